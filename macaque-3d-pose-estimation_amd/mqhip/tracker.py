"""Step-1 multi-object tracker: boxmot 12.0.7 ``BotSort`` as step 1 configures it (BOTSORT_CFG,
``src/pipeline/step1_proc2d.py``:75-89; one tracker per camera, :430; ``tracker.update(dets6, img)``,
:239-252): IoU association only (``with_reid=False``), track_high_thresh = new_track_thresh = 0.85,
track_low_thresh 0.10, match_thresh 0.80, track_buffer 72 at 24 fps, camera-motion compensation
``cmc_method='sift'``.

Host logic, as in the reference: a frame carries a handful of boxes, so the per-frame Kalman
predict / update and the assignment are a few microseconds of numpy -- there is nothing for the GPU
(the detector that feeds it and the ID / pose models after it run on MI355X).

Restated from boxmot's published BoT-SORT (boxmot is absent here):
* ``KalmanFilterXYWH`` (state x, y, w, h and their velocities; position / velocity noise weights
  1/20, 1/160 scaled by w / h);
* three association rounds -- high-score detections vs tracked + lost tracks (cost 1 - IoU, limit
  0.8), low-score detections vs the remaining tracked tracks (limit 0.5), the remaining high-score
  detections vs unconfirmed tracks (1 - IoU * score, limit 0.7) -- each an optimal assignment with a
  per-pair cost limit (lap.lapjv(extend_cost=True, cost_limit) semantics, solved on the same extended
  matrix with scipy's linear_sum_assignment);
* new tracks from unmatched detections above new_track_thresh (confirmed at once only on the first
  frame), lost tracks dropped after int(frame_rate / 30 * track_buffer) frames, duplicate removal
  (IoU > 0.85 between a tracked and a lost track keeps the older one);
* output rows ``[x1, y1, x2, y2, id, conf, cls, det_ind]`` from the Kalman posterior of every
  activated track.

Camera-motion compensation: the SIFT + RANSAC affine of boxmot needs OpenCV (absent here).  ``cmc``
is a callable (img, dets) -> 2x3 warp; the default is the identity, which is what the estimate tends
to for the reference's fixed cage cameras.  Parity with boxmot is unpinned.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg
from scipy.optimize import linear_sum_assignment

TRACKED, LOST, REMOVED = 1, 2, 3

BOTSORT_CFG = dict(track_high_thresh=0.85, track_low_thresh=0.10, new_track_thresh=0.85, track_buffer=72,
                   match_thresh=0.80, frame_rate=24, proximity_thresh=0.5, fuse_first_associate=False)


class KalmanFilterXYWH:
    """boxmot KalmanFilterXYWH: constant velocity in (x, y, w, h), noise proportional to w / h."""

    def __init__(self):
        nd, dt = 4, 1.0
        self._motion_mat = np.eye(2 * nd)
        for i in range(nd):
            self._motion_mat[i, nd + i] = dt
        self._update_mat = np.eye(nd, 2 * nd)
        self._w_pos, self._w_vel = 1.0 / 20, 1.0 / 160

    def initiate(self, m):
        mean = np.r_[m, np.zeros_like(m)]
        p, v = self._w_pos, self._w_vel
        std = [2 * p * m[2], 2 * p * m[3], 2 * p * m[2], 2 * p * m[3],
               10 * v * m[2], 10 * v * m[3], 10 * v * m[2], 10 * v * m[3]]
        return mean, np.diag(np.square(std))

    def _q(self, mean):
        p, v = self._w_pos, self._w_vel
        return np.square([p * mean[2], p * mean[3], p * mean[2], p * mean[3],
                          v * mean[2], v * mean[3], v * mean[2], v * mean[3]])

    def multi_predict(self, mean, cov):
        q = np.stack([self._q(m) for m in mean])
        motion_cov = np.asarray([np.diag(q[i]) for i in range(len(mean))])
        mean = np.dot(mean, self._motion_mat.T)
        left = np.dot(self._motion_mat, cov).transpose((1, 0, 2))
        return mean, np.dot(left, self._motion_mat.T) + motion_cov

    def project(self, mean, cov):
        p = self._w_pos
        r = np.diag(np.square([p * mean[2], p * mean[3], p * mean[2], p * mean[3]]))
        return np.dot(self._update_mat, mean), np.linalg.multi_dot((self._update_mat, cov, self._update_mat.T)) + r

    def update(self, mean, cov, m):
        pm, pc = self.project(mean, cov)
        cf, lower = scipy.linalg.cho_factor(pc, lower=True, check_finite=False)
        gain = scipy.linalg.cho_solve((cf, lower), np.dot(cov, self._update_mat.T).T, check_finite=False).T
        new_mean = mean + np.dot(m - pm, gain.T)
        return new_mean, cov - np.linalg.multi_dot((gain, pc, gain.T))


def xyxy2xywh(b):
    b = np.asarray(b, dtype=np.float64)
    return np.array([(b[0] + b[2]) / 2, (b[1] + b[3]) / 2, b[2] - b[0], b[3] - b[1]])


def xywh2xyxy(b):
    return np.array([b[0] - b[2] / 2, b[1] - b[3] / 2, b[0] + b[2] / 2, b[1] + b[3] / 2])


class STrack:
    def __init__(self, det):
        self.xywh = xyxy2xywh(det[0:4])
        self.conf, self.cls, self.det_ind = float(det[4]), det[5], int(det[6])
        self.kf = None
        self.mean = self.cov = None
        self.is_activated = False
        self.state = 0
        self.id = 0
        self.frame_id = self.start_frame = 0
        self.tracklet_len = 0

    @property
    def end_frame(self):
        return self.frame_id

    @property
    def xyxy(self):
        return xywh2xyxy(self.xywh.copy() if self.mean is None else self.mean[:4].copy())

    def activate(self, kf, frame_id, new_id):
        self.kf = kf
        self.id = new_id
        self.mean, self.cov = kf.initiate(self.xywh)
        self.tracklet_len = 0
        self.state = TRACKED
        if frame_id == 1:
            self.is_activated = True
        self.frame_id = self.start_frame = frame_id

    def _take(self, det):
        self.conf, self.cls, self.det_ind = det.conf, det.cls, det.det_ind

    def re_activate(self, det, frame_id):
        self.mean, self.cov = self.kf.update(self.mean, self.cov, det.xywh)
        self.tracklet_len = 0
        self.state = TRACKED
        self.is_activated = True
        self.frame_id = frame_id
        self._take(det)

    def update(self, det, frame_id):
        self.frame_id = frame_id
        self.tracklet_len += 1
        self.mean, self.cov = self.kf.update(self.mean, self.cov, det.xywh)
        self.state = TRACKED
        self.is_activated = True
        self._take(det)


def iou_batch(a, b):
    """boxmot iou_batch (no +1 pixel convention): (len(a), len(b))."""
    a = np.asarray(a, dtype=np.float64).reshape(-1, 4)[:, None]
    b = np.asarray(b, dtype=np.float64).reshape(-1, 4)[None]
    w = np.maximum(0.0, np.minimum(a[..., 2], b[..., 2]) - np.maximum(a[..., 0], b[..., 0]))
    h = np.maximum(0.0, np.minimum(a[..., 3], b[..., 3]) - np.maximum(a[..., 1], b[..., 1]))
    wh = w * h
    return wh / ((a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1]) + (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
                 - wh)


def iou_distance(ta, tb):
    if len(ta) == 0 or len(tb) == 0:
        return np.zeros((len(ta), len(tb)), dtype=np.float32)
    return 1 - iou_batch([t.xyxy for t in ta], [t.xyxy for t in tb])


def fuse_score(cost, dets):
    if cost.size == 0:
        return cost
    return 1 - (1 - cost) * np.array([d.conf for d in dets])[None, :]


def linear_assignment(cost, thresh):
    """lap.lapjv(cost, extend_cost=True, cost_limit=thresh): the (n+m) x (n+m) extension with thresh / 2 for
    leaving a row or a column unmatched; a pair is matched only when that is cheaper."""
    n, m = cost.shape
    if cost.size == 0:
        return np.empty((0, 2), dtype=int), np.arange(n), np.arange(m)
    ext = np.zeros((n + m, n + m))
    ext[:n, :m] = cost
    ext[:n, m:] = thresh / 2.0
    ext[n:, :m] = thresh / 2.0
    r, c = linear_sum_assignment(ext)
    x = np.full(n, -1)
    y = np.full(m, -1)
    for i, j in zip(r, c):
        if i < n and j < m:
            x[i], y[j] = j, i
    matches = np.array([[i, x[i]] for i in range(n) if x[i] >= 0], dtype=int).reshape(-1, 2)
    return matches, np.where(x < 0)[0], np.where(y < 0)[0]


def joint_stracks(a, b):
    seen, res = set(), []
    for t in list(a) + list(b):
        if t.id not in seen:
            seen.add(t.id)
            res.append(t)
    return res


def sub_stracks(a, b):
    drop = {t.id for t in b}
    return [t for t in a if t.id not in drop]


def remove_duplicate_stracks(sa, sb):
    pdist = iou_distance(sa, sb)
    dupa, dupb = set(), set()
    for p, q in zip(*np.where(pdist < 0.15)):
        if sa[p].frame_id - sa[p].start_frame > sb[q].frame_id - sb[q].start_frame:
            dupb.add(q)
        else:
            dupa.add(p)
    return [t for i, t in enumerate(sa) if i not in dupa], [t for i, t in enumerate(sb) if i not in dupb]


def identity_cmc(img, dets):
    return np.eye(2, 3)


class BotSort:
    """``BotSort(**BOTSORT_CFG).update(dets (N, 6) [x1, y1, x2, y2, conf, cls], img)`` -> (M, 8) rows
    [x1, y1, x2, y2, id, conf, cls, det_ind] of the activated tracks."""

    def __init__(self, track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6, track_buffer=30,
                 match_thresh=0.8, frame_rate=30, proximity_thresh=0.5, fuse_first_associate=False, cmc=None,
                 with_reid=False, **_ignored):
        if with_reid:
            raise NotImplementedError("with_reid=True (step 1 runs BoT-SORT without ReID, step1_proc2d.py:81)")
        self.track_high_thresh, self.track_low_thresh = track_high_thresh, track_low_thresh
        self.new_track_thresh, self.match_thresh = new_track_thresh, match_thresh
        self.proximity_thresh, self.fuse_first_associate = proximity_thresh, fuse_first_associate
        self.max_time_lost = int(frame_rate / 30.0 * track_buffer)
        self.kf = KalmanFilterXYWH()
        self.cmc = cmc or identity_cmc
        self.active_tracks, self.lost_stracks, self.removed_stracks = [], [], []
        self.frame_count = 0
        self._next = 0

    def _new_id(self):
        self._next += 1
        return self._next

    def _predict(self, tracks):
        if not tracks:
            return
        mean = np.asarray([t.mean.copy() for t in tracks])
        cov = np.asarray([t.cov for t in tracks])
        for i, t in enumerate(tracks):
            if t.state != TRACKED:
                mean[i][6] = mean[i][7] = 0
        mean, cov = self.kf.multi_predict(mean, cov)
        for t, mu, c in zip(tracks, mean, cov):
            t.mean, t.cov = mu, c

    @staticmethod
    def _gmc(tracks, H):
        if not tracks:
            return
        R8 = np.kron(np.eye(4), H[:2, :2])
        for t in tracks:
            mean = R8.dot(t.mean)
            mean[:2] += H[:2, 2]
            t.mean, t.cov = mean, R8.dot(t.cov).dot(R8.T)

    def update(self, dets, img=None):
        dets = np.asarray(dets, dtype=np.float64).reshape(-1, 6)
        self.frame_count += 1
        fc = self.frame_count
        activated, refind, lost, removed = [], [], [], []
        dets = np.hstack([dets, np.arange(len(dets)).reshape(-1, 1)])
        confs = dets[:, 4]
        dets_second = dets[(confs > self.track_low_thresh) & (confs < self.track_high_thresh)]
        dets_first = dets[confs > self.track_high_thresh]
        detections = [STrack(d) for d in dets_first]
        unconfirmed = [t for t in self.active_tracks if not t.is_activated]
        tracked = [t for t in self.active_tracks if t.is_activated]

        # 1st association: high-score detections vs tracked + lost tracks
        pool = joint_stracks(tracked, self.lost_stracks)
        self._predict(pool)
        warp = self.cmc(img, dets_first)
        self._gmc(pool, warp)
        self._gmc(unconfirmed, warp)
        dists = iou_distance(pool, detections)
        if self.fuse_first_associate:
            dists = fuse_score(dists, detections)
        matches, u_track, u_det = linear_assignment(dists, self.match_thresh)
        for it, idet in matches:
            t, d = pool[it], detections[idet]
            if t.state == TRACKED:
                t.update(d, fc)
                activated.append(t)
            else:
                t.re_activate(d, fc)
                refind.append(t)

        # 2nd association: low-score detections vs the remaining tracked tracks
        det2 = [STrack(d) for d in dets_second]
        r_tracked = [pool[i] for i in u_track if pool[i].state == TRACKED]
        matches, u_track2, _ = linear_assignment(iou_distance(r_tracked, det2), 0.5)
        for it, idet in matches:
            t, d = r_tracked[it], det2[idet]
            if t.state == TRACKED:
                t.update(d, fc)
                activated.append(t)
            else:
                t.re_activate(d, fc)
                refind.append(t)
        for it in u_track2:
            t = r_tracked[it]
            if t.state != LOST:
                t.state = LOST
                lost.append(t)

        # unconfirmed tracks (one frame old) vs the remaining high-score detections
        detections = [detections[i] for i in u_det]
        dists = fuse_score(iou_distance(unconfirmed, detections), detections)
        matches, u_unconf, u_det = linear_assignment(dists, 0.7)
        for it, idet in matches:
            unconfirmed[it].update(detections[idet], fc)
            activated.append(unconfirmed[it])
        for it in u_unconf:
            unconfirmed[it].state = REMOVED
            removed.append(unconfirmed[it])

        # new tracks
        for inew in u_det:
            t = detections[inew]
            if t.conf < self.new_track_thresh:
                continue
            t.activate(self.kf, fc, self._new_id())
            activated.append(t)

        for t in self.lost_stracks:
            if fc - t.end_frame > self.max_time_lost:
                t.state = REMOVED
                removed.append(t)

        self.active_tracks = [t for t in self.active_tracks if t.state == TRACKED]
        self.active_tracks = joint_stracks(self.active_tracks, activated)
        self.active_tracks = joint_stracks(self.active_tracks, refind)
        self.lost_stracks = sub_stracks(self.lost_stracks, self.active_tracks)
        self.lost_stracks.extend(lost)
        self.lost_stracks = sub_stracks(self.lost_stracks, self.removed_stracks)
        self.removed_stracks.extend(removed)
        self.active_tracks, self.lost_stracks = remove_duplicate_stracks(self.active_tracks, self.lost_stracks)

        out = [list(t.xyxy) + [t.id, t.conf, t.cls, t.det_ind] for t in self.active_tracks if t.is_activated]
        return np.asarray(out, dtype=np.float64).reshape(-1, 8)
