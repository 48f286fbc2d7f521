"""Step 1 -- the pose slice of ``src/pipeline/step1_proc2d.py`` on MI355X.

Kept from the reference (same constants, same row format, same files):
  * box filtering and dynamic-margin expansion with aspect fix (step1:255-292),
  * top-down ViTPose-H with heatmap flip test (step1:100-101, :294-298) --
    through ``mqhip.apis`` (crop -> 32-layer ViT -> UDP/DARK decode in libmq_hip),
  * keypoint threshold (KP_THR) and the recursive per-track EMA (step1:300-343),
  * ``alldata.json`` rows ``[tid, x1, y1, x2, y2, [[x, y, s] x 17], id, id_score]``
    and ``frame_num.npy`` (step1:345-395).

MI355X-first: ``process_frame_multiview`` sends every box of every view of a
frame through ONE batched launch sequence instead of one ``inference_topdown``
per camera.

The Swin-S Mask R-CNN detector runs on MI355X too (``init_detector`` / ``inference_detector``,
step1:98, :226-237 -> ``mqhip.detector``); ``detect_stores`` gives, per camera and processed frame,
the detections above SCORE_THR that the reference hands to its tracker (step1:229-240).

The ResNet-152 collar-ID classifier runs on MI355X too (``init_id_model`` / ``classify_patches``,
step1:125-163 -> ``mqhip.resnet_id``); ``process_stores(..., id_model=...)`` classifies every tracked
box of a batch of time steps x cameras in one launch sequence.

The BoT-SORT tracker (``mqhip.tracker.BotSort`` with BOTSORT_CFG, host logic as in the reference)
turns the detections into tracker rows: ``track_stores`` runs detector -> tracker per camera over the
frame plan, and ``step1_proc2d_custom(..., detector=...)`` chains detector -> tracker -> pose -> ID.
Without a detector the tracker rows enter as data: per-frame ``(N, >=5)`` [x1, y1, x2, y2,
track_id, ...] carried by the per-camera ``mqhip.io.FrameStore`` that ``proc`` reads (imgstore video
decoding is out of scope).
Without an ID model or stored ID predictions every box gets ``assigned_id = -1`` (the reference's
"not confident" value).
"""
from __future__ import annotations

import json
import os
from collections import deque
from pathlib import Path

import numpy as np

from mqhip.apis import inference_topdown, inference_topdown_batch, init_model

DETECT_CONFIG = "./model/detection/SWIN-Mask_R-CNN_bbox_only.py"
DETECT_CHECKPOINT = "./model/detection/detection.pth"
POSE_CONFIG = "./model/pose/ViTPose_huge_macaque_256x192.py"
POSE_CHECKPOINT = "./model/pose/pose.pth"

SCORE_THR = 0.85
KP_THR = 0.30
EMA_ALPHA = 0.50
DISP_THR = 20.0
MIN_MARGIN = 0.20
MAX_MARGIN = 0.50
DESIRED_AR = 192.0 / 256.0
ID_CONF_THR = 0.80

TRACK_BUFFER = 72  # frames to buffer lost tracks (~3 s at 24 fps), step1:75
BOTSORT_CFG = dict(with_reid=False, track_high_thresh=SCORE_THR, track_low_thresh=0.10, new_track_thresh=SCORE_THR,
                   track_buffer=TRACK_BUFFER, match_thresh=0.80, frame_rate=24, cmc_method="sift")

ID_CONFIGS = {
    "normal": "./model/id/sn_resnet152_8xb32_in1k_pretrained_optimized_finetuned.py",
    "mff1y": "./model/id/sn_resnet152_8xb32_in1k_mff1y_pretrained_optimized.py",
}
ID_CKPTS = {
    "normal": "./model/id/id_finetuned.pth",
    "mff1y": "./model/id/id_mff1y.pth",
}

KP_PARAMS = {"score_thr": SCORE_THR, "kp_thr": KP_THR, "ema_alpha": EMA_ALPHA, "disp_thr": DISP_THR,
             "min_margin": MIN_MARGIN, "max_margin": MAX_MARGIN, "desired_ar": DESIRED_AR,
             "id_conf_thr": ID_CONF_THR}


def init_detector(config=DETECT_CONFIG, checkpoint=DETECT_CHECKPOINT, device="cuda:0", weights=None):
    """mmdet init_detector (step1:98) -> the MI355X Swin-S Mask R-CNN.  The checkpoint is read with
    torch.load(weights_only=True) when it exists (mmdet keys under 'state_dict'); otherwise seeded
    random weights (no checkpoint ships with the reference)."""
    from mqhip.detector import SwinDetectorHip, make_random_weights
    dev = int(device.split(":")[1]) if ":" in device else 0
    if weights is None:
        if checkpoint and os.path.exists(checkpoint):
            import torch
            ck = torch.load(checkpoint, map_location="cpu", weights_only=True)
            weights = {k: v.float() for k, v in ck.get("state_dict", ck).items()}
        else:
            weights = make_random_weights(seed=0)
    return SwinDetectorHip(weights, device=dev)


def inference_detector(detector, imgs, test_pipeline=None):
    """mmdet inference_detector(detector, [img], test_pipeline) (step1:226): per image
    (bboxes (k, 4) float32, scores (k,)) in original pixels, score-ordered; the test pipeline is the
    detector's own (Resize 800x800 keep-ratio + DetDataPreprocessor, step1:104-109)."""
    from mqhip.detector import inference_detector as _inf
    return _inf(detector, imgs)


def detect_stores(detector, stores, T, score_thr=SCORE_THR):
    """Detections per camera over step 1's frame plan (the boxes the reference's tracker receives,
    step1:210-240): {cam: [(frame_number, boxes (k, 4), scores (k,))]} for every frame a camera
    processes (repeats of the time-sync walk are skipped, as there); the cameras that process a frame
    at the same time step go through one detector batch."""
    plans = [_frame_plan(st, T) for st in stores]
    out = {i: [] for i in range(len(stores))}
    for k in range(len(T)):
        cams = [i for i, p in enumerate(plans) if not p[k][1]]
        if not cams:
            continue
        by_shape = {}
        for i in cams:  # one detector batch per image size (cameras may differ in resolution)
            img = stores[i].image(plans[i][k][0])
            by_shape.setdefault(img.shape, []).append((i, img))
        for items in by_shape.values():
            for (i, _), (b, sc) in zip(items, inference_detector(detector, [im for _, im in items])):
                keep = sc > score_thr
                out[i].append((plans[i][k][0], b[keep], sc[keep]))
    return out


def init_id_model(device: str = "cuda:0", id_variant: str = "normal", weights=None, random_weights=False):
    """step1:125-136: the ResNet-152 ID classifier of ``id_variant`` (None for an unknown variant, as
    there).  The checkpoint is read with torch.load(weights_only=True) (mmpretrain keys under
    'state_dict').  A missing checkpoint raises FileNotFoundError, as the reference's init_model does,
    unless ``random_weights`` asks for seeded random weights (tests and bench only: no checkpoint ships
    with the reference)."""
    from mqhip.resnet_id import ResNetIdHip, make_random_weights
    if ID_CONFIGS.get(id_variant) is None or ID_CKPTS.get(id_variant) is None:
        return None
    dev = int(device.split(":")[1]) if ":" in device else 0
    if weights is None:
        ck = ID_CKPTS[id_variant]
        if os.path.exists(ck):
            import torch
            sd = torch.load(ck, map_location="cpu", weights_only=True)
            weights = {k: v.float() for k, v in sd.get("state_dict", sd).items()}
        elif random_weights:  # one seed per variant, so a camera's variant shows in its predictions
            weights = make_random_weights(152, seed={"normal": 0, "mff1y": 1}[id_variant])
        else:
            raise FileNotFoundError(f"ID checkpoint of variant {id_variant!r} not found: {ck}")
    return ResNetIdHip(weights, depth=152, device=dev)


def classify_patches(id_model, patches, input_size: int = 224):
    """step1:140-163: crop-and-classify patches through the ID model -> [{pred_label, pred_score}] (label -1,
    score 0 for an empty patch or without a model).  All non-empty patches go through one batch."""
    if id_model is None or not patches:
        return [{"pred_label": -1, "pred_score": 0.0} for _ in patches]
    if input_size != 224:
        raise NotImplementedError("the ID pipeline is built for input_size 224 (ResizeEdge 256, CenterCrop 224)")
    return id_model.classify_patches(patches)


def classify_boxes(id_model, imgs, boxes_per_view):
    """The ID half of step1:301-302 for all views of a frame: ``img[y1:y2, x1:x2]`` per int box, classified
    in one batch -> per view [{pred_label, pred_score}]."""
    if id_model is None:
        return [[{"pred_label": -1, "pred_score": 0.0} for _ in b] for b in boxes_per_view]
    return id_model.classify(imgs, boxes_per_view)


def init_tracker(cfg=None):
    """step1:99 / :430 ``BotSort(**BOTSORT_CFG)`` -- one per camera (camera-motion compensation: identity,
    see mqhip.tracker)."""
    from mqhip.tracker import BotSort
    return BotSort(**(cfg or BOTSORT_CFG))


def track_stores(detector, stores, T, score_thr=SCORE_THR, tracker_cfg=None):
    """Detector -> tracker per camera over step 1's frame plan (step1:225-252): a frame whose detections are
    all <= score_thr gets no tracker update and no rows; otherwise ``tracker.update(dets6, img)`` with
    dets6 = [boxes, scores, 0].  Returns per camera {frame_number: tracker rows (k, 8)}."""
    dets = detect_stores(detector, stores, T, score_thr)
    out = []
    for c, st in enumerate(stores):
        tr = init_tracker(tracker_cfg)
        rows = {}
        for fn, b, sc in dets[c]:
            if len(sc) == 0:
                rows[fn] = np.zeros((0, 8))
                continue
            d6 = np.hstack([np.asarray(b, np.float64), np.asarray(sc, np.float64)[:, None], np.zeros((len(sc), 1))])
            rows[fn] = tr.update(d6, st.image(fn))
        out.append(rows)
    return out


def init_pose_model(config=POSE_CONFIG, checkpoint=POSE_CHECKPOINT, device="cuda:0"):
    """step1:100-101: the pose model with the reference's test_cfg."""
    model = init_model(config, checkpoint, device=device)
    model.test_cfg = dict(flip_test=True, flip_mode="heatmap", shift_heatmap=False)
    return model


def filter_tracks(tracks):
    """step1:255-268: tracker rows -> int32 boxes with positive extent + their track ids."""
    t = np.asarray(tracks, dtype=np.float64)
    if t.size == 0:
        return np.zeros((0, 4), np.int32), np.zeros((0,), np.int32)
    t = t.reshape(len(t), -1)
    b = t[:, :4].astype(np.int64)                     # int() truncation toward zero
    ok = (b[:, 2] > b[:, 0]) & (b[:, 3] > b[:, 1])
    return b[ok].astype(np.int32), t[ok, 4].astype(int).astype(np.int32)


def expand_boxes(boxes, kp_params=KP_PARAMS):
    """step1:270-292: margin 0.5 -> 0.2 as the box height grows 50 -> 200 px, aspect fixed to
    0.75 when off by > 0.2, centre kept.  int32 (N,4) xyxy -> float32 (N,4) xyxy."""
    b = np.asarray(boxes, dtype=np.float64).reshape(-1, 4)
    w, h = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
    cx, cy = b[:, 0] + 0.5 * w, b[:, 1] + 0.5 * h
    frac = np.clip((h - 50.0) / (200.0 - 50.0), 0.0, 1.0)
    mx, mn, ar_t = kp_params["max_margin"], kp_params["min_margin"], kp_params["desired_ar"]
    m = mx - (mx - mn) * frac
    wn, hn = w * (1 + m), h * (1 + m)
    ar = wn / hn
    fix = np.abs(ar - ar_t) > 0.20
    wide = ar >= ar_t
    wn = np.where(fix & ~wide, hn * ar_t, wn)
    hn = np.where(fix & wide, wn / ar_t, hn)
    xywh = np.stack([cx, cy, wn, hn], axis=1).astype(np.float32).astype(np.float64)
    half = 0.5 * xywh[:, 2:]
    return np.concatenate([xywh[:, :2] - half, xywh[:, :2] + half], axis=1).astype(np.float32)


class KeypointSmoother:
    """step1:300-343: KP_THR masking, then the recursive EMA over a per-track deque(5)."""

    def __init__(self, kp_params=KP_PARAMS):
        self.p = kp_params
        self.buffers: dict[int, deque] = {}

    def clear(self):
        self.buffers.clear()

    def update(self, tid, frame_number, kpt_xy, kpt_score):
        return self.update_many([tid], frame_number, np.asarray(kpt_xy)[None], np.asarray(kpt_score)[None])[0]

    def update_many(self, tids, frame_number, kpt_xy, kpt_score):
        """``update`` for the n boxes of one frame at once (n, J, 2) / (n, J) -> (n, J, 3): the same
        element-wise float64 / float32 arithmetic, vectorised over the boxes.  Boxes sharing a track id
        within the frame (the second one smooths against the first) take the sequential path."""
        tids = [t if isinstance(t, tuple) else int(t) for t in tids]   # (camera, track) keys: several cameras
        if len(set(tids)) != len(tids):
            return np.stack([self.update_many([t], frame_number, np.asarray(kpt_xy)[i:i + 1],
                                              np.asarray(kpt_score)[i:i + 1])[0] for i, t in enumerate(tids)])
        xy = np.array(kpt_xy, dtype=np.float64, copy=True)
        sc = np.array(kpt_score, dtype=np.float32, copy=True)
        low = sc < self.p["kp_thr"]
        xy[low] = np.nan
        sc[low] = 0.0
        kp = np.concatenate([xy, sc[..., None]], axis=-1)                    # (n, J, 3)
        hist = []
        for i, t in enumerate(tids):
            buf = self.buffers.setdefault(t, deque(maxlen=5))
            if buf:
                hist.append(i)
        if hist:
            prev = np.stack([self.buffers[tids[i]][-1][1] for i in hist])     # (h, J, 3) smoothed previous
            cur = kp[hist]
            both = ~np.isnan(prev[..., 0]) & ~np.isnan(cur[..., 0])
            disp = np.zeros(both.shape, dtype=np.float32)
            if both.any():
                disp[both] = np.linalg.norm(cur[both][:, :2] - prev[both][:, :2], axis=1)
            sm = (disp < self.p["disp_thr"]) & both
            a = self.p["ema_alpha"]
            cur[sm, :2] = a * prev[sm][:, :2] + (1 - a) * cur[sm][:, :2]
            kp[hist] = cur
        for i, t in enumerate(tids):
            self.buffers[t].append((frame_number, kp[i].copy()))
        return kp


def _rows(pose_results, boxes, tids, smoother, frame_number, id_preds, kp_params):
    n = len(pose_results)
    if n == 0:
        return []
    kps, scs = [], []
    for pr in pose_results:
        kp = pr.pred_instances.keypoints[0]
        try:
            sc = pr.pred_instances.keypoint_scores[0]
        except AttributeError:
            sc = np.ones(kp.shape[0], dtype=np.float32)
        kps.append(np.asarray(kp, dtype=np.float64))
        scs.append(np.asarray(sc, dtype=np.float32))
    return _rows_arrays(np.stack(kps), np.stack(scs), boxes, tids, smoother, frame_number, id_preds, kp_params)


def _rows_arrays(kp, sc, boxes, tids, smoother, frame_number, id_preds, kp_params):
    """alldata rows [tid, x1, y1, x2, y2, [[x, y, s] x J], assigned_id, id_score] (step1:345-362) of the
    n boxes of one frame from their keypoints (n, J, 2) float64 and scores (n, J) float32."""
    n = len(kp)
    if n == 0:
        return []
    sm = smoother.update_many([int(tids[i]) for i in range(n)], frame_number, kp, sc).tolist()
    return _rows_smoothed(sm, boxes, tids, id_preds, kp_params)


def _rows_smoothed(sm, boxes, tids, id_preds, kp_params):
    """alldata rows from the smoothed keypoints ``sm`` (n lists of J [x, y, s])."""
    n = len(sm)
    bx = np.asarray(boxes[:n], dtype=np.float64).tolist()
    rows = []
    for i in range(n):
        if id_preds is None:
            label, score = -1, 0.0
        else:
            label, score = int(id_preds[i]["pred_label"]), float(id_preds[i]["pred_score"])
        assigned = label if score >= kp_params["id_conf_thr"] else -1
        rows.append([int(tids[i])] + bx[i] + [sm[i], assigned, score])
    return rows


def process_frame(pose_model, img, tracks, smoother, frame_number, id_preds=None, kp_params=KP_PARAMS,
                  id_model=None):
    """One camera frame: tracker rows -> alldata.json rows (step1:255-364).  With ``id_model`` the
    tracked boxes' patches are classified here (step1:301-302); else ``id_preds`` (or none)."""
    boxes, tids = filter_tracks(tracks)
    if len(boxes) == 0:
        return []
    bb = expand_boxes(boxes, kp_params)
    res = inference_topdown(pose_model, img, bboxes=bb, bbox_format="xyxy")
    if id_model is not None:
        id_preds = classify_patches(id_model, [img[y1:y2, x1:x2] for (x1, y1, x2, y2) in boxes])
    return _rows(res, boxes, tids, smoother, frame_number, id_preds, kp_params)


def process_frame_multiview(pose_model, imgs, tracks_per_view, smoothers, frame_number, id_preds_per_view=None,
                            kp_params=KP_PARAMS, id_model=None):
    """All views of one frame in one batched crop -> ViT -> decode pass (and, with ``id_model``, one
    batched ID pass over every tracked box).  imgs: list of HxWx3 uint8 or a (V,H,W,3) uint8 GPU tensor;
    smoothers: one KeypointSmoother per view."""
    per_view = [filter_tracks(t) for t in tracks_per_view]
    bbs = [expand_boxes(b, kp_params) if len(b) else np.zeros((0, 4), np.float32) for b, _ in per_view]
    results = inference_topdown_batch(pose_model, imgs, bbs)
    if id_model is not None:
        id_preds_per_view = classify_boxes(id_model, imgs if not isinstance(imgs, list) else np.stack(imgs),
                                           [b for b, _ in per_view])
    out = []
    for v, ((boxes, tids), res) in enumerate(zip(per_view, results)):
        ids = None if id_preds_per_view is None else id_preds_per_view[v]
        out.append(_rows(res, boxes, tids, smoothers[v], frame_number, ids, kp_params) if len(boxes) else [])
    return out


def process_single_cam(frames, tracks, out_dir, pose_model, frame_numbers=None, id_preds=None,
                       kp_params=KP_PARAMS, id_model=None):
    """Pose half of step1:166-410 for one camera.  frames: iterable of BGR uint8 images;
    tracks: per-frame tracker rows; writes alldata.json + frame_num.npy to out_dir."""
    os.makedirs(out_dir, exist_ok=True)
    smoother = KeypointSmoother(kp_params)
    results, fnums = [], []
    for k, (img, trk) in enumerate(zip(frames, tracks)):
        fn = k if frame_numbers is None else int(frame_numbers[k])
        ids = None if id_preds is None else id_preds[k]
        results.append(process_frame(pose_model, img, trk, smoother, fn, ids, kp_params, id_model=id_model))
        fnums.append(fn)
    np.save(Path(out_dir) / "frame_num.npy", np.array(fnums, dtype=np.int32))
    with open(Path(out_dir) / "alldata.json", "w") as fp:
        fp.write(json.dumps(results))  # same text as json.dump, C encoder
    return results


def _frame_plan(store, T):
    """The reference's per-camera walk over the time grid (step1_proc2d.py:210-223): for each t the
    stored frame nearest in time; a t whose nearest frame is not newer than the last one processed
    repeats the previous result.  Returns [(frame_number, is_repeat)] per t."""
    md = store.get_frame_metadata()
    t_cam, fnums = md["frame_time"], md["frame_number"]
    plan, frame_number = [], -1
    for t in T:
        idx = int(np.abs(t_cam - t).argmin())
        if frame_number >= fnums[idx]:
            plan.append((frame_number, True))
            continue
        frame_number = int(fnums[idx])
        plan.append((frame_number, False))
    return plan


def plan_jobs(stores, T, kp_params=KP_PARAMS, tracks=None):
    """Per camera the time-grid walk (_frame_plan) and, per time step, the pose jobs of the frames
    it newly reaches: {step: [(cam, frame_number, boxes int32, track ids, expanded boxes f32)]}
    (degenerate-box filter and margin expansion of step1:254-292).  ``tracks``: per camera
    {frame_number: tracker rows} (track_stores) instead of the stores' rows."""
    plans = [_frame_plan(st, T) for st in stores]
    jobs = {}
    for k in range(len(T)):
        for c, st in enumerate(stores):
            fn, rep = plans[c][k]
            if rep:
                continue
            rows = st.tracks_of(fn) if tracks is None else tracks[c].get(fn, np.zeros((0, 8)))
            boxes, tids = filter_tracks(rows)
            if len(boxes):
                jobs.setdefault(k, []).append((c, fn, boxes, tids, expand_boxes(boxes, kp_params)))
    return plans, jobs


def run_pose(pose_model, stores, jobs, steps, steps_per_batch=8):
    """The ViTPose work of the given time steps: every job of ``steps_per_batch`` consecutive steps
    (all cameras) in ONE batched crop -> ViT -> decode launch sequence per image size.
    Returns {(step, cam): (keypoints float64 (n, J, 2), scores float32 (n, J))}."""
    steps = [k for k in steps if k in jobs]
    raw = {}
    for b0 in range(0, len(steps), steps_per_batch):
        by_shape = {}
        for k in steps[b0:b0 + steps_per_batch]:
            for (c, fn, _, _, bb) in jobs[k]:
                img = stores[c].image(fn)
                by_shape.setdefault(img.shape, []).append(((k, c), img, bb))
        for items in by_shape.values():
            out = inference_topdown_batch(pose_model, [im for _, im, _ in items], [bb for _, _, bb in items])
            for (key, _, _), r in zip(items, out):
                kp = np.stack([np.asarray(x.pred_instances.keypoints[0], dtype=np.float64) for x in r])
                sc = np.stack([np.asarray(x.pred_instances.keypoint_scores[0], dtype=np.float32) for x in r])
                raw[key] = (kp, sc)
    return raw


def id_variant_of(store):
    """step1:425-426: the ID checkpoint of a camera -- 'mff1y' when its store folder name contains it."""
    return "mff1y" if "mff1y" in os.path.basename(str(store.filename)).lower() else "normal"


def resolve_id_models(stores, id_model, device_str="cuda:0"):
    """One ID model (or None) per store.  ``id_model``: None (no classification: the stores' own ID
    predictions, if any); ``"auto"`` -- the reference's rule, ``init_id_model(device, id_variant_of(store))``
    per camera (step1:424-427), each variant built once; a variant whose checkpoint is missing warns and
    keeps the stores' own predictions (None) instead of classifying with random weights;
    ``"random"`` -- the same per-variant models with seeded random weights (tests and bench only);
    a dict {variant: model}; or one model for every camera."""
    if id_model is None:
        return None
    if isinstance(id_model, str):
        if id_model not in ("auto", "random"):
            raise ValueError(f"id_model must be None, 'auto', 'random', a dict or a model, not {id_model!r}")
        cache = {}
        for st in stores:
            v = id_variant_of(st)
            if v in cache:
                continue
            if id_model == "random":
                cache[v] = init_id_model(device_str, v, random_weights=True)
                continue
            try:
                cache[v] = init_id_model(device_str, v)
            except FileNotFoundError as e:
                import warnings
                warnings.warn(f"{e}; cameras of variant {v!r} keep their stores' ID predictions")
                cache[v] = None
        return [cache[id_variant_of(st)] for st in stores]
    if isinstance(id_model, dict):
        return [id_model.get(id_variant_of(st)) for st in stores]
    return [id_model] * len(stores)


def run_id(id_model, stores, jobs, steps, steps_per_batch=8):
    """The ID classification of the given time steps' tracked boxes (step1:301-302): every job of
    ``steps_per_batch`` consecutive steps (all cameras) in ONE batched patch -> ResNet launch sequence
    per (ID model, image size).  ``id_model``: one model, or a list with one model (or None) per store
    (``resolve_id_models``).  Returns {(step, cam): [{pred_label, pred_score}] per box}; cameras without a
    model get the reference's "not classified" value (label -1, score 0)."""
    models = id_model if isinstance(id_model, (list, tuple)) else [id_model] * len(stores)
    steps = [k for k in steps if k in jobs]
    out = {}
    for b0 in range(0, len(steps), steps_per_batch):
        by_key = {}
        for k in steps[b0:b0 + steps_per_batch]:
            for (c, fn, boxes, _, _) in jobs[k]:
                if models[c] is None:
                    out[(k, c)] = [{"pred_label": -1, "pred_score": 0.0} for _ in boxes]
                    continue
                img = stores[c].image(fn)
                by_key.setdefault((id(models[c]), img.shape), (models[c], []))[1].append(((k, c), img, boxes))
        for model, items in by_key.values():
            preds = model.classify(np.stack([im for _, im, _ in items]), [bx for _, _, bx in items])
            for (key, _, _), p in zip(items, preds):
                out[key] = p
    return out


_PINNED = {}
_SIDE = {}


def _pinned_frames(shape, key):
    """A reusable page-locked host buffer of at least ``shape`` (n, H, W, 3) u8 per ``key``."""
    import torch
    n = int(np.prod(shape))
    buf = _PINNED.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        _PINNED[key] = buf
    return buf[:n].view(*shape)


def _to_host(t):
    """Device -> page-locked host copy, queued on the current stream (read it after the batch's event)."""
    import torch
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    return h


def run_pose_id(pose_model, id_model, stores, jobs, steps, steps_per_batch=8):
    """``run_pose`` and ``run_id`` over the same batches, pipelined: every frame of a batch is read once
    into a page-locked buffer (two, alternating) and uploaded once on a side stream; the pose crops and the
    ID patches are cut from that device copy; the outputs come back by queued copies, and the host reads
    batch b - 1's results while the GPU runs batch b (the two passes stacked and uploaded every frame twice
    and waited on each batch).  Batches, their order and their box order are the two passes' own, so the
    results are theirs bit for bit.  Returns (raw, id_raw); id_raw is None without an ``id_model``."""
    if getattr(pose_model, "device_index", None) is None:  # a stand-in model (host tests): the two passes
        return (run_pose(pose_model, stores, jobs, steps, steps_per_batch),
                None if id_model is None else run_id(id_model, stores, jobs, steps, steps_per_batch))
    import torch
    from mqhip.apis import _sample
    from mqhip.resnet_id import patch_bounds
    models = None if id_model is None else (
        id_model if isinstance(id_model, (list, tuple)) else [id_model] * len(stores))
    steps = [k for k in steps if k in jobs]
    di = pose_model.device_index
    dev = torch.device("cuda", di)
    cs = torch.cuda.current_stream(dev)
    xs = _SIDE.get(di)
    if xs is None:
        xs = _SIDE[di] = torch.cuda.Stream(device=dev)
    raw, id_raw = {}, (None if models is None else {})

    def launch(items, key):
        host = _pinned_frames((len(items),) + tuple(items[0][1].shape), key)
        for i, (_, img, _, _) in enumerate(items):
            host[i].numpy()[...] = img
        with torch.cuda.stream(xs):
            frames = host.to(dev, non_blocking=True)
            up = torch.cuda.Event()
            up.record(xs)
        cs.wait_event(up)
        frames.record_stream(cs)
        # pose: inference_topdown_batch's batch, outputs left on the device
        boxes, owner = [], []
        for i, (_, _, _, bb) in enumerate(items):
            b = np.asarray(bb, dtype=np.float32).reshape(-1, 4)
            boxes.append(b)
            owner += [i] * len(b)
        pose_out = None
        if owner:
            allb = np.concatenate(boxes)
            kp, score, _ = pose_model.net.topdown(frames, torch.from_numpy(allb).to(dev),
                                                  torch.tensor(owner, dtype=torch.int32, device=dev),
                                                  flip_test=pose_model.flip_test)
            pose_out = (allb, owner, _to_host(kp), _to_host(score))
        # ID: run_id's grouping (per model, items in step / camera order) and classify's box order
        id_out = []
        if models is not None:
            groups = {}
            for i, ((k, c), _, bxs, _) in enumerate(items):
                if models[c] is None:
                    id_raw[(k, c)] = [{"pred_label": -1, "pred_score": 0.0} for _ in bxs]
                else:
                    groups.setdefault(id(models[c]), (models[c], []))[1].append(i)
            for model, idx in groups.values():
                res = {i: [{"pred_label": -1, "pred_score": 0.0} for _ in range(len(items[i][2]))] for i in idx}
                rows, where = [], []
                for i in idx:
                    for j, b in enumerate(np.asarray(items[i][2]).reshape(-1, 4)):
                        pb = patch_bounds(frames.shape[1:3], b)
                        if pb is not None:
                            y0, y1, x0, x1 = pb
                            rows.append((i, x0, y0, x1, y1))
                            where.append((i, j))
                probs = None
                if rows:
                    x, _ = model.preprocess(frames, rows)
                    probs = _to_host(model.forward(x)[1])
                id_out.append((res, where, probs))
        return items, pose_out, id_out

    def finish(batch, ev):
        ev.synchronize()
        for items, pose_out, id_out in batch:
            per = [[] for _ in items]
            if pose_out is not None:
                allb, owner, kp, score = pose_out
                kp, score = kp.numpy(), score.numpy()
                for k, i in enumerate(owner):
                    per[i].append(_sample(kp[k], score[k], allb[k]))
            for (key, _, _, _), r in zip(items, per):
                kpa = np.stack([np.asarray(x.pred_instances.keypoints[0], dtype=np.float64) for x in r])
                sca = np.stack([np.asarray(x.pred_instances.keypoint_scores[0], dtype=np.float32) for x in r])
                raw[key] = (kpa, sca)
            for res, where, probs in id_out:
                if probs is not None:
                    p = probs.numpy()
                    for (i, j), pr in zip(where, p):
                        res[i][j] = {"pred_label": int(np.argmax(pr)), "pred_score": float(np.max(pr))}
                for i, r in res.items():
                    id_raw[items[i][0]] = r

    pending = None
    for bi, b0 in enumerate(range(0, len(steps), steps_per_batch)):
        by_shape = {}
        for k in steps[b0:b0 + steps_per_batch]:
            for (c, fn, bxs, _, bb) in jobs[k]:
                img = stores[c].image(fn)
                by_shape.setdefault(img.shape, []).append(((k, c), img, bxs, bb))
        batch = [launch(items, (di, bi & 1, gi)) for gi, items in enumerate(by_shape.values())]
        ev = torch.cuda.Event()
        ev.record(cs)
        if pending is not None:
            finish(*pending)
        pending = (batch, ev)
    if pending is not None:
        finish(*pending)
    return raw, id_raw


class CameraRows:
    """One camera's alldata rows (step1:345-375) as arrays: per kept frame ``nrows[f]`` rows; per row the
    track id, the int box (as float), the smoothed keypoints (J, 3) [x, y, score], the assigned ID and its
    score.  ``rows()`` gives the reference's nested lists (what json.dump writes), ``json_text()`` the file
    text (libmq_hip's formatter, byte for byte json.dumps of those lists, run without the interpreter lock)."""

    def __init__(self, nrows, tid, box, kp, assigned, score, fnums):
        self.nrows = np.asarray(nrows, dtype=np.int32)
        self.tid = np.asarray(tid, dtype=np.int64)
        self.box = np.asarray(box, dtype=np.float64).reshape(-1, 4)
        self.kp = np.asarray(kp, dtype=np.float64)
        self.assigned = np.asarray(assigned, dtype=np.int64)
        self.score = np.asarray(score, dtype=np.float64)
        self.fnums = list(fnums)
        self.offsets = np.concatenate([[0], np.cumsum(self.nrows)]).astype(np.int64)

    def __len__(self):
        return len(self.nrows)

    def frame(self, f):
        """(first row, row count) of kept frame f."""
        return int(self.offsets[f]), int(self.nrows[f])

    def track_ids(self):
        t = self.tid.tolist()
        return [t[self.offsets[f]:self.offsets[f + 1]] for f in range(len(self.nrows))]

    def rows(self):
        tid, box, kp = self.tid.tolist(), self.box.tolist(), self.kp.tolist()
        assigned, score = self.assigned.tolist(), self.score.tolist()
        out = []
        for f in range(len(self.nrows)):
            a, b = self.offsets[f], self.offsets[f + 1]
            out.append([[tid[r]] + box[r] + [kp[r], assigned[r], score[r]] for r in range(a, b)])
        return out

    def json_text(self):
        import ctypes
        from mqhip import _lib
        try:
            lib = _lib.load()
        except _lib.MqError:  # no library: the Python encoder (same text)
            return json.dumps(self.rows())
        J = self.kp.shape[1] if self.kp.ndim == 3 and len(self.kp) else 17
        cap = len(self.tid) * ((5 + 3 * J) * 26 + 64) + len(self.nrows) * 4 + 16
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_int64()
        c = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        arrs = [np.ascontiguousarray(x) for x in (self.nrows, self.tid, self.box, self.kp, self.assigned, self.score)]
        _lib.check(lib.mq_alldata_json(len(self.nrows), c(arrs[0]), c(arrs[1]), c(arrs[2]), c(arrs[3]), J, c(arrs[4]),
                                       c(arrs[5]), buf, cap, ctypes.byref(n)), "mq_alldata_json")
        return buf.raw[:n.value].decode()


def assemble_records(stores, T, plans, jobs, raw, kp_params=KP_PARAMS, id_raw=None, cams=None):
    """KP_THR, the recursive per-track EMA and the alldata rows (step1:300-370), per camera in time order,
    from the pose results of ``run_pose``, as ``CameraRows`` (after the reference's "valid frames only"
    filter).  ``cams``: only these cameras (the EMA state is per camera, so a subset gives the same rows;
    ``raw`` needs entries for them only); the result is aligned with ``cams``."""
    cams = list(range(len(stores))) if cams is None else list(cams)
    job_at = {(k, j[0]): j for k, js in jobs.items() for j in js}
    thr = kp_params["id_conf_thr"]
    # one smoother for the cameras, keyed (camera, track): the cameras' EMA states are independent, and every
    # time step's boxes of all cameras go through ONE vectorised update (same element-wise arithmetic)
    smoother = KeypointSmoother(kp_params)
    frames = {c: [] for c in cams}       # per camera, per time step: (tid, box, kp, assigned, score) arrays
    fnums = {c: [] for c in cams}
    empty = None
    for k in range(len(T)):
        batch = []
        for c in cams:
            fn, rep = plans[c][k]
            fnums[c].append(fn)
            job = job_at.get((k, c))
            if rep:
                frames[c].append(frames[c][-1] if frames[c] else empty)
            elif job is None:  # no tracks / only degenerate boxes in this frame (step1:229-265)
                frames[c].append(empty)
            else:
                batch.append((c, fn, job))
                frames[c].append(None)
        if not batch:
            continue
        keys, kps, scs = [], [], []
        for c, fn, (_, _, boxes, tids, _) in batch:
            kp, sc = raw[(k, c)]
            keys += [(c, int(t)) for t in tids[:len(kp)]]
            kps.append(np.asarray(kp, dtype=np.float64))
            scs.append(np.asarray(sc, dtype=np.float32))
        sm = smoother.update_many(keys, k, np.concatenate(kps), np.concatenate(scs))
        o = 0
        for (c, fn, (_, _, boxes, tids, _)), kp in zip(batch, kps):
            n = len(kp)
            ids = id_raw[(k, c)] if id_raw is not None else stores[c].id_preds_of(fn)
            if ids is None:
                lab, scr = np.full(n, -1, np.int64), np.zeros(n)
            else:
                lab = np.array([int(ids[i]["pred_label"]) for i in range(n)], dtype=np.int64)
                scr = np.array([float(ids[i]["pred_score"]) for i in range(n)], dtype=np.float64)
            frames[c][-1] = (np.asarray(tids[:n], dtype=np.int64), np.asarray(boxes[:n], dtype=np.float64),
                             sm[o:o + n], np.where(scr >= thr, lab, -1), scr)
            o += n
    out = []
    J = None
    for c in cams:
        valid = set(int(x) for x in stores[c].get_frame_metadata()["frame_number"])  # "valid frames only" (:364-370)
        keep = [(fr, f) for fr, f in zip(frames[c], fnums[c]) if f in valid]
        parts = [fr for fr, _ in keep if fr is not None]
        if J is None:
            J = next((p[2].shape[1] for ps in frames.values() for p in ps if p is not None), 17)
        out.append(CameraRows(
            [0 if fr is None else len(fr[0]) for fr, _ in keep],
            np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.int64),
            np.concatenate([p[1] for p in parts]) if parts else np.zeros((0, 4)),
            np.concatenate([p[2] for p in parts]) if parts else np.zeros((0, J, 3)),
            np.concatenate([p[3] for p in parts]) if parts else np.zeros(0, np.int64),
            np.concatenate([p[4] for p in parts]) if parts else np.zeros(0),
            [f for _, f in keep]))
    return out


def assemble_rows(stores, T, plans, jobs, raw, kp_params=KP_PARAMS, id_raw=None, cams=None):
    """``assemble_records`` as the reference's nested row lists: per camera (rows per kept frame, frame
    numbers)."""
    return [(cr.rows(), cr.fnums) for cr in assemble_records(stores, T, plans, jobs, raw, kp_params, id_raw, cams)]


def kept_track_ids(stores, T, plans, jobs):
    """Per camera, per kept frame of ``assemble_rows``, the track ids of its rows -- from the frame plan
    alone (no pose results): what step 3's known assignment needs from the cameras a rank does not
    assemble itself."""
    out = []
    for c, st in enumerate(stores):
        ids, fnums = [], []
        for k in range(len(T)):
            fn, rep = plans[c][k]
            job = next((j for j in jobs.get(k, ()) if j[0] == c), None)
            if rep:
                ids.append(ids[-1] if ids else [])
            elif job is None:
                ids.append([])
            else:
                ids.append([int(t) for t in job[3]])
            fnums.append(fn)
        valid = set(int(x) for x in st.get_frame_metadata()["frame_number"])
        out.append([i for i, f in zip(ids, fnums) if f in valid])
    return out


def process_stores(pose_model, stores, T, kp_params=KP_PARAMS, steps_per_batch=8, id_model=None, tracks=None,
                   records=False):
    """Pose half of step1_proc2d_custom / process_single_cam (step1_proc2d.py:166-447) for every
    camera at once.  Per camera the reference's time-grid walk, degenerate-box filter, margin
    expansion, KP_THR and recursive EMA are kept exactly (the EMA state is per camera and runs in
    time order); the ViTPose work of ``steps_per_batch`` time steps x all cameras goes through ONE
    batched crop -> ViT -> decode launch sequence (the reference: one inference_topdown per camera
    frame).  With ``id_model`` the tracked boxes are classified on the GPU the same way (else the stores'
    ID predictions, if any).  Returns per camera (alldata rows per kept frame, frame numbers)."""
    plans, jobs = plan_jobs(stores, T, kp_params, tracks)
    raw, id_raw = run_pose_id(pose_model, id_model, stores, jobs, range(len(T)), steps_per_batch)
    if records:  # CameraRows per camera (arrays) instead of (rows, frame numbers)
        return assemble_records(stores, T, plans, jobs, raw, kp_params, id_raw)
    return assemble_rows(stores, T, plans, jobs, raw, kp_params, id_raw)


class Step1Output:
    """What step 1 computed in this call, for steps 3-4 in memory (run_demo): per processed camera (store
    index) its alldata rows as ``CameraRows`` -- on a sharded rank only the cameras it owns
    (``mqhip.shard.camera_shard``) -- and every camera's kept-frame track ids; ``wait()`` joins the
    background writer of the alldata.json / frame_num.npy files."""

    def __init__(self, names, todo, rows, fnums, ids, writer):
        self.names = names            # camera id (results sub-directory) per store, in store order
        self.todo = todo              # store indices processed in this call
        self.rows = rows              # {store index: CameraRows}
        self.fnums = fnums            # {store index: kept frame numbers}
        self.ids = ids                # per store (every camera): per kept frame, the rows' track ids
        self._writer = writer

    @property
    def complete(self):
        return len(self.todo) == len(self.names)

    def wait(self):
        if self._writer is not None:
            self._writer.join()
            self._writer = None
        err = getattr(self, "_error", None)
        if err is not None:
            self._error = None
            raise err


def _write_step1_files(out_dirs, items, into):
    try:
        for i, rec in items:
            os.makedirs(out_dirs[i], exist_ok=True)
            np.save(Path(out_dirs[i]) / "frame_num.npy", np.array(rec.fnums, dtype=np.int32))
            with open(Path(out_dirs[i]) / "alldata.json", "w") as fp:
                fp.write(rec.json_text())  # json.dumps' text of the rows, formatted natively (GIL released)
    except BaseException as e:  # re-raised by Step1Output.wait()
        into._error = e


def step1_proc2d_custom(data_name, results_root, raw_root, fps=24.0, t_intv=None, redo=False, pose_model=None,
                        device_str="cuda:0", steps_per_batch=8, id_model=None, detector=None, world=1, rank=0,
                        group=None, sharded=False, gather_device=None, background_writes=False, timings=None):
    """step1_proc2d.py:389-447 with the frame stores of ``mqhip.io.FrameStore`` and the tracker
    rows they carry (or, with ``detector``, the detector -> tracker chain).  ``id_model``: see
    ``resolve_id_models`` ("auto" = the reference's per-camera variant).  Writes
    <results_root>/<data_name>/<cam>/alldata.json and frame_num.npy, and returns a ``Step1Output``
    (None when every camera was already done).

    Multi-GPU (BASELINE config 3; ``world`` > 1, or ``sharded`` at world 1): every rank calls this with
    its ``rank``; the clip's time steps are sharded over the ranks (``mqhip.shard.pose_clip_sharded``:
    one all-gather of the raw keypoints over ``group``, buffers on ``gather_device`` -- the rank's GPU for
    RCCL, None for gloo); then rank r post-processes (KP_THR / EMA) and writes the cameras
    c = r (mod world) only.  The files equal the single-process ones bit for bit.
    ``background_writes``: the files are written by a thread (``Step1Output.wait()`` joins it) while the
    caller goes on with the rows in memory."""
    import glob
    import threading
    from mqhip.io import FrameStore
    meta_paths = sorted(glob.glob(os.path.join(raw_root, f"{data_name}.*", "metadata.yaml")))
    if not meta_paths:
        raise FileNotFoundError(f'No imgstore metadata for "{data_name}" in {raw_root}')
    stores = [FrameStore(os.path.dirname(p)) for p in meta_paths]
    md0 = stores[0].get_frame_metadata()
    t0 = md0["frame_time"][0]
    if t_intv is None:
        t_start, t_end = t0, md0["frame_time"][-1]
    else:
        t_start, t_end = t0 + t_intv[0], t0 + t_intv[1]
    T = np.arange(t_start, t_end, 1.0 / fps)
    suffix = "" if t_intv is None else f".{int(t_intv[0]):04d}-{int(t_intv[1]):04d}"
    names = [os.path.basename(st.filename).split(".")[-1] for st in stores]
    out_dirs = [os.path.join(results_root, data_name + suffix, n) for n in names]
    todo = [i for i, d in enumerate(out_dirs)
            if redo or not (os.path.exists(os.path.join(d, "alldata.json"))
                            and os.path.exists(os.path.join(d, "frame_num.npy")))]
    if not todo:
        return None
    if pose_model is None:
        pose_model = init_pose_model(device=device_str)
    sel = [stores[i] for i in todo]
    tracks = None if detector is None else track_stores(detector, sel, T)
    id_models = resolve_id_models(sel, id_model, device_str)
    ids_sel = None
    if world > 1 or sharded:
        from mqhip.shard import camera_shard, pose_clip_sharded
        own = camera_shard(len(sel), world, rank)
        res, ids_sel = pose_clip_sharded(pose_model, sel, T, world, rank, group=group,
                                         steps_per_batch=steps_per_batch, device=gather_device, id_model=id_models,
                                         tracks=tracks, cams=own, with_ids=True, timings=timings, records=True)
        done = [todo[j] for j in own]
    else:
        res = process_stores(pose_model, sel, T, steps_per_batch=steps_per_batch, id_model=id_models, tracks=tracks,
                             records=True)
        done = list(todo)
    items = list(zip(done, res))
    out = Step1Output(names, todo, {i: r for i, r in items}, {i: r.fnums for i, r in items}, None, None)
    if ids_sel is None:
        ids_sel = [out.rows[i].track_ids() for i in todo]
    out.ids = [None] * len(stores)
    for j, i in enumerate(todo):
        out.ids[i] = ids_sel[j]
    if background_writes:
        out._writer = threading.Thread(target=_write_step1_files, args=(out_dirs, items, out), daemon=False)
        out._writer.start()
    else:
        _write_step1_files(out_dirs, items, out)
        out.wait()
    return out


def proc(data_name, results_root, raw_root, device_str="cuda:0", fps=24.0, pose_model=None, detector=None,
         id_model="auto", **shard):
    """step1.proc (step1_proc2d.py:450) over every camera's frame store: pose and ID on the stores' tracker
    rows, or the full detector -> tracker -> pose -> ID chain with ``detector``.  ``id_model="auto"`` is the
    reference's rule (every camera classified by the ID model of its variant, step1:424-427); None keeps
    the stores' own ID predictions (``resolve_id_models``).  Unlike the reference (which hard-codes cuda:1,
    step1:50,421) the device argument is honoured."""
    return step1_proc2d_custom(data_name, results_root, raw_root, fps=fps, pose_model=pose_model,
                               device_str=device_str, detector=detector, id_model=id_model, **shard)
