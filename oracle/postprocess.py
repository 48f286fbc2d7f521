"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the step-1 host logic around the pose model.

Rows a1 (box expansion, step1_proc2d.py:270-292, constants :67-73) and a10
(keypoint threshold + recursive EMA, :300-343, frame row layout :353-362),
written as plain per-box Python loops so the product's vectorised version
(src/pipeline/step1_proc2d.py) can be checked against it.  Never imported by the
product path.
"""
from collections import deque

import numpy as np

KP_THR = 0.30
EMA_ALPHA = 0.50
DISP_THR = 20.0
MIN_MARGIN = 0.20
MAX_MARGIN = 0.50
DESIRED_AR = 192.0 / 256.0
ID_CONF_THR = 0.80


def filter_tracks(tracks):
    """step1_proc2d.py:255-268: int-truncate, keep boxes with positive extent."""
    boxes, tids = [], []
    for row in tracks:
        x1, y1, x2, y2 = (int(v) for v in row[:4])
        if x2 > x1 and y2 > y1:
            boxes.append((x1, y1, x2, y2))
            tids.append(int(row[4]))
    return np.array(boxes, dtype=np.int32).reshape(-1, 4), np.array(tids, dtype=np.int32)


def expand_boxes(boxes):
    """step1_proc2d.py:270-292 (+ :286-292 back to xyxy); float64 host math, float32 storage
    (numpy 1.x promotes np.float32 scalar (op) python float to float64)."""
    xywh = []
    for (x1, y1, x2, y2) in boxes:
        w, h = float(x2 - x1), float(y2 - y1)
        cx, cy = x1 + 0.5 * w, y1 + 0.5 * h
        frac = min(max((h - 50.0) / (200.0 - 50.0), 0.0), 1.0)
        m = MAX_MARGIN - (MAX_MARGIN - MIN_MARGIN) * frac
        wn, hn = w * (1 + m), h * (1 + m)
        ar = wn / hn
        if abs(ar - DESIRED_AR) > 0.20:
            if ar < DESIRED_AR:
                wn = hn * DESIRED_AR
            else:
                hn = wn / DESIRED_AR
        xywh.append([cx, cy, wn, hn])
    xywh = np.array(xywh, dtype=np.float32).reshape(-1, 4)
    out = []
    for cx, cy, w, h in xywh:
        cx, cy, w, h = float(cx), float(cy), float(w), float(h)
        out.append([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h])
    return np.array(out, dtype=np.float32).reshape(-1, 4)


class Smoother:
    """step1_proc2d.py:314-343: per-track deque(5) holding the SMOOTHED previous value."""

    def __init__(self):
        self.buf = {}

    def update(self, tid, frame_number, kpt_xy, kpt_score):
        kpt_xy = np.array(kpt_xy, dtype=np.float64, copy=True)
        kpt_score = np.array(kpt_score, dtype=np.float32, copy=True)
        for j in range(len(kpt_score)):
            if kpt_score[j] < KP_THR:
                kpt_xy[j, :] = np.nan
                kpt_score[j] = 0.0
        kp = np.concatenate([kpt_xy, kpt_score.reshape(-1, 1)], axis=1)
        b = self.buf.setdefault(tid, deque(maxlen=5))
        b.append((frame_number, kp.copy()))
        if len(b) >= 2:
            (_, prev), (fc, cur) = b[-2], b[-1]
            for j in range(prev.shape[0]):
                if np.isnan(prev[j, 0]) or np.isnan(cur[j, 0]):
                    continue
                d = np.float32(np.sqrt((cur[j, 0] - prev[j, 0]) ** 2 + (cur[j, 1] - prev[j, 1]) ** 2))
                if d < DISP_THR:
                    cur[j, :2] = EMA_ALPHA * prev[j, :2] + (1 - EMA_ALPHA) * cur[j, :2]
            b[-1] = (fc, cur)
        return b[-1][1]


def frame_rows(kps, scores, boxes, tids, smoother, frame_number, id_label=None, id_score=None):
    """Rows [tid, x1, y1, x2, y2, [[x, y, s] x J], assigned_id, id_score] (step1:345-362)."""
    rows = []
    for i in range(len(tids)):
        sm = smoother.update(int(tids[i]), frame_number, kps[i], scores[i])
        lab = -1 if id_label is None else int(id_label[i])
        sc = 0.0 if id_score is None else float(id_score[i])
        assigned = lab if sc >= ID_CONF_THR else -1
        x1, y1, x2, y2 = boxes[i]
        rows.append([int(tids[i]), float(x1), float(y1), float(x2), float(y2),
                     [[float(x), float(y), float(s)] for (x, y, s) in sm], assigned, sc])
    return rows
