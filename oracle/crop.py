"""ORACLE (test infrastructure only): top-down crop of a detection.

Restates, for ``mmpose.apis.inference_topdown`` with the test pipeline of
``model/pose/td-hm_ViTPose-huge_8xb64-210e_coco-256x192_sn_macaque.py``:151-159:

* ``GetBBoxCenterScale(padding=1.25)`` -> ``bbox_xyxy2cs`` (float32),
* ``TopdownAffine(input_size=(192,256), use_udp=True)``: ``_fix_aspect_ratio`` then
  ``get_udp_warp_matrix`` (numpy 1.x scalar promotion: the scalar parts are float64,
  the matrix is stored float32) and ``cv2.warpAffine(INTER_LINEAR, BORDER_CONSTANT 0)``,
* ``PoseDataPreprocessor``: bgr->rgb, ``(x - mean) / std`` in float32 (config :72-84).

cv2.warpAffine on uint8 is restated as OpenCV's fixed-point path: the 2x3 matrix
is inverted in double, source coordinates are formed with AB_BITS=10 and rounded
half-to-even (cvRound), INTER_BITS=5 sub-pixel phases, 15-bit bilinear weights
(INTER_REMAP_COEF_SCALE = 32768; exact for the linear table), out-of-image taps 0,
``(sum + 16384) >> 15``.  Integer-exact; parity vs the real cv2 build unpinned.
"""
from __future__ import annotations

import numpy as np

INPUT_W, INPUT_H = 192, 256
MEAN = np.array([123.675, 116.28, 103.53], dtype=np.float32)
STD = np.array([58.395, 57.12, 57.375], dtype=np.float32)


def bbox_xyxy2cs(bbox, padding=1.25):
    bbox = np.asarray(bbox, dtype=np.float32).reshape(-1, 4)
    scale = ((bbox[:, 2:] - bbox[:, :2]) * np.float32(padding)).astype(np.float32)
    center = ((bbox[:, 2:] + bbox[:, :2]) * np.float32(0.5)).astype(np.float32)
    return center, scale


def fix_aspect_ratio(scale, aspect_ratio=INPUT_W / INPUT_H):
    w = scale[:, 0:1]
    h = scale[:, 1:2]
    ar = np.float32(aspect_ratio)
    return np.where(w > h * ar, np.hstack([w, w / ar]), np.hstack([h * ar, h])).astype(np.float32)


def udp_warp_matrix(center, scale, output_size=(INPUT_W, INPUT_H)):
    """mmpose get_udp_warp_matrix with rot = 0 (numpy 1.x scalar promotion)."""
    c0, c1 = float(np.float32(center[0])), float(np.float32(center[1]))
    s0, s1 = float(np.float32(scale[0])), float(np.float32(scale[1]))
    in0, in1 = float(np.float32(c0 * 2)), float(np.float32(c1 * 2))
    sx = (output_size[0] - 1) / s0
    sy = (output_size[1] - 1) / s1
    m = np.zeros((2, 3), dtype=np.float32)
    m[0, 0] = 1.0 * sx
    m[0, 1] = -0.0 * sx
    m[0, 2] = sx * (-0.5 * in0 * 1.0 + 0.5 * in1 * 0.0 + 0.5 * s0)
    m[1, 0] = 0.0 * sy
    m[1, 1] = 1.0 * sy
    m[1, 2] = sy * (-0.5 * in0 * 0.0 - 0.5 * in1 * 1.0 + 0.5 * s1)
    return m


def invert_affine(m32):
    M = m32.astype(np.float64).ravel().copy()
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11 = M[4] * D
    A22 = M[0] * D
    M[0] = A11
    M[1] *= -D
    M[3] *= -D
    M[4] = A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2] = b1
    M[5] = b2
    return M


def warp_affine_linear_u8(img, m32, out_w=INPUT_W, out_h=INPUT_H):
    """cv2.warpAffine(img u8 HxWx3, m32, (out_w,out_h), INTER_LINEAR, BORDER_CONSTANT=0)."""
    H, W, C = img.shape
    M = invert_affine(m32)
    xs = np.arange(out_w, dtype=np.float64)
    ys = np.arange(out_h, dtype=np.float64)
    adelta = np.rint(M[0] * xs * 1024.0).astype(np.int64)
    bdelta = np.rint(M[3] * xs * 1024.0).astype(np.int64)
    X0 = np.rint((M[1] * ys + M[2]) * 1024.0).astype(np.int64) + 16
    Y0 = np.rint((M[4] * ys + M[5]) * 1024.0).astype(np.int64) + 16
    X = (X0[:, None] + adelta[None, :]) >> 5
    Y = (Y0[:, None] + bdelta[None, :]) >> 5
    sx = X >> 5
    sy = Y >> 5
    fx = X & 31
    fy = Y & 31
    w00 = (32 - fy) * (32 - fx) * 32
    w01 = (32 - fy) * fx * 32
    w10 = fy * (32 - fx) * 32
    w11 = fy * fx * 32
    src = img.astype(np.int64)

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = src[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]
        return np.where(ok[..., None], v, 0)

    s = (tap(sy, sx) * w00[..., None] + tap(sy, sx + 1) * w01[..., None]
         + tap(sy + 1, sx) * w10[..., None] + tap(sy + 1, sx + 1) * w11[..., None])
    out = (s + 16384) >> 15
    return np.clip(out, 0, 255).astype(np.uint8)


def topdown_crop(img, bbox_xyxy):
    """One detection -> (crop u8 256x192x3 BGR, input_center f32 (2,), input_scale f32 (2,))."""
    center, scale = bbox_xyxy2cs(np.asarray(bbox_xyxy, dtype=np.float32)[None])
    scale = fix_aspect_ratio(scale)
    c, s = center[0], scale[0]
    m = udp_warp_matrix(c, s)
    return warp_affine_linear_u8(img, m), c, s


def preprocess(crop_bgr_u8):
    """PoseDataPreprocessor: HWC BGR u8 -> CHW RGB float32 normalised."""
    x = crop_bgr_u8[:, :, ::-1].astype(np.float32).transpose(2, 0, 1)
    return ((x - MEAN[:, None, None]) / STD[:, None, None]).astype(np.float32)
