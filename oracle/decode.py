"""ORACLE (test infrastructure only): UDP heatmap decode with DARK-UDP refinement.

Restates mmpose 1.3.2 (not installed here; the reference selects it via
``model/pose/td-hm_ViTPose-huge_8xb64-210e_coco-256x192_sn_macaque.py``:4-14, 85-110):

* ``flip_heatmaps(flip_mode='heatmap', shift_heatmap=False)`` + ``(H + H_flip) * 0.5``
  (``TopdownPoseEstimator`` flip test, config :109, ``step1_proc2d.py``:101),
* ``UDPHeatmap.decode`` -> ``get_heatmap_maximum`` + ``refine_keypoints_dark_udp``
  (blur_kernel_size 11) -> ``kp / (W-1, H-1) * input_size``,
* ``TopdownPoseEstimator.add_pred_to_datasample``:
  ``kp / input_size * input_scale + input_center - 0.5 * input_scale``.

Precision is kept exactly as in mmpose: blur / log / derivatives in float32, the
Hessian gets ``np.finfo(np.float32).eps * np.eye(2)`` (float64), so the 2x2 inverse
and the Newton step are float64 and stored back to float32.  The 11x11 Gaussian
(cv2.GaussianBlur, sigma 0 -> 2.0) is restated as a separable float32 filter with
the kernel computed in float64 and rounded to float32 (OpenCV's getGaussianKernel),
taps accumulated in ascending order, rows first (parity vs cv2 unpinned).
Low-confidence joints (val <= 0) keep loc -1 and still receive a Newton step read
through numpy's negative-index wrap-around of the flattened padded maps; that is
reproduced here (and in the HIP kernel).
"""
from __future__ import annotations

import numpy as np

FLIP_INDICES = [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15]


def flip_average(h, h_flip_raw, flip_indices=FLIP_INDICES):
    """(N,K,H,W) float32 heatmaps of the plain and the flipped forward -> averaged."""
    hf = h_flip_raw[:, :, :, ::-1][:, flip_indices]
    return ((h + hf) * np.float32(0.5)).astype(np.float32)


def gaussian_kernel_1d(ksize=11, sigma=0.0):
    """cv2.getGaussianKernel(ksize, sigma<=0 -> 0.3*((ksize-1)*0.5-1)+0.8), float64 -> float32."""
    if sigma <= 0:
        sigma = ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8
    scale2 = -0.5 / (sigma * sigma)
    k = np.empty(ksize, dtype=np.float64)
    s = 0.0
    for i in range(ksize):
        x = i - (ksize - 1) * 0.5
        t = np.exp(scale2 * x * x)
        k[i] = t
        s += t
    s = 1.0 / s
    return (k * s).astype(np.float32)


def gaussian_blur(heatmaps, kernel=11):
    """mmpose ``gaussian_blur``: zero-pad by (k-1)/2, blur, crop, rescale to the old max."""
    K, H, W = heatmaps.shape
    b = (kernel - 1) // 2
    g = gaussian_kernel_1d(kernel)
    out = heatmaps.copy()
    for k in range(K):
        origin_max = np.max(heatmaps[k])
        dr = np.zeros((H + 2 * b, W + 2 * b), dtype=np.float32)
        dr[b:-b, b:-b] = heatmaps[k]
        # rows (horizontal taps), only the rows that feed the kept window are needed
        rows = np.zeros((H + 2 * b, W), dtype=np.float32)
        acc = g[0] * dr[:, 0:W]
        for t in range(1, kernel):
            acc = (acc + g[t] * dr[:, t:t + W]).astype(np.float32)
        rows[:] = acc
        acc = g[0] * rows[0:H, :]
        for t in range(1, kernel):
            acc = (acc + g[t] * rows[t:t + H, :]).astype(np.float32)
        blurred = acc.astype(np.float32)
        ratio = np.float32(origin_max / np.max(blurred))
        out[k] = (blurred * ratio).astype(np.float32)
    return out


def get_heatmap_maximum(heatmaps):
    """mmpose ``get_heatmap_maximum`` for (K,H,W): first max of the flattened map."""
    K, H, W = heatmaps.shape
    flat = heatmaps.reshape(K, -1)
    idx = np.argmax(flat, axis=1)
    y, x = np.unravel_index(idx, (H, W))
    locs = np.stack((x, y), axis=-1).astype(np.float32)
    vals = np.amax(flat, axis=1)
    locs[vals <= 0.] = -1
    return locs, vals, idx.astype(np.int32)


def refine_keypoints_dark_udp(keypoints, heatmaps, blur_kernel_size=11):
    """mmpose ``refine_keypoints_dark_udp`` for one instance (keypoints (1,K,2) float32)."""
    N, K = keypoints.shape[:2]
    H, W = heatmaps.shape[1:]
    hm = gaussian_blur(heatmaps, blur_kernel_size)
    np.clip(hm, 1e-3, 50., hm)
    np.log(hm, hm)
    pad = np.pad(hm, ((0, 0), (1, 1), (1, 1)), mode='edge').flatten()
    for n in range(N):
        index = keypoints[n, :, 0] + 1 + (keypoints[n, :, 1] + 1) * (W + 2)
        index += (W + 2) * (H + 2) * np.arange(0, K)
        index = index.astype(int).reshape(-1, 1)
        i_ = pad[index]
        ix1 = pad[index + 1]
        iy1 = pad[index + W + 2]
        ix1y1 = pad[index + W + 3]
        ix1_y1_ = pad[index - W - 3]
        ix1_ = pad[index - 1]
        iy1_ = pad[index - 2 - W]
        dx = 0.5 * (ix1 - ix1_)
        dy = 0.5 * (iy1 - iy1_)
        derivative = np.concatenate([dx, dy], axis=1).reshape(K, 2, 1)
        dxx = ix1 - 2 * i_ + ix1_
        dxy = 0.5 * (ix1y1 - ix1 - iy1 + i_ + i_ - ix1_ - iy1_ + ix1_y1_)
        dyy = iy1 - 2 * i_ + iy1_
        hessian = np.concatenate([dxx, dxy, dxy, dyy], axis=1).reshape(K, 2, 2)
        hessian = np.linalg.inv(hessian + np.finfo(np.float32).eps * np.eye(2))
        keypoints[n] -= np.einsum('imn,ink->imk', hessian, derivative).squeeze()
    return keypoints


def udp_decode(heatmaps, input_size=(192, 256), blur_kernel_size=11):
    """UDPHeatmap.decode for one instance: (K,H,W) float32 -> kp (1,K,2) float64 input
    space (``keypoints / [W-1, H-1] * input_size`` promotes to float64), scores (1,K) f32."""
    K, H, W = heatmaps.shape
    hm = heatmaps.copy()
    locs, vals, idx = get_heatmap_maximum(hm)
    kp = locs[None].copy()
    kp = refine_keypoints_dark_udp(kp, hm, blur_kernel_size)
    kp = kp / np.array([W - 1, H - 1]) * np.array(input_size)
    return kp, vals[None].astype(np.float32), idx


def to_image_space(kp_input, input_center, input_scale, input_size=(192, 256)):
    """add_pred_to_datasample (float64 like mmpose):
    ``kp / input_size * input_scale + input_center - 0.5 * input_scale``."""
    c = np.asarray(input_center, dtype=np.float32)
    s = np.asarray(input_scale, dtype=np.float32)
    half = (np.float32(0.5) * s).astype(np.float32)
    return kp_input / np.array(input_size) * s + c - half


def decode_batch(heatmaps, centers, scales, input_size=(192, 256)):
    """(N,K,H,W) averaged heatmaps -> image-space kp (N,K,2) f64, scores (N,K) f32, argmax (N,K)."""
    N = heatmaps.shape[0]
    kps, scs, idxs = [], [], []
    for n in range(N):
        kp, sc, idx = udp_decode(heatmaps[n], input_size)
        kps.append(to_image_space(kp[0], centers[n], scales[n], input_size))
        scs.append(sc[0])
        idxs.append(idx)
    return np.stack(kps), np.stack(scs), np.stack(idxs)
