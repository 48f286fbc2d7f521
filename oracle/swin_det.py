"""ORACLE (test infrastructure only): float32 PyTorch restatement of the step-1 detector,
Swin-S Mask R-CNN (bbox only), as configured by
``/root/reference/model/detection/SWIN-Mask_R-CNN_bbox_only.py``:29-226 and called by
``src/pipeline/step1_proc2d.py``:98,104-109,226-237 (mmdet==3.2.0, mmcv==2.1.0; absent here, so
the semantics below are restated from their published algorithms and **parity is unpinned**
against them):

* test pipeline (step1:104-109): ``Resize(scale=(800, 800), keep_ratio=True)`` = mmcv
  ``imrescale`` -> ``cv2.resize(INTER_LINEAR)`` on the uint8 BGR frame (restated: OpenCV's fixed-point
  bilinear, 11-bit coefficients, the 8-bit vertical pass of ``VResizeLinearVec_32s8u``);
* ``DetDataPreprocessor`` (config :61-77): BGR->RGB, (x - mean) / std, zero pad to a multiple of 32;
* ``SwinTransformer`` (config :29-60): patch 4 + LN, depths [2, 2, 18, 2], heads [3, 6, 12, 24],
  window 7, shifted windows on odd blocks (torch.roll, zero pad after norm1, -100 mask),
  relative position bias, qkv bias, MLP ratio 4 (exact GELU), PatchMerging (nn.Unfold 2x2 order,
  LN(4C), Linear 4C->2C without bias), LN on every output stage;
* ``FPN`` (:78-87): 1x1 laterals, nearest top-down, 3x3 outputs, P6 = max_pool(k1, s2);
* ``RPNHead`` (:163-199, test_cfg :208-213): 3x3 conv + ReLU, 3 anchors (ratios 0.5/1/2, scale 8,
  strides 4..64), sigmoid, top 1000 per level, delta2bbox (stds 1, wh clamp log(1000/16)), clip,
  w,h > 0, NMS 0.7 per level (batched_nms offsets), top 1000;
* ``StandardRoIHead`` (:88-162, test_cfg :201-207): RoIAlign 7x7 (sampling 0 = adaptive,
  aligned=True) on the level of ``map_roi_levels`` (finest_scale 56), Shared2FC (1024, ReLU), softmax,
  delta2bbox (stds 0.1/0.1/0.2/0.2), rescale by 1/scale_factor, score_thr 0.05, NMS 0.5, top 100.

Weights are seeded random (``make_weights``) under the mmdet state_dict key names.  Never
imported by the product path.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

MEAN = (123.675, 116.28, 103.53)
STD = (58.395, 57.12, 57.375)
SWIN_S = dict(embed=96, depths=(2, 2, 18, 2), heads=(3, 6, 12, 24), window=7, mlp_ratio=4)
FPN_OUT = 256
ANCHOR_RATIOS = (0.5, 1.0, 2.0)
ANCHOR_SCALE = 8
STRIDES = (4, 8, 16, 32, 64)
RPN_NMS_PRE, RPN_MAX, RPN_IOU = 1000, 1000, 0.7
RCNN_SCORE_THR, RCNN_IOU, RCNN_MAX = 0.05, 0.5, 100
FC_OUT = 1024
NUM_CLASSES = 1
WH_RATIO_CLIP = 16 / 1000
RPN_CLS_STD = 0.02   # random-weight scales that spread the logits (no tied scores)
FC_CLS_STD = 0.05


# ----------------------------------------------------------------------------- resize (cv2)

def rescale_size(w, h, scale=(800, 800)):
    """mmcv rescale_size for keep_ratio: the largest factor that fits both edges."""
    long_e, short_e = max(scale), min(scale)
    f = min(long_e / max(h, w), short_e / min(h, w))
    return int(w * f + 0.5), int(h * f + 0.5), f


def _linear_coeffs(dst, src):
    """cv::resize INTER_LINEAR coefficient tables: source index and 11-bit weights per output."""
    scale = 1.0 / (dst / src)  # resize.cpp: scale_x = 1. / inv_scale_x, inv_scale_x = dsize.width / ssize.width
    ofs = np.zeros(dst, np.int64)
    a = np.zeros((dst, 2), np.int64)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0), 0
        if s >= src - 1:
            f, s = np.float32(0), src - 1
        c0 = np.float32(1.0) - f
        # saturate_cast<short>(float) rounds half to even
        a[d, 0] = int(np.rint(np.float32(c0 * np.float32(2048))))
        a[d, 1] = int(np.rint(np.float32(f * np.float32(2048))))
        ofs[d] = s
    return ofs, a


def resize_linear_u8(img, new_w, new_h):
    """cv2.resize(img, (new_w, new_h), INTER_LINEAR) for uint8 HxWx3 (OpenCV native fixed point:
    integer horizontal pass, vertical pass ((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16), +2 >> 2; an exact
    2x downscale is INTER_AREA).  The vertical rounding is the SIMD kernel's (VResizeLinearVec_32s8u);
    OpenCV's scalar tail, (S0*b0 + S1*b1 + 2^21) >> 22, can differ by one in the last pixels of a row:
    parity with cv2 itself is unpinned (cv2 is absent here)."""
    H, W, C = img.shape
    if W == 2 * new_w and H == 2 * new_h:
        # resize.cpp: INTER_LINEAR with an exact 2x downscale takes the INTER_AREA fast path
        # (resizeAreaFast_: (a + b + c + d + 2) >> 2)
        s = img.astype(np.int64)
        v = s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2]
        return ((v + 2) >> 2).astype(np.uint8)
    xo, xa = _linear_coeffs(new_w, W)
    yo, ya = _linear_coeffs(new_h, H)
    src = img.astype(np.int64)
    x1 = np.minimum(xo + 1, W - 1)
    rows = src[:, xo, :] * xa[None, :, 0, None] + src[:, x1, :] * xa[None, :, 1, None]  # (H, new_w, C)
    y1 = np.minimum(yo + 1, H - 1)
    s0 = rows[yo] >> 4
    s1 = rows[y1] >> 4
    v = ((s0 * ya[:, 0, None, None]) >> 16) + ((s1 * ya[:, 1, None, None]) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def preprocess(img_bgr, scale=(800, 800), pad_divisor=32):
    """Resize + DetDataPreprocessor -> (1, 3, Hp, Wp) float32, img_shape (h, w), scale_factor (sw, sh)."""
    H, W, _ = img_bgr.shape
    nw, nh, _ = rescale_size(W, H, scale)
    r = resize_linear_u8(img_bgr, nw, nh)
    x = torch.from_numpy(r[..., ::-1].copy()).float().permute(2, 0, 1)
    x = (x - torch.tensor(MEAN).view(3, 1, 1)) / torch.tensor(STD).view(3, 1, 1)
    hp = int(math.ceil(nh / pad_divisor)) * pad_divisor
    wp = int(math.ceil(nw / pad_divisor)) * pad_divisor
    x = F.pad(x, (0, wp - nw, 0, hp - nh), value=0.0)
    return x[None], (nh, nw), (nw / W, nh / H)


# ----------------------------------------------------------------------------- weights

def make_weights(cfg=SWIN_S, seed=0, std=0.02):
    """Seeded random weights under the mmdet state_dict names (LN 1/0 perturbed, biases small)."""
    g = torch.Generator().manual_seed(seed)

    def rn(*shape, s=std):
        return (torch.randn(*shape, generator=g) * s).float()

    w = {}
    C = cfg["embed"]
    w["backbone.patch_embed.projection.weight"] = rn(C, 3, 4, 4, s=0.1)
    w["backbone.patch_embed.projection.bias"] = rn(C)
    w["backbone.patch_embed.norm.weight"] = 1 + rn(C, s=0.1)
    w["backbone.patch_embed.norm.bias"] = rn(C)
    ws = cfg["window"]
    for si, (depth, heads) in enumerate(zip(cfg["depths"], cfg["heads"])):
        Cs = C * 2 ** si
        for bi in range(depth):
            k = f"backbone.stages.{si}.blocks.{bi}."
            w[k + "norm1.weight"] = 1 + rn(Cs, s=0.1)
            w[k + "norm1.bias"] = rn(Cs)
            w[k + "attn.w_msa.relative_position_bias_table"] = rn((2 * ws - 1) ** 2, heads, s=0.5)
            w[k + "attn.w_msa.qkv.weight"] = rn(3 * Cs, Cs, s=1.0 / math.sqrt(Cs))
            w[k + "attn.w_msa.qkv.bias"] = rn(3 * Cs)
            w[k + "attn.w_msa.proj.weight"] = rn(Cs, Cs, s=0.5 / math.sqrt(Cs))
            w[k + "attn.w_msa.proj.bias"] = rn(Cs)
            w[k + "norm2.weight"] = 1 + rn(Cs, s=0.1)
            w[k + "norm2.bias"] = rn(Cs)
            w[k + "ffn.layers.0.0.weight"] = rn(4 * Cs, Cs, s=1.0 / math.sqrt(Cs))
            w[k + "ffn.layers.0.0.bias"] = rn(4 * Cs)
            w[k + "ffn.layers.1.weight"] = rn(Cs, 4 * Cs, s=0.5 / math.sqrt(4 * Cs))
            w[k + "ffn.layers.1.bias"] = rn(Cs)
        if si < 3:
            k = f"backbone.stages.{si}.downsample."
            w[k + "norm.weight"] = 1 + rn(4 * Cs, s=0.1)
            w[k + "norm.bias"] = rn(4 * Cs)
            w[k + "reduction.weight"] = rn(2 * Cs, 4 * Cs, s=1.0 / math.sqrt(4 * Cs))
        w[f"backbone.norm{si}.weight"] = 1 + rn(Cs, s=0.1)
        w[f"backbone.norm{si}.bias"] = rn(Cs)
    for i in range(4):
        cin = C * 2 ** i
        w[f"neck.lateral_convs.{i}.conv.weight"] = rn(FPN_OUT, cin, 1, 1, s=1.0 / math.sqrt(cin))
        w[f"neck.lateral_convs.{i}.conv.bias"] = rn(FPN_OUT)
        w[f"neck.fpn_convs.{i}.conv.weight"] = rn(FPN_OUT, FPN_OUT, 3, 3, s=1.0 / math.sqrt(9 * FPN_OUT))
        w[f"neck.fpn_convs.{i}.conv.bias"] = rn(FPN_OUT)
    na = len(ANCHOR_RATIOS)
    w["rpn_head.rpn_conv.weight"] = rn(FPN_OUT, FPN_OUT, 3, 3, s=1.0 / math.sqrt(9 * FPN_OUT))
    w["rpn_head.rpn_conv.bias"] = rn(FPN_OUT)
    w["rpn_head.rpn_cls.weight"] = rn(na, FPN_OUT, 1, 1, s=RPN_CLS_STD)
    w["rpn_head.rpn_cls.bias"] = rn(na)
    w["rpn_head.rpn_reg.weight"] = rn(4 * na, FPN_OUT, 1, 1, s=0.2 / math.sqrt(FPN_OUT))
    w["rpn_head.rpn_reg.bias"] = rn(4 * na)
    k = "roi_head.bbox_head."
    w[k + "shared_fcs.0.weight"] = rn(FC_OUT, FPN_OUT * 49, s=1.0 / math.sqrt(FPN_OUT * 49))
    w[k + "shared_fcs.0.bias"] = rn(FC_OUT)
    w[k + "shared_fcs.1.weight"] = rn(FC_OUT, FC_OUT, s=1.0 / math.sqrt(FC_OUT))
    w[k + "shared_fcs.1.bias"] = rn(FC_OUT)
    w[k + "fc_cls.weight"] = rn(NUM_CLASSES + 1, FC_OUT, s=FC_CLS_STD)
    w[k + "fc_cls.bias"] = rn(NUM_CLASSES + 1)
    w[k + "fc_reg.weight"] = rn(4 * NUM_CLASSES, FC_OUT, s=0.3 / math.sqrt(FC_OUT))
    w[k + "fc_reg.bias"] = rn(4 * NUM_CLASSES)
    return w


# ----------------------------------------------------------------------------- Swin

def relative_position_index(ws):
    """WindowMSA: double_step_seq(2ws-1, ws, 1, ws), index = c + c^T, flipped on dim 1."""
    seq1 = torch.arange(0, (2 * ws - 1) * ws, 2 * ws - 1)
    seq2 = torch.arange(0, ws, 1)
    c = (seq1[:, None] + seq2[None, :]).reshape(1, -1)
    idx = c + c.T
    return idx.flip(1).contiguous()


def shift_mask(Hp, Wp, ws, shift):
    """ShiftWindowMSA attention mask on the padded size: region ids from the three slices per
    axis, -100 between tokens of different regions.  (nW, N, N)"""
    img = torch.zeros(1, Hp, Wp, 1)
    cnt = 0
    for h in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for w in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img[:, h, w, :] = cnt
            cnt += 1
    win = window_partition(img, ws).view(-1, ws * ws)
    m = win[:, None, :] - win[:, :, None]
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


def window_partition(x, ws):
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, ws, ws, C)


def window_reverse(win, Hp, Wp, ws):
    B = int(win.shape[0] / (Hp * Wp / ws / ws))
    x = win.view(B, Hp // ws, Wp // ws, ws, ws, -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(B, Hp, Wp, -1)


def swin_block(x, H, W, w, k, heads, ws, shift):
    """SwinBlock: x + ShiftWindowMSA(norm1 x); x + FFN(norm2 x).  x (B, H*W, C)."""
    B, L, C = x.shape
    ident = x
    q = F.layer_norm(x, (C,), w[k + "norm1.weight"], w[k + "norm1.bias"], eps=1e-5).view(B, H, W, C)
    pad_r = (ws - W % ws) % ws
    pad_b = (ws - H % ws) % ws
    q = F.pad(q, (0, 0, 0, pad_r, 0, pad_b))
    Hp, Wp = H + pad_b, W + pad_r
    if shift > 0:
        q = torch.roll(q, shifts=(-shift, -shift), dims=(1, 2))
        mask = shift_mask(Hp, Wp, ws, shift).to(q.device)
    else:
        mask = None
    win = window_partition(q, ws).view(-1, ws * ws, C)
    Bw, N, _ = win.shape
    hd = C // heads
    qkv = F.linear(win, w[k + "attn.w_msa.qkv.weight"], w[k + "attn.w_msa.qkv.bias"])
    qkv = qkv.reshape(Bw, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    qq, kk, vv = qkv[0], qkv[1], qkv[2]
    qq = qq * (hd ** -0.5)
    attn = qq @ kk.transpose(-2, -1)
    table = w[k + "attn.w_msa.relative_position_bias_table"]
    bias = table[relative_position_index(ws).view(-1).to(table.device)].view(N, N, -1).permute(2, 0, 1)
    attn = attn + bias[None]
    if mask is not None:
        nW = mask.shape[0]
        attn = attn.view(Bw // nW, nW, heads, N, N) + mask[None, :, None]
        attn = attn.view(-1, heads, N, N)
    attn = attn.softmax(dim=-1)
    o = (attn @ vv).transpose(1, 2).reshape(Bw, N, C)
    o = F.linear(o, w[k + "attn.w_msa.proj.weight"], w[k + "attn.w_msa.proj.bias"])
    o = window_reverse(o.view(-1, ws, ws, C), Hp, Wp, ws)
    if shift > 0:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    o = o[:, :H, :W, :].reshape(B, H * W, C)
    x = ident + o
    h = F.layer_norm(x, (C,), w[k + "norm2.weight"], w[k + "norm2.bias"], eps=1e-5)
    h = F.gelu(F.linear(h, w[k + "ffn.layers.0.0.weight"], w[k + "ffn.layers.0.0.bias"]))
    h = F.linear(h, w[k + "ffn.layers.1.weight"], w[k + "ffn.layers.1.bias"])
    return x + h


def patch_merging(x, H, W, w, k):
    """mmcv PatchMerging: nn.Unfold(2, stride 2) channel order c*4 + kh*2 + kw, LN(4C), Linear."""
    B, L, C = x.shape
    xi = x.view(B, H, W, C).permute(0, 3, 1, 2)
    if H % 2 or W % 2:  # AdaptivePadding 'corner'
        xi = F.pad(xi, (0, W % 2, 0, H % 2))
    u = F.unfold(xi, kernel_size=2, stride=2).transpose(1, 2)
    u = F.layer_norm(u, (4 * C,), w[k + "norm.weight"], w[k + "norm.bias"], eps=1e-5)
    return F.linear(u, w[k + "reduction.weight"]), ((H + 1) // 2, (W + 1) // 2)


def swin_forward(img, w, cfg=SWIN_S):
    """-> list of 4 NCHW feature maps (after norm0..norm3)."""
    x = F.conv2d(img, w["backbone.patch_embed.projection.weight"], w["backbone.patch_embed.projection.bias"],
                 stride=4)
    B, C, H, W = x.shape
    x = x.flatten(2).transpose(1, 2)
    x = F.layer_norm(x, (C,), w["backbone.patch_embed.norm.weight"], w["backbone.patch_embed.norm.bias"], eps=1e-5)
    outs = []
    ws = cfg["window"]
    for si, (depth, heads) in enumerate(zip(cfg["depths"], cfg["heads"])):
        for bi in range(depth):
            x = swin_block(x, H, W, w, f"backbone.stages.{si}.blocks.{bi}.", heads, ws, ws // 2 if bi % 2 else 0)
        Cs = x.shape[-1]
        o = F.layer_norm(x, (Cs,), w[f"backbone.norm{si}.weight"], w[f"backbone.norm{si}.bias"], eps=1e-5)
        outs.append(o.view(B, H, W, Cs).permute(0, 3, 1, 2).contiguous())
        if si < 3:
            x, (H, W) = patch_merging(x, H, W, w, f"backbone.stages.{si}.downsample.")
    return outs


def fpn_forward(feats, w):
    lat = [F.conv2d(f, w[f"neck.lateral_convs.{i}.conv.weight"], w[f"neck.lateral_convs.{i}.conv.bias"])
           for i, f in enumerate(feats)]
    for i in range(3, 0, -1):
        lat[i - 1] = lat[i - 1] + F.interpolate(lat[i], size=lat[i - 1].shape[2:], mode="nearest")
    outs = [F.conv2d(lat[i], w[f"neck.fpn_convs.{i}.conv.weight"], w[f"neck.fpn_convs.{i}.conv.bias"], padding=1)
            for i in range(4)]
    outs.append(F.max_pool2d(outs[-1], 1, stride=2))
    return outs


# ----------------------------------------------------------------------------- RPN

def base_anchors(stride, ratios=ANCHOR_RATIOS, scale=ANCHOR_SCALE):
    """AnchorGenerator.gen_single_level_base_anchors (center offset 0): ratios outer, scales inner."""
    r = torch.tensor(ratios, dtype=torch.float32)
    h_r = torch.sqrt(r)
    w_r = 1 / h_r
    ws = (stride * w_r[:, None] * torch.tensor([float(scale)])[None, :]).view(-1)
    hs = (stride * h_r[:, None] * torch.tensor([float(scale)])[None, :]).view(-1)
    return torch.stack([-0.5 * ws, -0.5 * hs, 0.5 * ws, 0.5 * hs], dim=-1)


def grid_anchors(feat_h, feat_w, stride):
    """(H*W*A, 4): position-major (y, x), anchor-minor."""
    b = base_anchors(stride)
    sx = torch.arange(0, feat_w, dtype=torch.float32) * stride
    sy = torch.arange(0, feat_h, dtype=torch.float32) * stride
    yy, xx = torch.meshgrid(sy, sx, indexing="ij")
    shifts = torch.stack([xx.reshape(-1), yy.reshape(-1), xx.reshape(-1), yy.reshape(-1)], dim=-1)
    return (b[None, :, :] + shifts[:, None, :]).view(-1, 4)


def delta2bbox(rois, deltas, stds, max_shape):
    """DeltaXYWHBBoxCoder.decode (means 0, clip_border, wh_ratio_clip 16/1000)."""
    d = deltas * torch.tensor(stds, dtype=torch.float32)
    dx, dy, dw, dh = d[:, 0], d[:, 1], d[:, 2], d[:, 3]
    max_ratio = abs(math.log(WH_RATIO_CLIP))
    dw = dw.clamp(min=-max_ratio, max=max_ratio)
    dh = dh.clamp(min=-max_ratio, max=max_ratio)
    px = (rois[:, 0] + rois[:, 2]) * 0.5
    py = (rois[:, 1] + rois[:, 3]) * 0.5
    pw = rois[:, 2] - rois[:, 0]
    ph = rois[:, 3] - rois[:, 1]
    gw = pw * dw.exp()
    gh = ph * dh.exp()
    gx = px + pw * dx
    gy = py + ph * dy
    x1 = gx - gw * 0.5
    y1 = gy - gh * 0.5
    x2 = gx + gw * 0.5
    y2 = gy + gh * 0.5
    b = torch.stack([x1, y1, x2, y2], dim=-1)
    b[:, 0::2] = b[:, 0::2].clamp(min=0, max=max_shape[1])
    b[:, 1::2] = b[:, 1::2].clamp(min=0, max=max_shape[0])
    return b


def nms(boxes, scores, iou_thr):
    """mmcv nms (CUDA kernel semantics, offset 0): visit boxes in descending score order (ties:
    lower index first); a later box is suppressed when inter > thr * (area_a + area_b - inter),
    all in float32.  -> kept indices in visiting order."""
    sc = np.asarray(scores, np.float32)
    order = np.lexsort((np.arange(len(sc)), -sc.astype(np.float64)))
    b = np.asarray(boxes, np.float32)[order]
    thr = np.float32(iou_thr)
    area = ((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])).astype(np.float32)
    supp = np.zeros(len(order), bool)
    keep = []
    for i in range(len(order)):
        if supp[i]:
            continue
        keep.append(int(order[i]))
        rest = np.arange(i + 1, len(order))
        rest = rest[~supp[rest]]
        if rest.size == 0:
            continue
        w = np.maximum(np.minimum(b[i, 2], b[rest, 2]) - np.maximum(b[i, 0], b[rest, 0]), np.float32(0))
        h = np.maximum(np.minimum(b[i, 3], b[rest, 3]) - np.maximum(b[i, 1], b[rest, 1]), np.float32(0))
        inter = (w * h).astype(np.float32)
        uni = ((area[i] + area[rest]).astype(np.float32) - inter).astype(np.float32)
        supp[rest[inter > (thr * uni).astype(np.float32)]] = True
    return keep


def batched_nms(boxes, scores, idxs, iou_thr):
    """mmcv batched_nms (class_agnostic False): offset boxes by idx * (max + 1), then nms."""
    if boxes.numel() == 0:
        return boxes.new_zeros((0, 5)), boxes.new_zeros((0,), dtype=torch.long)
    max_c = boxes.max()
    offsets = idxs.to(boxes) * (max_c + torch.tensor(1).to(boxes))
    keep = nms(boxes + offsets[:, None], scores, iou_thr)
    keep = torch.tensor(keep, dtype=torch.long)
    return torch.cat([boxes[keep], scores[keep][:, None]], -1), keep


def rpn_forward(feats, w, img_shape):
    """RPNHead + _predict_by_feat_single -> proposals (n, 4), scores (n,)."""
    boxes_all, scores_all, lvl_all = [], [], []
    for lvl, (f, stride) in enumerate(zip(feats, STRIDES)):
        h = F.relu(F.conv2d(f, w["rpn_head.rpn_conv.weight"], w["rpn_head.rpn_conv.bias"], padding=1))
        cls = F.conv2d(h, w["rpn_head.rpn_cls.weight"], w["rpn_head.rpn_cls.bias"])
        reg = F.conv2d(h, w["rpn_head.rpn_reg.weight"], w["rpn_head.rpn_reg.bias"])
        s, d = rpn_level_outputs(cls, reg)
        b, sc = rpn_level_select(s, d, f.shape[2], f.shape[3], stride, img_shape)
        boxes_all.append(b)
        scores_all.append(sc)
        lvl_all.append(torch.full((sc.numel(),), lvl, dtype=torch.long))
    return rpn_merge(torch.cat(boxes_all), torch.cat(scores_all), torch.cat(lvl_all))


def rpn_level_outputs(cls, reg):
    """(1, A, H, W) logits, (1, 4A, H, W) deltas -> sigmoid scores (H*W*A,), deltas (H*W*A, 4)."""
    s = cls[0].permute(1, 2, 0).reshape(-1).sigmoid()
    d = reg[0].permute(1, 2, 0).reshape(-1, 4)
    return s, d


def rpn_level_select(scores, deltas, feat_h, feat_w, stride, img_shape):
    """top nms_pre by score (descending; ties -> lower index), decode, clip."""
    anchors = grid_anchors(feat_h, feat_w, stride)
    if scores.numel() > RPN_NMS_PRE:
        order = sorted(range(scores.numel()), key=lambda i: (-float(scores[i]), i))[:RPN_NMS_PRE]
        order = torch.tensor(order, dtype=torch.long)
        scores, deltas, anchors = scores[order], deltas[order], anchors[order]
    return delta2bbox(anchors, deltas, (1.0, 1.0, 1.0, 1.0), img_shape), scores


def rpn_merge(boxes, scores, lvl):
    w = boxes[:, 2] - boxes[:, 0]
    h = boxes[:, 3] - boxes[:, 1]
    valid = (w > 0) & (h > 0)
    if not bool(valid.all()):
        boxes, scores, lvl = boxes[valid], scores[valid], lvl[valid]
    dets, keep = batched_nms(boxes, scores, lvl, RPN_IOU)
    return boxes[keep][:RPN_MAX], dets[:RPN_MAX, -1]


# ----------------------------------------------------------------------------- RoI head

def map_roi_levels(rois, num_levels=4, finest_scale=56):
    scale = torch.sqrt((rois[:, 2] - rois[:, 0]) * (rois[:, 3] - rois[:, 1]))
    lv = torch.floor(torch.log2(scale / finest_scale + 1e-6))
    return lv.clamp(min=0, max=num_levels - 1).long()


def roi_align(feat, rois, spatial_scale, out=7):
    """mmcv roi_align forward, aligned=True, sampling_ratio 0 (adaptive), avg.  feat (C, H, W)."""
    C, H, W = feat.shape
    res = torch.zeros(rois.shape[0], C, out, out)
    for r in range(rois.shape[0]):
        x1, y1, x2, y2 = [float(v) for v in rois[r]]
        sx = np.float32(np.float32(x1) * np.float32(spatial_scale) - np.float32(0.5))
        sy = np.float32(np.float32(y1) * np.float32(spatial_scale) - np.float32(0.5))
        ex = np.float32(np.float32(x2) * np.float32(spatial_scale) - np.float32(0.5))
        ey = np.float32(np.float32(y2) * np.float32(spatial_scale) - np.float32(0.5))
        rw, rh = np.float32(ex - sx), np.float32(ey - sy)
        bw, bh = np.float32(rw / np.float32(out)), np.float32(rh / np.float32(out))
        gh = int(np.ceil(np.float32(rh / np.float32(out))))
        gw = int(np.ceil(np.float32(rw / np.float32(out))))
        cnt = max(gh * gw, 1)
        for ph in range(out):
            for pw in range(out):
                acc = torch.zeros(C)
                for iy in range(gh):
                    y = np.float32(sy + np.float32(ph) * bh + np.float32(np.float32(iy + 0.5) * bh / np.float32(gh)))
                    for ix in range(gw):
                        x = np.float32(sx + np.float32(pw) * bw + np.float32(np.float32(ix + 0.5) * bw / np.float32(gw)))
                        acc += _bilinear(feat, H, W, y, x)
                res[r, :, ph, pw] = acc / cnt
    return res


def _bilinear(feat, H, W, y, x):
    if y < -1.0 or y > H or x < -1.0 or x > W:
        return torch.zeros(feat.shape[0])
    y = max(y, np.float32(0))
    x = max(x, np.float32(0))
    yl, xl = int(y), int(x)
    if yl >= H - 1:
        yh = yl = H - 1
        y = np.float32(yl)
    else:
        yh = yl + 1
    if xl >= W - 1:
        xh = xl = W - 1
        x = np.float32(xl)
    else:
        xh = xl + 1
    ly, lx = np.float32(y - yl), np.float32(x - xl)
    hy, hx = np.float32(1 - ly), np.float32(1 - lx)
    return (float(hy * hx) * feat[:, yl, xl] + float(hy * lx) * feat[:, yl, xh]
            + float(ly * hx) * feat[:, yh, xl] + float(ly * lx) * feat[:, yh, xh])


def roi_extract(feats, rois):
    """SingleRoIExtractor over P2..P5 -> (n, 256, 7, 7)."""
    lv = map_roi_levels(rois)
    out = torch.zeros(rois.shape[0], feats[0].shape[1], 7, 7)
    for i in range(4):
        idx = torch.nonzero(lv == i).view(-1)
        if idx.numel():
            out[idx] = roi_align(feats[i][0], rois[idx], 1.0 / STRIDES[i])
    return out


def bbox_head(roi_feats, w):
    k = "roi_head.bbox_head."
    x = roi_feats.flatten(1)
    x = F.relu(F.linear(x, w[k + "shared_fcs.0.weight"], w[k + "shared_fcs.0.bias"]))
    x = F.relu(F.linear(x, w[k + "shared_fcs.1.weight"], w[k + "shared_fcs.1.bias"]))
    return F.linear(x, w[k + "fc_cls.weight"], w[k + "fc_cls.bias"]), F.linear(x, w[k + "fc_reg.weight"],
                                                                                  w[k + "fc_reg.bias"])


def rcnn_post(rois, cls, reg, img_shape, scale_factor):
    """_predict_by_feat_single + multiclass_nms (1 class) -> boxes (n, 4) original pixels, scores."""
    scores = F.softmax(cls, dim=-1)
    boxes = delta2bbox(rois, reg, (0.1, 0.1, 0.2, 0.2), img_shape)
    inv = torch.tensor([1 / scale_factor[0], 1 / scale_factor[1]], dtype=torch.float32).repeat(2)
    boxes = boxes * inv
    s = scores[:, 0]
    valid = s > RCNN_SCORE_THR
    boxes, s = boxes[valid], s[valid]
    if boxes.numel() == 0:
        return boxes.view(0, 4), s
    dets, keep = batched_nms(boxes, s, torch.zeros(s.numel(), dtype=torch.long), RCNN_IOU)
    return dets[:RCNN_MAX, :4], dets[:RCNN_MAX, 4]


def detect(img_bgr, w, cfg=SWIN_S, scale=(800, 800)):
    """inference_detector on one BGR frame -> (boxes (n, 4) original pixels, scores (n,))."""
    x, img_shape, sf = preprocess(img_bgr, scale)
    feats = swin_forward(x, w, cfg)
    p = fpn_forward(feats, w)
    props, _ = rpn_forward(p, w, img_shape)
    rf = roi_extract(p[:4], props)
    cls, reg = bbox_head(rf, w)
    return rcnn_post(props, cls, reg, img_shape, sf)
