"""Step-1 detector on MI355X: Swin-S Mask R-CNN (bbox only), ``inference_detector`` of
``src/pipeline/step1_proc2d.py``:226-237 with the model of
``model/detection/SWIN-Mask_R-CNN_bbox_only.py``:29-226 and the test pipeline of step1:104-109.

Every arithmetic step runs in libmq_hip (``include/mq_hip.h``, detector section + ``mq_gemm_bf16`` /
``mq_layernorm``); this module owns the weights (bf16 [N][K] GEMM operands, f32 biases / norms) and
sequences the launches on the caller's stream.  Per batch of frames (all views of a frame):

  resize + normalise + patch im2col -> patch GEMM -> LN                        (PatchEmbed)
  per Swin block: LN1 -> qkv GEMM -> window attention -> proj GEMM (+= x)
                  LN2 -> fc1 GEMM (GELU) -> fc2 GEMM (+= x)                      (SwinBlock)
  per stage: LN_s -> FPN lateral GEMM; merge gather -> LN(4C) -> reduction GEMM  (norm_s, PatchMerging)
  FPN: nearest top-down adds, 3x3 im2col -> GEMM, P6 = every other pixel of P5
  RPN: 3x3 im2col of every level -> one GEMM (ReLU) -> one GEMM (3 logits + 12 deltas)
       -> sigmoid / per-level top 1000 / decode / NMS 0.7 / top 1000          (mq_rpn_proposals)
  RoIAlign 7x7 -> fc 1024 (ReLU) -> fc 1024 (ReLU) -> cls + reg GEMM -> softmax / decode / rescale /
       score > 0.05 / NMS 0.5 / top 100                                         (mq_rcnn_post)

GEMM operands are bf16 with f32 accumulation; the residual stream, LayerNorm statistics, feature
maps and all box arithmetic are f32.  No CPU fallback: without the HIP library the calls raise.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib

EPI_BF16, EPI_GELU, EPI_RESID, EPI_F32, EPI_RELU = 0, 1, 2, 4, 6
SWIN_S = dict(embed=96, depths=(2, 2, 18, 2), heads=(3, 6, 12, 24), window=7)
STRIDES = (4, 8, 16, 32, 64)
ANCHOR_RATIOS = (0.5, 1.0, 2.0)
ANCHOR_SCALE = 8
RPN_NMS_PRE, RPN_MAX, RPN_IOU = 1000, 1000, 0.7
RCNN_SCORE_THR, RCNN_IOU, RCNN_MAX = 0.05, 0.5, 100
LN_EPS = 1e-5


def make_random_weights(cfg=SWIN_S, seed=0, std=0.02):
    """Seeded random detector weights under the mmdet state_dict names (no checkpoint is available
    offline).  Scales keep the logits spread (no tied scores) so NMS / top-k see distinct inputs."""
    g = torch.Generator().manual_seed(seed)

    def rn(*shape, s=std):
        return (torch.randn(*shape, generator=g) * s).float()

    w = {}
    C, ws = cfg["embed"], cfg["window"]
    w["backbone.patch_embed.projection.weight"] = rn(C, 3, 4, 4, s=0.1)
    w["backbone.patch_embed.projection.bias"] = rn(C)
    w["backbone.patch_embed.norm.weight"] = 1 + rn(C, s=0.1)
    w["backbone.patch_embed.norm.bias"] = rn(C)
    for si, (depth, heads) in enumerate(zip(cfg["depths"], cfg["heads"])):
        Cs = C * 2 ** si
        for bi in range(depth):
            k = f"backbone.stages.{si}.blocks.{bi}."
            w[k + "norm1.weight"], w[k + "norm1.bias"] = 1 + rn(Cs, s=0.1), rn(Cs)
            w[k + "attn.w_msa.relative_position_bias_table"] = rn((2 * ws - 1) ** 2, heads, s=0.5)
            w[k + "attn.w_msa.qkv.weight"], w[k + "attn.w_msa.qkv.bias"] = rn(3 * Cs, Cs, s=Cs ** -0.5), rn(3 * Cs)
            w[k + "attn.w_msa.proj.weight"], w[k + "attn.w_msa.proj.bias"] = rn(Cs, Cs, s=0.5 * Cs ** -0.5), rn(Cs)
            w[k + "norm2.weight"], w[k + "norm2.bias"] = 1 + rn(Cs, s=0.1), rn(Cs)
            w[k + "ffn.layers.0.0.weight"], w[k + "ffn.layers.0.0.bias"] = rn(4 * Cs, Cs, s=Cs ** -0.5), rn(4 * Cs)
            w[k + "ffn.layers.1.weight"], w[k + "ffn.layers.1.bias"] = rn(Cs, 4 * Cs, s=0.5 * (4 * Cs) ** -0.5), rn(Cs)
        if si < 3:
            k = f"backbone.stages.{si}.downsample."
            w[k + "norm.weight"], w[k + "norm.bias"] = 1 + rn(4 * Cs, s=0.1), rn(4 * Cs)
            w[k + "reduction.weight"] = rn(2 * Cs, 4 * Cs, s=(4 * Cs) ** -0.5)
        w[f"backbone.norm{si}.weight"], w[f"backbone.norm{si}.bias"] = 1 + rn(Cs, s=0.1), rn(Cs)
    for i in range(4):
        cin = C * 2 ** i
        w[f"neck.lateral_convs.{i}.conv.weight"] = rn(256, cin, 1, 1, s=cin ** -0.5)
        w[f"neck.lateral_convs.{i}.conv.bias"] = rn(256)
        w[f"neck.fpn_convs.{i}.conv.weight"] = rn(256, 256, 3, 3, s=(9 * 256) ** -0.5)
        w[f"neck.fpn_convs.{i}.conv.bias"] = rn(256)
    w["rpn_head.rpn_conv.weight"], w["rpn_head.rpn_conv.bias"] = rn(256, 256, 3, 3, s=(9 * 256) ** -0.5), rn(256)
    w["rpn_head.rpn_cls.weight"], w["rpn_head.rpn_cls.bias"] = rn(3, 256, 1, 1, s=0.02), rn(3)
    w["rpn_head.rpn_reg.weight"], w["rpn_head.rpn_reg.bias"] = rn(12, 256, 1, 1, s=0.2 * 256 ** -0.5), rn(12)
    k = "roi_head.bbox_head."
    w[k + "shared_fcs.0.weight"], w[k + "shared_fcs.0.bias"] = rn(1024, 256 * 49, s=(256 * 49) ** -0.5), rn(1024)
    w[k + "shared_fcs.1.weight"], w[k + "shared_fcs.1.bias"] = rn(1024, 1024, s=1024 ** -0.5), rn(1024)
    w[k + "fc_cls.weight"], w[k + "fc_cls.bias"] = rn(2, 1024, s=0.05), rn(2)
    w[k + "fc_reg.weight"], w[k + "fc_reg.bias"] = rn(4, 1024, s=0.3 * 1024 ** -0.5), rn(4)
    return w


def rescale_size(w, h, scale=(800, 800)):
    """mmcv rescale_size (keep_ratio): (new_w, new_h)."""
    long_e, short_e = max(scale), min(scale)
    f = min(long_e / max(h, w), short_e / min(h, w))
    return int(w * f + 0.5), int(h * f + 0.5)


def linear_coeffs(dst, src):
    """cv::resize INTER_LINEAR tables: source offset and the two 11-bit weights per output index."""
    scale = 1.0 / (dst / src)  # resize.cpp: 1. / inv_scale_x
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = np.float32(0), 0
    hi = s >= src - 1
    f[hi], s[hi] = np.float32(0), src - 1
    c0 = (np.float32(1.0) - f).astype(np.float32)
    a = np.stack([np.rint((c0 * np.float32(2048)).astype(np.float32)),
                  np.rint((f * np.float32(2048)).astype(np.float32))], axis=1).astype(np.int32)
    return s.astype(np.int32), a


def base_anchors(stride):
    """AnchorGenerator base anchors (center offset 0, ratios outer, scale 8), float32 as torch computes them."""
    r = torch.tensor(ANCHOR_RATIOS, dtype=torch.float32)
    h_r = torch.sqrt(r)
    w_r = 1 / h_r
    sc = torch.tensor([float(ANCHOR_SCALE)])
    ws = (stride * w_r[:, None] * sc[None, :]).view(-1)
    hs = (stride * h_r[:, None] * sc[None, :]).view(-1)
    return torch.stack([-0.5 * ws, -0.5 * hs, 0.5 * ws, 0.5 * hs], dim=-1)


class SwinDetectorHip:
    """Swin-S Mask R-CNN bbox detector.  ``weights``: mmdet state_dict names -> float tensors."""

    def __init__(self, weights, cfg=SWIN_S, device: int = 0, scale=(800, 800)):
        self.cfg = cfg
        self.device = device
        self.scale = scale
        self.implicit_conv = True  # FPN / RPN 3x3 convolutions as implicit GEMMs (False: im2col + GEMM)
        self.dev = torch.device("cuda", device)
        self.ctx = _lib.Context.get(device)
        self.w = {}
        d = self.dev

        def f32(name):
            return weights[name].detach().float().contiguous().to(d)

        def bf16(t):
            return t.detach().float().contiguous().to(d).to(torch.bfloat16).contiguous()

        pe = weights["backbone.patch_embed.projection.weight"].float().reshape(cfg["embed"], 48)
        self.w["patch_w"] = bf16(torch.nn.functional.pad(pe, (0, 16)))
        for k in ("backbone.patch_embed.projection.bias", "backbone.patch_embed.norm.weight",
                  "backbone.patch_embed.norm.bias"):
            self.w[k] = f32(k)
        for si, depth in enumerate(cfg["depths"]):
            for bi in range(depth):
                p = f"backbone.stages.{si}.blocks.{bi}."
                for k in ("norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias", "attn.w_msa.qkv.bias",
                          "attn.w_msa.proj.bias", "ffn.layers.0.0.bias", "ffn.layers.1.bias",
                          "attn.w_msa.relative_position_bias_table"):
                    self.w[p + k] = f32(p + k)
                for k in ("attn.w_msa.qkv.weight", "attn.w_msa.proj.weight", "ffn.layers.0.0.weight",
                          "ffn.layers.1.weight"):
                    self.w[p + k] = bf16(weights[p + k])
            if si < 3:
                p = f"backbone.stages.{si}.downsample."
                self.w[p + "norm.weight"] = f32(p + "norm.weight")
                self.w[p + "norm.bias"] = f32(p + "norm.bias")
                self.w[p + "reduction.weight"] = bf16(weights[p + "reduction.weight"])
            self.w[f"backbone.norm{si}.weight"] = f32(f"backbone.norm{si}.weight")
            self.w[f"backbone.norm{si}.bias"] = f32(f"backbone.norm{si}.bias")

        def conv3(name):  # (Cout, Cin, 3, 3) -> [Cout][(ky * 3 + kx) * Cin + c]
            t = weights[name].float()
            return bf16(t.permute(0, 2, 3, 1).reshape(t.shape[0], -1))

        for i in range(4):
            self.w[f"lat{i}"] = bf16(weights[f"neck.lateral_convs.{i}.conv.weight"].float().flatten(1))
            self.w[f"lat{i}_b"] = f32(f"neck.lateral_convs.{i}.conv.bias")
            self.w[f"fpn{i}"] = conv3(f"neck.fpn_convs.{i}.conv.weight")
            self.w[f"fpn{i}_b"] = f32(f"neck.fpn_convs.{i}.conv.bias")
        self.w["rpn_conv"] = conv3("rpn_head.rpn_conv.weight")
        self.w["rpn_conv_b"] = f32("rpn_head.rpn_conv.bias")
        self.w["rpn_out"] = bf16(torch.cat([weights["rpn_head.rpn_cls.weight"].float().flatten(1),
                                            weights["rpn_head.rpn_reg.weight"].float().flatten(1)]))
        self.w["rpn_out_b"] = torch.cat([weights["rpn_head.rpn_cls.bias"].float(),
                                         weights["rpn_head.rpn_reg.bias"].float()]).contiguous().to(d)
        k = "roi_head.bbox_head."
        self.w["fc0"] = bf16(weights[k + "shared_fcs.0.weight"])
        self.w["fc0_b"] = f32(k + "shared_fcs.0.bias")
        self.w["fc1"] = bf16(weights[k + "shared_fcs.1.weight"])
        self.w["fc1_b"] = f32(k + "shared_fcs.1.bias")
        self.w["fcout"] = bf16(torch.cat([weights[k + "fc_cls.weight"].float(), weights[k + "fc_reg.weight"].float()]))
        self.w["fcout_b"] = torch.cat([weights[k + "fc_cls.bias"].float(),
                                       weights[k + "fc_reg.bias"].float()]).contiguous().to(d)
        self._geom = {}

    # ------------------------------------------------------------------ launch helpers
    def _s(self):
        return _lib.stream_ptr(self.dev)

    def _gemm(self, A, W, C, bias, M, N, K, epi, ldc=None):
        _lib.check(self.ctx.lib.mq_gemm_bf16(self.ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(C),
                                             _lib.ptr(bias) if bias is not None else None, None, M, N, K, K, K,
                                             N if ldc is None else ldc, 0, epi, self._s()), "mq_gemm_bf16")

    def _conv3x3(self, x, n, h, w, wt, bias, out, epi):
        """3x3 / pad 1 conv of the f32 NHWC map x (256 channels): implicit GEMM on its bf16 copy (default), or
        im2col + GEMM (``self.implicit_conv = False``); both give the same bits."""
        rows = n * h * w
        if self.implicit_conv:
            xb = torch.empty((rows, 256), dtype=torch.bfloat16, device=self.dev)
            _lib.check(self.ctx.lib.mq_f32_to_bf16(self.ctx.handle, _lib.ptr(x), _lib.ptr(xb), rows * 256, self._s()),
                       "mq_f32_to_bf16")
            _lib.check(self.ctx.lib.mq_conv3x3_bf16(self.ctx.handle, _lib.ptr(xb), n, h, w, 256, _lib.ptr(wt),
                                                    _lib.ptr(bias), _lib.ptr(out), out.shape[1], out.shape[1], epi,
                                                    self._s()), "mq_conv3x3_bf16")
            return
        cols = torch.empty((rows, 9 * 256), dtype=torch.bfloat16, device=self.dev)
        _lib.check(self.ctx.lib.mq_im2col3x3(self.ctx.handle, _lib.ptr(x), n, h, w, 256, _lib.ptr(cols), self._s()),
                   "mq_im2col3x3")
        self._gemm(cols, wt, out, bias, rows, out.shape[1], 9 * 256, epi)

    def _add_ln(self, x, p1, p2, store, g, b, y, rows, dim):
        _lib.check(self.ctx.lib.mq_add_layernorm(self.ctx.handle, _lib.ptr(x), _lib.ptr(p1),
                                                 None if p2 is None else _lib.ptr(p2), 1 if store else 0, _lib.ptr(g),
                                                 _lib.ptr(b), _lib.ptr(y), rows, dim, LN_EPS, self._s()),
                   "mq_add_layernorm")

    def _ln(self, x, g, b, y, rows, dim, out_f32=False):
        _lib.check(self.ctx.lib.mq_layernorm(self.ctx.handle, _lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), rows,
                                             dim, LN_EPS, 1 if out_f32 else 0, self._s()), "mq_layernorm")

    def geometry(self, H, W):
        """Resize tables and feature sizes for (H, W) frames (cached)."""
        key = (H, W)
        if key not in self._geom:
            nw, nh = rescale_size(W, H, self.scale)
            hp, wp = int(math.ceil(nh / 32)) * 32, int(math.ceil(nw / 32)) * 32
            xo, xa = linear_coeffs(nw, W)
            yo, ya = linear_coeffs(nh, H)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)  # noqa: E731
            sizes = [(hp // 4, wp // 4)]
            for _ in range(3):
                h, w = sizes[-1]
                sizes.append(((h + 1) // 2, (w + 1) // 2))
            h5, w5 = sizes[3]
            levels = sizes + [((h5 + 1) // 2, (w5 + 1) // 2)]
            anchors = torch.stack([base_anchors(s) for s in STRIDES]).contiguous()
            self._geom[key] = dict(nh=nh, nw=nw, hp=hp, wp=wp, xo=t(xo), xa=t(xa), yo=t(yo), ya=t(ya), sizes=sizes,
                                   levels=levels, anchors=anchors.numpy().astype(np.float32),
                                   scale_factor=(nw / W, nh / H))
        return self._geom[key]

    # ------------------------------------------------------------------ forward
    def backbone(self, frames):
        """frames uint8 (n, H, W, 3) BGR on the device -> (4 NHWC f32 stage outputs after norm_s as
        FPN laterals' inputs are produced inside fpn(); here: list of bf16 normed stage maps)."""
        n, H, W, _ = frames.shape
        g = self.geometry(H, W)
        dev = self.dev
        C = self.cfg["embed"]
        th, tw = g["sizes"][0]
        T = n * th * tw
        A0 = torch.empty((T, 64), dtype=torch.bfloat16, device=dev)
        _lib.check(self.ctx.lib.mq_det_resize_patch(self.ctx.handle, _lib.ptr(frames), H * W * 3, n, H, W, g["nh"],
                                                    g["nw"], g["hp"], g["wp"], _lib.ptr(g["xo"]), _lib.ptr(g["xa"]),
                                                    _lib.ptr(g["yo"]), _lib.ptr(g["ya"]), _lib.ptr(A0), self._s()),
                   "mq_det_resize_patch")
        x0 = torch.empty((T, C), dtype=torch.float32, device=dev)
        self._gemm(A0, self.w["patch_w"], x0, self.w["backbone.patch_embed.projection.bias"], T, C, 64, EPI_F32)
        x = torch.empty_like(x0)
        self._ln(x0, self.w["backbone.patch_embed.norm.weight"], self.w["backbone.patch_embed.norm.bias"], x, T, C,
                 out_f32=True)
        outs = []
        for si, (depth, heads) in enumerate(zip(self.cfg["depths"], self.cfg["heads"])):
            Cs = C * 2 ** si
            Hs, Ws = g["sizes"][si]
            T = n * Hs * Ws
            h = torch.empty((T, Cs), dtype=torch.bfloat16, device=dev)
            qkv = torch.empty((T, 3 * Cs), dtype=torch.bfloat16, device=dev)
            att = torch.empty((T, Cs), dtype=torch.bfloat16, device=dev)
            mlp = torch.empty((T, 4 * Cs), dtype=torch.bfloat16, device=dev)
            # residual updates as in the ViT: proj and fc2 write their branch outputs in
            # bf16 (bias included) and the next LayerNorm adds them to the f32 stream x (x += p1; x += p2)
            p1 = torch.empty((T, Cs), dtype=torch.bfloat16, device=dev)
            p2 = torch.empty((T, Cs), dtype=torch.bfloat16, device=dev)
            for bi in range(depth):
                p = f"backbone.stages.{si}.blocks.{bi}."
                if bi == 0:
                    self._ln(x, self.w[p + "norm1.weight"], self.w[p + "norm1.bias"], h, T, Cs)
                else:
                    self._add_ln(x, p1, p2, True, self.w[p + "norm1.weight"], self.w[p + "norm1.bias"], h, T, Cs)
                self._gemm(h, self.w[p + "attn.w_msa.qkv.weight"], qkv, self.w[p + "attn.w_msa.qkv.bias"], T, 3 * Cs,
                           Cs, EPI_BF16)
                shift = self.cfg["window"] // 2 if bi % 2 else 0
                _lib.check(self.ctx.lib.mq_window_attention(
                    self.ctx.handle, _lib.ptr(qkv), _lib.ptr(self.w[p + "attn.w_msa.qkv.bias"]),
                    _lib.ptr(self.w[p + "attn.w_msa.relative_position_bias_table"]), _lib.ptr(att), n, Hs, Ws, Cs,
                    heads, shift, self._s()), "mq_window_attention")
                self._gemm(att, self.w[p + "attn.w_msa.proj.weight"], p1, self.w[p + "attn.w_msa.proj.bias"], T, Cs,
                           Cs, EPI_BF16)
                self._add_ln(x, p1, None, False, self.w[p + "norm2.weight"], self.w[p + "norm2.bias"], h, T, Cs)
                self._gemm(h, self.w[p + "ffn.layers.0.0.weight"], mlp, self.w[p + "ffn.layers.0.0.bias"], T, 4 * Cs,
                           Cs, EPI_GELU)
                self._gemm(mlp, self.w[p + "ffn.layers.1.weight"], p2, self.w[p + "ffn.layers.1.bias"], T, Cs,
                           4 * Cs, EPI_BF16)
            o = torch.empty((T, Cs), dtype=torch.bfloat16, device=dev)
            # the last block's updates, stored (patch merging reads x), and the stage's output norm
            self._add_ln(x, p1, p2, True, self.w[f"backbone.norm{si}.weight"], self.w[f"backbone.norm{si}.bias"], o, T,
                         Cs)
            del p1, p2
            outs.append(o)
            if si < 3:
                H2, W2 = g["sizes"][si + 1]
                T2 = n * H2 * W2
                m = torch.empty((T2, 4 * Cs), dtype=torch.float32, device=dev)
                _lib.check(self.ctx.lib.mq_patch_merge_gather(self.ctx.handle, _lib.ptr(x), n, Hs, Ws, Cs, _lib.ptr(m),
                                                              self._s()), "mq_patch_merge_gather")
                p = f"backbone.stages.{si}.downsample."
                mh = torch.empty((T2, 4 * Cs), dtype=torch.bfloat16, device=dev)
                self._ln(m, self.w[p + "norm.weight"], self.w[p + "norm.bias"], mh, T2, 4 * Cs)
                x = torch.empty((T2, 2 * Cs), dtype=torch.float32, device=dev)
                self._gemm(mh, self.w[p + "reduction.weight"], x, None, T2, 2 * Cs, 4 * Cs, EPI_F32)
        return outs

    def fpn(self, outs, n, g):
        dev = self.dev
        C = self.cfg["embed"]
        lat = []
        for i, o in enumerate(outs):
            Hs, Ws = g["sizes"][i]
            t = torch.empty((n * Hs * Ws, 256), dtype=torch.float32, device=dev)
            self._gemm(o, self.w[f"lat{i}"], t, self.w[f"lat{i}_b"], n * Hs * Ws, 256, C * 2 ** i, EPI_F32)
            lat.append(t)
        for i in range(3, 0, -1):
            (hl, wl), (hh, wh) = g["sizes"][i - 1], g["sizes"][i]
            _lib.check(self.ctx.lib.mq_upsample_add(self.ctx.handle, _lib.ptr(lat[i - 1]), _lib.ptr(lat[i]), n, hl, wl,
                                                    hh, wh, 256, self._s()), "mq_upsample_add")
        P = []
        for i in range(4):
            Hs, Ws = g["sizes"][i]
            t = torch.empty((n * Hs * Ws, 256), dtype=torch.float32, device=dev)
            self._conv3x3(lat[i], n, Hs, Ws, self.w[f"fpn{i}"], self.w[f"fpn{i}_b"], t, EPI_F32)
            P.append(t)
        h5, w5 = g["sizes"][3]
        h6, w6 = g["levels"][4]
        p6 = torch.empty((n * h6 * w6, 256), dtype=torch.float32, device=dev)
        _lib.check(self.ctx.lib.mq_subsample2(self.ctx.handle, _lib.ptr(P[3]), n, h5, w5, 256, _lib.ptr(p6), self._s()),
                   "mq_subsample2")
        P.append(p6)
        return P

    def rpn_head(self, P, n, g):
        """-> head f32 (rows level-major over the batch, 15)."""
        dev = self.dev
        rows = [n * h * w for h, w in g["levels"]]
        M = sum(rows)
        hid = torch.empty((M, 256), dtype=torch.bfloat16, device=dev)
        off = 0
        for (h, w), p, r in zip(g["levels"], P, rows):
            self._conv3x3(p, n, h, w, self.w["rpn_conv"], self.w["rpn_conv_b"], hid[off:off + r], EPI_RELU)
            off += r
        head = torch.empty((M, 15), dtype=torch.float32, device=dev)
        self._gemm(hid, self.w["rpn_out"], head, self.w["rpn_out_b"], M, 15, 256, EPI_F32)
        return head

    def proposals(self, head, n, g):
        dev = self.dev
        lv = np.array(g["levels"], dtype=np.int32).reshape(-1)
        st = np.array(STRIDES, dtype=np.int32)
        an = np.ascontiguousarray(g["anchors"], dtype=np.float32)
        props = torch.empty((n, RPN_MAX, 4), dtype=torch.float32, device=dev)
        sc = torch.empty((n, RPN_MAX), dtype=torch.float32, device=dev)
        cnt = torch.empty((n,), dtype=torch.int32, device=dev)
        _lib.check(self.ctx.lib.mq_rpn_proposals(
            self.ctx.handle, _lib.ptr(head), n, len(STRIDES), lv.ctypes.data, st.ctypes.data, an.ctypes.data,
            RPN_NMS_PRE, float(g["nh"]), float(g["nw"]), RPN_IOU, RPN_MAX, _lib.ptr(props), _lib.ptr(sc), _lib.ptr(cnt),
            self._s()), "mq_rpn_proposals")
        return props, sc, cnt

    def roi_features(self, P, props, cnt, n, g):
        dev = self.dev
        lv = np.array(g["sizes"], dtype=np.int32).reshape(-1)
        st = np.array(STRIDES[:4], dtype=np.int32)
        out = torch.empty((n * RPN_MAX, 256 * 49), dtype=torch.bfloat16, device=dev)
        _lib.check(self.ctx.lib.mq_roi_align(self.ctx.handle, _lib.ptr(P[0]), _lib.ptr(P[1]), _lib.ptr(P[2]),
                                             _lib.ptr(P[3]), lv.ctypes.data, st.ctypes.data, _lib.ptr(props),
                                             _lib.ptr(cnt), n, RPN_MAX, _lib.ptr(out), self._s()), "mq_roi_align")
        return out

    def bbox_head(self, rf):
        dev = self.dev
        M = rf.shape[0]
        h0 = torch.empty((M, 1024), dtype=torch.bfloat16, device=dev)
        self._gemm(rf, self.w["fc0"], h0, self.w["fc0_b"], M, 1024, 256 * 49, EPI_RELU)
        h1 = torch.empty((M, 1024), dtype=torch.bfloat16, device=dev)
        self._gemm(h0, self.w["fc1"], h1, self.w["fc1_b"], M, 1024, 1024, EPI_RELU)
        out = torch.empty((M, 6), dtype=torch.float32, device=dev)
        self._gemm(h1, self.w["fcout"], out, self.w["fcout_b"], M, 6, 1024, EPI_F32)
        return out

    def detections(self, props, head, cnt, n, g):
        dev = self.dev
        sw, sh = g["scale_factor"]
        boxes = torch.empty((n, RCNN_MAX, 4), dtype=torch.float32, device=dev)
        scores = torch.empty((n, RCNN_MAX), dtype=torch.float32, device=dev)
        dcnt = torch.empty((n,), dtype=torch.int32, device=dev)
        _lib.check(self.ctx.lib.mq_rcnn_post(self.ctx.handle, _lib.ptr(props), _lib.ptr(head), _lib.ptr(cnt), n,
                                             RPN_MAX, float(g["nh"]), float(g["nw"]), float(np.float32(1 / sw)),
                                             float(np.float32(1 / sh)), RCNN_SCORE_THR, RCNN_IOU, RCNN_MAX,
                                             _lib.ptr(boxes), _lib.ptr(scores), _lib.ptr(dcnt), self._s()),
                   "mq_rcnn_post")
        return boxes, scores, dcnt

    def forward(self, frames, keep_intermediates=False):
        """frames uint8 (n, H, W, 3) BGR device tensor -> boxes (n, 100, 4), scores (n, 100), counts (n,)
        in original-image pixels (device tensors); with keep_intermediates also the stage tensors."""
        assert frames.dtype == torch.uint8 and frames.dim() == 4 and frames.shape[3] == 3, "frames (n, H, W, 3) uint8"
        frames = frames.contiguous()
        n, H, W, _ = frames.shape
        g = self.geometry(H, W)
        outs = self.backbone(frames)
        P = self.fpn(outs, n, g)
        head = self.rpn_head(P, n, g)
        props, psc, cnt = self.proposals(head, n, g)
        rf = self.roi_features(P, props, cnt, n, g)
        bh = self.bbox_head(rf)
        boxes, scores, dcnt = self.detections(props, bh, cnt, n, g)
        if keep_intermediates:
            return boxes, scores, dcnt, dict(outs=outs, P=P, head=head, props=props, prop_scores=psc, prop_counts=cnt,
                                             roi_feats=rf, bbox_head=bh)
        return boxes, scores, dcnt


def inference_detector(model: SwinDetectorHip, imgs):
    """mmdet.apis.inference_detector(model, [img]) for uint8 BGR frames (numpy HxWx3 or a device
    tensor batch): list of (bboxes (k, 4) float32, scores (k,)) numpy per image, like
    ``det.pred_instances.bboxes / .scores`` (step1_proc2d.py:226-228)."""
    if isinstance(imgs, torch.Tensor):
        fr = imgs
    else:
        fr = torch.from_numpy(np.stack([np.ascontiguousarray(i) for i in imgs])).to(model.dev)
    boxes, scores, cnt = model.forward(fr)
    b, s, c = boxes.cpu().numpy(), scores.cpu().numpy(), cnt.cpu().numpy()
    return [(b[i, :c[i]], s[i, :c[i]]) for i in range(b.shape[0])]
