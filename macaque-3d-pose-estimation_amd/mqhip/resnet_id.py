"""Step-1 collar-ID classifier on MI355X: ResNet-152 + GlobalAveragePooling + LinearClsHead(6), the
model of ``model/id/sn_resnet152_8xb32_in1k_pretrained_optimized_finetuned.py``:40-73 as
``classify_patches`` (``src/pipeline/step1_proc2d.py``:140-163) runs it through mmpretrain's
``ImageClassificationInferencer``.

Every arithmetic step runs in libmq_hip (``include/mq_hip.h``, ID-classifier section +
``mq_gemm_bf16``); this module folds BatchNorm into the convolution weights (bf16 [Cout][kh kw Cin]
GEMM operands, f32 bias), and sequences the launches on the caller's stream:

  patch slice + cv2.resize(224) (mq_id_crop_resize) -> ResizeEdge(256) + CenterCrop(224) + to_rgb +
  normalise (mq_id_preprocess) -> stem 7x7/2 im2col + GEMM (ReLU) -> MaxPool 3x3/2
  per Bottleneck: 1x1 GEMM (ReLU) -> 3x3/s im2col + GEMM (ReLU) -> [downsample: 1x1/s GEMM -> f32]
                  -> 1x1 GEMM accumulated into the f32 identity (+=) -> ReLU + bf16 copy
  -> GAP + fc + softmax (mq_id_head) -> pred_label = argmax, pred_score = max

Maps are NHWC; convolution operands bf16 with f32 accumulation; each stage's residual stream f32.
No CPU fallback: without the HIP library the calls raise.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

EPI_F32, EPI_RELU = 4, 6
ID_CLASSES = ("b", "d", "g", "r", "unknown", "w")
DEPTH_BLOCKS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}
STAGE_WIDTHS = (64, 128, 256, 512)
BN_EPS = 1e-5
INPUT_SIZE, EDGE, CROP = 224, 256, 224  # classify_patches input_size; ResizeEdge(256); CenterCrop(224)


def _kpad(k):
    return (k + 31) // 32 * 32


def make_random_weights(depth=152, num_classes=6, seed=0):
    """Seeded random weights under mmpretrain's ResNet state_dict names, with non-trivial BN statistics (no
    checkpoint is available offline)."""
    g = torch.Generator().manual_seed(seed)

    def conv(co, ci, k):
        return torch.randn(co, ci, k, k, generator=g) * (2.0 / (ci * k * k)) ** 0.5

    def bn(prefix, c, sd, gamma=1.0):
        sd[prefix + ".weight"] = gamma * (1 + 0.1 * torch.randn(c, generator=g))
        sd[prefix + ".bias"] = 0.1 * torch.randn(c, generator=g)
        sd[prefix + ".running_mean"] = 0.1 * torch.randn(c, generator=g)
        sd[prefix + ".running_var"] = 1 + 0.2 * torch.rand(c, generator=g)
        sd[prefix + ".num_batches_tracked"] = torch.tensor(1)

    sd = {}
    sd["backbone.conv1.weight"] = conv(64, 3, 7)
    bn("backbone.bn1", 64, sd)
    cin = 64
    for si, nb in enumerate(DEPTH_BLOCKS[depth]):
        w = STAGE_WIDTHS[si]
        for bi in range(nb):
            p = f"backbone.layer{si + 1}.{bi}"
            sd[p + ".conv1.weight"] = conv(w, cin, 1)
            bn(p + ".bn1", w, sd)
            sd[p + ".conv2.weight"] = conv(w, w, 3)
            bn(p + ".bn2", w, sd)
            sd[p + ".conv3.weight"] = conv(4 * w, w, 1)
            bn(p + ".bn3", 4 * w, sd, gamma=0.3)  # residual branches start small, as in a trained net
            if bi == 0:
                sd[p + ".downsample.0.weight"] = conv(4 * w, cin, 1)
                bn(p + ".downsample.1", 4 * w, sd)
            cin = 4 * w
    sd["head.fc.weight"] = torch.randn(num_classes, 2048, generator=g) * (1.0 / 2048) ** 0.5
    sd["head.fc.bias"] = 0.1 * torch.randn(num_classes, generator=g)
    return sd


def patch_bounds(shape, box):
    """``img[y1:y2, x1:x2]`` for an int box with Python slice semantics -> (y0, y1, x0, x1) or None if empty
    (classify_patches then reports label -1, score 0)."""
    x1, y1, x2, y2 = (int(v) for v in box)
    H, W = shape[:2]
    ys, xs = range(H)[slice(y1, y2)], range(W)[slice(x1, x2)]
    if len(ys) == 0 or len(xs) == 0:
        return None
    return ys.start, ys.stop, xs.start, xs.stop


def fold_conv_bn(weights, conv, bn):
    """Eval-mode BatchNorm folded into the bias-free convolution before it: W' = W * s, b' = beta - mean * s with
    s = gamma / sqrt(var + eps); W' as the GEMM operand [Cout][(ky * kw + kx) * Cin + c], K zero-padded to a
    multiple of 32.  Returns f32 (W', b') on the host."""
    w = weights[conv].detach().float()
    s = weights[bn + ".weight"].float() / torch.sqrt(weights[bn + ".running_var"].float() + BN_EPS)
    b = weights[bn + ".bias"].float() - weights[bn + ".running_mean"].float() * s
    co, ci, kh, kw = w.shape
    k = kh * kw * ci
    wm = (w * s[:, None, None, None]).permute(0, 2, 3, 1).reshape(co, k)
    return torch.nn.functional.pad(wm, (0, _kpad(k) - k)).contiguous(), b.contiguous()


class ResNetIdHip:
    """ResNet-``depth`` ID classifier.  ``weights``: mmpretrain state_dict names -> float tensors."""

    def __init__(self, weights, depth=152, num_classes=6, device: int = 0, classes=ID_CLASSES):
        if num_classes > 16:
            raise ValueError("at most 16 classes (mq_id_head)")
        self.depth, self.num_classes, self.classes = depth, num_classes, tuple(classes)
        self.dev = torch.device("cuda", device)
        self.ctx = _lib.Context.get(device)
        d = self.dev

        def fold(conv, bn, stride, pad):
            wm, b = fold_conv_bn(weights, conv, bn)
            co, ci, kh, kw = weights[conv].shape
            return dict(w=wm.to(d).to(torch.bfloat16).contiguous(), b=b.to(d), co=co, ci=ci, kh=kh, kw=kw,
                        stride=stride, pad=pad, kpad=wm.shape[1])

        self.stem = fold("backbone.conv1.weight", "backbone.bn1", 2, 3)
        self.blocks = []
        for si, nb in enumerate(DEPTH_BLOCKS[depth]):
            for bi in range(nb):
                p = f"backbone.layer{si + 1}.{bi}"
                stride = 2 if (bi == 0 and si > 0) else 1
                blk = dict(c1=fold(p + ".conv1.weight", p + ".bn1", 1, 0),
                           c2=fold(p + ".conv2.weight", p + ".bn2", stride, 1),
                           c3=fold(p + ".conv3.weight", p + ".bn3", 1, 0), stride=stride)
                if bi == 0:
                    blk["down"] = fold(p + ".downsample.0.weight", p + ".downsample.1", stride, 0)
                self.blocks.append(blk)
        self.implicit_conv = True  # 3x3 / strided 1x1 convolutions as implicit GEMMs (False: im2col + GEMM)
        self.fc_w = weights["head.fc.weight"].detach().float().contiguous().to(d)
        self.fc_b = weights["head.fc.bias"].detach().float().contiguous().to(d)

    # ------------------------------------------------------------------ launch helpers
    def _s(self):
        return _lib.stream_ptr(self.dev)

    def _gemm(self, A, cv, C, M, epi):
        _lib.check(self.ctx.lib.mq_gemm_bf16(self.ctx.handle, _lib.ptr(A), _lib.ptr(cv["w"]), _lib.ptr(C),
                                             _lib.ptr(cv["b"]), None, M, cv["co"], cv["kpad"], cv["kpad"],
                                             cv["kpad"], cv["co"], 0, epi, self._s()), "mq_gemm_bf16")

    def _conv(self, x, n, h, w, cv, epi, dtype=torch.bfloat16):
        """k x k / stride convolution of the NHWC bf16 map x: an implicit GEMM when the input channels are a
        multiple of 64 (every 3x3 and strided 1x1 of the bottlenecks), else im2col + GEMM (the stem);
        both give the same bits.  Returns (y (n*oh*ow, co), oh, ow)."""
        oh = (h + 2 * cv["pad"] - cv["kh"]) // cv["stride"] + 1
        ow = (w + 2 * cv["pad"] - cv["kw"]) // cv["stride"] + 1
        y = torch.empty((n * oh * ow, cv["co"]), device=self.dev, dtype=dtype)
        if self.implicit_conv and cv["ci"] % 64 == 0 and cv["kh"] == cv["kw"] and cv["kpad"] == cv["kh"] ** 2 * cv["ci"]:
            _lib.check(self.ctx.lib.mq_id_conv_bf16(self.ctx.handle, _lib.ptr(x), n, h, w, cv["ci"], cv["kh"],
                                                    cv["stride"], cv["pad"], _lib.ptr(cv["w"]), _lib.ptr(cv["b"]),
                                                    _lib.ptr(y), cv["co"], epi, self._s()), "mq_id_conv_bf16")
        else:
            cols, _, _ = self._im2col(x, n, h, w, cv)
            self._gemm(cols, cv, y, n * oh * ow, epi)
        return y, oh, ow

    def _im2col(self, x, n, h, w, cv):
        oh = (h + 2 * cv["pad"] - cv["kh"]) // cv["stride"] + 1
        ow = (w + 2 * cv["pad"] - cv["kw"]) // cv["stride"] + 1
        out = torch.empty((n * oh * ow, cv["kpad"]), device=self.dev, dtype=torch.bfloat16)
        _lib.check(self.ctx.lib.mq_id_im2col(self.ctx.handle, _lib.ptr(x), n, h, w, cv["ci"], cv["kh"], cv["kw"],
                                             cv["stride"], cv["pad"], cv["kpad"], _lib.ptr(out), self._s()),
                   "mq_id_im2col")
        return out, oh, ow

    # ------------------------------------------------------------------ stages
    def preprocess(self, frames, boxes):
        """frames u8 (V, H, W, 3) on the device; boxes int (n, 5) = (view, x0, y0, x1, y1) non-empty slices
        -> normalised bf16 NHWC (n, 224, 224, 3) and the 224x224 u8 patches."""
        V, H, W, _ = frames.shape
        n = len(boxes)
        b = np.asarray(boxes, dtype=np.int64).reshape(n, 5)
        ok = ((b[:, 0] >= 0) & (b[:, 0] < V) & (b[:, 1] >= 0) & (b[:, 1] < b[:, 3]) & (b[:, 3] <= W) &
              (b[:, 2] >= 0) & (b[:, 2] < b[:, 4]) & (b[:, 4] <= H))
        if n == 0 or not ok.all():
            raise ValueError("boxes must be non-empty slices inside their frame: (view, x0, y0, x1, y1)")
        bx = torch.as_tensor(b.astype(np.int32)).to(self.dev)
        pat = torch.empty((n, INPUT_SIZE, INPUT_SIZE, 3), device=self.dev, dtype=torch.uint8)
        _lib.check(self.ctx.lib.mq_id_crop_resize(self.ctx.handle, _lib.ptr(frames), H * W * 3, H, W, _lib.ptr(bx), n,
                                                  INPUT_SIZE, _lib.ptr(pat), self._s()), "mq_id_crop_resize")
        x = torch.empty((n, CROP, CROP, 3), device=self.dev, dtype=torch.bfloat16)
        _lib.check(self.ctx.lib.mq_id_preprocess(self.ctx.handle, _lib.ptr(pat), n, INPUT_SIZE, EDGE, CROP,
                                                 _lib.ptr(x), self._s()), "mq_id_preprocess")
        return x, pat

    def forward(self, x):
        """x bf16 NHWC (n, 224, 224, 3) -> logits, probs f32 (n, num_classes) on the device."""
        n, h, w, _ = x.shape
        cols, h, w = self._im2col(x, n, h, w, self.stem)
        y = torch.empty((n * h * w, 64), device=self.dev, dtype=torch.bfloat16)
        self._gemm(cols, self.stem, y, n * h * w, EPI_RELU)
        oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        a = torch.empty((n * oh * ow, 64), device=self.dev, dtype=torch.bfloat16)
        _lib.check(self.ctx.lib.mq_id_maxpool(self.ctx.handle, _lib.ptr(y), n, h, w, 64, _lib.ptr(a), self._s()),
                   "mq_id_maxpool")
        h, w = oh, ow
        xs = None  # f32 residual stream of the current stage
        for blk in self.blocks:
            c1, c2, c3 = blk["c1"], blk["c2"], blk["c3"]
            M = n * h * w
            h1 = torch.empty((M, c1["co"]), device=self.dev, dtype=torch.bfloat16)
            self._gemm(a, c1, h1, M, EPI_RELU)
            h2, oh, ow = self._conv(h1, n, h, w, c2, EPI_RELU)
            Mo = n * oh * ow
            if "down" in blk:
                dn = blk["down"]
                if dn["stride"] == 1:
                    xs = torch.empty((Mo, dn["co"]), device=self.dev, dtype=torch.float32)
                    self._gemm(a, dn, xs, Mo, EPI_F32)
                else:
                    xs = self._conv(a, n, h, w, dn, EPI_F32, dtype=torch.float32)[0]
            # conv3 + residual + ReLU in one epilogue: the f32 stream and the next block's bf16 operand
            a = torch.empty((Mo, c3["co"]), device=self.dev, dtype=torch.bfloat16)
            _lib.check(self.ctx.lib.mq_gemm_resid_relu_bf16(self.ctx.handle, _lib.ptr(h2), _lib.ptr(c3["w"]),
                                                            _lib.ptr(xs), _lib.ptr(c3["b"]), _lib.ptr(a), Mo,
                                                            c3["co"], c3["kpad"], c3["kpad"], c3["kpad"], c3["co"],
                                                            self._s()), "mq_gemm_resid_relu_bf16")
            h, w = oh, ow
        logits = torch.empty((n, self.num_classes), device=self.dev, dtype=torch.float32)
        probs = torch.empty_like(logits)
        _lib.check(self.ctx.lib.mq_id_head(self.ctx.handle, _lib.ptr(xs), n, h * w, xs.shape[1], _lib.ptr(self.fc_w),
                                           _lib.ptr(self.fc_b), self.num_classes, _lib.ptr(logits), _lib.ptr(probs),
                                           self._s()), "mq_id_head")
        return logits, probs

    def classify(self, frames, boxes_per_view):
        """All tracked boxes of all views of a frame in one batch.  frames u8 (V, H, W, 3) (numpy or device),
        boxes_per_view[v]: int (n_v, 4) xyxy -> per view a list of {pred_label, pred_score}."""
        if not torch.is_tensor(frames) or frames.device != self.dev:
            frames = torch.as_tensor(np.ascontiguousarray(frames)).to(self.dev)
        frames = frames.contiguous()
        out, rows, where = [], [], []
        for v, bxs in enumerate(boxes_per_view):
            res = [{"pred_label": -1, "pred_score": 0.0} for _ in range(len(bxs))]
            out.append(res)
            for i, b in enumerate(np.asarray(bxs).reshape(-1, 4)):
                pb = patch_bounds(frames.shape[1:3], b)
                if pb is not None:
                    y0, y1, x0, x1 = pb
                    rows.append((v, x0, y0, x1, y1))
                    where.append((v, i))
        if rows:
            x, _ = self.preprocess(frames, rows)
            _, probs = self.forward(x)
            p = probs.cpu().numpy()
            for (v, i), pr in zip(where, p):
                out[v][i] = {"pred_label": int(np.argmax(pr)), "pred_score": float(np.max(pr))}
        return out


    def classify_patches(self, patches):
        """classify_patches (step1_proc2d.py:140-163) on a list of HxWx3 uint8 BGR patches: every non-empty one
        resized and classified in one batch -> [{pred_label, pred_score}] (label -1, score 0 for empty)."""
        out = [{"pred_label": -1, "pred_score": 0.0} for _ in patches]
        valid = [i for i, p in enumerate(patches) if p.shape[0] > 0 and p.shape[1] > 0]
        if not valid:
            return out
        pat = torch.empty((len(valid), INPUT_SIZE, INPUT_SIZE, 3), device=self.dev, dtype=torch.uint8)
        for j, i in enumerate(valid):
            p = torch.as_tensor(np.ascontiguousarray(patches[i])).to(self.dev)
            h, w = p.shape[:2]
            bx = torch.tensor([[0, 0, 0, w, h]], dtype=torch.int32).to(self.dev)
            _lib.check(self.ctx.lib.mq_id_crop_resize(self.ctx.handle, _lib.ptr(p), h * w * 3, h, w, _lib.ptr(bx), 1,
                                                      INPUT_SIZE, _lib.ptr(pat[j]), self._s()), "mq_id_crop_resize")
        x = torch.empty((len(valid), CROP, CROP, 3), device=self.dev, dtype=torch.bfloat16)
        _lib.check(self.ctx.lib.mq_id_preprocess(self.ctx.handle, _lib.ptr(pat), len(valid), INPUT_SIZE, EDGE, CROP,
                                                 _lib.ptr(x), self._s()), "mq_id_preprocess")
        _, probs = self.forward(x)
        pr = probs.cpu().numpy()
        for j, i in enumerate(valid):
            out[i] = {"pred_label": int(np.argmax(pr[j])), "pred_score": float(np.max(pr[j]))}
        return out


def init_id_model(weights=None, device: int = 0, depth=152):
    """The model ``init_id_model`` returns (step1_proc2d.py:125-136), with random weights when none are given."""
    return ResNetIdHip(weights if weights is not None else make_random_weights(depth), depth=depth, device=device)
