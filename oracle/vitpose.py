"""ORACLE (test infrastructure only): float32 PyTorch restatement of ViTPose top-down.

Restates the model selected by
``/root/reference/model/pose/td-hm_ViTPose-huge_8xb64-210e_coco-256x192_sn_macaque.py``:54-110
as mmpretrain 1.2.0 ``VisionTransformer`` + mmpose 1.3.2 ``HeatmapHead`` /
``TopdownPoseEstimator`` compute it at eval time (neither library is installed here,
so parity against them is UNPINNED -- see DESIGN.md):

* patch embed: Conv2d(3, D, k16, s16, padding 2) -> 16x12 = 192 tokens, + pos_embed
  (no cls token, no pre-norm, dropouts/drop-path off at eval),
* L x pre-LN encoder layers (LN eps 1e-6): ``x += proj(softmax(q k^T / sqrt(dh)) v)``,
  ``x += fc2(GELU_erf(fc1(ln2 x)))``; final ``ln1``; out_type 'featmap' -> (B, D, 16, 12),
* head: 2 x [ConvTranspose2d(k4, s2, p1, no bias) -> BatchNorm2d(eps 1e-5, eval) -> ReLU],
  Conv2d 1x1 -> (B, 17, 64, 48),
* flip test: second forward on ``x.flip(-1)``, heatmaps flipped back on W and
  re-indexed by the macaque flip pairs (``model/pose/macaque.py``:15-130), averaged.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def vit_features(x, w, cfg):
    """x (B,3,256,192) float32 normalised -> final-LN tokens (B, T, D)."""
    D, H = cfg.embed_dims, cfg.num_heads
    dh = D // H
    y = F.conv2d(x, w["backbone.patch_embed.projection.weight"], w["backbone.patch_embed.projection.bias"],
                 stride=cfg.patch, padding=cfg.patch_pad)
    B = y.shape[0]
    t = y.flatten(2).transpose(1, 2)  # (B, T, D)
    t = t + w["backbone.pos_embed"]
    for i in range(cfg.num_layers):
        p = f"backbone.layers.{i}."
        h = F.layer_norm(t, (D,), w[p + "ln1.weight"], w[p + "ln1.bias"], cfg.ln_eps)
        qkv = F.linear(h, w[p + "attn.qkv.weight"], w[p + "attn.qkv.bias"])
        qkv = qkv.reshape(B, -1, 3, H, dh).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        att = torch.softmax((q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(dh)), dim=-1)
        o = (att @ v).transpose(1, 2).reshape(B, -1, D)
        t = t + F.linear(o, w[p + "attn.proj.weight"], w[p + "attn.proj.bias"])
        h = F.layer_norm(t, (D,), w[p + "ln2.weight"], w[p + "ln2.bias"], cfg.ln_eps)
        h = F.gelu(F.linear(h, w[p + "ffn.layers.0.0.weight"], w[p + "ffn.layers.0.0.bias"]))
        t = t + F.linear(h, w[p + "ffn.layers.1.weight"], w[p + "ffn.layers.1.bias"])
    t = F.layer_norm(t, (D,), w["backbone.ln1.weight"], w["backbone.ln1.bias"], cfg.ln_eps)
    return t


def heatmap_head(t, w, cfg):
    """tokens (B,T,D) -> heatmaps (B,17,64,48)."""
    B = t.shape[0]
    gh, gw = cfg.grid
    x = t.transpose(1, 2).reshape(B, cfg.embed_dims, gh, gw)
    for dc, bn in ((0, 1), (3, 4)):
        x = F.conv_transpose2d(x, w[f"head.deconv_layers.{dc}.weight"], None, stride=2, padding=1)
        x = F.batch_norm(x, w[f"head.deconv_layers.{bn}.running_mean"], w[f"head.deconv_layers.{bn}.running_var"],
                         w[f"head.deconv_layers.{bn}.weight"], w[f"head.deconv_layers.{bn}.bias"],
                         training=False, eps=cfg.bn_eps)
        x = F.relu(x)
    return F.conv2d(x, w["head.final_layer.weight"], w["head.final_layer.bias"])


def forward_heatmaps(x, w, cfg):
    return heatmap_head(vit_features(x, w, cfg), w, cfg)


def forward_flip_test(x, w, cfg, flip_indices=None):
    """TopdownPoseEstimator flip test: returns (avg, plain, flipped_raw) heatmaps."""
    from .decode import FLIP_INDICES
    fi = FLIP_INDICES if flip_indices is None else flip_indices
    h = forward_heatmaps(x, w, cfg)
    hf_raw = forward_heatmaps(x.flip(-1), w, cfg)
    hf = hf_raw.flip(-1)[:, fi]
    return (h + hf) * 0.5, h, hf_raw
