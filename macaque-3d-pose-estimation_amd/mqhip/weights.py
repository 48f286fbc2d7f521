"""ViTPose weight sets in the mmpose state_dict naming ("Weights").

The real ``model/pose/pose.pth`` is not shipped with the reference (``.gitignore``:10,
README.md:86), so benchmarks and parity tests use seeded random weights.  Values are
rounded to bf16-representable float32 so that the bf16 HIP path and the float32
oracle see bit-identical parameters and differ only in activation rounding.

Key names follow mmpretrain ``VisionTransformer`` / mmpose ``HeatmapHead``:
``backbone.patch_embed.projection.*``, ``backbone.pos_embed``,
``backbone.layers.{i}.{ln1,attn.qkv,attn.proj,ln2,ffn.layers.0.0,ffn.layers.1}.*``,
``backbone.ln1.*``, ``head.deconv_layers.{0,1,3,4}.*``, ``head.final_layer.*``.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class VitPoseConfig:
    name: str
    embed_dims: int
    num_layers: int
    num_heads: int
    ffn: int
    img_h: int = 256
    img_w: int = 192
    patch: int = 16
    patch_pad: int = 2
    deconv_ch: int = 256
    n_joints: int = 17
    ln_eps: float = 1e-6
    bn_eps: float = 1e-5

    @property
    def grid(self):
        gh = (self.img_h + 2 * self.patch_pad - self.patch) // self.patch + 1
        gw = (self.img_w + 2 * self.patch_pad - self.patch) // self.patch + 1
        return gh, gw

    @property
    def tokens(self):
        gh, gw = self.grid
        return gh * gw

    @property
    def head_dim(self):
        return self.embed_dims // self.num_heads

    def flops_per_forward(self) -> int:
        """Algorithmic FLOPs of one forward (2 per MAC; elementwise ops excluded).

        ViT-H 256x192: 251,659,812,864 (BASELINE.md / SURVEY.md section 8(d))."""
        T, D, Fd = self.tokens, self.embed_dims, self.ffn
        gh, gw = self.grid
        patch = 2 * T * D * 3 * self.patch * self.patch
        layer = 2 * T * D * 3 * D + 2 * 2 * T * T * D + 2 * T * D * D + 2 * 2 * T * D * Fd
        c = self.deconv_ch
        dc1 = 2 * (gh * gw) * D * c * 16
        dc2 = 2 * (4 * gh * gw) * c * c * 16
        fin = 2 * (16 * gh * gw) * c * self.n_joints
        return patch + self.num_layers * layer + dc1 + dc2 + fin


VIT_H = VitPoseConfig("huge", 1280, 32, 16, 5120)
VIT_B = VitPoseConfig("base", 768, 12, 12, 3072)
VIT_TINY = VitPoseConfig("tiny", 320, 2, 4, 640)   # d_head 80 like ViT-H; for fast tests
CONFIGS = {c.name: c for c in (VIT_H, VIT_B, VIT_TINY)}


def _bf16(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


def make_random_weights(cfg: VitPoseConfig, seed: int = 0, device="cpu", std: float = 0.02):
    """Seeded random weights (trunc-normal-ish linear/conv, random LN/BN affine)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    D, Fd, T = cfg.embed_dims, cfg.ffn, cfg.tokens

    def rn(*shape, s=std, mean=0.0):
        x = torch.randn(*shape, generator=g, device=device, dtype=torch.float32)
        return _bf16(x.clamp_(-2.0, 2.0) * s + mean)

    def ru(*shape, lo=0.5, hi=1.5):
        x = torch.rand(*shape, generator=g, device=device, dtype=torch.float32)
        return _bf16(lo + (hi - lo) * x)

    w = {}
    w["backbone.patch_embed.projection.weight"] = rn(D, 3, cfg.patch, cfg.patch)
    w["backbone.patch_embed.projection.bias"] = rn(D)
    w["backbone.pos_embed"] = rn(1, T, D)
    for i in range(cfg.num_layers):
        p = f"backbone.layers.{i}."
        w[p + "ln1.weight"] = rn(D, s=0.1, mean=1.0)
        w[p + "ln1.bias"] = rn(D)
        w[p + "attn.qkv.weight"] = rn(3 * D, D)
        w[p + "attn.qkv.bias"] = rn(3 * D)
        w[p + "attn.proj.weight"] = rn(D, D)
        w[p + "attn.proj.bias"] = rn(D)
        w[p + "ln2.weight"] = rn(D, s=0.1, mean=1.0)
        w[p + "ln2.bias"] = rn(D)
        w[p + "ffn.layers.0.0.weight"] = rn(Fd, D)
        w[p + "ffn.layers.0.0.bias"] = rn(Fd)
        w[p + "ffn.layers.1.weight"] = rn(D, Fd)
        w[p + "ffn.layers.1.bias"] = rn(D)
    w["backbone.ln1.weight"] = rn(D, s=0.1, mean=1.0)
    w["backbone.ln1.bias"] = rn(D)
    c = cfg.deconv_ch
    w["head.deconv_layers.0.weight"] = rn(D, c, 4, 4)
    w["head.deconv_layers.1.weight"] = rn(c, s=0.1, mean=1.0)
    w["head.deconv_layers.1.bias"] = rn(c, s=0.1)
    w["head.deconv_layers.1.running_mean"] = rn(c, s=0.1)
    w["head.deconv_layers.1.running_var"] = ru(c)
    w["head.deconv_layers.3.weight"] = rn(c, c, 4, 4)
    w["head.deconv_layers.4.weight"] = rn(c, s=0.1, mean=1.0)
    w["head.deconv_layers.4.bias"] = rn(c, s=0.1)
    w["head.deconv_layers.4.running_mean"] = rn(c, s=0.1)
    w["head.deconv_layers.4.running_var"] = ru(c)
    w["head.final_layer.weight"] = rn(cfg.n_joints, c, 1, 1, s=0.05)
    w["head.final_layer.bias"] = rn(cfg.n_joints, s=0.05)
    return w


def load_mmpose_checkpoint(path: str):
    """Load a real mmpose ``pose.pth`` (weights_only, no pickle code) -> state_dict of f32 tensors."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck.get("state_dict", ck)
    return {k: v.float() for k, v in sd.items() if k.startswith(("backbone.", "head."))}
