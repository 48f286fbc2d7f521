"""ctypes binding of libmq_hip.so (include/mq_hip.h).

The shared library is built in-tree (``macaque-3d-pose-estimation_amd/lib/``) by
``__graft_entry__.build()`` / ``make -C macaque-3d-pose-estimation_amd/csrc``.
There is no CPU fallback: if the library or a GPU is missing, every product call
raises ``MqError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "lib", "libmq_hip.so"))
ABI_VERSION = 8  # include/mq_hip.h MQ_ABI_VERSION

EXPORTED = [
    "mq_abi_version", "mq_last_error", "mq_set_tuning", "mq_get_tuning", "mq_create", "mq_destroy",
    "mq_vitpose_create", "mq_vitpose_destroy", "mq_vitpose_set_param", "mq_vitpose_finalize",
    "mq_vitpose_set_graph", "mq_vitpose_timing", "mq_vitpose_timing_result", "mq_crop_udp", "mq_vitpose_forward", "mq_decode_udp", "mq_topdown",
    "mq_gemm_bf16", "mq_omnidir_undistort", "mq_omnidir_project", "mq_camera_undistort", "mq_camera_project", "mq_triangulate_dlt", "mq_reproj_error",
    "mq_triangulate_ransac", "mq_triangulate_pinv", "mq_geometry_affinity", "mq_match_svt", "mq_viterbi_filter",
    "mq_det_resize_patch", "mq_layernorm", "mq_add_layernorm", "mq_window_attention", "mq_patch_merge_gather", "mq_upsample_add",
    "mq_im2col3x3", "mq_conv3x3_bf16", "mq_gemm_resid_relu_bf16", "mq_id_conv_bf16", "mq_deconv_subpixel_pack", "mq_deconv_subpixel_bf16", "mq_f32_to_bf16", "mq_subsample2", "mq_nms", "mq_rpn_proposals", "mq_roi_align", "mq_rcnn_post", "mq_det_topk_boxes", "mq_optim_prepare", "mq_trust_region_2d", "mq_optim_points", "mq_attention_bf16", "mq_alldata_json",
    "mq_id_crop_resize", "mq_id_preprocess", "mq_id_im2col", "mq_id_maxpool", "mq_id_relu_bf16", "mq_id_head",
]


class MqError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_int64
f64 = C.c_double
f32 = C.c_float

_SIGS = {
    "mq_abi_version": (i32, []),
    "mq_alldata_json": (i32, [i32, vp, vp, vp, vp, i32, vp, vp, vp, i64, C.POINTER(i64)]),
    "mq_last_error": (C.c_char_p, []),
    "mq_set_tuning": (i32, [i32, i32]),
    "mq_get_tuning": (i32, [i32]),
    "mq_create": (i32, [i32, C.POINTER(vp)]),
    "mq_destroy": (i32, [vp]),
    "mq_vitpose_create": (i32, [vp, i32, i32, i32, i32, i32, C.POINTER(vp)]),
    "mq_vitpose_destroy": (i32, [vp]),
    "mq_vitpose_set_param": (i32, [vp, C.c_char_p, vp, i64, i32]),
    "mq_vitpose_finalize": (i32, [vp]),
    "mq_vitpose_set_graph": (i32, [vp, i32]),
    "mq_vitpose_timing": (i32, [vp, i32]),
    "mq_vitpose_timing_result": (i32, [vp, C.POINTER(f64), C.POINTER(i32), C.POINTER(i64)]),
    "mq_crop_udp": (i32, [vp, vp, i64, i32, i32, vp, vp, i32, vp, vp, vp, vp]),
    "mq_vitpose_forward": (i32, [vp, vp, i32, i32, vp, vp]),
    "mq_decode_udp": (i32, [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]),
    "mq_topdown": (i32, [vp, vp, i64, i32, i32, vp, vp, i32, i32, vp, vp, vp, vp, vp]),
    "mq_gemm_bf16": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
    "mq_omnidir_undistort": (i32, [vp, vp, i32, vp, i32, vp, vp]),
    "mq_omnidir_project": (i32, [vp, vp, i32, vp, i32, vp, vp]),
    "mq_camera_undistort": (i32, [vp, vp, i32, vp, i32, vp, vp]),
    "mq_camera_project": (i32, [vp, vp, i32, vp, i32, vp, vp]),
    "mq_triangulate_dlt": (i32, [vp, vp, i32, vp, i32, i32, vp, vp]),
    "mq_reproj_error": (i32, [vp, vp, i32, vp, vp, i32, i32, vp, vp]),
    "mq_triangulate_ransac": (i32, [vp, vp, i32, vp, i32, i32, f64, vp, vp, vp, vp, vp]),
    "mq_triangulate_pinv": (i32, [vp, vp, i32, vp, vp, i32, vp, vp]),
    "mq_geometry_affinity": (i32, [vp, vp, i32, vp, vp, i32, i32, i32, f64, vp, vp]),
    "mq_match_svt": (i32, [vp, vp, vp, vp, i32, i32, f64, f64, f64, f64, i32, i32, vp, vp, vp, vp]),
    "mq_det_resize_patch": (i32, [vp, vp, i64, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]),
    "mq_layernorm": (i32, [vp, vp, vp, vp, vp, i32, i32, f32, i32, vp]),
    "mq_add_layernorm": (i32, [vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, f32, vp]),
    "mq_window_attention": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mq_patch_merge_gather": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "mq_upsample_add": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mq_im2col3x3": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "mq_conv3x3_bf16": (i32, [vp, vp, i32, i32, i32, i32, vp, vp, vp, i32, i32, i32, vp]),
    "mq_deconv_subpixel_pack": (i32, [vp, vp, vp, vp, i32, i32, vp]),
    "mq_gemm_resid_relu_bf16": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mq_id_conv_bf16": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, i32, i32, vp]),
    "mq_deconv_subpixel_bf16": (i32, [vp, vp, i32, i32, i32, i32, vp, vp, vp, i32, i32, vp]),
    "mq_f32_to_bf16": (i32, [vp, vp, vp, i64, vp]),
    "mq_subsample2": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "mq_nms": (i32, [vp, vp, vp, vp, vp, i32, i32, f32, i32, vp, vp, vp]),
    "mq_id_crop_resize": (i32, [vp, vp, i64, i32, i32, vp, i32, i32, vp, vp]),
    "mq_id_preprocess": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "mq_id_im2col": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
    "mq_id_maxpool": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "mq_id_relu_bf16": (i32, [vp, vp, vp, i64, vp]),
    "mq_id_head": (i32, [vp, vp, i32, i32, i32, vp, vp, i32, vp, vp, vp]),
    "mq_rpn_proposals": (i32, [vp, vp, i32, i32, vp, vp, vp, i32, f32, f32, f32, i32, vp, vp, vp, vp]),
    "mq_roi_align": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp]),
    "mq_rcnn_post": (i32, [vp, vp, vp, vp, i32, i32, f32, f32, f32, f32, f32, f32, i32, vp, vp, vp, vp]),
    "mq_det_topk_boxes": (i32, [vp, vp, vp, vp, i32, i32, i32, f32, f64, f64, f64, vp, vp, vp, vp, vp]),
    "mq_optim_prepare": (i32, [vp, i32, i32, i32, vp, i32, i32, f64, vp, vp]),
    "mq_trust_region_2d": (i32, [vp, vp, f64, vp]),
    "mq_viterbi_filter": (i32, [vp, vp, i32, i32, i32, i32, f64, i32, f64, vp, vp]),
    "mq_attention_bf16": (i32, [vp, vp, vp, i32, i32, i32, i32, vp]),
    "mq_optim_points": (i32, [vp, vp, i32, vp, vp, i32, i32, i32, vp, i32, i32, vp, f64, f64, f64, i32, i32, i32,
                              i32, f64, i32, vp, vp]),
}


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library with every signature bound."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise MqError(f"libmq_hip.so not found at {path}: run __graft_entry__.build() "
                          f"or `make -C macaque-3d-pose-estimation_amd/csrc` first")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.mq_abi_version() != ABI_VERSION:
            raise MqError("libmq_hip ABI version mismatch")
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.mq_last_error().decode() if _lib is not None else "?"
        raise MqError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Raw device/host pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def apply_tuning_env(lib) -> None:
    """MQ_TUNING="key=value,key=value" (include/mq_hip.h MQ_TUNE_* keys): kernel-routing knobs for
    A/B runs in the measurement tools (tools/).  Product code never reads the environment: every
    knob the library accepts gives the same results, but nothing is switched behind a caller."""
    spec = os.environ.get("MQ_TUNING", "").strip()
    if not spec:
        return
    for item in spec.split(","):
        k, v = item.split("=")
        check(lib.mq_set_tuning(int(k), int(v)), f"mq_set_tuning({k}, {v})")


class Context:
    """One mq_ctx per device (threading)."""

    _per_device: dict = {}

    def __init__(self, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise MqError("no HIP device visible: the MI355X path has no CPU fallback")
        self.lib = load()
        self.device = device
        h = C.c_void_p()
        check(self.lib.mq_create(device, C.byref(h)), "mq_create")
        self.handle = h

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        ctx = cls._per_device.get(device)
        if ctx is None:
            ctx = cls(device)
            cls._per_device[device] = ctx
        return ctx

    def __del__(self):
        try:
            if getattr(self, "handle", None) is not None and _lib is not None:
                _lib.mq_destroy(self.handle)
        except Exception:
            pass
