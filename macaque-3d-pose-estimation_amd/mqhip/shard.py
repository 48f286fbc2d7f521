"""Frame sharding across GPUs: one process per GPU, contiguous frame blocks,
one collective -- the all-gather of per-view 2D keypoints before the temporally coupled
step-4 stages.

Everything per frame (crop -> ViT -> decode -> per-frame triangulation) is rank-local;
weights are replicated.  ``pose_clip_sharded`` is the clip driver of BASELINE config 3: step 1
over a clip's time steps sharded across ranks, one all-gather, then the sequential per-track
post-process and (by the caller) step 4 on the gathered keypoints.  ``gather_keypoints`` moves fixed-size per-rank buffers
([F_block, C, A, J, 3] f32, zero-padded to the largest block) so the collective is a single
RCCL all-gather over xGMI (backend "nccl") -- or gloo in the CPU tests.
"""
from __future__ import annotations

import torch


def frame_block(n_frames: int, world: int, rank: int):
    """Contiguous [start, stop) of rank's frames; the first n_frames % world ranks get one extra."""
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_keypoints(kp_local: torch.Tensor, n_frames: int, world: int, group=None):
    """kp_local (F_local, ...) on this rank -> (n_frames, ...) on every rank, in frame order."""
    import torch.distributed as dist
    block = frame_block(n_frames, world, 0)[1]          # largest block (rank 0 never has fewer)
    shape = (block,) + tuple(kp_local.shape[1:])
    buf = torch.zeros(shape, dtype=kp_local.dtype, device=kp_local.device)
    buf[:kp_local.shape[0]] = kp_local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = []
    for r in range(world):
        s, e = frame_block(n_frames, world, r)
        out.append(parts[r][:e - s])
    return torch.cat(out, dim=0)


def n_joints_of(pose_model, default=17):
    """Keypoints per instance of a pose model (PoseModelHip / VitPoseHip: cfg.n_joints; an mmpose-style
    model: dataset_meta['num_keypoints'])."""
    cfg = getattr(pose_model, "cfg", None)
    if cfg is not None and getattr(cfg, "n_joints", None):
        return int(cfg.n_joints)
    meta = getattr(pose_model, "dataset_meta", None) or {}
    return int(meta.get("num_keypoints", default))


def _all_gather(buf, world, group=None):
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return [buf]  # no process group (a process group of one, e.g. an RCCL rehearsal, still gathers)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return parts


def camera_shard(n_cams: int, world: int, rank: int):
    """The cameras whose post-process (KP_THR / EMA, alldata.json, step 3's kp2d slice) rank owns:
    c = rank (mod world)."""
    return list(range(rank, n_cams, world))


def gather_cameras(part, n_cams: int, world: int, group=None, device=None):
    """kp2d slices (A, F, C_own, J, 3) of every rank's ``camera_shard`` -> the whole (A, F, C, J, 3) on every
    rank: ONE all-gather of fixed-size buffers (padded to the largest shard; ~2 MB for a 300-frame clip)."""
    import numpy as np
    per = len(camera_shard(n_cams, world, 0))
    A, F, _, J, D = part.shape
    buf = torch.zeros((A, F, per, J, D), dtype=torch.float64)
    buf[:, :, :part.shape[2]] = torch.from_numpy(np.ascontiguousarray(part))
    if device is not None:
        buf = buf.to(device)
    parts = _all_gather(buf, world, group)
    out = np.zeros((A, F, n_cams, J, D))
    for r in range(world):
        own = camera_shard(n_cams, world, r)
        out[:, :, own] = parts[r][:, :, :len(own)].cpu().numpy()
    return out


def pose_clip_sharded(pose_model, stores, T, world: int, rank: int, group=None, steps_per_batch=8,
                      kp_params=None, device=None, id_model=None, tracks=None, cams=None, with_ids=False, timings=None, records=False):
    """BASELINE config 3: the step-1 pose slice of a clip, time steps sharded across ranks.

    Every rank walks the same per-camera time grid (``step1_proc2d.plan_jobs``); rank r runs the
    ViTPose jobs (and, with ``id_model``, the ID classification) of its contiguous block of time steps
    (``frame_block``); one all-gather moves every rank's raw keypoints and scores ([steps, C, boxes, J, 3]
    float64, padded to the largest block and box count; + [steps, C, boxes, 2] ID label / score) to every
    rank, which then runs the sequential KP_THR / EMA / alldata post-process over the whole clip -- the EMA
    is recursive in time per track, so it runs after the gather and the result equals the single-GPU
    ``process_stores`` exactly.  ``device``: where the gathered buffers live (a CUDA device for RCCL;
    None = host tensors, gloo).  ``world == 1`` needs no process group.  Returns what ``process_stores``
    returns (per camera: rows per kept frame, frame numbers); with ``cams`` only for those cameras (the
    post-process of the other cameras is left to their owning ranks, ``camera_shard``), aligned with
    ``cams``; ``with_ids`` adds every camera's kept-frame track ids (``step1_proc2d.kept_track_ids``); ``records``
    returns ``step1_proc2d.CameraRows`` per camera instead of row lists; ``timings``
    (dict) receives ``gather_end``, the perf_counter at which the all-gather completed."""
    import numpy as np
    from src.pipeline import step1_proc2d as s1
    kp_params = s1.KP_PARAMS if kp_params is None else kp_params
    plans, jobs = s1.plan_jobs(stores, T, kp_params, tracks)
    n_steps, C = len(T), len(stores)
    s0, e0 = frame_block(n_steps, world, rank)
    raw, id_raw = s1.run_pose_id(pose_model, id_model, stores, jobs, range(s0, e0), steps_per_batch)
    # the buffer shape must agree on every rank, also on a rank whose block holds no pose job:
    # take J from the model, never from this rank's results
    J = n_joints_of(pose_model)
    nb = max([len(j[2]) for js in jobs.values() for j in js] or [1])
    block = frame_block(n_steps, world, 0)[1]
    buf = torch.full((block, C, nb, J * 3 + 2), float("nan"), dtype=torch.float64)
    for (k, c), (kp, sc) in raw.items():
        n = len(kp)
        buf[k - s0, c, :n, :J * 3] = torch.from_numpy(
            np.concatenate([kp, sc.astype(np.float64)[..., None]], axis=-1).reshape(n, J * 3))
        if id_raw is not None:
            buf[k - s0, c, :n, J * 3:] = torch.tensor([[p["pred_label"], p["pred_score"]] for p in id_raw[(k, c)]],
                                                      dtype=torch.float64)
    if device is not None:
        buf = buf.to(device)
    parts = _all_gather(buf, world, group)
    if timings is not None:
        import time
        if device is not None:
            torch.cuda.synchronize(device)
        timings["gather_end"] = time.perf_counter()
    allraw, allid = {}, ({} if id_model is not None else None)
    keep = set(range(C) if cams is None else cams)
    for r in range(world):
        s, e = frame_block(n_steps, world, r)
        part = parts[r].cpu().numpy()
        for k in range(s, e):
            for (c, _, boxes, _, _) in jobs.get(k, []):
                if c not in keep:
                    continue
                v = part[k - s, c, :len(boxes)]
                kp = v[:, :J * 3].reshape(len(boxes), J, 3)
                allraw[(k, c)] = (kp[..., :2].copy(), kp[..., 2].astype(np.float32))
                if allid is not None:
                    allid[(k, c)] = [{"pred_label": int(lab), "pred_score": float(scr)} for lab, scr in v[:, J * 3:]]
    if records:  # step1_proc2d.CameraRows (arrays) instead of the nested row lists
        out = s1.assemble_records(stores, T, plans, jobs, allraw, kp_params, allid, cams=cams)
    else:
        out = s1.assemble_rows(stores, T, plans, jobs, allraw, kp_params, allid, cams=cams)
    if with_ids:
        return out, s1.kept_track_ids(stores, T, plans, jobs)
    return out
