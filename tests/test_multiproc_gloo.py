"""CPU, world_size 2 over gloo: the frame-shard partition and the 2D-keypoint all-gather
(mqhip.shard) that bench.py and the multi-GPU pipeline use between the per-frame pose stage
and the clip-level step-4 stages."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_frames, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "macaque-3d-pose-estimation_amd"))
    import torch.distributed as dist
    from mqhip.shard import frame_block, gather_keypoints
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(n_frames * 8 * 4 * 17 * 3, dtype=torch.float32).reshape(n_frames, 8, 4, 17, 3)
        s, e = frame_block(n_frames, world, rank)
        got = gather_keypoints(full[s:e].clone(), n_frames, world)
        q.put((rank, bool(torch.equal(got, full)), s, e))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [7, 300])
def test_gather_keypoints_world2(n_frames):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(ok for _, ok, _, _ in res)
    assert res[0][2] == 0 and res[0][3] == res[1][2] and res[1][3] == n_frames


def test_frame_block_partition():
    from mqhip.shard import frame_block
    for n in (1, 7, 37, 300):
        for w in (1, 2, 3, 8):
            blocks = [frame_block(n, w, r) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            sizes = [e - s for s, e in blocks]
            assert max(sizes) - min(sizes) <= 1 and sizes[0] == max(sizes)
    assert frame_block(300, 8, 0) == (0, 38) and frame_block(300, 8, 7) == (263, 300)


def _clip_worker(rank, world, port, root, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "macaque-3d-pose-estimation_amd")]
    import json
    import torch.distributed as dist
    from _fakes import fake_pose_batch, open_stores
    from mqhip.shard import pose_clip_sharded
    from src.pipeline import step1_proc2d as s1
    s1.inference_topdown_batch = fake_pose_batch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stores = open_stores(root)
        T = np.arange(stores[0].frame_time[0], stores[0].frame_time[-1], 1.0 / 24)
        got = pose_clip_sharded(None, stores, T, world, rank, steps_per_batch=4)
        q.put((rank, json.dumps(got)))
    finally:
        dist.destroy_process_group()


def test_pose_clip_sharded_world2_equals_single_rank(tmp_path):
    """BASELINE config 3's clip driver: time steps sharded over 2 ranks (gloo), one all-gather of
    the raw keypoints, then the sequential KP_THR / EMA post-process -- identical alldata rows on
    every rank and identical to the single-rank step-1 pass."""
    import json
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from _fakes import fake_pose_batch, make_stores
    from src.pipeline import step1_proc2d as s1
    stores = make_stores(str(tmp_path), n_cams=3, n_frames=23, seed=5)
    T = np.arange(stores[0].frame_time[0], stores[0].frame_time[-1], 1.0 / 24)
    orig = s1.inference_topdown_batch
    s1.inference_topdown_batch = fake_pose_batch
    try:
        ref = json.dumps(s1.process_stores(None, stores, T, steps_per_batch=5))
    finally:
        s1.inference_topdown_batch = orig
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_clip_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(T) > 10
    for _, got in res:
        assert got == ref
