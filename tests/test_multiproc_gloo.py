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


def _tail_worker(rank, world, port, root, res, cam_order, q):
    import sys
    from types import SimpleNamespace
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "macaque-3d-pose-estimation_amd")]
    import torch.distributed as dist
    from _fakes import fake_pose_batch
    from src.pipeline import step1_proc2d as s1
    from src.pipeline import step3_crossframematching as step3
    s1.inference_topdown_batch = fake_pose_batch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stub = SimpleNamespace(cfg=SimpleNamespace(n_joints=17))
        out = s1.step1_proc2d_custom("demo", res, root, pose_model=stub, world=world, rank=rank,
                                     steps_per_batch=4, background_writes=True)
        kp2d = step3.kp2d_from_step1(out, cam_order, n_animal=2, world=world)
        out.wait()
        q.put((rank, sorted(out.rows), kp2d))
    finally:
        dist.destroy_process_group()


def test_sharded_tail_world2_equals_single_rank_files(tmp_path):
    """VERDICT r3 item 4, the host half of the config-3 tail: rank r post-processes (KP_THR / EMA) and
    writes alldata.json for the cameras c = r (mod 2) only; step 3's kp2d is assembled per camera from the
    rows in memory on the owning rank and all-gathered (gloo), in config.yaml's camera order.  Every rank's
    kp2d and every written file equal the single-rank run that reads the files back (step3:872-915)."""
    import sys
    from types import SimpleNamespace
    import yaml
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from _fakes import fake_pose_batch, make_stores
    from src.pipeline import step1_proc2d as s1
    from src.pipeline import step3_crossframematching as step3
    make_stores(str(tmp_path), n_cams=3, n_frames=23, seed=5)
    cam_order = ["1002", "1000", "1001"]
    cfg = tmp_path / "config.yaml"
    cfg.write_text(yaml.safe_dump({"camera_id": [int(c) for c in cam_order]}))
    ref_res = str(tmp_path / "res_single")
    orig = s1.inference_topdown_batch
    s1.inference_topdown_batch = fake_pose_batch
    try:
        stub = SimpleNamespace(cfg=SimpleNamespace(n_joints=17))
        single = s1.step1_proc2d_custom("demo", ref_res, str(tmp_path), pose_model=stub, steps_per_batch=5)
        ref = step3.proc_known_assignment("demo", ref_res, str(cfg), n_animal=2)
        mem = step3.kp2d_from_step1(single, cam_order, n_animal=2)
    finally:
        s1.inference_topdown_batch = orig
    assert np.abs(ref[..., 2]).sum() > 0                          # the fake model's rows reach kp2d
    np.testing.assert_array_equal(mem, ref)                       # in memory == re-read files, world 1
    res = str(tmp_path / "res_w2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tail_worker, args=(r, 2, port, str(tmp_path), res, cam_order, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = {r: own for r, own, _ in got}
    assert owned == {0: [0, 2], 1: [1]}                          # stores demo.1000/1001/1002 -> c = r (mod 2)
    for _, _, kp2d in got:
        np.testing.assert_array_equal(kp2d, ref)
    for cam in ("1000", "1001", "1002"):
        for name in ("alldata.json", "frame_num.npy"):
            a = open(os.path.join(ref_res, "demo", cam, name), "rb").read()
            b = open(os.path.join(res, "demo", cam, name), "rb").read()
            assert a == b, (cam, name)
