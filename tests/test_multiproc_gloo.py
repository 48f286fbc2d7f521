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


def _fake_filter_2d(kp2d, filter_config=None, device=0):
    """CPU stand-in for step 4's Viterbi filter: the (A,F,C,J,3) -> (F,J,A,3,C) layout, per individual."""
    return np.ascontiguousarray(np.asarray(kp2d).transpose(1, 3, 0, 4, 2))


def _fake_reconstruct_3d(kp2d_f, cgroup, config, bodyparts=None, joint_len_median=None, verbose=False,
                         return_run=False):
    """CPU stand-in for step 4's lift (the GPU part): a deterministic function of each individual's own 2D, with
    `run` (the refined individuals) depending on the data, so the split / assembly is exercised as on the GPU."""
    kp = np.asarray(kp2d_f).transpose(2, 4, 0, 1, 3)                     # (A, C, F, J, 3)
    kp3d = kp.mean(axis=1)
    S = kp[..., 2].min(axis=1)
    E = kp[..., 0].std(axis=1)
    run = [a for a in range(kp.shape[0]) if np.nansum(np.abs(kp3d[a])) > 0]
    jl = [kp3d[a].reshape(-1)[:5].copy() for a in run]
    return (kp3d, S, E, jl, run) if return_run else (kp3d, S, E, jl)


class _FakeCameraGroup:
    @staticmethod
    def load(path, device=0):
        return _FakeCameraGroup()

    def subset_cameras_names(self, names):
        return self


def _demo_worker(rank, world, port, raw, res, cfg, fps, slow_rank, q, n_animal=2):
    """run_demo.proc on one gloo rank with the fake pose model.  Step 4 runs for real -- its split of the
    individuals over the ranks, the object all-gather and rank 0's assembly and files -- with its GPU stages
    (Viterbi filter, lift, camera loading) replaced by deterministic per-individual CPU stand-ins."""
    import sys
    import time
    from types import SimpleNamespace
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(os.path.dirname(here), "macaque-3d-pose-estimation_amd")
    sys.path[:0] = [here, pkg]
    import torch.distributed as dist
    from _fakes import fake_pose_batch
    import run_demo
    from src.pipeline import step1_proc2d as s1
    from src.pipeline import step4_aniposefiltering as step4
    s1.inference_topdown_batch = fake_pose_batch
    step4.filter_2d = _fake_filter_2d
    step4.reconstruct_3d = _fake_reconstruct_3d
    step4.CameraGroup = _FakeCameraGroup
    if rank == 0:                  # (step 4 needs a calibration.toml when there is no cam_intrinsic.h5)
        os.makedirs(os.path.join(res, "demo"), exist_ok=True)
        open(os.path.join(res, "demo", "calibration.toml"), "w").close()
    if rank == slow_rank:          # a slow writer: rank 0 must not read the files before it has finished
        orig = s1._write_step1_files

        def slow(*a, **k):
            time.sleep(2.0)
            return orig(*a, **k)
        s1._write_step1_files = slow
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stub = SimpleNamespace(cfg=SimpleNamespace(n_joints=17))
        tm = {}
        out = run_demo.proc("demo", fps, res, "cuda:0", cfg, raw, 17, n_animal=n_animal, pose_model=stub, id_model=None,
                            world=world, rank=rank, timings=tm)
        q.put((rank, out, sorted(tm)))
    finally:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()


def _run_demo_ranks(world, raw, res, cfg, fps, slow_rank=-1, n_animal=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_demo_worker, args=(r, world, port, raw, res, cfg, fps, slow_rank, q, n_animal))
             for r in range(world)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def _demo_inputs(tmp_path, n_cams, n_frames, steps=None):
    import yaml
    from _fakes import make_stores
    stores = make_stores(str(tmp_path / "raw"), n_cams=n_cams, n_frames=n_frames, seed=5)
    cams = [str(1000 + c) for c in range(n_cams)][::-1]          # config order differs from the store order
    cfg = tmp_path / "config.yaml"
    cfg.write_text(yaml.safe_dump({"camera_id": [int(c) for c in cams]}))
    t = stores[0].frame_time
    fps = 24.0 if steps is None else (steps - 0.5) / (t[-1] - t[0])
    return str(tmp_path / "raw"), str(cfg), fps, np.arange(t[0], t[-1], 1.0 / fps)


def _files(res, n_cams):
    return {(c, n): open(os.path.join(res, "demo", str(1000 + c), n), "rb").read()
            for c in range(n_cams) for n in ("alldata.json", "frame_num.npy")}


def _same_step4(a, b):
    assert sorted(a) == sorted(b)
    for k in ("kp3d", "kp3d_score", "kp3d_err"):
        np.testing.assert_array_equal(a[k], b[k])
    assert len(a["joint_len"]) == len(b["joint_len"])
    for x, y in zip(a["joint_len"], b["joint_len"]):
        np.testing.assert_array_equal(x, y)


def _step4_files(res):
    """Step 4's files (config.toml differs by the results path it records; kp3d.pickle is compared loaded, by
    _same_step4: its bytes also encode which arrays share a dtype object)."""
    return {n: open(os.path.join(res, "demo", n), "rb").read() for n in ("kp2d.pickle", "kp2d_f.pickle", "joint_len.npy")}


def test_run_demo_world8_config3_equals_single_rank(tmp_path):
    """the whole config-3 sharded path at world 8 (gloo, CPU): a 300-step clip split by
    frame_block(300, 8) (38 / 37 steps) through pose_clip_sharded, 3 cameras so ranks 3-7 own no camera
    (camera_shard / gather_cameras with empty parts), then step 4 split by individual (2 individuals: ranks 2-7
    own none) and assembled on rank 0.  Bit for bit the single-rank run: rank 0's step-4 data, every step-4 file,
    kp2d.pickle and every alldata.json / frame_num.npy."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from mqhip.shard import camera_shard, frame_block
    raw, cfg, fps, T = _demo_inputs(tmp_path, 3, 290, steps=300)
    assert len(T) == 300 and frame_block(300, 8, 0) == (0, 38) and frame_block(300, 8, 7) == (263, 300)
    assert [camera_shard(3, 8, r) for r in range(8)][3:] == [[]] * 5
    ref = _run_demo_ranks(1, raw, str(tmp_path / "res1"), cfg, fps)[0][1]
    got = _run_demo_ranks(8, raw, str(tmp_path / "res8"), cfg, fps)
    assert got[0][1] is not None and all(out is None for _, out, _ in got[1:])
    _same_step4(got[0][1], ref)
    assert np.nansum(np.abs(ref["kp3d"])) > 0 and len(ref["joint_len"]) == 2
    assert _files(str(tmp_path / "res1"), 3) == _files(str(tmp_path / "res8"), 3)
    assert _step4_files(str(tmp_path / "res1")) == _step4_files(str(tmp_path / "res8"))
    from mqhip import io as mqio
    _same_step4(mqio.load_array_pickle(os.path.join(tmp_path, "res8", "demo", "kp3d.pickle")), ref)
    assert "after_gather_s" in got[0][2]


def test_run_demo_world2_file_path_waits_for_every_writer(tmp_path):
    """when some cameras' outputs are already on disk, step 1 covers only the others and
    steps 3-4 read the files; rank 1 writes its cameras from a background thread (slowed down here), so rank 0
    may read only after every rank's writer has finished (run_demo's barrier).  Rank 0's step-4 input equals
    the single-rank run's."""
    import shutil
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    raw, cfg, fps, _ = _demo_inputs(tmp_path, 3, 23)
    ref = _run_demo_ranks(1, raw, str(tmp_path / "res1"), cfg, fps)[0][1]
    res = tmp_path / "res2"
    (res / "demo").mkdir(parents=True)
    shutil.copytree(tmp_path / "res1" / "demo" / "1001", res / "demo" / "1001")   # one camera already done
    got = _run_demo_ranks(2, raw, str(res), cfg, fps, slow_rank=1)
    _same_step4(got[0][1], ref)
    assert got[1][1] is None
    assert _files(str(tmp_path / "res1"), 3) == _files(str(res), 3)


def test_run_demo_world3_uneven_step4_split(tmp_path):
    """Step 4 split unevenly: 4 individuals over 3 ranks (individuals 0 and 3 on rank 0), two of them without a
    track (nothing to lift, so outside the refined set whose joint lengths are listed): rank 0's assembled data
    and step-4 files equal the single-rank run's."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    raw, cfg, fps, _ = _demo_inputs(tmp_path, 3, 23)
    ref = _run_demo_ranks(1, raw, str(tmp_path / "res1"), cfg, fps, n_animal=4)[0][1]
    got = _run_demo_ranks(3, raw, str(tmp_path / "res3"), cfg, fps, n_animal=4)
    assert got[0][1] is not None and got[1][1] is None and got[2][1] is None
    _same_step4(got[0][1], ref)
    assert ref["kp3d"].shape[0] == 4 and len(ref["joint_len"]) == 2
    assert _step4_files(str(tmp_path / "res1")) == _step4_files(str(tmp_path / "res3"))


def _step4_fail_worker(rank, world, port, res, cfg, stage, q):
    """step4.proc at world `world` over gloo with the CPU stand-ins, failing on purpose: "setup" -- rank 0 finds no
    calibration; "lift" -- rank 1's lift raises; "config" -- rank 1 cannot read config.yaml (before the
    first exchange).  Reports what each rank raised."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "macaque-3d-pose-estimation_amd")]
    import torch.distributed as dist
    from src.pipeline import step4_aniposefiltering as step4
    step4.filter_2d = _fake_filter_2d
    step4.CameraGroup = _FakeCameraGroup

    def lift(*a, **k):
        if rank == 1:
            raise ValueError("lift failed on purpose")
        return _fake_reconstruct_3d(*a, **k)
    step4.reconstruct_3d = lift
    if rank == 0 and stage == "lift":
        os.makedirs(os.path.join(res, "demo"), exist_ok=True)
        open(os.path.join(res, "demo", "calibration.toml"), "w").close()
    if stage == "config" and rank == 1:   # this rank's view of config.yaml is missing
        cfg = cfg + ".missing"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kp2d = np.random.default_rng(3).random((3, 6, 2, 17, 3))
        step4.proc("demo", res, cfg, 17, kp2d=kp2d, world=world, rank=rank)
        q.put((rank, "ok", ""))
    except Exception as e:  # noqa: BLE001
        q.put((rank, type(e).__name__, str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("stage", ["setup", "lift", "config"])
def test_step4_split_failure_raises_on_every_rank(tmp_path, stage):
    """A sharded step 4 whose setup (rank 0: no calibration) or lift (rank 1) fails raises on every rank instead of
    leaving the others waiting in the exchange: the failing rank its own exception, the others a RuntimeError
    naming it."""
    import yaml
    cfg = tmp_path / "config.yaml"
    cfg.write_text(yaml.safe_dump({"camera_id": [1000, 1001]}))
    res = str(tmp_path / "res")
    os.makedirs(os.path.join(res, "demo"), exist_ok=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step4_fail_worker, args=(r, 2, port, res, str(cfg), stage, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (kind, msg)) for r, kind, msg in [q.get(timeout=120) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
    bad = 0 if stage == "setup" else 1
    assert got[bad][0] == {"setup": "FileNotFoundError", "lift": "ValueError", "config": "FileNotFoundError"}[stage]
    other = 1 - bad
    assert got[other][0] == "RuntimeError" and f"rank(s) {bad}:" in got[other][1], got


# ---------------------------------------------------------------------------------------------------------------
# bench.py's N > 1 exchange: every rank's per-view 2D keypoints of its own frames -> the keypoint
# all-gather (mqhip.shard.gather_keypoints, as in bench.main) -> bench.clip_lift with the individuals split over the
# ranks.  The exchange logic runs for real over gloo; the lift's GPU stages are oracle stand-ins (oracle/viterbi.py's
# batched Viterbi for step 4's filter_2d, oracle/geometry.py's CameraGroupOracle DLT and reprojection error inside
# step 4's own reconstruct_3d, optim_points off).  The GPU-side checks of the same path stay in tests/test_gpu_*.

def _bench_rank_frames(rank, n_frames, cams):
    """A rank's (n_frames, C, A, J, 3) f32 keypoint log, laid out as bench.main's kp_log per frame."""
    from mqhip import synth
    kp = synth.make_kp2d(cams, synth.make_skeletons(4, n_frames, seed=2 + rank), seed=3 + rank)   # (A, F, C, J, 3)
    return np.ascontiguousarray(kp.transpose(1, 2, 0, 3, 4)).astype(np.float32)


def _bench_lift_setup():
    import bench
    from mqhip import io as mqio
    from oracle.viterbi import step4_filter_batched
    from src.pipeline import step4_aniposefiltering as step4
    step4.filter_2d = lambda kp2d, filter_config=None, device=0: step4_filter_batched(kp2d)
    cfg = mqio.load_toml(step4.CONFIG_TMPL)
    cfg["triangulation"]["optim"] = False
    cfg["triangulation"]["ransac"] = False
    return bench, cfg


def _bench_exchange_worker(rank, world, port, n_frames, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "macaque-3d-pose-estimation_amd")]
    import torch.distributed as dist
    from mqhip import synth
    from mqhip.shard import gather_keypoints
    from oracle.geometry import CameraGroupOracle
    bench, cfg = _bench_lift_setup()
    cams = synth.make_cameras(8)
    per_frame = torch.from_numpy(_bench_rank_frames(rank, n_frames, cams))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gathered = gather_keypoints(per_frame, world * n_frames, world)
        cl = bench.clip_lift(gathered.numpy(), cams, None, clips=world, rank=rank, world=world, config=cfg,
                             camera_group=CameraGroupOracle(cams), return_kp3d=True)
        q.put((rank, gathered.numpy(), cl["kp3d"], cl["individuals_per_rank"], cl["individuals"]))
    finally:
        dist.destroy_process_group()


def test_bench_exchange_world4_equals_single_rank():
    """World 4, 3 frames per rank (12 gathered frames = 4 clips x 4 individuals): every rank holds the same
    gathered keypoints, in rank-then-frame order, equal to the concatenation of the ranks' own logs; rank r lifts
    the individuals r, r + 4, ... of the 16 and its 3D joints equal the single-rank lift's rows bit for bit."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "macaque-3d-pose-estimation_amd")]
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle
    world, n_frames = 4, 3
    cams = synth.make_cameras(8)
    full = np.concatenate([_bench_rank_frames(r, n_frames, cams) for r in range(world)])
    bench, cfg = _bench_lift_setup()
    ref = bench.clip_lift(full, cams, None, clips=world, rank=0, world=1, config=cfg,
                          camera_group=CameraGroupOracle(cams), return_kp3d=True)["kp3d"]
    assert ref.shape == (world * 4, n_frames, 17, 3) and np.isfinite(ref).mean() > 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_exchange_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, gathered, kp3d, per_rank, total in got:
        np.testing.assert_array_equal(gathered, full)
        assert per_rank == 4 and total == 16
        np.testing.assert_array_equal(kp3d, ref[r::world])
