"""GPU: BASELINE config 3 end to end -- a 300-frame x 8-view x 4-individual clip (cameras at 2048x1536)
through ``run_demo.proc`` with the real ViTPose-H (seeded random weights, head made confident so the
3D stage has work) and the ResNet-152 ID classifier of each camera's variant:

  step 1 (crop -> ViT-H flip test -> UDP decode, ID) -> alldata.json -> step 3's kp2d writer (known
  assignment) -> step 4 (Viterbi, DLT, optim_points) -> kp3d.pickle          (run_demo.py:21-30)

Parity: the frame-sharded path (time steps split over ranks, one all-gather of the raw 2D keypoints,
the EMA post-process on the gathered clip, steps 3-4 on rank 0) must reproduce the single-process
run BIT FOR BIT -- every alldata.json, kp2d.pickle, kp2d_f.pickle and kp3d.pickle:
  * world 1 through the sharded code path, in this process;
  * world 2 as two fresh processes under torch.distributed.run sharing device 0 (gloo; RCCL refuses
    two ranks on one GPU), which checks that a different batch composition per rank changes no bit.
The single-process kp2d / kp3d themselves are checked against the oracle composition elsewhere
(test_gpu_run_demo.py for the 2D stage, test_gpu_pipeline.py for step 4 at this clip size).
"""
import json
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

N_FRAMES, N_VIEWS, N_ANIMALS = 300, 8, 4


@pytest.fixture(scope="module")
def clip(tmp_path_factory):
    from mqhip import synth
    root = tmp_path_factory.mktemp("config3")
    cams, raw, res, cfg, truth = synth.write_clip(str(root), "clip", n_frames=N_FRAMES, n_views=N_VIEWS,
                                                  n_animals=N_ANIMALS)
    return str(root), raw, cfg


def _results(root, name):
    res = os.path.join(root, name)
    os.makedirs(os.path.join(res, "clip"), exist_ok=True)
    shutil.copy(os.path.join(root, "results3D", "clip", "calibration.toml"), os.path.join(res, "clip"))
    return res


@pytest.fixture(scope="module")
def pose():
    import torch
    from mqhip import synth
    from mqhip.apis import PoseModelHip
    from mqhip.weights import VIT_H, make_random_weights
    w = synth.confident_head(make_random_weights(VIT_H, seed=0, device=torch.device("cuda", 0)))
    return PoseModelHip(VIT_H, w, 0)


@pytest.fixture(scope="module")
def single(clip, pose):
    import run_demo
    root, raw, cfg = clip
    res = _results(root, "res_single")
    data = run_demo.proc("clip", 24, res, "cuda:0", cfg, raw, 17, n_animal=N_ANIMALS, pose_model=pose,
                         id_model="random")
    return res, data


def _assert_same_outputs(a, b, cams):
    from mqhip import io as mqio
    for cam in cams:
        with open(os.path.join(a, "clip", cam, "alldata.json")) as f:
            ra = f.read()
        with open(os.path.join(b, "clip", cam, "alldata.json")) as f:
            rb = f.read()
        assert ra == rb, cam
        np.testing.assert_array_equal(np.load(os.path.join(a, "clip", cam, "frame_num.npy")),
                                      np.load(os.path.join(b, "clip", cam, "frame_num.npy")))
    for name in ("kp2d.pickle", "kp2d_f.pickle"):
        x = mqio.load_array_pickle(os.path.join(a, "clip", name))
        y = mqio.load_array_pickle(os.path.join(b, "clip", name))
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), name
    ka = mqio.load_array_pickle(os.path.join(a, "clip", "kp3d.pickle"))
    kb = mqio.load_array_pickle(os.path.join(b, "clip", "kp3d.pickle"))
    for k in ("kp3d", "kp3d_score", "kp3d_err"):
        x, y = np.asarray(ka[k]), np.asarray(kb[k])
        assert x.shape == y.shape and x.dtype == y.dtype and x.tobytes() == y.tobytes(), k  # bitwise, NaNs too
    np.testing.assert_array_equal(np.asarray(ka["joint_len"]), np.asarray(kb["joint_len"]))


def test_config3_single_process_clip_is_populated(clip, single):
    """The clip really exercises the chain: every time step has 32 boxes, step 4 triangulates and
    refines most joints (optim_points runs: the clip has far more than 20 points per animal)."""
    from mqhip import io as mqio
    from src.pipeline.step3_crossframematching import camera_ids
    root, raw, cfg = clip
    res, data = single
    cams = camera_ids(cfg)
    assert len(cams) == N_VIEWS
    with open(os.path.join(res, "clip", cams[0], "alldata.json")) as f:
        rows = json.load(f)
    assert len(rows) == N_FRAMES and all(len(r) == N_ANIMALS for r in rows)
    assert all(r[6] in range(-1, 6) and 0 <= r[7] <= 1 for fr in rows for r in fr)   # ID columns
    kp2d = mqio.load_array_pickle(os.path.join(res, "clip", "kp2d.pickle"))
    assert kp2d.shape == (N_ANIMALS, N_FRAMES, N_VIEWS, 17, 3)
    assert data["kp3d"].shape == (N_ANIMALS, N_FRAMES, 17, 3)
    assert np.isfinite(data["kp3d"]).mean() > 0.5
    assert len(data["joint_len"]) == N_ANIMALS


def test_config3_world1_sharded_equals_single_process(clip, single, pose):
    import run_demo
    from src.pipeline.step3_crossframematching import camera_ids
    root, raw, cfg = clip
    res = _results(root, "res_world1")
    times = {}
    run_demo.proc("clip", 24, res, "cuda:0", cfg, raw, 17, n_animal=N_ANIMALS, pose_model=pose, id_model="random",
                  world=1, rank=0, sharded=True, timings=times)
    _assert_same_outputs(single[0], res, camera_ids(cfg))
    # steps 3-4 took step 1's rows in memory: the kp2d.pickle they wrote equals step 3 run on the files
    from mqhip import io as mqio
    from src.pipeline import step3_crossframematching as step3
    mem = mqio.load_array_pickle(os.path.join(res, "clip", "kp2d.pickle"))
    np.testing.assert_array_equal(step3.proc_known_assignment("clip", res, cfg, n_animal=N_ANIMALS), mem)
    print("config-3 world-1 sharded timings:", times)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(900)
def test_config3_two_ranks_shared_gpu_equals_single_process(clip, single):
    """Two fresh processes (torch.distributed.run, gloo) on device 0, the same CLI the 8-GPU run uses
    (tools/run_clip_sharded.py -> run_demo.proc(world=2, rank=r)); rank 0's files equal the
    single-process run bit for bit."""
    from src.pipeline.step3_crossframematching import camera_ids
    root, raw, cfg = clip
    res = os.path.join(root, "res_world2")
    env = dict(os.environ, MQ_DIST_BACKEND="gloo", MQ_SHARE_GPU="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tools", "run_clip_sharded.py"), "--root", root, "--results", res]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=800)
    assert p.returncode == 0, p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    info = json.loads(line)
    assert info["world"] == 2 and info["frames"] == N_FRAMES
    _assert_same_outputs(single[0], res, camera_ids(cfg))


def test_run_pose_id_equals_separate_passes(clip, pose):
    """step 1's single-upload batch loop (run_pose_id: each batch's frames uploaded once, pose crops and
    ID patches cut from that copy) gives run_pose's keypoints / scores and run_id's predictions bit for bit
    on the first 24 time steps of the clip (3 batches, 8 cameras, each camera's ID variant)."""
    import glob

    from mqhip.io import FrameStore
    from src.pipeline import step1_proc2d as s1
    root, raw_dir, cfg = clip
    stores = [FrameStore(os.path.dirname(p)) for p in sorted(glob.glob(os.path.join(raw_dir, "clip.*", "metadata.yaml")))]
    md0 = stores[0].get_frame_metadata()
    T = np.arange(md0["frame_time"][0], md0["frame_time"][-1], 1.0 / 24)
    _, jobs = s1.plan_jobs(stores, T)
    ids = s1.resolve_id_models(stores, "random", "cuda:0")
    steps = range(24)
    raw_a = s1.run_pose(pose, stores, jobs, steps, 8)
    id_a = s1.run_id(ids, stores, jobs, steps, 8)
    raw_b, id_b = s1.run_pose_id(pose, ids, stores, jobs, steps, 8)
    assert raw_a.keys() == raw_b.keys() and len(raw_a) > 0
    for k in raw_a:
        assert np.array_equal(raw_a[k][0], raw_b[k][0]) and np.array_equal(raw_a[k][1], raw_b[k][1]), k
    assert id_a == id_b and len(id_a) == len(raw_a)
