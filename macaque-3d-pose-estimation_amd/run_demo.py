"""run_demo.proc mirror (reference run_demo.py:21-39) for the 2D->3D hot path.

The reference chains step 1 (detect / track / pose / ID) -> step 2 (cross-view association) ->
step 3 (cross-frame association, kp2d.pickle) -> step 4 (2D filter + 3D lift) -> visualisation,
and imports the Cython ``pictorial`` module (run_demo.py:3-11) that no step calls.

This build runs the same chain on MI355X with the parts outside its scope replaced by data:

* step 1 (``src.pipeline.step1_proc2d.proc``): the pose slice over every camera's frame store
  and the ID classifier of each camera's variant; the detector / tracker output arrives as the
  stores' tracker rows;
* steps 2-3: association is bypassed -- ``kp2d.pickle`` is written by step 3's own
  ``create_kp2dfile`` from a known track -> individual map
  (``src.pipeline.step3_crossframematching.proc_known_assignment``);
* step 4 (``src.pipeline.step4_aniposefiltering.proc``): unchanged drop-in;
* visualisation (video rendering) is out of scope and the ``pictorial`` import is not needed.

Multi-GPU (BASELINE config 3): run one process per GPU under ``torch.distributed.run``; every rank
calls ``proc(..., world=W, rank=r, group=g)``.  Step 1's time steps are sharded over the ranks with
one all-gather of the 2D keypoints (RCCL over xGMI); rank 0 runs step 3, and step 4 runs on every rank for
its individuals (individual a on rank a mod world -- step 4 couples the frames of an individual, not the
individuals), whose results one object all-gather brings to rank 0.  The files and kp3d equal the
single-process run bit for bit (tests/test_gpu_config3.py).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \\
        run_demo.py --data example --raw ./videos --results ./results3D --config ./calib/config.yaml
"""
import argparse
import os

from src.pipeline import step1_proc2d as step1
from src.pipeline import step3_crossframematching as step3
from src.pipeline import step4_aniposefiltering as step4


def proc(data_name, fps, results_dir_root, device_str, config_path, raw_data_dir, n_kp, vidfile_prefix='',
         n_animal=4, track_to_animal=None, pose_model=None, id_model="auto", world=1, rank=0, group=None,
         sharded=False, gather_device=None, timings=None):
    """run_demo.py:21-30: step 1 -> (known assignment) -> step 4; returns step 4's kp3d dict (on rank 0;
    None on the other ranks of a sharded run).  ``timings``: optional dict filled with wall seconds per
    stage.

    Steps 3-4 take step 1's rows in memory (the files are still written, by a background thread joined
    before returning).  On a sharded run (``world`` > 1 or ``sharded``) rank r post-processes and writes
    the cameras c = r (mod world) and assembles their kp2d slices; one all-gather of the slices gives
    every rank step 3's array; rank 0 writes kp2d.pickle, every rank runs step 4 (Viterbi, DLT / RANSAC,
    optim_points: tens of ms of GPU work for a 300-frame clip) for the individuals a = r (mod world), and
    rank 0 assembles and writes step 4's files.  When step 1 had nothing to do (files present) steps 3-4
    read the files on rank 0, as the reference does."""
    import time
    device = int(device_str.split(':')[1]) if ':' in device_str else 0
    t0 = time.perf_counter()
    s1out = step1.proc(data_name, results_dir_root, raw_data_dir, device_str, fps, pose_model=pose_model,
                       id_model=id_model, world=world, rank=rank, group=group, sharded=sharded,
                       gather_device=gather_device, background_writes=True, timings=timings)
    t1 = time.perf_counter()
    try:
        kp2d = step3.kp2d_from_step1(s1out, step3.camera_ids(config_path), n_animal=n_animal, n_kp=n_kp,
                                     track_to_animal=track_to_animal, world=world if (world > 1 or sharded) else 1,
                                     group=group if (world > 1 or sharded) else None,
                                     device=gather_device if (world > 1 or sharded) else None)
        t2 = time.perf_counter()
        sharded_run = world > 1 or sharded
        if kp2d is None and sharded_run:
            # the file path of a sharded run (some cameras' outputs were already on disk): rank r
            # writes the cameras c = r (mod world), so every rank's writer must have finished before rank 0
            # reads any file (the decision above is the same on every rank: same stores, same files)
            if s1out is not None:
                s1out.wait()
            _barrier(group)
        # step 4 over the ranks (individual a on rank a mod world, the results assembled on rank 0) when every
        # rank holds the gathered keypoints; the file path (kp2d None) runs it on rank 0 alone
        split = sharded_run and kp2d is not None and world > 1
        if rank != 0 and not split:
            return None
        result_dir = os.path.join(results_dir_root, data_name)
        if kp2d is None:
            if s1out is not None:
                s1out.wait()               # the files are the input of the file path
            kp2d = step3.proc_known_assignment(data_name, results_dir_root, config_path, n_animal=n_animal,
                                               n_kp=n_kp, track_to_animal=track_to_animal)
        elif rank == 0:
            from mqhip import io as mqio
            os.makedirs(result_dir, exist_ok=True)
            mqio.dump_pickle(kp2d, os.path.join(result_dir, "kp2d.pickle"))
        t3 = time.perf_counter()
        out = step4.proc(data_name, results_dir_root, config_path, n_kp, redo=True, device=device, kp2d=kp2d,
                         world=world if split else 1, rank=rank if split else 0, group=group if split else None)
        t4 = time.perf_counter()
    finally:
        if s1out is not None:
            s1out.wait()
    t5 = time.perf_counter()
    if timings is not None:
        timings.update(step1_s=t1 - t0, step3_s=t3 - t1, step4_s=t4 - t3, kp2d_gather_s=t2 - t1,
                       after_step1_s=t4 - t1, files_join_s=t5 - t4)
        if "gather_end" in timings:   # the sharded path: rank 0's timeline after the keypoint all-gather
            timings["after_gather_s"] = t4 - timings.pop("gather_end")
    return out


def _barrier(group):
    """A barrier over the run's ranks when a process group exists (a ``sharded`` run at world 1 has none)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=group)


def _dist_from_env(backend=None):
    """torch.distributed.run environment -> (world, rank, local_rank, group, gather_device).  Backend
    "nccl" (RCCL over xGMI, one GPU per rank) unless MQ_DIST_BACKEND=gloo (host tensors: a rehearsal
    of several ranks on one GPU, MQ_SHARE_GPU=1).  MQ_DIST_FORCE=1 builds the process group also at world
    size 1 (an RCCL rehearsal of the gather on a one-GPU box; never needed for a real run)."""
    import datetime

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or os.environ.get("MQ_DIST_BACKEND", "nccl")
    if os.environ.get("MQ_SHARE_GPU") == "1":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world == 1 and os.environ.get("MQ_DIST_FORCE") != "1":
        return 1, 0, local, None, None
    # rank 0 runs step 4 alone after the last collective while the others wait in the closing barrier:
    # a timeout well past any clip's step 4
    timeout = datetime.timedelta(seconds=float(os.environ.get("MQ_DIST_TIMEOUT_S", "7200")))
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        return world, rank, local, None, torch.device("cuda", local)
    dist.init_process_group(backend, timeout=timeout)
    return world, rank, local, None, None


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default="example")
    ap.add_argument("--fps", type=float, default=24)
    ap.add_argument("--results", default="./results3D")
    ap.add_argument("--config", default="./calib/config.yaml")
    ap.add_argument("--raw", default="./videos")
    ap.add_argument("--n-kp", type=int, default=17)
    a = ap.parse_args()
    W, R, L, G, dev = _dist_from_env()
    proc(a.data, a.fps, a.results, f"cuda:{L}", a.config, a.raw, a.n_kp, world=W, rank=R, group=G,
         gather_device=dev)
    if W > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
