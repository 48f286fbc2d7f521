"""Step 4 -- 2D Viterbi filtering + anipose 3D lift, on MI355X (row a18 glue).

Mirrors ``src/pipeline/step4_aniposefiltering.py`` of the reference: same
``proc(data_name, results_dir_root, config_path, n_kp, redo)`` entry point, same
files in and out (``kp2d.pickle`` -> ``kp2d_f.pickle``, ``calibration.toml``,
``config.toml``, ``joint_len.npy``, ``kp3d.pickle`` / ``kp3d_fxdJointLen.pickle``)
and the same numbers, but batched MI355X-first:

* the Viterbi filter runs every (animal, camera, joint) chain in one launch
  (reference: a spawn pool per animal x camera, step4:145-167);
* initial triangulation / RANSAC / reprojection errors run over all animals'
  points in one launch each (reference: per animal, per point);
* optim_points refines all animals in one batched solve (reference: scipy
  per animal);
* on a sharded run (``world`` > 1, every rank holding the gathered kp2d) the
  individuals are split over the ranks (individual a on rank a mod world) and
  rank 0 assembles and writes the outputs: the same bits as one rank, since
  every stage is independent per individual.

Calibration: if the reference's ``cam_intrinsic.h5`` / ``cam_extrinsic_optim.h5``
sit next to ``config_path`` and h5py is importable, ``calibration.toml`` is
rebuilt from them as in step4:101-138; otherwise an existing
``<result_dir>/calibration.toml`` is used.
"""
from __future__ import annotations

import os

import numpy as np
import yaml

from mqhip import io as mqio
from mqhip.geometry import CameraGroup, viterbi_filter

BODYPARTS = ['nose', 'left_eye', 'right_eye', 'left_ear', 'right_ear',
             'left_shoulder', 'right_shoulder', 'left_elbow', 'right_elbow',
             'left_wrist', 'right_wrist', 'left_hip', 'right_hip',
             'left_knee', 'right_knee', 'left_ankle', 'right_ankle']

_HERE = os.path.dirname(os.path.abspath(__file__))
CONFIG_TMPL = os.path.join(_HERE, "..", "..", "configs", "config_tmpl.toml")

# cameras.py:1250: optim_points_jointlenfix runs scipy with max_nfev=15, i.e. the initial
# evaluation plus at most 14 trial steps; one LM iteration here is one trial evaluation.
JOINTLENFIX_MAX_TRIALS = 14   # LM solver: trial steps
JOINTLENFIX_MAX_NFEV = 15     # trf solver: scipy's max_nfev of optim_points_jointlenfix (cameras.py:1246-1260)

# step4:142-147 -- the filter settings are hard-coded there, not read from the TOML
FILTER_CONFIG = {"filter": {"score_threshold": 0.3, "n_back": 3, "offset_threshold": 25, "multiprocessing": True}}


def load_constraints(config, bodyparts, key='constraints'):
    """step4:40-49: bodypart-name pairs -> index pairs (AssertionError on unknown names)."""
    names = config['triangulation'].get(key, [])
    idx = {b: i for i, b in enumerate(bodyparts)}
    out = []
    for a, b in names:
        assert a in idx, 'Bodypart {} from constraints not found in list of bodyparts'.format(a)
        assert b in idx, 'Bodypart {} from constraints not found in list of bodyparts'.format(b)
        out.append([idx[a], idx[b]])
    return out


def _median_valid(p3, ix):
    pts = p3[:, ix]
    pts = pts[~np.isnan(pts[:, 0])]
    return np.median(pts, axis=0)


def correct_coordinate_frame(config, all_points_3d, bodyparts):
    """step4:51-87: rotate/translate into the frame named by triangulation.reference_point / axes."""
    bp = {b: i for i, b in enumerate(bodyparts)}
    axis_of = {'x': 0, 'y': 1, 'z': 2}
    ref = config['triangulation']['reference_point']
    (ad, al, ar), (bd, bl, br) = config['triangulation']['axes'][:2]
    a_dir, b_dir = axis_of[ad], axis_of[bd]
    c_dir = [i for i in range(3) if i not in (a_dir, b_dir)][0]
    a_vec = _median_valid(all_points_3d, bp[ar]) - _median_valid(all_points_3d, bp[al])
    b_raw = _median_valid(all_points_3d, bp[br]) - _median_valid(all_points_3d, bp[bl])
    b_vec = b_raw - a_vec * np.dot(b_raw, a_vec) / np.dot(a_vec, a_vec)
    M = np.zeros((3, 3))
    M[a_dir], M[b_dir] = a_vec, b_vec
    M[c_dir] = np.cross(a_vec, b_vec) if (a_dir, b_dir) in [(0, 1), (2, 0), (1, 2)] else np.cross(b_vec, a_vec)
    M /= np.linalg.norm(M, axis=1)[:, None]
    adj = all_points_3d.dot(M.T)
    center = _median_valid(adj, bp[ref])
    return adj - center, M, center


# configs/calibration_tmpl.toml of the reference: eight omnidir entries cam_0..cam_7 named "1".."8",
# zero intrinsics / extrinsics; step4:106 loads it and overwrites the fields of the listed cameras.
N_CALIB_TEMPLATE_CAMS = 8


def calibration_template(n_cams=N_CALIB_TEMPLATE_CAMS):
    """The reference's calibration template as a dict (key order = the template's)."""
    return {f'cam_{i}': {'name': str(i + 1), 'size': [2048, 1536], 'matrix': [[0.0] * 3 for _ in range(3)],
                         'distortions': [0.0] * 4, 'rotation': [0, 0, 0], 'translation': [0, 0, 0],
                         'fisheye': False, 'omnidir': True} for i in range(n_cams)}


def write_calibration(config_path, result_dir, cam_ids):
    """step4:101-138: calibration.toml from the h5 intrinsics / extrinsics (needs h5py).

    Same semantics as the reference: start from the 8-camera template, then per listed camera
    matrix = mtx with its first two rows halved (the h5 intrinsics are at 2x resolution),
    distortions / xi / D raveled, K as stored, name = the camera id; rotation / translation
    = the raveled rvec / tvec of cam_extrinsic_optim.h5.  Template entries past len(cam_ids)
    keep their zeros (step 4 subsets the group by name afterwards); a camera index past the
    template raises KeyError, as the reference's ``calib['cam_'+str(i_cam)]`` does."""
    import h5py  # absent in this image; only reached when the h5 files exist
    base = os.path.dirname(config_path)
    calib = calibration_template()
    with h5py.File(os.path.join(base, 'cam_intrinsic.h5'), 'r') as f:
        for i, k in enumerate(cam_ids):
            mtx = np.array(f[k]['mtx'][()])
            mtx[:2, :] /= 2
            ent = calib[f'cam_{i}']
            ent['matrix'] = mtx.tolist()
            ent['distortions'] = np.asarray(f[k]['dist'][()]).ravel().tolist()
            ent['name'] = k
            ent['xi'] = np.asarray(f[k]['xi'][()]).ravel().tolist()
            ent['K'] = np.asarray(f[k]['K'][()]).tolist()
            ent['D'] = np.asarray(f[k]['D'][()]).ravel().tolist()
    with h5py.File(os.path.join(base, 'cam_extrinsic_optim.h5'), 'r') as f:
        for i, k in enumerate(cam_ids):
            ent = calib[f'cam_{i}']
            ent['rotation'] = np.asarray(f[k]['rvec'][()]).ravel().tolist()
            ent['translation'] = np.asarray(f[k]['tvec'][()]).ravel().tolist()
            ent['name'] = k
    mqio.dump_toml(calib, os.path.join(result_dir, 'calibration.toml'))


def filter_2d(kp2d, filter_config=FILTER_CONFIG, device: int = 0):
    """step4:140-170: kp2d (A,F,C,J,3) -> kp2d_f (F,J,A,3,C) (filtered points + Viterbi scores)."""
    fc = filter_config['filter']
    out = viterbi_filter(kp2d, score_threshold=fc['score_threshold'], n_back=fc['n_back'],
                         offset_threshold=fc['offset_threshold'], device=device)
    return np.ascontiguousarray(out.transpose(1, 3, 0, 4, 2))


def reconstruct_3d(kp2d_f, cgroup, config, bodyparts=BODYPARTS, joint_len_median=None, verbose=False,
                   return_run=False):
    """step4:185-331 for all animals at once.  kp2d_f (F,J,A,3,C) ->
    (kp3d (A,F,J,3), S (A,F,J), E (A,F,J), joint_len list (one entry per refined animal, in animal order)
    [, the refined animals when ``return_run``])."""
    tri = config['triangulation']
    n_frame, n_kp, n_animal, _, n_cam = kp2d_f.shape
    kp = np.array(kp2d_f.transpose((2, 4, 0, 1, 3)), dtype=np.float64)   # (A,C,F,J,3)
    run = []
    pts_raw = kp[..., :2].copy()
    scores = kp[..., 2].copy()
    pts_raw[scores < tri['score_threshold']] = np.nan
    kp3d = np.zeros((n_animal, n_frame, n_kp, 3))
    S = np.zeros((n_animal, n_frame, n_kp))
    E = np.zeros((n_animal, n_frame, n_kp))
    joint_len = []
    # (C, A*F*J, 2): every animal's points in one launch; per-point results are independent
    flat = np.ascontiguousarray(pts_raw.transpose(1, 0, 2, 3, 4).reshape(n_cam, -1, 2))
    good = ~np.isnan(pts_raw[..., 0])                                     # (A,C,F,J)
    if tri['optim']:
        cons = load_constraints(config, bodyparts)
        weak = load_constraints(config, bodyparts, 'constraints_weak')
        if tri['ransac']:
            init = cgroup.triangulate_ransac(flat)[0]
        else:
            init = cgroup.triangulate(flat)
        init = init.reshape(n_animal, n_frame, n_kp, 3)
        p3 = init.copy()
        run = [a for a in range(n_animal) if np.sum(np.isfinite(init[a, :, :, 0])) >= 20]
        for a in range(n_animal):
            if a not in run:
                print("warning: not enough 3D points to run optimization")
        if run:
            from mqhip.optim import optim_points_batch
            jl_fix = None if joint_len_median is None else np.asarray(joint_len_median, dtype=np.float64)
            res, jls = optim_points_batch(
                cgroup, pts_raw[run], init[run], cons, weak, scale_smooth=tri['scale_smooth'],
                scale_length=tri['scale_length'], scale_length_weak=tri['scale_length_weak'],
                reproj_error_threshold=tri['reproj_error_threshold'], n_deriv_smooth=tri['n_deriv_smooth'],
                joint_len=jl_fix, max_iter=200 if jl_fix is None else JOINTLENFIX_MAX_TRIALS,
                max_nfev=None if jl_fix is None else JOINTLENFIX_MAX_NFEV, verbose=verbose)
            for i, a in enumerate(run):
                p3[a] = res[i]
                joint_len.append(jls[i] if jl_fix is None else jl_fix)
        p3_flat = np.ascontiguousarray(p3.reshape(-1, 3))
        err = cgroup.reprojection_error(p3_flat, flat, mean=True).reshape(n_animal, n_frame, n_kp)
        num_cams = good.sum(axis=1).astype(float)                         # (A,F,J)
        sc = scores.copy()
        sc[~good] = 2
        s3 = sc.min(axis=1)
        s3[num_cams < 1] = np.nan
        err[num_cams < 1] = np.nan
    else:
        if tri['ransac']:
            p3, picked, p2s, err = cgroup.triangulate_ransac(flat, min_cams=3)
            p2s = p2s.reshape(n_cam, n_animal, n_frame, n_kp, 2).transpose(1, 0, 2, 3, 4)
            good = ~np.isnan(p2s[..., 0])
            num_cams = picked.reshape(n_cam, n_animal, n_frame, n_kp).sum(axis=0).astype(float)
        else:
            p3 = cgroup.triangulate(flat)
            err = cgroup.reprojection_error(p3, flat, mean=True)
            num_cams = good.sum(axis=1).astype(float)
        p3 = p3.reshape(n_animal, n_frame, n_kp, 3)
        err = np.asarray(err, dtype=np.float64).reshape(n_animal, n_frame, n_kp)
        sc = scores.copy()
        sc[~good] = 2
        s3 = sc.min(axis=1)
        s3[num_cams < 2] = np.nan
        err[num_cams < 2] = np.nan
    for a in range(n_animal):
        if 'reference_point' in tri and 'axes' in tri:
            kp3d[a] = correct_coordinate_frame(config, p3[a], bodyparts)[0]
        else:
            kp3d[a] = p3[a]
        S[a] = s3[a]
        E[a] = err[a]
    if return_run:
        return kp3d, S, E, joint_len, run
    return kp3d, S, E, joint_len


def proc(data_name, results_dir_root, config_path, n_kp, redo=False, device: int = 0, verbose=False, kp2d=None,
         world=1, rank=0, group=None):
    """step4_aniposefiltering.proc (step4:89).  ``kp2d``: step 3's (A, F, C, J, 3) array in memory (as
    written to kp2d.pickle) instead of reading the file back.

    ``world`` > 1 (every rank calls this with the same gathered ``kp2d``): rank r filters and lifts the
    individuals a with a % world == r, one object all-gather brings their results to rank 0, which writes the
    files and returns the data (None elsewhere).  Rank 0 writes config.toml / calibration.toml before the other
    ranks read them.  An exception on any rank is raised on every rank (each waiting point exchanges the ranks'
    errors), so a failure ends the run instead of leaving the others waiting."""
    result_dir = results_dir_root + '/' + data_name
    fixed = os.path.exists(os.path.dirname(config_path) + '/joint_len.npy')
    out_name = 'kp3d_fxdJointLen.pickle' if fixed else 'kp3d.pickle'
    split = world > 1
    if split and kp2d is None:
        raise ValueError("step4.proc: a sharded run needs the gathered kp2d in memory on every rank")
    if split:
        # the ranks' objects (failures, per-individual results) travel over a gloo group: a rank whose device has
        # faulted can still report, and nothing waits on a collective over a dead device
        group = _object_group(group)

    def skip():
        return os.path.exists(os.path.join(result_dir, out_name)) and not redo

    def read_cam_ids():
        with open(config_path, 'r') as f:
            return [str(i) for i in yaml.safe_load(f)['camera_id']]

    if not split:
        if skip():
            print(f'Skip as exist:{data_name:s}/{out_name}')
            return
        cam_ids = read_cam_ids()
    else:
        # every rank reads the camera ids and rank 0 decides the skip, inside the first exchange: a rank that fails
        # here (a missing or malformed config.yaml) ends the run on every rank, and all ranks follow rank 0's skip
        own = _attempt(lambda: (read_cam_ids(), skip() if rank == 0 else None), rank)
        parts = _gather_objects(own if isinstance(own, _Failure) else (None if rank else own[1]), world, group)
        _raise_if_any(parts, own)
        cam_ids = own[0]
        if parts[0]:
            if rank == 0:
                print(f'Skip as exist:{data_name:s}/{out_name}')
            return None

    # ---- configuration + calibration (step4:101-138)
    def setup():
        config = mqio.load_toml(CONFIG_TMPL)
        config['model_folder'] = os.path.abspath(os.path.dirname(result_dir))
        mqio.dump_toml(config, result_dir + '/config.toml')
        h5_in = os.path.dirname(config_path) + '/cam_intrinsic.h5'
        if os.path.exists(h5_in):
            write_calibration(config_path, result_dir, cam_ids)
        elif not os.path.exists(result_dir + '/calibration.toml'):
            raise FileNotFoundError(f'need {h5_in} (+ h5py) or {result_dir}/calibration.toml')
    if not split:
        setup()
    else:
        own = _attempt(setup, rank) if rank == 0 else None
        _raise_if_any(_gather_objects(own, world, group), own)

    # ---- 2D filtering (step4:140-170)
    print('##### 2D filtering....', flush=True)
    if kp2d is None:
        kp2d = mqio.load_array_pickle(result_dir + '/kp2d.pickle')
    kp2d = np.asarray(kp2d, dtype=np.float64)
    n_animal = kp2d.shape[0]
    mine = [a for a in range(n_animal) if a % world == rank] if split else list(range(n_animal))
    joint_len_median = None
    if fixed:
        joint_len_median = np.median(np.load(os.path.dirname(config_path) + '/joint_len.npy'), axis=0)

    def lift():
        kp2d_f = filter_2d(kp2d[mine], device=device) if mine else None
        if not split:
            mqio.dump_pickle(kp2d_f, result_dir + '/kp2d_f.pickle')
        # ---- 3D reconstruction (step4:172-339)
        print('##### 3D reconstruction....', flush=True)
        config = mqio.load_toml(result_dir + '/config.toml')
        if not mine:
            return config, None
        cgroup = CameraGroup.load(result_dir + '/calibration.toml', device=device).subset_cameras_names(cam_ids)
        if not split:
            return config, (kp2d_f,) + tuple(reconstruct_3d(kp2d_f, cgroup, config, joint_len_median=joint_len_median,
                                                            verbose=verbose))
        kp3d, S, E, joint_len, run = reconstruct_3d(kp2d_f, cgroup, config, joint_len_median=joint_len_median,
                                                    verbose=verbose, return_run=True)
        return config, (mine, kp2d_f, kp3d, S, E, joint_len, [mine[i] for i in run])

    if not split:
        config, (kp2d_f, kp3d, S, E, joint_len) = lift()
    else:
        out = _attempt(lift, rank)
        parts = _gather_objects(out if isinstance(out, _Failure) else out[1], world, group)
        _raise_if_any(parts, out)
        if rank != 0:
            return None
        config = out[0]
        kp2d_f, kp3d, S, E, joint_len = _assemble(parts, n_animal)
        if joint_len_median is not None:   # as one rank builds it: the fixed lengths, once per refined individual
            jl_fix = np.asarray(joint_len_median, dtype=np.float64)
            joint_len = [jl_fix for _ in joint_len]
        mqio.dump_pickle(kp2d_f, result_dir + '/kp2d_f.pickle')
    if config['triangulation']['optim']:
        np.save(result_dir + '/joint_len.npy', np.array(joint_len))
    data = {'kp3d': kp3d, 'kp3d_score': S, 'kp3d_err': E, 'joint_len': joint_len}
    mqio.dump_pickle(data, os.path.join(result_dir, out_name))
    return data


class _Failure:
    """A rank's exception, as sent to the other ranks (the original object stays on its own rank)."""

    def __init__(self, rank, exc):
        self.rank, self.text = rank, f'{type(exc).__name__}: {exc}'
        self.exc = exc

    def __getstate__(self):
        return {'rank': self.rank, 'text': self.text, 'exc': None}


def _attempt(fn, rank):
    """fn() or the _Failure it raised (sent to every rank before anyone raises)."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 -- re-raised by _raise_if_any on every rank
        return _Failure(rank, e)


def _raise_if_any(parts, own):
    """After the exchange: this rank's own exception as it was raised, else one naming every failed rank."""
    if isinstance(own, _Failure):
        raise own.exc
    bad = [p for p in parts if isinstance(p, _Failure)]
    if not bad:
        return
    raise RuntimeError('step4.proc failed on rank(s) ' + '; '.join(f'{p.rank}: {p.text}' for p in bad))


_OBJECT_GROUPS = {}


def _object_group(group):
    """The group step 4's object exchanges use: the caller's group when it has one, the default group when that is
    gloo already, else a gloo group over every rank (created once, collectively, at the first sharded call)."""
    import datetime
    import torch.distributed as dist
    if group is not None or dist.get_backend() == 'gloo':
        return group
    key = dist.get_world_size()
    if key not in _OBJECT_GROUPS:
        timeout = datetime.timedelta(seconds=float(os.environ.get('MQ_DIST_TIMEOUT_S', '7200')))
        _OBJECT_GROUPS[key] = dist.new_group(backend='gloo', timeout=timeout)
    return _OBJECT_GROUPS[key]


def _gather_objects(obj, world, group):
    """Every rank's part (or None) on every rank, in rank order (torch.distributed.all_gather_object over the gloo
    object group: pickled numpy arrays through host memory)."""
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj, group=group)
    return out


def _assemble(parts, n_animal):
    """Rank 0: the ranks' per-individual results back in individual order -- kp2d_f (F,J,A,3,C), kp3d / S / E
    (A,...) and joint_len (one entry per refined individual, in individual order, as one rank produces it)."""
    first = next(p for p in parts if p is not None)
    kf0, k0, s0, e0 = first[1], first[2], first[3], first[4]
    kp2d_f = np.zeros(kf0.shape[:2] + (n_animal,) + kf0.shape[3:], dtype=kf0.dtype)
    kp3d = np.zeros((n_animal,) + k0.shape[1:], dtype=k0.dtype)
    S = np.zeros((n_animal,) + s0.shape[1:], dtype=s0.dtype)
    E = np.zeros((n_animal,) + e0.shape[1:], dtype=e0.dtype)
    jl = {}
    for p in parts:
        if p is None:
            continue
        mine, kf, k3, s3, e3, joint_len, run = p
        for i, a in enumerate(mine):
            kp2d_f[:, :, a] = kf[:, :, i]
            kp3d[a], S[a], E[a] = k3[i], s3[i], e3[i]
        for a, j in zip(run, joint_len):
            jl[a] = np.array(j, dtype=np.float64)
    return kp2d_f, kp3d, S, E, [jl[a] for a in sorted(jl)]
