"""Step 3 -- the kp2d.pickle writer of ``src/pipeline/step3_crossframematching.py``.

The reference's step 3 builds tracklets, stitches them with a min-cost flow and votes IDs
(step3_crossframematching.py:36-94, 313-402); that association is outside this build's scope
(SURVEY 8(f) row 2).  What the 3D lift consumes from it is ``kp2d.pickle``: (A, F, C, J, 3)
per-view keypoints of every individual, zero where an individual is not seen, written by
``create_kp2dfile`` (step3:872-915).  This module keeps that writer and its semantics, and
feeds it from a KNOWN track -> individual assignment instead of the association (the
benchmark's "association bypassed" path):

* ``load_alldata``: step 1's per-camera ``alldata.json`` rows, the T[i_cam][i_frame] of step 3;
* ``known_assignment``: Trk / Cid (step 3's per-track box ids per camera and individual ids)
  from a {track id -> individual} map (default: track id == individual index);
* ``create_kp2dfile``: step3:872-915 (every matching row of a camera is written, so the last one
  stays; zero fill);
* ``proc_known_assignment``: the three above for a results directory.

The reference hard-codes 4 individuals and 8 cameras (step3:879-880); here both come from the
arguments / the camera list of config.yaml, so the 4-view config 1 also runs.
"""
from __future__ import annotations

import json
import os

import numpy as np
import yaml

from mqhip import io as mqio


def camera_ids(config_path):
    with open(config_path, "r") as f:
        return [str(i) for i in yaml.safe_load(f)["camera_id"]]


def load_alldata(result_dir, cam_ids):
    """T[i_cam][i_frame] = list of rows [tid, x1, y1, x2, y2, [[x, y, s] x J], id, id_score]."""
    T = []
    for cam in cam_ids:
        with open(os.path.join(result_dir, cam, "alldata.json")) as f:
            T.append(json.load(f))
    return T


def track_ids(T):
    """Per camera, per frame, the track ids of the alldata rows T[i_cam][i_frame]."""
    return [[[int(row[0]) for row in frame] for frame in cam] for cam in T]


def default_track_map(T, n_animal, ids=None):
    """{track id -> individual} for the smallest ``n_animal`` track ids present in the alldata rows, in
    ascending order (synthetic stores number tracks from 0, the BoT-SORT tracker from 1).  ``ids``: the
    rows' track ids (``track_ids``) in place of the rows."""
    ids = track_ids(T) if ids is None else ids
    tids = sorted({t for cam in ids for frame in cam for t in frame})
    if not tids:  # nothing tracked: every individual stays zero-filled
        return {a: a for a in range(n_animal)}
    return {t: a for a, t in enumerate(tids[:n_animal])}


def known_assignment(T, n_animal, track_to_animal=None, ids=None):
    """Trk[k] (F, C) box id of track k in each camera (-1 = absent) and Cid[k] (F,) its individual,
    for a known {track id -> individual} map shared by all cameras (default: ``default_track_map``, the
    ``n_animal`` smallest track ids present -> 0..n_animal-1).  ``ids`` (``track_ids``) may stand in for
    the rows: a rank of a sharded run holds the rows of its own cameras only."""
    ids = track_ids(T) if ids is None else ids
    n_cam = len(ids)
    n_frame = len(ids[0])
    if track_to_animal is None:
        track_to_animal = default_track_map(None, n_animal, ids)
    Trk, Cid = {}, {}
    for tid, a in track_to_animal.items():
        trk = np.full((n_frame, n_cam), -1, dtype=np.int64)
        for c in range(n_cam):
            for f in range(min(n_frame, len(ids[c]))):
                if int(tid) in ids[c][f]:
                    trk[f, c] = int(tid)
        Trk[tid] = trk
        Cid[tid] = np.full(n_frame, int(a), dtype=np.int64)
    return Trk, Cid


def kp2d_of_camera(rows_c, Trk, Cid, i_cam, n_frame, n_animal=4, n_kp=17):
    """Camera ``i_cam``'s slice kp2d[:, :, i_cam] of create_kp2dfile (step3:872-915) from that camera's rows
    alone: the writer touches camera i_cam only through T[i_cam] and Trk[k][:, i_cam], so the cameras can
    be assembled independently (on different ranks) and stacked, with the same bits."""
    out = np.zeros([n_animal, n_frame, n_kp, 3])
    is_done = np.zeros([n_animal, n_frame], dtype=bool)
    for i_frame in range(n_frame):
        for k in Trk.keys():
            i_animal = Cid[k][i_frame]
            if i_animal < 0:
                continue
            trk = Trk[k][i_frame, :]
            if np.sum(trk >= 0) == 0 or is_done[i_animal, i_frame]:
                continue
            for tt in rows_c[i_frame]:
                if tt[0] == trk[i_cam]:
                    out[i_animal, i_frame, :, :] = np.array(tt[5], dtype=np.float64)
                    is_done[i_animal, i_frame] = True
    return out


def kp2d_of_camera_rows(cr, Trk, Cid, i_cam, n_frame, n_animal=4, n_kp=17):
    """``kp2d_of_camera`` from a camera's rows as arrays (``step1_proc2d.CameraRows``): the same selection --
    per frame and track (Trk order) the last row carrying the track's box id -- on the arrays, bit for bit."""
    out = np.zeros([n_animal, n_frame, n_kp, 3])
    is_done = np.zeros([n_animal, n_frame], dtype=bool)
    tid = cr.tid
    for i_frame in range(min(n_frame, len(cr))):
        a0, n = cr.frame(i_frame)
        if n == 0:
            continue
        ft = tid[a0:a0 + n]
        for k in Trk.keys():
            i_animal = Cid[k][i_frame]
            if i_animal < 0:
                continue
            trk = Trk[k][i_frame, :]
            if np.sum(trk >= 0) == 0 or is_done[i_animal, i_frame]:
                continue
            hit = np.nonzero(ft == trk[i_cam])[0]
            if len(hit):
                out[i_animal, i_frame] = cr.kp[a0 + hit[-1]]
                is_done[i_animal, i_frame] = True
    return out


def assemble_kp2d(T, Trk, Cid, n_animal=4, n_kp=17):
    """create_kp2dfile's (A, F, C, J, 3) array without writing it."""
    n_cam = len(T)
    n_frame = Trk[list(Trk.keys())[0]].shape[0]
    kp2d = np.zeros([n_animal, n_frame, n_cam, n_kp, 3])
    for i_cam in range(n_cam):
        kp2d[:, :, i_cam] = kp2d_of_camera(T[i_cam], Trk, Cid, i_cam, n_frame, n_animal, n_kp)
    return kp2d


def create_kp2dfile(result_dir, T, Trk, Cid, n_animal=4, n_kp=17):
    """step3_crossframematching.py:872-915 -> <result_dir>/kp2d.pickle (A, F, C, J, 3): per individual,
    frame and camera the keypoints of the first track (in Trk's order) mapped to that individual that has a
    box in the camera; among that camera's rows carrying the box id, the last one; zero fill."""
    kp2d = assemble_kp2d(T, Trk, Cid, n_animal, n_kp)
    mqio.dump_pickle(kp2d, os.path.join(result_dir, "kp2d.pickle"))
    return kp2d


def kp2d_from_step1(s1out, cam_ids, n_animal=4, n_kp=17, track_to_animal=None, world=1, group=None, device=None):
    """create_kp2dfile's array from step 1's rows in memory (``step1_proc2d.Step1Output``) instead of the
    alldata.json files, in the camera order of config.yaml.  On a sharded run every rank assembles the
    kp2d slices of the cameras it post-processed (``mqhip.shard.camera_shard``) -- the known assignment
    needs only every camera's track ids, which every rank has -- and one all-gather
    (``mqhip.shard.gather_cameras``) gives every rank the whole array.  Same bits as the file path.
    Returns None when the rows do not cover config.yaml's cameras (the caller then reads the files)."""
    if s1out is None or not s1out.complete or any(c not in s1out.names for c in cam_ids):
        return None
    store_of = [s1out.names.index(c) for c in cam_ids]          # store index of each config camera
    pos = {i: p for p, i in enumerate(store_of)}
    ids = [s1out.ids[i] for i in store_of]
    Trk, Cid = known_assignment(None, n_animal, track_to_animal, ids=ids)
    n_frame = len(ids[0])
    n_st = len(s1out.names)
    own = sorted(s1out.rows)
    part = np.zeros((n_animal, n_frame, len(own), n_kp, 3))
    for j, i in enumerate(own):
        if i in pos:
            part[:, :, j] = kp2d_of_camera_rows(s1out.rows[i], Trk, Cid, pos[i], n_frame, n_animal, n_kp)
    if len(own) == n_st and world == 1 and group is None:
        full = part
    else:
        from mqhip.shard import gather_cameras
        full = gather_cameras(part, n_st, world, group=group, device=device)
    return np.ascontiguousarray(full[:, :, store_of])


def proc_known_assignment(data_name, results_dir_root, config_path, n_animal=4, n_kp=17, track_to_animal=None):
    """alldata.json of every camera -> kp2d.pickle through a known track -> individual map."""
    result_dir = os.path.join(results_dir_root, data_name)
    cams = camera_ids(config_path)
    T = load_alldata(result_dir, cams)
    Trk, Cid = known_assignment(T, n_animal, track_to_animal)
    return create_kp2dfile(result_dir, T, Trk, Cid, n_animal=n_animal, n_kp=n_kp)
