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


def default_track_map(T, n_animal):
    """{track id -> individual} for the smallest ``n_animal`` track ids present in the alldata rows, in
    ascending order (synthetic stores number tracks from 0, the BoT-SORT tracker from 1)."""
    tids = sorted({int(row[0]) for cam in T for frame in cam for row in frame})
    if not tids:  # nothing tracked: every individual stays zero-filled
        return {a: a for a in range(n_animal)}
    return {t: a for a, t in enumerate(tids[:n_animal])}


def known_assignment(T, n_animal, track_to_animal=None):
    """Trk[k] (F, C) box id of track k in each camera (-1 = absent) and Cid[k] (F,) its individual,
    for a known {track id -> individual} map shared by all cameras (default: ``default_track_map``, the
    ``n_animal`` smallest track ids present -> 0..n_animal-1)."""
    n_cam = len(T)
    n_frame = len(T[0])
    if track_to_animal is None:
        track_to_animal = default_track_map(T, n_animal)
    Trk, Cid = {}, {}
    for tid, a in track_to_animal.items():
        trk = np.full((n_frame, n_cam), -1, dtype=np.int64)
        for c in range(n_cam):
            for f in range(min(n_frame, len(T[c]))):
                if any(int(row[0]) == int(tid) for row in T[c][f]):
                    trk[f, c] = int(tid)
        Trk[tid] = trk
        Cid[tid] = np.full(n_frame, int(a), dtype=np.int64)
    return Trk, Cid


def create_kp2dfile(result_dir, T, Trk, Cid, n_animal=4, n_kp=17):
    """step3_crossframematching.py:872-915 -> <result_dir>/kp2d.pickle (A, F, C, J, 3)."""
    n_cam = len(T)
    n_frame = Trk[list(Trk.keys())[0]].shape[0]
    kp2d = np.zeros([n_animal, n_frame, n_cam, n_kp, 3])
    is_done = np.zeros([n_animal, n_frame, n_cam])
    for i_frame in range(n_frame):
        for k in Trk.keys():
            i_animal = Cid[k][i_frame]
            if i_animal < 0:
                continue
            trk = Trk[k][i_frame, :]
            if np.sum(trk >= 0) == 0:
                continue
            for i_cam in range(n_cam):
                if is_done[i_animal, i_frame, i_cam]:
                    continue
                for tt in T[i_cam][i_frame]:
                    if tt[0] == trk[i_cam]:
                        kp2d[i_animal, i_frame, i_cam, :, :] = np.array(tt[5], dtype=np.float64)
                        is_done[i_animal, i_frame, i_cam] = True
    mqio.dump_pickle(kp2d, os.path.join(result_dir, "kp2d.pickle"))
    return kp2d


def proc_known_assignment(data_name, results_dir_root, config_path, n_animal=4, n_kp=17, track_to_animal=None):
    """alldata.json of every camera -> kp2d.pickle through a known track -> individual map."""
    result_dir = os.path.join(results_dir_root, data_name)
    cams = camera_ids(config_path)
    T = load_alldata(result_dir, cams)
    Trk, Cid = known_assignment(T, n_animal, track_to_animal)
    return create_kp2dfile(result_dir, T, Trk, Cid, n_animal=n_animal, n_kp=n_kp)
