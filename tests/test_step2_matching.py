"""Step-2 matching (step2_crossviewmatching.py): matchSVT (:130-216), get_best_comb / calc_3dpose
(:436-461, :610-646), predict_data (:502-713), the 2D-tracklet ID voting (:717-850) and proc
(:854-959).

CPU: the oracle's matchSVT recovers planted clusters and its SVD thresholding equals the eigen
thresholding the kernel uses; the host ID voting equals the oracle; calibration loading.
GPU: mq_match_svt vs the oracle (binary match bit-exact, X within 1e-9, same iteration count);
predict_batch vs the oracle's predict_data per keyframe (same clusters and bcomb, 3D within 1e-6);
proc end to end from alldata.json."""
import copy
import json
import os

import numpy as np
import pytest

from conftest import gpu_available
from oracle import association as orc


def _planted_w(rng, n_cam=8, n_ind=4, p_seen=0.85, noise=0.15, dup=False):
    ids, cams = [], []
    for c in range(n_cam):
        seen = [a for a in range(n_ind) if rng.random() < p_seen]
        if dup and seen:
            seen.append(seen[0])
        rng.shuffle(seen)
        ids += seen
        cams += [c] * len(seen)
    ids, cams = np.array(ids, dtype=int), np.array(cams, dtype=int)
    M = len(ids)
    W = np.where(ids[:, None] == ids[None, :], 0.9, 0.1) + noise * rng.standard_normal((M, M))
    W = np.clip(W, 0, 1)
    W[cams[:, None] == cams[None, :]] = 0
    dim = np.concatenate([[0], np.cumsum([np.sum(cams == c) for c in range(n_cam)])]).astype(int)
    return W, dim, ids, cams


def test_oracle_matchsvt_recovers_planted_clusters():
    rng = np.random.default_rng(0)
    for _ in range(4):
        W, dim, ids, cams = _planted_w(rng, noise=0.1)
        match = orc.matchSVT(W.copy(), dim, alpha=0.5, _lambda=50, dual_stochastic_SVT=False)
        truth = (ids[:, None] == ids[None, :]).astype(np.uint8)
        assert np.array_equal(match, truth)


def test_svd_threshold_equals_eigen_threshold():
    # the kernel's identity: for symmetric M, U max(s - tau, 0) V^T = E sign(l) max(|l| - tau, 0) E^T
    rng = np.random.default_rng(1)
    for n in (1, 5, 32):
        A = rng.standard_normal((n, n))
        M = (A + A.T) / 2
        U, s, Vh = np.linalg.svd(M)
        Q1 = U @ np.diag(np.maximum(s - 0.7, 0)) @ Vh
        l, E = np.linalg.eigh(M)
        Q2 = (E * (np.sign(l) * np.maximum(np.abs(l) - 0.7, 0))) @ E.T
        assert np.abs(Q1 - Q2).max() < 1e-12


def _tracklets(rng, n_frame, n_trk):
    Cid = {}
    for k in range(n_trk):
        arr = -2 * np.ones(n_frame, dtype=int)
        a, b = sorted(rng.integers(0, n_frame, 2))
        b = max(b, a + 5)
        seg = rng.choice([0, 2, 3, 5, -1, 1], size=b - a, p=[0.3, 0.1, 0.1, 0.1, 0.3, 0.1])
        if k % 3 == 2:  # an ID switch half-way
            seg[: (b - a) // 2] = np.where(rng.random((b - a) // 2) < 0.9, 2, -1)
            seg[(b - a) // 2:] = np.where(rng.random(b - a - (b - a) // 2) < 0.9, 5, -1)
        elif k % 3 == 1:
            seg = np.where(rng.random(b - a) < 0.85, 3, seg)
        arr[a:b] = seg
        Cid[k] = arr
    return Cid


def test_id_voting_host_equals_oracle():
    from src.pipeline.step2_crossviewmatching import set_id_for_each_frame_of_2dtracklets as host
    rng = np.random.default_rng(2)
    for trial in range(6):
        n_frame = int(rng.integers(60, 400))
        Cid = _tracklets(rng, n_frame, 6)
        wsize = 24 * 5 if trial % 2 == 0 else 30
        a = host(Cid, n_frame, wsize)
        b = orc.set_id_for_each_frame_of_2dtracklets(Cid, n_frame, wsize)
        for k in Cid:
            assert np.array_equal(a[k], b[k]), (trial, k)


def test_id_sequences_host_equals_oracle():
    from mqhip import synth
    from src.pipeline.step2_crossviewmatching import _id_sequences
    cams = synth.make_cameras(4)
    skel = synth.make_skeletons(4, 150)
    T = synth.make_alldata(cams, skel, p_dup=0.2)
    a = _id_sequences(copy.deepcopy(T))
    b = orc.get_id_of_2dtrack(copy.deepcopy(T))
    for c in range(4):
        assert a[c].keys() == b[c].keys()
        for k in a[c]:
            assert np.array_equal(a[c][k], b[c][k])


def test_get_camparam_from_calibration_toml(tmp_path):
    from mqhip import io as mqio, synth
    from src.pipeline.step2_crossviewmatching import get_camparam
    cams = synth.make_cameras(3)
    ref = synth.camparam_from_cams(cams)
    calib = {f"cam_{i}": {"name": c["name"], "size": c["size"], "matrix": c["K"].tolist(), "K": c["K"].tolist(),
                          "xi": [float(c["xi"][0])], "D": c["D"].tolist(), "distortions": [0.0] * 5,
                          "rotation": c["rvec"].tolist(), "translation": c["tvec"].tolist(), "omnidir": True}
             for i, c in enumerate(cams)}
    mqio.dump_toml(calib, str(tmp_path / "calibration.toml"))
    with open(tmp_path / "config.yaml", "w") as f:
        f.write("camera_id: [" + ", ".join(c["name"] for c in cams) + "]\n")
    got = get_camparam(str(tmp_path / "config.yaml"))
    for key in ("K", "xi", "D", "rvecs", "tvecs", "pmat"):
        for a, b in zip(got[key], ref[key]):
            assert np.allclose(np.asarray(a, dtype=float).ravel(), np.asarray(b, dtype=float).ravel(), atol=1e-12)


# ----------------------------------------------------------------------------- GPU

def _oracle_info_dicts(T, Cid2d, camparam, frames, n_kp=17):
    ocams = orc.camparam_cams(camparam)
    out = []
    for f in frames:
        info = {}
        for c in range(len(T)):
            ents = []
            for det in T[c][f]:
                raw = np.array(det[5], dtype=np.float64)
                ents.append({"pose2d": ocams[c].undistort_points(raw[:, :2] + 0.0), "pose2d_raw": raw,
                             "bbox": det[1:5], "bbox_id": [c, det[0]], "cid": Cid2d[c][det[0]][f]})
            info[c] = {0: ents, "image_data": []}
        out.append(info)
    return out


def _assert_same_result(got, exp, tol=1e-6):
    m1, p1, b1 = got
    m2, p2, b2 = exp
    assert len(m1) == len(m2)
    for a, b in zip(m1, m2):
        assert np.array_equal(np.asarray(a, dtype=int), np.asarray(b, dtype=int))
    for a, b in zip(b1, b2):
        assert np.array_equal(a, b)
    for a, b in zip(p1, p2):
        assert a.shape == b.shape
        assert np.array_equal(np.isnan(a), np.isnan(b))
        ok = ~np.isnan(b)
        assert np.abs(a[ok] - b[ok]).max() < tol * max(1.0, np.abs(b[ok]).max())


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_match_svt_matches_oracle():
    from mqhip.association import match_svt_batch
    rng = np.random.default_rng(3)
    cases = [_planted_w(rng, noise=0.05 + 0.03 * i, dup=(i % 3 == 0)) for i in range(10)]
    cases.append(_planted_w(rng, n_cam=2, n_ind=1, p_seen=1.0))           # N = 2
    cases.append(_planted_w(rng, n_cam=3, n_ind=3, p_seen=0.7))           # small, maybe odd
    cases.append(_planted_w(rng, n_cam=8, n_ind=8, p_seen=1.0, noise=0.2))  # N = 64
    rand = rng.uniform(0, 1, (31, 31))
    cams31 = np.sort(rng.integers(0, 8, 31))
    rand[cams31[:, None] == cams31[None, :]] = 0
    dim31 = np.concatenate([[0], np.cumsum([np.sum(cams31 == c) for c in range(8)])])
    cases.append((rand, dim31, None, cams31))                              # unstructured, odd N
    B = len(cases) + 1  # + one empty keyframe
    Nmax = max(c[0].shape[0] for c in cases)
    W = np.zeros((B, Nmax, Nmax))
    nd = np.zeros(B, dtype=np.int32)
    cod = np.full((B, Nmax), -1, dtype=np.int32)
    for b, (w, dim, _, cams) in enumerate(cases):
        n = w.shape[0]
        W[b, :n, :n] = w
        nd[b] = n
        cod[b, :n] = cams
    match, iters, X = match_svt_batch(W, nd, cod, alpha=0.5, _lambda=50, return_x=True)
    for b, (w, dim, ids, cams) in enumerate(cases):
        n = w.shape[0]
        m_o, X_o, it_o = orc.matchSVT(w.copy(), dim, alpha=0.5, _lambda=50, dual_stochastic_SVT=False,
                                      return_info=True)
        assert iters[b] == it_o, (b, iters[b], it_o)
        assert np.abs(X[b, :n, :n] - X_o).max() < 1e-9, b
        assert np.array_equal(match[b, :n, :n], m_o), b
        assert not match[b, n:, :].any() and not match[b, :, n:].any()
    assert iters[B - 1] == -1 and not match[B - 1].any()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_match_svt_reference_signature():
    from src.pipeline.step2_crossviewmatching import matchSVT
    rng = np.random.default_rng(4)
    W, dim, ids, cams = _planted_w(rng)
    S = W.copy()
    got = matchSVT(S, dim, alpha=0.5, _lambda=50, dual_stochastic_SVT=False)
    assert np.all(np.diag(S) == 0)
    assert np.array_equal(got, orc.matchSVT(W.copy(), dim, alpha=0.5, _lambda=50, dual_stochastic_SVT=False))
    with pytest.raises(NotImplementedError):
        matchSVT(W.copy(), dim, dual_stochastic_SVT=True)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_calc_3dpose_and_reproject_match_oracle():
    from mqhip import synth
    from src.pipeline.step2_crossviewmatching import calc_3dpose, reproject
    cams = synth.make_cameras(8)
    cp = synth.camparam_from_cams(cams)
    skel = synth.make_skeletons(2, 3)
    T = synth.make_alldata(cams, skel, p_seen=0.8, p_dup=0.0)
    for f in range(3):
        kp = np.zeros((8, 17, 3))
        for c in range(8):
            for det in T[c][f]:
                if det[0] == 0:
                    kp[c] = np.array(det[5])
        got = calc_3dpose(kp, "", camparam=cp)
        exp = orc.calc_3dpose(kp, cp)
        ok = ~np.isnan(exp)
        assert np.array_equal(np.isnan(got), ~ok)
        assert np.abs(got[ok] - exp[ok]).max() < 1e-6
        for c in range(8):
            r1 = reproject(c, np.nan_to_num(exp), camparam=cp)
            r2 = orc.reproject(c, np.nan_to_num(exp), cp)
            assert np.abs(r1 - r2).max() < 1e-7


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("n_cam,p_dup", [(8, 0.15), (4, 0.3)])
def test_predict_batch_matches_oracle(n_cam, p_dup):
    from mqhip import synth
    from src.pipeline.step2_crossviewmatching import MultiEstimator, _id_sequences
    cams = synth.make_cameras(n_cam)
    cp = synth.camparam_from_cams(cams)
    skel = synth.make_skeletons(4, 40, seed=7)
    T = synth.make_alldata(cams, skel, p_dup=p_dup, seed=8)
    Cid2d = _id_sequences(copy.deepcopy(T), wsize=10)
    frames = list(range(1, 40 - 12, 3))
    infos = _oracle_info_dicts(T, Cid2d, cp, frames)
    infos.append({c: {0: [], "image_data": []} for c in range(n_cam)})  # an empty keyframe
    got = MultiEstimator("", device=0).predict_batch(infos, camparam=cp)
    n_multi = 0
    for g, info in zip(got, infos):
        exp = orc.predict_data(info, cp)
        _assert_same_result(g, exp)
        n_multi += len(exp[0])
    assert n_multi > 0
    assert got[-1] == ([], [], [])


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_step2_proc_end_to_end(tmp_path):
    from mqhip import synth
    from src.pipeline.step2_crossviewmatching import proc
    n_cam = 6
    cams = synth.make_cameras(n_cam)
    cp = synth.camparam_from_cams(cams)
    skel = synth.make_skeletons(4, 50, seed=9)
    T = synth.make_alldata(cams, skel, p_dup=0.1, seed=10)
    res = tmp_path / "clip"
    for c, cam in enumerate(cams):
        os.makedirs(res / cam["name"])
        with open(res / cam["name"] / "alldata.json", "w") as f:
            json.dump(T[c], f)
    with open(tmp_path / "config.yaml", "w") as f:
        f.write("camera_id: [" + ", ".join(c["name"] for c in cams) + "]\n")
    out = proc("clip", str(tmp_path), "", str(tmp_path / "config.yaml"), camparam=cp)
    frames = list(range(1, 50 - 12, 12))
    assert [r["frame"] for r in out] == frames
    Cid2d = orc.get_id_of_2dtrack(copy.deepcopy(T))
    infos = _oracle_info_dicts(T, Cid2d, cp, frames)
    for r, info in zip(out, infos):
        _, p3, bc = orc.predict_data(info, cp)
        assert len(bc) == len(r["bcomb"])
        for a, b in zip(r["bcomb"], bc):
            assert np.array_equal(a, b)
        for a, b in zip(r["pose3d"], p3):
            ok = ~np.isnan(b)
            assert np.array_equal(np.isnan(a), ~ok)
            assert np.abs(a[ok] - b[ok]).max() < 1e-6
    assert os.path.exists(res / "match_keyframe.pickle")
