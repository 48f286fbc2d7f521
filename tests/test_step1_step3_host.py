"""CPU: the host logic of the step-1 pose slice over frame stores and of step 3's kp2d writer.

* step 1's time-grid walk (step1_proc2d.py:210-223: nearest stored frame, repeats keep the
  previous result) and the batched multi-camera ``process_stores`` against a camera-by-camera
  loop written the reference's way -- the ViTPose call is replaced by a deterministic stand-in
  that depends on the image and the box, so batching / ordering / EMA state are what is tested;
* step 3's ``create_kp2dfile`` (step3_crossframematching.py:872-915) fed by a known assignment.
"""
import json
from types import SimpleNamespace

import numpy as np


from _fakes import fake_pose_batch as _fake_pose


def _stores(tmp_path, n_cams=3, n_frames=9, seed=0):
    from _fakes import make_stores
    return make_stores(str(tmp_path), n_cams, n_frames, seed)


def test_frame_plan_repeats_like_the_reference():
    from src.pipeline.step1_proc2d import _frame_plan
    st = SimpleNamespace(get_frame_metadata=lambda: {"frame_time": np.array([0.0, 0.1, 0.2]),
                                                      "frame_number": np.array([4, 5, 6])})
    T = np.arange(0.0, 0.2, 1 / 24)
    plan = _frame_plan(st, T)
    assert plan == [(4, False), (4, True), (5, False), (5, True), (6, False)]


def test_process_stores_equals_camera_by_camera_loop(tmp_path, monkeypatch):
    from src.pipeline import step1_proc2d as s1
    monkeypatch.setattr(s1, "inference_topdown_batch", _fake_pose)
    stores = _stores(tmp_path)
    t0 = stores[0].frame_time[0]
    T = np.arange(t0, stores[0].frame_time[-1], 1.0 / 24)
    got = s1.process_stores(None, stores, T, steps_per_batch=3)
    for c, st in enumerate(stores):           # the reference's per-camera walk (step1:210-362)
        sm = s1.KeypointSmoother()
        md = st.get_frame_metadata()
        res, fns, fn = [], [], -1
        for t in T:
            idx = int(np.abs(md["frame_time"] - t).argmin())
            if fn >= md["frame_number"][idx]:
                res.append(res[-1] if res else [])
                fns.append(fn)
                continue
            fn = int(md["frame_number"][idx])
            boxes, tids = s1.filter_tracks(st.tracks_of(fn))
            if len(boxes) == 0:
                res.append([])
            else:
                r = _fake_pose(None, [st.image(fn)], [s1.expand_boxes(boxes)])[0]
                res.append(s1._rows(r, boxes, tids, sm, fn, None, s1.KP_PARAMS))
            fns.append(fn)
        assert got[c][1] == fns
        assert json.dumps(got[c][0]) == json.dumps(res)


def test_known_assignment_kp2d_writer(tmp_path):
    from mqhip import io as mqio
    from src.pipeline import step3_crossframematching as s3
    kp = lambda v: [[v, v + 1, 0.5]] * 17
    T = [[[[0, 0, 0, 1, 1, kp(1.0), -1, 0.0], [1, 0, 0, 1, 1, kp(2.0), -1, 0.0]], []],
         [[[1, 0, 0, 1, 1, kp(3.0), -1, 0.0]], [[0, 0, 0, 1, 1, kp(4.0), -1, 0.0], [0, 0, 0, 1, 1, kp(5.0), -1, 0.0]]]]
    Trk, Cid = s3.known_assignment(T, 2)
    assert Trk[0].tolist() == [[0, -1], [-1, 0]] and Trk[1].tolist() == [[1, 1], [-1, -1]]
    k = s3.create_kp2dfile(str(tmp_path), T, Trk, Cid, n_animal=2)
    assert k.shape == (2, 2, 2, 17, 3)
    assert k[0, 0, 0, 0, 0] == 1.0 and k[1, 0, 0, 0, 0] == 2.0 and k[1, 0, 1, 0, 0] == 3.0
    assert k[0, 1, 1, 0, 0] == 5.0     # every matching row of the camera is written: the last one stays
    assert not k[0, 0, 1].any() and not k[1, 1].any()  # zero fill where absent
    np.testing.assert_array_equal(mqio.load_array_pickle(str(tmp_path / "kp2d.pickle")), k)


class _FakeId:
    """Deterministic stand-in for the ID model: label and score from the patch's mean value."""

    def classify(self, imgs, boxes_per_view):
        out = []
        for img, bxs in zip(imgs, boxes_per_view):
            res = []
            for (x1, y1, x2, y2) in np.asarray(bxs).reshape(-1, 4):
                p = np.asarray(img)[y1:y2, x1:x2]
                if p.size == 0:
                    res.append({"pred_label": -1, "pred_score": 0.0})
                    continue
                m = float(p.mean())
                res.append({"pred_label": int(m) % 6, "pred_score": 0.5 + (m % 1.0) * 0.5})
            out.append(res)
        return out

    def classify_patches(self, patches):
        return [self.classify([p], [np.array([[0, 0, p.shape[1], p.shape[0]]])])[0][0] for p in patches]


def test_process_stores_with_id_model_classifies_every_tracked_box(tmp_path, monkeypatch):
    """step1:301-350: the tracked boxes' patches are classified (here by a stand-in) and the id columns
    follow ID_CONF_THR; the batched run_id equals a per-frame classify_patches of the boxes."""
    from src.pipeline import step1_proc2d as s1
    monkeypatch.setattr(s1, "inference_topdown_batch", _fake_pose)
    stores = _stores(tmp_path)
    t0 = stores[0].frame_time[0]
    T = np.arange(t0, stores[0].frame_time[-1], 1.0 / 24)
    fake = _FakeId()
    got = s1.process_stores(None, stores, T, steps_per_batch=3, id_model=fake)
    plans, jobs = s1.plan_jobs(stores, T)
    n_rows = 0
    for c, st in enumerate(stores):
        rows_by_fn = dict(zip(got[c][1], got[c][0]))
        for k, js in jobs.items():
            for (cc, fn, boxes, tids, _) in js:
                if cc != c:
                    continue
                img = st.image(fn)
                ref = s1.classify_patches(fake, [img[y1:y2, x1:x2] for (x1, y1, x2, y2) in boxes])
                for row, r in zip(rows_by_fn[fn], ref):
                    assert row[7] == r["pred_score"]
                    assert row[6] == (r["pred_label"] if r["pred_score"] >= s1.ID_CONF_THR else -1)
                    n_rows += 1
    assert n_rows > 0
    assert s1.classify_patches(None, [np.zeros((3, 3, 3), np.uint8)]) == [{"pred_label": -1, "pred_score": 0.0}]


def test_id_model_per_camera_variant(tmp_path, monkeypatch):
    """step1:424-427: each camera is classified by the ID model of its variant -- 'mff1y' when the store
    folder name contains it, else 'normal' (ADVICE r2); ``resolve_id_models`` builds one model per variant."""
    from mqhip import io as mqio
    from src.pipeline import step1_proc2d as s1
    monkeypatch.setattr(s1, "inference_topdown_batch", _fake_pose)
    stores = _stores(tmp_path)
    # rename camera 1's store to an mff1y folder
    import os
    import shutil
    src = stores[1].filename
    dst = os.path.join(os.path.dirname(src), "demo_mff1y.1001")
    shutil.move(src, dst)
    stores[1] = mqio.FrameStore(dst)
    assert [s1.id_variant_of(st) for st in stores] == ["normal", "mff1y", "normal"]

    class _Shifted(_FakeId):
        def classify(self, imgs, boxes_per_view):
            return [[{"pred_label": (r["pred_label"] + 3) % 6, "pred_score": r["pred_score"]} for r in v]
                    for v in super().classify(imgs, boxes_per_view)]

    normal, mff = _FakeId(), _Shifted()
    models = s1.resolve_id_models(stores, {"normal": normal, "mff1y": mff})
    assert models[0] is normal and models[1] is mff and models[2] is normal
    built = []
    monkeypatch.setattr(s1, "init_id_model", lambda dev, v: built.append(v) or {"normal": normal, "mff1y": mff}[v])
    assert s1.resolve_id_models(stores, "auto") == models and sorted(built) == ["mff1y", "normal"]
    assert s1.resolve_id_models(stores, None) is None
    t0 = stores[0].frame_time[0]
    T = np.arange(t0, stores[0].frame_time[-1], 1.0 / 24)
    got = s1.process_stores(None, stores, T, steps_per_batch=3, id_model=models)
    plans, jobs = s1.plan_jobs(stores, T)
    n_rows = 0
    for c, st in enumerate(stores):
        rows_by_fn = dict(zip(got[c][1], got[c][0]))
        for js in jobs.values():
            for (cc, fn, boxes, _, _) in js:
                if cc != c:
                    continue
                img = st.image(fn)
                ref = s1.classify_patches(models[c], [img[y1:y2, x1:x2] for (x1, y1, x2, y2) in boxes])
                for row, r in zip(rows_by_fn[fn], ref):
                    assert row[7] == r["pred_score"]
                    assert row[6] == (r["pred_label"] if r["pred_score"] >= s1.ID_CONF_THR else -1)
                    n_rows += 1
    assert n_rows > 0


def test_detect_stores_groups_cameras_by_resolution(tmp_path, monkeypatch):
    """detect_stores sends the cameras of a time step to the detector in one batch per image size
    (np.stack of mixed resolutions raised)."""
    from mqhip import io as mqio
    from src.pipeline import step1_proc2d as s1
    times = np.arange(4) * 0.04 + 10.0
    for c, (h, w) in enumerate([(8, 8), (6, 10), (8, 8)]):
        fr = np.full((4, h, w, 3), 10 * c, np.uint8)
        mqio.write_frame_store(str(tmp_path / f"demo.{100 + c}"), fr, times, np.arange(4), [[]] * 4, 100 + c)
    from _fakes import open_stores
    stores = open_stores(str(tmp_path))
    batches = []

    def fake_det(det, imgs):
        assert len({im.shape for im in imgs}) == 1
        batches.append(len(imgs))
        return [(np.array([[1.0, 1.0, 4.0, 4.0], [0, 0, 2, 2]], np.float32),
                 np.array([0.9, 0.5 + im[0, 0, 0] / 100.0], np.float32)) for im in imgs]

    monkeypatch.setattr(s1, "inference_detector", fake_det)
    T = np.arange(times[0], times[-1], 1.0 / 24)
    out = s1.detect_stores(None, stores, T)
    assert batches and max(batches) == 2 and sum(batches) == 3 * len(out[0])
    for c in range(3):
        assert [fn for fn, _, _ in out[c]] == list(range(len(out[c])))
        for _, b, sc in out[c]:
            assert len(sc) == (2 if 0.5 + 10 * c / 100.0 > s1.SCORE_THR else 1)


def test_default_track_map_follows_the_track_ids_present():
    """BoT-SORT numbers tracks from 1, so the default individual map is built from the track
    ids in alldata (the n_animal smallest), not assumed to be 0..n_animal-1."""
    from src.pipeline import step3_crossframematching as s3
    kp = [[1.0, 2.0, 0.9]] * 17
    T = [[[[tid, 0, 0, 1, 1, kp, -1, 0.0] for tid in (1, 2, 3, 4, 5)]], [[[2, 0, 0, 1, 1, kp, -1, 0.0]]]]
    assert s3.default_track_map(T, 4) == {1: 0, 2: 1, 3: 2, 4: 3}
    Trk, Cid = s3.known_assignment(T, 4)
    assert sorted(Trk) == [1, 2, 3, 4] and Trk[2].tolist() == [[2, 2]] and Cid[4].tolist() == [3]
    assert s3.default_track_map([[[]]], 2) == {0: 0, 1: 1}


def test_auto_id_model_without_checkpoint_warns_and_keeps_store_ids(tmp_path, monkeypatch):
    """"auto" never classifies with random weights.  A missing checkpoint raises in
    init_id_model (the reference's init_model fails loudly); resolve_id_models("auto") warns and keeps
    the stores' own ID predictions (None) for that variant; "random" is the explicit opt-in."""
    import pytest
    from src.pipeline import step1_proc2d as s1
    monkeypatch.setattr(s1, "ID_CKPTS", {"normal": str(tmp_path / "missing.pth"), "mff1y": str(tmp_path / "m2.pth")})
    with pytest.raises(FileNotFoundError):
        s1.init_id_model("cuda:0", "normal")
    stores = _stores(tmp_path, n_cams=2)
    with pytest.warns(UserWarning, match="keep their stores' ID predictions"):
        assert s1.resolve_id_models(stores, "auto") == [None, None]
    built = []
    monkeypatch.setattr(s1, "init_id_model", lambda dev, v, random_weights=False: built.append((v, random_weights)) or v)
    assert s1.resolve_id_models(stores, "random") == ["normal", "normal"] and built == [("normal", True)]
    with pytest.raises(ValueError):
        s1.resolve_id_models(stores, "bogus")
