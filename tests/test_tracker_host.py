"""Step-1 tracker (mqhip/tracker.py, boxmot BotSort as BOTSORT_CFG configures it, step1_proc2d.py:75-89):
known-answer behaviour of the three association rounds, track life cycle and the cost-limited
assignment (parity with boxmot itself is unpinned: boxmot / OpenCV are absent)."""
import itertools

import numpy as np

from mqhip import tracker as trk


def _run(seq, **cfg):
    t = trk.BotSort(**dict(trk.BOTSORT_CFG, **cfg))
    return [t.update(np.asarray(d, float).reshape(-1, 6), None) for d in seq]


def _box(cx, cy, w=80, h=120, s=0.95):
    return [cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2, s, 0]


def test_linear_assignment_is_the_cost_limited_optimum():
    rng = np.random.default_rng(0)
    for _ in range(60):
        n, m = rng.integers(1, 5), rng.integers(1, 5)
        c = rng.uniform(0, 1, (n, m))
        thr = 0.6
        matches, ua, ub = trk.linear_assignment(c, thr)
        got = sum(c[i, j] for i, j in matches) + (len(ua) + len(ub)) * thr / 2
        best = np.inf
        for k in range(0, min(n, m) + 1):
            for rows in itertools.combinations(range(n), k):
                for cols in itertools.permutations(range(m), k):
                    best = min(best, sum(c[r, q] for r, q in zip(rows, cols)) + (n + m - 2 * k) * thr / 2)
        assert abs(got - best) < 1e-9
        assert len(matches) + len(ua) == n and len(matches) + len(ub) == m


def test_moving_box_keeps_one_id_and_follows_the_detections():
    seq = [[_box(100 + 4 * f, 200 + 2 * f)] for f in range(40)]
    out = _run(seq)
    assert all(len(o) == 1 and o[0, 4] == 1 for o in out)
    last = out[-1][0]
    assert np.abs(last[:4] - np.array(seq[-1][0][:4])).max() < 1.0
    assert np.all(out[5][:, 7] == 0)                      # det_ind of the matched detection


def test_first_frame_tracks_are_confirmed_later_ones_after_a_second_hit():
    seq = [[_box(100, 100)], [_box(101, 100), _box(500, 300)], [_box(102, 100), _box(501, 300)]]
    out = _run(seq)
    assert sorted(out[0][:, 4]) == [1]
    assert sorted(out[1][:, 4]) == [1]                    # the new box is unconfirmed on its first frame
    assert sorted(out[2][:, 4]) == [1, 2]


def test_occlusion_shorter_than_the_buffer_keeps_the_id_longer_gets_a_new_one():
    gap = lambda n: [_box(300, 300)] * 5 + [[]] * n + [_box(302, 301)] * 3
    out = _run([[b] if b else [] for b in gap(30)])
    assert out[-1][0, 4] == 1
    out = _run([[b] if b else [] for b in gap(80)])       # > int(24 / 30 * 72) = 57 frames lost
    assert out[-1][0, 4] == 2


def test_low_score_detections_keep_tracks_but_never_start_them():
    seq = [[_box(200, 200)]] + [[_box(200 + f, 200, s=0.5)] for f in range(1, 6)] + [[_box(600, 100, s=0.5)]] * 3
    out = _run(seq)
    assert all(len(o) == 1 and o[0, 4] == 1 for o in out[:6])
    assert all(set(o[:, 4].astype(int)) <= {1} for o in out[6:])    # no track starts from a low score


def test_two_crossing_boxes_keep_their_ids():
    seq = [[_box(100 + 10 * f, 200), _box(400 - 10 * f, 200 + 60)] for f in range(31)]
    out = _run(seq)
    for f, o in enumerate(out):
        assert len(o) == 2
        by_id = {int(r[4]): r for r in o}
        assert abs((by_id[1][0] + by_id[1][2]) / 2 - (100 + 10 * f)) < 3
        assert abs((by_id[2][0] + by_id[2][2]) / 2 - (400 - 10 * f)) < 3


# ----------------------------------------------------------------------------- known-answer fixtures
# Hand-derived from boxmot 12.0.7's published BoT-SORT (KalmanFilterXYWH, the three association rounds,
# lap.lapjv(extend_cost=True, cost_limit)); the numbers below are exact binary fractions, so the checks
# are equalities, not tolerances.

def test_kalman_xywh_initiate_predict_known_answer():
    """initiate: std = (2/20 w, 2/20 h, 2/20 w, 2/20 h, 10/160 w, 10/160 h, 10/160 w, 10/160 h);
    predict: F = [[I, I], [0, I]], Q = diag((w/20)^2, (h/20)^2, (w/20)^2, (h/20)^2, (w/160)^2, ...)."""
    from mqhip.tracker import KalmanFilterXYWH
    kf = KalmanFilterXYWH()
    mean, cov = kf.initiate(np.array([100.0, 200.0, 50.0, 80.0]))
    np.testing.assert_array_equal(mean, [100, 200, 50, 80, 0, 0, 0, 0])
    np.testing.assert_array_equal(np.diag(cov), [25, 64, 25, 64, 9.765625, 25, 9.765625, 25])
    assert np.count_nonzero(cov - np.diag(np.diag(cov))) == 0
    m2, c2 = kf.multi_predict(mean[None], cov[None])
    np.testing.assert_array_equal(m2[0], mean)
    # position: P_pp + P_vv + Q_p ; velocity: P_vv + Q_v ; cross: P_vv
    np.testing.assert_array_equal(np.diag(c2[0])[:4], [25 + 9.765625 + 6.25, 64 + 25 + 16, 25 + 9.765625 + 6.25,
                                                       64 + 25 + 16])
    np.testing.assert_array_equal(np.diag(c2[0])[4:], [9.765625 + 0.09765625, 25 + 0.25, 9.765625 + 0.09765625,
                                                       25 + 0.25])
    for i in range(4):
        assert c2[0][i, i + 4] == c2[0][i + 4, i] == cov[i + 4, i + 4]


def test_kalman_xywh_update_equals_textbook_gain():
    """update: S = H P H^T + R (R = diag((w/20)^2, (h/20)^2, ...)), K = P H^T S^-1, x' = x + K (z - H x),
    P' = P - K S K^T, against an explicit inverse."""
    from mqhip.tracker import KalmanFilterXYWH
    kf = KalmanFilterXYWH()
    mean, cov = kf.initiate(np.array([100.0, 200.0, 50.0, 80.0]))
    mean, cov = kf.multi_predict(mean[None], cov[None])
    mean, cov = mean[0], cov[0]
    mean[4:] = [3.0, -2.0, 0.5, 0.25]
    z = np.array([104.0, 197.0, 52.0, 79.0])
    H = np.eye(4, 8)
    R = np.diag(np.square([mean[2] / 20, mean[3] / 20, mean[2] / 20, mean[3] / 20]))
    S = H @ cov @ H.T + R
    K = cov @ H.T @ np.linalg.inv(S)
    m_ref = mean + K @ (z - H @ mean)
    c_ref = cov - K @ S @ K.T
    m, c = kf.update(mean, cov, z)
    np.testing.assert_allclose(m, m_ref, rtol=0, atol=1e-10)
    np.testing.assert_allclose(c, c_ref, rtol=0, atol=1e-10)


def test_lapjv_cost_limit_boundary():
    """extend_cost + cost_limit: a pair is matched iff its cost is below the limit (leaving both unmatched
    costs limit/2 + limit/2); with competing pairs the total is minimised."""
    from mqhip.tracker import linear_assignment
    m, ut, ud = linear_assignment(np.array([[0.79]]), 0.8)
    assert m.tolist() == [[0, 0]] and len(ut) == len(ud) == 0
    m, ut, ud = linear_assignment(np.array([[0.81]]), 0.8)
    assert len(m) == 0 and ut.tolist() == [0] and ud.tolist() == [0]
    # greedy would take (0, 0) = 0.1 and leave (1, 1) = 0.9 over the limit; the optimum is (0,1)+(1,0) = 0.5
    m, ut, ud = linear_assignment(np.array([[0.1, 0.2], [0.3, 0.9]]), 0.8)
    assert sorted(m.tolist()) == [[0, 1], [1, 0]]
    # a pair under the limit is still dropped when matching it would cost more overall than leaving it
    m, ut, ud = linear_assignment(np.array([[0.7, 0.05], [0.05, 0.7]]), 0.8)
    assert sorted(m.tolist()) == [[0, 1], [1, 0]]


def _kbox(cx, cy, w=40.0, h=60.0):
    return [cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2]


def test_three_association_rounds_known_answer():
    """A scripted sequence through BOTSORT_CFG (high 0.85, low 0.10, new 0.85, match 0.8):
    f1: two high detections -> tracks 1, 2 confirmed at once (first frame);
    f2: track 1's detection high (round 1), track 2's at 0.5 (round 2: low-score vs remaining tracked,
        IoU limit 0.5) -> both keep their ids; a far high detection starts track 3, unconfirmed (not shown);
    f3: track 3's detection again -> round 3 (unconfirmed vs remaining high, 1 - IoU*score) confirms it;
        track 2 absent -> lost (not shown);
    f4: track 2's detection back at 0.95 -> round 1 re-finds it among the lost tracks with its id."""
    from mqhip.tracker import BOTSORT_CFG, BotSort
    t = BotSort(**BOTSORT_CFG)
    out = t.update(np.array([_kbox(100, 100) + [0.95, 0], _kbox(300, 100) + [0.95, 0]]))
    assert sorted(out[:, 4].tolist()) == [1, 2]
    out = t.update(np.array([_kbox(102, 101) + [0.95, 0], _kbox(301, 99) + [0.5, 0], _kbox(700, 400) + [0.9, 0]]))
    rows = {int(r[4]): r for r in out}
    assert sorted(rows) == [1, 2]
    assert rows[1][7] == 0 and rows[2][7] == 1 and rows[2][5] == 0.5     # det_ind, conf of the matched detection
    out = t.update(np.array([_kbox(104, 102) + [0.95, 0], _kbox(702, 401) + [0.9, 0]]))
    assert sorted(int(r[4]) for r in out) == [1, 3]
    assert [tr.id for tr in t.lost_stracks] == [2]
    out = t.update(np.array([_kbox(106, 103) + [0.95, 0], _kbox(302, 99) + [0.95, 0], _kbox(704, 402) + [0.9, 0]]))
    assert sorted(int(r[4]) for r in out) == [1, 2, 3]
    assert not t.lost_stracks


def test_max_time_lost_is_int_frame_rate_over_30_times_buffer():
    """BOTSORT_CFG: track_buffer 72 at 24 fps -> max_time_lost = int(24 / 30 * 72) = 57 frames."""
    from mqhip.tracker import BOTSORT_CFG, BotSort
    assert BotSort(**BOTSORT_CFG).max_time_lost == 57
