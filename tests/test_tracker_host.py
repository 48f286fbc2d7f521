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
