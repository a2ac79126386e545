"""Interval trial decisions (sections.trial_decided): the bounded -7/-9
encode tries fqz / sequence-model candidates for their size intervals only
and takes the trial's choices from them when the intervals separate the
candidates of every decision metrics_method / compress_with_methods make
(fqzcomp5.c:1899-2127).  Host logic only, no GPU."""
import numpy as np

from fqzcomp5_amd import sections as S

Q = 3                       # quality sections
R0, F0, F1 = S.RANS0, S.FQZ0, S.FQZ1
MASK = (1 << R0) | (1 << F0) | (1 << F1)


def case(n, lo_f0, hi_f0, lo_f1, hi_f1, r0):
    lo = np.full((n, S.M_LAST), np.iinfo(np.uint32).max, np.uint32)
    hi = lo.copy()
    for i in range(n):
        lo[i, R0] = hi[i, R0] = r0
        lo[i, F0], hi[i, F0] = lo_f0, hi_f0
        lo[i, F1], hi[i, F1] = lo_f1, hi_f1
    ids = np.full(n, Q, np.int32)
    ins = np.full(n, 10_000, np.uint32)
    sched = np.array([MASK if i < S.TRIAL_WINDOW else 0 for i in range(n)], np.uint32)
    tried = np.array([MASK if i < S.TRIAL_WINDOW else (1 << F0) for i in range(n)], np.uint32)
    return lo, hi, ids, ins, tried, sched


def test_first_min_fixed():
    assert S._first_min_fixed([5, 10], [6, 12])
    assert not S._first_min_fixed([5, 6], [7, 8])          # overlap
    assert S._first_min_fixed([5, 5], [5, 5])              # exact tie: the first wins
    assert S._first_min_fixed([7, 5], [7, 6])              # exact first, interval later
    assert not S._first_min_fixed([6, 5], [6, 6])          # a later one ties the first
    assert S._first_min_fixed([6, 5], [6, 5])              # exact values: decided


def test_separated_intervals_decide():
    st = S.new_state()
    assert S.trial_decided(*case(4, 100, 110, 200, 220, 500), st, final=True)


def test_overlap_is_not_decided():
    st = S.new_state()
    assert not S.trial_decided(*case(4, 100, 150, 140, 220, 500), st, final=True)


def test_window_sum_decides_later_blocks():
    # per section F0 wins clearly; the window's ratio too
    st = S.new_state()
    lo, hi, ids, ins, tried, sched = case(5, 1000, 1001, 1100, 1102, 5000)
    assert S.trial_decided(lo, hi, ids, ins, tried, sched, st, final=True)
    # a decision after the window needs the next section inside the call
    lo, hi, ids, ins, tried, sched = case(3, 1000, 1001, 1100, 1102, 5000)
    assert S.trial_decided(lo, hi, ids, ins, tried, sched, st, final=True)
    assert not S.trial_decided(lo, hi, ids, ins, tried, sched, st, final=False)


def test_mid_trial_state_is_not_decided():
    st = S.new_state()
    st.sec[Q].trial = 2          # a window begun in an earlier call
    assert not S.trial_decided(*case(4, 100, 110, 200, 220, 500), st, final=True)


def test_replay_of_lower_ends_matches_exact_sizes():
    """When decided, replaying the lower ends picks what any exact sizes
    inside the intervals pick."""
    rng = np.random.default_rng(3)
    av = np.zeros(4, np.uint32)
    av[Q] = MASK
    for _ in range(20):
        n = 7
        lo, hi, ids, ins, tried, sched = case(n, 0, 0, 0, 0, 0)
        for i in range(n):
            lo[i, R0] = hi[i, R0] = rng.integers(4000, 6000)
            a = rng.integers(1000, 5000)
            lo[i, F0], hi[i, F0] = a, a + rng.integers(0, 50)
            b = rng.integers(1000, 5000)
            lo[i, F1], hi[i, F1] = b, b + rng.integers(0, 50)
        sched = S.trial_schedule(ids, av, S.new_state())
        st = S.new_state()
        tried = np.zeros(n, np.uint32)
        m_lo = S.trial_replay(ids, ins, lo, av, st, tried)
        if not S.trial_decided(lo, hi, ids, ins, tried, sched, S.new_state(), final=True):
            continue
        for _ in range(5):
            ex = lo.copy()
            for i in range(n):
                for m in (F0, F1):
                    ex[i, m] = rng.integers(int(lo[i, m]), int(hi[i, m]) + 1)
            assert list(S.trial_replay(ids, ins, ex, av, S.new_state())) == list(m_lo)
