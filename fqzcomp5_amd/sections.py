"""Block-section coding on the GPU (include/fqz5_block.h) from Python.

A "run" is a list of blocks in file order; each block has a name, a
sequence and a quality section (fqzcomp5.c:2167-2257).  Encoding follows fqzcomp5's codec
trial (metrics_method / compress_with_methods, fqzcomp5.c:1899-2144):

    ids    = exchange(section ids)          # multi-GPU: all_gather (RCCL)
    masks  = schedule(all sections)         # which sections try every method
    sizes  = try(local sections, masks)     # trial candidates, one GPU batch
    sizes  = exchange(sizes)
    meth   = replay(all sections, sizes)    # host state machine, file order
    commit(local sections, meth)            # the rest encoded once, framed

so the choices are those of a single-threaded reference run over the whole
file, whichever GPU holds which block.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import lib as _lib

M_LAST = 31
SEC_NAME, SEC_SEQ, SEC_QUAL = 0, 2, 3
RANS0, RANS1, RANS64, RANS65, RANS128, RANS129, RANS192, RANS193, RANSXN1 = range(1, 10)
LZP3 = 10
TLZP3 = 11
TOK3_3, TOK3_5, TOK3_7, TOK3_9 = range(12, 16)
TOK3_3_LZP, TOK3_5_LZP, TOK3_7_LZP, TOK3_9_LZP = range(16, 20)
NAME_MASK = sum(1 << m for m in range(TLZP3, TOK3_9_LZP + 1))
SEQ10, SEQ12, SEQ12B, SEQ13B, SEQ14B = range(20, 25)
FQZ0, FQZ1, FQZ2, FQZ3, FQZ4 = range(26, 31)
RANS_MASK = sum(1 << m for m in range(RANS0, RANSXN1 + 1))
FQZ_MASK = sum(1 << m for m in range(FQZ0, FQZ4 + 1))
SEQ_MASK = sum(1 << m for m in range(SEQ10, SEQ14B + 1))
# candidates whose cost grows with their work: tried only where the trial
# schedule names them (see encode_run)
WORK_MASK = FQZ_MASK | SEQ_MASK | (1 << LZP3)

# Method masks of the level presets (name: arg.nauto, sequence, quality;
# fqzcomp5.c:4886-4932, :2750-2793) and their block sizes.
PRESET_MASKS = {
    1: {SEC_NAME: [TLZP3],
        SEC_SEQ: [RANS0, RANS1, RANS129, RANS193, LZP3],
        SEC_QUAL: [RANS0, RANS1, RANS129, RANS193]},
    3: {SEC_NAME: [TLZP3, TOK3_3_LZP],
        SEC_SEQ: [RANS0, RANS1, RANS129, RANS193, LZP3],
        SEC_QUAL: [RANS0, RANS1, RANS129, RANS193, RANSXN1]},
    5: {SEC_NAME: [TLZP3, TOK3_5_LZP],
        SEC_SEQ: [RANS0, RANS1, RANS129, RANS193, LZP3, SEQ10, SEQ12B],
        SEC_QUAL: [RANS0, RANS1, RANS129, RANS193, RANSXN1, FQZ1, FQZ3]},
    7: {SEC_NAME: [TLZP3, TOK3_7_LZP, TOK3_7],
        SEC_SEQ: [RANS0, RANS1, RANS129, RANS193, LZP3, RANS65, SEQ10, SEQ12B, SEQ13B],
        SEC_QUAL: [RANS0, RANS1, RANS129, RANS193, RANS65, FQZ0, FQZ1, FQZ2, FQZ3, FQZ4]},
    9: {SEC_NAME: [TLZP3, TOK3_9_LZP, TOK3_9],
        SEC_SEQ: [RANS0, RANS1, RANS129, RANS193, RANS64, RANS65, RANS128, LZP3,
                  SEQ10, SEQ12, SEQ12B, SEQ13B, SEQ14B],
        SEC_QUAL: [RANS0, RANS1, RANS129, RANS193, RANS64, RANS65, RANS128,
                   FQZ0, FQZ1, FQZ2, FQZ3, FQZ4]},
}
BLOCK_SIZE = {1: 10_000_000, 3: 100_000_000, 5: 100_000_000, 7: 500_000_000,
              9: 1_000_000_000}
# encode_seq's (k, both strands) per method (fqzcomp5.c:2047-2062)
SEQ_PARAMS = {SEQ10: (10, 0), SEQ12: (12, 0), SEQ12B: (12, 1), SEQ13B: (13, 1),
              SEQ14B: (14, 1)}
# methods this build codes: every method of the presets (rANS, LZP3, the
# name methods, the sequence context models, fqz)
BUILT = set(range(RANS0, TOK3_9_LZP + 1)) | set(SEQ_PARAMS) | set(range(FQZ0, FQZ4 + 1))


def preset_methods(level: int, names: bool = True) -> list[int]:
    """Every method of the preset, (section, method) flattened."""
    return sorted({m for sec, ms in PRESET_MASKS[level].items()
                   for m in ms if names or sec != SEC_NAME})


def level_methods(level: int, names: bool = True) -> list[int]:
    """The preset's methods that this build codes."""
    return [m for m in preset_methods(level, names) if m in BUILT]


class Section(C.Structure):
    """fqz5_section; the record fields are needed by the FQZ methods only
    (host lengths / flags, the block's device sequence bytes)."""
    _fields_ = [("in_", C.c_void_p), ("out", C.c_void_p),
                ("in_size", C.c_uint32), ("out_cap", C.c_uint32),
                ("fixed_len", C.c_uint32), ("sec", C.c_int32),
                ("rec_len", C.POINTER(C.c_uint32)), ("rec_flags", C.POINTER(C.c_uint32)),
                ("nrec", C.c_int32), ("seq", C.c_void_p)]


class SectionResult(C.Structure):
    _fields_ = [("method", C.c_int32), ("strat", C.c_int32),
                ("status", C.c_int32), ("clen", C.c_uint32),
                ("usize", C.c_uint32)]


class SectionStats(C.Structure):
    _fields_ = [("usize", C.c_uint64 * M_LAST), ("csize", C.c_uint64 * M_LAST),
                ("review", C.c_int32), ("trial", C.c_int32),
                ("count", C.c_int32 * M_LAST), ("method_used", C.c_int32)]


class TrialState(C.Structure):
    _fields_ = [("sec", SectionStats * 4)]


_bound = False


TRIAL_WINDOW = 3      # FQZ5_METRICS_TRIAL (fqzcomp5.c:152)
last_bounds_decided = None   # whether the last bounded run's intervals decided its trial
bounds_widen = 0             # tests: bytes added to every interval's upper end


def trial_counts() -> tuple[int, int]:
    """(fqz candidates tried, of which pruned) since the library was loaded."""
    out = (C.c_uint64 * 2)()
    _load().fqz5_trial_counts(out)
    return int(out[0]), int(out[1])


def _load():
    global _bound
    so = _lib.load()
    if not _bound:
        so.fqz5_trial_init.argtypes = [C.POINTER(TrialState)]
        so.fqz5_set_trial_prune.restype = C.c_int
        so.fqz5_set_trial_prune.argtypes = [C.c_int]
        so.fqz5_set_trial_bounds.restype = C.c_int
        so.fqz5_set_trial_bounds.argtypes = [C.c_int]
        so.fqz5_arenas_release.restype = C.c_int
        so.fqz5_arenas_release.argtypes = []
        so.fqz5_sections_try_upper.restype = C.c_int
        so.fqz5_sections_try_upper.argtypes = [C.POINTER(C.c_uint32), C.c_int]
        so.fqz5_trial_counts.argtypes = [C.POINTER(C.c_uint64)]
        so.fqz5_trial_schedule.argtypes = [C.POINTER(C.c_int32), C.c_int,
                                           C.POINTER(C.c_uint32), C.POINTER(TrialState),
                                           C.POINTER(C.c_uint32)]
        so.fqz5_sections_try.argtypes = [C.POINTER(Section), C.c_int,
                                         C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32)]
        so.fqz5_sections_try.restype = C.c_int
        so.fqz5_trial_replay.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32), C.c_int,
                                         C.POINTER(C.c_uint32), C.POINTER(TrialState),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]
        so.fqz5_sections_commit.argtypes = [C.POINTER(Section), C.c_int,
                                            C.POINTER(C.c_int32),
                                            C.POINTER(SectionResult)]
        so.fqz5_sections_commit.restype = C.c_int
        so.fqz5_decode_sections.argtypes = [C.POINTER(Section), C.c_int,
                                            C.POINTER(SectionResult)]
        so.fqz5_decode_sections.restype = C.c_int
        _bound = True
    return so


def masks(level: int, seq_cm: bool = False, full: bool = False) -> np.ndarray:
    """Per-section method masks of a level preset, restricted to the built
    methods.  Without `full` the sequence context models (SEQ*) are left out
    unless `seq_cm` is set (the reduced trial of earlier tests)."""
    av = np.zeros(4, np.uint32)
    for sec, ms in PRESET_MASKS[level].items():
        for m in ms:
            if m not in BUILT or (m in SEQ_PARAMS and not (seq_cm or full)):
                continue
            av[sec] |= np.uint32(1 << m)
    return av


def new_state() -> TrialState:
    st = TrialState()
    _load().fqz5_trial_init(C.byref(st))
    return st


def _arr(t, xs):
    return (t * len(xs))(*xs)


def trial_schedule(sec_ids, avail: np.ndarray, state: TrialState) -> np.ndarray:
    """Per section (file order) the methods it tries: avail in trial and
    re-trial blocks, 0 where the trial sizes decide (state unchanged)."""
    so = _load()
    ids = np.ascontiguousarray(sec_ids, np.int32)
    av = np.ascontiguousarray(avail, np.uint32)
    out = np.zeros(len(ids), np.uint32)
    so.fqz5_trial_schedule(ids.ctypes.data_as(C.POINTER(C.c_int32)), len(ids),
                           av.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(state),
                           out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def sections_try(secs: list[Section], masks: np.ndarray) -> np.ndarray:
    """Candidates of masks[i] (per section) for every section."""
    so = _load()
    sizes = np.zeros(len(secs) * M_LAST, np.uint32)
    av = np.ascontiguousarray(masks, np.uint32)
    assert len(av) == len(secs)
    _lib.after_torch()
    rc = so.fqz5_sections_try(_arr(Section, secs), len(secs),
                              av.ctypes.data_as(C.POINTER(C.c_uint32)),
                              sizes.ctypes.data_as(C.POINTER(C.c_uint32)))
    if rc:
        raise _lib.NativeError("fqz5_sections_try: " + _lib.last_error())
    return sizes.reshape(len(secs), M_LAST)


def trial_replay(sec_ids, in_sizes, sizes: np.ndarray, avail: np.ndarray,
                 state: TrialState, tried: np.ndarray | None = None) -> np.ndarray:
    """Host-only replay of metrics_method/compress_with_methods; `tried`
    (optional, uint32[n]) receives the method mask each section tried."""
    so = _load()
    n = len(sec_ids)
    ids = np.ascontiguousarray(sec_ids, np.int32)
    ins = np.ascontiguousarray(in_sizes, np.uint32)
    sz = np.ascontiguousarray(sizes, np.uint32).reshape(-1)
    av = np.ascontiguousarray(avail, np.uint32)
    out = np.zeros(n, np.int32)
    so.fqz5_trial_replay(ids.ctypes.data_as(C.POINTER(C.c_int32)),
                         ins.ctypes.data_as(C.POINTER(C.c_uint32)),
                         sz.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                         av.ctypes.data_as(C.POINTER(C.c_uint32)),
                         C.byref(state), out.ctypes.data_as(C.POINTER(C.c_int32)),
                         None if tried is None else
                         tried.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def sections_try_bounds(secs: list[Section], masks: np.ndarray):
    """sections_try with every fqz / sequence-model candidate's range chain
    skipped (fqz5_set_trial_bounds): (lower, upper) size matrices, equal
    wherever the size is exact."""
    so = _load()
    prev = so.fqz5_set_trial_bounds(1)
    try:
        lo = sections_try(secs, masks)
    finally:
        so.fqz5_set_trial_bounds(prev)
    hi = np.zeros(len(secs) * M_LAST, np.uint32)
    if so.fqz5_sections_try_upper(hi.ctypes.data_as(C.POINTER(C.c_uint32)), len(secs)):
        raise _lib.NativeError("fqz5_sections_try_upper: " + _lib.last_error())
    return lo, hi.reshape(len(secs), M_LAST)


def _first_min_open(lo, hi, ratios: bool = False) -> list:
    """Which candidates keep the first smallest of values known only within
    [lo[j], hi[j]] open (compress_with_methods keeps the first smallest size,
    fqzcomp5.c:2111-2119; metrics_method the first smallest ratio,
    :1913-1920): empty when the winner is the same for every choice of
    values, else the winner and every candidate whose interval lets it tie or
    win.  Pairs of exact values are always decided.  Values are Fractions or
    ints."""
    w = min(range(len(lo)), key=lambda j: (lo[j], j))
    out = []
    for j in range(len(lo)):
        if j == w or (lo[j] == hi[j] and lo[w] == hi[w]):
            continue
        # ratios: a margin for the reference's double arithmetic
        gap = hi[w] * (1 + 1e-9) if ratios else hi[w]
        if (j < w and not gap < lo[j]) or (j > w and not gap <= lo[j]):
            out.append(j)
    return out + [w] if out else []


def _first_min_fixed(lo, hi, ratios: bool = False) -> bool:
    return not _first_min_open(lo, hi, ratios)


def trial_decided(lo: np.ndarray, hi: np.ndarray, ids, ins, tried, sched, state_in: TrialState,
                  final: bool, why: list | None = None, open_pairs: set | None = None) -> bool:
    """Whether the trial replay (metrics_method / compress_with_methods,
    fqzcomp5.c:1899-2127) picks the same methods for every size matrix
    between lo and hi (per section and method).  The decisions that read
    sizes: each tried section keeps its first smallest candidate, and each
    completed trial window (TRIAL_WINDOW tried sections of a kind) picks the
    first smallest (csize + 1) / usize summed over it, at the next section of
    its kind (sched: the trial schedule, nonzero on trial and re-trial
    sections; tried: the methods each section tried).  Interval sizes stand
    in for exact ones only when every such decision falls inside this call
    (or the input ends with it: `final`), so the state carried out holds no
    interval-derived sums a later call could read; and not when the call
    starts inside a trial window.  open_pairs (if given) receives the
    (section, method) pairs of interval sizes that leave a decision open:
    exact sizes for them decide it."""
    from fractions import Fraction
    ids = [int(x) for x in ids]
    n = len(ids)
    for k in range(4):
        if 0 < state_in.sec[k].trial < TRIAL_WINDOW:
            return False
    ok = True

    def no(msg, pairs):
        if why is not None:
            why.append(msg)
        if open_pairs is not None:
            open_pairs.update((i, m) for i, m in pairs if lo[i, m] != hi[i, m])
        return False

    for i in range(n):
        ms = [m for m in range(M_LAST) if (int(tried[i]) >> m) & 1]
        op = _first_min_open([int(lo[i, m]) for m in ms], [int(hi[i, m]) for m in ms]) \
            if len(ms) > 1 else []
        if op:
            ok = no(f"section {i} (kind {ids[i]}): " + ", ".join(
                f"m{m} [{int(lo[i, m])}, {int(hi[i, m])}]" for m in ms),
                [(i, ms[j]) for j in op])
    for k in sorted(set(ids)):
        rows = [i for i in range(n) if ids[i] == k and sched[i]]
        for g0 in range(0, len(rows), TRIAL_WINDOW):
            grp = rows[g0:g0 + TRIAL_WINDOW]
            later = any(ids[j] == k for j in range(grp[-1] + 1, n))
            if not later:
                if final:
                    continue          # no decision follows within the input
                return False
            if len(grp) < TRIAL_WINDOW:
                return False          # (cannot happen: a window completes first)
            us, cl, ch = {}, {}, {}
            for i in grp:
                for m in range(M_LAST):
                    if (int(tried[i]) >> m) & 1:
                        us[m] = us.get(m, 0) + int(ins[i])
                        cl[m] = cl.get(m, 0) + int(lo[i, m])
                        ch[m] = ch.get(m, 0) + int(hi[i, m])
            ms = sorted(m for m in us if us[m])
            op = _first_min_open([Fraction(cl[m] + 1, us[m]) for m in ms],
                                 [Fraction(ch[m] + 1, us[m]) for m in ms], ratios=True) \
                if len(ms) > 1 else []
            if op:
                ok = no(f"window of kind {k} at sections {grp}: " + ", ".join(
                    f"m{m} [{cl[m]}, {ch[m]}]" for m in ms),
                    [(i, ms[j]) for j in op for i in grp if (int(tried[i]) >> ms[j]) & 1])
    return ok


def refine_session(secs: list, ids, sched, lo: np.ndarray, hi: np.ndarray, pairs, ins,
                   chunk_bytes: int, commit_bytes: int | None = None) -> bool:
    """refine_exact as one try session over every section, which the commit
    can then use: the open pairs exactly, and each section outside the trial
    of a kind with open candidates tries those candidates too (its method is
    the window's pick, one of them when it is open), so a decided trial
    commits with the winners already coded.  Returns False, trying nothing,
    when the session would not fit the device memory budget (~60 B per input
    byte and work candidate, 5 x chunk_bytes of such bytes), counting the
    sections the commit then codes late in the same session (one candidate
    each), and when all sections' inputs exceed the commit's chunk
    (commit_bytes): the commit of a reused session is not chunked."""
    want, kinds = {}, {}
    for i, m in pairs:
        want[i] = want.get(i, 0) | (1 << m)
        kinds[int(ids[i])] = kinds.get(int(ids[i]), 0) | (1 << m)
    for j in range(len(secs)):
        if not sched[j] and int(ids[j]) in kinds:
            want[j] = want.get(j, 0) | kinds[int(ids[j])]
    cost = sum(int(ins[i]) * max(1, bin(want[i] & WORK_MASK).count("1")) for i in want)
    cost += sum(int(ins[j]) for j in range(len(secs)) if j not in want)   # coded late
    if cost > 5 * chunk_bytes:
        return False
    if commit_bytes is not None and sum(int(x) for x in ins[:len(secs)]) > commit_bytes:
        return False
    so = _load()
    if so.fqz5_arenas_release():
        raise _lib.NativeError("fqz5_arenas_release: " + _lib.last_error())
    prev = so.fqz5_set_trial_prune(0)
    try:
        got = sections_try(secs, np.array([want.get(i, 0) for i in range(len(secs))], np.uint32))
    finally:
        so.fqz5_set_trial_prune(prev)
    for i, m in pairs:
        lo[i, m] = hi[i, m] = got[i, m]
    return True


def refine_exact(secs: list, lo: np.ndarray, hi: np.ndarray, pairs, ins, chunk_bytes: int):
    """Exact sizes for the (section, method) pairs whose intervals left a
    trial decision open: those sections try just those methods with their
    range chains (sections_try, no pruning), lo = hi = the size."""
    so = _load()
    want = {}
    for i, m in pairs:
        want[i] = want.get(i, 0) | (1 << m)
    rows = sorted(want)
    # a chunk's device memory goes with its work candidates (~60 B per input
    # byte each); a full try chunk holds ~5 of them per chunk_bytes
    cost = {i: int(ins[i]) * max(1, bin(want[i] & WORK_MASK).count("1")) for i in rows}
    prev = so.fqz5_set_trial_prune(0)
    try:
        for ch in _chunks(rows, cost, 5 * chunk_bytes):
            got = sections_try([secs[i] for i in ch], np.array([want[i] for i in ch], np.uint32))
            for r, i in enumerate(ch):
                for m in range(M_LAST):
                    if (want[i] >> m) & 1:
                        lo[i, m] = hi[i, m] = got[r, m]
    finally:
        so.fqz5_set_trial_prune(prev)


def bounds_usable(ids, sched, state_in: TrialState, final: bool) -> bool:
    """The structural half of trial_decided, known before any try: the call
    does not start inside a trial window, and every window's decision falls
    inside the call (or the input ends with it)."""
    ids = [int(x) for x in ids]
    for k in range(4):
        if 0 < state_in.sec[k].trial < TRIAL_WINDOW:
            return False
    if final:
        return True
    for k in sorted(set(ids)):
        rows = [i for i in range(len(ids)) if ids[i] == k and sched[i]]
        for g0 in range(0, len(rows), TRIAL_WINDOW):
            grp = rows[g0:g0 + TRIAL_WINDOW]
            if not any(ids[j] == k for j in range(grp[-1] + 1, len(ids))):
                return False
    return True


def _copy_state(st: TrialState) -> TrialState:
    out = TrialState()
    C.memmove(C.byref(out), C.byref(st), C.sizeof(TrialState))
    return out


def sections_commit(secs: list[Section], methods: np.ndarray) -> list[SectionResult]:
    so = _load()
    res = (SectionResult * len(secs))()
    m = np.ascontiguousarray(methods, np.int32)
    _lib.after_torch()
    rc = so.fqz5_sections_commit(_arr(Section, secs), len(secs),
                                 m.ctypes.data_as(C.POINTER(C.c_int32)), res)
    if rc:
        raise _lib.NativeError("fqz5_sections_commit: " + _lib.last_error())
    return list(res)


def decode(secs: list[Section]) -> list[SectionResult]:
    so = _load()
    res = (SectionResult * len(secs))()
    _lib.after_torch()
    if so.fqz5_decode_sections(_arr(Section, secs), len(secs), res):
        raise _lib.NativeError("fqz5_decode_sections: " + _lib.last_error())
    return list(res)


class PeerError(RuntimeError):
    """Another rank of the group failed (its error envelope arrived in an
    exchange); raised on every rank that was waiting for it."""


def xchg(obj, group=None) -> list:
    """Every rank's `obj` (rank order): the one collective of the encode and
    decode paths, all_gather_object with an error envelope.  All the paths'
    exchanges (sizes, minima, barriers) go through it, so a failing rank's
    error envelope (ranks_fail_together) always pairs with the exchange its
    peers are waiting in, whichever it is, and every rank raises."""
    ws, _ = _world(group)
    if ws == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * ws
    dist.all_gather_object(out, ("ok", obj), group=group)
    for r, (st, m) in enumerate(out):
        if st != "ok":
            raise PeerError(f"rank {r} failed: {m}")
    return [m for _, m in out]


class ranks_fail_together:
    """Context of one multi-rank call (compress_file, decompress_file, a
    bench step): every rank calls it with the same exchanges.  A rank whose
    body raises sends one error envelope as its next exchange: its peers are
    all blocked in that same exchange (no rank can pass an exchange this
    rank has not joined), receive the error and raise PeerError, so every
    rank fails at once instead of waiting for the process group's timeout.
    The body must end with an exchange (a final barrier) so that no peer can
    have left before a failure inside it."""

    def __init__(self, group=None):
        self.group = group

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        if ev is None or isinstance(ev, PeerError) or _world(self.group)[0] == 1:
            return False
        import torch.distributed as dist
        out = [None] * _world(self.group)[0]
        try:
            dist.all_gather_object(out, ("err", repr(ev)[:400]), group=self.group)
        except Exception:          # the group itself is gone: nothing to tell
            pass
        return False


def barrier(group=None) -> None:
    """A barrier as an exchange (xchg), so that it can carry a peer's error."""
    xchg(None, group)


def exchange_sizes(local: np.ndarray, in_sizes: np.ndarray, sec_ids: np.ndarray,
                   group=None):
    """All-gather the candidate sizes of every rank's sections (rank-major =
    file order).  This is the only exchange of the encode path: the trial
    state of later blocks depends on the first blocks' candidates (KB
    messages: latency-bound, so one all_gather_object, xchg)."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return local, in_sizes, sec_ids, 0
    if group is None:             # (here: the default group, all ranks)
        group = dist.group.WORLD
    ws, rk = _world(group)
    if ws == 1:
        return local, in_sizes, sec_ids, 0
    pack = np.zeros((local.shape[0], M_LAST + 2), np.int64)
    pack[:, :M_LAST] = local
    pack[:, M_LAST] = in_sizes
    pack[:, M_LAST + 1] = sec_ids
    rows = xchg(pack, group)
    allp = np.concatenate(rows, 0)
    off = sum(int(r.shape[0]) for r in rows[:rk])
    return (allp[:, :M_LAST].astype(np.uint32), allp[:, M_LAST].astype(np.uint32),
            allp[:, M_LAST + 1].astype(np.int32), off)


def encode_run(secs: list[Section], avail: np.ndarray, state: TrialState,
               group=None, speculate: bool = True, prune: bool = True,
               bounds: bool = False):
    """try -> (exchange) -> replay -> commit for this rank's sections.

    speculate: every section tries every method in one GPU launch.  A launch
    lasts as long as its longest rANS chain, so the extra candidates cost
    little, while encoding the non-trial sections after the replay would add
    a second chain-length launch.  speculate=False tries only the sections
    the schedule names (trial and re-trial blocks) and encodes the others
    once at commit, for candidates that do cost in proportion to their work.

    prune: fqz and sequence-model candidates that provably cannot win the
    trial skip their range chain (fqz5_set_trial_prune), when this rank holds
    every section the schedule has try them and they form one whole trial
    window per family.

    bounds: first try with every fqz / sequence-model range chain skipped
    (their size intervals, fqz5_set_trial_bounds); when the intervals decide
    every choice of the trial (trial_decided), the commit codes the winners
    in the same session, the trial blocks' beside the others' in one launch,
    instead of the trial's chains first and the other blocks' after them.
    Otherwise the exact tries below run as without it.  One rank, the whole
    input in this call (bounds_usable with final=True)."""
    ins = np.array([s.in_size for s in secs], np.uint32)
    ids = np.array([s.sec for s in secs], np.int32)
    av = np.asarray(avail, np.uint32)
    # name candidates are speculative too: their host tokenising runs on a
    # helper thread beside the rANS batch, and none is left for commit
    SPEC = RANS_MASK | NAME_MASK
    if speculate and not (av & WORK_MASK).any():
        masks = av[ids]
        prune = False
    else:
        blank = np.zeros((len(secs), M_LAST), np.uint32)
        _, _, g_ids0, off = exchange_sizes(blank, ins, ids, group)
        sched_all = trial_schedule(g_ids0, avail, state)
        sched = sched_all[off:off + len(secs)]
        # rANS candidates stay speculative (chain-bound, nearly free in one
        # launch); fqz candidates cost in proportion to their work, so only
        # the scheduled trial sections try them.  So does TLZP3 here: its lzp
        # pass and order-5 chain over every block's names ended after the
        # tokenisers, the names helper's long pole at -5 (a block after the
        # trial codes it at commit if it wins)
        NAME_WORK = 1 << TLZP3
        masks = ((av[ids] & np.uint32(SPEC & ~NAME_WORK & 0xFFFFFFFF)) |
                 (sched & np.uint32(WORK_MASK | NAME_WORK)) if speculate else sched)
        # pruning needs each family's trial window whole on this rank
        for fam in (FQZ_MASK, SEQ_MASK):
            rows = np.nonzero(sched_all & fam)[0]
            if len(rows) == 0:
                continue
            prune = prune and speculate and len(rows) == TRIAL_WINDOW and \
                bool(((rows >= off) & (rows < off + len(secs))).all())
        if bounds and _world(group)[0] == 1 and (sched_all & WORK_MASK).any() and \
                bounds_usable(g_ids0, sched_all, state, final=True):
            global last_bounds_decided
            state0 = _copy_state(state)
            lo, hi = sections_try_bounds(secs, masks)
            tried = np.zeros(len(secs), np.uint32)
            meth_all = trial_replay(ids, ins, lo, avail, state, tried)
            last_bounds_decided = trial_decided(lo, hi, ids, ins, tried, sched_all, state0,
                                                final=True)
            if last_bounds_decided:
                return sections_commit(secs, meth_all), meth_all, lo, tried, 0
            C.memmove(C.byref(state), C.byref(state0), C.sizeof(TrialState))
    so = _load()
    prev = so.fqz5_set_trial_prune(1 if prune else 0)
    try:
        local = sections_try(secs, masks)
    finally:
        so.fqz5_set_trial_prune(prev)
    g_sizes, g_ins, g_ids, off = exchange_sizes(local, ins, ids, group)
    tried = np.zeros(len(g_ids), np.uint32)
    meth_all = trial_replay(g_ids, g_ins, g_sizes, avail, state, tried)
    meth = meth_all[off:off + len(secs)]
    res = sections_commit(secs, meth)
    return res, meth_all, g_sizes, tried, off


def _chunks(rows, sizes, budget: int):
    """Consecutive runs of `rows` whose `sizes` sum to at most `budget`
    (at least one row each)."""
    out, cur, tot = [], [], 0
    for i in rows:
        if cur and tot + int(sizes[i]) > budget:
            out.append(cur)
            cur, tot = [], 0
        cur.append(i)
        tot += int(sizes[i])
    if cur:
        out.append(cur)
    return out


def encode_run_bounded(secs: list[Section], avail: np.ndarray, state: TrialState,
                       group=None, chunk_bytes: int = 600_000_000,
                       commit_bytes: int = 2_400_000_000, bounds: bool = True,
                       merge_commit: bool = True):
    """encode_run for the large-block presets (-7: 500 MB, -9: 1 GB blocks),
    in bounded device memory: the same choices and bytes, at the cost of
    coding each trial section's winner twice.

    A trial section of -7/-9 tries up to 13 methods, five of them fqz (about
    60 B of events, sort buffers and coder records per quality byte) and five
    sequence models (about as much per base): a trial window of 500 MB blocks
    tried at once needs more than one GPU's 288 GB.  Here the sections the
    schedule has try methods are tried a chunk at a time (input bytes summed
    up to `chunk_bytes`, one section at least), only their sizes kept (each
    try rewinds the last one's buffers); the replay picks every section's
    method from the sizes as encode_run does; then every section is coded
    with its one method a chunk at a time (fqz5_sections_commit codes the
    methods a session did not try, "late").  A commit codes one candidate
    per section (at most ~64 B of device memory per input byte, an fqz
    section's), so its chunks are `commit_bytes` of input: the range chains
    of several blocks' fqz / sequence-model sections then run side by side
    instead of one chunk after another (-7: the four 250 MB quality
    sections' FQZ0 chains in one launch).

    bounds: the tries skip every fqz / sequence-model range chain and give
    size intervals (fqz5_set_trial_bounds); trial_decided checks that the
    intervals fix every choice the trial makes (else the tries run again with
    exact sizes), so the choices are those of exact sizes.  The returned
    sizes then hold the intervals' lower ends for those candidates.  The
    call is taken to hold the whole input (a decision left for a later call
    would read interval sums from the state).  merge_commit: on one rank, the
    refinement of open decisions is one session over every section
    (refine_session) that the commit then reuses."""
    ins = np.array([s.in_size for s in secs], np.uint32)
    ids = np.array([s.sec for s in secs], np.int32)
    blank = np.zeros((len(secs), M_LAST), np.uint32)
    _, _, g_ids0, off = exchange_sizes(blank, ins, ids, group)
    sched_all = trial_schedule(g_ids0, avail, state)
    session = False
    sched = sched_all[off:off + len(secs)]
    so = _load()
    state0 = _copy_state(state)
    tries = [i for i in range(len(secs)) if sched[i]]

    def try_all(use_bounds: bool):
        lo = np.full((len(secs), M_LAST), np.iinfo(np.uint32).max, np.uint32)
        hi = lo.copy()
        prev = so.fqz5_set_trial_prune(0)     # pruning needs a whole trial window per try
        try:
            for ch in _chunks(tries, ins, chunk_bytes):
                part = [secs[i] for i in ch]
                if use_bounds:
                    lo[ch], hi[ch] = sections_try_bounds(part, sched[ch])
                else:
                    lo[ch] = hi[ch] = sections_try(part, sched[ch])
        finally:
            so.fqz5_set_trial_prune(prev)
        if use_bounds and bounds_widen:        # tests: leave decisions open
            iv = lo != hi
            hi[iv] = np.minimum(hi[iv].astype(np.int64) + bounds_widen, 2**32 - 2).astype(np.uint32)
        return lo, hi

    # First the fqz / sequence-model candidates' size intervals only (no
    # range chains): when they separate the candidates of every decision
    # the trial makes, the winners are coded once at commit; else the tries
    # run again with exact sizes.
    bounds = bounds and bounds_usable(g_ids0, sched_all, state, final=True)
    lo, hi = try_all(bounds)
    g_sizes, g_ins, g_ids, off = exchange_sizes(lo, ins, ids, group)
    tried = np.zeros(len(g_ids), np.uint32)
    meth_all = trial_replay(g_ids, g_ins, g_sizes, avail, state, tried)
    if bounds:
        g_hi = exchange_sizes(hi, ins, ids, group)[0]
        # every rank sees the same rows, so every rank decides the same
        import sys
        single = group is None or _world(group)[0] == 1
        ok = False
        session = False      # the last try session covers every section
        for _ in range(M_LAST):
            why, pairs = [], set()
            ok = trial_decided(g_sizes, g_hi, g_ids, g_ins, tried, sched_all, state0,
                               final=True, why=why, open_pairs=pairs)
            if ok or not pairs or not single:
                break
            # exact sizes for the candidates that leave a decision open,
            # then the replay again from the entry state
            print(f"[sections] size intervals leave a trial decision open ({why[0]}): "
                  f"{len(pairs)} candidates coded exactly", file=sys.stderr, flush=True)
            session = merge_commit and not session and refine_session(
                secs, ids, sched, lo, hi, sorted(pairs), ins, chunk_bytes, commit_bytes)
            if not session:
                refine_exact(secs, lo, hi, sorted(pairs), ins, chunk_bytes)
            g_sizes, g_hi = lo, hi
            C.memmove(C.byref(state), C.byref(state0), C.sizeof(TrialState))
            tried = np.zeros(len(g_ids), np.uint32)
            meth_all = trial_replay(g_ids, g_ins, g_sizes, avail, state, tried)
        global last_bounds_decided
        last_bounds_decided = ok
        if not ok:
            print(f"[sections] size intervals do not decide the trial ({why[0] if why else ''}): "
                  "trying again with exact sizes", file=sys.stderr, flush=True)
            C.memmove(C.byref(state), C.byref(state0), C.sizeof(TrialState))
            lo, _ = try_all(False)
            g_sizes, g_ins, g_ids, off = exchange_sizes(lo, ins, ids, group)
            tried = np.zeros(len(g_ids), np.uint32)
            meth_all = trial_replay(g_ids, g_ins, g_sizes, avail, state, tried)
    meth = meth_all[off:off + len(secs)]
    if bounds and last_bounds_decided and session:
        # the refinement's session tried every section's possible winners:
        # the commit codes the rest (late) and reuses those
        return sections_commit(secs, meth), meth_all, g_sizes, tried, off
    # the tries' arenas (helper contexts) back to the device before the
    # commit's candidates take theirs
    if so.fqz5_arenas_release():
        raise _lib.NativeError("fqz5_arenas_release: " + _lib.last_error())
    res = []
    for ch in _chunks(range(len(secs)), ins, max(commit_bytes, chunk_bytes)):
        part = [secs[i] for i in ch]
        sections_try(part, np.zeros(len(ch), np.uint32))    # an empty session
        res += sections_commit(part, meth[ch])
    return res, meth_all, g_sizes, tried, off


def _world(group):
    import torch.distributed as dist
    if group is None or not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def allreduce_min(a: np.ndarray, group) -> np.ndarray:
    """Element-wise minimum over the ranks of `group` (an exchange, xchg)."""
    if _world(group)[0] == 1:
        return a
    parts = xchg(np.ascontiguousarray(a, np.int64), group)
    return np.minimum.reduce(parts).astype(a.dtype)


def work_share(methods: list[int], world: int, rank: int) -> int:
    """The work-candidate methods (fqz, sequence models, LZP3) this rank
    tries for the trial sections: method j of the sorted list goes to rank
    j mod world, so one rank holds a method for the whole trial window (the
    exact pruning needs that) and the ranks split the windows' chains."""
    m = 0
    for j, meth in enumerate(sorted(methods)):
        if j % world == rank:
            m |= 1 << meth
    return m


def encode_window(secs: list, ids, ins, owner, avail: np.ndarray,
                  state: TrialState, group=None, bounded: bool = False,
                  chunk_bytes: int = 600_000_000, prune: bool = True,
                  commit_bytes: int = 2_400_000_000, bounds: bool = True,
                  final: bool = False, bounds_first: bool = False):
    """Code the sections of consecutive blocks (file order) over the ranks of
    `group`; every rank passes the same section ids / input sizes / owners,
    its Section for every section it holds the data of (None elsewhere) and
    the same state.  owner[i] is the rank that commits
    section i; the trial sections (the schedule's trial and re-trial blocks)
    are tried on every rank that holds them, each rank trying its share of
    the work candidates (work_share) plus every rANS / name candidate, so
    that the serial fqz and sequence-model chains of a trial window run on
    as many GPUs as there are methods, not all on the first block's owner.
    One collective, an element-wise minimum of the candidate sizes (a size
    is the same wherever it is computed; untried candidates are UINT32_MAX),
    then every rank replays the trial (fqz5_trial_replay, file order) and
    commits its own sections.

    bounded: the -7/-9 path of encode_run_bounded (tries chunked by
    chunk_bytes, no pruning, every section coded again at commit, in chunks
    of commit_bytes; with `bounds`, the work candidates' size intervals
    first, as in encode_run_bounded; final: the input ends with this call).
    bounds_first (not bounded, one rank): encode_run's bounds option, the
    work candidates' size intervals first and, when they decide the trial,
    the commit in the same session (-5: the trial blocks' fqz chains beside
    the other blocks' in one launch).
    Returns (results: SectionResult per section or None when not owned,
    methods of every section, sizes)."""
    ws, rk = _world(group)
    n = len(secs)
    ids = np.asarray(ids, np.int32)
    ins = np.asarray(ins, np.uint32)
    owner = np.asarray(owner, np.int64)
    av = np.asarray(avail, np.uint32)
    sched = trial_schedule(ids, av, state)
    SPEC = RANS_MASK | NAME_MASK
    work = sorted({m for i in range(n) for m in range(M_LAST) if (int(sched[i]) >> m) & 1
                   and (1 << m) & WORK_MASK})
    share = work_share(work, ws, rk)
    masks = np.zeros(n, np.uint32)
    for i in range(n):
        mine = owner[i] == rk
        if bounded:
            # the scheduled sections only (their rANS on the owner), the
            # rest coded once at commit
            if sched[i]:
                masks[i] = (int(sched[i]) & ~WORK_MASK & (SPEC if mine else 0)) | \
                    (int(sched[i]) & share)
        else:
            if mine:
                masks[i] = int(av[ids[i]]) & SPEC
            if sched[i] and (int(sched[i]) & share):
                # the exact pruning of this rank's methods needs the earlier
                # methods' sizes of the whole trial window here
                masks[i] |= (int(sched[i]) & SPEC) | (int(sched[i]) & share)
    rows = [i for i in range(n) if masks[i] or owner[i] == rk]
    for i in rows:
        if secs[i] is None:
            raise ValueError(f"section {i}: rank {rk} needs its data")
    local = np.full((n, M_LAST), np.iinfo(np.uint32).max, np.uint32)
    hi_local = None
    so = _load()
    state0 = _copy_state(state)
    use_bounds = bounded and bounds and bounds_usable(ids, sched, state, final)

    def bounded_tries(with_bounds: bool):
        lo = np.full((n, M_LAST), np.iinfo(np.uint32).max, np.uint32)
        hi = lo.copy()
        prev = so.fqz5_set_trial_prune(0)
        try:
            tried_rows = [i for i in rows if masks[i]]
            for ch in _chunks(tried_rows, ins, chunk_bytes):
                part = [secs[i] for i in ch]
                if with_bounds:
                    lo[ch], hi[ch] = sections_try_bounds(part, masks[ch])
                else:
                    lo[ch] = hi[ch] = sections_try(part, masks[ch])
        finally:
            so.fqz5_set_trial_prune(prev)
        return lo, hi

    pre = None                     # (sizes, tried, methods) decided by bounds_first
    if bounded:
        local, hi_local = bounded_tries(use_bounds)
    else:
        if bounds_first and ws == 1 and rows and bool((sched & WORK_MASK).any()) and \
                bounds_usable(ids, sched, state, final):
            global last_bounds_decided
            lo = np.full((n, M_LAST), np.iinfo(np.uint32).max, np.uint32)
            hi = lo.copy()
            lo[rows], hi[rows] = sections_try_bounds([secs[i] for i in rows], masks[rows])
            t0 = np.zeros(n, np.uint32)
            m0 = trial_replay(ids, ins, lo, av, state, t0)
            last_bounds_decided = trial_decided(lo, hi, ids, ins, t0, sched, state0, final)
            if last_bounds_decided:
                pre = (lo, t0, m0)
            else:
                C.memmove(C.byref(state), C.byref(state0), C.sizeof(TrialState))
        if pre is None:
            # pruning of a family: its trial window whole in this call
            for fam in (FQZ_MASK, SEQ_MASK):
                frows = np.nonzero(sched & fam)[0]
                if len(frows):
                    prune = prune and len(frows) == TRIAL_WINDOW
            prev = so.fqz5_set_trial_prune(1 if prune else 0)
            try:
                if rows:
                    local[rows] = sections_try([secs[i] for i in rows], masks[rows])
            finally:
                so.fqz5_set_trial_prune(prev)
    if pre is not None:
        sizes, tried, meth = pre
    else:
        sizes = allreduce_min(local, group)
        tried = np.zeros(n, np.uint32)
        meth = trial_replay(ids, ins, sizes, av, state, tried)
    if use_bounds:
        hi_all = allreduce_min(hi_local, group)
        for _ in range(M_LAST):
            pairs = set()
            last_bounds_decided = trial_decided(sizes, hi_all, ids, ins, tried, sched, state0,
                                                final, open_pairs=pairs)
            if last_bounds_decided or not pairs:
                break
            # exact sizes for the candidates left open (every rank holds the
            # trial sections; the pairs are dealt out over the ranks and the
            # sizes combined by the same element-wise minimum), replay again
            held = [pr for pr in sorted(pairs) if secs[pr[0]] is not None]
            # stop refining on every rank together when any rank lacks a
            # section's data (the collectives below must pair up)
            if ws > 1 and int(allreduce_min(np.array([int(len(held) == len(pairs))]), group)[0]) == 0:
                break
            mine_p = held[rk::ws]
            ex = np.full((n, M_LAST), np.iinfo(np.uint32).max, np.uint32)
            ex_hi = ex.copy()
            if mine_p:
                refine_exact(secs, ex, ex_hi, mine_p, ins, chunk_bytes)
            ex = allreduce_min(ex, group)
            for i, m in pairs:
                sizes[i, m] = hi_all[i, m] = ex[i, m]
            C.memmove(C.byref(state), C.byref(state0), C.sizeof(TrialState))
            tried = np.zeros(n, np.uint32)
            meth = trial_replay(ids, ins, sizes, av, state, tried)
        if not last_bounds_decided:        # the intervals overlap: exact sizes
            C.memmove(C.byref(state), C.byref(state0), C.sizeof(TrialState))
            local, _ = bounded_tries(False)
            sizes = allreduce_min(local, group)
            tried = np.zeros(n, np.uint32)
            meth = trial_replay(ids, ins, sizes, av, state, tried)
    res: list = [None] * n
    mine = [i for i in rows if owner[i] == rk]
    if bounded:
        if so.fqz5_arenas_release():
            raise _lib.NativeError("fqz5_arenas_release: " + _lib.last_error())
        for ch in _chunks(mine, ins, max(commit_bytes, chunk_bytes)):
            part = [secs[i] for i in ch]
            sections_try(part, np.zeros(len(ch), np.uint32))    # an empty session
            for i, r in zip(ch, sections_commit(part, meth[ch])):
                res[i] = r
    elif rows:
        m = np.where(owner[rows] == rk, meth[rows], 0).astype(np.int32)
        for i, r in zip(rows, sections_commit([secs[i] for i in rows], m)):
            if owner[i] == rk:
                res[i] = r
    return res, meth, sizes


def fqz_bound(n: int) -> int:
    """Room the fqz encoder needs: the coder's bound (fqz_codec.cpp) plus
    the parameter header."""
    return int(n * 1.1) + 100000 + 16384


class BlockParts(C.Structure):
    """fqz5_block_parts"""
    _fields_ = [("nrec", C.c_int32), ("name", C.c_void_p), ("name_size", C.c_uint32),
                ("lengths", C.c_void_p), ("lengths_size", C.c_uint32),
                ("seq", C.c_void_p), ("seq_size", C.c_uint32),
                ("qual", C.c_void_p), ("qual_size", C.c_uint32)]


class BlockView(C.Structure):
    """fqz5_block_view"""
    _fields_ = [("block_size", C.c_uint32), ("nrec", C.c_uint32), ("crc_ok", C.c_int32),
                ("name_off", C.c_uint32), ("name_size", C.c_uint32), ("name_ulen", C.c_uint32),
                ("fixed_len", C.c_int32), ("seq_off", C.c_uint32), ("seq_size", C.c_uint32),
                ("seq_ulen", C.c_uint32), ("qual_off", C.c_uint32), ("qual_size", C.c_uint32),
                ("qual_ulen", C.c_uint32)]


_bound_blk = False


def _load_blk():
    global _bound_blk
    so = _load()
    if not _bound_blk:
        so.fqz5_name_flags.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]
        so.fqz5_block_lengths.restype = C.c_int
        so.fqz5_block_lengths.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.c_int32,
                                          C.c_void_p, C.c_uint32]
        so.fqz5_block_size.restype = C.c_uint64
        so.fqz5_block_size.argtypes = [C.POINTER(BlockParts)]
        so.fqz5_blocks_assemble.restype = C.c_int
        so.fqz5_blocks_assemble.argtypes = [C.POINTER(BlockParts), C.c_int, C.c_void_p,
                                            C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        so.fqz5_block_parse.restype = C.c_int
        so.fqz5_block_parse.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(BlockView),
                                        C.POINTER(C.c_uint32), C.c_uint32]
        so.fqz5_blocks_parse_v.restype = C.c_int
        so.fqz5_blocks_parse_v.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_int,
                                           C.c_int, C.POINTER(BlockView),
                                           C.POINTER(C.POINTER(C.c_uint32)),
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_int32)]
        so.fqz5_block_parse_v.restype = C.c_int
        so.fqz5_block_parse_v.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.POINTER(BlockView),
                                          C.POINTER(C.c_uint32), C.c_uint32]
        _bound_blk = True
    return so


def name_flags(names: np.ndarray, nrec: int) -> np.ndarray:
    """load_seqs_kseq's per-record flags from the names (fqz5_name_flags)."""
    out = np.zeros(nrec, np.uint32)
    nb = np.ascontiguousarray(names, np.uint8)
    _load_blk().fqz5_name_flags(nb.ctypes.data, len(nb), nrec,
                                out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def block_lengths(lens: np.ndarray, fixed_len: int) -> bytes:
    ln = np.ascontiguousarray(lens, np.uint32)
    buf = C.create_string_buffer(5 * len(ln) + 16)
    n = _load_blk().fqz5_block_lengths(ln.ctypes.data_as(C.POINTER(C.c_uint32)), len(ln),
                                       fixed_len, buf, len(buf))
    if n < 0:
        raise _lib.NativeError("fqz5_block_lengths")
    return buf.raw[:n]


def parse_blocks(ptrs, sizes, nrecs, version: int = 0, lens_out=None):
    """fqz5_blocks_parse_v over device blocks (addresses, byte sizes, record
    counts from the headers): per block its BlockView and record lengths.
    lens_out: the callers' length arrays to fill (uint32, one per block, at
    least max(nrec, 1) long; a caller that parses the same blocks every step
    keeps them, instead of ~45 MB of fresh pages a -5 NovaSeq step)."""
    so = _load_blk()
    n = len(ptrs)
    views = (BlockView * max(n, 1))()
    if lens_out is not None:
        lens = lens_out
        if len(lens) != n or any(len(x) < max(k, 1) or x.dtype != np.uint32
                                 for x, k in zip(lens, nrecs)):
            raise ValueError("parse_blocks: lens_out does not fit the blocks")
    else:
        lens = [np.zeros(max(k, 1), np.uint32) for k in nrecs]
    lp = (C.POINTER(C.c_uint32) * max(n, 1))(*[x.ctypes.data_as(C.POINTER(C.c_uint32)) for x in lens])
    caps = (C.c_uint32 * max(n, 1))(*[len(x) for x in lens])
    st = (C.c_int32 * max(n, 1))()
    _lib.after_torch()
    if so.fqz5_blocks_parse_v((C.c_void_p * max(n, 1))(*ptrs), (C.c_uint64 * max(n, 1))(*sizes), n,
                              version, views, lp, caps, st):
        raise _lib.NativeError("fqz5_block_parse: " + _lib.last_error())
    return [(views[i], lens[i][:views[i].nrec]) for i in range(n)]


class Run:
    """Device buffers and sections of a run of blocks in file order, each
    block a name (when the reads carry names), a sequence and a quality
    section (encode_block order).  The quality sections carry the records
    (FQZ methods) and point at their block's sequence bytes: the input when
    encoding, the decoded sequence section when decoding.

    With names, `assemble` writes whole .fqz5 blocks (fqz5_blocks_assemble:
    header, CRC32, lengths) and `parse` reads them back (fqz5_block_parse)."""

    def __init__(self, reads, blocks, device, names: bool | None = None):
        import torch
        from . import synth
        self.reads, self.blocks = reads, blocks
        self.names = reads.has_names() if names is None else names
        offs = np.concatenate([[0], np.cumsum(reads.lens.astype(np.int64))])
        self.seq_d = torch.from_numpy(reads.seq).to(device)
        self.qual_d = torch.from_numpy(reads.qual).to(device)
        self.name_h = self.name_off = self.name_d = None
        if self.names:
            self.name_h, self.name_off = synth.all_names(reads)
            self.name_d = torch.from_numpy(self.name_h).to(device)
        lens, flags, nranges, sranges = [], [], [], []
        for a, b in blocks:
            lens.append(np.ascontiguousarray(reads.lens[a:b], np.uint32))
            sranges.append((int(offs[a]), int(offs[b])))
            if self.names:          # load_seqs_kseq derives them from the names
                ns, ne = int(self.name_off[a]), int(self.name_off[b])
                nranges.append((ns, ne))
                flags.append(name_flags(self.name_h[ns:ne], b - a))
            elif getattr(reads, "flags", None) is not None:
                flags.append(np.ascontiguousarray(reads.flags[a:b], np.uint32))
            else:
                flags.append(None)
        self._setup(lens, flags, nranges if self.names else None, sranges)

    @classmethod
    def from_device(cls, name_d, seq_d, qual_d, name_ranges, seq_ranges, lens, flags,
                    fasta=None):
        """A run over section inputs already in device memory (the FASTQ
        parser's gathered blocks, fqz5file.py): per block its name and
        sequence/quality byte ranges, record lengths and READ2 flags.
        fasta: per block, no quality section (load_seqs_kseq's per-block
        rule, fqzcomp5.c:574-578); every block when qual_d is None."""
        run = cls.__new__(cls)
        run.reads = None
        run.blocks = [(0, len(ln)) for ln in lens]
        run.names = True
        run.name_d, run.seq_d, run.qual_d = name_d, seq_d, qual_d   # qual_d None: FASTA
        run.name_h = run.name_off = None
        run.blk_fasta = list(fasta) if fasta is not None else None
        run._setup([np.ascontiguousarray(ln, np.uint32) for ln in lens],
                   [np.ascontiguousarray(f, np.uint32) for f in flags], name_ranges, seq_ranges)
        return run

    def _setup(self, lens, flags, name_ranges, seq_ranges):
        """Sections (name, seq, qual per block), their encode / decode buffers."""
        import torch
        device = self.seq_d.device
        nblk = len(lens)
        bf = getattr(self, "blk_fasta", None)
        self.blk_fasta = [self.qual_d is None or bool(bf is not None and bf[k])
                          for k in range(nblk)]
        self.blk_sec0 = []            # per block: its first section's index
        self.spans, self.lens, self.flags, self.fixed, self.lengths = [], [], [], [], []
        for k, (ln, fg, (s, e)) in enumerate(zip(lens, flags, seq_ranges)):
            fl = int(ln[0]) if len(ln) and bool(np.all(ln == ln[0])) else 0
            self.blk_sec0.append(len(self.spans))
            self.lens.append(ln)
            self.flags.append(fg)
            self.fixed.append(fl)
            if name_ranges is not None:
                self.lengths.append(block_lengths(ln, fl if len(ln) else -1))
                ns, ne = name_ranges[k]
                self.spans.append((SEC_NAME, ns, ne, 0, k))
            self.spans.append((SEC_SEQ, s, e, fl, k))
            if not self.blk_fasta[k]:         # FASTA blocks: no quality section
                self.spans.append((SEC_QUAL, s, e, fl, k))
        caps = []
        for sec, s, e, fl, _ in self.spans:
            n = e - s
            if sec == SEC_NAME:    # encode_names' buffer (fqzcomp5.c:1412) and then some
                caps.append(2 * n + 1000 + 65536)
                continue
            caps.append(9 + max(max(_lib.compress_bound(n, o) for o in
                                    (0, 1, 64, 65, 128, 129, 192, 193, (fl << 8) + 9)),
                                fqz_bound(n)))
        self.enc_buf = torch.empty(sum(caps), dtype=torch.uint8, device=device)
        self._dec_buf = None          # decode outputs, allocated on first use
        self.enc, self.dec = [], []
        eo = do = 0
        for (sec, s, e, fl, k), cap in zip(self.spans, caps):
            self.enc.append((eo, cap))
            self.dec.append(do)
            eo += cap
            do += e - s
        self.in_bytes = sum(e - s for _, s, e, _, _ in self.spans)
        self.blk_buf = None
        self.blk_off = None

    @property
    def dec_buf(self):
        import torch
        if self._dec_buf is None:
            self._dec_buf = torch.empty(max(sum(e - s for _, s, e, _, _ in self.spans), 1),
                                        dtype=torch.uint8, device=self.seq_d.device)
        return self._dec_buf

    def _src(self, sec):
        return {SEC_NAME: self.name_d, SEC_SEQ: self.seq_d, SEC_QUAL: self.qual_d}[sec]

    def _rec(self, k):
        ln = self.lens[k]
        return ln.ctypes.data_as(C.POINTER(C.c_uint32)), len(ln)

    def _flags(self, k):
        f = self.flags[k]
        return None if f is None else f.ctypes.data_as(C.POINTER(C.c_uint32))

    def enc_secs(self) -> list[Section]:
        out = []
        for (sec, s, e, fl, k), (eo, cap) in zip(self.spans, self.enc):
            src = self._src(sec)
            rl, nr = self._rec(k)
            out.append(Section(src.data_ptr() + s, self.enc_buf.data_ptr() + eo, e - s, cap,
                               fl, sec, rl, self._flags(k), nr,
                               self.seq_d.data_ptr() + s if sec == SEC_QUAL else None))
        return out

    def _seq_dec(self, i):
        """The decoded sequence section of the block of section i."""
        j = i - 1
        while self.spans[j][0] != SEC_SEQ:
            j -= 1
        return self.dec_buf.data_ptr() + self.dec[j]

    def dec_secs(self, res) -> list[Section]:
        out = []
        for i, ((sec, s, e, fl, k), (eo, cap), do, r) in enumerate(
                zip(self.spans, self.enc, self.dec, res)):
            rl, nr = self._rec(k)
            seq = self._seq_dec(i) if sec == SEC_QUAL else None
            size = r.clen if sec == SEC_NAME else 9 + r.clen
            out.append(Section(self.enc_buf.data_ptr() + eo, self.dec_buf.data_ptr() + do,
                               size, e - s, 0, sec, rl, self._flags(k), nr, seq))
        return out

    def chosen(self, res, i) -> bytes:
        """The i-th section's chosen stream (without the 9-byte frame; a name
        section whole)."""
        eo, _ = self.enc[i]
        skip = 0 if self.spans[i][0] == SEC_NAME else 9
        return self.enc_buf[eo + skip:eo + 9 + res[i].clen].cpu().numpy().tobytes() \
            if skip else self.enc_buf[eo:eo + res[i].clen].cpu().numpy().tobytes()

    def roundtrip_ok(self) -> bool:
        import torch
        ok = True
        for (sec, s, e, _, _), do in zip(self.spans, self.dec):
            src = self._src(sec)
            ok = ok and bool(torch.equal(self.dec_buf[do:do + e - s], src[s:e]))
        return ok

    # ---- whole blocks (encode_block / decode_block) -----------------------
    def _parts(self, res, which=None) -> list[BlockParts]:
        assert self.names, "blocks need the name sections"
        parts = []
        base = self.enc_buf.data_ptr()
        for b in (range(len(self.blocks)) if which is None else which):
            i = self.blk_sec0[b]
            (eo_n, _), (eo_s, _) = self.enc[i], self.enc[i + 1]
            ln = self.lengths[b]
            q, qs = None, 0                   # FASTA: 9 zero bytes (fqzcomp5.c:2258-2264)
            if not self.blk_fasta[b]:
                q, qs = base + self.enc[i + 2][0], 9 + res[i + 2].clen
            parts.append(BlockParts(len(self.lens[b]), base + eo_n, res[i].clen,
                                    C.cast(C.c_char_p(ln), C.c_void_p), len(ln),
                                    base + eo_s, 9 + res[i + 1].clen, q, qs))
        return parts

    def secs_per_block(self, b: int = 0) -> int:
        """Sections of block b: name, seq, qual (2 for a FASTA block)."""
        return 2 if self.blk_fasta[b] else 3

    def assemble(self, res, which=None):
        """Write every block (or the blocks `which`, in that order) with
        fqz5_blocks_assemble into self.blk_buf at self.blk_off; returns the
        block sizes."""
        import torch
        so = _load_blk()
        parts = self._parts(res, which)
        sizes = [int(so.fqz5_block_size(C.byref(p))) for p in parts]
        off = np.zeros(len(parts) + 1, np.uint64)
        np.cumsum(sizes, out=off[1:])
        if self.blk_buf is None or self.blk_buf.numel() < int(off[-1]):
            self.blk_buf = torch.empty(int(off[-1]) + 64, dtype=torch.uint8,
                                       device=self.seq_d.device)
        self.blk_off = off
        out = np.zeros(len(parts), np.uint32)
        _lib.after_torch(self.seq_d.device)
        rc = so.fqz5_blocks_assemble(_arr(BlockParts, parts), len(parts), self.blk_buf.data_ptr(),
                                     off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                     out.ctypes.data_as(C.POINTER(C.c_uint32)))
        if rc:
            raise _lib.NativeError("fqz5_blocks_assemble: " + _lib.last_error())
        return out

    def block_bytes(self, b: int) -> bytes:
        s, e = int(self.blk_off[b]), int(self.blk_off[b + 1])
        return self.blk_buf[s:e].cpu().numpy().tobytes()

    def parse(self, b: int) -> tuple[BlockView, np.ndarray]:
        """fqz5_block_parse of block b of blk_buf: its view and lengths."""
        so = _load_blk()
        v = BlockView()
        s, e = int(self.blk_off[b]), int(self.blk_off[b + 1])
        nrec = len(self.lens[b])
        lens = np.zeros(max(nrec, 1), np.uint32)
        _lib.after_torch(self.seq_d.device)
        if so.fqz5_block_parse(self.blk_buf.data_ptr() + s, e - s, C.byref(v),
                               lens.ctypes.data_as(C.POINTER(C.c_uint32)), len(lens)):
            raise _lib.NativeError("fqz5_block_parse: " + _lib.last_error())
        return v, lens[:v.nrec]

    def block_dec_secs(self) -> list[Section]:
        """Decode sections that read the assembled blocks (after parse: one
        batched fqz5_blocks_parse_v for all of them)."""
        out = []
        base = self.blk_buf.data_ptr()
        nrecs = [len(self.lens[b]) for b in range(len(self.blocks))]
        if getattr(self, "_plens", None) is None:
            self._plens = [np.zeros(max(k, 1), np.uint32) for k in nrecs]
        parsed = parse_blocks([base + int(self.blk_off[b]) for b in range(len(self.blocks))],
                              [int(self.blk_off[b + 1] - self.blk_off[b])
                               for b in range(len(self.blocks))],
                              nrecs, lens_out=self._plens)
        for b in range(len(self.blocks)):
            v, lens = parsed[b]
            if not v.crc_ok:
                raise _lib.NativeError(f"block {b}: CRC mismatch")
            if not np.array_equal(lens, self.lens[b]):
                raise _lib.NativeError(f"block {b}: lengths differ")
            bo = int(self.blk_off[b])
            per = self.secs_per_block(b)
            for j, (off, size) in enumerate(((v.name_off, v.name_size),
                                             (v.seq_off, v.seq_size),
                                             (v.qual_off, v.qual_size))[:per]):
                i = self.blk_sec0[b] + j
                sec, s, e, fl, k = self.spans[i]
                rl, nr = self._rec(k)
                seq = self._seq_dec(i) if sec == SEC_QUAL else None
                out.append(Section(base + bo + off, self.dec_buf.data_ptr() + self.dec[i],
                                   size, e - s, 0, sec, rl, self._flags(k), nr, seq))
        return out
