"""Seeded fqzcomp_qual test blocks (inputs are regenerated, not stored).

Each case is (name, qual bytes as q-33 values, lens, flags, seq or None).
The mix covers the branches of fqz_pick_parameters / fqz_qual_stats
(htscodecs/fqzcomp_qual.c:424-1001): symbol counts <=4 / <=8 / >8, input
sizes below 300000 and 5000000, fixed and variable lengths, READ2 flags
(the r2 split), duplicate records (dedup), HiFi '~'-dominant quals (strat
3 qtab), sequence context (strats 3/4) and degenerate blocks.
"""
from __future__ import annotations

import numpy as np

F_READ2 = 128
ILLUMINA8 = np.array([2, 6, 15, 22, 27, 33, 37, 40], np.uint8)
NOVA4 = np.array([2, 12, 23, 37], np.uint8)


def _walk(rng, n, lo=2, hi=41):
    steps = rng.integers(-3, 4, n)
    q = np.clip(np.cumsum(steps) % (hi - lo + 1) + lo, lo, hi)
    return q.astype(np.uint8)


def _records(rng, nrec, lens, kind):
    out = []
    for L in lens:
        if kind == "bin8":
            q = _walk(rng, L)
            q = ILLUMINA8[np.searchsorted(ILLUMINA8, q, side="right") - 1]
        elif kind == "nova":
            q = rng.choice(NOVA4, L, p=[.01, .04, .10, .85])
        elif kind == "q40":
            q = _walk(rng, L)
        elif kind == "hifi":
            q = np.where(rng.random(L) < 0.7, 93, rng.integers(5, 60, L)).astype(np.uint8)
        else:
            raise ValueError(kind)
        out.append(q.astype(np.uint8))
    return out


def _seq(rng, lens):
    return np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(sum(lens)))].tobytes()


def cases():
    rng = np.random.default_rng(20240601)
    res = []

    def add(name, recs, flags=None, seq=False):
        lens = np.array([len(r) for r in recs], np.uint32)
        q = np.concatenate(recs).tobytes() if recs else b""
        fl = np.zeros(len(recs), np.uint32) if flags is None else np.asarray(flags, np.uint32)
        res.append((name, q, lens, fl, _seq(rng, lens) if seq else None))

    add("bin8_small", _records(rng, 0, [150] * 500, "bin8"))
    add("bin8_mid", _records(rng, 0, [150] * 2400, "bin8"))
    add("nova_mid", _records(rng, 0, [150] * 2400, "nova"))
    add("nova_small", _records(rng, 0, [100] * 300, "nova"))
    add("q40_mid", _records(rng, 0, [150] * 2400, "q40"))
    add("q40_var", _records(rng, 0, list(rng.integers(30, 260, 2000)), "q40"))
    add("bin8_paired", _records(rng, 0, [150] * 2400, "bin8"),
        flags=[F_READ2 * (i & 1) for i in range(2400)])
    recs = _records(rng, 0, [120] * 2000, "q40")
    for i in range(1, 2000, 7):
        recs[i] = recs[i - 1].copy()
    add("q40_dups", recs)
    add("hifi", _records(rng, 0, list(rng.integers(800, 1500, 300)), "hifi"), seq=True)
    add("bin8_seq", _records(rng, 0, [150] * 2400, "bin8"), seq=True)
    add("q40_seq_var", _records(rng, 0, list(rng.integers(50, 400, 1200)), "q40"), seq=True)
    add("bin8_big", _records(rng, 0, [150] * 36000, "bin8"))
    add("one_record", _records(rng, 0, [150], "q40"))
    add("tiny_var", _records(rng, 0, [1, 2, 3, 200, 5], "q40"))
    return res


STRATS = (0, 1, 2, 3, 4)
