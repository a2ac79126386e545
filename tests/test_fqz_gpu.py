"""GPU parity of fqz_compress / fqz_decompress through the C-ABI: the
reference-generated golden vectors (tests/golden/fqz.json), random blocks
against the oracle restatement, and round trips."""
import hashlib
import json
import os

import numpy as np
import pytest

from fqz_cases import cases
from fqzcomp5_amd import lib
from oracle import binding

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


@pytest.fixture(scope="module")
def golden():
    vec = json.load(open(os.path.join(HERE, "golden", "fqz.json")))
    blob = open(os.path.join(HERE, "golden", "fqz_small.bin"), "rb").read()
    return {c[0]: c for c in cases()}, vec, blob


def test_fqz_golden_compress(golden):
    cs, vec, _ = golden
    bad = []
    for v in vec:
        if v["case"] == "bin8_big":
            continue                      # covered by the round-trip test
        name, q, lens, flags, seq = cs[v["case"]]
        fl = flags.copy()
        out = lib.fqz_compress(q, lens.copy(), fl, v["strat"], seq)
        if (len(out), hashlib.md5(out).hexdigest()) != (v["len"], v["md5"]):
            bad.append((v["case"], v["strat"], len(out), v["len"]))
        assert (fl == flags).all()        # selector bits cleared again
    assert not bad, bad


def test_fqz_golden_decompress(golden):
    cs, vec, blob = golden
    for v in vec:
        if v["off"] is None:
            continue
        name, q, lens, flags, seq = cs[v["case"]]
        comp = blob[v["off"]:v["off"] + v["len"]]
        out, got_lens = lib.fqz_decompress(comp, lens.copy(), flags.copy(), seq)
        assert out == q, (name, v["strat"])
        assert got_lens == [int(x) for x in lens], (name, v["strat"])


def test_fqz_random_vs_oracle():
    ora = binding.oracle()
    rng = np.random.default_rng(77)
    for it in range(12):
        nrec = int(rng.integers(1, 400))
        lens = rng.integers(1, 300, nrec).astype(np.uint32)
        nsym = int(rng.choice([2, 4, 8, 20, 40]))
        alpha = np.sort(rng.choice(np.arange(2, 60), nsym, replace=False)).astype(np.uint8)
        q = alpha[rng.integers(0, nsym, int(lens.sum()))].tobytes()
        flags = (rng.integers(0, 2, nrec) * 128).astype(np.uint32)
        seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, int(lens.sum()))].tobytes() \
            if it % 3 == 0 else None
        strat = it % 5
        exp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        got = lib.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        assert got == exp, (it, strat, len(got), len(exp))
        back, _ = lib.fqz_decompress(got, lens.copy(), flags.copy(), seq)
        assert back == q, it


@pytest.mark.parametrize("kind,strat", [("novaseq", 3), ("novaseq", 4), ("ont", 0), ("ont", 3),
                                        ("hifi", 0), ("illumina", 1)])
def test_fqz_decoder_paths_roundtrip(kind, strat):
    """Blocks long enough that hot models halve many times (FL_MAX) and the
    decoder's fast run leaves for the reference arithmetic, the cache
    misses and the input refills mid-run; with sequence context (strats 3
    and 4) the run's context state must survive every such exit."""
    from fqzcomp5_amd import synth
    r = {"novaseq": lambda: synth.novaseq(12000, seed=9),
         "illumina": lambda: synth.illumina(12000, seed=9),
         "ont": lambda: synth.ont(160, seed=9),
         "hifi": lambda: synth.hifi(40, seed=9)}[kind]()
    q, lens, seq = r.qual.tobytes(), r.lens.astype(np.uint32), r.seq.tobytes()
    flags = np.asarray(r.flags if getattr(r, "flags", None) is not None
                       else np.zeros(len(lens)), np.uint32)
    got = lib.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
    back, _ = lib.fqz_decompress(got, lens.copy(), flags.copy(), seq)
    assert back == q


def test_fqz_large_roundtrip(golden):
    cs, vec, _ = golden
    name, q, lens, flags, seq = cs["bin8_big"]
    want = {v["strat"]: v for v in vec if v["case"] == "bin8_big"}
    for st in (0, 2):
        out = lib.fqz_compress(q, lens.copy(), flags.copy(), st, seq)
        assert hashlib.md5(out).hexdigest() == want[st]["md5"]
        back, _ = lib.fqz_decompress(out, lens.copy(), flags.copy(), seq)
        assert back == q


def test_fqz_div_selftest():
    assert lib.fqz_div_selftest() == 0


def test_fqz_truncated_vs_oracle(golden):
    """Damaged streams: the decoder follows the reference's arithmetic past
    the end of the input and on out-of-range targets."""
    ora = binding.oracle()
    cs, _, _ = golden
    name, q, lens, flags, seq = cs["q40_var"]
    rng = np.random.default_rng(5)
    for strat in (0, 1, 3):
        comp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        for cut in (1, 3, 9, 40):
            bad = comp[:-cut]
            try:
                exp = ora.fqz_decompress(bad, lens.copy(), flags.copy(), seq)
            except RuntimeError:
                exp = None
            try:
                got, _ = lib.fqz_decompress(bad, lens.copy(), flags.copy(), seq)
            except RuntimeError:
                got = None
            assert got == exp, (strat, cut)
        # flipped bytes in the coder payload
        for _ in range(3):
            b = bytearray(comp)
            at = int(rng.integers(len(b) // 2, len(b)))
            b[at] ^= 0x5A
            try:
                exp = ora.fqz_decompress(bytes(b), lens.copy(), flags.copy(), seq)
            except RuntimeError:
                exp = None
            try:
                got, _ = lib.fqz_decompress(bytes(b), lens.copy(), flags.copy(), seq)
            except RuntimeError:
                got = None
            assert got == exp, (strat, at)


@pytest.mark.parametrize("hot_min", [1, 0])
def test_fqz_model_pass_paths(golden, hot_min):
    """The encoder's model pass has two forms (fqz5_set_hot_min): one wave per
    quality model with the list in lanes (runs of head hits coded in closed
    form) and one lane per model.  hot_min=1 sends every eligible model
    through the first, 0 none: both give the reference's bytes, including a
    skewed block whose hottest models halve their lists many times."""
    so = lib.load()
    prev = so.fqz5_set_hot_min(hot_min)
    try:
        cs, vec, _ = golden
        bad = []
        for v in vec:
            name, q, lens, flags, seq = cs[v["case"]]
            out = lib.fqz_compress(q, lens.copy(), flags.copy(), v["strat"], seq)
            if (len(out), hashlib.md5(out).hexdigest()) != (v["len"], v["md5"]):
                bad.append((v["case"], v["strat"]))
        assert not bad, bad
        ora = binding.oracle()
        rng = np.random.default_rng(5)
        nrec = 3000
        lens = np.full(nrec, 150, np.uint32)
        p = np.array([.90, .06, .03, .01])
        q = np.array([2, 12, 23, 37], np.uint8)[rng.choice(4, int(lens.sum()), p=p)].tobytes()
        for strat in (1, 3):
            exp = ora.fqz_compress(q, lens.copy(), np.zeros(nrec, np.uint32), strat)
            got = lib.fqz_compress(q, lens.copy(), np.zeros(nrec, np.uint32), strat)
            assert got == exp, strat
    finally:
        so.fqz5_set_hot_min(prev)
