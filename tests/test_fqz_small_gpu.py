"""GPU parity of the small-alphabet fqz decoder (fqz_decode_small.hip):
24-byte models of at most 9 live symbols in a 4-way set-associative LDS
cache.

Every case decodes through the C-ABI (fqz_decompress) with the small decoder
on, with its cache cut to a few 4-way sets (FQZ5_DEC_SETS: nearly every symbol
misses, so the write-back / fetch path and its HBM backing store carry the
decode), and off (the general decoder); all must give the reference's
bytes.  fqz5_fqz_dec_counts shows which decoder ran."""
import ctypes as C
import json
import os

import numpy as np
import pytest

from fqz_cases import cases
from fqzcomp5_amd import lib, synth
from oracle import binding

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


def _counts():
    so = lib.load()
    out = (C.c_uint64 * 2)()
    so.fqz5_fqz_dec_counts(out)
    return int(out[0]), int(out[1])


MODES = ["small", "small_sets16", "small_sets1", "general"]


@pytest.fixture(params=MODES)
def mode(request):
    so = lib.load()
    prev = so.fqz5_set_dec_small(0 if request.param == "general" else 1)
    old = os.environ.pop("FQZ5_DEC_SETS", None)
    if request.param.startswith("small_sets"):
        os.environ["FQZ5_DEC_SETS"] = request.param[len("small_sets"):]
    try:
        yield request.param
    finally:
        so.fqz5_set_dec_small(prev)
        os.environ.pop("FQZ5_DEC_SETS", None)
        if old is not None:
            os.environ["FQZ5_DEC_SETS"] = old


def _decode(comp, lens, flags, seq, mode):
    g0, s0 = _counts()
    out, got_lens = lib.fqz_decompress(comp, lens.copy(), flags.copy(), seq)
    g1, s1 = _counts()
    return out, got_lens, (g1 - g0, s1 - s0)


def _small_eligible(q: bytes) -> bool:
    return len(set(q)) <= 8


def test_small_golden_decompress(mode):
    cs = {c[0]: c for c in cases()}
    vec = json.load(open(os.path.join(HERE, "golden", "fqz.json")))
    blob = open(os.path.join(HERE, "golden", "fqz_small.bin"), "rb").read()
    used_small = 0
    for v in vec:
        if v["off"] is None:
            continue
        name, q, lens, flags, seq = cs[v["case"]]
        comp = blob[v["off"]:v["off"] + v["len"]]
        out, got_lens, (ng, ns) = _decode(comp, lens, flags, seq, mode)
        assert out == q, (name, v["strat"], mode)
        assert got_lens == [int(x) for x in lens], (name, v["strat"])
        used_small += ns
        if mode == "general":
            assert ns == 0
    if mode != "general":
        assert used_small > 0, "no golden stream took the small decoder"


@pytest.mark.parametrize("kind", ["illumina", "novaseq"])
@pytest.mark.parametrize("strat", [0, 1, 2])
def test_small_synth_vs_oracle(mode, kind, strat):
    """Illumina 8-level and NovaSeq blocks (the configs[1] / configs[2]
    shapes) at every non-sequence strategy: encoded by the reference
    restatement, decoded on the GPU; long enough that hot models halve and
    bubble and the position contexts cycle through the cache."""
    r = synth.illumina(9000, seed=21) if kind == "illumina" else synth.novaseq(9000, seed=21)
    q, lens = r.qual.tobytes(), r.lens.astype(np.uint32)
    flags = np.zeros(len(lens), np.uint32)
    flags[1::2] = 128
    comp = binding.oracle().fqz_compress(q, lens.copy(), flags.copy(), strat)
    out, got_lens, (ng, ns) = _decode(comp, lens, flags, None, mode)
    assert out == q
    assert got_lens == [int(x) for x in lens]
    if mode == "general":
        assert (ng, ns) == (1, 0)
    else:
        assert (ng, ns) == (0, 1)


def test_small_random_vs_oracle(mode):
    """Random small alphabets (2..8 symbols, so 3..9 live with qmap), ragged
    records, READ2 flags, sequence bases given (strategies 3 and 4 keep the
    general decoder)."""
    ora = binding.oracle()
    rng = np.random.default_rng(1234)
    for it in range(10):
        nrec = int(rng.integers(1, 500))
        lens = rng.integers(1, 400, nrec).astype(np.uint32)
        nsym = int(rng.choice([2, 3, 4, 5, 7, 8]))
        alpha = np.sort(rng.choice(np.arange(2, 45), nsym, replace=False)).astype(np.uint8)
        p = rng.dirichlet(np.ones(nsym) * 0.5)
        q = alpha[rng.choice(nsym, int(lens.sum()), p=p)].tobytes()
        flags = (rng.integers(0, 2, nrec) * 128).astype(np.uint32)
        strat = it % 5
        seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, int(lens.sum()))].tobytes()
        comp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        out, _, _ = _decode(comp, lens, flags, seq, mode)
        assert out == q, (it, strat, nsym)


def test_small_truncated_vs_oracle(mode):
    """Damaged streams follow the reference's arithmetic (the slow path at
    the input's end, t >= total, symbol 0 without an update)."""
    ora = binding.oracle()
    r = synth.illumina(600, seed=4)
    q, lens = r.qual.tobytes(), r.lens.astype(np.uint32)
    flags = np.zeros(len(lens), np.uint32)
    rng = np.random.default_rng(9)
    for strat in (0, 1, 2):
        comp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat)
        bads = [comp[:-cut] for cut in (1, 3, 9, 40)]
        for _ in range(3):
            b = bytearray(comp)
            b[int(rng.integers(len(b) // 2, len(b)))] ^= 0x5A
            bads.append(bytes(b))
        for bad in bads:
            try:
                exp = ora.fqz_decompress(bad, lens.copy(), flags.copy())
            except RuntimeError:
                exp = None
            try:
                got, _, _ = _decode(bad, lens, flags, None, mode)
            except RuntimeError:
                got = None
            assert got == exp, (strat, len(bad))
