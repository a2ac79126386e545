"""The adaptive-model decode chains on a host core (host_dec.cpp behind
fqz5_fqz_decompress_host / fqz5_seq_decode_host): the block decoder's host
leg.  CPU tests: the library's own C++ decoders (not the oracle) against the
reference's golden vectors (tests/golden/fqz.json, seq.json), and streams the
oracle restatement encodes from seeded inputs, damaged ones included."""
import json
import os

import numpy as np
import pytest

from fqz_cases import cases as fqz_cases
from fqzcomp5_amd import lib, synth
from oracle import binding
from seq_cases import METHODS, cases as seq_cases

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_fqz_host_golden():
    cs = {c[0]: c for c in fqz_cases()}
    vec = json.load(open(os.path.join(GOLD, "fqz.json")))
    blob = open(os.path.join(GOLD, "fqz_small.bin"), "rb").read()
    n = 0
    for v in vec:
        if v["off"] is None:
            continue
        name, q, lens, flags, seq = cs[v["case"]]
        comp = blob[v["off"]:v["off"] + v["len"]]
        out, got_lens = lib.fqz_decompress(comp, lens.copy(), flags.copy(), seq, host=True)
        assert out == q, (name, v["strat"])
        assert got_lens == [int(x) for x in lens], (name, v["strat"])
        n += 1
    assert n > 10


@pytest.mark.parametrize("kind", ["illumina", "novaseq", "ont", "hifi"])
def test_fqz_host_synth_vs_oracle(kind):
    """Every strategy on each data shape (sequence contexts for 3 and 4, READ2
    flags for the paired HiFi reads), long enough for halvings and bubbles."""
    r = {"illumina": lambda: synth.illumina(3000, seed=2),
         "novaseq": lambda: synth.novaseq(3000, seed=2),
         "ont": lambda: synth.ont(40, seed=2),
         "hifi": lambda: synth.hifi(16, seed=2)}[kind]()
    q, lens, seq = r.qual.tobytes(), r.lens.astype(np.uint32), r.seq.tobytes()
    flags = np.asarray(r.flags if getattr(r, "flags", None) is not None
                       else np.zeros(len(lens)), np.uint32)
    ora = binding.oracle()
    for strat in range(5):
        comp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        out, got = lib.fqz_decompress(comp, lens.copy(), flags.copy(), seq, host=True)
        assert out == q, (kind, strat)
        assert got == [int(x) for x in lens]


def test_fqz_host_random_and_damaged():
    ora = binding.oracle()
    rng = np.random.default_rng(31)
    for it in range(12):
        nrec = int(rng.integers(1, 300))
        lens = rng.integers(1, 300, nrec).astype(np.uint32)
        nsym = int(rng.choice([2, 4, 8, 20, 40, 90]))
        alpha = np.sort(rng.choice(np.arange(2, 94), nsym, replace=False)).astype(np.uint8)
        q = alpha[rng.integers(0, nsym, int(lens.sum()))].tobytes()
        flags = (rng.integers(0, 2, nrec) * 128).astype(np.uint32)
        seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, int(lens.sum()))].tobytes() \
            if it % 2 else None
        strat = it % 5
        comp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        out, _ = lib.fqz_decompress(comp, lens.copy(), flags.copy(), seq, host=True)
        assert out == q, (it, strat, nsym)
        # damaged: truncated streams give the reference's result (or both
        # fail); a flipped payload byte must not bring the decoder down
        flipped = bytearray(comp)
        flipped[len(comp) * 3 // 4] ^= 0x33
        try:
            lib.fqz_decompress(bytes(flipped), lens.copy(), flags.copy(), seq, host=True)
        except RuntimeError:
            pass
        # (with sequences given, a damaged stream that decodes more records
        # than the slice has makes the reference read past s->seq: compare
        # those without sequences only)
        for bad in ((comp[:-3], comp[:-17]) if seq is None else ()):
            try:
                exp = ora.fqz_decompress(bad, lens.copy(), flags.copy(), seq)
            except RuntimeError:
                exp = None
            try:
                got, _ = lib.fqz_decompress(bad, lens.copy(), flags.copy(), seq, host=True)
            except RuntimeError:
                got = None
            assert got == exp, (it, strat, len(bad))


@pytest.mark.parametrize("meth,k,both", METHODS)
def test_seq_host_golden(meth, k, both):
    g = json.load(open(os.path.join(GOLD, "seq.json")))
    gold = {(r["case"], r["method"]): r for r in g}
    blob = open(os.path.join(GOLD, "seq_small.bin"), "rb").read()
    n = 0
    for name, seq, lens in seq_cases():
        r = gold[(name, meth)]
        if r["off"] is None:
            continue
        c = blob[r["off"]:r["off"] + r["len"]]
        assert lib.seq_decode(c, lens, both, k, len(seq), host=True) == seq, name
        n += 1
    assert n > 0


def test_seq_host_random_vs_oracle():
    o = binding.seq_oracle()
    rng = np.random.default_rng(19)
    alpha = np.frombuffer(b"ACGTACGTACGTACGTacgtNNRY", np.uint8)
    for t in range(10):
        nrec = int(rng.integers(1, 80))
        lens = [int(x) for x in rng.integers(0, 400, nrec)]
        seq = rng.choice(alpha, sum(lens)).tobytes()
        meth, k, both = METHODS[t % len(METHODS)]
        c = o.encode(seq, lens, both, k)
        assert lib.seq_decode(c, lens, both, k, len(seq), host=True) == seq, (t, meth)


def test_seq_host_damaged():
    """Cut and byte-flipped SEQ streams: the host decoder returns an error or
    some bytes, and never reads past its k-mer model table (host_dec.cpp's
    symbol search is bounded by the model total)."""
    o = binding.seq_oracle()
    rng = np.random.default_rng(23)
    alpha = np.frombuffer(b"ACGTACGTACGTacgtNN", np.uint8)
    for t in range(24):
        nrec = int(rng.integers(1, 60))
        lens = [int(x) for x in rng.integers(1, 300, nrec)]
        seq = rng.choice(alpha, sum(lens)).tobytes()
        meth, k, both = METHODS[t % len(METHODS)]
        c = o.encode(seq, lens, both, k)
        bad = bytearray(c)
        for j in rng.integers(4, len(c), 1 + t % 5):
            bad[int(j)] ^= int(rng.integers(1, 256))
        for stream in (bytes(bad), c[:len(c) // 2], c[:7]):
            try:
                lib.seq_decode(stream, lens, both, k, len(seq), host=True)
            except RuntimeError:
                pass
