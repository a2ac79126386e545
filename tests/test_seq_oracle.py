"""The sequence context model oracle (oracle/seq_oracle.c) against the
reference's own encode_seq / decode_seq: the committed golden vectors
(tests/golden/make_golden_seq.py) always, and the compiled reference
(oracle/_ref/libfqz5ref.so) on further seeded inputs when it is present."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import binding
from seq_cases import METHODS, cases

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _golden():
    g = json.load(open(os.path.join(GOLD, "seq.json")))
    return {(r["case"], r["method"]): r for r in g}, open(os.path.join(GOLD, "seq_small.bin"), "rb").read()


@pytest.mark.parametrize("meth,k,both", METHODS)
def test_seq_oracle_golden(meth, k, both):
    gold, blob = _golden()
    o = binding.seq_oracle()
    for name, seq, lens in cases():
        r = gold[(name, meth)]
        c = o.encode(seq, lens, both, k)
        assert (len(c), hashlib.md5(c).hexdigest()) == (r["len"], r["md5"]), name
        if r["off"] is not None:
            ref_bytes = blob[r["off"]:r["off"] + r["len"]]
            assert o.decode(ref_bytes, lens, both, k, len(seq)) == seq, name


def test_seq_oracle_bad_records():
    # more symbols than the records cover: the reference returns NULL
    o = binding.seq_oracle()
    with pytest.raises(RuntimeError):
        o.encode(b"ACGT" * 10, [8, 8], 0, 10)


@pytest.mark.skipif(not binding.have_seq_ref(), reason="oracle/_ref not built")
def test_seq_oracle_vs_reference_random():
    o, ref = binding.seq_oracle(), binding.seq_ref()
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(b"ACGTACGTACGTACGTacgtNNRY", np.uint8)
    for t in range(12):
        nrec = int(rng.integers(1, 60))
        lens = [int(x) for x in rng.integers(0, 300, nrec)]
        seq = rng.choice(alpha, sum(lens)).tobytes()
        meth, k, both = METHODS[t % len(METHODS)]
        c = ref.encode(seq, lens, both, k)
        assert o.encode(seq, lens, both, k) == c, (t, meth)
        assert o.decode(c, lens, both, k, len(seq)) == seq


@pytest.mark.skipif(not binding.have_seq_ref(), reason="oracle/_ref not built")
def test_seq_oracle_vs_reference_k14():
    o, ref = binding.seq_oracle(), binding.seq_ref()
    name, seq, lens = cases()[0]
    c = ref.encode(seq, lens, 1, 14)
    assert o.encode(seq, lens, 1, 14) == c
