"""The sequence context model on the GPU (fqz5_seq_encode / fqz5_seq_decode,
the drop-ins of fqzcomp5.c's encode_seq / decode_seq) against the reference's
golden vectors (tests/golden/make_golden_seq.py) and the oracle
(oracle/seq_oracle.c) on seeded inputs."""
import hashlib
import json
import os

import numpy as np
import pytest

from fqzcomp5_amd import lib
from oracle import binding
from seq_cases import METHODS, cases

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _golden():
    g = json.load(open(os.path.join(GOLD, "seq.json")))
    return {(r["case"], r["method"]): r for r in g}, open(os.path.join(GOLD, "seq_small.bin"), "rb").read()


@pytest.mark.parametrize("meth,k,both", METHODS)
def test_seq_encode_golden(meth, k, both):
    gold, _ = _golden()
    for name, seq, lens in cases():
        r = gold[(name, meth)]
        c = lib.seq_encode(seq, lens, both, k)
        assert (len(c), hashlib.md5(c).hexdigest()) == (r["len"], r["md5"]), name


@pytest.mark.parametrize("meth,k,both", METHODS[:3])
def test_seq_decode_golden(meth, k, both):
    gold, blob = _golden()
    for name, seq, lens in cases():
        r = gold[(name, meth)]
        if r["off"] is None or len(seq) > 200_000:
            continue
        c = blob[r["off"]:r["off"] + r["len"]]
        assert lib.seq_decode(c, lens, both, k, len(seq)) == seq, name


def test_seq_random_vs_oracle():
    o = binding.seq_oracle()
    rng = np.random.default_rng(9)
    alpha = np.frombuffer(b"ACGTACGTACGTACGTacgtNNRY", np.uint8)
    for t in range(8):
        nrec = int(rng.integers(1, 80))
        lens = [int(x) for x in rng.integers(0, 400, nrec)]
        seq = rng.choice(alpha, sum(lens)).tobytes()
        meth, k, both = METHODS[t % len(METHODS)]
        c = o.encode(seq, lens, both, k)
        assert lib.seq_encode(seq, lens, both, k) == c, (t, meth)
        assert lib.seq_decode(c, lens, both, k, len(seq)) == seq, (t, meth)


def test_seq_k14_and_large():
    # SEQ14B (1 GiB of context counts) and a 2 MB Illumina-like block with
    # repeated reads: encode against the oracle, decode round trip
    o = binding.seq_oracle()
    rng = np.random.default_rng(3)
    g = rng.choice(np.frombuffer(b"ACGT", np.uint8), 300_000)
    st = rng.integers(0, len(g) - 150, 14_000)
    seq = b"".join(g[s:s + 150].tobytes() for s in st)
    lens = [150] * len(st)
    for k, both in ((14, 1), (12, 1)):
        c = o.encode(seq, lens, both, k)
        assert lib.seq_encode(seq, lens, both, k) == c, k
    assert lib.seq_decode(c, lens, 1, 12, len(seq)) == seq


def test_seq_errors():
    with pytest.raises(lib.NativeError):
        lib.seq_encode(b"ACGT" * 10, [8, 8], 0, 10)   # records run out (NULL)
    with pytest.raises(lib.NativeError):
        lib.seq_encode(b"ACGT", [4], 0, 15)             # context size out of range
    with pytest.raises(lib.NativeError):
        lib.seq_decode(b"\x00\x01", [4], 0, 10, 4)   # damaged stream
