"""The LZP restatement (oracle/lzp_oracle.c) against the reference's own lzp
/ unlzp (lzp16e.c) and the LZP3 method (fqzcomp5.c:2013-2021): the committed
golden vectors (made from oracle/_ref), and live against oracle/_ref when it
is built.  CPU only."""
import hashlib
import json
import os
import random

import pytest

from lzp_cases import cases
from oracle import binding

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "lzp.json")))
SMALL = open(os.path.join(HERE, "golden", "lzp_small.bin"), "rb").read()


def test_oracle_vs_golden():
    ora = binding.oracle()
    got = dict(cases())
    for g in GOLD:
        data = got[g["case"]]
        z = ora.lzp(data)
        assert (len(z), hashlib.md5(z).hexdigest()) == (g["lzp_len"], g["lzp_md5"]), g["case"]
        c = ora.lzp3_compress(data)
        assert (len(c), hashlib.md5(c).hexdigest()) == (g["lzp3_len"], g["lzp3_md5"]), g["case"]
        assert ora.unlzp(z, len(data)) == data
        if g["off"] is not None:
            stream = SMALL[g["off"]:g["off"] + g["lzp3_len"]]
            assert ora.lzp3_uncompress(stream, len(data)) == data


@pytest.mark.skipif(not binding.have_ref(), reason="oracle/_ref not built")
def test_oracle_vs_reference_random():
    ora, ref = binding.oracle(), binding.ref()
    rng = random.Random(7)
    for it in range(60):
        n = rng.choice([0, 1, 3, 4, 10, 100, 1000, 5000])
        alpha = rng.choice([b"AC", b"ACGT", b"ACGTN", bytes([233, 234, 0]), bytes(range(256))])
        rep = rng.random() < 0.5
        if rep and n:
            unit = bytes(rng.choice(alpha) for _ in range(rng.randint(1, 40)))
            data = (unit * (n // len(unit) + 1))[:n]
        else:
            data = bytes(rng.choice(alpha) for _ in range(n))
        assert ora.lzp(data) == ref.lzp(data), it
        assert ora.unlzp(ref.lzp(data), n) == data


def test_unlzp_bounds():
    """Damaged streams: the restatement stops at its capacity or at a token
    cut short instead of writing past the buffer."""
    ora = binding.oracle()
    data = b"ACGTACGTACGTACGTACGT" * 10
    z = ora.lzp(data)
    assert ora.unlzp(z, len(data)) == data
    with pytest.raises(RuntimeError):
        ora.unlzp(z, len(data) - 1)
    last = max(z.rfind(bytes([233])), z.rfind(bytes([234])))
    cut = z[:last + 1]                            # ends on a marker
    with pytest.raises(RuntimeError):
        ora.unlzp(cut, len(data))
