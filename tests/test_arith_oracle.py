"""The arith_dynamic restatement (oracle/arith_oracle.c) against the
reference-generated vectors (tests/golden/arith.json, made by
tests/golden/make_golden_arith.py from oracle/_ref): every order of every
golden input byte-exact, NULL where the reference returns NULL, the
capacity semantics of caller buffers, and round trips."""
import hashlib
import json
import os

import pytest

from oracle import binding

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    g = os.path.join(HERE, "golden")
    man = json.load(open(os.path.join(g, "rans.json")))
    blob = open(os.path.join(g, "rans_inputs.bin"), "rb").read()
    ins = {k: blob[o:o + n] for k, (o, n, _) in man["inputs"].items()}
    arith = json.load(open(os.path.join(g, "arith.json")))
    outs = open(os.path.join(g, "arith_outputs.bin"), "rb").read()
    return ins, arith, outs


def test_arith_oracle_golden(golden):
    ins, arith, outs = golden
    ora = binding.oracle()
    bad = []
    for c in arith["cases"]:
        data = ins[c["input"]]
        got = ora.arith_compress(data, c["order"])
        if c.get("null"):
            if got is not None:
                bad.append((c["input"], c["order"], "not NULL"))
            continue
        if got is None or len(got) != c["len"] or hashlib.md5(got).hexdigest() != c["md5"]:
            bad.append((c["input"], c["order"]))
            continue
        if "off" in c:
            assert got == outs[c["off"]:c["off"] + c["len"]]
        nosz = c["order"] & 0x10 and not c["order"] & 0x08
        back = ora.arith_uncompress(got, len(data) if nosz else None)
        if back != data:
            bad.append((c["input"], c["order"], "roundtrip"))
    assert not bad, bad[:10]


def test_arith_oracle_capacity(golden):
    ins, arith, _ = golden
    ora = binding.oracle()
    for c in arith["caps"]:
        got = ora.arith_compress(ins[c["input"]], c["order"], cap=c["cap"])
        assert (got is None) == c["null"], c
        if got is not None:
            assert hashlib.md5(got).hexdigest() == c["md5"], c


def test_arith_oracle_truncated():
    """Decoding past the end of the input is an error (RC_FinishDecode)."""
    ora = binding.oracle()
    data = bytes((i * 7) % 13 + 40 for i in range(5000))
    for od in (0, 1, 64, 65):
        comp = ora.arith_compress(data, od)
        assert ora.arith_uncompress(comp[:-3]) is None
