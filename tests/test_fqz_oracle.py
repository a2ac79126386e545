"""The fqzcomp_qual restatement (oracle/fqz_oracle.c) against the golden
vectors generated from the compiled reference (tests/golden/fqz.json), and
its decoder on the reference's own streams."""
import hashlib
import json
import os

import pytest

from fqz_cases import cases
from oracle import binding

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    vec = json.load(open(os.path.join(HERE, "golden", "fqz.json")))
    blob = open(os.path.join(HERE, "golden", "fqz_small.bin"), "rb").read()
    return {c[0]: c for c in cases()}, vec, blob


def test_oracle_encodes_golden(golden):
    cs, vec, _ = golden
    ora = binding.oracle()
    bad = []
    for v in vec:
        name, q, lens, flags, seq = cs[v["case"]]
        fl = flags.copy()
        out = ora.fqz_compress(q, lens.copy(), fl, v["strat"], seq)
        if (len(out), hashlib.md5(out).hexdigest()) != (v["len"], v["md5"]):
            bad.append((v["case"], v["strat"], len(out), v["len"]))
        assert not fl.any() or (fl == flags).all()   # selector bits cleared
    assert not bad, bad


def test_oracle_decodes_golden(golden):
    cs, vec, blob = golden
    ora = binding.oracle()
    for v in vec:
        if v["off"] is None:
            continue
        name, q, lens, flags, seq = cs[v["case"]]
        comp = blob[v["off"]:v["off"] + v["len"]]
        assert ora.fqz_decompress(comp, lens, flags, seq) == q, (name, v["strat"])


def test_oracle_roundtrip_large(golden):
    cs, vec, _ = golden
    ora = binding.oracle()
    name, q, lens, flags, seq = cs["bin8_big"]
    for st in (0, 1, 2):
        c = ora.fqz_compress(q, lens.copy(), flags.copy(), st, seq)
        assert ora.fqz_decompress(c, lens, flags, seq) == q
