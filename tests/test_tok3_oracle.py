"""The tok3 golden vectors (tests/golden/make_golden_tok3.py) against the
reference tokeniser compiled from /root/reference (oracle/_ref): the stored
streams decode to the input names and re-encoding reproduces them.  CPU
only; skipped where oracle/_ref is not built."""
import hashlib
import json
import os

import pytest

from oracle import binding
from tok3_cases import cases, bad_cases

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "tok3.json")))
BLOB = open(os.path.join(HERE, "golden", "tok3_small.bin"), "rb").read()

need_ref = pytest.mark.skipif(not binding.have_ref(), reason="oracle/_ref not built")


def test_golden_table_covers_cases():
    names = {c for c, _ in cases()}
    assert {g["case"] for g in GOLD} == names
    assert all(g["off"] is None or g["off"] + g["len"] <= len(BLOB) for g in GOLD)


@need_ref
def test_ref_decodes_golden():
    ref = binding.ref()
    data = dict(cases())
    for g in GOLD:
        if g["off"] is None:
            continue
        z = BLOB[g["off"]:g["off"] + g["len"]]
        assert hashlib.md5(z).hexdigest() == g["md5"]
        exp = data[g["case"]][:g["last_start"]].replace(b"\n", b"\0")
        assert ref.tok3_decode(z) == exp, g


@need_ref
def test_ref_reencodes_golden():
    ref = binding.ref()
    data = dict(cases())
    for g in GOLD:
        if g["len"] > 50000:
            continue
        z, ls = ref.tok3_encode(data[g["case"]], g["level"], g["arith"])
        assert (len(z), hashlib.md5(z).hexdigest(), ls) == (g["len"], g["md5"], g["last_start"])


@need_ref
def test_ref_refuses_bad_blocks():
    ref = binding.ref()
    for name, data in bad_cases():
        assert ref.tok3_encode(data, 5, 0) is None, name
