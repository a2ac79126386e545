"""The tok3 read-name tokeniser behind the product C-ABI (tok3.cpp:
tok3_encode_names / tok3_decode_names, token streams coded as one GPU
batch) against the reference's tokenise_name3.c: byte-identical streams on
the golden vectors (tests/golden/make_golden_tok3.py) and on seeded random
blocks (reference run live from oracle/_ref when present), decodes of the
reference's streams, and the reference's refusals."""
import hashlib
import json
import os
import random

import pytest

from fqzcomp5_amd import lib
from oracle import binding
from tok3_cases import bad_cases, cases, _illumina, _srr, _mixed, block

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "tok3.json")))
BLOB = open(os.path.join(HERE, "golden", "tok3_small.bin"), "rb").read()


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


def _streams(z):
    """(ttype byte, descriptor bytes) per descriptor of a tok3 stream, for
    naming the first descriptor that differs."""
    out, o = [], 9
    while o < len(z):
        t = z[o]
        o += 1
        if t & 64:
            out.append((t, z[o:o + 2]))
            o += 2
            continue
        v, s, nb = 0, 0, 0
        while True:
            c = z[o + nb]
            v |= (c & 127) << s
            s += 7
            nb += 1
            if not c & 128:
                break
        out.append((t, z[o:o + nb + v]))
        o += nb + v
    return out


def _first_diff(a, b):
    sa, sb = _streams(a), _streams(b)
    for i, (x, y) in enumerate(zip(sa, sb)):
        if x != y:
            return i, x[0], y[0], len(x[1]), len(y[1])
    return len(sa), len(sb)


def test_encode_golden():
    data = dict(cases())
    for g in GOLD:
        r = lib.tok3_encode(data[g["case"]], g["level"], g["arith"])
        assert r is not None, (g, lib.last_error())
        z, ls = r
        if g["off"] is not None and hashlib.md5(z).hexdigest() != g["md5"]:
            ref = BLOB[g["off"]:g["off"] + g["len"]]
            pytest.fail(f"{g['case']} level {g['level']} arith {g['arith']}: "
                        f"first differing descriptor {_first_diff(z, ref)}")
        assert (len(z), hashlib.md5(z).hexdigest(), ls) == (g["len"], g["md5"], g["last_start"]), g


def test_decode_golden():
    data = dict(cases())
    for g in GOLD:
        if g["off"] is None:
            continue
        z = BLOB[g["off"]:g["off"] + g["len"]]
        exp = data[g["case"]][:g["last_start"]].replace(b"\n", b"\0")
        assert lib.tok3_decode(z) == exp, g


def test_large_block_roundtrip():
    data = dict(cases())["illumina_20k"]
    for g in GOLD:
        if g["case"] != "illumina_20k":
            continue
        z, ls = lib.tok3_encode(data, g["level"], g["arith"])
        assert lib.tok3_decode(z) == data[:ls].replace(b"\n", b"\0")


def test_refusals():
    for name, data in bad_cases():
        assert lib.tok3_encode(data, 5, 0) is None, name
    assert lib.tok3_decode(b"\0" * 8) is None
    assert lib.tok3_decode(b"") is None


def test_truncated_stream_fails_cleanly():
    data = dict(cases())["illumina_1k"]
    z, _ = lib.tok3_encode(data, 5, 0)
    for cut in (9, 10, 20, len(z) // 2, len(z) - 1):
        r = lib.tok3_decode(z[:cut])
        assert r is None or isinstance(r, bytes)


@pytest.mark.skipif(not binding.have_ref(), reason="oracle/_ref not built")
def test_random_blocks_vs_reference():
    ref = binding.ref()
    rng = random.Random(4242)
    for it in range(24):
        kind = rng.choice([_illumina, _srr, _mixed])
        names = kind(rng, rng.choice([1, 2, 3, 17, 256, 1000, 4000]))
        data = block(names, sep=rng.choice(["\n", "\0"]), tail=rng.random() < 0.9)
        lv = rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9])
        exp = ref.tok3_encode(data, lv, 0)
        got = lib.tok3_encode(data, lv, 0)
        if exp is None:
            assert got is None, it
            continue
        assert got is not None, (it, lib.last_error())
        assert got == exp, (it, lv, _first_diff(got[0], exp[0]))
        assert lib.tok3_decode(exp[0]) == ref.tok3_decode(exp[0]), it
