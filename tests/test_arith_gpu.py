"""arith_dynamic on the GPU (include/fqz5_mi355x.h: arith_compress_to &c.,
arith_kernels.hip + arith_codec.cpp) against the reference-generated
vectors (tests/golden/arith.json) and the oracle (oracle/arith_oracle.c):
byte-exact streams, NULL exactly where the reference returns NULL, the
capacity semantics of caller buffers, truncated input, and round trips."""
import hashlib
import json
import os
import random

import pytest

from oracle import binding

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def L():
    from fqzcomp5_amd import lib
    if not lib.device_ok():
        pytest.fail("no HIP device: " + lib.last_error())
    return lib


@pytest.fixture(scope="module")
def golden():
    g = os.path.join(HERE, "golden")
    man = json.load(open(os.path.join(g, "rans.json")))
    blob = open(os.path.join(g, "rans_inputs.bin"), "rb").read()
    ins = {k: blob[o:o + n] for k, (o, n, _) in man["inputs"].items()}
    return ins, json.load(open(os.path.join(g, "arith.json")))


def test_arith_gpu_golden(L, golden):
    ins, arith = golden
    bad = []
    for c in arith["cases"]:
        data = ins[c["input"]]
        got = L.arith_compress(data, c["order"])
        if c.get("null"):
            if got is not None:
                bad.append((c["input"], c["order"], "not NULL"))
            continue
        if got is None or len(got) != c["len"] or hashlib.md5(got).hexdigest() != c["md5"]:
            bad.append((c["input"], c["order"], None if got is None else len(got), c["len"]))
            continue
        nosz = c["order"] & 0x10 and not c["order"] & 0x08
        back = L.arith_uncompress(got, len(data) if nosz else None)
        if back != data:
            bad.append((c["input"], c["order"], "roundtrip"))
    assert not bad, (len(bad), bad[:10])


def test_arith_gpu_capacity(L, golden):
    ins, arith = golden
    for c in arith["caps"]:
        got = L.arith_compress(ins[c["input"]], c["order"], cap=c["cap"])
        assert (got is None) == c["null"], c
        if got is not None:
            assert hashlib.md5(got).hexdigest() == c["md5"], c


def _streams(rng):
    """Inputs the golden set is short of: long runs, wide alphabets (order-1
    models in HBM), quality-like values, sizes across the 4 KB ring/page."""
    yield bytes(rng.randrange(256) for _ in range(70000))
    yield bytes(rng.choice(b"ACGTN") for _ in range(30000))
    q, v = bytearray(), 30
    for _ in range(50000):
        v = min(70, max(2, v + rng.choice((-3, -1, 0, 0, 0, 1, 2))))
        q.append(v)
    yield bytes(q)
    r = bytearray()
    while len(r) < 40000:
        r += bytes([rng.randrange(8)]) * rng.choice((1, 2, 3, 4, 5, 9, 300))
    yield bytes(r)
    for n in (4095, 4096, 4097, 8193):
        yield bytes(rng.randrange(200) for _ in range(n))


@pytest.mark.parametrize("order", [0, 1, 0x40, 0x41, 0x80, 0x81, 0xC1, 0x08 | 0x100 * 4,
                                   0x09 | 0x100 * 3, 0x20])
def test_arith_gpu_vs_oracle(L, order):
    ora = binding.oracle()
    rng = random.Random(order)
    for data in _streams(rng):
        exp = ora.arith_compress(data, order)
        got = L.arith_compress(data, order)
        assert got == exp, (order, len(data))
        if exp is not None:      # CAT alone is NULL in the reference (:743-752)
            assert L.arith_uncompress(got) == data


def test_arith_gpu_truncated(L):
    data = bytes((i * 7) % 13 + 40 for i in range(5000))
    ora = binding.oracle()
    for od in (0, 1, 64, 65):
        comp = L.arith_compress(data, od)
        assert comp == ora.arith_compress(data, od)
        assert L.arith_uncompress(comp[:-3]) is None
        assert L.arith_uncompress(comp, len(data) - 1) is None


def test_arith_gpu_bad_streams(L):
    """Cut and corrupted streams give what the oracle gives (mostly NULL),
    without faulting."""
    ora = binding.oracle()
    data = bytes(range(200)) * 50
    rng = random.Random(5)
    for order in (0x08 | 0x100 * 4, 0x81, 0x41, 0x01):
        comp = ora.arith_compress(data, order)
        cases = [comp[:cut] for cut in (1, 2, 3, 5, 8, 13, len(comp) // 2)]
        for _ in range(6):
            b = bytearray(comp)
            b[rng.randrange(8, min(len(b), 40))] ^= 1 << rng.randrange(8)   # past the size
            cases.append(bytes(b))
        for c in cases:
            assert L.arith_uncompress(c) == ora.arith_uncompress(c), (order, len(c))
    assert L.arith_uncompress(b"") is None
