"""CPU tests: the oracle restatement against the reference's golden vectors
(and against the compiled reference itself when oracle/_ref is present)."""
import hashlib

import numpy as np
import pytest

from oracle import binding


def test_golden_inputs_intact(golden_rans):
    import json, os
    from conftest import ROOT
    man = json.load(open(os.path.join(ROOT, "tests/golden/rans.json")))
    inputs, _ = golden_rans
    for k, (_, n, m) in man["inputs"].items():
        assert hashlib.md5(inputs[k]).hexdigest() == m


def test_oracle_matches_golden(golden_rans):
    ora = binding.oracle()
    inputs, cases = golden_rans
    bad = []
    for name, order, ln, md5, exp in cases:
        data = inputs[name]
        out = ora.rans_compress(data, order)
        if hashlib.md5(out).hexdigest() != md5:
            bad.append((name, order))
            continue
        if ora.rans_uncompress(out) != data:
            bad.append((name, order, "dec"))
    assert not bad, bad[:20]


def test_oracle_decodes_golden(golden_rans):
    ora = binding.oracle()
    inputs, cases = golden_rans
    for name, order, ln, md5, exp in cases:
        if exp is not None:
            assert ora.rans_uncompress(exp) == inputs[name], (name, order)


@pytest.mark.skipif(not binding.have_ref(), reason="oracle/_ref not built")
def test_oracle_vs_reference_fuzz():
    ora, ref = binding.oracle(), binding.ref()
    rng = np.random.default_rng(99)
    for it in range(400):
        n = int(rng.choice([rng.integers(0, 64), rng.integers(0, 5000)]))
        k = it % 4
        if k == 0:
            d = rng.integers(0, 256, n, dtype=np.uint8)
        elif k == 1:
            d = (rng.integers(0, 1 + it % 17, n) + 30).astype(np.uint8)
        elif k == 2:
            d = np.repeat(rng.integers(0, 4, n), rng.integers(1, 25, n))[:n]
        else:
            d = np.minimum(rng.zipf(1.4, n), 255)
        d = d.astype(np.uint8).tobytes()
        o = int(rng.choice([0, 1, 4, 5, 64, 65, 128, 129, 192, 193, 197]))
        if it % 5 == 0:
            o = (int(rng.integers(1, 260)) << 8) | 9
        try:
            a = ref.rans_compress(d, o)
        except RuntimeError:
            a = None
        try:
            b = ora.rans_compress(d, o)
        except RuntimeError:
            b = None
        assert a == b, (n, k, hex(o))


@pytest.mark.skipif(not binding.have_ref(), reason="oracle/_ref not built")
def test_oracle_capacity_semantics_vs_reference():
    """rans_compress_to_4x16 with tight caller buffers: the restatement
    fails (NULL) exactly when the reference does, else same bytes."""
    import ctypes as C
    ora, ref = binding.oracle(), binding.ref()
    fo = ora.lib.ora_rans_compress_to_4x16
    fr = ref.lib.rans_compress_to_4x16
    for f in (fo, fr):
        f.restype = C.c_void_p
        f.argtypes = [C.c_char_p, C.c_uint, C.c_void_p, C.POINTER(C.c_uint), C.c_int]
    rng = np.random.default_rng(5)
    for it in range(200):
        n = int(rng.integers(0, 3000))
        d = (rng.integers(0, 1 + it % 20, n) + it % 3).astype(np.uint8).tobytes()
        o = int(rng.choice([0, 1, 5, 65, 128, 129, 193, (12 << 8) | 9, (40 << 8) | 9]))
        try:
            full = len(ref.rans_compress(d, o))
        except RuntimeError:
            continue
        for cap in (full, full - 1, full + 2, 1, 6, full // 2):
            if cap <= 0:
                continue
            res = []
            for f in (fo, fr):
                buf = C.create_string_buffer(cap + 4096)
                k = C.c_uint(cap)
                p = f(d, len(d), buf, C.byref(k), o)
                res.append(buf.raw[:k.value] if p else None)
            assert res[0] == res[1], (n, hex(o), cap)
