"""GPU parity: the HIP rANS path through the C-ABI against the reference's
golden vectors and the oracle (bit-exact), plus round trips."""
import hashlib

import numpy as np
import pytest

from fqzcomp5_amd import lib
from oracle import binding

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


def test_golden_compress(golden_rans):
    inputs, cases = golden_rans
    bad = []
    for name, order, ln, md5, exp in cases:
        out = lib.rans_compress(inputs[name], order)
        if hashlib.md5(out).hexdigest() != md5:
            bad.append((name, hex(order), len(out), ln))
    assert not bad, f"{len(bad)} mismatches: {bad[:25]}"


def test_golden_decompress(golden_rans):
    inputs, cases = golden_rans
    bad = []
    for name, order, ln, md5, exp in cases:
        if exp is None:
            continue
        try:
            back = lib.rans_uncompress(exp)
        except lib.NativeError as e:
            bad.append((name, hex(order), str(e)[:80]))
            continue
        if back != inputs[name]:
            bad.append((name, hex(order), "mismatch"))
    assert not bad, f"{len(bad)} failures: {bad[:25]}"


def _rand_case(rng, it):
    n = int(rng.choice([rng.integers(0, 64), rng.integers(0, 4000),
                        rng.integers(0, 300000)]))
    k = it % 5
    if k == 0:
        d = rng.integers(0, 256, n, dtype=np.uint8)
    elif k == 1:
        d = (rng.integers(0, 1 + it % 17, n) + 30).astype(np.uint8)
    elif k == 2:
        d = np.repeat(rng.integers(0, 4, n), rng.integers(1, 25, n))[:n]
    elif k == 3:
        d = np.minimum(rng.zipf(1.4, n), 255)
    else:
        d = rng.choice(np.array([2, 12, 23, 37]), n, p=[.01, .04, .1, .85])
    o = int(rng.choice([0, 1, 4, 5, 64, 65, 68, 69, 128, 129, 132, 133,
                        192, 193, 196, 197]))
    if it % 6 == 0:
        o = (int(rng.integers(1, 300)) << 8) | int(rng.choice([8, 9, 13]))
    return d.astype(np.uint8).tobytes(), o


def _or_none(f, *a):
    try:
        return f(*a)
    except (RuntimeError, lib.NativeError):
        return None


def test_random_vs_oracle():
    ora = binding.oracle()
    rng = np.random.default_rng(2024)
    bad = []
    for it in range(150):
        d, o = _rand_case(rng, it)
        exp = _or_none(ora.rans_compress, d, o)
        got = _or_none(lib.rans_compress, d, o)
        if got != exp:
            bad.append((len(d), hex(o), got and len(got), exp and len(exp)))
            continue
        if got is not None and lib.rans_uncompress(got) != d:
            bad.append((len(d), hex(o), "roundtrip"))
    assert not bad, bad[:20]


def test_capacity_semantics_vs_oracle():
    """rans_compress_to_4x16 with tight caller buffers fails exactly when
    the reference does."""
    ora = binding.oracle()
    rng = np.random.default_rng(7)
    import ctypes as C
    olib = ora.lib
    olib.ora_rans_compress_to_4x16.restype = C.c_void_p
    olib.ora_rans_compress_to_4x16.argtypes = [C.c_char_p, C.c_uint, C.c_void_p,
                                               C.POINTER(C.c_uint), C.c_int]
    for it in range(60):
        d, o = _rand_case(rng, it)
        if len(d) > 20000:
            d = d[:20000]
        full = _or_none(ora.rans_compress, d, o)
        if full is None:
            continue
        for cap in (len(full), len(full) - 1, len(full) + 3, 1,
                    lib.compress_bound(len(d), o) // 2):
            if cap <= 0:
                continue
            buf = C.create_string_buffer(cap)
            n = C.c_uint(cap)
            p = olib.ora_rans_compress_to_4x16(d, len(d), buf, C.byref(n), o)
            exp = buf.raw[:n.value] if p else None
            got = lib.rans_compress_to(d, o, cap)
            assert got == exp, (len(d), hex(o), cap)


def test_o1_big_alphabet_counter_spills():
    """O1 pair counts of a >= 128-symbol alphabet (k_hist1<true>: 16-bit LDS
    counters that spill at 0x8000, 4 MB slices): one pair repeated ~3M times
    (many spills of one bin), a second hot pair, and a 9 MB input (three
    slices), against the oracle's bytes, O1 alone and after PACK/RLE."""
    ora = binding.oracle()
    rng = np.random.default_rng(11)
    n = 9_000_000
    d = rng.integers(0, 200, n, dtype=np.uint8)
    d[1_000_000:4_000_000] = 7                      # pair (7, 7): ~3M counts
    d[5_000_000:7_000_000:2] = 9                    # pairs (9, x) / (x, 9)
    d[5_000_001:7_000_000:2] = 250
    data = d.tobytes()
    for o in (1, 5, 65):
        exp = ora.rans_compress(data, o)
        got = lib.rans_compress(data, o)
        assert got == exp, hex(o)
        assert lib.rans_uncompress(got) == data, hex(o)
    # packed bytes: 16 symbols, 2 per byte -> up to 256 packed values
    q = (rng.integers(0, 16, n, dtype=np.uint8) + 33)
    q[2_000_000:6_000_000] = 40
    qd = q.tobytes()
    for o in (129, 193):
        exp = ora.rans_compress(qd, o)
        got = lib.rans_compress(qd, o)
        assert got == exp, hex(o)
        assert lib.rans_uncompress(got) == qd, hex(o)


def test_large_q40_roundtrip():
    from fqzcomp5_amd import synth
    r = synth.illumina(20000, seed=3, binned=False)
    q = r.qual.tobytes()
    ora = binding.oracle()
    for o in (0, 1, 129, 193, (150 << 8) | 9):
        got = lib.rans_compress(q, o)
        assert got == ora.rans_compress(q, o), hex(o)
        assert lib.rans_uncompress(got) == q


def test_hedged_launches_same_bytes():
    """fqz5_set_hedge: the decode launch (and the fqz range chain) runs each
    chain on several CUs and keeps the first copy to finish.  Off and on
    give the same bytes, for several streams of several orders at once and
    for a stream too short to reach a group boundary."""
    import torch
    from fqzcomp5_amd import synth
    so = lib.load()
    r = synth.illumina(20000, seed=9)
    datas = [r.qual.tobytes(), r.seq.tobytes(), r.qual.tobytes()[:777]]
    orders = [0, 1, 129, 193]
    comps = [(d, lib.rans_compress(d, o)) for d in datas for o in orders]
    prev = so.fqz5_set_hedge(1)
    try:
        outs = {}
        for hedge in (0, 1):
            so.fqz5_set_hedge(hedge)
            cin = [torch.frombuffer(bytearray(c), dtype=torch.uint8).cuda() for _, c in comps]
            cout = [torch.zeros(len(d), dtype=torch.uint8, device="cuda") for d, _ in comps]
            jobs = [lib.RansJob(a.data_ptr(), b.data_ptr(), a.numel(), b.numel(), 0, 0, 0, 0)
                    for a, b in zip(cin, cout)]
            lib.uncompress_batch_dev(jobs)
            assert all(j.status == 0 for j in jobs)
            outs[hedge] = [bytes(b.cpu().numpy()) for b in cout]
        assert outs[0] == outs[1]
        assert outs[1] == [d for d, _ in comps]
        q = r.qual.tobytes()
        lens = r.lens.astype(np.uint32)
        fq = {}
        for hedge in (0, 1):
            so.fqz5_set_hedge(hedge)
            fq[hedge] = lib.fqz_compress(q, lens.copy(), np.zeros(len(lens), np.uint32), 1)
        assert fq[0] == fq[1]
    finally:
        so.fqz5_set_hedge(prev)


def test_o1_register_decoder_alphabets():
    """Small O1 alphabets (the O1 register decoder's domain, rans_chain.hip
    dec4_o1reg_body: <= 8 contexts at 12-bit slots, <= 16 at 10, <= 64
    (context, symbol) pairs; it runs when $FQZ5_O1REG=1 was set when the
    library loaded, else the table decoders do) against the oracle's
    streams: alphabets of 1-16 symbols, skewed and flat, lengths with every
    tail n % 4 and inputs short enough for 10-bit slots, with RLE / PACK in
    front."""
    from fqzcomp5_amd import synth
    ora = binding.oracle()
    rng = np.random.default_rng(77)
    q = synth.novaseq(30000, seed=4).qual
    cases = [q.tobytes(), q[:100003].tobytes(), q[:4097].tobytes()]
    for nsym in (1, 2, 3, 4, 5, 7, 8, 11, 16):
        alpha = rng.choice(np.arange(1, 90), nsym, replace=False)
        p = rng.dirichlet(np.full(nsym, 0.4))
        for n in (5, 63, 1001, 65538, 400001):
            cases.append(rng.choice(alpha, n, p=p).astype(np.uint8).tobytes())
    bad = []
    for d in cases:
        for o in (1, 65, 129, 193):
            c = ora.rans_compress(d, o)
            got = _or_none(lib.rans_uncompress, c)
            if got != d:
                bad.append((len(d), hex(o), len(set(d))))
    assert not bad, bad[:20]
