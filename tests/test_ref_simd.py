"""The SIMD-dispatching reference build (oracle/Makefile libhtsref_simd.so,
bench.py's AVX2-enabled CPU baseline) writes the same bytes
as the as-shipped scalar build: the X32 orders it dispatches to SSE4 / AVX2
/ AVX-512 and the 4x16 orders it leaves scalar."""
import numpy as np
import pytest

from oracle import binding


@pytest.mark.skipif(not binding.have_ref_simd(), reason="oracle/_ref/libhtsref_simd.so not built")
@pytest.mark.parametrize("order", [0, 1, 4, 5, 133, 197])
def test_simd_build_same_bytes(order):
    rng = np.random.default_rng(order)
    data = rng.choice(np.frombuffer(b"#+5?FFIIII", np.uint8), 200_003).tobytes()
    a = binding.ref().rans_compress(data, order)
    b = binding.ref_simd().rans_compress(data, order)
    assert a == b
    assert binding.ref_simd().rans_uncompress(a) == data
