"""zlib's crc32 on the GPU (fqz5_crc32 / fqz5_crc32_dev):
equal to zlib.crc32 for sizes around the 256-byte segments and 64 KiB
tiles, unaligned device buffers, chained initial values, and a 300 MB
buffer spanning several combine passes."""
import zlib

import numpy as np
import pytest
import torch

from fqzcomp5_amd import lib

pytestmark = pytest.mark.gpu


def test_crc32_host_sizes():
    rng = np.random.default_rng(1)
    for n in (0, 1, 3, 15, 16, 255, 256, 257, 4095, 65535, 65536, 65537, 200_001, 1 << 20):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for crc in (0, 0xDEADBEEF):
            assert lib.crc32(b, crc) == zlib.crc32(b, crc), (n, crc)


def test_crc32_device_unaligned_and_large():
    rng = np.random.default_rng(2)
    n = 300_000_003
    h = rng.integers(0, 256, n, dtype=np.uint8)
    d = torch.from_numpy(h).to("cuda:0")
    hb = h.tobytes()
    torch.cuda.synchronize()
    for off, ln in ((0, n), (1, n - 7), (13, 65536 * 3 + 5), (7, 100)):
        got = lib.crc32_dev(d.data_ptr() + off, ln, 0x1234)
        assert got == zlib.crc32(hb[off:off + ln], 0x1234), (off, ln)


def test_crc32_block_checksum_form():
    # fqzcomp5.c:2268-2269: crc32(crc32(0, NULL, 0), comp + 12, size - 12)
    b = bytes(range(256)) * 1000
    assert lib.crc32(b[12:], lib.crc32(b"", 0)) == zlib.crc32(b[12:])
