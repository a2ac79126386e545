"""Ordering contract of the device-pointer entry points (include/fqz5_mi355x.h,
fqz5_stream_wait; VERDICT r02 weak #9, the 48a269b race): a producer writes
the input on another stream, with no host synchronisation, after a long
queue of work on that stream; fqz5_stream_wait orders the library's stream
after it and the device-pointer call reads the finished bytes."""
import zlib

import numpy as np
import pytest
import torch

from fqzcomp5_amd import lib

pytestmark = pytest.mark.gpu


def test_producer_on_other_stream():
    n = 64 << 20
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, n, dtype=np.uint8)
    want = zlib.crc32(host.tobytes())
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    a = torch.randn(4096, 4096, device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(40):          # tens of ms of queued work before the copy
            a = torch.tanh(a @ a)
        dst.copy_(src)
    lib.stream_wait(side.cuda_stream)
    got = lib.crc32_dev(dst.data_ptr(), n)
    side.synchronize()
    assert got == want


def test_outputs_ready_on_return():
    """Outputs are complete when the call returns: another stream reads them
    without waiting on the library's stream."""
    data = bytes(range(256)) * 4096
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    for _ in range(3):
        c = lib.crc32_dev(d.data_ptr(), d.numel())
        with torch.cuda.stream(side):
            x = d.sum()
        side.synchronize()
        assert c == zlib.crc32(data) and int(x) == sum(data)
