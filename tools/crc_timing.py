"""fqz5_crc32_dev throughput on a device-resident buffer (wall time of the
whole call: table upload, tile kernel, combine passes, sync)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib  # noqa: E402

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(gb * (1 << 30))
d = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda:0")
torch.cuda.synchronize()
lib.crc32_dev(d.data_ptr(), n)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    lib.crc32_dev(d.data_ptr(), n)
    ts.append(time.perf_counter() - t0)
t = min(ts)
print(f"crc32 {n} bytes: {t*1e3:.3f} ms (best of 5) = {n/t/1e9:.1f} GB/s", flush=True)
