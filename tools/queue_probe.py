"""Hardware-queue probe ("Hardware queues"): one fqz
quality stream (block 0 of the level5_illumina workload, FQZ strategy 1 --
the bytes the -5 trial picks) decoded before and after a -5 encode of the
1 GB workload in the same process.  Run once per setting, e.g.
  FQZ5_HW_QUEUES=32 python tools/queue_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fqzcomp5_amd import lib, sections as S, synth  # noqa: E402

reads = bench.make_reads(1.0, 1, "illumina")
blocks = synth.split_blocks(reads, bench.BLK)
r0 = synth.block(reads, *blocks[0])
q = r0.qual.tobytes()
n = len(r0.lens)
lens = r0.lens.astype(np.uint32)
c = lib.fqz_compress(q, lens.copy(), np.zeros(n, np.uint32), 1)
tag = os.environ.get("GPU_MAX_HW_QUEUES")


def dec(what):
    ts = []
    for _ in range(2):
        t0 = time.perf_counter()
        out, _ = lib.fqz_decompress(c, lens.copy(), np.zeros(n, np.uint32))
        ts.append(time.perf_counter() - t0)
        assert out == q
    print(f"queues {tag} {what}: " + " ".join(f"{t / len(q) * 1e9:.1f}" for t in ts)
          + " ns/symbol", flush=True)


dec("fresh")
run = S.Run(reads, blocks, torch.device("cuda", 0))
t0 = time.perf_counter()
S.encode_run(run.enc_secs(), S.masks(5, full=True), S.new_state())
torch.cuda.synchronize()
print(f"queues {tag} encode {time.perf_counter() - t0:.2f} s", flush=True)
dec("after encode")
