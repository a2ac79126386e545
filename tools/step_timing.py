"""Phases of one bench step (FQZ5_STEP_TRACE=1 prints the library's own
phase lines): where the wall time between GPU launches goes.
Usage: step_timing.py [3|5]  (-3: 1 GB Illumina, -5: 4 GB NovaSeq, the
bench's workloads, full preset masks)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
torch.cuda.init()
import bench  # noqa: E402
from fqzcomp5_amd import sections as S, synth  # noqa: E402

level = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reads = (bench.make_reads(1.0, 1, "illumina") if level == 3 else bench.make_reads(4.0, 2, "novaseq"))
blocks = synth.split_blocks(reads, bench.BLK)
run = S.Run(reads, blocks, torch.device("cuda", 0))
enc = run.enc_secs()
if "prof" in sys.argv[2:]:              # the bench's live kernel timing (HIP events)
    from fqzcomp5_amd import lib
    lib.load().fqz5_profile(1)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = S.new_state()
    res, meth, sizes, tried, off = S.encode_run(enc, S.masks(level, full=True), st)
    t1 = time.perf_counter()
    ds = run.dec_secs(res)
    t2 = time.perf_counter()
    dres = S.decode(ds)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"encode_run {1e3*(t1-t0):.1f} ms  dec_secs {1e3*(t2-t1):.1f} ms  decode {1e3*(t3-t2):.1f} ms",
          flush=True)
