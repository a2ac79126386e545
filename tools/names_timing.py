"""One -3 whole-block step on the bench's 1 GB workload with the library's
phase trace (FQZ5_STEP_TRACE): where the name-section time goes."""
import os
import sys
import time

os.environ.setdefault("FQZ5_STEP_TRACE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
torch.cuda.init()
import bench  # noqa: E402
from fqzcomp5_amd import sections as S, synth  # noqa: E402

level = int(sys.argv[1]) if len(sys.argv) > 1 else 3
gb = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
reads = bench.make_reads(gb, 1, "illumina" if level == 3 else "novaseq")
blocks = synth.split_blocks(reads, bench.BLK)
run = S.Run(reads, blocks, torch.device("cuda", 0))
enc = run.enc_secs()
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res, meth, sizes, tried, off = S.encode_run(enc, S.masks(level, full=True), S.new_state())
    t1 = time.perf_counter()
    run.assemble(res)
    t2 = time.perf_counter()
    ds = run.block_dec_secs()
    t3 = time.perf_counter()
    dres = S.decode(ds)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"encode_run {1e3*(t1-t0):.1f} ms  assemble {1e3*(t2-t1):.1f} ms  parse {1e3*(t3-t2):.1f} ms"
          f"  decode {1e3*(t4-t3):.1f} ms", flush=True)
print("roundtrip", run.roundtrip_ok())
