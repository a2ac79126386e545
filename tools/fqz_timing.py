"""fqz_compress / fqz_decompress timing through the C-ABI on one block of
synthetic quality data (host buffers, so PCIe copies are included)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib, synth  # noqa: E402

nreads = int(sys.argv[1]) if len(sys.argv) > 1 else 290000
dec_reads = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
for kind in ("illumina8", "novaseq"):
    r = synth.illumina(nreads, seed=3) if kind == "illumina8" else synth.novaseq(nreads, seed=3)
    q = r.qual.tobytes()
    lens = r.lens.astype(np.uint32)
    for st in (0, 1, 2):
        lib.fqz_compress(q[:100000], lens[:100000 // 150].copy(), np.zeros(100000 // 150, np.uint32), st)
        t0 = time.perf_counter()
        c = lib.fqz_compress(q, lens.copy(), np.zeros(len(lens), np.uint32), st)
        t1 = time.perf_counter()
        nd = dec_reads
        cd = lib.fqz_compress(q[:nd * 150], lens[:nd].copy(), np.zeros(nd, np.uint32), st)
        t2 = time.perf_counter()
        back, _ = lib.fqz_decompress(cd, lens[:nd].copy(), np.zeros(nd, np.uint32))
        t3 = time.perf_counter()
        assert back == q[:nd * 150]
        print(f"{kind:9s} strat {st}: enc {len(q)/1e6:.1f} MB -> {len(c)/1e6:.2f} MB in "
              f"{t1-t0:.3f} s ({len(q)/(t1-t0)/1e6:.1f} MB/s); dec {nd*150/1e6:.1f} MB in "
              f"{t3-t2:.3f} s ({nd*150/(t3-t2)/1e6:.2f} MB/s)", flush=True)
