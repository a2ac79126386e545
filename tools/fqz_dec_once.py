"""One fqz_compress + fqz_decompress of a synthetic block (for rocprof /
FQZ5_DEBUG=1 counters): python tools/fqz_dec_once.py {novaseq|illumina} STRAT [NREADS]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib, synth  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "novaseq"
strat = int(sys.argv[2]) if len(sys.argv) > 2 else 0
nreads = int(sys.argv[3]) if len(sys.argv) > 3 else 290000
r = synth.novaseq(nreads, seed=3) if kind == "novaseq" else synth.illumina(nreads, seed=3)
q = r.qual.tobytes()
lens = r.lens.astype(np.uint32)
c = lib.fqz_compress(q, lens.copy(), np.zeros(len(lens), np.uint32), strat)
t0 = time.perf_counter()
back, _ = lib.fqz_decompress(c, lens.copy(), np.zeros(len(lens), np.uint32))
t1 = time.perf_counter()
assert back == q
print(f"{kind} strat {strat}: {len(q)/1e6:.1f} MB dec in {t1-t0:.3f} s "
      f"({(t1-t0)/len(q)*1e9:.1f} ns/symbol)", flush=True)
