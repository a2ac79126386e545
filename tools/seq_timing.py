"""Wall time of the sequence context model on the GPU (host-buffer entry
points, so copies included) for an Illumina-like sequence section.
Usage: python tools/seq_timing.py [MB]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib  # noqa: E402

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 4
rng = np.random.default_rng(1)
g = rng.choice(np.frombuffer(b"ACGT", np.uint8), 50_000_000)
nrec = int(mb * 1e6 / 150)
st = rng.integers(0, len(g) - 150, nrec)
seq = g[(st[:, None] + np.arange(150)[None, :])].tobytes()
lens = [150] * nrec
lib.seq_encode(seq[:15000], lens[:100], 0, 10)        # warm up
for k, both in ((10, 0), (12, 1)):
    t0 = time.time()
    c = lib.seq_encode(seq, lens, both, k)
    t1 = time.time()
    d = lib.seq_decode(c, lens, both, k, len(seq))
    t2 = time.time()
    assert d == seq
    print(f"k={k} both={both} n={len(seq)} comp={len(c)} enc {t1-t0:.3f} s "
          f"({len(seq)/(t1-t0)/1e6:.1f} MB/s) dec {t2-t1:.3f} s ({len(seq)/(t2-t1)/1e6:.2f} MB/s)",
          flush=True)
