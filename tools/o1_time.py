"""Wall time of one O1 4x16 stream decode (rans_uncompress_4x16, host
buffers) on NovaSeq-like qualities: ns per step of the chain."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib, synth  # noqa: E402

r = synth.novaseq(290_000, seed=2)
q = r.qual.tobytes()
for order in (1, 0):
    c = lib.rans_compress(q, order)
    lib.rans_uncompress(c)
    t0 = time.time()
    for _ in range(3):
        d = lib.rans_uncompress(c)
    t = (time.time() - t0) / 3
    assert d == q
    print(f"order {order} n={len(q)} steps={len(q)//4} {t*1e3:.1f} ms {t/(len(q)/4)*1e9:.1f} ns/step", flush=True)
