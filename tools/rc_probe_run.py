"""Cycles of the fqz range chain (library built with tools/build_variant.sh
rcprobe fqz_kernels -DFQZ5_RC_PROBE): whole kernel vs the lane-0 chain."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/variants/libfqz5_rcprobe.so"))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import lib, synth  # noqa: E402
r = synth.novaseq(290000, seed=3)
so = lib.load()
for st in (1, 3):
    c = lib.fqz_compress(r.qual.tobytes(), r.lens.astype(np.uint32), np.zeros(len(r.lens), np.uint32), st)
    p = (C.c_uint64 * 4)()
    so.fqz5_rc_probe_read(p)
    print(f"strat {st}: {len(c)} B; rc total {p[0]/max(p[2],1):.1f} cyc/event, chain {p[1]/max(p[2],1):.1f} cyc/event over {p[2]} events", flush=True)
