"""Per-stream kernel timing: encode and decode one stream at a time through
the C-ABI with the library's HIP-event profile, so the per-step cost of a
chain is seen without other streams sharing its SIMD."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib, synth  # noqa: E402

r = synth.illumina(int(sys.argv[1]) if len(sys.argv) > 1 else 290000, seed=1)
so = lib.load()
for name, data, orders in (("seq", r.seq.tobytes(), (0, 1, 129)),
                           ("qual", r.qual.tobytes(), (0, 1, 129, 193))):
    for o in orders:
        comp = lib.rans_compress(data, o)          # warm
        so.fqz5_profile(1)
        comp = lib.rans_compress(data, o)
        back = lib.rans_uncompress(comp)
        p = (C.c_double * 6)()
        so.fqz5_profile_read(p)
        so.fqz5_profile(0)
        steps = len(data) / 4
        if o & 0x80:
            steps /= 2 if name == "qual" else 2
        print(f"{name:4s} o={o:3d} n={len(data)} c={len(comp)} enc {p[0]:8.2f} ms "
              f"dec {p[3]:8.2f} ms  enc ns/step {p[0]*1e6/steps:6.2f} "
              f"dec ns/step {p[3]*1e6/steps:6.2f} ok={back == data}", flush=True)
