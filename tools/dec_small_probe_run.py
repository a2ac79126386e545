"""Per-symbol cycle split of k_fqz_dec_small, from the
probe build's s_memtime stamps (fqz_decode_small.hip, FQZ5_SMALL_PROBE):

  VARIANT_DIR=tools/vbuild tools/build_variant.sh sprobe fqz_decode_small -DFQZ5_SMALL_PROBE
  FQZ5_LIB_VARIANT=tools/vbuild/libfqz5_sprobe.so python tools/dec_small_probe_run.py [MSYM]

For NovaSeq 4-level and Illumina 8-level qualities, strategies 0-2: the
segments' cycles per fast symbol (A..E as in the kernel's comment), the
stamped build's ns per symbol, and the decoder's miss / slow counters."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/vbuild/libfqz5_sprobe.so"))
os.environ.setdefault("FQZ5_DEBUG", "1")
sys.path.insert(0, ROOT)
from fqzcomp5_amd import lib, synth  # noqa: E402

msym = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
so = lib.load()
so.fqz5_small_probe_read.argtypes = [C.POINTER(C.c_uint64)]
NAMES = ["division (A-B)", "p_i + ballot + next set (B-C)", "readlanes + coder + update (C-D)",
         "next model read issue (D-E)", "model read wait + loop (E-A)"]
for kind in ("novaseq", "illumina8"):
    n = int(msym * 1e6)
    r = synth.novaseq(n // 150, seed=3) if kind == "novaseq" else synth.illumina(n // 150, seed=3)
    q, lens = r.qual.tobytes(), r.lens.astype(np.uint32)
    fl = np.zeros(len(lens), np.uint32)
    for st in (0, 1, 2):
        c = lib.fqz_compress(q, lens.copy(), fl.copy(), st)
        lib.fqz_decompress(c, lens.copy(), fl.copy())          # warm
        p = (C.c_uint64 * 6)()
        so.fqz5_small_probe_read(p)                             # (clears)
        t0 = time.perf_counter()
        back, _ = lib.fqz_decompress(c, lens.copy(), fl.copy())
        dt = time.perf_counter() - t0
        assert back == q
        so.fqz5_small_probe_read(p)
        nsym = max(int(p[5]), 1)
        segs = [p[i] / nsym for i in range(5)]
        print(f"{kind:9s} strat {st}: {len(q)/1e6:.2f} M symbols, {nsym/1e6:.2f} M on the fast path; "
              f"stamped build {dt/len(q)*1e9:.1f} ns/sym; cycles per symbol: "
              + ", ".join(f"{nm} {v:.1f}" for nm, v in zip(NAMES, segs))
              + f"; sum {sum(segs):.1f}", flush=True)
