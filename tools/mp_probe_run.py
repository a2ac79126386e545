"""The fqz model pass's slowest lane (library built with
VARIANT_DIR=tools/vbuild tools/build_variant.sh mprobe fqz_kernels -DFQZ5_MP_PROBE):
one -5 Illumina-style block encoded with FQZ1, the model id, its events and
its cycles."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/vbuild/libfqz5_mprobe.so"))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import lib, synth  # noqa: E402
so = lib.load()
so.fqz5_mp_probe_read.argtypes = [C.POINTER(C.c_uint64)]
for kind, n in (("illumina", 296000), ("novaseq", 296000)):
    r = synth.illumina(n, seed=3) if kind == "illumina" else synth.novaseq(n, seed=3)
    for st in (1, 3):
        p = (C.c_uint64 * 2)()
        so.fqz5_mp_probe_read(p)
        c = lib.fqz_compress(r.qual.tobytes(), r.lens.astype(np.uint32), np.zeros(len(r.lens), np.uint32), st)
        so.fqz5_mp_probe_read(p)
        cyc = (p[0] >> 24) << 4
        print(f"{kind} strat {st}: {len(c)} B; slowest lane: model {p[0] & 0xffffff}, {p[1]} events, "
              f"{cyc} cycles ({cyc / 2.4e6:.1f} ms at 2.4 GHz, {cyc / max(p[1], 1):.0f} cycles per event)", flush=True)
