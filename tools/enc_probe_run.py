"""Encoder chain cycle split (a library built with
tools/build_variant.sh cprobe rans_chain -DFQZ5_CHAIN_PROBE): shader cycles
of k_enc_chain spent in the chain loop vs. staging, per step, for one O0
stream of a -3 block's sequence section (44 MB)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/variants/libfqz5_cprobe.so"))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import lib, synth  # noqa: E402

r = synth.illumina(int(sys.argv[1]) if len(sys.argv) > 1 else 290000, seed=1)
so = lib.load()
for name, data, order in (("seq", r.seq.tobytes(), 0), ("qual", r.qual.tobytes(), 0),
                          ("qual", r.qual.tobytes(), 1)):
    for rep in range(2):
        z = (C.c_uint64 * 8)()
        so.fqz5_chain_probe_read(z)
        base = list(z)
        so.fqz5_profile(1)
        comp = lib.rans_compress(data, order)
        p = (C.c_double * 6)()
        so.fqz5_profile_read(p)
        so.fqz5_profile(0)
        so.fqz5_chain_probe_read(z)
        st, ch = z[0] - base[0], z[1] - base[1]
        steps = len(data) / 4
        print(f"{name} o{order} n={len(data)} launch {p[0]:.1f} ms ({p[0]*1e6/steps:.2f} ns/step) "
              f"chain {ch/steps:.1f} cyc/step stage {st/steps:.1f} cyc/step", flush=True)
