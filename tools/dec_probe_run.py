"""Cycle stamps of the O0 NX=4 decoder (a library built with
tools/build_variant.sh cprobe rans_chain -DFQZ5_CHAIN_PROBE): total and
full-step-loop shader cycles of the first stream of the launch, the
in-kernel clock from s_memrealtime (100 MHz), cycles per step."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/variants/libfqz5_cprobe.so"))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import lib, synth  # noqa: E402

r = synth.illumina(int(sys.argv[1]) if len(sys.argv) > 1 else 290000, seed=1)
so = lib.load()
for name, data in (("seq", r.seq.tobytes()), ("qual", r.qual.tobytes())):
    comp = lib.rans_compress(data, 0)
    back = lib.rans_uncompress(comp)
    p = (C.c_uint64 * 8)()
    so.fqz5_chain_probe_read(p)
    tot, real, ts, ns, T = p[2], p[3], p[4], p[5], p[6]
    ghz = tot / (real * 10.0) if real else 0
    print(f"{name} O0 ok={back == data} steps={T} total {tot} cyc ({tot/max(T,1):.1f}/step) "
          f"loop {ts} cyc over {ns} steps ({ts/max(ns,1):.1f}/step) clock {ghz:.3f} GHz "
          f"wall {real/100:.0f} us", flush=True)
