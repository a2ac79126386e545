"""fqz decoder timing per data kind and strategy.

python tools/fqz_dec_bench.py [MSYM] [kinds] [strats]
  MSYM   quality symbols per block in millions (default 4)
  kinds  comma list of novaseq,illumina8,ont,hifi (default all)
  strats comma list (default 0,1,2,3,4)

For each case: encode on the GPU, decode on the GPU through the C-ABI
(fqz_decompress, host buffers: one upload + one download of a few MB, small
next to the chain), print ns per symbol; the reference's own fqz_decompress
(oracle/_ref/libhtsref.so, one core) decodes the same stream beside it when
present.  FQZ5_DEBUG=1 adds the decoder's miss / slow-path counters.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib, synth  # noqa: E402

msym = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
kinds = (sys.argv[2] if len(sys.argv) > 2 else "novaseq,illumina8,ont,hifi").split(",")
strats = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,1,2,3,4").split(",")]
ref = None
try:
    from oracle import binding
    if binding.have_ref():
        ref = binding.ref()
except Exception:  # noqa: BLE001 - the CPU column is optional
    ref = None


def make(kind: str, n: int):
    if kind == "novaseq":
        r = synth.novaseq(max(1, n // 150), seed=3)
    elif kind == "illumina8":
        r = synth.illumina(max(1, n // 150), seed=3)
    elif kind == "ont":
        r = synth.ont(max(1, n // 12000), seed=3)
    else:
        r = synth.hifi(max(1, n // 30000), seed=5)
    flags = r.flags if getattr(r, "flags", None) is not None else np.zeros(len(r.lens), np.uint32)
    return r.qual.tobytes(), r.lens.astype(np.uint32), np.asarray(flags, np.uint32), r.seq.tobytes()


for kind in kinds:
    q, lens, flags, seq = make(kind, int(msym * 1e6))
    for st in strats:
        c = lib.fqz_compress(q, lens.copy(), flags.copy(), st, seq=seq)
        best = 1e9
        for _ in range(2):
            t0 = time.perf_counter()
            back, _ = lib.fqz_decompress(c, lens.copy(), flags.copy(), seq=seq)
            best = min(best, time.perf_counter() - t0)
        assert back == q, f"{kind} strat {st}: round trip"
        line = (f"{kind:9s} strat {st}: {len(q)/1e6:6.2f} MB -> {len(c)/1e6:6.3f} MB  "
                f"GPU dec {best:7.3f} s = {best/len(q)*1e9:6.1f} ns/sym")
        if ref is not None:
            t0 = time.perf_counter()
            rb = ref.fqz_decompress(c, lens.copy(), flags.copy(), seq=seq)
            t1 = time.perf_counter()
            rb = rb[0] if isinstance(rb, tuple) else rb
            line += f"  | ref 1 core {(t1-t0)/len(q)*1e9:6.1f} ns/sym ({'ok' if rb == q else 'DIFF'})"
        print(line, flush=True)
