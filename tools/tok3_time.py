"""Time the host tokeniser (fqz5_tok3_tokenise_bytes: tok3_tokenise without
the GPU stages) on one 100 MB block's names (~280 000 Illumina names), on
the CPU.  Usage: python tools/tok3_time.py [n_names]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 280000
so = C.CDLL(os.path.join(ROOT, "fqzcomp5_amd", "libfqz5_mi355x.so"))
so.fqz5_tok3_tokenise_bytes.restype = C.c_longlong
so.fqz5_tok3_tokenise_bytes.argtypes = [C.c_char_p, C.c_int, C.c_int]
r = synth.illumina(n, seed=1)
buf, off = synth.all_names(r)
data = bytes(buf)
for rep in range(3):
    t0 = time.perf_counter()
    tot = so.fqz5_tok3_tokenise_bytes(data, len(data), 3)
    t1 = time.perf_counter()
    print(f"{n} names, {len(data)} B: {1e3*(t1-t0):.1f} ms, {tot} stream bytes")
