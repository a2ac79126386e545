"""Cycle breakdown of the sequence CM decoder's base step (a library built
with -DFQZ5_SEQ_PROBE for seq_cm.hip, loaded through FQZ5_LIB_VARIANT):
load + symbol / renorm + stores / next counts + reverse update / between
steps, in shader cycles per base, for one Illumina-like block."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/v2/libfqz5_seqprobe.so"))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import lib  # noqa: E402

rng = np.random.default_rng(1)
g = rng.choice(np.frombuffer(b"ACGT", np.uint8), 5_000_000)
nrec = 6667
st = rng.integers(0, len(g) - 150, nrec)
seq = g[(st[:, None] + np.arange(150)[None, :])].tobytes()
lens = [150] * nrec
so = lib.load()
so.fqz5_seq_probe_read.argtypes = [C.POINTER(C.c_uint64)]
for k, both in ((10, 0), (12, 1)):
    c = lib.seq_encode(seq, lens, both, k)
    assert lib.seq_decode(c, lens, both, k, len(seq)) == seq
    p = (C.c_uint64 * 8)()
    so.fqz5_seq_probe_read(p)
    n = max(p[4], 1)
    print(f"k={k} both={both} steps={p[4]}: load+symbol {p[0]/n:.0f}  renorm+stores {p[1]/n:.0f}  "
          f"next+reverse {p[2]/n:.0f}  between steps {p[3]/n:.0f} cycles/base", flush=True)
