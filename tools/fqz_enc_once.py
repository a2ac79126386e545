"""One fqz_compress of a 43.5 MB quality block (for kernel profiling)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import lib, synth  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "novaseq"
st = int(sys.argv[2]) if len(sys.argv) > 2 else 0
r = synth.illumina(290000, seed=3) if kind == "illumina8" else synth.novaseq(290000, seed=3)
c = lib.fqz_compress(r.qual.tobytes(), r.lens.astype(np.uint32), np.zeros(len(r.lens), np.uint32), st)
print(kind, st, len(c))
