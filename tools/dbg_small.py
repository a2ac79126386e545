"""Debug the small-alphabet fqz decoder: first mismatch per variant."""
import os, sys, subprocess
os.environ.setdefault("FQZ5_DEC_SMALL", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
from fqz_cases import cases
from fqzcomp5_amd import lib, synth
from oracle import binding
ora = binding.oracle()
cs = {c[0]: c for c in cases()}
items = []
for name in ("bin8_small", "bin4_small"):
    if name in cs:
        items.append(cs[name])
r = synth.illumina(3000, seed=21)
items.append(("illum3000", r.qual.tobytes(), r.lens.astype(np.uint32), np.zeros(3000, np.uint32), None))
for name, q, lens, flags, seq in items:
    for strat in (0, 1, 2):
        comp = ora.fqz_compress(q, lens.copy(), flags.copy(), strat, seq)
        out, _ = lib.fqz_decompress(comp, lens.copy(), flags.copy(), seq)
        if out == q:
            print(name, strat, "OK", len(q), flush=True)
        else:
            a = np.frombuffer(out, np.uint8); b = np.frombuffer(q, np.uint8)
            i = int(np.nonzero(a[:len(b)] != b[:len(a)])[0][0]) if len(a) and len(b) else -1
            print(name, strat, "MISMATCH at", i, "of", len(q), "lens0", int(lens[0]), "got", list(a[max(0,i-3):i+5]), "want", list(b[max(0,i-3):i+5]), flush=True)
