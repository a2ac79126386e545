"""Trial candidate sizes of the section coder at -5 against the oracle's
sizes for the same blocks (debugging aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import sections as S, synth  # noqa: E402
from oracle import binding  # noqa: E402

torch.cuda.init()
reads = synth.illumina(72000, seed=11)
blocks = synth.split_blocks(reads, 4_000_000)
run = S.Run(reads, blocks, torch.device("cuda", 0))
res, meth, sizes, tried, _ = S.encode_run(run.enc_secs(), S.masks(5), S.new_state())
o = binding.oracle()
for i, (sec, s, e, fl, k) in enumerate(run.spans[:6]):
    if sec != S.SEC_QUAL:
        continue
    a, b = blocks[k]
    q = reads.qual[s:e].tobytes()
    row = {m: int(sizes[i, m]) for m in range(S.M_LAST) if sizes[i, m] != 0xFFFFFFFF}
    exp = {1: len(o.rans_compress(q, 0)), 6: len(o.rans_compress(q, 129)),
           27: len(o.fqz_compress(q, reads.lens[a:b].copy(), np.zeros(b - a, np.uint32), 1,
                                  reads.seq[s:e].tobytes()))}
    print(i, e - s, "gpu", row, "oracle", exp, "chosen", int(meth[i]))
print("methods", meth.tolist())
