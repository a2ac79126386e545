import numpy as np, torch, sys
sys.path.insert(0, '.')
from fqzcomp5_amd import lib, sections as S, synth
reads = synth.novaseq(6000, seed=11)
blocks = synth.split_blocks(reads, 200_000)
run = S.Run(reads, blocks, torch.device("cuda", 0))
res, meth_all, sizes, tried, _ = S.encode_run(run.enc_secs(), S.masks(5), S.new_state())
for i, r in enumerate(res):
    print(i, run.spans[i][0], 'meth', int(meth_all[i]), 'status', r.status, 'clen', r.clen, 'tried', hex(int(tried[i])))
print('sizes fqz', sizes[:6, S.FQZ1], sizes[:6, S.FQZ3], sizes[:6, S.RANS0])
