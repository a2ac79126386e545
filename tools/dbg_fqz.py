import sys; sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import numpy as np
from fqz_cases import cases
from fqzcomp5_amd import lib
from oracle import binding
ora=binding.oracle()
cs={c[0]:c for c in cases()}
for nm in ("bin8_small","one_record","tiny_var","nova_small"):
    name,q,lens,flags,seq=cs[nm]
    exp=ora.fqz_compress(q,lens.copy(),flags.copy(),2,seq)
    got=lib.fqz_compress(q,lens.copy(),flags.copy(),2,seq)
    d=[i for i in range(min(len(exp),len(got))) if exp[i]!=got[i]]
    print(nm,len(exp),len(got),"ndiff",len(d),"first",d[:12])
    if d:
        i=d[0]; print(" exp",exp[max(0,i-4):i+12].hex()); print(" got",got[max(0,i-4):i+12].hex())
