"""Drive tools/fqz_stats.c: compress synthetic blocks with the reference
(oracle/_ref) and print decoder design statistics per kind and strategy.
python tools/fqz_stats.py [MSYM]"""
import json
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
exec(open(os.path.join(os.path.dirname(__file__), "fqz_dec_bench.py")).read().split("for kind in kinds:")[0]
     .replace("msym = float(sys.argv[1])", "msym = 0 and float(sys.argv[1])"))
msym = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
exe = "/tmp/fqz_stats"
subprocess.run(["gcc", "-O2", "-I", f"{root}/oracle", f"{root}/tools/fqz_stats.c",
                f"{root}/oracle/rans_oracle.c", "-lm", "-o", exe], check=True)
for kind in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("novaseq", "illumina8", "ont", "hifi")):
    q, lens, flags, seq = make(kind, int(msym * 1e6))
    for st in range(5):
        c = ref.fqz_compress(q, lens.copy(), flags.copy(), st, seq=None)
        with tempfile.NamedTemporaryFile(delete=False) as f:
            f.write(c)
        r = json.loads(subprocess.run([exe, f.name], capture_output=True, text=True, check=True).stdout)
        os.unlink(f.name)
        print(f"{kind:9s} {st}: k {r['k_mean']:.2f} k>1 {r['k_gt'][0]:.2f} k>2 {r['k_gt'][1]:.2f} "
              f"k>4 {r['k_gt'][2]:.2f} k>32 {r['k_gt'][5]:.4f} k>62 {r['k_gt'][6]:.4f} swap {r['swap']:.3f} halve {r['halve']:.4f} same {r['same_ctx']:.3f} "
              f"ctx {r['contexts']} miss " + " ".join(f"{k}:{v:.3f}" for k, v in r['miss'].items()), flush=True)
        print("          assoc (miss, refetch): " + " ".join(f"{k}:{v[0]:.3f}/{v[1]:.3f}" for k, v in r['assoc'].items()), flush=True)
