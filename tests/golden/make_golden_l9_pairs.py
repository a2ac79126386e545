"""The configs[4] golden at reduced size: seeded
synthetic PacBio HiFi pairs as two FASTQ files (R1: the /1 reads, R2: the /2
reads) of >= 2.2 GB together, coded by the reference CLI as shipped
(oracle/_ref/fqzcomp5 -9 -t1 r1 r2 out: load_seqs_interleaved,
fqzcomp5.c:627-865, the -9 preset's 1 GB blocks, :4931), recorded as the
inputs' and output's md5 and sizes in l9_pairs.json.  The inputs are
regenerated from the seed on the GPU box (synth.hifi), so only this record
travels.
python tests/golden/make_golden_l9_pairs.py [workdir]"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import synth  # noqa: E402

NPAIRS, SEED = 38_000, 17


def make_inputs(p1: str, p2: str) -> tuple[int, int]:
    """R1 and R2 of the seeded HiFi pairs, written a chunk of pairs at a time
    (bounded host memory)."""
    import numpy as np
    r = synth.hifi(NPAIRS, seed=SEED, with_names=True)
    names = synth.all_names(r)
    buf, off = names
    n1 = n2 = 0
    with open(p1, "wb") as f1, open(p2, "wb") as f2:
        step = 2000
        for a in range(0, r.num_records, step):
            b = min(a + step, r.num_records)
            txt = synth.fastq_chunk(r, a, b, names)
            rec = (off[a + 1:b + 1] - off[a:b] - 1) + 2 * r.lens[a:b].astype(np.int64) + 6
            st = np.concatenate([[0], np.cumsum(rec)])
            for k in range(b - a):
                piece = txt[st[k]:st[k + 1]].tobytes()
                if (a + k) % 2 == 0:
                    f1.write(piece)
                    n1 += len(piece)
                else:
                    f2.write(piece)
                    n2 += len(piece)
    return n1, n2


def md5(path: str) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for c in iter(lambda: f.read(1 << 24), b""):
            h.update(c)
    return h.hexdigest()


if __name__ == "__main__":
    wd = sys.argv[1] if len(sys.argv) > 1 else "/tmp/l9p"
    os.makedirs(wd, exist_ok=True)
    r1, r2, out = (os.path.join(wd, x) for x in ("r1.fastq", "r2.fastq", "pairs.fqz5"))
    n1, n2 = make_inputs(r1, r2)
    t0 = time.time()
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "fqzcomp5"), "-9", "-t1", r1, r2, out],
                   check=True)
    rec = dict(npairs=NPAIRS, seed=SEED, r1_bytes=n1, r2_bytes=n2, r1_md5=md5(r1),
               r2_md5=md5(r2), out_bytes=os.path.getsize(out), out_md5=md5(out), level=9,
               ref_seconds=round(time.time() - t0, 1),
               cmd="oracle/_ref/fqzcomp5 -9 -t1 r1.fastq r2.fastq pairs.fqz5")
    json.dump(rec, open(os.path.join(ROOT, "tests", "golden", "l9_pairs.json"), "w"), indent=1)
    print(rec)
