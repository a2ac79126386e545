"""The -5 file-path golden: a seeded synthetic
random-walk Illumina FASTQ of >= 1.5 GB coded by the reference CLI as shipped
(oracle/_ref/fqzcomp5 -5 -t1, its preset blocks), recorded as the input's and
output's md5 and sizes in l5_illumina.json.  The input is regenerated from
the seed on the GPU box (synth.illumina), so only this record travels.
python tests/golden/make_golden_l5.py [workdir]"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fqzcomp5_amd import synth  # noqa: E402

NREADS, SEED = 4_300_000, 13


def make_input(path: str) -> int:
    r = synth.illumina(NREADS, seed=SEED, with_names=True)
    return synth.write_fastq(r, path)


def md5(path: str) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for c in iter(lambda: f.read(1 << 24), b""):
            h.update(c)
    return h.hexdigest()


if __name__ == "__main__":
    wd = sys.argv[1] if len(sys.argv) > 1 else "/tmp/l5"
    os.makedirs(wd, exist_ok=True)
    src, out = os.path.join(wd, "illumina.fastq"), os.path.join(wd, "illumina.fqz5")
    n = make_input(src)
    t0 = time.time()
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "fqzcomp5"), "-5", "-t1", src, out],
                   check=True)
    rec = dict(nreads=NREADS, seed=SEED, in_bytes=n, in_md5=md5(src),
               out_bytes=os.path.getsize(out), out_md5=md5(out), level=5,
               ref_seconds=round(time.time() - t0, 1),
               cmd="oracle/_ref/fqzcomp5 -5 -t1 illumina.fastq illumina.fqz5")
    json.dump(rec, open(os.path.join(ROOT, "tests", "golden", "l5_illumina.json"), "w"), indent=1)
    print(rec)
