"""configs[2]'s whole -5 file pinned to the single-threaded reference
(VERDICT r05 item 1): the bench's seeded 4 GB NovaSeq FASTQ (bench.make_reads
(4.0, seed 2, "novaseq"), the `level5` item's rank-0 workload) coded by the
reference CLI as shipped, `oracle/_ref/fqzcomp5 -5 -t1 -b 100000000` (its
trial in file order, fqzcomp5.c:1899-1958; block framing :2147-2280).
Recorded in l5_novaseq.json: the input's md5 and size, the output's md5, the
md5 of the block bytes (the file between its 16-byte header and the index,
which is what the bench's assembled blocks concatenate to) and each block's
own md5, so the bench can say which blocks match.  The input is regenerated
from the seed on the GPU box; only this record travels.
python tests/golden/make_golden_l5_novaseq.py [workdir]"""
import hashlib
import json
import os
import struct
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

GB, SEED, KIND, BLK = 4.0, 2, "novaseq", 100_000_000


def md5(path: str) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for c in iter(lambda: f.read(1 << 24), b""):
            h.update(c)
    return h.hexdigest()


def block_md5s(path: str):
    """(md5 of all block bytes, [md5 of each block]) of a .fqz5 file."""
    buf = open(path, "rb").read()
    (idx,) = struct.unpack_from("<Q", buf, 8)
    end = idx if idx else len(buf)
    p, each = 16, []
    while p < end:
        (bsz,) = struct.unpack_from("<I", buf, p)
        each.append(hashlib.md5(buf[p:p + 4 + bsz]).hexdigest())
        p += 4 + bsz
    return hashlib.md5(buf[16:end]).hexdigest(), each


if __name__ == "__main__":
    import bench
    from fqzcomp5_amd import synth
    wd = sys.argv[1] if len(sys.argv) > 1 else "/tmp/l5n"
    os.makedirs(wd, exist_ok=True)
    src, out = os.path.join(wd, "novaseq.fastq"), os.path.join(wd, "novaseq.fqz5")
    reads = bench.make_reads(GB, SEED, KIND)
    n = synth.write_fastq(reads, src)
    nblk = len(synth.split_blocks(reads, BLK))
    del reads
    t0 = time.time()
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "fqzcomp5"), "-5", "-t1", "-b",
                    str(BLK), src, out], check=True)
    secs = time.time() - t0
    all_md5, each = block_md5s(out)
    assert len(each) == nblk, (len(each), nblk)
    rec = dict(gb=GB, seed=SEED, kind=KIND, block_size=BLK, in_bytes=n, in_md5=md5(src),
               out_bytes=os.path.getsize(out), out_md5=md5(out), blocks=len(each),
               blocks_md5=all_md5, block_md5s=each, level=5, ref_seconds=round(secs, 1),
               cmd=f"oracle/_ref/fqzcomp5 -5 -t1 -b {BLK} novaseq.fastq novaseq.fqz5")
    json.dump(rec, open(os.path.join(ROOT, "tests", "golden", "l5_novaseq.json"), "w"), indent=1)
    print({k: v for k, v in rec.items() if k != "block_md5s"})
