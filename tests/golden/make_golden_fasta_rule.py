"""Reference bytes for load_seqs_kseq's per-block FASTA rule (VERDICT r03
item 4): a block whose first record has no quality (in FASTQ text, an empty
sequence) is coded without a quality section (fqzcomp5.c:574-578, :805-809,
:2237-2264) and decodes to FASTA text (:2477-2483, :3833).  Cases: a tiny
file, a multi-block file (-b 1M) whose second and fourth blocks start with an
empty record, and a pair of files whose second block starts with one.  The
CLI as shipped (oracle/_ref/fqzcomp5 -t1) records the .fqz5 and decoded md5s
in fasta_rule.json; the inputs are rebuilt from make_inputs() on the GPU box.
python tests/golden/make_golden_fasta_rule.py"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref", "fqzcomp5")
BLK = 1_000_000
TINY = b"@r1\n\n+\n\n@r2\nACGT\n+\nIIII\n@r3\nGG\n+\n#I\n"


def _records(n: int, seed: int, tag: bytes):
    """(name, seq, qual) of n Illumina-like records (150 bp, 8 levels)."""
    rng = np.random.default_rng(seed)
    lv = np.frombuffer(b"#',7<AFJ", np.uint8)
    out = []
    for i in range(n):
        L = 150
        s = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)].tobytes()
        q = lv[np.clip(7 - rng.geometric(0.5, L) + 1, 0, 7)].tobytes()
        out.append((b"%s:%d" % (tag, i), s, q))
    return out


def _starts(recs, blk: int, pair=None):
    """Record indices that start a block (load_seqs_kseq / _interleaved)."""
    size = lambda r: len(r[0]) + 1 + len(r[1]) + len(r[2])
    out, tot = [0], 0
    for i, r in enumerate(recs):
        rs = size(r) + (size(pair[i]) if pair else 0)
        if tot > 0 and tot + rs > blk:
            out.append(i)
            tot = 0
        tot += rs
    return out


def _fastq(recs) -> bytes:
    return b"".join(b"@%s\n%s\n+\n%s\n" % r for r in recs)


def _empty_at(recs, idx):
    """Empty the sequences of records idx, their names grown by the bases
    taken out so the block split stays where it was."""
    for i in idx:
        n, s, q = recs[i]
        recs[i] = (n + b"_" * (len(s) + len(q)), b"", b"")


def make_inputs() -> dict:
    """name -> list of input texts (one, or R1 and R2)."""
    multi = _records(22000, 7, b"m")
    st = _starts(multi, BLK)
    _empty_at(multi, [st[1], st[2]])
    assert _starts(multi, BLK) == st and len(st) >= 4
    r1, r2 = _records(7000, 8, b"p/1"), _records(7000, 9, b"p/2")
    sp = _starts(r1, BLK, r2)
    _empty_at(r1, [sp[1]])
    assert _starts(r1, BLK, r2) == sp
    return {"tiny": [TINY], "multi": [_fastq(multi)], "pair": [_fastq(r1), _fastq(r2)]}


CASES = [("tiny", 1), ("tiny", 3), ("tiny", 5), ("multi", 3), ("multi", 5), ("pair", 3)]


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


if __name__ == "__main__":
    ins = make_inputs()
    out = []
    with tempfile.TemporaryDirectory() as wd:
        for name, level in CASES:
            srcs = []
            for k, t in enumerate(ins[name]):
                p = os.path.join(wd, f"{name}{k}.fq")
                open(p, "wb").write(t)
                srcs.append(p)
            z = os.path.join(wd, "o.fqz5")
            subprocess.run([REF, f"-{level}", "-t1", "-b", "1M", *srcs, z], check=True,
                           capture_output=True)
            zb = open(z, "rb").read()
            dec = [os.path.join(wd, f"d{k}") for k in range(len(srcs))]
            subprocess.run([REF, "-d", "-t1", z, *dec], check=True, capture_output=True)
            out.append(dict(case=name, level=level, in_md5=[md5(t) for t in ins[name]],
                            fqz5_md5=md5(zb), fqz5_bytes=len(zb),
                            dec_md5=[md5(open(d, "rb").read()) for d in dec],
                            dec_bytes=[os.path.getsize(d) for d in dec]))
            print(out[-1])
    json.dump(out, open(os.path.join(HERE, "fasta_rule.json"), "w"), indent=1)
