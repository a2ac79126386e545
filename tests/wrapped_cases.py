"""Wrapped (multi-line) FASTQ inputs for the kseq_read parity tests
(kseq.h:194-216: sequence lines up to '+', quality lines until their bytes
reach the sequence's length).  Deterministic: tests/golden/make_wrapped.py
codes them with the reference CLI and stores the md5s.

Cases:
  illumina70    the synthetic Illumina reads (fqzcomp5_amd.synth, seed 21)
                with sequence and quality lines wrapped at 70 columns;
                several 1 MB blocks at -b 1M
  mixed         hand-made records: wrap widths 1..200, quality lines that
                start with '@' and '+', empty sequences (3-line records),
                single-line records among wrapped ones, empty lines inside
                the sequence and quality blocks, CRLF line ends, no final
                newline
"""
import numpy as np

from fqzcomp5_amd import synth


def wrap(b: bytes, width: int, nl: bytes = b"\n") -> bytes:
    if not b:
        return nl
    return b"".join(b[i:i + width] + nl for i in range(0, len(b), width))


def illumina70() -> bytes:
    r = synth.illumina(9000, seed=21, with_names=True)
    text = synth.fastq_chunk(r, 0, r.num_records).tobytes()
    lines = text.split(b"\n")
    out = []
    for i in range(0, len(lines) - 3, 4):
        h, s, _, q = lines[i:i + 4]
        out.append(h + b"\n" + wrap(s, 70) + b"+\n" + wrap(q, 70))
    return b"".join(out)


def mixed() -> bytes:
    rng = np.random.default_rng(77)
    out = []
    for r in range(600):
        n = int(rng.choice([0, 1, 2, 63, 64, 65, 150, 151, 300, 1000]))
        if r == 0:          # (a block whose first record has no bases is FASTA, :575-578)
            n = 150
        seq = bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), n))
        # qualities from '!'..'J' with '@' and '+' common, so that quality
        # lines start with them
        qual = bytes(rng.choice(np.frombuffer(b"@+@+!#5?ABCDEFGHIJ", np.uint8), n))
        # (CRLF records: no empty lines, no empty sequence: kseq keeps the
        # '\r' of a lone-'\r' line that starts a block, kseq.h:141, which
        # fqz5_fastq_index_any refuses)
        crlf = r % 7 == 3 and n > 0
        nl = b"\r\n" if crlf else b"\n"
        w = int(rng.choice([1, 7, 60, 70, 80, 200, 10_000]))
        head = b"@r%d" % r + (b" c%d" % (r * 3) if r % 3 == 0 else b"") + nl
        sq = wrap(seq, w, nl)
        qq = wrap(qual, w, nl)
        if r % 11 == 5 and n > 2 and not crlf:   # empty lines inside both blocks
            sq = nl + sq
            cut = qq.index(nl) + len(nl)
            qq = qq[:cut] + nl + qq[cut:]
        plus = b"+" + (b"r%d" % r if r % 5 == 0 else b"") + nl
        out.append(head + sq + plus + qq)
    text = b"".join(out)
    return text[:-1] if text.endswith(b"\n") and not text.endswith(b"\r\n") else text


CASES = {"illumina70": illumina70, "mixed": mixed}
