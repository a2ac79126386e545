"""Wrapped (multi-line) FASTQ inputs for the kseq_read parity tests
(kseq.h:194-216: sequence lines up to '+', quality lines until their bytes
reach the sequence's length).  Deterministic: tests/golden/make_wrapped.py
codes them with the reference CLI and stores the md5s.

Cases:
  junk          4-line and wrapped records with lines kseq skips before,
                between and after them (round 6)
  lonecr        lone '\r' lines that kseq keeps as the first byte of a
                sequence or quality block, and ones it drops (round 6)
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


def junk() -> bytes:
    """kseq's skip to the next header (kseq.h:180-186): lines before the
    first record, between records and after the last that hold neither '@'
    nor '>' (text, '+' lines, empty lines, lone '\r' and CRLF lines), among
    4-line and 70-column wrapped records; two 1 MB blocks at -b 1M."""
    r = synth.illumina(4200, seed=23, with_names=True)
    text = synth.fastq_chunk(r, 0, r.num_records).tobytes()
    lines = text.split(b"\n")
    junks = [b"junk between records\n", b"+ a plus line\n", b"\n\n", b"\r\n", b"x y z\r\n",
             b"+\n", b"0123456789\n"]
    out = [b"# a first line that is no header\nmore text\n\n"]
    for n, i in enumerate(range(0, len(lines) - 3, 4)):
        h, sq, _, q = lines[i:i + 4]
        if n % 3 == 1:
            out.append(h + b"\n" + wrap(sq, 70) + b"+\n" + wrap(q, 70))
        else:
            out.append(h + b"\n" + sq + b"\n+\n" + q + b"\n")
        if n % 5 == 2:
            out.append(junks[(n // 5) % len(junks)])
    out.append(b"trailing text\n")
    return b"".join(out)


def lonecr() -> bytes:
    """A lone '\r' line before the first kept byte of a sequence or quality
    block: kseq keeps that '\r' (its strip of a trailing '\r' needs two bytes
    in the string, kseq.h:141), later ones it drops; with empty lines before
    it, in CRLF records, as the whole sequence or quality."""
    rng = np.random.default_rng(29)
    out = []
    for r in range(900):
        n = int(rng.choice([1, 2, 5, 70, 71, 150]))
        seq = bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), n))
        qual = bytes(rng.choice(np.frombuffer(b"#,:FIJ", np.uint8), n))
        kind = r % 6
        crlf = r % 4 == 3
        nl = b"\r\n" if crlf else b"\n"
        head = b"@cr%d" % r + nl
        if kind == 0:        # both blocks start with the kept '\r'
            sq, qq = b"\r\n" + wrap(seq[1:], 60, nl), b"\r\n" + wrap(qual[1:], 60, nl)
        elif kind == 1:      # the qualities only
            sq, qq = wrap(seq, 60, nl), b"\r\n" + wrap(qual[1:], 60, nl)
        elif kind == 2:      # the bases only, empty lines before it
            sq, qq = b"\n\n\r\n" + wrap(seq[1:], 60, nl), wrap(qual, 60, nl)
        elif kind == 3:      # a second lone '\r' line is dropped
            sq, qq = b"\r\n\r\n" + wrap(seq[1:], 60, nl), b"\n\r\n\r\n" + wrap(qual[1:], 60, nl)
        elif kind == 4:      # no '\r'
            sq, qq = wrap(seq, 60, nl), wrap(qual, 60, nl)
        else:                # a lone '\r' after the first bases is dropped
            sq, qq = wrap(seq, 60, nl) + b"\r\n", wrap(qual, 60, nl) + b"\r\n"
        if n == 1 and kind in (0, 3):        # the '\r' is the whole block
            sq, qq = b"\r\n", b"\r\n"
        out.append(head + sq + b"+" + nl + qq)
    return b"".join(out)


CASES = {"illumina70": illumina70, "mixed": mixed, "junk": junk, "lonecr": lonecr}
