"""Seeded inputs of the sequence context model tests (fqzcomp5.c:1073-1406):
record-structured base strings with the cases the coder distinguishes —
uppercase / lowercase / literal runs and their switches, runs of 255 and
more, record resets, a zero-length record (after which the reference sees
no more record boundaries), an empty block, a block starting with a literal,
and repeated reads (k-mer contexts that recur)."""
import numpy as np

# (method name, k, both strands) of SEQ10, SEQ12, SEQ12B, SEQ13B
# (fqzcomp5.c:2047-2062); SEQ14B needs a 1 GB model table per call and is
# covered by one case below.
METHODS = [("SEQ10", 10, 0), ("SEQ12", 12, 0), ("SEQ12B", 12, 1), ("SEQ13B", 13, 1)]


def _reads(rng, nrec, rlen, genome_len=200_000):
    g = rng.choice(np.frombuffer(b"ACGT", np.uint8), genome_len)
    st = rng.integers(0, genome_len - rlen, nrec)
    reads = [g[s:s + rlen].copy() for s in st]
    for r in reads[::2]:          # reverse complements
        r[:] = np.frombuffer(bytes(r[::-1]).translate(bytes.maketrans(b"ACGT", b"TGCA")), np.uint8)
    return reads


def cases():
    rng = np.random.default_rng(11)
    out = []
    # illumina-like: fixed 150 bp, rare N
    reads = _reads(rng, 800, 150)
    for r in reads[::37]:
        r[rng.integers(0, 150)] = ord("N")
    out.append(("illumina", b"".join(bytes(r) for r in reads), [150] * len(reads)))
    # variable lengths, lowercase stretches, IUPAC codes, long runs
    rng2 = np.random.default_rng(12)
    recs = []
    for i in range(300):
        L = int(rng2.integers(1, 400))
        r = bytearray(rng2.choice(np.frombuffer(b"ACGT", np.uint8), L).tobytes())
        if i % 5 == 0:
            a = int(rng2.integers(0, L))
            r[a:a + 40] = r[a:a + 40].lower()
        if i % 7 == 0:
            a = int(rng2.integers(0, L))
            r[a:a + 3] = b"NRY"[: len(r[a:a + 3])]
        if i % 50 == 3:
            r += b"N" * 600           # literal run of more than 255
        if i % 60 == 1:
            r += b"a" * 510           # lowercase run of exactly 2 x 255
        recs.append(bytes(r))
    out.append(("mixed", b"".join(recs), [len(r) for r in recs]))
    # starts with a literal, then lowercase first
    out.append(("lead_n", b"NNACGTacgtNNNNacgtACGT" * 20, [22] * 20))
    out.append(("lead_lc", b"acgtACGT" * 50, [40] * 10))
    # a zero-length record in the middle: no boundary after it
    s = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 1000).tobytes())
    out.append(("zero_len", s, [100, 100, 0, 300, 500]))
    out.append(("single", b"G", [1]))
    out.append(("empty", b"", [0]))
    return out
