"""Seeded synthetic FASTQ generator.

The reference ships no large inputs, so every benchmark and large parity
case is generated here from a seed.  The shapes follow SURVEY.md §8(d) d2:

* ``illumina``  (config C2): 150 bp, Illumina-style names, uniform ACGT with
  1 % of reads carrying one ``N``; qualities are a clipped random walk over
  Q2..Q41 binned to the 8 Illumina levels {2,6,15,22,27,33,37,40}.
* ``q40walk``   : as ``illumina`` but the walk is left un-binned (~40 levels).
* ``novaseq``   (config C3): qualities i.i.d. from {2,12,23,37} with
  p = {.01,.04,.10,.85}.
* ``ont``       (config C4): Oxford Nanopore-like long reads: log-normal
  lengths with N50 ~ 20 kb, homopolymer-rich sequence, qualities Q3..Q30 as
  an AR(1) walk around a per-read mean near Q12.
* ``hifi``      (config C5): PacBio HiFi-like pairs, interleaved R1/R2 (names
  ending /1 and /2, so the second of each pair carries FQZ_FREAD2 by the
  reference's rule, fqzcomp5.c:518-526); lengths ~ N(15 kb, 3 kb); over half
  of the qualities are '~' (Q93), so fqz's HiFi table applies
  (fqzcomp_qual.c:919-938).

Records are returned in the reference's in-memory SoA layout
(``fastq`` struct, fqzcomp5.c:235-249): concatenated sequence bytes,
concatenated quality bytes stored as ``q-33``... except that here the
qualities are returned as *raw phred values* (already ``q-33``, exactly what
``load_seqs_kseq`` stores at fqzcomp5.c:564), per-record lengths and flags.
Block splitting follows ``load_seqs_kseq`` (fqzcomp5.c:471-477): a record of
``name.l + 1 + seq.l + qual.l`` bytes starts a new block when it would push
a non-empty block past ``blk_size``.
"""
from __future__ import annotations

import dataclasses
import numpy as np

ILLUMINA_BINS = np.array([2, 6, 15, 22, 27, 33, 37, 40], dtype=np.uint8)


COMMENT = b" 1:N:0:ACGTACGT"      # the comment every synthetic name carries


def _illumina_bin(q: np.ndarray) -> np.ndarray:
    # Illumina 8-level binning: 2-9 -> 6, 10-19 -> 15, 20-24 -> 22,
    # 25-29 -> 27, 30-34 -> 33, 35-39 -> 37, >=40 -> 40; <2 -> 2.
    edges = np.array([2, 10, 20, 25, 30, 35, 40], dtype=np.int16)
    idx = np.searchsorted(edges, q.astype(np.int16), side="right")
    return ILLUMINA_BINS[idx]


@dataclasses.dataclass
class Reads:
    """One set of records in the reference's SoA layout."""
    seq: np.ndarray        # uint8, concatenated bases
    qual: np.ndarray       # uint8, concatenated phred values (q-33)
    lens: np.ndarray       # uint32 per record
    names: list | None     # list[bytes] without '@' (name + ' ' + comment)
    name_l: np.ndarray     # int32: kseq name.l (name part before the space)
    flags: np.ndarray | None = None   # uint32 per record (FQZ_FREAD2), None = all 0
    comment_l: int = 15    # bytes of ' ' + comment per name (0: no comment)
    name_buf: np.ndarray | None = None   # uint8: every name, '\0' after each
    name_off: np.ndarray | None = None   # int64 [n + 1]: offsets into name_buf

    @property
    def num_records(self) -> int:
        return int(self.lens.shape[0])

    @property
    def fixed_len(self) -> int:
        if self.num_records == 0:
            return 0
        l0 = int(self.lens[0])
        return l0 if bool(np.all(self.lens == l0)) else 0

    def has_names(self) -> bool:
        return self.names is not None or self.name_buf is not None

    def name(self, i: int) -> bytes:
        if self.names is not None:
            return self.names[i]
        return self.name_buf[self.name_off[i]:self.name_off[i + 1] - 1].tobytes()

    def to_fastq(self) -> bytes:
        assert self.has_names()
        out = []
        off = 0
        for i, ln in enumerate(self.lens.tolist()):
            s = self.seq[off:off + ln].tobytes()
            q = (self.qual[off:off + ln] + 33).astype(np.uint8).tobytes()
            out.append(b"@" + self.name(i) + b"\n" + s + b"\n+\n" + q + b"\n")
            off += ln
        return b"".join(out)


def _digits(v: np.ndarray, width: int) -> tuple[np.ndarray, np.ndarray]:
    """Decimal digits of v (< 10**width) right-aligned in `width` columns,
    and the mask of the significant ones."""
    cols = np.empty((v.shape[0], width), np.uint8)
    t = v.astype(np.int64).copy()
    for c in range(width - 1, -1, -1):
        cols[:, c] = (t % 10 + 48).astype(np.uint8)
        t //= 10
    nd = np.floor(np.log10(np.maximum(v, 1))).astype(np.int64) + 1
    mask = np.arange(width)[None, :] >= (width - nd)[:, None]
    return cols, mask


def _names_buf(lane, tile, x, y) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The names 'A00123:45:HXXXXXXX:lane:tile:x:y 1:N:0:ACGTACGT', '\0'
    after each, built column-wise: (buffer, offsets [n + 1], name.l)."""
    n = lane.shape[0]
    parts, masks = [], []

    def lit(b):
        parts.append(np.broadcast_to(np.frombuffer(b, np.uint8), (n, len(b))))
        masks.append(np.ones((n, len(b)), bool))
    lit(b"A00123:45:HXXXXXXX:")
    for i, (v, w) in enumerate(((lane, 1), (tile, 4), (x, 5), (y, 5))):
        c, m = _digits(v, w)
        parts.append(c)
        masks.append(m)
        if i < 3:
            lit(b":")
    lit(COMMENT + b"\0")
    rows = np.concatenate(parts, 1)
    mask = np.concatenate(masks, 1)
    buf = rows[mask]
    per = mask.sum(1).astype(np.int64)
    off = np.zeros(n + 1, np.int64)
    np.cumsum(per, out=off[1:])
    name_l = (per - 1 - len(COMMENT)).astype(np.int32)
    return np.ascontiguousarray(buf), off, name_l


def _names(rng: np.random.Generator, n: int, as_list: bool):
    lane = rng.integers(1, 5, n)
    tile = rng.integers(1101, 2679, n)
    x = np.sort(rng.integers(1000, 32000, n))
    y = rng.integers(1000, 40000, n)
    buf, off, name_l = _names_buf(lane, tile, x, y)
    names = None
    if as_list:
        names = [b"A00123:45:HXXXXXXX:%d:%d:%d:%d 1:N:0:ACGTACGT" % t
                 for t in zip(lane.tolist(), tile.tolist(), x.tolist(), y.tolist())]
    return names, name_l, buf, off


def illumina(n_reads: int, seed: int = 1, read_len: int = 150,
             binned: bool = True, with_names: bool = False) -> Reads:
    rng = np.random.default_rng(seed)
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[
        rng.integers(0, 4, n_reads * read_len, dtype=np.uint8)].copy()
    has_n = np.nonzero(rng.random(n_reads) < 0.01)[0]
    seq[has_n * read_len + rng.integers(0, read_len, has_n.shape[0])] = ord("N")

    start = rng.integers(30, 42, (n_reads, 1)).astype(np.int16)
    steps = rng.choice(np.array([-3, -1, 0, 0, 0, 0, 1, 2], dtype=np.int16),
                       size=(n_reads, read_len))
    steps[:, 0] = 0
    q = np.clip(start + np.cumsum(steps, axis=1), 2, 41)
    # quality tails off towards the 3' end, like a real run
    q = np.clip(q - (np.arange(read_len) // 30)[None, :], 2, 41)
    q = q.reshape(-1)
    qual = _illumina_bin(q) if binned else q.astype(np.uint8)
    lens = np.full(n_reads, read_len, dtype=np.uint32)
    names, name_l, nbuf, noff = _names(rng, n_reads, with_names)
    return Reads(seq, qual.astype(np.uint8), lens, names, name_l, name_buf=nbuf, name_off=noff)


def novaseq(n_reads: int, seed: int = 2, read_len: int = 150,
            with_names: bool = False) -> Reads:
    rng = np.random.default_rng(seed)
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[
        rng.integers(0, 4, n_reads * read_len, dtype=np.uint8)].copy()
    levels = np.array([2, 12, 23, 37], dtype=np.uint8)
    qual = levels[rng.choice(4, size=n_reads * read_len,
                             p=[.01, .04, .10, .85])]
    lens = np.full(n_reads, read_len, dtype=np.uint32)
    names, name_l, nbuf, noff = _names(rng, n_reads, with_names)
    return Reads(seq, qual, lens, names, name_l, name_buf=nbuf, name_off=noff)




def fastq_size(r: Reads, a: int = 0, b: int | None = None) -> int:
    """Bytes of the FASTQ text of records [a, b) as to_fastq writes it:
    '@' name [' ' comment] '\\n' seq '\\n' '+\\n' qual '\\n'."""
    b = r.num_records if b is None else b
    return int((r.name_l[a:b].astype(np.int64) + r.comment_l + 6).sum()
               + 2 * r.lens[a:b].astype(np.int64).sum())


def split_blocks(r: Reads, blk_size: int) -> list[tuple[int, int]]:
    """Record ranges [a, b) per block, by the load_seqs_kseq rule
    (fqzcomp5.c:471-477): ``record_size = name.l + 1 + seq.l + qual.l``."""
    rec = (r.name_l.astype(np.int64) + 1 + 2 * r.lens.astype(np.int64))
    out, a, tot = [], 0, 0
    csum = np.cumsum(rec)
    n = r.num_records
    while a < n:
        base = csum[a - 1] if a else 0
        # first index b>a with csum[b]-base > blk_size (record b overflows)
        b = int(np.searchsorted(csum, base + blk_size, side="right"))
        b = max(b, a + 1)
        out.append((a, b))
        a = b
    del tot
    return out


def block(r: Reads, a: int, b: int) -> Reads:
    offs = np.concatenate([[0], np.cumsum(r.lens.astype(np.int64))])
    s, e = int(offs[a]), int(offs[b])
    nb = no = None
    if r.name_buf is not None:
        nb = r.name_buf[r.name_off[a]:r.name_off[b]]
        no = r.name_off[a:b + 1] - r.name_off[a]
    return Reads(r.seq[s:e], r.qual[s:e], r.lens[a:b],
                 r.names[a:b] if r.names is not None else None,
                 r.name_l[a:b], None if r.flags is None else r.flags[a:b], r.comment_l,
                 nb, no)


def fastq_chunk(r: Reads, a: int, b: int, names=None) -> np.ndarray:
    """FASTQ text of records [a, b) as to_fastq writes it, built with
    vectorised scatters: '@' name '\\n' seq '\\n+\\n' qual+33 '\\n'."""
    buf, off = names if names is not None else all_names(r)
    n = b - a
    nl = (off[a + 1:b + 1] - off[a:b] - 1).astype(np.int64)
    L = r.lens[a:b].astype(np.int64)
    rec = nl + 2 * L + 6
    start = np.zeros(n + 1, np.int64)
    np.cumsum(rec, out=start[1:])
    out = np.empty(int(start[-1]), np.uint8)
    st = start[:-1]
    out[st] = ord("@")

    def scatter(src, lengths, base):
        tot = int(lengths.sum())
        if not tot:
            return
        ri = np.repeat(np.arange(n), lengths)
        first = np.zeros(n, np.int64)
        np.cumsum(lengths[:-1], out=first[1:])
        within = np.arange(tot, dtype=np.int64) - first[ri]
        out[base[ri] + within] = src
    nb = buf[off[a]:off[b]]
    scatter(nb[nb != 0], nl, st + 1)
    out[st + 1 + nl] = ord("\n")
    boff = np.concatenate([[0], np.cumsum(r.lens.astype(np.int64))])
    s, e = int(boff[a]), int(boff[b])
    scatter(r.seq[s:e], L, st + nl + 2)
    q0 = st + nl + 2 + L
    out[q0] = ord("\n")
    out[q0 + 1] = ord("+")
    out[q0 + 2] = ord("\n")
    scatter((r.qual[s:e] + 33).astype(np.uint8), L, q0 + 3)
    out[st + rec - 1] = ord("\n")
    return out


def write_fastq(r: Reads, path: str, chunk: int = 200_000) -> int:
    """Write the reads as FASTQ text (to_fastq's bytes) in chunks; returns
    the bytes written."""
    names = all_names(r)
    tot = 0
    with open(path, "wb") as f:
        for a in range(0, r.num_records, chunk):
            c = fastq_chunk(r, a, min(a + chunk, r.num_records), names)
            f.write(c.tobytes())
            tot += c.shape[0]
    return tot


def all_names(r: Reads) -> tuple[np.ndarray, np.ndarray]:
    """(buffer, offsets [n + 1]) of every name, '\0' after each: the name
    section input of load_seqs_kseq (name [' ' comment] '\0')."""
    if r.name_buf is not None:
        return r.name_buf, r.name_off
    assert r.names is not None
    buf = np.frombuffer(b"".join(nm + b"\0" for nm in r.names), np.uint8).copy()
    off = np.zeros(r.num_records + 1, np.int64)
    np.cumsum([len(nm) + 1 for nm in r.names], out=off[1:])
    return buf, off


def _homopolymer_seq(rng: np.random.Generator, n: int) -> np.ndarray:
    """ACGT with geometric homopolymer runs (mean ~1.8 bases)."""
    out = np.empty(0, np.uint8)
    parts, got = [], 0
    while got < n:
        m = max(1024, (n - got) // 2 + 64)
        runs = rng.geometric(0.55, m)
        step = rng.integers(1, 4, m)                  # next base differs
        base = np.cumsum(step) % 4
        parts.append(np.repeat(base.astype(np.uint8), runs))
        got += int(runs.sum())
    out = np.concatenate(parts)[:n]
    return np.frombuffer(b"ACGT", dtype=np.uint8)[out]


def ont(n_reads: int, seed: int = 3, with_names: bool = False, median: float = 10500.0,
        sigma: float = 0.8) -> Reads:
    rng = np.random.default_rng(seed)
    lens = np.clip(rng.lognormal(np.log(median), sigma, n_reads), 200, 400000).astype(np.uint32)
    tot = int(lens.sum())
    seq = _homopolymer_seq(rng, tot)
    # qualities: an AR(1) walk (phi 0.8) around a per-read mean near Q12,
    # clipped to Q3..Q30 (one filter over the whole run of records)
    from scipy.signal import lfilter
    mu = np.repeat(np.clip(rng.normal(12.0, 2.5, n_reads), 6, 20), lens)
    d = lfilter([1.0], [1.0, -0.8], rng.normal(0.0, 2.8, tot))
    q = np.clip(np.rint(mu + d), 3, 30).astype(np.uint8)
    ids = rng.integers(0, 1 << 62, (n_reads, 2))
    names = None
    if with_names:                                # read ids, no comment
        names = [b"%016x-%016x" % (int(a), int(b)) for a, b in ids.tolist()]
    return Reads(seq, q, lens, names, np.full(n_reads, 33, np.int32), None, 0)


def hifi(n_pairs: int, seed: int = 5, with_names: bool = False) -> Reads:
    rng = np.random.default_rng(seed)
    n = 2 * n_pairs
    lens = np.clip(np.rint(rng.normal(15000.0, 3000.0, n)), 3000, 40000).astype(np.uint32)
    tot = int(lens.sum())
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, tot, dtype=np.uint8)].copy()
    q = np.where(rng.random(tot) < 0.62, 93, rng.integers(10, 60, tot)).astype(np.uint8)
    flags = np.tile(np.array([0, 128], np.uint32), n_pairs)        # FQZ_FREAD2 on /2
    zmw = np.sort(rng.integers(1, 1 << 24, n_pairs))
    if with_names:
        names = [b"m84011_220902_175841_s1/%d/ccs/%d" % (int(z), k)
                 for z in zmw.tolist() for k in (1, 2)]
        name_l = np.array([len(nm) for nm in names], dtype=np.int32)
    else:
        names = None
        name_l = np.repeat((len(b"m84011_220902_175841_s1//ccs/1")
                            + np.floor(np.log10(zmw)).astype(np.int32) + 1), 2).astype(np.int32)
    return Reads(seq, q, lens, names, name_l, flags, 0)
