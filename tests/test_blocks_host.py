"""Host-side block framing of the library on the CPU (no GPU call): the
lengths section (fqz5_block_lengths, fqzcomp5.c:2189-2214), the READ2 flags
(fqz5_name_flags, :518-527), the block split (fqz5_fastq_blocks, :471-479)
against plain Python restatements and the reference CLI's own files, and the
container framing of fqz5file.py (:2563-2630, :2959-2969)."""
import ctypes as C
import os
import struct
import subprocess

import numpy as np
import pytest

import fqz5_container as F
from fqzcomp5_amd import fqz5file, sections as S, synth
from oracle import binding

CLI = os.path.join(os.path.dirname(binding.REF_BIN), "fqzcomp5")


def _varint(v):                       # htscodecs var_put_u32 (varint.h:206)
    out = [v & 0x7f]
    v >>= 7
    while v:
        out.append(0x80 | (v & 0x7f))
        v >>= 7
    return bytes(reversed(out))


def _lengths_py(lens, fixed):
    if fixed:
        v = _varint(fixed & 0xffffffff)
        return bytes([len(v)]) + v
    body = b"".join(_varint(int(x)) for x in lens)
    return b"\0" + struct.pack("<I", len(body)) + body


def _flags_py(names):
    out, last = [], None
    for nm in names:
        f = 0
        name_l = nm.find(b" ") if b" " in nm else len(nm)
        if name_l > 1 and len(nm) >= 2 and nm[-2:] == b"/2":
            f = 128
        if last is not None and nm == last:
            f = 128
        out.append(f)
        last = nm
    return out


def test_lengths_section():
    rng = np.random.default_rng(5)
    for n in (1, 2, 17, 1000):
        lens = rng.integers(0, 300000, n).astype(np.uint32)
        assert S.block_lengths(lens, 0) == _lengths_py(lens, 0)
        assert S.block_lengths(lens[:1], 150) == _lengths_py(lens[:1], 150)
    assert S.block_lengths(np.zeros(0, np.uint32), -1) == _lengths_py([], -1)


def test_name_flags():
    names = [b"r1/1", b"r1/2", b"r1/2", b"x y/2", b"a", b"a", b"/2", b"q/2 c", b"q/2 c"]
    buf = np.frombuffer(b"".join(n + b"\0" for n in names), np.uint8)
    assert S.name_flags(buf, len(names)).tolist() == _flags_py(names)


def test_block_split_matches_synth():
    so = fqz5file._load()
    r = synth.ont(400, seed=9, with_names=True)
    rs = (r.name_l.astype(np.int64) + 1 + 2 * r.lens.astype(np.int64)).astype(np.uint32)
    for blk in (1_000_000, 3_000_000, 10**9):
        first = np.zeros(len(rs) + 2, np.uint64)
        nb = so.fqz5_fastq_blocks(rs.ctypes.data, len(rs), blk, first.ctypes.data, len(rs) + 1)
        got = [(int(first[k]), int(first[k + 1])) for k in range(nb)]
        assert got == synth.split_blocks(r, blk)


@pytest.mark.skipif(not os.path.exists(CLI), reason="oracle/_ref not built")
def test_container_framing_vs_cli(tmp_path):
    r = synth.illumina(20000, seed=3, with_names=True)
    src, out = str(tmp_path / "in.fastq"), str(tmp_path / "o.fqz5")
    synth.write_fastq(r, src)
    subprocess.run([CLI, "-3", "-t1", "-b", "1M", src, out], check=True, capture_output=True)
    data = open(out, "rb").read()
    blocks = F.raw_blocks(out)
    assert len(blocks) > 3
    ranges = fqz5file._blocks_of(data)
    assert [data[a:b] for a, b in ranges] == blocks
    bases, nrec = [], []
    for b in blocks:
        (n,) = struct.unpack_from("<I", b, 4)
        nrec.append(n)
    for a, b in synth.split_blocks(r, 1_000_000):
        bases.append(int(r.lens[a:b].sum()))
    assert fqz5file.container(blocks, bases, nrec) == data


def _pair_split_py(s1, s2, blk):
    """load_seqs_interleaved's rule (fqzcomp5.c:703-711): a pair that would
    take a non-empty block past blk starts the next one."""
    out, a, tot = [], 0, 0
    for k in range(len(s1)):
        rs = int(s1[k]) + int(s2[k])
        if tot > 0 and tot + rs > blk:
            out.append((2 * a, 2 * k))
            a, tot = k, 0
        tot += rs
    if len(s1):
        out.append((2 * a, 2 * len(s1)))
    return out


@pytest.mark.skipif(not os.path.exists(CLI), reason="oracle/_ref not built")
def test_pair_split_vs_cli(tmp_path):
    """The paired block split fqz5file.parse_paired uses (pair sizes through
    fqz5_fastq_blocks, record indices doubled) against the restated rule and
    against the records per block in the reference CLI's index for two files."""
    so = fqz5file._load()
    r = synth.illumina(12000, seed=5, with_names=True)
    text = synth.fastq_chunk(r, 0, r.num_records).tobytes().split(b"\n")
    recs = [b"\n".join(text[k:k + 4]) + b"\n" for k in range(0, len(text) - 1, 4)]
    r1, r2 = recs[0::2], recs[1::2]
    size = lambda rec: len(rec.split(b"\n")[0].split(b" ")[0]) + len(rec.split(b"\n")[1]) * 2
    s1 = np.array([size(x) for x in r1], np.uint32)      # name.l + 1 + seq.l + qual.l
    s2 = np.array([size(x) for x in r2], np.uint32)
    blk = 1_000_000
    first = fqz5file._blocks(so, (s1 + s2).astype(np.uint32), blk) * 2
    got = [(int(first[k]), int(first[k + 1])) for k in range(len(first) - 1)]
    assert got == _pair_split_py(s1, s2, blk) and len(got) > 1
    a, b, out = str(tmp_path / "a.fq"), str(tmp_path / "b.fq"), str(tmp_path / "o.fqz5")
    open(a, "wb").write(b"".join(r1))
    open(b, "wb").write(b"".join(r2))
    subprocess.run([CLI, "-1", "-t1", "-b", "1M", a, b, out], check=True, capture_output=True)
    data = open(out, "rb").read()
    (idx,) = struct.unpack_from("<Q", data, 8)
    (n,) = struct.unpack_from("<I", data, idx + 8)
    nrec = [struct.unpack_from("<QII", data, idx + 12 + 16 * k)[2] for k in range(n)]
    assert nrec == [e - s for s, e in got]
