"""FASTQ file <-> .fqz5 file on the GPU: the container
fqzcomp5 writes, produced and read by this library alone.

    compress_file(src, dst, level[, src2=])  FASTQ text -> HBM -> fqz5_fastq_index /
                                     blocks / gather (fastq.hip) -> the
                                     section coder with the level's trial
                                     (sections.encode_run) -> whole blocks
                                     (fqz5_blocks_assemble) -> file
    decompress_file(src, dst[, dst2=])  file -> HBM -> fqz5_block_parse ->
                                     sections decoded -> fqz5_fastq_format
                                     (_pairs: deinterleaved to two files)
    compress_paired_bytes / decompress_paired_bytes: the same for R1/R2
    pairs (encode_interleaved / decode_deinterleaved, fqzcomp5.c:3211,
    :4049): records interleaved R1, R2, R1, ... with READ2 on the R2 ones.

File layout (fqzcomp5.c:2563-2630, :2959-2969): "FQZ5\\1\\1\\0\\0", u64 index
offset, the blocks, then "FQZ5IDX\\0", u32 nblocks and per block {u64 file
offset, u32 bases, u32 records}.  Encoding follows a single-threaded (-t1)
reference run: the codec trial runs over the blocks in file order, so the
file equals the reference CLI's `-<level> -t1` output byte for byte.

Scope: 4-line FASTQ and FASTA with any line wrapping (text starting with
'>': blocks without a quality section, decoded to output_fasta's one-line
text, fqzcomp5.c:2258-2264, :3503-3517); the parser refuses multi-line FASTQ
records with an error (there is no host parse); files that fit in device
memory.
"""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np

from . import lib as _lib
from . import sections as S

MAGIC = b"FQZ5\x01\x01\x00\x00"                 # fqzcomp5.c:156
INDEX_MAGIC = b"FQZ5IDX\x00"                    # :158


class FastqRec(C.Structure):
    """fqz5_fastq_rec (include/fqz5_fastq.h)"""
    _fields_ = [("name", C.c_uint64), ("comment", C.c_uint64), ("seq", C.c_uint64),
                ("qual", C.c_uint64), ("name_len", C.c_uint32), ("comment_len", C.c_uint32),
                ("seq_len", C.c_uint32), ("fasta", C.c_uint32)]


_bound = False


def _load():
    global _bound
    so = _lib.load()
    if not _bound:
        so.fqz5_fastq_index.restype = C.c_int
        so.fqz5_fastq_index.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                        C.POINTER(C.c_uint64), C.c_void_p]
        so.fqz5_fastq_blocks.restype = C.c_int
        so.fqz5_fastq_blocks.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_int]
        so.fqz5_fastq_gather.restype = C.c_int
        so.fqz5_fastq_gather.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.POINTER(C.c_uint64)]
        so.fqz5_fastq_format.restype = C.c_int
        so.fqz5_fastq_format.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                                         C.c_uint64, C.POINTER(C.c_uint64)]
        so.fqz5_fastq_format_pairs.restype = C.c_int
        so.fqz5_fastq_format_pairs.argtypes = so.fqz5_fastq_format.argtypes + [
            C.POINTER(C.c_uint64)]
        _bound = True
    return so


def _check(rc, what):
    if rc < 0:
        raise _lib.NativeError(f"{what}: {_lib.last_error()}")
    return rc


def _index_text(text_d, at: int, n: int):
    """fqz5_fastq_index of text_d[at:at+n]: (records as bytes on the
    device, their load_seqs_kseq sizes, count, is FASTA)."""
    import torch
    so = _load()
    part = text_d[at:at + n]
    # records <= lines / 4, FASTA records <= lines (+1 for a last line
    # without '\n')
    lpr = 1 if n and int(part[0].item()) == ord(">") else 4
    max_rec = (int((part == 10).sum().item()) + 1) // lpr + 1 if n else 1
    recs = torch.empty(max_rec * C.sizeof(FastqRec), dtype=torch.uint8, device=text_d.device)
    rsz = np.zeros(max_rec, np.uint32)
    nrec = C.c_uint64(0)
    fasta = _check(so.fqz5_fastq_index(text_d.data_ptr() + at, n, recs.data_ptr(), max_rec,
                                       C.byref(nrec), rsz.ctypes.data), "fqz5_fastq_index") == 1
    nrec = int(nrec.value)
    if at and nrec:                     # offsets into the whole text
        v = recs[:nrec * C.sizeof(FastqRec)].view(torch.int64).view(nrec, -1)
        v[:, :4] += at
    return recs[:nrec * C.sizeof(FastqRec)], rsz[:nrec], nrec, fasta


def _gather(text_d, recs, first, fasta: bool, pair_flags: bool):
    """The blocks [first[k], first[k+1]) of the records as a sections.Run,
    every section input gathered in HBM.  pair_flags: READ2 on the odd
    records (load_seqs_interleaved, fqzcomp5.c:763) instead of from the names."""
    import torch
    so = _load()
    nb = len(first) - 1
    sizes = []
    for k in range(nb):
        sz = (C.c_uint64 * 3)()
        _check(so.fqz5_fastq_gather(text_d.data_ptr(), recs.data_ptr(), int(first[k]),
                                    int(first[k + 1]), None, None, None, None, None, sz),
               "fqz5_fastq_gather")
        sizes.append((int(sz[0]), int(sz[1])))
    tot_n = sum(a for a, _ in sizes)
    tot_s = sum(b for _, b in sizes)
    name_d = torch.empty(max(tot_n, 1), dtype=torch.uint8, device=text_d.device)
    seq_d = torch.empty(max(tot_s, 1), dtype=torch.uint8, device=text_d.device)
    qual_d = None if fasta else torch.empty(max(tot_s, 1), dtype=torch.uint8, device=text_d.device)
    lens, flags, nr, sr = [], [], [], []
    no = so_ = 0
    for k in range(nb):
        a, b = int(first[k]), int(first[k + 1])
        ln = np.zeros(max(b - a, 1), np.uint32)
        fl = np.zeros(max(b - a, 1), np.uint32)
        sz = (C.c_uint64 * 3)()
        _check(so.fqz5_fastq_gather(text_d.data_ptr(), recs.data_ptr(), a, b,
                                    name_d.data_ptr() + no, seq_d.data_ptr() + so_,
                                    None if fasta else qual_d.data_ptr() + so_, ln.ctypes.data,
                                    fl.ctypes.data, sz),
               "fqz5_fastq_gather")
        if pair_flags:
            fl[:] = 0
            fl[1::2] = 128                  # FQZ_FREAD2
        lens.append(ln[:b - a])
        flags.append(fl[:b - a])
        nr.append((no, no + sizes[k][0]))
        sr.append((so_, so_ + sizes[k][1]))
        no += sizes[k][0]
        so_ += sizes[k][1]
    return S.Run.from_device(name_d, seq_d, qual_d, nr, sr, lens, flags)


def _blocks(so, sizes: np.ndarray, blk_size: int) -> np.ndarray:
    n = len(sizes)
    first = np.zeros(n + 2, np.uint64)
    sz = np.ascontiguousarray(sizes, np.uint32)
    nb = _check(so.fqz5_fastq_blocks(sz.ctypes.data, n, blk_size, first.ctypes.data, n + 1),
                "fqz5_fastq_blocks")
    return first[:nb + 1]


def parse_fastq(text_d, blk_size: int):
    """FASTQ (or FASTA) text (a device uint8 tensor) -> a sections.Run of
    its blocks, every section input gathered in HBM.  FASTA blocks have no
    quality section (fqzcomp5.c:2237-2264)."""
    so = _load()
    recs, rsz, nrec, fasta = _index_text(text_d, 0, int(text_d.numel()))
    run = _gather(text_d, recs, _blocks(so, rsz, blk_size), fasta, False)
    del recs
    return run


def parse_paired(text_d, len1: int, blk_size: int):
    """Two files' text in one device buffer (R1 in [0, len1), R2 after it)
    -> the Run of their interleaved records (load_seqs_interleaved,
    fqzcomp5.c:627-848): records R1[0], R2[0], R1[1], ...; a block ends
    before the pair that would take it past blk_size; READ2 on R2 records.
    R2 ending before R1 is an error; R2 records past R1's end are not read."""
    import torch
    so = _load()
    r1, rs1, n1, fa1 = _index_text(text_d, 0, len1)
    r2, rs2, n2, fa2 = _index_text(text_d, len1, int(text_d.numel()) - len1)
    if n2 < n1:
        raise _lib.NativeError("unpaired read detected: R2 file ended before R1")
    if n1 and fa1 != fa2:
        raise _lib.NativeError("paired files: one FASTA, one FASTQ")
    w = C.sizeof(FastqRec)
    recs = torch.stack([r1.view(n1, w), r2[:n1 * w].view(n1, w)], 1).reshape(-1) if n1 else r1
    del r1, r2
    pair = rs1.astype(np.uint64) + rs2[:n1].astype(np.uint64)
    if n1 and int(pair.max()) >= 2 ** 32:
        raise _lib.NativeError("paired record larger than 4 GB")
    first = _blocks(so, pair.astype(np.uint32), blk_size) * 2
    run = _gather(text_d, recs, first, fa1, True)
    del recs
    return run


def container(blocks: list[bytes], bases: list[int], nrec: list[int]) -> bytes:
    """The file: header with the index offset, the blocks, the index
    (write_header / write_index, fqzcomp5.c:2563-2630, :2959-2969)."""
    out = [MAGIC, b"\0" * 8]
    off = 16
    idx = []
    for blk, nb, nr in zip(blocks, bases, nrec):
        idx.append(struct.pack("<QII", off, nb, nr))
        out.append(blk)
        off += len(blk)
    if blocks:
        out.append(INDEX_MAGIC + struct.pack("<I", len(blocks)) + b"".join(idx))
    out[1] = struct.pack("<Q", off)
    return b"".join(out)


def _pinned(n: int):
    import torch
    return torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True)[:n]


def _read_pinned(path: str):
    """The file's bytes in page-locked host memory (one read, no copy).  A
    gzip file (the reference reads every input through zlib's gzopen,
    fqzcomp5.c:5075-5110) is inflated on the host first: zlib's stream
    format is serial and stays host I/O; the FASTQ text is still parsed on
    the GPU only."""
    import os
    with open(path, "rb") as f:
        magic = f.read(2)
    if magic == b"\x1f\x8b":
        import gzip
        with open(path, "rb") as f:
            raw = gzip.decompress(f.read())
        buf = _pinned(len(raw))
        if raw:
            buf.numpy()[:] = np.frombuffer(raw, np.uint8)
        return buf
    n = os.path.getsize(path)
    buf = _pinned(n)
    mv = memoryview(buf.numpy())
    with open(path, "rb", buffering=0) as f:
        got = 0
        while got < n:
            k = f.readinto(mv[got:])
            if not k:
                raise OSError(f"{path}: short read")
            got += k
    return buf


def _encode(text_d, level: int, blk_size: int | None, len1: int | None = None):
    """FASTQ text in HBM -> (the Run holding the encoded blocks, bases,
    records); with len1, the paired files R1 = text_d[:len1], R2 after it."""
    blk = blk_size or S.BLOCK_SIZE[level]
    run = parse_fastq(text_d, blk) if len1 is None else parse_paired(text_d, len1, blk)
    if not run.blocks:
        return None, [], []
    res, *_ = S.encode_run(run.enc_secs(), S.masks(level, full=True), S.new_state())
    if any(r.status != 0 for r in res):
        raise _lib.NativeError("section coding failed: " + _lib.last_error())
    run.assemble(res)
    return run, [int(ln.sum()) for ln in run.lens], [len(ln) for ln in run.lens]


def _index(offs, bases, nrec) -> bytes:
    return INDEX_MAGIC + struct.pack("<I", len(offs)) + b"".join(
        struct.pack("<QII", o, nb, nr) for o, nb, nr in zip(offs, bases, nrec))


def compress_bytes(text: bytes, level: int = 3, blk_size: int | None = None,
                   device: str = "cuda") -> bytes:
    """fqzcomp5 -<level> (-t1 semantics) of FASTQ text, on the GPU."""
    import torch
    text_d = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(device) if text else \
        torch.empty(0, dtype=torch.uint8, device=device)
    run, bases, nrec = _encode(text_d, level, blk_size)
    del text_d
    if run is None:
        return container([], [], [])
    blocks = [run.block_bytes(b) for b in range(len(run.blocks))]
    return container(blocks, bases, nrec)


def compress_paired_bytes(text1: bytes, text2: bytes, level: int = 3,
                          blk_size: int | None = None, device: str = "cuda") -> bytes:
    """fqzcomp5 -<level> in1 in2 out (-t1 semantics): the two files'
    records interleaved (encode_interleaved, fqzcomp5.c:3211-3440)."""
    import torch
    both = text1 + text2
    text_d = torch.frombuffer(bytearray(both), dtype=torch.uint8).to(device) if both else \
        torch.empty(0, dtype=torch.uint8, device=device)
    run, bases, nrec = _encode(text_d, level, blk_size, len(text1))
    del text_d
    if run is None:
        return container([], [], [])
    return container([run.block_bytes(b) for b in range(len(run.blocks))], bases, nrec)


def compress_file(src: str, dst: str, level: int = 3, blk_size: int | None = None,
                  device: str = "cuda", src2: str | None = None) -> int:
    """The file path without host copies of the data: the FASTQ read into
    page-locked memory, one copy to HBM, the encoded blocks back in one copy
    and written behind the header, then the index.  src2: the R2 file of a
    pair, interleaved with src (fqzcomp5 in1 in2 out)."""
    import torch
    # a blocking copy: the library's kernels run on its own streams, which
    # do not wait for torch's (a non-blocking copy raced the FASTQ parse)
    len1 = None
    if src2 is None:
        text_d = _read_pinned(src).to(device)
    else:
        a, b = _read_pinned(src), _read_pinned(src2)
        len1 = a.numel()
        text_d = torch.empty(max(a.numel() + b.numel(), 1), dtype=torch.uint8,
                             device=device)[:a.numel() + b.numel()]
        text_d[:len1].copy_(a)
        text_d[len1:].copy_(b)
        torch.cuda.synchronize(text_d.device)
        del a, b
    run, bases, nrec = _encode(text_d, level, blk_size, len1)
    del text_d
    if run is None:
        out = container([], [], [])
        with open(dst, "wb") as f:
            f.write(out)
        return len(out)
    end = int(run.blk_off[-1])
    host = _pinned(end)
    host.copy_(run.blk_buf[:end])
    offs = [16 + int(run.blk_off[b]) for b in range(len(run.blocks))]
    idx = _index(offs, bases, nrec)
    with open(dst, "wb") as f:
        f.write(MAGIC + struct.pack("<Q", 16 + end))
        f.write(memoryview(host.numpy()))
        f.write(idx)
    return 16 + end + len(idx)


def _blocks_of(data):
    """Block byte ranges of a .fqz5 (walking block_size fields up to the
    index, fqzcomp5.c:3754-3772)."""
    data = memoryview(data).cast("B")
    if bytes(data[:8]) != MAGIC:
        raise ValueError("not an FQZ5 v1.1 file")
    (idx,) = struct.unpack_from("<Q", data, 8)
    end = idx if idx else len(data)
    p, out = 16, []
    while p < end:
        (bsz,) = struct.unpack_from("<I", data, p)
        out.append((p, p + 4 + bsz))
        p += 4 + bsz
    return out


def _decode(data, buf, plus_name: bool, device: str, pairs: bool = False):
    """Blocks of a .fqz5 (host view `data`, device copy `buf`) -> the FASTQ
    text of every block in one device buffer; pairs: (the R1 text, the R2
    text) of output_fastq_deinterleaved (fqzcomp5.c:3612-3676), even records
    of every block to R1 and odd ones to R2."""
    import torch
    so = _load()
    ranges = _blocks_of(data)
    if not ranges:
        return torch.empty(0, dtype=torch.uint8, device=device)
    views, lens = [], []
    for s, e in ranges:
        v = S.BlockView()
        (nrec,) = struct.unpack_from("<I", data, s + 4)
        ln = np.zeros(max(nrec, 1), np.uint32)
        _check(S._load_blk().fqz5_block_parse(buf.data_ptr() + s, e - s, C.byref(v),
                                              ln.ctypes.data_as(C.POINTER(C.c_uint32)), len(ln)),
               "fqz5_block_parse")
        if not v.crc_ok:
            raise _lib.NativeError("block CRC mismatch")
        views.append(v)
        lens.append(ln[:v.nrec])
    # FASTA: a quality section of u_len 0 and c_len 0 (decode_block,
    # fqzcomp5.c:2477-2483); the text is then output_fasta's (:3503-3517)
    fasta = [v.qual_ulen == 0 and v.qual_size == 9 for v in views]
    if any(fasta) and not all(fasta):
        raise _lib.NativeError("FASTA and FASTQ blocks in one file")
    nsz = [v.name_ulen for v in views]
    ssz = [v.seq_ulen for v in views]
    out_d = torch.empty(sum(nsz) + 2 * sum(ssz) + 1, dtype=torch.uint8, device=device)
    secs, places = [], []
    o = 0
    base = buf.data_ptr()
    for (s, e), v, ln in zip(ranges, views, lens):
        rl = ln.ctypes.data_as(C.POINTER(C.c_uint32))
        po = (o, o + v.name_ulen, o + v.name_ulen + v.seq_ulen)
        secs.append(S.Section(base + s + v.name_off, out_d.data_ptr() + po[0], v.name_size,
                              v.name_ulen, 0, S.SEC_NAME, rl, None, len(ln), None))
        secs.append(S.Section(base + s + v.seq_off, out_d.data_ptr() + po[1], v.seq_size,
                              v.seq_ulen, 0, S.SEC_SEQ, rl, None, len(ln), None))
        if not fasta[0]:
            secs.append(S.Section(base + s + v.qual_off, out_d.data_ptr() + po[2], v.qual_size,
                                  v.qual_ulen, 0, S.SEC_QUAL, rl, None, len(ln),
                                  out_d.data_ptr() + po[1]))
        places.append(po)
        o = po[2] + v.seq_ulen
    res = S.decode(secs)
    if any(r.status != 0 for r in res):
        raise _lib.NativeError("section decoding failed: " + _lib.last_error())
    # the text of every block, one after the other in one device buffer
    fmt = so.fqz5_fastq_format_pairs if pairs else so.fqz5_fastq_format
    args, sizes, r1 = [], [], []
    for v, ln, po in zip(views, lens, places):
        size, s1 = C.c_uint64(0), C.c_uint64(0)
        a = (out_d.data_ptr() + po[0], v.name_ulen, out_d.data_ptr() + po[1],
             None if fasta[0] else out_d.data_ptr() + po[2], ln.ctypes.data, len(ln),
             int(plus_name))
        _check(fmt(*a, None, 0, C.byref(size), *((C.byref(s1),) if pairs else ())),
               "fqz5_fastq_format")
        args.append(a)
        sizes.append(int(size.value))
        r1.append(int(s1.value))
    text = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device=device)
    at = 0
    for a, n in zip(args, sizes):
        size, s1 = C.c_uint64(0), C.c_uint64(0)
        _check(fmt(*a, text.data_ptr() + at, n, C.byref(size),
                   *((C.byref(s1),) if pairs else ())), "fqz5_fastq_format")
        at += n
    if not pairs:
        return text[:at]
    idx1, idx2, at = [], [], 0
    for n, k in zip(sizes, r1):
        idx1.append((at, at + k))
        idx2.append((at + k, at + n))
        at += n
    cat = lambda rs: torch.cat([text[a:b] for a, b in rs]) if rs else text[:0]
    return cat(idx1), cat(idx2)


def decompress_bytes(data: bytes, plus_name: bool = False, device: str = "cuda") -> bytes:
    """fqzcomp5 -d of a .fqz5 (its blocks parsed, CRC-checked and decoded on
    the GPU, the FASTQ text formatted there)."""
    import torch
    if not _blocks_of(data):
        return b""
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device)
    return _decode(data, buf, plus_name, device).cpu().numpy().tobytes()


def decompress_paired_bytes(data: bytes, plus_name: bool = False,
                            device: str = "cuda") -> tuple[bytes, bytes]:
    """fqzcomp5 -d in out1 out2: the records deinterleaved into R1 / R2."""
    import torch
    if not _blocks_of(data):
        return b"", b""
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device)
    t1, t2 = _decode(data, buf, plus_name, device, pairs=True)
    return t1.cpu().numpy().tobytes(), t2.cpu().numpy().tobytes()


def decompress_file(src: str, dst: str, plus_name: bool = False, device: str = "cuda",
                    dst2: str | None = None) -> int:
    """The file path: the .fqz5 read into page-locked memory, one copy to
    HBM, the FASTQ text back in one copy and written.  dst2: deinterleave,
    R1 records to dst and R2 records to dst2 (fqzcomp5 -d in out1 out2)."""
    host = _read_pinned(src)
    hv = host.numpy()
    if not _blocks_of(hv):
        for d in (dst, dst2):
            if d is not None:
                _write_out(d, b"")
        return 0
    buf = host.to(device)     # blocking: block parsing runs on the library's streams
    texts = _decode(hv, buf, plus_name, device, pairs=dst2 is not None)
    if dst2 is None:
        texts = (texts,)
    total = 0
    for text, d in zip(texts, (dst, dst2)):
        out = _pinned(int(text.numel()))
        out.copy_(text)
        _write_out(d, memoryview(out.numpy()))
        total += int(text.numel())
    return total


def _write_out(path: str, data) -> None:
    """Decoded text to `path`; gzip-compressed when the name ends in ".gz"
    (gzopen(name, "wb"), zlib's default level, fqzcomp5.c:5113-5160)."""
    if path.endswith(".gz"):
        import gzip
        with gzip.open(path, "wb", compresslevel=6) as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)
