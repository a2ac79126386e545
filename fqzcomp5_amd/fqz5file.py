"""FASTQ file <-> .fqz5 file on the GPU: the container
fqzcomp5 writes, produced and read by this library alone.

    compress_file(src, dst, level)   FASTQ text -> HBM -> fqz5_fastq_index /
                                     blocks / gather (fastq.hip) -> the
                                     section coder with the level's trial
                                     (sections.encode_run) -> whole blocks
                                     (fqz5_blocks_assemble) -> file
    decompress_file(src, dst)        file -> HBM -> fqz5_block_parse ->
                                     sections decoded -> fqz5_fastq_format

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
        _bound = True
    return so


def _check(rc, what):
    if rc < 0:
        raise _lib.NativeError(f"{what}: {_lib.last_error()}")
    return rc


def parse_fastq(text_d, blk_size: int):
    """FASTQ (or 2-line FASTA) text (a device uint8 tensor) -> a
    sections.Run of its blocks, every section input gathered in HBM.  FASTA
    blocks have no quality section (fqzcomp5.c:2237-2264)."""
    import torch
    so = _load()
    n = int(text_d.numel())
    # records <= lines / 4, FASTA records <= lines (+1 for a last line
    # without '\n')
    lpr = 1 if n and int(text_d[0].item()) == ord(">") else 4
    max_rec = (int((text_d == 10).sum().item()) + 1) // lpr + 1 if n else 1
    recs = torch.empty(max_rec * C.sizeof(FastqRec), dtype=torch.uint8, device=text_d.device)
    rsz = np.zeros(max_rec, np.uint32)
    nrec = C.c_uint64(0)
    fasta = _check(so.fqz5_fastq_index(text_d.data_ptr(), n, recs.data_ptr(), max_rec,
                                       C.byref(nrec), rsz.ctypes.data), "fqz5_fastq_index") == 1
    nrec = int(nrec.value)
    max_blocks = nrec + 1
    first = np.zeros(max_blocks + 1, np.uint64)
    nb = _check(so.fqz5_fastq_blocks(rsz.ctypes.data, nrec, blk_size, first.ctypes.data,
                                     max_blocks), "fqz5_fastq_blocks")
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
        lens.append(ln[:b - a])
        flags.append(fl[:b - a])
        nr.append((no, no + sizes[k][0]))
        sr.append((so_, so_ + sizes[k][1]))
        no += sizes[k][0]
        so_ += sizes[k][1]
    del recs
    return S.Run.from_device(name_d, seq_d, qual_d, nr, sr, lens, flags)


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
    """The file's bytes in page-locked host memory (one read, no copy)."""
    import os
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


def _encode(text_d, level: int, blk_size: int | None):
    """FASTQ text in HBM -> (the Run holding the encoded blocks, bases, records)."""
    blk = blk_size or S.BLOCK_SIZE[level]
    run = parse_fastq(text_d, blk)
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


def compress_file(src: str, dst: str, level: int = 3, blk_size: int | None = None,
                  device: str = "cuda") -> int:
    """The file path without host copies of the data: the FASTQ read into
    page-locked memory, one copy to HBM, the encoded blocks back in one copy
    and written behind the header, then the index."""
    # a blocking copy: the library's kernels run on its own streams, which
    # do not wait for torch's (a non-blocking copy raced the FASTQ parse)
    text_d = _read_pinned(src).to(device)
    run, bases, nrec = _encode(text_d, level, blk_size)
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


def _decode(data, buf, plus_name: bool, device: str):
    """Blocks of a .fqz5 (host view `data`, device copy `buf`) -> the FASTQ
    text of every block in one device buffer."""
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
    args, sizes = [], []
    for v, ln, po in zip(views, lens, places):
        size = C.c_uint64(0)
        a = (out_d.data_ptr() + po[0], v.name_ulen, out_d.data_ptr() + po[1],
             None if fasta[0] else out_d.data_ptr() + po[2], ln.ctypes.data, len(ln),
             int(plus_name))
        _check(so.fqz5_fastq_format(*a, None, 0, C.byref(size)), "fqz5_fastq_format")
        args.append(a)
        sizes.append(int(size.value))
    text = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device=device)
    at = 0
    for a, n in zip(args, sizes):
        size = C.c_uint64(0)
        _check(so.fqz5_fastq_format(*a, text.data_ptr() + at, n, C.byref(size)),
               "fqz5_fastq_format")
        at += n
    return text[:at]


def decompress_bytes(data: bytes, plus_name: bool = False, device: str = "cuda") -> bytes:
    """fqzcomp5 -d of a .fqz5 (its blocks parsed, CRC-checked and decoded on
    the GPU, the FASTQ text formatted there)."""
    import torch
    if not _blocks_of(data):
        return b""
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device)
    return _decode(data, buf, plus_name, device).cpu().numpy().tobytes()


def decompress_file(src: str, dst: str, plus_name: bool = False, device: str = "cuda") -> int:
    """The file path: the .fqz5 read into page-locked memory, one copy to
    HBM, the FASTQ text back in one copy and written."""
    host = _read_pinned(src)
    hv = host.numpy()
    if not _blocks_of(hv):
        open(dst, "wb").close()
        return 0
    buf = host.to(device)     # blocking: block parsing runs on the library's streams
    text = _decode(hv, buf, plus_name, device)
    out = _pinned(int(text.numel()))
    out.copy_(text)
    with open(dst, "wb") as f:
        f.write(memoryview(out.numpy()))
    return int(text.numel())
