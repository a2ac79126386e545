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

Scope: 4-line FASTQ, wrapped (multi-line) FASTQ as kseq_read reads it
(kseq.h:194-216; fastq.hip's record chain) and FASTA with any line wrapping
(text starting with '>': blocks without a quality section, decoded to
output_fasta's one-line text, fqzcomp5.c:2258-2264, :3503-3517).  Files of
any size stream through in windows of whole records (see below), on one or
several ranks; over several ranks a window of 4-line FASTQ or FASTA is read
once (each rank its share), a window holding wrapped FASTQ whole by every
rank.  Refused with an error (there is no host parse): the two layouts of
kseq's that fastq.hip does not follow (a lone '\\r' line before a block's
first kept byte, kseq.h:141; bytes between records, :180-186).
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
                ("seq_len", C.c_uint32), ("fasta", C.c_uint32), ("end", C.c_uint64)]


_bound = False


def _load():
    global _bound
    so = _lib.load()
    if not _bound:
        so.fqz5_fastq_index.restype = C.c_int
        so.fqz5_fastq_index.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                        C.POINTER(C.c_uint64), C.c_void_p]
        so.fqz5_fastq_index_any.restype = C.c_int
        so.fqz5_fastq_index_any.argtypes = so.fqz5_fastq_index.argtypes
        so.fqz5_fastq_record_ends.restype = C.c_int
        so.fqz5_fastq_record_ends.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                                              C.c_uint64, C.POINTER(C.c_uint64)]
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


# $FQZ5_FILE_TRACE: host wall time per stage of compress_file /
# decompress_file on stderr (read, upload, parse, gather, codec, assemble,
# download, write); the stages end with what the library synchronises
_TRACE = {}


class _stage:
    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        import time
        self.t = time.perf_counter()

    def __exit__(self, *a):
        import time
        _TRACE[self.name] = _TRACE.get(self.name, 0.0) + time.perf_counter() - self.t


def _trace_dump(what: str) -> None:
    import os
    import sys
    if os.environ.get("FQZ5_FILE_TRACE") and _TRACE:
        print(f"[fqz5file] {what}: " + ", ".join(f"{k} {1e3 * v:.1f} ms" for k, v in _TRACE.items()),
              file=sys.stderr, flush=True)
    _TRACE.clear()


def _check(rc, what):
    if rc < 0:
        raise _lib.NativeError(f"{what}: {_lib.last_error()}")
    return rc


def _index_text(text_d, at: int, n: int, wrapped: bool = False):
    """fqz5_fastq_index of text_d[at:at+n]: (records as bytes on the
    device, their load_seqs_kseq sizes, count, is FASTA).  wrapped: any
    layout kseq reads, wrapped FASTQ included (fqz5_fastq_index_any; the
    multi-rank windows, which count records in lines, keep 4-line FASTQ)."""
    import torch
    so = _load()
    part = text_d[at:at + n]
    # records <= lines / 4 (wrapped: / 3, a record without bases), FASTA
    # records <= lines (+1 for a last line without '\n')
    lpr = 1 if n and int(part[0].item()) == ord(">") else (3 if wrapped else 4)
    max_rec = (int((part == 10).sum().item()) + 1) // lpr + 1 if n else 1
    recs = torch.empty(max_rec * C.sizeof(FastqRec), dtype=torch.uint8, device=text_d.device)
    rsz = np.zeros(max_rec, np.uint32)
    nrec = C.c_uint64(0)
    _lib.after_torch(text_d.device)
    fn = so.fqz5_fastq_index_any if wrapped else so.fqz5_fastq_index
    fasta = _check(fn(text_d.data_ptr() + at, n, recs.data_ptr(), max_rec,
                      C.byref(nrec), rsz.ctypes.data), "fqz5_fastq_index") == 1
    nrec = int(nrec.value)
    if at and nrec:                     # offsets into the whole text
        v = recs[:nrec * C.sizeof(FastqRec)].view(torch.int64).view(nrec, -1)
        v[:, :4] += at
        v[:, 6] += at                   # (end)
    return recs[:nrec * C.sizeof(FastqRec)], rsz[:nrec], nrec, fasta


def _seq_lens_of(recs, rids) -> np.ndarray:
    """Sequence lengths of the records `rids` (the device record table)."""
    import torch
    if not len(rids):
        return np.zeros(0, np.uint32)
    w = C.sizeof(FastqRec)
    tab = recs.view(-1, w)
    idx = torch.as_tensor(np.asarray(rids, np.int64), device=recs.device)
    return tab[idx, 40:44].contiguous().view(torch.int32).flatten().cpu().numpy().astype(np.uint32)


def _fasta_blocks(recs, starts, fasta: bool) -> list[bool]:
    """load_seqs_kseq's per-block rule (fqzcomp5.c:574-578, :805-809): a
    block is FASTA (no quality section) when its first record has no
    quality, i.e. in FASTQ text when that record's sequence is empty."""
    if fasta:
        return [True] * len(starts)
    return [bool(x == 0) for x in _seq_lens_of(recs, starts)]


def _gather(text_d, recs, first, fasta: bool, pair_flags: bool):
    """The blocks [first[k], first[k+1]) of the records as a sections.Run,
    every section input gathered in HBM.  pair_flags: READ2 on the odd
    records (load_seqs_interleaved, fqzcomp5.c:763) instead of from the names."""
    return _gather_ranges(text_d, recs, [(int(first[k]), int(first[k + 1]))
                                         for k in range(len(first) - 1)], fasta, pair_flags)


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
    recs, rsz, nrec, fasta = _index_text(text_d, 0, int(text_d.numel()), wrapped=True)
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
    r1, rs1, n1, fa1 = _index_text(text_d, 0, len1, wrapped=True)
    r2, rs2, n2, fa2 = _index_text(text_d, len1, int(text_d.numel()) - len1, wrapped=True)
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


def _index(offs, bases, nrec) -> bytes:
    return INDEX_MAGIC + struct.pack("<I", len(offs)) + b"".join(
        struct.pack("<QII", o, nb, nr) for o, nb, nr in zip(offs, bases, nrec))


# ---------------------------------------------------------------------------
# streaming and multi-GPU encode
#
# The reference reads its input block by block (load_seqs_kseq per block,
# fqzcomp5.c:3051, dispatched at :3077) and writes each block behind the
# last, the index at the end (:3108-3115, write_index :2606).  Here the text
# comes in windows of whole records (a FASTQ window ends after 4k lines, a
# FASTA window before a header line); the last block of a window that is not
# the end of the input may be incomplete, so it is not coded: the next window
# starts at its first record.  The codec trial's state carries from window
# to window, so the blocks and their methods are those of one pass over the
# whole input.
#
# Over several ranks (group = a torch.distributed group, one process per
# GPU), every rank reads and parses every window (the block split needs the
# records in order), the window's blocks are split contiguously over the
# ranks, each rank codes its own blocks and its share of the trial blocks'
# work candidates (sections.encode_window), and the blocks are written with
# positioned writes at offsets from an all-gather of the block sizes and an
# exclusive scan; rank 0 writes the header and the index.
# ---------------------------------------------------------------------------
DEFAULT_WINDOW = 2_000_000_000
# Device bytes the encode of a window takes per input byte, by level (the
# arenas' pool peak over the input size, bench.py's arena_bytes.peak): the
# candidates' outputs and the fqz / sequence-model event tables of the trial
# blocks dominate.
FOOTPRINT = {1: 24, 2: 24, 3: 40, 4: 40, 5: 64, 6: 64, 7: 64, 8: 64, 9: 64}


def window_bytes_for(level: int, blk: int, ws: int = 1, hbm: int | None = None) -> int:
    """The encode window: as much input as fits 0.8 x HBM at the level's
    footprint on every rank (each codes about window / ws of it), at least
    two blocks per rank and one over (the last block of a window waits for
    the next), at most 8 GB per rank."""
    if hbm is None:
        import torch
        hbm = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory \
            if torch.cuda.is_available() else 64 << 30
    per_rank = int(0.8 * hbm) // FOOTPRINT.get(level, 64)
    per_rank = min(per_rank, 8_000_000_000)
    return max(ws * per_rank, 2 * ws * blk + blk)


class _Src:
    """One input read sequentially (plain or gzip; a path or bytes), holding
    the unread text from the start of the next window on (`buf`).

    A plain file is memory-mapped: `buf` is a view of the mapping and the
    window's text goes to the device straight from the page cache in 32 MB
    parts on several threads (fill(device=...)), with no host copy of the
    text to make, fault in and free (the copy ran at ~4.3 GB/s, and freeing
    a 1 GB window's copy took ~90 ms).  gzip and bytes sources keep a host
    buffer."""

    def __init__(self, path: str | None = None, data: bytes | None = None):
        import gzip
        import io
        import os
        self.path, self.gz = path, False
        self.mm = None
        if data is not None:
            self.f = io.BytesIO(data)
            self.size = len(data)
        else:
            with open(path, "rb") as f:
                magic = f.read(2)
            self.gz = magic == b"\x1f\x8b"
            self.f = gzip.open(path, "rb") if self.gz else open(path, "rb")
            self.size = None if self.gz else os.fstat(self.f.fileno()).st_size
            if not self.gz and self.size:
                import mmap
                self.mm = mmap.mmap(self.f.fileno(), 0, access=mmap.ACCESS_READ)
        self.pos = 0                          # bytes read so far (plain / bytes)
        self.base = 0                         # mapped: file offset of buf's start
        self._buf = bytearray()
        self.dev = None                       # fill(device=...): the buffer on the device
        self.eof = False

    @property
    def buf(self):
        if self.mm is not None:
            return memoryview(self.mm)[self.base:self.pos]
        return self._buf

    def fill(self, want: int, device=None) -> None:
        """The buffer up to `want` bytes (or the end of the input).  device
        (a mapped file): also self.dev, the whole buffer on the device
        (otherwise self.dev is None and the caller uploads)."""
        self.dev = None
        if self.mm is not None:
            end = min(self.base + max(want, 0), self.size)
            if end > self.pos:
                self.pos = end
            self.eof = self.pos >= self.size
            if device is not None and self.pos > self.base:
                self.dev = self._upload(device)
            return
        need = want - len(self._buf)
        if need <= 0 or self.eof:
            return
        if self.size is None:                 # gzip: chunks
            while len(self._buf) < want and not self.eof:
                c = self.f.read(min(want - len(self._buf), 1 << 28))
                if not c:
                    self.eof = True
                    break
                self._buf += c
            return
        at = len(self._buf)                   # bytes: into a buffer of the exact size
        left = self.size - self.pos
        want = at + min(need, left)
        nb = bytearray(want)
        nb[:at] = self._buf
        self._buf = nb
        got = self.f.readinto(memoryview(self._buf)[at:want])
        self.pos += got
        if at + got < want:
            del self._buf[at + got:]
        if self.pos >= self.size:
            self.eof = True

    def _upload(self, device):
        """buf on the device: 32 MB parts copied from the mapping by several
        threads (the copies fault the page-cache pages in and release the
        GIL)."""
        import warnings
        from concurrent.futures import ThreadPoolExecutor
        import torch
        a, b = self.base, self.pos
        dev = torch.empty(b - a, dtype=torch.uint8, device=device)
        mv = memoryview(self.mm)
        step = 32 << 20
        parts = [(o, min(o + step, b)) for o in range(a, b, step)]

        def one(p):
            o, e = p
            with warnings.catch_warnings():   # (a read-only mapping: torch only reads it)
                warnings.simplefilter("ignore")
                src = torch.frombuffer(mv[o:e], dtype=torch.uint8)
            dev[o - a:e - a].copy_(src)
        try:
            if len(parts) == 1:
                one(parts[0])
            else:
                with ThreadPoolExecutor(max_workers=min(16, len(parts))) as ex:
                    list(ex.map(one, parts))
        finally:
            del mv
        return dev

    def advance(self, n: int) -> None:
        if self.mm is not None:
            self.base += n
        else:
            del self._buf[:n]

    def close(self) -> None:
        if self.mm is not None:
            self.mm.close()
            self.mm = None
        self.f.close()


class _Sink:
    """Positioned writes into the output file (or a bytearray).  A pipe, FIFO
    or terminal (/dev/stdout) cannot take pwrite (ESPIPE): there the writes
    go out sequentially, any that arrive ahead of the stream position held
    until the bytes before them have been written."""

    def __init__(self, path: str | None, create: bool):
        import os
        import stat
        self.path, self.mem, self.fd = path, None, None
        self.seq, self.pos, self.held = False, 0, {}
        if path is None:
            self.mem = bytearray()
        else:
            flags = os.O_WRONLY | (os.O_CREAT | os.O_TRUNC if create else 0)
            self.fd = os.open(path, flags, 0o644)
            self.seq = not stat.S_ISREG(os.fstat(self.fd).st_mode)

    def _write_seq(self, off: int, mv) -> None:
        import os
        if off != self.pos:
            if off < self.pos:
                raise ValueError("sequential output: a write before the stream position")
            self.held[off] = bytes(mv)
            return
        while True:
            while len(mv):
                k = os.write(self.fd, mv)
                mv = mv[k:]
                self.pos += k
            nxt = self.held.pop(self.pos, None)
            if nxt is None:
                return
            mv = memoryview(nxt)

    def write_at(self, off: int, data) -> None:
        import os
        mv = memoryview(data).cast("B")
        if self.mem is not None:
            if len(self.mem) < off + len(mv):
                self.mem.extend(b"\0" * (off + len(mv) - len(self.mem)))
            self.mem[off:off + len(mv)] = mv
            return
        if self.seq:
            self._write_seq(off, mv)
            return
        if len(mv) >= (64 << 20):
            # large writes in 32 MB parts on several threads (the page-cache
            # copy runs at ~4 GB/s on one core; pwrite releases the GIL)
            from concurrent.futures import ThreadPoolExecutor
            step = 32 << 20
            parts = [(o, min(o + step, len(mv))) for o in range(0, len(mv), step)]

            def one(p):
                a, b = p
                part, at = mv[a:b], off + a
                while len(part):
                    k = os.pwrite(self.fd, part, at)
                    part, at = part[k:], at + k
            with ThreadPoolExecutor(max_workers=min(16, len(parts))) as ex:
                list(ex.map(one, parts))
            return
        while len(mv):
            k = os.pwrite(self.fd, mv, off)
            mv, off = mv[k:], off + k

    def close(self) -> None:
        import os
        if self.fd is not None:
            held, self.held = self.held, {}
            os.close(self.fd)
            self.fd = None
            if held:
                raise ValueError("sequential output: a gap before the held writes")


def _allgather_obj(x, group):
    return S.xchg(x, group)


def _barrier(group):
    S.barrier(group)


def _complete_records(text_d, n: int, eof: bool):
    """Record ends of text_d[:n] (exclusive offsets, increasing; a list or a
    uint64 array) that are known to be complete, and whether the text is
    FASTA.  FASTQ: after each record (fqz5_fastq_record_ends: 4-line or
    wrapped); FASTA: before every header line after the first; at the end of
    the input, the end of the text closes the last record."""
    import torch
    if n == 0:
        return [], False
    t = text_d[:n]
    fasta = int(t[0].item()) == ord(">")
    if fasta:
        starts = ((t[1:] == ord(">")) & (t[:-1] == 10)).nonzero().flatten() + 1
        ends = starts.cpu().tolist()
    else:
        # 4-line records, or kseq's wrapped ones (fqz5_fastq_record_ends)
        cap = int((t == 10).sum().item()) // 3 + 2
        buf = np.zeros(cap, np.uint64)
        cnt = C.c_uint64(0)
        _lib.after_torch()
        _check(_load().fqz5_fastq_record_ends(text_d.data_ptr(), n, int(bool(eof)), buf.ctypes.data,
                                              cap, C.byref(cnt)), "fqz5_fastq_record_ends")
        # (an array: the window needs the count and one end, not 3M Python ints)
        ends = buf[:int(cnt.value)]
        if eof and (not len(ends) or int(ends[-1]) != n):
            ends = np.append(ends, np.uint64(n))
        return ends, fasta
    if eof and (not ends or ends[-1] != n):
        ends.append(n)
    del torch
    return ends, fasta


def _rec_start(recs, r: int) -> int:
    """Text offset of record r's header line (its name field less one)."""
    import torch
    w = C.sizeof(FastqRec)
    return int(recs[r * w:r * w + 8].view(torch.int64).item()) - 1


class _Window:
    """One window of the input, parsed: record table, block starts (records),
    the blocks to code now, and the text to consume after them."""
    pass


def _next_window(srcs: list, blk: int, wbytes: int, device: str):
    """Parse the next window of whole records from the source(s); returns a
    _Window or None at the end of the input.  Grows the window until it holds
    one complete block (or the rest of the input)."""
    import torch
    so = _load()
    paired = len(srcs) == 2
    want = wbytes
    while True:
        with _stage("read"):                  # (the parts go up as they are read)
            for s in srcs:
                s.fill(want, device)
        devs, ends = [], []
        for s in srcs:
            with _stage("upload"):
                if getattr(s, "dev", None) is not None and int(s.dev.numel()) == len(s.buf):
                    d = s.dev
                    s.dev = None
                    H2D[0] += int(d.numel())
                elif len(s.buf):
                    cpu = torch.frombuffer(s.buf, dtype=torch.uint8)
                    d = cpu.to(device)            # blocking (pageable): done before the parse
                    H2D[0] += int(cpu.numel())
                    del cpu
                else:
                    d = torch.empty(0, dtype=torch.uint8, device=device)
            devs.append(d)
            with _stage("record_ends"):
                ends.append(_complete_records(d, int(d.numel()), s.eof)[0])
        k = min(len(e) for e in ends) if paired else len(ends[0])
        r1_done = srcs[0].eof and k == len(ends[0])      # all of R1 in the window
        if paired and not r1_done and srcs[1].eof and k == len(ends[1]):
            raise _lib.NativeError("unpaired read detected: R2 file ended before R1")
        if k == 0:
            if r1_done:
                return None
            want *= 2
            continue
        cut = [int(e[k - 1]) for e in ends]
        if paired:
            text_d = torch.cat([devs[0][:cut[0]], devs[1][:cut[1]]])
            len1 = cut[0]
        else:
            text_d, len1 = devs[0][:cut[0]], None
        del devs
        if len1 is None:
            with _stage("parse"):
                recs, rsz, nrec, fasta = _index_text(text_d, 0, int(text_d.numel()), wrapped=True)
                first = _blocks(so, rsz, blk)
        else:
            r1, rs1, n1, fa1 = _index_text(text_d, 0, len1, wrapped=True)
            r2, rs2, n2, fa2 = _index_text(text_d, len1, int(text_d.numel()) - len1, wrapped=True)
            if n2 < n1:
                raise _lib.NativeError("unpaired read detected: R2 file ended before R1")
            if n1 and fa1 != fa2:
                raise _lib.NativeError("paired files: one FASTA, one FASTQ")
            w = C.sizeof(FastqRec)
            recs = (torch.stack([r1.view(n1, w), r2[:n1 * w].view(n1, w)], 1).reshape(-1)
                    if n1 else r1)
            del r1, r2
            pair = rs1.astype(np.uint64) + rs2[:n1].astype(np.uint64)
            if n1 and int(pair.max()) >= 2 ** 32:
                raise _lib.NativeError("paired record larger than 4 GB")
            first = _blocks(so, pair.astype(np.uint32), blk) * 2
            fasta = fa1
        nb = len(first) - 1
        keep = nb if r1_done else nb - 1
        if keep <= 0:
            want *= 2
            continue
        W = _Window()
        W.text_d, W.recs, W.first, W.fasta, W.pairs = text_d, recs, first[:keep + 1], fasta, paired
        W.final = bool(r1_done and keep == nb)   # the input ends with this window
        if keep < nb:                          # the next window starts at block `keep`
            r = int(first[keep])
            W.consume = [_rec_start(recs, r)] + \
                ([_rec_start(recs, r + 1) - len1] if paired else [])
        else:
            W.consume = [len(srcs[0].buf)] + ([len(srcs[1].buf)] if paired else [])
        return W


# ---------------------------------------------------------------------------
# Windows read once over the ranks (plain files, several ranks).  The window
# [P, P + Wn) of each input is cut into one byte range per rank; each rank
# reads and uploads only its range (and the byte before it), counts its
# newlines on the GPU, and after one exchange of the counts knows which of
# its line starts are record starts (FASTQ: every 4th line from the window
# start; FASTA: a '>' line).  It parses the records that start in its range
# (fqz5_fastq_index), and a second exchange gives every rank every record's
# start, load_seqs_kseq size, name-section and sequence bytes: the block
# split (fqz5_fastq_blocks) is then computed alike on every rank.  A block
# belongs to the rank holding its first record; a rank then gathers its own
# blocks (and the trial blocks whose work candidates it shares) from the text
# it already holds, reading from the file only the bytes it lacks (the end of
# its last block, other ranks' trial blocks).  Reference: load_seqs_kseq's
# split, fqzcomp5.c:423-623; dispatch :3051-3120.
# ---------------------------------------------------------------------------
H2D = [0]          # input text bytes this process uploaded (tests, bench)


def _upload(buf, device: str):
    import torch
    a = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    H2D[0] += int(a.size)
    if not a.size:
        return torch.empty(0, dtype=torch.uint8, device=device)
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


class _PosFile:
    """A plain input file read at positions."""

    def __init__(self, path: str):
        import os
        self.fd = os.open(path, os.O_RDONLY)
        self.size = os.fstat(self.fd).st_size

    def read(self, a: int, b: int) -> np.ndarray:
        import os
        out = np.empty(max(b - a, 0), np.uint8)
        got = 0
        while got < out.size:
            c = os.pread(self.fd, out.size - got, a + got)
            if not c:
                raise _lib.NativeError("input file shrank while being read")
            out[got:got + len(c)] = np.frombuffer(c, np.uint8)
            got += len(c)
        return out

    def close(self) -> None:
        import os
        os.close(self.fd)


def _allgather_np(x, group):
    return _allgather_obj(x, group)


def _record_end(f: _PosFile, s: int, fasta: bool) -> int:
    """End (exclusive) of the record starting at file offset s: FASTQ after
    its 4th line, FASTA before the next '>' line; the end of the file closes
    the last record."""
    need, at, piece = 4, s, 1 << 16
    while at < f.size:
        b = f.read(at, min(f.size, at + piece))
        if fasta:
            hit = np.flatnonzero((b[:-1] == 10) & (b[1:] == ord(">")))
            if hit.size:
                return at + int(hit[0]) + 1
            at += max(b.size - 1, 1)
        else:
            nl = np.flatnonzero(b == 10)
            if nl.size >= need:
                return at + int(nl[need - 1]) + 1
            need -= nl.size
            at += b.size
        piece *= 2
    return f.size


class _Scan:
    """One input's window scanned over the ranks (see above)."""
    pass


def _scan(f: _PosFile, P: int, Wn: int, device: str, group, fasta=None) -> _Scan:
    import torch
    ws, rk = S._world(group)
    lo, hi = P + rk * Wn // ws, P + (rk + 1) * Wn // ws
    # bytes [lo - 1, hi): the byte before the range decides whether lo
    # starts a line (a newline stands in before the window start)
    h = f.read(max(lo - 1, P), hi)
    if lo == P:
        h = np.concatenate([np.array([10], np.uint8), h])
    t = _upload(h, device)
    n = hi - lo
    nl = (t[:n] == 10) if n else torch.zeros(0, dtype=torch.bool, device=device)
    head = int(t[1].item()) if rk == 0 and t.numel() > 1 else -1
    cnt = int(nl.sum().item()) if n else 0
    got = _allgather_np((cnt, head), group)
    if fasta is None:
        fasta = got[0][1] == ord(">")
    base = sum(c for c, _ in got[:rk])
    # four: this range reads as 4-line FASTQ (every line 4k a '@' line, every
    # line 4k + 2 a '+' line), where kseq's record is exactly those 4 lines;
    # wrapped FASTQ (or blank lines among the records) fails it and the
    # window is read whole instead (_next_window_ranks)
    four = True
    if n:
        if fasta:
            st = nl & (t[1:n + 1] == ord(">"))
        else:
            # (an '@' line: blank lines after the last record start none)
            line = torch.cumsum(nl.to(torch.int64), 0) + (base - 1)
            st = nl & (line % 4 == 0) & (t[1:n + 1] == ord("@"))
            four = not bool((nl & (line % 4 == 2) & (t[1:n + 1] != ord("+"))).any().item()) \
                and not bool((nl & (line % 4 == 0) & (t[1:n + 1] != ord("@"))).any().item())
        starts = (st.nonzero().flatten() + lo).cpu().numpy().astype(np.int64)
    else:
        starts = np.zeros(0, np.int64)
    firsts = _allgather_np(int(starts[0]) if starts.size else -1, group)
    # the end of this rank's last record: the next rank's first start, or
    # (the window's last record) found by reading on
    nxt = [x for x in firsts[rk + 1:] if x >= 0]
    sc = _Scan()
    sc.fasta = fasta
    sc.lo = int(starts[0]) if starts.size else hi
    nrec = -1
    if starts.size and four:
        end = nxt[0] if nxt else _record_end(f, int(starts[-1]), fasta)
        text = t[int(starts[0]) - (lo - 1):]
        if end > hi:
            text = torch.cat([text, _upload(f.read(hi, end), device)])
        else:
            text = text[:end - int(starts[0])]
        sc.hi = end
        try:
            recs, rsz, nrec, fa = _index_text(text, 0, int(text.numel()))
        except _lib.NativeError:
            four = False              # (every rank still takes the exchanges below)
        four = four and nrec == starts.size
    if starts.size and four:
        w = C.sizeof(FastqRec)
        u = recs.view(nrec, w)[:, 32:44].contiguous().view(torch.int32).view(nrec, 3).cpu().numpy()
        nsz = (u[:, 0] + np.where(u[:, 1] > 0, u[:, 1] + 1, 0) + 1).astype(np.uint64)
        slen = u[:, 2].astype(np.uint64)
    else:
        text, sc.hi = t[:0], hi
        rsz = np.zeros(0, np.uint32)
        nsz = slen = np.zeros(0, np.uint64)
        if not four:
            starts = np.zeros(0, np.int64)
    del t, nl
    sc.text = text                       # this rank's records' text, [lo, hi) of the file
    parts = _allgather_np((starts, rsz.astype(np.uint32), nsz, slen, sc.hi, four), group)
    sc.four = all(p[5] for p in parts)
    if not sc.four:
        return sc
    sc.start = np.concatenate([p[0] for p in parts]).astype(np.int64)
    sc.rsz = np.concatenate([p[1] for p in parts]).astype(np.uint32)
    sc.nsz = np.concatenate([p[2] for p in parts]).astype(np.uint64)
    sc.slen = np.concatenate([p[3] for p in parts]).astype(np.uint64)
    counts = [len(p[0]) for p in parts]
    sc.rank_of = np.repeat(np.arange(ws), counts)
    ends = [p[4] for p in parts if len(p[0])]
    sc.end = np.append(sc.start[1:], ends[-1] if ends else P).astype(np.int64)   # per record
    sc.n = int(sc.start.size)
    return sc


def _need_text(f: _PosFile, sc: _Scan, ranges, device: str):
    """The text of the byte ranges (file order, disjoint) as one device
    buffer: the parts this rank holds from its scan sliced, the rest read."""
    import torch
    pieces = []
    for a, e in ranges:
        x0, x1 = max(a, sc.lo), min(e, sc.hi)
        if x0 < x1:
            if a < x0:
                pieces.append(_upload(f.read(a, x0), device))
            pieces.append(sc.text[x0 - sc.lo:x1 - sc.lo])
            if x1 < e:
                pieces.append(_upload(f.read(x1, e), device))
        else:
            pieces.append(_upload(f.read(a, e), device))
    if not pieces:
        return torch.empty(0, dtype=torch.uint8, device=device)
    return torch.cat(pieces) if len(pieces) > 1 else pieces[0]


def _merge(ranges):
    out = []
    for a, e in ranges:
        if out and out[-1][1] == a:
            out[-1] = (out[-1][0], e)
        else:
            out.append((a, e))
    return out


class _RankWindow:
    """A window read once over the ranks: the per-block fields every rank
    knows, and gather() for the blocks this rank codes or tries."""

    def __init__(self, files, pos, scans, k, first, keep, final, group, device):
        ws, rk = S._world(group)
        self.files, self.pos, self.scans, self.device = files, pos, scans, device
        self.paired = len(files) == 2
        self.first, self.nb, self.final = first, keep, final
        mul = 2 if self.paired else 1
        fa = scans[0].fasta
        self.text_fasta = fa
        self.fasta, self.name_bytes, self.seq_bytes, self.nrec, self.owner = [], [], [], [], []
        for b in range(keep):
            a, e = int(first[b]) // mul, int(first[b + 1]) // mul
            self.fasta.append(fa or int(scans[0].slen[a]) == 0)
            self.name_bytes.append(int(sum(int(s.nsz[a:e].sum()) for s in scans)))
            self.seq_bytes.append(int(sum(int(s.slen[a:e].sum()) for s in scans)))
            self.nrec.append((e - a) * mul)
            self.owner.append(int(scans[0].rank_of[a]))
        self.owner = np.array(self.owner, np.int64)
        # the next window starts at block `keep` (R1 and R2 at the same pair)
        if keep < len(first) - 1:
            r = int(first[keep]) // mul
            self.next_pos = [int(s.start[r]) for s in scans]
        else:
            self.next_pos = [int(s.end[k - 1]) if k else p for s, p in zip(scans, pos)]

    def gather(self, need):
        """A sections.Run of the blocks `need` (in that order)."""
        import torch
        mul = 2 if self.paired else 1
        texts, lens = [], []
        for f, sc in zip(self.files, self.scans):
            rng = []
            for b in need:
                a, e = int(self.first[b]) // mul, int(self.first[b + 1]) // mul
                rng.append((int(sc.start[a]), int(sc.end[e - 1])))
            t = _need_text(f, sc, _merge(rng), self.device)
            texts.append(t)
            lens.append(int(t.numel()))
        nrecs = [self.nrec[b] for b in need]
        loc = np.concatenate([[0], np.cumsum(nrecs)]).astype(np.int64)
        if not self.paired:
            text_d = texts[0]
            recs, _, nrec, _ = _index_text(text_d, 0, lens[0])
        else:
            text_d = torch.cat(texts) if lens[1] else texts[0]
            r1, _, n1, _ = _index_text(text_d, 0, lens[0])
            r2, _, n2, _ = _index_text(text_d, lens[0], lens[1])
            if n1 != n2:
                raise _lib.NativeError("window gather: R1 and R2 record counts differ")
            w = C.sizeof(FastqRec)
            recs = torch.stack([r1.view(n1, w), r2.view(n2, w)], 1).reshape(-1) if n1 else r1
            nrec = 2 * n1
        if nrec != int(loc[-1]):
            raise _lib.NativeError("window gather: record count differs from the scan")
        run = _gather_ranges(text_d, recs, [(int(loc[j]), int(loc[j + 1]))
                                            for j in range(len(need))],
                             self.text_fasta, self.paired)
        for j, b in enumerate(need):          # the scan's sizes are the ones coded
            i = run.blk_sec0[j]
            if (run.spans[i][2] - run.spans[i][1], run.spans[i + 1][2] - run.spans[i + 1][1]) != \
                    (self.name_bytes[b], self.seq_bytes[b]):
                raise _lib.NativeError("window gather: section sizes differ from the scan")
        return run

    def advance(self):
        self.pos[:] = self.next_pos


WRAPPED = object()


def _next_window_ranks(files, pos, blk: int, wbytes: int, device: str, group):
    """The next window of the inputs at file offsets `pos`, read once over
    the ranks; None at the end of the input; WRAPPED when the window is not
    4-line FASTQ (or FASTA), whose record starts the line count cannot give:
    wrapped FASTQ, whose kseq records (kseq.h:194-216) only a walk from a
    known record start finds (the caller then reads the window whole on
    every rank, _LocalWindow)."""
    so = _load()
    paired = len(files) == 2
    want = wbytes
    if pos[0] >= files[0].size:
        return None
    while True:
        wn = [min(want, f.size - p) for f, p in zip(files, pos)]
        eof = [p + w >= f.size for f, p, w in zip(files, pos, wn)]
        scans = [_scan(files[0], pos[0], wn[0], device, group)]
        if paired:
            scans.append(_scan(files[1], pos[1], wn[1], device, group))
        if not all(sc.four for sc in scans):
            return WRAPPED
            if scans[0].n and scans[1].n and scans[0].fasta != scans[1].fasta:
                raise _lib.NativeError("paired files: one FASTA, one FASTQ")
        k = min(s.n for s in scans)
        r1_done = eof[0] and k == scans[0].n
        if paired and not r1_done and eof[1] and k == scans[1].n:
            raise _lib.NativeError("unpaired read detected: R2 file ended before R1")
        if k == 0:
            if r1_done:
                return None
            want *= 2
            continue
        if paired:
            pair = scans[0].rsz[:k].astype(np.uint64) + scans[1].rsz[:k].astype(np.uint64)
            if int(pair.max()) >= 2 ** 32:
                raise _lib.NativeError("paired record larger than 4 GB")
            first = _blocks(so, pair.astype(np.uint32), blk) * 2
        else:
            first = _blocks(so, scans[0].rsz[:k], blk)
        nb = len(first) - 1
        keep = nb if r1_done else nb - 1
        if keep <= 0:
            want *= 2
            continue
        return _RankWindow(files, pos, scans, k, first, keep, bool(r1_done and keep == nb),
                           group, device)


class _LocalWindow:
    """A window every rank reads whole (one rank, or gzip / in-memory
    input): the same per-block fields as _RankWindow."""

    def __init__(self, W, srcs, ws):
        so = _load()
        self.W, self.srcs = W, srcs
        nb = len(W.first) - 1
        self.nb, self.final = nb, W.final
        self.fasta = _fasta_blocks(W.recs, [int(W.first[b]) for b in range(nb)], W.fasta)
        self.name_bytes, self.seq_bytes, self.nrec = [], [], []
        for b in range(nb):
            a, e = int(W.first[b]), int(W.first[b + 1])
            sz = (C.c_uint64 * 3)()
            _lib.after_torch()
            _check(so.fqz5_fastq_gather(W.text_d.data_ptr(), W.recs.data_ptr(), a, e, None,
                                        None, None, None, None, sz), "fqz5_fastq_gather")
            self.name_bytes.append(int(sz[0]))
            self.seq_bytes.append(int(sz[1]))
            self.nrec.append(e - a)
        self.owner = (np.arange(nb) * ws) // nb

    def gather(self, need):
        W = self.W
        return _gather_ranges(W.text_d, W.recs, [(int(W.first[b]), int(W.first[b + 1]))
                                                 for b in need], W.fasta, W.pairs)

    def advance(self):
        for s, c in zip(self.srcs, self.W.consume):
            s.advance(c)


def _code_window(W, sink: _Sink, level: int, pos: int, index: list, av, state, group) -> int:
    """Code the window's blocks over the ranks and write them at file
    offset `pos` on (see above); appends their index entries and returns
    the offset after them."""
    ws, rk = S._world(group)
    nb = W.nb
    # per block the sections in encode_block order (no quality section in a
    # FASTA block)
    per = [2 if f else 3 for f in W.fasta]
    sec0 = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    ids, ins = [], []
    for b in range(nb):
        ids += [S.SEC_NAME, S.SEC_SEQ] + ([] if W.fasta[b] else [S.SEC_QUAL])
        ins += [W.name_bytes[b], W.seq_bytes[b]] + ([] if W.fasta[b] else [W.seq_bytes[b]])
    ids = np.array(ids, np.int32)
    ins = np.array(ins, np.uint32)
    blk_owner = np.asarray(W.owner, np.int64)
    owner = np.repeat(blk_owner, per)
    sched = S.trial_schedule(ids, av, state)
    need = sorted({b for b in range(nb)
                   if blk_owner[b] == rk or sched[sec0[b]:sec0[b + 1]].any()})
    # the needed blocks' section inputs, gathered in HBM
    with _stage("gather"):
        run = W.gather(need)
    secs = [None] * int(sec0[-1])
    local = run.enc_secs()
    for j, b in enumerate(need):
        for q in range(per[b]):
            secs[sec0[b] + q] = local[run.blk_sec0[j] + q]
    with _stage("codec"):
        res, meth, _ = S.encode_window(secs, ids, ins, owner, av, state, group,
                                       bounded=level >= 7, final=W.final,
                                       bounds_first=5 <= level < 7)
    mine = [j for j, b in enumerate(need) if blk_owner[b] == rk]
    full_res = [None] * len(local)
    for j, b in enumerate(need):
        for q in range(per[b]):
            full_res[run.blk_sec0[j] + q] = res[sec0[b] + q]
    for j in mine:
        for q in range(per[need[j]]):
            r = full_res[run.blk_sec0[j] + q]
            if r is None or r.status != 0:
                raise _lib.NativeError("section coding failed: " + _lib.last_error())
    sizes = []
    if mine:
        with _stage("assemble"):
            run.assemble(full_res, mine)
        sizes = [int(run.blk_off[i + 1] - run.blk_off[i]) for i in range(len(mine))]
    all_sizes = _allgather_obj(sizes, group)
    # blocks in file order: rank-contiguous, so rank-major order
    flat = [z for zs in all_sizes for z in zs]
    assert len(flat) == nb
    starts = np.concatenate([[0], np.cumsum(flat)]).astype(np.int64) + pos
    if mine:
        end = int(run.blk_off[len(mine)])
        with _stage("download"):
            host = _pinned(end)
            host.copy_(run.blk_buf[:end])
        b0 = need[mine[0]]
        with _stage("write"):
            sink.write_at(int(starts[b0]), host.numpy())
        del host
    for b in range(nb):
        index.append((int(starts[b]), W.seq_bytes[b], W.nrec[b]))
    return int(starts[-1])


def _encode_stream(srcs: list, sink: _Sink, level: int, blk_size: int | None, device: str,
                   group=None, window_bytes: int | None = None) -> int:
    """The sources' FASTQ -> .fqz5 written through `sink` (see above);
    returns the file size."""
    ws, rk = S._world(group)
    blk = blk_size or S.BLOCK_SIZE[level]
    # a window holds several blocks per rank, so that every GPU has blocks
    # whose serial chains run side by side
    wbytes = window_bytes or window_bytes_for(level, blk, ws)
    av = S.masks(level, full=True)
    state = S.new_state()
    pos = 16                                  # file offset of the next block
    index = []
    # several ranks on plain files: each reads its share of every window once
    files = [_PosFile(s.path) for s in srcs] \
        if ws > 1 and all(s.path and not s.gz for s in srcs) else None
    opened = list(files or [])
    at = [0] * len(srcs)
    try:
        while True:
            with _stage("window"):
                W = _next_window_ranks(files, at, blk, wbytes, device, group) if files else None
                if W is WRAPPED:
                    # wrapped FASTQ: from here on every rank reads each window
                    # whole and walks its records (fqz5_fastq_record_ends); the
                    # mapped sources start at the window's offsets
                    for s_, a in zip(srcs, at):
                        s_.base = s_.pos = a
                        s_.eof = False
                    files = None
                if not files:
                    w0 = _next_window(srcs, blk, wbytes, device)
                    W = _LocalWindow(w0, srcs, ws) if w0 is not None else None
            if W is None:
                break
            with _stage("code_window"):
                pos = _code_window(W, sink, level, pos, index, av, state, group)
            with _stage("advance"):
                W.advance()
                del W
    finally:
        for f in opened:
            f.close()
    if rk == 0:
        if index:
            idx = _index([o for o, _, _ in index], [b for _, b, _ in index],
                         [n for _, _, n in index])
            sink.write_at(pos, idx)
        else:
            idx = b""
        sink.write_at(0, MAGIC + struct.pack("<Q", pos))
        total = pos + len(idx)
    else:
        total = 0
    _trace_dump(f"encode -{level}")
    return int(_allgather_obj(total, group)[0])


def _gather_ranges(text_d, recs, ranges, fasta: bool, pair_flags: bool):
    """Blocks given as record ranges [a, b) (not necessarily adjacent) as a
    sections.Run, every section input gathered in HBM."""
    import torch
    so = _load()
    sizes = []
    for a, b in ranges:
        sz = (C.c_uint64 * 3)()
        _lib.after_torch()
        _check(so.fqz5_fastq_gather(text_d.data_ptr(), recs.data_ptr(), a, b, None, None, None,
                                    None, None, sz), "fqz5_fastq_gather")
        sizes.append((int(sz[0]), int(sz[1])))
    tot_n = sum(a for a, _ in sizes)
    tot_s = sum(b for _, b in sizes)
    name_d = torch.empty(max(tot_n, 1), dtype=torch.uint8, device=text_d.device)
    seq_d = torch.empty(max(tot_s, 1), dtype=torch.uint8, device=text_d.device)
    qual_d = None if fasta else torch.empty(max(tot_s, 1), dtype=torch.uint8, device=text_d.device)
    bfa = _fasta_blocks(recs, [a for a, _ in ranges], fasta)
    lens, flags, nr, sr = [], [], [], []
    no = so_ = 0
    for (a, b), (zn, zs) in zip(ranges, sizes):
        ln = np.zeros(max(b - a, 1), np.uint32)
        fl = np.zeros(max(b - a, 1), np.uint32)
        sz = (C.c_uint64 * 3)()
        _lib.after_torch()
        _check(so.fqz5_fastq_gather(text_d.data_ptr(), recs.data_ptr(), a, b,
                                    name_d.data_ptr() + no, seq_d.data_ptr() + so_,
                                    None if fasta else qual_d.data_ptr() + so_, ln.ctypes.data,
                                    fl.ctypes.data, sz),
               "fqz5_fastq_gather")
        if pair_flags:
            fl[:] = 0
            fl[1::2] = 128                  # FQZ_FREAD2 (a range starts at an R1 record)
        lens.append(ln[:b - a])
        flags.append(fl[:b - a])
        nr.append((no, no + zn))
        sr.append((so_, so_ + zs))
        no += zn
        so_ += zs
    return S.Run.from_device(name_d, seq_d, qual_d, nr, sr, lens, flags, bfa)


def compress_bytes(text: bytes, level: int = 3, blk_size: int | None = None,
                   device: str = "cuda", window_bytes: int | None = None) -> bytes:
    """fqzcomp5 -<level> (-t1 semantics) of FASTQ text, on the GPU."""
    sink = _Sink(None, True)
    _encode_stream([_Src(data=text)], sink, level, blk_size, device, None, window_bytes)
    return bytes(sink.mem)


def compress_paired_bytes(text1: bytes, text2: bytes, level: int = 3,
                          blk_size: int | None = None, device: str = "cuda",
                          window_bytes: int | None = None) -> bytes:
    """fqzcomp5 -<level> in1 in2 out (-t1 semantics): the two files'
    records interleaved (encode_interleaved, fqzcomp5.c:3211-3440)."""
    sink = _Sink(None, True)
    _encode_stream([_Src(data=text1), _Src(data=text2)], sink, level, blk_size, device, None,
                   window_bytes)
    return bytes(sink.mem)


def compress_file(src: str, dst: str, level: int = 3, blk_size: int | None = None,
                  device: str = "cuda", src2: str | None = None, group=None,
                  window_bytes: int | None = None) -> int:
    """fqzcomp5 -<level> src [src2] dst on the GPU(s): the input streamed in
    windows of whole records, each window's complete blocks coded and written
    behind the last (see above); src2: the R2 file of a pair, interleaved
    with src (fqzcomp5 in1 in2 out).  group: a torch.distributed group, one
    process per GPU, every rank calling with the same arguments; the file
    equals the single-process one byte for byte.  Returns the file size."""
    ws, rk = S._world(group)
    # every rank fails together (S.ranks_fail_together): the body's last
    # exchange is the final barrier, taken on every path
    with S.ranks_fail_together(group):
        if rk == 0:
            _Sink(dst, True).close()              # create / truncate before anyone writes
        _barrier(group)
        sink = _Sink(dst, False)
        srcs = [_Src(src)] + ([_Src(src2)] if src2 else [])
        try:
            n = _encode_stream(srcs, sink, level, blk_size, device, group, window_bytes)
        finally:
            sink.close()
            for s in srcs:
                s.close()
        _barrier(group)
        return n


V11, V10, VOLD = 0, 1, 2                        # read_header's results (fqzcomp5.c:2577)
MAGIC_V10 = b"FQZ5\x01\x00\x00\x00"             # :155


class Blocks(list):
    """Block byte ranges of a container, with its version: V11 (CRC field in
    every block), V10 or VOLD (none; VOLD files have no file header either)."""
    version = V11

    def __init__(self, ranges=(), version: int = V11):
        super().__init__(ranges)
        self.version = version


def _version_of(head: bytes, size: int):
    """read_header (fqzcomp5.c:2578-2603): (version, first block offset,
    index offset or 0).  A file with neither magic is the old headerless
    format: blocks from offset 0 to the end, no index.  Fewer than 8 bytes
    (an empty file included) is an error, as read_header's short fread of
    the magic is (:2581-2582)."""
    if len(head) < 8 or size < 8:
        raise ValueError("not an .fqz5 file: shorter than the 8-byte magic")
    if head[:8] in (MAGIC, MAGIC_V10):
        if len(head) < 16:
            raise ValueError("truncated .fqz5: no index offset after the magic")
        (idx,) = struct.unpack_from("<Q", head, 8)
        if idx > size or (idx and idx < 16):
            raise ValueError("truncated .fqz5: index offset past the end of the file")
        return (V11 if head[:8] == MAGIC else V10), 16, idx
    return VOLD, 0, 0


def _walk(read4, start: int, end: int, version: int) -> Blocks:
    """The block_size walk of decode (fqzcomp5.c:3769-3797) from `start` up
    to `end` (the index or the end of the file); a block that runs past it is
    an error (the reference's read fails there)."""
    hd = 12 if version == V11 else 8
    p, out = start, Blocks(version=version)
    while p < end:
        h = read4(p) if p + 4 <= end else b""
        if len(h) < 4:
            raise ValueError("truncated .fqz5: a block header runs past the end")
        (bsz,) = struct.unpack("<I", h)
        if p + 4 + bsz > end or bsz + 4 < hd:
            raise ValueError("truncated .fqz5: a block runs past the end of the file")
        out.append((p, p + 4 + bsz))
        p += 4 + bsz
    return out


def _blocks_of(data) -> Blocks:
    """Block byte ranges of a .fqz5 held in memory (any version the
    reference reads)."""
    data = memoryview(data).cast("B")
    version, start, idx = _version_of(bytes(data[:16]), len(data))
    return _walk(lambda p: bytes(data[p:p + 4]), start, idx if idx else len(data), version)


def block_fields(data, s: int, e: int, version: int = V11) -> dict:
    """The header fields of the block data[s:e] read on the host, as
    decode_block reads them (fqzcomp5.c:2290-2420): record count, the name,
    sequence and quality sections' sizes, the lengths section.  Raises
    ValueError when a field points past the block or the sizes disagree
    (the decoders write u_len bytes into outputs sized by these fields)."""
    d = memoryview(data).cast("B")

    def get(fmt, at):
        z = struct.calcsize(fmt)
        if at + z > e:
            raise ValueError("corrupt block: header runs past the block")
        return struct.unpack_from(fmt, d, at), at + z

    (bsz, nrec), p = get("<II", s)
    if version == V11:
        _crc, p = get("<I", p)
    if s + 4 + bsz != e:
        raise ValueError("corrupt block: block size field")
    (nu, _st, nc), p = get("<IBI", p)
    p += nc

    def varint(at, end):
        # var_get_u32 as the reference's lengths walk reads it
        # (fqzcomp5.c:2384-2404; csrc/rans_format.hpp varint_get): the bytes
        # it reads, not the header's own count, set the offsets
        if at >= end:
            raise ValueError("corrupt block: bad length varint")
        v = n = 0
        while True:
            c = d[at + n]
            n += 1
            v = ((v << 7) | (c & 0x7f)) & 0xffffffff
            if not (c & 0x80 and n < 6 and at + n < end):
                return v, at + n

    (nb,), p = get("<B", p)
    lens_sum = None
    if nb:
        fixed, p = varint(p, min(e, p + 5))
        lens_sum = fixed * nrec
    else:
        (_lz,), p = get("<I", p)
        lens_sum = 0
        end = min(e, p + 5 * nrec)
        for _ in range(nrec):
            x, p = varint(p, end)
            lens_sum += x
    (_s1, su, sc), p = get("<BII", p)
    p += sc
    (_s2, qu, qc), p = get("<BII", p)
    p += qc
    if p > e:
        raise ValueError("corrupt block: a section runs past the block")
    fasta = qu == 0 and qc == 0
    if not fasta and qu != su:
        raise ValueError("corrupt block: quality and sequence sizes differ")
    if lens_sum != su:
        raise ValueError("corrupt block: record lengths do not sum to the bases")
    return dict(nrec=nrec, name_ulen=nu, seq_ulen=su, qual_ulen=qu, fasta=fasta)


def check_blocks(data, ranges=None) -> list[dict]:
    """block_fields of every block (host only)."""
    if ranges is None:
        ranges = _blocks_of(data)
    v = getattr(ranges, "version", V11)
    return [block_fields(data, s, e, v) for s, e in ranges]


def _decode(data, buf, plus_name: bool, device: str, pairs: bool = False, ranges=None):
    """Blocks of a .fqz5 (host view `data`, device copy `buf`; `ranges` the
    block byte ranges within them, all blocks of the file by default) ->
    the FASTQ text of every block in one device buffer; pairs: (the R1
    text, the R2 text) of output_fastq_deinterleaved (fqzcomp5.c:3612-3676),
    even records of every block to R1 and odd ones to R2."""
    import torch
    so = _load()
    if ranges is None:
        ranges = _blocks_of(data)
    version = getattr(ranges, "version", V11)
    if not ranges:
        return torch.empty(0, dtype=torch.uint8, device=device)
    try:
        check_blocks(data, ranges)
    except ValueError as err:
        raise _lib.NativeError(str(err)) from None
    views, lens = [], []
    nrecs = [struct.unpack_from("<I", data, s + 4)[0] for s, _ in ranges]
    parsed = S.parse_blocks([buf.data_ptr() + s for s, _ in ranges], [e - s for s, e in ranges],
                            nrecs, version)
    for v, ln in parsed:
        if not v.crc_ok:
            raise _lib.NativeError("block CRC mismatch")
        # the decoders write u_len bytes into outputs sized by the block's
        # own fields: refuse fields that disagree (decode_block allocates
        # from them, fqzcomp5.c:2433-2519)
        if int(ln.astype(np.uint64).sum()) != v.seq_ulen:
            raise _lib.NativeError("corrupt block: record lengths do not sum to the bases")
        if not (v.qual_ulen == 0 and v.qual_size == 9) and v.qual_ulen != v.seq_ulen:
            raise _lib.NativeError("corrupt block: quality and sequence sizes differ")
        views.append(v)
        lens.append(ln)
    # FASTA: a quality section of u_len 0 and c_len 0 (decode_block,
    # fqzcomp5.c:2477-2483); the text is then output_fasta's (:3503-3517)
    fasta = [v.qual_ulen == 0 and v.qual_size == 9 for v in views]
    nsz = [v.name_ulen for v in views]
    ssz = [v.seq_ulen for v in views]
    out_d = torch.empty(sum(nsz) + 2 * sum(ssz) + 1, dtype=torch.uint8, device=device)
    secs, places = [], []
    o = 0
    base = buf.data_ptr()
    for (s, e), v, ln, fa in zip(ranges, views, lens, fasta):
        rl = ln.ctypes.data_as(C.POINTER(C.c_uint32))
        po = (o, o + v.name_ulen, o + v.name_ulen + v.seq_ulen)
        secs.append(S.Section(base + s + v.name_off, out_d.data_ptr() + po[0], v.name_size,
                              v.name_ulen, 0, S.SEC_NAME, rl, None, len(ln), None))
        secs.append(S.Section(base + s + v.seq_off, out_d.data_ptr() + po[1], v.seq_size,
                              v.seq_ulen, 0, S.SEC_SEQ, rl, None, len(ln), None))
        if not fa:
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
    for v, ln, po, fa in zip(views, lens, places, fasta):
        size, s1 = C.c_uint64(0), C.c_uint64(0)
        a = (out_d.data_ptr() + po[0], v.name_ulen, out_d.data_ptr() + po[1],
             None if fa else out_d.data_ptr() + po[2], ln.ctypes.data, len(ln),
             int(plus_name))
        _check(fmt(*a, None, 0, C.byref(size), *((C.byref(s1),) if pairs else ())),
               "fqz5_fastq_format")
        args.append(a)
        sizes.append(int(size.value))
        r1.append(int(s1.value))
    text = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device=device)
    _lib.after_torch(device)
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


def _file_blocks(f, size: int) -> Blocks:
    """Block byte ranges of a .fqz5 file (any version the reference reads),
    walking the block size fields up to the index; checked against the file
    size."""
    f.seek(0)
    version, start, idx = _version_of(f.read(16), size)

    def read4(p):
        f.seek(p)
        return f.read(4)
    return _walk(read4, start, idx if idx else size, version)


def _block_text_size(f, s: int, e: int, plus_name: bool, version: int = V11) -> int:
    """The FASTQ (or FASTA) text size of block [s, e) of an open .fqz5, from
    its headers alone (a few small reads): output_fastq writes '@' name '\n'
    seq '\n' '+' [name] '\n' qual '\n' per record (fqzcomp5.c:3441-3480),
    output_fasta '>' name '\n' seq '\n' (:3503-3517); the name section
    decodes to each name and a '\0'."""
    hd = 12 if version == V11 else 8
    f.seek(s)
    h = f.read(hd + 9)
    if len(h) < hd + 9:
        raise ValueError("truncated .fqz5: a block header runs past the end")
    nrec, = struct.unpack_from("<I", h, 4)
    name_ulen, = struct.unpack_from("<I", h, hd)
    c_len, = struct.unpack_from("<I", h, hd + 5)
    p = s + hd + 9 + c_len
    f.seek(p)
    nb = f.read(1)
    if not nb:
        raise ValueError("truncated .fqz5: lengths past the block")
    if nb[0]:
        vl = f.read(5)
        n = 1
        while n < len(vl) and vl[n - 1] & 0x80:
            n += 1
        p += 1 + n
    else:
        # [0][u32][a varint per record]: walk them (read in one go)
        f.seek(p + 5)
        v = f.read(min(5 * nrec, max(e - p - 5, 0)))
        k = 0
        for _ in range(nrec):
            while k < len(v) and v[k] & 0x80:
                k += 1
            k += 1
        p += 5 + k
    f.seek(p)
    sh = f.read(9)
    if len(sh) < 9:
        raise ValueError("truncated .fqz5: sequence header past the block")
    seq_ulen, seq_clen = struct.unpack_from("<II", sh, 1)
    f.seek(p + 9 + seq_clen)
    qh = f.read(9)
    if len(qh) < 9:
        raise ValueError("truncated .fqz5: quality header past the block")
    qual_ulen, qual_clen = struct.unpack_from("<II", qh, 1)
    names = name_ulen - nrec
    if qual_ulen == 0 and qual_clen == 0:                    # FASTA
        return names + seq_ulen + 2 * nrec
    return names * (2 if plus_name else 1) + 2 * seq_ulen + 6 * nrec


def decompress_file(src: str, dst: str, plus_name: bool = False, device: str = "cuda",
                    dst2: str | None = None, group=None, window_bytes: int | None = None) -> int:
    """fqzcomp5 -d src dst [dst2] on the GPU(s): blocks read and decoded in
    windows of at most `window_bytes` of compressed data (the reference
    decodes block by block, fqzcomp5.c:3754-3800), the text written behind
    the last.  dst2: deinterleave, R1 records to dst and R2 records to dst2
    (fqzcomp5 -d in out1 out2).  group: one process per GPU, the blocks split
    contiguously over the ranks; every window's text goes out as soon as it
    is decoded (host memory stays one window): at its offset from the block
    headers' text sizes (one output), or into a per-rank spill file copied
    into place at the end (R1/R2: the split of a block's text between the two
    files needs its decoded names).  Returns the text bytes written."""
    import os
    ws, rk = S._world(group)
    with S.ranks_fail_together(group):
        outs = [dst] + ([dst2] if dst2 is not None else [])
        if ws > 1 and any(d.endswith(".gz") for d in outs):
            raise ValueError("gzip output needs a single process")
        size = os.path.getsize(src)
        single = ws == 1
        spill = not single and dst2 is not None
        with open(src, "rb") as f:
            with _stage("index"):
                ranges = _file_blocks(f, size)
            nb = len(ranges)
            mine = [b for b in range(nb) if (b * ws) // max(nb, 1) == rk] if nb else []
            wb = window_bytes or DEFAULT_WINDOW
            groups, cur, tot = [], [], 0
            for b in mine:
                z = ranges[b][1] - ranges[b][0]
                if cur and tot + z > wb:
                    groups.append(cur)
                    cur, tot = [], 0
                cur.append(b)
                tot += z
            if cur:
                groups.append(cur)
            gz = [d.endswith(".gz") for d in outs]
            streams, sinks, at = [], [], 0
            plain = []                        # single process: plain outputs by positioned writes
            st_open = _stage("open")
            st_open.__enter__()
            if single:
                import gzip
                streams = [gzip.GzipFile(filename="", mode="wb", compresslevel=6, mtime=0,
                                         fileobj=open(d, "wb")) if z else None
                           for d, z in zip(outs, gz)]
                plain = [None if z else _Sink(d, True) for d, z in zip(outs, gz)]
            elif spill:
                streams = [open(f"{d}.part{rk}", "wb") for d in outs]
            else:
                # one output: every block's text size from its headers, so this
                # rank's text starts at the sum over the blocks before its first
                sizes = [_block_text_size(f, s, e, plus_name, ranges.version) for s, e in ranges]
                at = sum(sizes[:mine[0]]) if mine else 0
                if rk == 0:
                    _Sink(dst, True).close()
                _barrier(group)
                sinks = [_Sink(dst, False)]
            st_open.__exit__()
            written = [0 for _ in outs]
            try:
                for gb in groups:
                    a, e = ranges[gb[0]][0], ranges[gb[-1]][1]
                    with _stage("read"):
                        host = _pinned(e - a)
                        f.seek(a)
                        mv = memoryview(host.numpy())
                        got = 0
                        while got < e - a:
                            k = f.readinto(mv[got:])
                            if not k:
                                raise OSError(f"{src}: short read")
                            got += k
                        hv = host.numpy()
                    with _stage("upload"):
                        buf = host.to(device)      # blocking: block parsing runs on the library's streams
                    with _stage("decode"):
                        texts = _decode(hv, buf, plus_name, device, pairs=dst2 is not None,
                                        ranges=Blocks([(ranges[b][0] - a, ranges[b][1] - a)
                                                       for b in gb], ranges.version))
                    if dst2 is None:
                        texts = (texts,)
                    for j, t in enumerate(texts):
                        with _stage("download"):
                            out = _pinned(int(t.numel()))
                            out.copy_(t)
                        st_w = _stage("write")
                        st_w.__enter__()
                        if sinks:
                            want = sum(sizes[b] for b in gb)
                            if int(t.numel()) != want:
                                raise _lib.NativeError("decoded text size differs from the block headers'")
                            sinks[j].write_at(at + written[j], out.numpy())
                        elif plain and plain[j] is not None:
                            plain[j].write_at(written[j], out.numpy())
                        else:
                            streams[j].write(memoryview(out.numpy()))
                        written[j] += int(t.numel())
                        st_w.__exit__()
                        del out
                    with _stage("free"):
                        del buf, host, texts
            finally:
                st_close = _stage("close")
                st_close.__enter__()
                for sk in plain:
                    if sk is not None:
                        sk.close()
                for st in streams:
                    if st is None:
                        continue
                    if isinstance(st, __import__("gzip").GzipFile):
                        raw = st.fileobj          # (close() drops the reference)
                        st.close()
                        raw.close()
                    else:
                        st.close()
                for sk in sinks:
                    sk.close()
                st_close.__exit__()
        _trace_dump("decode")
        if single:
            return sum(written)
        all_w = _allgather_obj(written, group)
        if spill:
            # the spill files into place at their offsets from the ranks' sizes
            for j, d in enumerate(outs):
                if rk == 0:
                    _Sink(d, True).close()
            _barrier(group)
            for j, d in enumerate(outs):
                off = sum(w[j] for w in all_w[:rk])
                sink = _Sink(d, False)
                part = f"{d}.part{rk}"
                try:
                    with open(part, "rb") as pf:
                        for c in iter(lambda: pf.read(1 << 26), b""):
                            sink.write_at(off, c)
                            off += len(c)
                finally:
                    sink.close()
                    os.unlink(part)
        _barrier(group)
        return sum(sum(w) for w in all_w)


def _write_out(path: str, data) -> None:
    """Decoded text to `path`; gzip-compressed when the name ends in ".gz"
    (gzopen(name, "wb"), zlib's default level, fqzcomp5.c:5113-5160)."""
    if path.endswith(".gz"):
        import gzip
        # no file name and mtime 0 in the header, as zlib's gzopen writes it
        with open(path, "wb") as raw, gzip.GzipFile(filename="", mode="wb", compresslevel=6,
                                                    mtime=0, fileobj=raw) as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)
