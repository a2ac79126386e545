"""ctypes binding of libfqz5_mi355x.so (include/fqz5_mi355x.h).

This is the only way the Python side reaches the codec: every call goes to
the HIP library.  There is no fallback — if the library or a GPU is missing
the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfqz5_mi355x.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

# helper contexts' streams need queues of their own (bench.py); effective
# only when nothing in the process has initialised HIP yet
# (the rule of capi.cpp's hw_queues_default: FQZ5_HW_QUEUES as given, else
# an unset value or HIP's default of 4 raised to 20, any other value kept)
if os.environ.get("FQZ5_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["FQZ5_HW_QUEUES"]
elif os.environ.get("GPU_MAX_HW_QUEUES", "") in ("", "4"):
    os.environ["GPU_MAX_HW_QUEUES"] = "20"

_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]


class RansJob(C.Structure):
    _fields_ = [("in_", C.c_void_p), ("out", C.c_void_p),
                ("in_size", C.c_uint32), ("out_cap", C.c_uint32),
                ("order", C.c_int32), ("out_size", C.c_uint32),
                ("status", C.c_int32), ("pad", C.c_int32)]


class FqzSlice(C.Structure):
    """fqz_slice (include/fqz5_mi355x.h; htscodecs fqzcomp_qual.h:59-64)."""
    _fields_ = [("num_records", C.c_int),
                ("len", C.POINTER(C.c_uint32)),
                ("flags", C.POINTER(C.c_uint32)),
                ("seq", C.POINTER(C.c_void_p))]


class NativeError(RuntimeError):
    pass


_lib = None


def load() -> C.CDLL:
    """Load the native library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("FQZ5_LIB_VARIANT") or LIB_PATH   # tools/build_variant.sh
    # torch bundles its own HIP runtime, and the package's device buffers
    # (sections.py, fqz5file.py) are torch tensors: its runtime must own the
    # device before this library's runtime starts (started the other way
    # round, torch later finds no GPU)
    try:
        import torch
    except ImportError:
        torch = None
    if torch is not None and torch.cuda.is_available():
        torch.cuda.init()
    if not os.path.exists(path):
        raise NativeError(f"{path} missing: run __graft_entry__.build()")
    lib = C.CDLL(path)
    lib.fqz5_set_hedge.restype = C.c_int
    lib.fqz5_set_hedge.argtypes = [C.c_int]
    lib.fqz5_set_dec_small.restype = C.c_int
    lib.fqz5_set_dec_small.argtypes = [C.c_int]
    lib.fqz5_set_host_decode.restype = C.c_int
    lib.fqz5_set_host_decode.argtypes = [C.c_int]
    lib.fqz5_host_threads.restype = C.c_int
    lib.fqz5_host_threads.argtypes = []
    lib.fqz5_set_hot_min.restype = C.c_uint
    lib.fqz5_set_hot_min.argtypes = [C.c_uint]
    lib.rans_compress_bound_4x16.restype = C.c_uint
    lib.rans_compress_bound_4x16.argtypes = [C.c_uint, C.c_int]
    lib.rans_compress_to_4x16.restype = C.c_void_p
    lib.rans_compress_to_4x16.argtypes = [C.c_char_p, C.c_uint, C.c_void_p,
                                          C.POINTER(C.c_uint), C.c_int]
    lib.rans_compress_4x16.restype = C.c_void_p
    lib.rans_compress_4x16.argtypes = [C.c_char_p, C.c_uint,
                                       C.POINTER(C.c_uint), C.c_int]
    lib.rans_uncompress_to_4x16.restype = C.c_void_p
    lib.rans_uncompress_to_4x16.argtypes = [C.c_char_p, C.c_uint, C.c_void_p,
                                            C.POINTER(C.c_uint)]
    lib.rans_uncompress_4x16.restype = C.c_void_p
    lib.rans_uncompress_4x16.argtypes = [C.c_char_p, C.c_uint,
                                         C.POINTER(C.c_uint)]
    lib.fqz5_rans_compress_batch.restype = C.c_int
    lib.fqz5_rans_compress_batch.argtypes = [C.POINTER(RansJob), C.c_int]
    lib.fqz5_rans_uncompress_batch.restype = C.c_int
    lib.fqz5_rans_uncompress_batch.argtypes = [C.POINTER(RansJob), C.c_int]
    lib.fqz5_stream.restype = C.c_void_p
    lib.fqz5_stream_wait.restype = C.c_int
    lib.fqz5_stream_wait.argtypes = [C.c_void_p]
    lib.fqz5_device_ok.restype = C.c_int
    lib.fqz5_last_error.restype = C.c_char_p
    lib.fqz_compress.restype = C.c_void_p
    lib.fqz_compress.argtypes = [C.c_int, C.POINTER(FqzSlice), C.c_char_p, C.c_size_t,
                                 C.POINTER(C.c_size_t), C.c_int, C.c_void_p]
    lib.fqz_decompress.restype = C.c_void_p
    lib.fqz_decompress.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t),
                                   C.POINTER(C.c_int), C.c_int, C.POINTER(FqzSlice)]
    lib.arith_compress_bound.restype = C.c_uint
    lib.arith_compress_bound.argtypes = [C.c_uint, C.c_int]
    lib.arith_compress_to.restype = C.c_void_p
    lib.arith_compress_to.argtypes = [C.c_char_p, C.c_uint, C.c_void_p,
                                      C.POINTER(C.c_uint), C.c_int]
    lib.arith_compress.restype = C.c_void_p
    lib.arith_compress.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint), C.c_int]
    lib.arith_uncompress_to.restype = C.c_void_p
    lib.arith_uncompress_to.argtypes = [C.c_char_p, C.c_uint, C.c_void_p,
                                        C.POINTER(C.c_uint)]
    lib.arith_uncompress.restype = C.c_void_p
    lib.arith_uncompress.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint)]
    lib.fqz5_crc32.restype = C.c_ulong
    lib.fqz5_crc32.argtypes = [C.c_ulong, C.c_char_p, C.c_uint]
    lib.fqz5_crc32_dev.restype = C.c_int
    lib.fqz5_crc32_dev.argtypes = [C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32)]
    lib.fqz5_seq_encode.restype = C.c_void_p
    lib.fqz5_seq_encode.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint32), C.c_int,
                                    C.c_int, C.c_int, C.POINTER(C.c_uint)]
    lib.fqz5_seq_decode.restype = C.c_void_p
    lib.fqz5_seq_decode.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint32), C.c_int,
                                    C.c_int, C.c_int, C.c_uint]
    lib.fqz5_seq_decode_host.restype = C.c_void_p
    lib.fqz5_seq_decode_host.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint32), C.c_int,
                                    C.c_int, C.c_int, C.c_uint]
    lib.fqz5_fqz_decompress_host.restype = C.c_void_p
    lib.fqz5_fqz_decompress_host.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t),
                                   C.POINTER(C.c_int), C.c_int, C.POINTER(FqzSlice)]
    _lib = lib
    return lib


def last_error() -> str:
    return load().fqz5_last_error().decode()


def fqz_div_selftest() -> int:
    """Mismatches of the fqz decoder's division on the device (0 expected)."""
    so = load()
    so.fqz5_fqz_div_selftest.restype = C.c_long
    return int(so.fqz5_fqz_div_selftest())


def device_ok() -> bool:
    return bool(load().fqz5_device_ok())


def arena_bytes() -> int:
    """Device bytes the arenas hold, process-wide (fqz5_arena_bytes)."""
    so = load()
    so.fqz5_arena_bytes.restype = C.c_uint64
    return int(so.fqz5_arena_bytes())


def arena_peak(reset: bool = False) -> int:
    """The most device bytes the arenas held since the last reset
    (fqz5_arena_peak)."""
    so = load()
    so.fqz5_arena_peak.restype = C.c_uint64
    so.fqz5_arena_peak.argtypes = [C.c_int]
    return int(so.fqz5_arena_peak(1 if reset else 0))


def arena_use_peak(reset: bool = False) -> int:
    """The most device bytes in use at once (held minus the pool's idle
    chunks) since the last reset (fqz5_arena_use_peak)."""
    so = load()
    so.fqz5_arena_use_peak.restype = C.c_uint64
    so.fqz5_arena_use_peak.argtypes = [C.c_int]
    return int(so.fqz5_arena_use_peak(1 if reset else 0))


def header_symbols() -> list[str]:
    """Function names declared in include/*.h."""
    import glob
    import re
    txt = "".join(open(f).read() for f in sorted(glob.glob(os.path.join(INCLUDE, "*.h"))))
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b([a-z_0-9]+)\s*\(", txt))
                  - {"if", "sizeof", "return"})


def compress_bound(n: int, order: int) -> int:
    return load().rans_compress_bound_4x16(n, order)


def rans_compress(data: bytes, order: int) -> bytes:
    """rans_compress_4x16 on the GPU (host buffers)."""
    lib = load()
    n = C.c_uint(0)
    p = lib.rans_compress_4x16(bytes(data), len(data), C.byref(n), order)
    if not p:
        raise NativeError("rans_compress_4x16 failed: " + last_error())
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out


def rans_compress_to(data: bytes, order: int, cap: int) -> bytes | None:
    """rans_compress_to_4x16 with a caller buffer of `cap` bytes."""
    lib = load()
    buf = C.create_string_buffer(max(cap, 1))
    n = C.c_uint(cap)
    p = lib.rans_compress_to_4x16(bytes(data), len(data), buf, C.byref(n),
                                  order)
    if not p:
        return None
    return buf.raw[:n.value]


def rans_uncompress(comp: bytes) -> bytes:
    lib = load()
    n = C.c_uint(0)
    p = lib.rans_uncompress_4x16(bytes(comp), len(comp), C.byref(n))
    if not p:
        raise NativeError("rans_uncompress_4x16 failed: " + last_error())
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out


def rans_uncompress_to(comp: bytes, size: int) -> bytes | None:
    lib = load()
    buf = C.create_string_buffer(max(size, 1))
    n = C.c_uint(size)
    p = lib.rans_uncompress_to_4x16(bytes(comp), len(comp), buf, C.byref(n))
    if not p:
        return None
    return buf.raw[:n.value]


def arith_compress(data: bytes, order: int, cap: int | None = None) -> bytes | None:
    """arith_compress (cap None) or arith_compress_to with a caller buffer
    of `cap` bytes, on the GPU; None where the reference returns NULL."""
    lib = load()
    if cap is None:
        n = C.c_uint(0)
        p = lib.arith_compress(bytes(data), len(data), C.byref(n), order)
        if not p:
            return None
        out = C.string_at(p, n.value)
        _libc.free(p)
        return out
    buf = C.create_string_buffer(max(cap, 1))
    n = C.c_uint(cap)
    p = lib.arith_compress_to(bytes(data), len(data), buf, C.byref(n), order)
    return None if not p else buf.raw[:n.value]


def arith_uncompress(comp: bytes, out_size: int | None = None) -> bytes | None:
    """arith_uncompress (out_size None) or arith_uncompress_to into a
    buffer of out_size bytes, on the GPU; None on failure."""
    lib = load()
    if out_size is None:
        n = C.c_uint(0)
        p = lib.arith_uncompress(bytes(comp), len(comp), C.byref(n))
        if not p:
            return None
        out = C.string_at(p, n.value)
        _libc.free(p)
        return out
    buf = C.create_string_buffer(max(out_size, 1))
    n = C.c_uint(out_size)
    p = lib.arith_uncompress_to(bytes(comp), len(comp), buf, C.byref(n))
    return None if not p else buf.raw[:n.value]


def compress_batch_dev(jobs: list[RansJob]) -> None:
    arr = (RansJob * len(jobs))(*jobs)
    if load().fqz5_rans_compress_batch(arr, len(jobs)) != 0:
        raise NativeError("fqz5_rans_compress_batch: " + last_error())
    for i, j in enumerate(jobs):
        j.out_size, j.status = arr[i].out_size, arr[i].status


def uncompress_batch_dev(jobs: list[RansJob]) -> None:
    arr = (RansJob * len(jobs))(*jobs)
    if load().fqz5_rans_uncompress_batch(arr, len(jobs)) != 0:
        raise NativeError("fqz5_rans_uncompress_batch: " + last_error())
    for i, j in enumerate(jobs):
        j.out_size, j.status = arr[i].out_size, arr[i].status


def _fqz_slice(lens, flags, seq: bytes | None):
    """Build an fqz_slice over numpy-like lens/flags (uint32, modified in
    place by fqz_compress as the reference does) and optional sequences."""
    import numpy as np
    lens = np.ascontiguousarray(lens, np.uint32)
    flags = np.ascontiguousarray(flags, np.uint32)
    nr = len(lens)
    keep = [lens, flags]
    S = None
    if seq is not None:
        sb = C.create_string_buffer(bytes(seq), len(seq) + 1)
        keep.append(sb)
        base = C.addressof(sb)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
        S = (C.c_void_p * max(nr, 1))(*[base + int(o) for o in offs[:-1]])
        keep.append(S)
    s = FqzSlice(nr, lens.ctypes.data_as(C.POINTER(C.c_uint32)),
                 flags.ctypes.data_as(C.POINTER(C.c_uint32)), S)
    return s, keep, lens, flags


def fqz_compress(qual: bytes, lens, flags, strat: int, seq: bytes | None = None,
                 vers: int = 4) -> bytes:
    """fqz_compress on the GPU (host buffers; values are q-33)."""
    s, keep, _, _ = _fqz_slice(lens, flags, seq)
    n = C.c_size_t(0)
    p = load().fqz_compress(vers, C.byref(s), bytes(qual), len(qual), C.byref(n), strat, None)
    if not p:
        raise NativeError("fqz_compress failed: " + last_error())
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out


def fqz_decompress(comp: bytes, lens=None, flags=None, seq: bytes | None = None,
                   host: bool = False):
    """fqz_decompress on the GPU (host=True: fqz5_fqz_decompress_host, the
    same decoder on a host core); returns (bytes, record lengths)."""
    import numpy as np
    lens = np.zeros(0, np.uint32) if lens is None else lens
    flags = np.zeros(len(lens), np.uint32) if flags is None else flags
    s, keep, lens_a, _ = _fqz_slice(lens, flags, seq)
    n = C.c_size_t(0)
    nl = len(lens_a)
    L = (C.c_int * max(nl, 1))()
    so = load()
    fn = so.fqz5_fqz_decompress_host if host else so.fqz_decompress
    p = fn(bytes(comp), len(comp), C.byref(n), L, nl, C.byref(s))
    if not p:
        raise NativeError("fqz_decompress failed: " + last_error())
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out, [L[i] for i in range(nl)]


def _seq_lens(lens):
    lens = [int(x) for x in lens] or [0]
    return (C.c_uint32 * len(lens))(*lens), len(lens)


def seq_encode(seq: bytes, lens, both: int, k: int) -> bytes:
    """fqz5_seq_encode (encode_seq, fqzcomp5.c:1073) on the GPU."""
    la, nr = _seq_lens(lens)
    n = C.c_uint(0)
    p = load().fqz5_seq_encode(bytes(seq), len(seq), la, nr, both, k, C.byref(n))
    if not p:
        raise NativeError("fqz5_seq_encode failed: " + last_error())
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out


def seq_decode(comp: bytes, lens, both: int, k: int, out_size: int, host: bool = False) -> bytes:
    """fqz5_seq_decode (decode_seq, fqzcomp5.c:1272) on the GPU (host=True:
    fqz5_seq_decode_host on a host core)."""
    la, nr = _seq_lens(lens)
    so = load()
    fn = so.fqz5_seq_decode_host if host else so.fqz5_seq_decode
    p = fn(bytes(comp), len(comp), la, nr, both, k, out_size)
    if not p:
        raise NativeError("fqz5_seq_decode failed: " + last_error())
    out = C.string_at(p, out_size)
    _libc.free(p)
    return out


def lzp(data: bytes) -> bytes:
    """fqz5_lzp (lzp16e.c:113 lzp) on the GPU."""
    so = load()
    so.fqz5_lzp.restype = C.c_int
    so.fqz5_lzp.argtypes = [C.c_char_p, C.c_int, C.c_void_p]
    buf = C.create_string_buffer(3 * len(data) + 16)
    n = so.fqz5_lzp(bytes(data), len(data), buf)
    if n < 0:
        raise NativeError("fqz5_lzp failed: " + last_error())
    return buf.raw[:n]


def unlzp(data: bytes, out_cap: int) -> bytes | None:
    """fqz5_unlzp (lzp16e.c:166 unlzp) on the GPU; None if the stream is
    damaged or decodes to more than out_cap bytes."""
    so = load()
    so.fqz5_unlzp.restype = C.c_int
    so.fqz5_unlzp.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int]
    buf = C.create_string_buffer(max(out_cap, 1))
    n = so.fqz5_unlzp(bytes(data), len(data), buf, out_cap)
    return None if n < 0 else buf.raw[:n]


def crc32(data: bytes, crc: int = 0) -> int:
    """zlib.crc32 computed on the GPU (fqz5_crc32, host buffer)."""
    return int(load().fqz5_crc32(crc, bytes(data), len(data)))


def stream_wait(stream: int) -> None:
    """Order the library's stream after the work enqueued so far on
    `stream` (a hipStream_t as int, e.g. torch's Stream.cuda_stream):
    fqz5_stream_wait, the ordering contract of the device-pointer calls."""
    if load().fqz5_stream_wait(C.c_void_p(stream)):
        raise NativeError("fqz5_stream_wait failed: " + last_error())


def after_torch(dev=None) -> None:
    """The ordering contract of the device-pointer calls for buffers torch
    made: the calling thread's library streams (and its helper contexts')
    wait, device-side, for the work enqueued so far on torch's current
    stream of the current device and, when `dev` (the device of the buffers
    the call reads) is another one, on that device's current stream too (a
    torch.cat output, a buffer the caching allocator reused).  Called before
    every device-pointer entry point of sections / fqz5file; a no-op while
    torch has not initialised the GPU."""
    import sys
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return
    cur = torch.cuda.current_device()
    stream_wait(torch.cuda.current_stream(cur).cuda_stream)
    if dev is not None:
        d = torch.device(dev)
        if d.type == "cuda" and d.index is not None and d.index != cur:
            stream_wait(torch.cuda.current_stream(d).cuda_stream)


def crc32_dev(ptr: int, n: int, crc: int = 0) -> int:
    """crc32 of n device bytes at ptr (fqz5_crc32_dev)."""
    out = C.c_uint32(0)
    if load().fqz5_crc32_dev(crc, C.c_void_p(ptr), n, C.byref(out)):
        raise NativeError("fqz5_crc32_dev failed: " + last_error())
    return int(out.value)


def tok3_encode(names: bytes, level: int, use_arith: int = 0):
    """tok3_encode_names (tokenise_name3.c:1451): tokenised on the host, the
    token streams entropy coded as one GPU batch.  Works on a private copy
    of `names` (the codec rewrites terminators): (stream, last_start), or
    None where the reference returns NULL."""
    so = load()
    f = so.tok3_encode_names
    f.restype = C.c_void_p
    f.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                  C.POINTER(C.c_int)]
    buf = C.create_string_buffer(bytes(names), max(len(names), 1))
    n, ls = C.c_int(0), C.c_int(-1)
    p = f(buf, len(names), level, use_arith, C.byref(n), C.byref(ls))
    if not p:
        return None
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out, ls.value


def tok3_decode(comp: bytes) -> bytes | None:
    """tok3_decode_names (tokenise_name3.c:1679): the '\\0'-terminated
    names, or None on a malformed stream."""
    so = load()
    f = so.tok3_decode_names
    f.restype = C.c_void_p
    f.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
    n = C.c_uint32(0)
    p = f(bytes(comp), len(comp), C.byref(n))
    if not p:
        return None
    out = C.string_at(p, n.value)
    _libc.free(p)
    return out
