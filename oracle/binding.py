"""ctypes bindings to the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.
Nothing in ``fqzcomp5_amd`` imports it; the product path never touches it.

Two libraries share the htscodecs C-ABI signatures
(htscodecs/rANS_static4x16.h:41-50, fqzcomp_qual.h:155-170):

* ``liboracle.so``        our plain-C restatement (oracle/*.c), symbols
                          prefixed ``ora_``;
* ``_ref/libhtsref.so``   the reference compiled from /root/reference by
                          oracle/Makefile (absent unless built here).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libhtsref.so")
REF_BIN = os.path.join(HERE, "_ref", "fqzcomp5")

_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]


class FqzSlice(C.Structure):
    # htscodecs/fqzcomp_qual.h:59-64 (fork ABI)
    _fields_ = [("num_records", C.c_int),
                ("len", C.POINTER(C.c_uint32)),
                ("flags", C.POINTER(C.c_uint32)),
                ("seq", C.POINTER(C.c_void_p))]


class _Codec:
    def __init__(self, path: str, prefix: str):
        self.path = path
        self.lib = C.CDLL(path)
        self._prefix = prefix
        p = prefix
        f = getattr(self.lib, p + "rans_compress_4x16")
        f.restype = C.c_void_p
        f.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint), C.c_int]
        self._rc = f
        f = getattr(self.lib, p + "rans_uncompress_4x16")
        f.restype = C.c_void_p
        f.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint)]
        self._ru = f
        self._fc = getattr(self.lib, p + "fqz_compress", None)
        if self._fc is not None:
            self._fc.restype = C.c_void_p
            self._fc.argtypes = [C.c_int, C.POINTER(FqzSlice), C.c_char_p,
                                 C.c_size_t, C.POINTER(C.c_size_t), C.c_int,
                                 C.c_void_p]
        self._fd = getattr(self.lib, p + "fqz_decompress", None)
        if self._fd is not None:
            self._fd.restype = C.c_void_p
            self._fd.argtypes = [C.c_char_p, C.c_size_t,
                                 C.POINTER(C.c_size_t), C.POINTER(C.c_int),
                                 C.c_int, C.POINTER(FqzSlice)]

    def _arith(self):
        if getattr(self, "_ac", None) is None:
            p = self._prefix
            f = getattr(self.lib, p + "arith_compress_to")
            f.restype = C.c_void_p
            f.argtypes = [C.c_char_p, C.c_uint, C.c_void_p, C.POINTER(C.c_uint), C.c_int]
            self._ac = f
            g = getattr(self.lib, p + "arith_uncompress_to")
            g.restype = C.c_void_p
            g.argtypes = [C.c_char_p, C.c_uint, C.c_void_p, C.POINTER(C.c_uint)]
            self._au = g
            b = getattr(self.lib, p + "arith_compress_bound")
            b.restype = C.c_uint
            b.argtypes = [C.c_uint, C.c_int]
            self._ab = b
        return self._ac, self._au, self._ab

    def arith_compress_bound(self, n: int, order: int) -> int:
        return int(self._arith()[2](n, order))

    def arith_compress(self, data: bytes, order: int, cap: int | None = None):
        """arith_compress_to; None when it returns NULL.  cap: caller buffer."""
        ac, _, _ = self._arith()
        if cap is None:
            n = C.c_uint(0)
            p = ac(bytes(data), len(data), None, C.byref(n), order)
            return None if not p else self._take(p, n.value)
        buf = C.create_string_buffer(max(cap, 1))
        n = C.c_uint(cap)
        p = ac(bytes(data), len(data), buf, C.byref(n), order)
        return None if not p else buf.raw[:n.value]

    def arith_uncompress(self, comp: bytes, out_size: int | None = None):
        """arith_uncompress_to; with out_size a caller buffer of that size."""
        _, au, _ = self._arith()
        if out_size is None:
            n = C.c_uint(0)
            p = au(bytes(comp), len(comp), None, C.byref(n))
            return None if not p else self._take(p, n.value)
        buf = C.create_string_buffer(max(out_size, 1))
        n = C.c_uint(out_size)
        p = au(bytes(comp), len(comp), buf, C.byref(n))
        return None if not p else buf.raw[:n.value]

    @staticmethod
    def _take(ptr, n) -> bytes:
        if not ptr:
            raise RuntimeError("codec returned NULL")
        b = C.string_at(ptr, n)
        _libc.free(ptr)
        return b

    def rans_compress(self, data: bytes, order: int) -> bytes:
        n = C.c_uint(0)
        p = self._rc(bytes(data), len(data), C.byref(n), order)
        return self._take(p, n.value)

    def rans_uncompress(self, comp: bytes) -> bytes:
        n = C.c_uint(0)
        p = self._ru(bytes(comp), len(comp), C.byref(n))
        return self._take(p, n.value)

    def tok3_encode(self, names: bytes, level: int, use_arith: int = 0):
        """tok3_encode_names (tokenise_name3.c:1451) on a private copy of
        `names`: (stream, last_start), or None where it returns NULL."""
        f = getattr(self.lib, self._prefix + "tok3_encode_names")
        f.restype = C.c_void_p
        f.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                      C.POINTER(C.c_int)]
        buf = C.create_string_buffer(bytes(names), max(len(names), 1))
        n, ls = C.c_int(0), C.c_int(-1)
        p = f(buf, len(names), level, use_arith, C.byref(n), C.byref(ls))
        return None if not p else (self._take(p, n.value), ls.value)

    def tok3_decode(self, comp: bytes):
        """tok3_decode_names (tokenise_name3.c:1679): the '\\0'-terminated
        names, or None."""
        f = getattr(self.lib, self._prefix + "tok3_decode_names")
        f.restype = C.c_void_p
        f.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
        n = C.c_uint32(0)
        p = f(bytes(comp), len(comp), C.byref(n))
        return None if not p else self._take(p, n.value)

    def _slice(self, lens, flags, seq: bytes | None):
        import numpy as np
        nr = len(lens)
        L = (C.c_uint32 * nr)(*[int(x) for x in lens])
        Fl = (C.c_uint32 * nr)(*[int(x) for x in flags])
        keep = [L, Fl]
        S = None
        if seq is not None:
            sb = C.create_string_buffer(bytes(seq), len(seq) + 1)
            keep.append(sb)
            base = C.addressof(sb)
            offs = np.concatenate([[0], np.cumsum(np.asarray(lens, np.int64))])
            S = (C.c_void_p * nr)(*[base + int(o) for o in offs[:-1]])
            keep.append(S)
        s = FqzSlice(nr, L, Fl, S)
        return s, keep

    def fqz_compress(self, qual: bytes, lens, flags, strat: int,
                     seq: bytes | None = None, vers: int = 4) -> bytes:
        s, keep = self._slice(lens, flags, seq)
        n = C.c_size_t(0)
        p = self._fc(vers, C.byref(s), bytes(qual), len(qual), C.byref(n),
                     strat, None)
        return self._take(p, n.value)

    def fqz_decompress(self, comp: bytes, lens, flags,
                       seq: bytes | None = None) -> bytes:
        s, keep = self._slice(lens, flags, seq)
        n = C.c_size_t(0)
        nl = len(lens)
        Larr = (C.c_int * max(nl, 1))()
        p = self._fd(bytes(comp), len(comp), C.byref(n), Larr, nl,
                     C.byref(s))
        return self._take(p, n.value)


    # ---- LZP (lzp16e.c) and LZP3 (fqzcomp5.c:2013-2021, :2431-2445) -------
    def _lzp_fns(self):
        if getattr(self, "_lz", None) is None:
            p = self._prefix
            f = getattr(self.lib, p + "lzp")
            f.restype = C.c_int
            f.argtypes = [C.c_char_p, C.c_int, C.c_void_p]
            g = getattr(self.lib, p + "unlzp")
            g.restype = C.c_int
            # the reference's unlzp has no capacity argument (extra args are
            # harmless under the C calling convention)
            g.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int]
            self._lz = (f, g)
        return self._lz

    def lzp(self, data: bytes) -> bytes:
        f, _ = self._lzp_fns()
        buf = C.create_string_buffer(3 * len(data) + 1000)
        n = f(bytes(data), len(data), buf)
        if n < 0:
            raise RuntimeError("lzp failed")
        return buf.raw[:n]

    def unlzp(self, data: bytes, out_size: int) -> bytes:
        """unlzp into a buffer of out_size bytes (the reference writes past
        it on a stream that decodes longer: size it generously there)."""
        _, g = self._lzp_fns()
        buf = C.create_string_buffer(max(out_size, 1))
        n = g(bytes(data), len(data), buf, out_size)
        if n < 0:
            raise RuntimeError("unlzp failed")
        return buf.raw[:n]

    def lzp3_compress(self, data: bytes) -> bytes:
        return self.rans_compress(self.lzp(data), 5)

    def lzp3_uncompress(self, comp: bytes, u_len: int) -> bytes:
        return self.unlzp(self.rans_uncompress(comp), u_len)


_cache: dict = {}


def oracle() -> _Codec:
    """Our restatement (liboracle.so)."""
    if "ora" not in _cache:
        _cache["ora"] = _Codec(ORACLE_SO, "ora_")
    return _cache["ora"]


def have_ref() -> bool:
    return os.path.exists(REF_SO)


def ref() -> _Codec:
    """The reference itself, compiled from /root/reference (oracle/_ref)."""
    if "ref" not in _cache:
        _cache["ref"] = _Codec(REF_SO, "")
    return _cache["ref"]


REF_SIMD_SO = os.path.join(HERE, "_ref", "libhtsref_simd.so")


def have_ref_simd() -> bool:
    return os.path.exists(REF_SIMD_SO)


def ref_simd() -> _Codec:
    """The reference with its x86 SIMD 32x16 codecs dispatched at run time
    (oracle/Makefile libhtsref_simd.so; the shipped config.h compiles the
    dispatcher out)."""
    if "ref_simd" not in _cache:
        _cache["ref_simd"] = _Codec(REF_SIMD_SO, "")
    return _cache["ref_simd"]


# ---- sequence context model (fqzcomp5.c:1073-1406) -------------------------
REF_CLI_SO = os.path.join(HERE, "_ref", "libfqz5ref.so")


class SeqCM:
    """encode_seq / decode_seq: ``ora_seq_*`` in liboracle.so, or the
    reference's own functions in ``_ref/libfqz5ref.so``."""

    def __init__(self, path: str, enc: str, dec: str):
        self.lib = C.CDLL(path)
        self._e = getattr(self.lib, enc)
        self._e.restype = C.c_void_p
        self._e.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint32), C.c_int,
                            C.c_int, C.c_int, C.POINTER(C.c_uint)]
        self._d = getattr(self.lib, dec)
        self._d.restype = C.c_void_p
        self._d.argtypes = [C.c_char_p, C.c_uint, C.POINTER(C.c_uint32), C.c_int,
                            C.c_int, C.c_int, C.c_uint]

    @staticmethod
    def _lens(lens):
        lens = list(lens) or [0]
        return (C.c_uint32 * len(lens))(*lens), len(lens)

    def encode(self, seq: bytes, lens, both: int, k: int):
        la, nr = self._lens(lens)
        n = C.c_uint(0)
        p = self._e(seq, len(seq), la, nr, both, k, C.byref(n))
        return _Codec._take(p, n.value)

    def decode(self, comp: bytes, lens, both: int, k: int, out_size: int):
        la, nr = self._lens(lens)
        p = self._d(comp, len(comp), la, nr, both, k, out_size)
        return _Codec._take(p, out_size)


def seq_oracle() -> SeqCM:
    if "seq_ora" not in _cache:
        _cache["seq_ora"] = SeqCM(ORACLE_SO, "ora_seq_encode", "ora_seq_decode")
    return _cache["seq_ora"]


def have_seq_ref() -> bool:
    return os.path.exists(REF_CLI_SO)


def seq_ref() -> SeqCM:
    if "seq_ref" not in _cache:
        _cache["seq_ref"] = SeqCM(REF_CLI_SO, "encode_seq", "decode_seq")
    return _cache["seq_ref"]
