"""CPU tests of the C-ABI boundary: the library loads and exports every
function declared in include/fqz5_mi355x.h.  No compute calls (no GPU)."""
import ctypes as C
import subprocess

from fqzcomp5_amd import lib


def test_header_declares_htscodecs_entry_points():
    syms = lib.header_symbols()
    for s in ("rans_compress_to_4x16", "rans_compress_4x16",
              "rans_uncompress_to_4x16", "rans_uncompress_4x16",
              "rans_compress_bound_4x16", "rans_set_cpu"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    so = lib.load()
    missing = [s for s in lib.header_symbols() if not hasattr(so, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH],
                         capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert set(lib.header_symbols()) <= exported


def test_bound_matches_oracle():
    from oracle import binding
    ora = C.CDLL(binding.ORACLE_SO)
    ora.ora_rans_compress_bound_4x16.restype = C.c_uint
    for n in (0, 1, 7, 100, 1000, 65536, 10**7):
        for o in (0, 1, 4, 5, 0x80, 0xc1, 0x45, (150 << 8) | 9):
            assert lib.compress_bound(n, o) == ora.ora_rans_compress_bound_4x16(n, o)
