"""Where the block decoder runs its adaptive-model chains (fqz quality,
SEQ10..SEQ14B sequence sections; fqz5_set_host_decode): every placement — all
on the GPU (0), all on host threads beside the GPU's rANS / LZP / name work
(1), by measured cost (2, the default), every other chain on the host (3:
a GPU sequence chain feeding a host quality chain and the reverse) — decodes
every file to its text, at the presets that choose those methods."""
import ctypes as C

import pytest

from fqzcomp5_amd import fqz5file, lib, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


def _text(kind, n):
    r = {"illumina": lambda: synth.illumina(n, seed=8, with_names=True),
         "novaseq": lambda: synth.novaseq(n, seed=8, with_names=True),
         "ont": lambda: synth.ont(max(1, n // 80), seed=8, with_names=True)}[kind]()
    return synth.fastq_chunk(r, 0, r.num_records).tobytes()


def _chains(so):
    c = (C.c_uint64 * 2)()
    so.fqz5_decode_chain_counts(c)
    return int(c[0]), int(c[1])


@pytest.mark.parametrize("kind,level", [("illumina", 5), ("novaseq", 5), ("illumina", 7),
                                        ("ont", 7), ("illumina", 9)])
def test_every_placement_decodes(kind, level):
    text = _text(kind, 6000)
    z = fqz5file.compress_bytes(text, level, blk_size=300_000)
    so = lib.load()
    prev = so.fqz5_set_host_decode(2)
    try:
        for mode in (0, 1, 2, 3):
            so.fqz5_set_host_decode(mode)
            h0, g0 = _chains(so)
            assert fqz5file.decompress_bytes(z) == text, mode
            h1, g1 = _chains(so)
            if mode == 0:
                assert h1 == h0
            if mode == 1:
                assert g1 == g0
    finally:
        so.fqz5_set_host_decode(prev)


def test_default_is_cost_model():
    so = lib.load()
    prev = so.fqz5_set_host_decode(2)
    so.fqz5_set_host_decode(prev)
    assert prev == 2
