"""The block decoder's host-core leg (fqz5_set_host_decode): with the
adaptive-model chains (fqz quality, SEQ10..SEQ14B sequence sections) on host
threads beside the GPU's rANS / LZP / name work, every file decodes to the
same text as the GPU-only decode, at the presets that choose those methods."""
import numpy as np
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


@pytest.mark.parametrize("kind,level", [("illumina", 5), ("novaseq", 5), ("illumina", 7),
                                        ("ont", 7), ("illumina", 9)])
def test_host_leg_equals_gpu(kind, level):
    text = _text(kind, 6000)
    z = fqz5file.compress_bytes(text, level, blk_size=300_000)
    so = lib.load()
    prev = so.fqz5_set_host_decode(1)
    try:
        host = fqz5file.decompress_bytes(z)
    finally:
        so.fqz5_set_host_decode(prev)
    so.fqz5_set_host_decode(0)
    try:
        gpu = fqz5file.decompress_bytes(z)
    finally:
        so.fqz5_set_host_decode(prev)
    assert host == text
    assert gpu == text
