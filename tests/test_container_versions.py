"""Older containers the reference still decodes (read_header,
fqzcomp5.c:2578-2603; decode_block skips the CRC field for them, :2300-2318):
v1.0 (`FQZ5\\1\\0\\0\\0`, no per-block CRC field) and the headerless old
format (blocks from offset 0, no index).

* the reference's own binary fixture, test_data/sample.fqz5 (v1.0, 241 B,
  copied to tests/golden/fastq/), decodes to sample.fastq;
* multi-block v1.0 / old files: the reference CLI's v1.1 output rewritten by
  tests/fqz5_container.downgrade; on the CPU the reference CLI itself decodes
  them back to its input (which pins the rewrite), on the GPU fqz5file must do
  the same."""
import os
import subprocess

import pytest

import fqz5_container as F
from fqzcomp5_amd import fqz5file, lib, synth

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CLI = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5")
SAMPLE = os.path.join(HERE, "golden", "fastq", "sample")
need_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def cli_files(tmp_path_factory):
    """(FASTQ text, {level: v1.1 bytes}) for a 4-block synthetic Illumina file
    coded by the reference CLI (-t1, 1 MB blocks)."""
    if not os.path.exists(CLI):
        pytest.skip("oracle/_ref not built")
    d = tmp_path_factory.mktemp("ver")
    src = str(d / "in.fastq")
    synth.write_fastq(synth.illumina(11000, seed=8, with_names=True), src)
    out = {}
    for level in (3, 5):
        dst = str(d / f"o{level}.fqz5")
        subprocess.run([CLI, f"-{level}", "-t1", "-b", "1M", src, dst], check=True,
                       capture_output=True, timeout=300)
        out[level] = open(dst, "rb").read()
    return open(src, "rb").read(), out


def test_sample_fqz5_is_v10_host():
    data = open(SAMPLE + ".fqz5", "rb").read()
    ranges = fqz5file._blocks_of(data)
    assert ranges.version == fqz5file.V10 and len(ranges) == 1
    (f,) = fqz5file.check_blocks(data, ranges)
    text = open(SAMPLE + ".fastq", "rb").read()
    assert f["nrec"] == text.count(b"\n") // 4 and f["seq_ulen"] == f["qual_ulen"] > 0


@need_cli
def test_reference_decodes_downgraded(cli_files, tmp_path):
    """The rewrite is a file the reference reads: its -d gives the input."""
    text, files = cli_files
    for level, z in files.items():
        ranges = fqz5file._blocks_of(z)
        assert len(ranges) >= 3
        for ver, tag in ((fqz5file.V10, "v1.0"), (fqz5file.VOLD, "old")):
            d = F.downgrade(z, tag)
            r = fqz5file._blocks_of(d)
            assert r.version == ver and len(r) == len(ranges)
            assert fqz5file.check_blocks(d, r) == fqz5file.check_blocks(z, ranges)
            src, back = str(tmp_path / f"{level}{tag}.fqz5"), str(tmp_path / "b.fastq")
            open(src, "wb").write(d)
            subprocess.run([CLI, "-d", "-t1", src, back], check=True, capture_output=True,
                           timeout=300)
            assert open(back, "rb").read() == text, (level, tag)


@pytest.mark.gpu
def test_sample_fqz5_decodes_gpu(tmp_path):
    """The reference's only binary fixture (v1.0) through the file path."""
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())
    text = open(SAMPLE + ".fastq", "rb").read()
    data = open(SAMPLE + ".fqz5", "rb").read()
    assert fqz5file.decompress_bytes(data) == text
    out = str(tmp_path / "s.fastq")
    assert fqz5file.decompress_file(SAMPLE + ".fqz5", out) == len(text)
    assert open(out, "rb").read() == text


@pytest.mark.gpu
@need_cli
def test_downgraded_multiblock_gpu(cli_files, tmp_path):
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())
    text, files = cli_files
    for level, z in files.items():
        for tag in ("v1.0", "old"):
            d = F.downgrade(z, tag)
            assert fqz5file.decompress_bytes(d) == text, (level, tag)
            src, out = str(tmp_path / "d.fqz5"), str(tmp_path / "d.fastq")
            open(src, "wb").write(d)
            # small windows: the blocks come in several groups
            fqz5file.decompress_file(src, out, window_bytes=len(d) // 3)
            assert open(out, "rb").read() == text, (level, tag)
