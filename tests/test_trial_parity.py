"""CPU checks of the container and block split the trial-parity test relies
on: the reference CLI (oracle/_ref/fqzcomp5, compiled from the reference
sources) writes the plumbing golden for sample.fastq at -1 (BASELINE
configs[0]), and its blocks hold exactly the records synth.split_blocks
assigns them (load_seqs_kseq's rule, fqzcomp5.c:471-477)."""
import hashlib
import os
import subprocess

import pytest

import fqz5_container as F
from fqzcomp5_amd import synth
from oracle import binding

HERE = os.path.dirname(os.path.abspath(__file__))
CLI = os.path.join(os.path.dirname(binding.REF_BIN), "fqzcomp5")
pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="oracle/_ref not built")


def test_sample_fastq_plumbing_golden(tmp_path):
    out = str(tmp_path / "s.fqz5")
    subprocess.run([CLI, "-1", "-t1", os.path.join(HERE, "golden", "fastq", "sample.fastq"), out],
                   check=True, capture_output=True)
    b = open(out, "rb").read()
    assert len(b) == 245 and hashlib.md5(b).hexdigest() == "8b5e07bf4c452ad206679f5e4bd7837a"


def test_block_split_matches_reference(tmp_path):
    reads = synth.illumina(12000, seed=4, with_names=True)
    src, out = str(tmp_path / "in.fastq"), str(tmp_path / "o.fqz5")
    open(src, "wb").write(reads.to_fastq())
    subprocess.run([CLI, "-3", "-b", "1M", "-t1", src, out], check=True, capture_output=True)
    blocks = F.read(out)
    split = synth.split_blocks(reads, 1_000_000)
    assert [b.nrec for b in blocks] == [e - a for a, e in split]
    assert all(b.crc_ok for b in blocks)
