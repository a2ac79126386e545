"""Trial-choice parity with the reference: the reference
CLI run single-threaded (-t1, the deterministic trial order) over a
109-block file (-b 1M) picks, per block, the name, sequence and quality
method by its codec trial (metrics_method / compress_with_methods,
fqzcomp5.c:1899-1958, :2106; the first 3 blocks try every method, block 4
fixes the winner, blocks 5-104 reuse it and block 105 re-trials,
METRICS_REVIEW = 100, :151-152).  The GPU section coder over the same
records must write, block for block, the same strat byte, the same sizes
and the same bytes for all three sections, and the assembled blocks
(header, CRC32, lengths: fqz5_blocks_assemble) must equal the file's
blocks byte for byte and decode back to the records."""
import hashlib
import os
import struct
import subprocess

import pytest
import torch

import fqz5_container as F
from fqzcomp5_amd import lib, sections as S, synth
from oracle import binding

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CLI = os.path.join(os.path.dirname(binding.REF_BIN), "fqzcomp5")
GPU_CLI = os.path.join(os.path.dirname(binding.REF_BIN), "fqzcomp5_gpu")


@pytest.fixture(scope="module", autouse=True)
def _need():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())
    if not os.path.exists(CLI):
        pytest.fail("oracle/_ref/fqzcomp5 not built (make -C oracle)")


GEN = {"illumina": lambda: synth.illumina(320000, seed=21, with_names=True),
       "novaseq": lambda: synth.novaseq(320000, seed=21, with_names=True),
       # configs[3] / [4] shapes at a few blocks (every preset method tried)
       "ont": lambda: synth.ont(700, seed=21, with_names=True),
       "hifi": lambda: synth.hifi(300, seed=21, with_names=True)}


@pytest.mark.parametrize("level,kind", [(3, "illumina"), (5, "illumina"), (5, "novaseq"),
                                        (7, "ont"), (9, "hifi")])
def test_trial_choices_match_reference(tmp_path, level, kind):
    reads = GEN[kind]()
    src, out = str(tmp_path / "in.fastq"), str(tmp_path / "ref.fqz5")
    open(src, "wb").write(reads.to_fastq())
    subprocess.run([CLI, f"-{level}", "-b", "1M", "-t1", src, out], check=True,
                   capture_output=True, timeout=600)
    ref = F.read(out)
    blocks = synth.split_blocks(reads, 1_000_000)
    assert len(ref) == len(blocks) >= (106 if level <= 5 else 5)   # -3/-5: re-trial at block 105
    run = S.Run(reads, blocks, torch.device("cuda", 0))
    res, meth_all, sizes, tried, _ = S.encode_run(run.enc_secs(), S.masks(level, full=True),
                                                  S.new_state())
    assert all(r.status == 0 for r in res)
    for i, (sec, s, e, fl, k) in enumerate(run.spans):
        if sec == S.SEC_NAME:                       # encode_names' bytes, whole
            want = ref[k].names
            exp = struct.pack("<IBI", want.u_len, want.strat, len(want.data)) + want.data
            assert (res[i].strat, res[i].clen) == (want.strat, len(exp)), (k, int(meth_all[i]))
            assert run.chosen(res, i) == exp, (k, sec)
            continue
        want = ref[k].seq if sec == S.SEC_SEQ else ref[k].qual
        assert (res[i].strat, res[i].usize, res[i].clen) == \
            (want.strat, want.u_len, len(want.data)), (k, sec, int(meth_all[i]))
        assert run.chosen(res, i) == want.data, (k, sec)
    # the run exercised a trial: blocks 1-3 and 105-107 tried every method
    for k in ((0, 1, 2, 104, 105, 106) if level <= 5 else (0, 1, 2)):
        assert all(bin(int(tried[3 * k + j])).count("1") > 1 for j in (1, 2))
    # whole blocks: header, CRC, lengths and sections as the file has them
    run.assemble(res)
    raw = F.raw_blocks(out)
    for k in range(len(blocks)):
        assert run.block_bytes(k) == raw[k], k
    # and back: parse every block, decode its sections
    dres = S.decode(run.block_dec_secs())
    assert all(r.status == 0 for r in dres)
    torch.cuda.synchronize()
    assert run.roundtrip_ok()


def test_sample_fastq_dropin_plumbing(tmp_path):
    """BASELINE configs[0]: the drop-in CLI (reference CLI on this library)
    writes the reference's 245-byte sample.fastq file at -1."""
    out = str(tmp_path / "s.fqz5")
    subprocess.run([GPU_CLI, "-1", "-t1", os.path.join(HERE, "golden", "fastq", "sample.fastq"),
                    out], check=True, capture_output=True, timeout=300)
    b = open(out, "rb").read()
    assert len(b) == 245 and hashlib.md5(b).hexdigest() == "8b5e07bf4c452ad206679f5e4bd7837a"
