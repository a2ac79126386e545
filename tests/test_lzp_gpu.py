"""The LZP pre-pass on the GPU (fqz5_lzp / fqz5_unlzp, lzp.hip) against the
reference's lzp / unlzp (golden vectors made from oracle/_ref by
tests/golden/make_golden_lzp.py) and the oracle restatement; and the LZP3
sequence method through the section coder: where it wins the trial
(repeated reads) the chosen stream equals the reference's and decodes back."""
import hashlib
import json
import os
import random

import numpy as np
import pytest
import torch

from fqzcomp5_amd import lib, sections as S, synth
from lzp_cases import cases
from oracle import binding

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "lzp.json")))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


def test_lzp_golden():
    got = dict(cases())
    for g in GOLD:
        data = got[g["case"]]
        z = lib.lzp(data)
        assert (len(z), hashlib.md5(z).hexdigest()) == (g["lzp_len"], g["lzp_md5"]), g["case"]
        assert lib.unlzp(z, len(data)) == data, g["case"]


def test_lzp_random_vs_oracle():
    ora = binding.oracle()
    rng = random.Random(11)
    for it in range(40):
        n = rng.choice([0, 1, 2, 5, 64, 65, 127, 1000, 70000, 140000])
        alpha = rng.choice([b"AC", b"ACGT", b"ACGTN", bytes([233, 234, 7]), bytes(range(256))])
        if rng.random() < 0.5 and n:
            unit = bytes(rng.choice(alpha) for _ in range(rng.randint(1, 300)))
            data = bytearray((unit * (n // len(unit) + 1))[:n])
            for _ in range(rng.randint(0, 5)):
                data[rng.randrange(n)] = rng.choice(alpha)
            data = bytes(data)
        else:
            data = bytes(rng.choice(alpha) for _ in range(n))
        exp = ora.lzp(data)
        assert lib.lzp(data) == exp, (it, n)
        assert lib.unlzp(exp, n) == data, (it, n)


def test_unlzp_damaged():
    data = b"ACGTTGCA" * 500
    z = lib.lzp(data)
    assert lib.unlzp(z, len(data) - 1) is None           # would write past out_cap
    last = max(z.rfind(bytes([233])), z.rfind(bytes([234])))
    assert last > 0
    cut = z[:last + 1]                                    # ends on a marker
    assert lib.unlzp(cut, len(data)) is None


def test_lzp3_wins_on_repeated_reads():
    """Amplicon sequences (3 reads repeated; with 40 distinct reads the 4-byte
    LZP contexts mispredict and PACK|O1 wins): LZP3 wins the -3 trial;
    the section coder's stream equals the reference's LZP3 and decodes."""
    rng = np.random.default_rng(3)
    reads = synth.illumina(30000, seed=3)
    pool = reads.seq[:150 * 3].reshape(3, 150).copy()     # 3 amplicons
    reads.seq[:] = pool[rng.integers(0, 3, reads.num_records)].reshape(-1)
    blocks = synth.split_blocks(reads, 2_000_000)
    run = S.Run(reads, blocks, torch.device("cuda", 0), names=False)
    res, meth_all, sizes, tried, _ = S.encode_run(run.enc_secs(), S.masks(3), S.new_state())
    codec = binding.ref() if binding.have_ref() else binding.oracle()
    seen = False
    for i, (sec, s, e, fl, k) in enumerate(run.spans):
        if sec != S.SEC_SEQ:
            continue
        assert int(meth_all[i]) == S.LZP3
        seen = True
        assert res[i].strat == S.LZP3
        assert run.chosen(res, i) == codec.lzp3_compress(reads.seq[s:e].tobytes())
    assert seen
    dres = S.decode(run.dec_secs(res))
    assert all(r.status == 0 for r in dres)
    torch.cuda.synchronize()
    assert run.roundtrip_ok()
