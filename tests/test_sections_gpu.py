"""The section coder on the GPU (include/fqz5_block.h) at -3 and -5: the
codec trial over a run of blocks, every chosen stream byte-equal to the
reference's codec for that method (oracle/_ref when built, else the oracle
restatement), and every section decoded back.  -5 adds the FQZ1/FQZ3
quality methods: trial blocks try them, later blocks are encoded with the
chosen method at commit."""
import numpy as np
import torch
import pytest

from fqzcomp5_amd import lib, sections as S, synth
from oracle import binding

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())


def _order(m, fl):
    return [0, 1, 64, 65, 128, 129, 192, 193][m - 1] if m <= 8 else (fl << 8) + 9


# fqz beats rANS on the random-walk (Illumina) qualities from ~2 MB blocks
# on; on i.i.d. NovaSeq qualities rANS O0 stays ahead at every size
GEN = {"illumina": synth.illumina, "novaseq": synth.novaseq, "ont": synth.ont,
       "hifi": lambda n, seed: synth.hifi(n // 2, seed=seed)}


# -7 (ONT) and -9 (HiFi pairs) are BASELINE configs[3]/[4] at small block
# sizes: every method of their presets (FQZ0..4, SEQ10..14B, RANS64/65/128)
@pytest.mark.parametrize("level,kind,nreads,blk,cm", [(3, "illumina", 6000, 200_000, False),
                                                      (5, "novaseq", 6000, 200_000, False),
                                                      (5, "illumina", 72000, 4_000_000, False),
                                                      (5, "novaseq", 6000, 200_000, True),
                                                      (7, "ont", 500, 1_500_000, True),
                                                      (9, "hifi", 600, 1_500_000, True)])
def test_run_vs_reference(level, kind, nreads, blk, cm):
    codec = binding.ref() if binding.have_ref() else binding.oracle()
    reads = GEN[kind](nreads, seed=11)
    blocks = synth.split_blocks(reads, blk)
    assert len(blocks) >= 5
    run = S.Run(reads, blocks, torch.device("cuda", 0), names=False)
    t0, p0 = S.trial_counts()
    res, meth_all, sizes, tried, _ = S.encode_run(run.enc_secs(), S.masks(level, cm), S.new_state())
    t1, p1 = S.trial_counts()
    assert all(r.status == 0 for r in res)
    offs = np.concatenate([[0], np.cumsum(reads.lens.astype(np.int64))])
    used = set()
    for i, ((sec, s, e, fl, k), r) in enumerate(zip(run.spans, res)):
        m = int(meth_all[i])
        used.add(m)
        data = (reads.seq if sec == S.SEC_SEQ else reads.qual)[s:e].tobytes()
        if m >= S.FQZ0:
            a, b = blocks[k]
            fl_ = np.zeros(b - a, np.uint32) if reads.flags is None else reads.flags[a:b].copy()
            exp = codec.fqz_compress(data, reads.lens[a:b].copy(), fl_,
                                     m - S.FQZ0, reads.seq[s:e].tobytes())
            assert r.strat == 1
        elif S.SEQ10 <= m <= S.SEQ14B:
            a, b = blocks[k]
            k_, both = S.SEQ_PARAMS[m]
            sc = binding.seq_ref() if binding.have_seq_ref() else binding.seq_oracle()
            exp = sc.encode(data, [int(x) for x in reads.lens[a:b]], both, k_)
            assert r.strat == (k_ << 4) | (both << 3) | 1
        elif m == S.LZP3:
            exp = codec.lzp3_compress(data)
            assert r.strat == S.LZP3
        else:
            exp = codec.rans_compress(data, _order(m, fl))
            assert r.strat == 0
        assert run.chosen(res, i) == exp, (i, m)
    if level == 5:
        # a reported fqz size is exact, or (pruned) a lower bound that is at
        # least the section's best rANS size: never above the true size
        for i, (sec, s, e, fl, k) in enumerate(run.spans):
            for m in (S.FQZ1, S.FQZ3):
                if sec != S.SEC_QUAL or int(sizes[i, m]) == 0xFFFFFFFF:
                    continue                        # not a try-phase candidate
                a, b = blocks[k]
                true = len(codec.fqz_compress((reads.qual)[s:e].tobytes(), reads.lens[a:b].copy(),
                                              np.zeros(b - a, np.uint32), m - S.FQZ0,
                                              reads.seq[s:e].tobytes()))
                assert int(sizes[i, m]) <= true, (i, m, int(sizes[i, m]), true)
        if kind == "novaseq" and not cm:            # rANS wins by a margin: fqz pruned
            assert p1 - p0 > 0 and t1 - t0 >= p1 - p0
        fqz_bits = (1 << S.FQZ1) | (1 << S.FQZ3)
        assert all(int(t) & fqz_bits for t, (sec, *_) in zip(tried[:6], run.spans)
                   if sec == S.SEC_QUAL)            # the trial blocks tried fqz
        if kind == "illumina":                      # random-walk qualities: fqz wins
            assert used & {S.FQZ1, S.FQZ3}, used
    if cm:                                          # trial blocks tried the CM
        cm_bits = (1 << S.SEQ10) | (1 << S.SEQ12B)
        assert all(int(t) & cm_bits for t, (sec, *_) in zip(tried[:6], run.spans)
                   if sec == S.SEC_SEQ)
    dres = S.decode(run.dec_secs(res))
    assert all(r.status == 0 for r in dres)
    torch.cuda.synchronize()
    assert run.roundtrip_ok()
    del offs


def test_arena_constant_over_steps():
    """Repeated -5 encode + decode steps (fqz trial candidates on the helper
    context) hold a constant amount of device arena memory: the r01 driver
    bench died with hipMalloc out of memory because the helper arena was
    never rewound after fqz5_sections_commit."""
    reads = synth.illumina(20000, seed=5)
    blocks = synth.split_blocks(reads, 1_000_000)
    run = S.Run(reads, blocks, torch.device("cuda", 0), names=False)
    sizes = []
    for _ in range(8):
        res, *_ = S.encode_run(run.enc_secs(), S.masks(5), S.new_state())
        dres = S.decode(run.dec_secs(res))
        assert all(r.status == 0 for r in res) and all(r.status == 0 for r in dres)
        sizes.append(lib.arena_bytes())
    assert run.roundtrip_ok()
    assert sizes[1:] == sizes[1:2] * (len(sizes) - 1), sizes


@pytest.mark.parametrize("bounds", [True, False, "widen"])
@pytest.mark.parametrize("level,kind,nreads,blk", [(7, "ont", 500, 1_500_000),
                                                   (9, "hifi", 600, 1_500_000)])
def test_bounded_run_equals_run(level, kind, nreads, blk, bounds):
    """encode_run_bounded (the trial a section at a time, then every section
    coded with its one method, for the -7/-9 block sizes) makes the choices
    and the bytes of encode_run; chunk_bytes small enough that every chunk
    holds one or two sections; the commit in one chunk (-7) or in chunks
    as small as the tries' (-9).  bounds: the tries give the fqz / sequence
    model candidates' size intervals only, decided by trial_decided (or
    tried again exactly).  "widen": every interval widened by 10 MB, so every
    decision is left open and refined by one session over all sections that
    the commit reuses (refine_session)."""
    reads = GEN[kind](nreads, seed=13)
    blocks = synth.split_blocks(reads, blk)
    assert len(blocks) >= 4
    dev = torch.device("cuda", 0)
    run = S.Run(reads, blocks, dev, names=False)
    av = S.masks(level, True)
    res_a, meth_a, _, tried_a, _ = S.encode_run(run.enc_secs(), av, S.new_state())
    got_a = [run.chosen(res_a, i) for i in range(len(res_a))]
    run_b = S.Run(reads, blocks, dev, names=False)
    S.bounds_widen = 10_000_000 if bounds == "widen" else 0
    try:
        res_b, meth_b, _, tried_b, _ = S.encode_run_bounded(run_b.enc_secs(), av, S.new_state(),
                                                        chunk_bytes=(50_000_000 if bounds == "widen"
                                                                     else 2 * blk // 3),
                                                        commit_bytes=(2 * blk // 3 if level == 9
                                                                      else 2_400_000_000),
                                                        bounds=bool(bounds))
    finally:
        S.bounds_widen = 0
    print(f"-{level} {kind}: intervals decided the trial: {S.last_bounds_decided}")
    assert all(r.status == 0 for r in res_b)
    assert list(meth_a) == list(meth_b)
    assert list(tried_a) == list(tried_b)
    for i in range(len(res_b)):
        assert run_b.chosen(res_b, i) == got_a[i], i
    dres = S.decode(run_b.dec_secs(res_b))
    assert all(r.status == 0 for r in dres)
    torch.cuda.synchronize()
    assert run_b.roundtrip_ok()


@pytest.mark.parametrize("level,kind,nreads,blk", [(5, "illumina", 60000, 2_000_000),
                                                   (5, "novaseq", 60000, 2_000_000),
                                                   (7, "ont", 500, 1_500_000)])
def test_run_bounds_first_equals_run(level, kind, nreads, blk):
    """encode_run(bounds=True): the tries give the fqz / sequence-model size
    intervals only; when they decide the trial the commit codes the winners
    in the same session (skipped candidates coded late, the rANS ones
    reused), else the exact tries run.  Same choices and bytes as
    encode_run, and the blocks decode back."""
    reads = GEN[kind](nreads, seed=17)
    blocks = synth.split_blocks(reads, blk)
    assert len(blocks) >= 4
    dev = torch.device("cuda", 0)
    av = S.masks(level, True)
    run = S.Run(reads, blocks, dev, names=False)
    res_a, meth_a, _, tried_a, _ = S.encode_run(run.enc_secs(), av, S.new_state())
    got_a = [run.chosen(res_a, i) for i in range(len(res_a))]
    run_b = S.Run(reads, blocks, dev, names=False)
    res_b, meth_b, _, tried_b, _ = S.encode_run(run_b.enc_secs(), av, S.new_state(), bounds=True)
    print(f"-{level} {kind}: intervals decided the trial: {S.last_bounds_decided}")
    assert all(r.status == 0 for r in res_b)
    assert list(meth_a) == list(meth_b)
    assert list(tried_a) == list(tried_b)
    for i in range(len(res_b)):
        assert run_b.chosen(res_b, i) == got_a[i], i
    dres = S.decode(run_b.dec_secs(res_b))
    assert all(r.status == 0 for r in dres)
    torch.cuda.synchronize()
    assert run_b.roundtrip_ok()
