#!/usr/bin/env python3
"""Benchmark: fqzcomp5 block coding on MI355X.

Metric (BASELINE.json): input MB/s encode+decode, 100 MB blocks, -3 and -5;
bit-exact vs CPU.  Default workload (configs[1]): a synthetic 1 GB Illumina
150 bp FASTQ with 8-level binned qualities and Illumina names at -3, split
into 100 MB blocks by the reference's record rule (fqzcomp5.c:471-477).  The
default run adds configs[2] as the `level5` item: a synthetic 4 GB NovaSeq
FASTQ per GPU at -5.  One step is one pass of the hot path over the whole
workload, the records resident in HBM (names, bases, qualities; lengths on
the host):

    encode  every block whole (encode_block, fqzcomp5.c:2147-2280): the name,
            sequence and quality sections with the level's method sets and
            the -t1 codec-trial state machine (fqzcomp5.c:1899-2144), the
            lengths section, the block header and its CRC32
    decode  every block parsed (CRC checked), every section back to bytes.

Encode and decode are timed separately inside each step (stream synchronised
between them).  Reported per workload:
    value     FASTQ input bytes of all ranks x steps / (t_enc + t_dec),
              the max over ranks of each (the metric's combined figure)
    enc_MBps, dec_MBps   the same bytes over t_enc and t_dec alone
    section_MBps         the name+seq+qual section bytes over t_enc + t_dec
The blocks equal the reference CLI's blocks byte for byte (checked against
the CPU baseline's file when it runs); the FASTQ parse and the file write
are outside the timed region (the records are already in HBM).

Methods: the level presets' name, sequence and quality masks
(fqzcomp5.c:4886-4932, :2750-2793), every one coded by this build.

Multi-GPU: `--gpus N` runs one process per GPU (it re-launches itself under
torch.distributed.run when not started by it).  Weak scaling by default:
each rank codes its own file of `--gb`, and the run's trial state covers the
blocks of all ranks in rank order (the only collective: an all-gather of the
candidate sizes, sections.exchange_sizes).  `--scaling strong` shards the
blocks of one fixed file contiguously over the ranks.

Also reported: the roofline of the dominant kernel from live HIP events on
the library's stream; the reference CLI (oracle/_ref, compiled from the
reference sources, as shipped and with its x86 SIMD dispatch) on the host
cores over the same FASTQ text, its blocks compared with the GPU's; and the
reference CLI relinked on this library (the drop-in) on the same file.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# The library runs the trial's work candidates on helper contexts, each with
# its own streams, beside the rANS batch; with HIP's default of 4 hardware
# queues per process those streams share queues and serialise (measured:
# the -3 encode waited 100 ms per step behind the LZP3 helper's chain).
# Must be set before anything initialises HIP.
# (the rule of capi.cpp's hw_queues_default: FQZ5_HW_QUEUES as given, else
# an unset value or HIP's default of 4 raised to 20, any other value kept)
if os.environ.get("FQZ5_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["FQZ5_HW_QUEUES"]
elif os.environ.get("GPU_MAX_HW_QUEUES", "") in ("", "4"):
    os.environ["GPU_MAX_HW_QUEUES"] = "20"

FASTQ_REC = 358          # bytes of FASTQ text per synthetic 150 bp record (avg)
GAP_S = float(os.environ.get("FQZ5_BENCH_GAP_S", "0") or 0)
STEP_TRACE = bool(os.environ.get("FQZ5_STEP_TRACE"))   # per-phase decode times on stderr
BLK = 100_000_000        # -3 / -5 block size (fqzcomp5.c:4896,4904)
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8 TB/s spec
# fqz5_profile_read_all's kernels, in its order (include/fqz5_mi355x.h); each
# launch timed by HIP events around it on its own stream.  k_enc_replay is
# the emitting pass (rocprof: k_enc_replay<true>), k_enc_replay0 the
# counting pass (k_enc_replay<false>); k_fqz_dec both fqz decoders
PROF_KERNELS = ["k_enc_chain", "k_rans_dec", "k_fqz_dec", "k_fqz_rc", "k_seq_dec",
                "k_enc_chain2w", "k_enc_replay", "k_seq_model", "k_fqz_model_hot",
                "k_fqz_ev_fill", "k_lzp_dec", "k_enc_replay0"]
# rocprof kernel names of a PROF_KERNELS entry (pmc_traffic)
ROCPROF_NAMES = {"k_fqz_dec": ["k_fqz_dec", "k_fqz_dec_small"],
                 "k_enc_replay": ["k_enc_replay<true>"],
                 "k_enc_replay0": ["k_enc_replay<false>"],
                 "k_seq_model": ["k_seq_model_runs", "k_seq_model"]}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def host_threads() -> int:
    """The host cores this process may use: its CPU affinity, capped by the
    box's per-GPU CPU share when one is set ($OMP_NUM_THREADS)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(n, 1)


def make_reads(gb: float, seed: int, kind: str):
    from fqzcomp5_amd import synth
    if kind == "ont":        # configs[3]: lognormal lengths, median 10.5 kb, read-id names
        return synth.ont(int(gb * 1e9 / 26_600), seed=seed, with_names=True)
    if kind == "hifi":       # configs[4]: ~15 kb pairs, READ2 flags from the /2 names
        return synth.hifi(int(gb * 1e9 / 60_100), seed=seed, with_names=True)
    n_reads = int(gb * 1e9 / FASTQ_REC)
    return (synth.novaseq if kind == "novaseq" else synth.illumina)(n_reads, seed=seed)


def pmc_traffic(kernel: str, tag: str = ""):
    """HBM bytes per dispatch of `kernel` from the newest committed PMC
    summary of this workload (profiles/rNN_pmc{tag}.json, written by
    tools/pmc_summary.py from separate rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of this bench; tag "" = configs[1] -3, "_l5" = configs[2] -5)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc{tag}.json")))
    if not files:
        return None, None, None
    js = json.load(open(files[-1]))
    names = ROCPROF_NAMES.get(kernel, [kernel])
    best = None
    for k, v in js["kernels"].items():
        if any(f"::{n}(" in k or (f"::{n}<" in k if "<" not in n else f"::{n}(" in k)
               for n in names):
            # the step's main launch of the kernel (the largest dispatch);
            # the file's "note" says how that launch ran (hedged copies)
            b = int(v.get("hbm_bytes_max_dispatch", v["hbm_bytes_per_dispatch"]))
            best = b if best is None else max(best, b)
    if best is None:
        return None, None, None
    return best, os.path.relpath(files[-1], ROOT), js.get("note")


def cpu_baseline(fastq: str, level: int, threads: int, gpu_blocks, exe_name="fqzcomp5",
                 timeout: int = 600):
    """The reference CLI (oracle/_ref/<exe_name>, compiled from the reference
    sources) on the workload's FASTQ text with -t<threads>: encode and decode
    wall time (file in the page cache, output to TMPDIR), its blocks compared
    with the GPU's blocks and its decoded FASTQ with the input."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fqz5_container as F
    exe = os.path.join(ROOT, "oracle", "_ref", exe_name)
    if not os.path.exists(exe):
        return {"error": f"oracle/_ref/{exe_name} not built"}
    nbytes = os.path.getsize(fastq)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        out, back = os.path.join(td, "c.fqz5"), os.path.join(td, "c.fastq")
        t0 = time.perf_counter()
        subprocess.run([exe, f"-{level}", f"-t{threads}", fastq, out], check=True,
                       capture_output=True, timeout=timeout)
        t1 = time.perf_counter()
        subprocess.run([exe, "-d", f"-t{threads}", out, back], check=True,
                       capture_output=True, timeout=timeout)
        t2 = time.perf_counter()
        raw = F.raw_blocks(out)
        same = len(raw) == len(gpu_blocks) and all(
            a == b for a, b in zip(raw, gpu_blocks))
        with open(back, "rb") as fb, open(fastq, "rb") as fs:
            rt = fb.read() == fs.read()
        fsize = os.path.getsize(out)
    return {"value": round(nbytes / (t2 - t0) / 1e6, 2), "unit": "MB/s",
            "cores": threads, "kind": "reference",
            "sample": f"the whole rank-0 workload: oracle/_ref/{exe_name} -{level} "
                      f"-t{threads} on its {nbytes} B FASTQ file, then -d",
            "enc_MBps": round(nbytes / (t1 - t0) / 1e6, 2),
            "dec_MBps": round(nbytes / (t2 - t1) / 1e6, 2),
            "enc_s": round(t1 - t0, 3), "dec_s": round(t2 - t1, 3),
            "fqz5_bytes": fsize, "blocks_match_gpu": bool(same), "roundtrip": bool(rt)}


def t1_check(reads, blocks, level, gpu_blocks, nblk: int, timeout: int = 900):
    """The reference CLI with one thread (-t1: its trial runs in file order,
    fqzcomp5.c:1911-1913) on the workload's first `nblk` blocks, their bytes
    compared with the GPU's first blocks.  The multi-threaded reference run
    of cpu_baseline decides its trial by timing, so its blocks can differ
    from -t1 ones; this is the deterministic comparison."""
    import tempfile
    from fqzcomp5_amd import synth
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fqz5_container as F
    exe = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5")
    if not os.path.exists(exe):
        return {"error": "oracle/_ref/fqzcomp5 not built"}
    from fqzcomp5_amd import sections as S
    nblk = min(nblk, len(blocks))
    try:
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
            src, out = os.path.join(td, "t1.fastq"), os.path.join(td, "t1.fqz5")
            with open(src, "wb") as f:
                f.write(synth.fastq_chunk(reads, blocks[0][0], blocks[nblk - 1][1]).tobytes())
            bs = BLK if level in (3, 5) else S.BLOCK_SIZE[level]
            t0 = time.perf_counter()
            subprocess.run([exe, f"-{level}", "-t1", "-b", str(bs), src, out], check=True,
                           capture_output=True, timeout=timeout)
            t1 = time.perf_counter()
            raw = F.raw_blocks(out)
        same = [bool(a == b) for a, b in zip(raw, gpu_blocks[:nblk])]
        return {"blocks": nblk, "blocks_match_gpu": same, "all_match": all(same) and len(raw) == nblk,
                "ref_enc_s": round(t1 - t0, 2),
                "cmd": f"oracle/_ref/fqzcomp5 -{level} -t1 -b {bs} (first {nblk} blocks)"}
    except Exception as e:       # never lose the line for the check
        return {"error": str(e)[-300:]}


def t1_pin(gpu_blocks, golden: str, fastq_md5=None):
    """The GPU's blocks of the whole workload against the md5s of the
    single-threaded reference's file recorded by a committed script
    (tests/golden/make_golden_l5_novaseq.py: oracle/_ref/fqzcomp5 -5 -t1 on
    the same seeded input): the md5 of all block bytes, and per block."""
    import hashlib
    g = json.load(open(os.path.join(ROOT, "tests", "golden", golden)))
    h = hashlib.md5()
    each = []
    for b in gpu_blocks:
        h.update(b)
        each.append(hashlib.md5(b).hexdigest())
    same = [a == b for a, b in zip(each, g["block_md5s"])]
    out = {"t1_file_md5_match": h.hexdigest() == g["blocks_md5"] and len(each) == g["blocks"],
           "t1_blocks_matching": f"{sum(same)}/{g['blocks']}",
           "gpu_blocks": len(each), "pinned_by": f"tests/golden/{golden} ({g['cmd']}, "
                                                 f"{g['ref_seconds']} s when made)"}
    if fastq_md5 is not None:
        out["input_md5_match"] = fastq_md5 == g["in_md5"]
    return out


def measure(level, kind, gb, steps, warmup, cpu, cpu_threads, world, rank, local, dist,
            scaling="weak", pmc_tag="", dropin=False, t1_blocks=0, gpu_only=False, pin=None):
    """One workload: warmup + `steps` timed steps (barrier + synchronize on
    both sides, max over ranks) and the result fields of its JSON line.  The
    decode places each adaptive-model chain (fqz quality, sequence model) on
    a host core or the GPU by its measured cost (fqz5_set_host_decode(2), the
    library's default).  gpu_only: then time the decode again with every
    chain on the GPU (fqz5_set_host_decode(0)), reported apart."""
    import torch
    from fqzcomp5_amd import lib, sections as S, synth

    t0 = time.time()
    # configs[1]'s seed for its Illumina data at any level, configs[2]'s otherwise
    seed = (1 if level <= 3 or kind == "illumina" else 2) + (rank if scaling == "weak" else 0)
    reads = make_reads(gb, seed, kind)
    blocks = synth.split_blocks(reads, BLK if level in (3, 5) else S.BLOCK_SIZE[level])
    if scaling == "strong":                      # contiguous shard of one file
        nb = len(blocks)
        blocks = blocks[rank * nb // world:(rank + 1) * nb // world]
    log(f"[bench] -{level} {kind} {gb:g} GB: {len(blocks)} blocks on rank 0, generated in "
        f"{time.time()-t0:.1f}s")
    fq_local = sum(synth.fastq_size(reads, a, b) for a, b in blocks)
    dev = torch.device("cuda", local)
    run = S.Run(reads, blocks, dev)
    enc_secs = run.enc_secs()
    avail = S.masks(level, full=True)

    def encode():
        if level >= 7:     # 500 MB / 1 GB blocks: the trial a section at a time
            res, meth_all, sizes, tried, off = S.encode_run_bounded(enc_secs, avail, S.new_state())
        else:
            # -5: the fqz / sequence-model candidates' size intervals first;
            # when they decide the trial, every block's winner is coded in one
            # launch (sections.encode_run, bounds)
            res, meth_all, sizes, tried, off = S.encode_run(enc_secs, avail, S.new_state(),
                                                            bounds=level == 5)
        run.assemble(res)                          # lengths, header, CRC32
        return res, meth_all, tried, off

    def decode(res):
        if not STEP_TRACE:
            return S.decode(run.block_dec_secs())  # parse + CRC check, sections
        a = time.perf_counter()
        secs = run.block_dec_secs()
        b = time.perf_counter()
        out = S.decode(secs)
        c = time.perf_counter()
        torch.cuda.synchronize()
        log(f"[bench] decode: parse {1e3*(b-a):.1f} ms, sections {1e3*(c-b):.1f} ms, "
            f"sync {1e3*(time.perf_counter()-c):.1f} ms")
        return out

    for _ in range(warmup):
        decode(encode()[0])
    arena0 = lib.arena_bytes()
    lib.arena_peak(reset=True)
    lib.arena_use_peak(reset=True)
    so = lib.load()
    fq0 = S.trial_counts()
    ch0 = (C.c_uint64 * 2)()
    so.fqz5_decode_chain_counts(ch0)
    so.fqz5_profile(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_enc = t_dec = 0.0
    enc_steps, dec_steps = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        res, meth_all, tried, off = encode()
        torch.cuda.synchronize()
        if GAP_S:                    # experiments: idle GPU between the phases (untimed)
            time.sleep(GAP_S)
            a += GAP_S
        b = time.perf_counter()
        dres = decode(res)
        torch.cuda.synchronize()
        c = time.perf_counter()
        t_enc += b - a
        t_dec += c - b
        enc_steps.append(b - a)
        dec_steps.append(c - b)
        log(f"[bench] -{level} step: encode {1e3*(b-a):.1f} ms, decode {1e3*(c-b):.1f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = (C.c_double * 6)()
    so.fqz5_profile_read(prof)
    kprof = (C.c_double * (3 * len(PROF_KERNELS)))()
    so.fqz5_profile_read_all(kprof, len(PROF_KERNELS))
    so.fqz5_profile(0)
    fq1 = S.trial_counts()
    arena1 = lib.arena_bytes()
    arena_pk, arena_use = lib.arena_peak(), lib.arena_use_peak()
    # the exchange's tensors live where the process group's backend wants them
    xdev = dev if world == 1 or dist.get_backend() == "nccl" else torch.device("cpu")
    tm = torch.tensor([dt, t_enc, t_dec], dtype=torch.float64, device=xdev)
    tot = torch.tensor([float(fq_local), float(run.in_bytes)], dtype=torch.float64, device=xdev)
    if world > 1:
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    dt, t_enc, t_dec = (float(x) for x in tm.tolist())
    fq_all, sec_all = (float(x) for x in tot.tolist())

    # ---- correctness: every decoded section equals its input -------------
    ok = all(r.status == 0 for r in res) and all(r.status == 0 for r in dres)
    ok = ok and run.roundtrip_ok()
    chains = (C.c_uint64 * 2)()
    so.fqz5_decode_chain_counts(chains)      # (the timed steps': less ch0)
    # ---- the same decode with every fqz / sequence-model chain on the GPU
    # (fqz5_set_host_decode(0)); the figures above stay the item's numbers --
    gonly = None
    if gpu_only:
        prev = so.fqz5_set_host_decode(0)
        try:
            decode(res)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            hs = []
            for _ in range(steps):
                b = time.perf_counter()
                hres = decode(res)
                torch.cuda.synchronize()
                hs.append(time.perf_counter() - b)
        finally:
            so.fqz5_set_host_decode(prev)
        g_ok = all(r.status == 0 for r in hres) and run.roundtrip_ok()
        th = torch.tensor([sum(hs)], dtype=torch.float64,
                          device=dev if world == 1 or dist.get_backend() == "nccl" else torch.device("cpu"))
        if world > 1:
            dist.all_reduce(th, op=dist.ReduceOp.MAX)
        t_gdec = float(th.item())
        gonly = {"dec_ms_per_step": round(t_gdec / steps * 1e3, 2),
                 "dec_MBps": round(fq_all * steps / t_gdec / 1e6, 2),
                 "value": round(fq_all * steps / (t_enc + t_gdec) / 1e6, 2),
                 "roundtrip_ok": bool(g_ok),
                 "note": "the same decode with every fqz / sequence-model chain on the GPU "
                         "(fqz5_set_host_decode(0)); encode as above; same bytes"}
    comp_bytes = int(run.blk_off[-1])
    # the md5 of this rank's block bytes, gathered in rank order: a strong
    # scaling run's list joined equals a one-process run's blocks (rehearsals
    # of the N > 1 path compare them); weak runs code one file per rank
    import hashlib
    bh = hashlib.md5(run.blk_buf[:comp_bytes].cpu().numpy().tobytes()).hexdigest()
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, bh)
    else:
        # FQZ5_BENCH_SPLIT=N: the md5s of the N contiguous shards a strong
        # run over N ranks would code (the comparison for its rehearsal)
        ns = int(os.environ.get("FQZ5_BENCH_SPLIT", "1") or 1)
        nb = len(blocks)
        got = [hashlib.md5(run.blk_buf[int(run.blk_off[r * nb // ns]):
                                       int(run.blk_off[(r + 1) * nb // ns])]
                           .cpu().numpy().tobytes()).hexdigest() for r in range(ns)]
    shape = {"illumina": "illumina 150 bp, Illumina names, 8-level binned quals",
             "novaseq": "novaseq 150 bp, Illumina names, NovaSeq 4-level i.i.d. quals",
             "ont": "ONT reads (lognormal lengths, median 10.5 kb; homopolymer-rich bases; "
                    "AR(1) quals near Q12), read-id names",
             "hifi": "HiFi pairs (~15 kb; 62 % Q93 quals), movie/zmw/ccs names with /1 /2"}[kind]
    blk_mb = (BLK if level in (3, 5) else S.BLOCK_SIZE[level]) // 1_000_000
    full = set(S.preset_methods(level))
    have = set(S.level_methods(level))
    out = {
        "value": round(fq_all * steps / (t_enc + t_dec) / 1e6, 2),
        "ms_per_step": round(dt / steps * 1e3, 2),
        "enc_MBps": round(fq_all * steps / t_enc / 1e6, 2),
        "dec_MBps": round(fq_all * steps / t_dec / 1e6, 2),
        "section_MBps": round(sec_all * steps / (t_enc + t_dec) / 1e6, 2),
        "enc_ms_per_step": round(t_enc / steps * 1e3, 2),
        "dec_ms_per_step": round(t_dec / steps * 1e3, 2),
        # rank 0's fastest / slowest step (spread between steps)
        "enc_ms_min_max": [round(min(enc_steps) * 1e3, 1), round(max(enc_steps) * 1e3, 1)],
        "dec_ms_min_max": [round(min(dec_steps) * 1e3, 1), round(max(dec_steps) * 1e3, 1)],
        "data": f"synthetic (seeded {shape}); records "
                f"resident in HBM; in the timed region only the names come to the host "
                f"(tokenising) and block headers / lengths cross PCIe",
        "config": {"workload": f"fqzcomp5 -{level} whole blocks (names, lengths, seq, qual, "
                               f"CRC) of a {gb:g} GB FASTQ "
                               f"{'per GPU' if scaling == 'weak' else 'in total'}, {blk_mb} MB blocks",
                   "blocks_rank0": len(blocks), "level": level,
                   "fastq_bytes_rank0": fq_local,
                   "section_bytes_rank0": run.in_bytes,
                   "fqz5_block_bytes_rank0": comp_bytes,
                   "methods_tried": sorted(have),
                   "methods_missing": sorted(full - have),
                   "methods_chosen": sorted({int(m) for m in meth_all}),
                   "blocks_md5_by_rank": got,
                   "roundtrip_ok": bool(ok),
                   "parallelism": f"blocks sharded over {world} GPU(s) ({scaling})",
                   "fqz_decoders": dict(zip(("general", "small"), _fqz_dec_counts(so))),
                   # device bytes of the arenas' shared chunk pool (idle
                   # chunks included): held before / after the timed steps
                   # and the peak during them
                   "arena_bytes": {"held_start": int(arena0), "held_end": int(arena1),
                                   "peak_held": int(arena_pk), "peak_in_use": int(arena_use)},
                   # candidates in the timed steps, and how many were provably
                   # losing and skipped their range chain (output unchanged)
                   "fqz_trial": {"tried": fq1[0] - fq0[0], "pruned": fq1[1] - fq0[1],
                                 # -7/-9: whether the candidates' size intervals
                                 # decided the trial (else tried again exactly)
                                 "intervals_decided": S.last_bounds_decided if level >= 5
                                 else None}},
    }
    out["decode_chains"] = {"host": int(chains[0] - ch0[0]), "gpu": int(chains[1] - ch0[1]),
                            "host_threads": int(so.fqz5_host_threads()),
                            "rule": "each fqz / sequence-model chain where its measured cost "
                                    "finishes the decode soonest (fqz5_set_host_decode(2))"}
    if gonly is not None:
        out["gpu_only"] = gonly
    # ---- roofline of the dominant kernel ---------------------------------
    # every chain kernel's launch time from HIP events on the stream it runs
    # on (fqz5_profile_read_all: rANS encode / decode, fqz decode, the fqz
    # and sequence-model range chain, sequence-model decode); the dominant
    # one is the kernel with the most time in the timed steps
    enc_ms, enc_n, enc_b, dec_ms, dec_n, dec_b = list(prof)
    kp = list(kprof)
    per_kernel = {k: {"ms": round(kp[3 * i], 3), "launches": int(kp[3 * i + 1]),
                      "bytes": int(kp[3 * i + 2])} for i, k in enumerate(PROF_KERNELS)}
    name = max(PROF_KERNELS, key=lambda k: per_kernel[k]["ms"])
    ms, n, b = per_kernel[name]["ms"], per_kernel[name]["launches"], per_kernel[name]["bytes"]
    avg_ms = ms / max(n, 1)
    # the algorithmic bytes of a step are the FASTQ text plus
    # the .fqz5 bytes it encodes or decodes (this rank's); the kernel's
    # launches of a step share them, so a launch's share is the step's bytes
    # over its launches per step (the kernel's own stream bytes beside it)
    alg_step = fq_local + comp_bytes
    alg_launch = alg_step * steps / max(n, 1)
    ach = alg_launch / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0
    traffic, tsrc, tnote = pmc_traffic(name, pmc_tag)
    # the decode launch is bound by its longest rANS chain: one step = one
    # symbol on each of the 4 interleaved states
    longest = max((e - s) for _, s, e, _, _ in run.spans)
    out["roofline"] = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 7),
                       "traffic": traffic, "traffic_source": tsrc,
                       "traffic_note": tnote, "kernel": name,
                       "avg_launch_ms": round(avg_ms, 3),
                       "bytes_per_launch": int(alg_launch),
                       "bytes_rule": "SURVEY §8 d3: FASTQ + .fqz5 bytes of a step "
                                     f"({fq_local} + {comp_bytes} B on rank 0) over the "
                                     "kernel's launches per step",
                       "launches_per_step": round(n / max(steps, 1), 3),
                       "kernel_ms_per_step": round(ms / max(steps, 1), 3),
                       "stream_bytes_per_launch": int(b / max(n, 1)),
                       "enc_avg_ms": round(enc_ms / max(enc_n, 1), 3),
                       "dec_avg_ms": round(dec_ms / max(dec_n, 1), 3),
                       "kernels": per_kernel,
                       "chains": {"streams_per_launch": len(run.spans),
                                  "longest_stream_steps": longest // 4,
                                  "dec_ns_per_step_longest": round(
                                      dec_ms / max(dec_n, 1) * 1e6 / max(longest // 4, 1), 2)}}
    # ---- CPU baseline (rank 0, N=1): the reference CLI on the same text -----
    # pinned: this workload's whole file was coded by the -t1 reference and
    # its md5s committed (the rank-0 file of a 1-GPU weak run is that input)
    pinned = pin is not None and rank == 0 and world == 1 and scaling == "weak"
    if pinned and not cpu:
        out["t1_pin"] = t1_pin([run.block_bytes(b) for b in range(len(blocks))], pin)
    if rank == 0 and world == 1 and cpu:
        import tempfile
        gpu_blocks = [run.block_bytes(b) for b in range(len(blocks))]
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
            fastq = os.path.join(td, "w.fastq")
            synth.write_fastq(reads, fastq)
            if pinned:
                import hashlib
                hm = hashlib.md5()
                with open(fastq, "rb") as fz:
                    for c in iter(lambda: fz.read(1 << 24), b""):
                        hm.update(c)
                pin_res = t1_pin(gpu_blocks, pin, hm.hexdigest())
            try:
                out["cpu_baseline"] = cpu_baseline(fastq, level, cpu_threads, gpu_blocks,
                                                   timeout=600 if level <= 5 else 1000)
                # the as-shipped build runs the scalar 32x16 code
                # (its config.h compiles the CPU dispatcher out); the same CLI
                # with the SSE4/AVX2/AVX-512 dispatch compiled in (-7/-9: the
                # fqz and sequence-model coders, which have no SIMD code, bound
                # the reference's time, so the second run is skipped)
                if level <= 5:
                    sb = cpu_baseline(fastq, level, cpu_threads, gpu_blocks, "fqzcomp5_simd")
                    out["cpu_baseline"]["simd_build"] = {
                        k: sb.get(k) for k in ("value", "enc_MBps", "dec_MBps", "blocks_match_gpu")}
            except Exception as e:       # never lose the line for the baseline
                out["cpu_baseline"] = {"error": str(e)[-300:]}
            if dropin:
                out["dropin_cli"] = dropin_item(fastq, level, cpu_threads)
        if pinned:
            out["cpu_baseline"].update(pin_res)
        elif t1_blocks:
            out["cpu_baseline"]["t1_blocks"] = t1_check(reads, blocks, level, gpu_blocks, t1_blocks)
    del run, reads
    # the pool's idle chunks back to the device between items (the next
    # item's arenas start empty)
    so.fqz5_arenas_release()
    torch.cuda.empty_cache()
    return out


def _fqz_dec_counts(so):
    out = (C.c_uint64 * 2)()
    so.fqz5_fqz_dec_counts(out)
    return [int(out[0]), int(out[1])]


def crc_item(lib, torch, gib: int = 4, reps: int = 5):
    """The block checksum (zlib crc32 of a block, fqzcomp5.c:2268-2269) on a
    device-resident 4 GiB buffer: fqz5_crc32_dev wall time per call (best of
    `reps`, table upload + tile kernel + combine passes + sync), checked
    against zlib on a 1 MiB prefix.  HBM-bound: 1 B read per input byte."""
    import zlib
    try:
        n = gib << 30
        d = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ok = lib.crc32_dev(d.data_ptr(), 1 << 20) == zlib.crc32(d[:1 << 20].cpu().numpy().tobytes())
        lib.crc32_dev(d.data_ptr(), n)
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            lib.crc32_dev(d.data_ptr(), n)
            best = min(best, time.perf_counter() - t0)
        del d
        gbs = n / best / 1e9
        return {"bytes": n, "ms": round(best * 1e3, 3), "GB/s": round(gbs, 1),
                "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0,
                             "unit": "GB/s", "frac": round(gbs / 8000.0, 4),
                             "kernel": "k_crc_tiles (whole call timed)"},
                "matches_zlib": bool(ok)}
    except Exception as e:   # the item is informative; never lose the line for it
        return {"error": str(e)}


def dropin_item(fastq: str, level: int, threads: int, timeout: int = 600):
    """The reference CLI relinked on libfqz5_mi355x.so (oracle/_ref/
    fqzcomp5_gpu, the drop-in of INTEGRATION.md) on the workload's FASTQ
    file with -t<threads>: wall time of encode and decode, its .fqz5 bytes
    compared with the CLI as shipped.  Host buffers: every codec call copies
    its block to the GPU and back (PCIe included).  Then the library's own
    file path (fqz5file.compress_file / decompress_file) on the same file:
    file to file, disk cache and PCIe included."""
    import hashlib
    import tempfile
    cpu = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5")
    gpu = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5_gpu")
    if not (os.path.exists(cpu) and os.path.exists(gpu)):
        return {"error": "oracle/_ref CLIs not built"}
    try:
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
            nbytes = os.path.getsize(fastq)
            res = {"fastq_bytes": nbytes, "level": level, "threads": threads}
            md5 = {}
            for tag, exe in (("gpu", gpu), ("cpu", cpu)):
                out = os.path.join(td, tag + ".fqz5")
                back = os.path.join(td, tag + ".fastq")
                t0 = time.perf_counter()
                subprocess.run([exe, f"-{level}", f"-t{threads}", fastq, out], check=True,
                               capture_output=True, timeout=timeout)
                t1 = time.perf_counter()
                subprocess.run([exe, "-d", f"-t{threads}", out, back], check=True,
                               capture_output=True, timeout=timeout)
                t2 = time.perf_counter()
                md5[tag] = hashlib.md5(open(out, "rb").read()).hexdigest()
                with open(back, "rb") as fb, open(fastq, "rb") as fs:
                    same = fb.read() == fs.read()
                res[tag] = {"enc_MBps": round(nbytes / (t1 - t0) / 1e6, 2),
                            "dec_MBps": round(nbytes / (t2 - t1) / 1e6, 2),
                            "enc_s": round(t1 - t0, 3), "dec_s": round(t2 - t1, 3),
                            "roundtrip": same}
                os.unlink(back)
            res["bytes_match"] = md5["cpu"] == md5["gpu"]
            # this library's own file path on the same file (fqz5file:
            # page-locked read, one copy to HBM, whole blocks, one copy back)
            from fqzcomp5_amd import fqz5file
            out = os.path.join(td, "native.fqz5")
            back = os.path.join(td, "native.fastq")
            t0 = time.perf_counter()
            fqz5file.compress_file(fastq, out, level)
            t1 = time.perf_counter()
            fqz5file.decompress_file(out, back)
            t2 = time.perf_counter()
            with open(back, "rb") as fb, open(fastq, "rb") as fs:
                same = fb.read() == fs.read()
            res["gpu_file_path"] = {
                "enc_MBps": round(nbytes / (t1 - t0) / 1e6, 2),
                "dec_MBps": round(nbytes / (t2 - t1) / 1e6, 2),
                "enc_s": round(t1 - t0, 3), "dec_s": round(t2 - t1, 3), "roundtrip": same,
                "bytes_match_cli": hashlib.md5(open(out, "rb").read()).hexdigest() == md5["cpu"]}
            os.unlink(back)
            return res
    except Exception as e:
        return {"error": str(e)[-300:]}


def relaunch(n: int) -> None:
    """Start `n` ranks of this script under torch.distributed.run (one
    process per GPU) and exit with its status.  Runs before anything has
    touched the GPU."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    raise SystemExit(subprocess.call(cmd, env=env))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--level", type=int, default=3, choices=[1, 3, 5, 7, 9])
    ap.add_argument("--kind", default="illumina", choices=["illumina", "novaseq", "ont", "hifi"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-level5", action="store_true",
                    help="skip the configs[2] (-5 NovaSeq 4 GB) line item")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the CPU baseline (0: all this process may use)")
    ap.add_argument("--no-crc", action="store_true", help="skip the block-checksum item")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in CLI item")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        relaunch(args.gpus)

    import torch
    import torch.distributed as dist
    from fqzcomp5_amd import lib

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # FQZ5_BENCH_SHARE_GPU=1 (rehearsal of the N > 1 path on a box with fewer
    # GPUs than ranks): ranks share the visible GPUs round-robin and exchange
    # over gloo, since RCCL refuses two ranks on one device
    share = os.environ.get("FQZ5_BENCH_SHARE_GPU") == "1"
    if share:
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if share:
            dist.init_process_group("gloo")
            chk = torch.ones(1)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            chk = torch.ones(1, device="cuda")
        dist.all_reduce(chk)
        assert int(chk.item()) == world, "the process group does not see every rank"
    if not lib.device_ok():
        raise SystemExit("no GPU: " + lib.last_error())
    threads = args.cpu_threads or host_threads()

    m = measure(args.level, args.kind, args.gb, args.steps, args.warmup, not args.no_cpu,
                threads, world, rank, local, dist, scaling=args.scaling,
                pmc_tag="" if args.level == 3 else f"_l{args.level}",
                dropin=not args.no_dropin and args.level == 3)
    out = {"metric": "input MB/s encode+decode, 100MB blocks, -3 and -5; bit-exact vs CPU",
           "value": m["value"], "unit": "MB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": m["ms_per_step"], "higher_is_better": True,
           "scaling": args.scaling, "vs_baseline": None, "dtype": "u8", "data": m["data"],
           "config": m["config"], "enc_MBps": m["enc_MBps"], "dec_MBps": m["dec_MBps"],
           "section_MBps": m["section_MBps"], "enc_ms_per_step": m["enc_ms_per_step"],
           "dec_ms_per_step": m["dec_ms_per_step"], "enc_ms_min_max": m["enc_ms_min_max"],
           "dec_ms_min_max": m["dec_ms_min_max"], "roofline": m["roofline"]}
    if "cpu_baseline" in m:
        out["cpu_baseline"] = m["cpu_baseline"]
    if "dropin_cli" in m:
        out["dropin_cli"] = m.pop("dropin_cli")
    # The metric covers -3 and -5: the default run adds configs[2] (-5,
    # 4 GB NovaSeq per GPU) as its own item with the same timing rules;
    # `value` stays configs[1] (-3).
    if not args.no_level5 and args.level == 3:
        out["level5"] = measure(5, "novaseq", 4.0 if args.scaling == "weak" else 4.0 * world,
                                args.steps, args.warmup, not args.no_cpu, threads, world,
                                rank, local, dist, scaling=args.scaling, pmc_tag="_l5",
                                t1_blocks=4, pin="l5_novaseq.json")
        # -5 on configs[1]'s data: the random-walk binned Illumina qualities,
        # where the trial picks fqz (FQZ1/FQZ3, fqzcomp5.c:4906-4907), so the
        # fqz range coder and decoder are in the timed region; each block's
        # quality section is one fqz chain, so a step lasts about one block's
        # decode: fewer steps
        out["level5_illumina"] = measure(5, "illumina", args.gb if args.scaling == "weak"
                                         else args.gb * world, min(args.steps, 2),
                                         min(args.warmup, 1), not args.no_cpu, threads, world,
                                         rank, local, dist, scaling=args.scaling,
                                         pmc_tag="_l5i", t1_blocks=4, gpu_only=True)
    if rank == 0 and world == 1 and not args.no_crc:
        out["crc32"] = crc_item(lib, torch)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
