#!/usr/bin/env python3
"""Benchmark: fqzcomp5 sequence+quality section coding on MI355X.

Metric (BASELINE.json): input MB/s encode+decode, 100 MB blocks, -3 and -5;
bit-exact vs CPU.  Default workload (configs[1]): a synthetic 1 GB Illumina
150 bp FASTQ with 8-level binned qualities at -3, split into 100 MB blocks
by the reference's record rule (fqzcomp5.c:471-477).  `--level 5 --kind
novaseq --gb 4` is configs[2] (the quality methods add FQZ1/FQZ3).  One step
is one pass of the hot path over the whole workload, inputs resident in HBM:

    encode  every block's seq and qual section with the level's method sets
            and the codec-trial state machine (fqzcomp5.c:1899-2144)
    decode  every chosen stream back to bytes.

`value` = seq+qual section bytes of all ranks / step time (max over ranks).
The default run adds configs[2] as the `level5` line item: a synthetic 4 GB
NovaSeq FASTQ per GPU at -5 (fqzcomp_qual FQZ1/FQZ3 in the codec trial),
timed with the same rules (`--no-level5` skips it).
Names (tok3/LZP) and LZP3 for sequences are the next rows of SURVEY §8f
and are not in the workload; the sequence context models SEQ10/SEQ12B of
the -5 preset are built (seq_cm.hip) but left out of the -5 masks while
their decoder is one slow chain per block.  The `crc32` item
times the block checksum (zlib crc32) over a 4 GiB device buffer.
Multi-GPU: one process per GPU, weak scaling
(each rank adds its own 1 GB file to the run); the only collective is the
all-gather of candidate sizes that the trial state needs.

Also reported: the roofline of the dominant kernel from live HIP events on
the library's stream, and the reference CPU path (oracle/_ref, compiled
from the reference sources) timed on the host cores on the same bytes,
whose output bytes are compared with the GPU's.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FASTQ_REC = 346          # bytes per synthetic 150 bp FASTQ record (avg)
BLK = 100_000_000        # -3 block size (fqzcomp5.c:4913)
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8 TB/s spec


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_blocks(gb: float, seed: int, kind: str):
    from fqzcomp5_amd import synth
    n_reads = int(gb * 1e9 / FASTQ_REC)
    r = (synth.novaseq if kind == "novaseq" else synth.illumina)(n_reads, seed=seed)
    return r, synth.split_blocks(r, BLK)


def pmc_traffic(kernel: str, tag: str = ""):
    """HBM bytes per dispatch of `kernel` from the newest committed PMC
    summary of this workload (profiles/rNN_pmc{tag}.json, written by
    tools/pmc_summary.py from separate rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of this bench; tag "" = configs[1] -3, "_l5" = configs[2] -5)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc{tag}.json")))
    if not files:
        return None, None
    ks = json.load(open(files[-1]))["kernels"]
    for k, v in ks.items():
        if f"::{kernel}(" in k:
            return int(v["hbm_bytes_per_dispatch"]), os.path.relpath(files[-1], ROOT)
    return None, None


def method_order(m: int, fixed_len: int) -> int:
    return [0, 1, 64, 65, 128, 129, 192, 193][m - 1] if m <= 8 else (fixed_len << 8) + 9


def cpu_baseline(run, tried, meth, gpu_out, threads):
    """The reference (oracle/_ref) on the same sections and schedule: every
    tried method of every section is compressed, the chosen stream is
    checked against the GPU's bytes and decoded again."""
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from oracle import binding
    from fqzcomp5_amd import sections as S
    kind = "reference" if binding.have_ref() else "port"
    codec = binding.ref() if kind == "reference" else binding.oracle()
    reads = run.reads
    secs = []
    for sec, s, e, fl, k in run.spans:
        arr = reads.seq if sec == S.SEC_SEQ else reads.qual
        a, b = run.blocks[k]
        secs.append((arr[s:e].tobytes(), fl, reads.lens[a:b].copy(),
                     reads.seq[s:e].tobytes()))

    def enc(i):
        data, fixed, lens, seq = secs[i]
        best = None
        for m in range(1, S.M_LAST):
            if not tried[i] & (1 << m) or (m == S.RANSXN1 and not fixed):
                continue
            if m >= S.FQZ0:
                out = codec.fqz_compress(data, lens.copy(), np.zeros(len(lens), np.uint32),
                                         m - S.FQZ0, seq)
            else:
                out = codec.rans_compress(data, method_order(m, fixed))
            if m == meth[i]:
                best = out
        return best

    def dec(i):
        data, fixed, lens, seq = secs[i]
        if meth[i] >= S.FQZ0:
            return codec.fqz_decompress(chosen[i], lens.copy(), np.zeros(len(lens), np.uint32), seq)
        return codec.rans_uncompress(chosen[i])

    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        chosen = list(ex.map(enc, range(len(secs))))
        t1 = time.perf_counter()
        back = list(ex.map(dec, range(len(secs))))
        t2 = time.perf_counter()
    same = all(c == g for c, g in zip(chosen, gpu_out))
    rt = all(b == h[0] for b, h in zip(back, secs))
    nbytes = sum(len(h[0]) for h in secs)
    return {"value": round(nbytes / (t2 - t0) / 1e6, 2), "unit": "MB/s",
            "cores": threads, "kind": kind,
            "sample": f"all {len(secs)} seq+qual sections of the rank-0 "
                      f"workload, the -t1 trial schedule (every tried "
                      f"candidate encoded), {threads} host threads",
            "enc_s": round(t1 - t0, 3), "dec_s": round(t2 - t1, 3),
            "bytes_match_gpu": bool(same), "roundtrip": bool(rt)}


def measure(level, kind, gb, steps, warmup, cpu, cpu_threads, world, rank, local, dist,
            pmc_tag=""):
    """One workload: warmup + `steps` timed steps (barrier + synchronize on
    both sides, max over ranks) and the result fields of the JSON line."""
    import torch
    from fqzcomp5_amd import lib, sections as S

    t0 = time.time()
    reads, blocks = make_blocks(gb, seed=(1 if level <= 3 else 2) + rank, kind=kind)
    log(f"[bench] -{level} {kind} {gb:g} GB: generated {len(blocks)} blocks/rank in "
        f"{time.time()-t0:.1f}s")
    dev = torch.device("cuda", local)
    run = S.Run(reads, blocks, dev)
    enc_secs = run.enc_secs()
    avail = S.masks(level)
    in_bytes_local = run.in_bytes

    def step():
        state = S.new_state()
        res, meth_all, sizes, tried, off = S.encode_run(enc_secs, avail, state)
        dres = S.decode(run.dec_secs(res))
        return res, dres, meth_all, tried, off

    for _ in range(warmup):
        step()
    so = lib.load()
    fq0 = S.trial_counts()
    so.fqz5_profile(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res, dres, meth_all, tried, off = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = (C.c_double * 6)()
    so.fqz5_profile_read(prof)
    so.fqz5_profile(0)
    fq1 = S.trial_counts()
    t_max = torch.tensor([dt], dtype=torch.float64, device=dev)
    tot_bytes = torch.tensor([float(in_bytes_local)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot_bytes, op=dist.ReduceOp.SUM)
    dt = float(t_max.item())

    # ---- correctness: every decoded section equals its input -------------
    ok = all(r.status == 0 for r in res) and all(r.status == 0 for r in dres)
    ok = ok and run.roundtrip_ok()
    comp_bytes = sum(9 + r.clen for r in res)
    quals = "8-level binned quals" if kind == "illumina" else "NovaSeq 4-level i.i.d. quals"
    out = {
        "value": round(float(tot_bytes.item()) * steps / dt / 1e6, 2),
        "ms_per_step": round(dt / steps * 1e3, 2),
        "data": f"synthetic (seeded {kind} 150 bp, {quals})",
        "config": {"workload": f"fqzcomp5 -{level} seq+qual sections of a "
                               f"{gb:g} GB FASTQ per GPU, 100 MB blocks",
                   "blocks_per_gpu": len(blocks), "level": level,
                   "section_bytes_per_gpu": in_bytes_local,
                   "compressed_bytes_per_gpu": comp_bytes,
                   "methods": sorted({int(m) for m in meth_all}),
                   "roundtrip_ok": bool(ok),
                   "parallelism": f"blocks sharded over {world} GPU(s)",
                   # fqz trial candidates in the timed steps, and how many
                   # were provably losing and skipped their range chain
                   # (fqz5_set_trial_prune; output bytes unchanged)
                   "fqz_trial": {"tried": fq1[0] - fq0[0], "pruned": fq1[1] - fq0[1]}},
    }
    # ---- roofline of the dominant kernel ---------------------------------
    enc_ms, enc_n, enc_b, dec_ms, dec_n, dec_b = list(prof)
    if enc_ms >= dec_ms:
        name, ms, n, b = "k_rans_enc", enc_ms, enc_n, enc_b
    else:
        name, ms, n, b = "k_rans_dec", dec_ms, dec_n, dec_b
    avg_ms = ms / max(n, 1)
    ach = (b / max(n, 1)) / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0
    traffic, tsrc = pmc_traffic(name, pmc_tag)
    # the decode launch is bound by its longest rANS chain: one step = one
    # symbol on each of the 4 interleaved states
    longest = max((e - s) for _, s, e, _, _ in run.spans)
    out["roofline"] = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 6),
                       "traffic": traffic, "traffic_source": tsrc, "kernel": name,
                       "avg_launch_ms": round(avg_ms, 3),
                       "bytes_per_launch": int(b / max(n, 1)),
                       "enc_avg_ms": round(enc_ms / max(enc_n, 1), 3),
                       "dec_avg_ms": round(dec_ms / max(dec_n, 1), 3),
                       "chains": {"streams_per_launch": len(run.spans),
                                  "longest_stream_steps": longest // 4,
                                  "dec_ns_per_step_longest": round(
                                      dec_ms / max(dec_n, 1) * 1e6 / max(longest // 4, 1), 2)}}
    # ---- CPU baseline (rank 0, N=1) -----------------------------------------
    if rank == 0 and world == 1 and cpu:
        gpu_streams = [run.chosen(res, i) for i in range(len(res))]
        threads = min(cpu_threads, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(run, tried[off:off + len(res)],
                                           meth_all[off:off + len(res)], gpu_streams, threads)
    del run, reads
    torch.cuda.empty_cache()
    return out


def crc_item(lib, torch, gib: int = 4, reps: int = 5):
    """The block checksum (zlib crc32 of a block, fqzcomp5.c:2268-2269) on a
    device-resident 4 GiB buffer: fqz5_crc32_dev wall time per call (best of
    `reps`, table upload + tile kernel + combine passes + sync), checked
    against zlib on a 1 MiB prefix.  HBM-bound: 1 B read per input byte."""
    import time
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--level", type=int, default=3, choices=[1, 3, 5])
    ap.add_argument("--kind", default="illumina", choices=["illumina", "novaseq"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-level5", action="store_true",
                    help="skip the configs[2] (-5 NovaSeq 4 GB) line item")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-crc", action="store_true", help="skip the block-checksum item")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from fqzcomp5_amd import lib

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if not lib.device_ok():
        raise SystemExit("no GPU: " + lib.last_error())

    m = measure(args.level, args.kind, args.gb, args.steps, args.warmup, not args.no_cpu,
                args.cpu_threads, world, rank, local, dist,
                pmc_tag="_l5" if args.level == 5 else "")
    out = {"metric": "input MB/s encode+decode, 100MB blocks, -3 and -5; bit-exact vs CPU",
           "value": m["value"], "unit": "MB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": m["ms_per_step"], "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": m["data"],
           "config": m["config"], "roofline": m["roofline"]}
    if "cpu_baseline" in m:
        out["cpu_baseline"] = m["cpu_baseline"]
    # The metric covers -3 and -5: the default run adds configs[2] (-5,
    # fqzcomp_qual candidates in the trial, 4 GB NovaSeq per GPU) as its own
    # line item with the same timing rules; `value` stays configs[1] (-3).
    if not args.no_level5 and args.level == 3:
        m5 = measure(5, "novaseq", 4.0, args.steps, args.warmup, not args.no_cpu,
                     args.cpu_threads, world, rank, local, dist, pmc_tag="_l5")
        out["level5"] = m5
    if rank == 0 and not args.no_crc:
        out["crc32"] = crc_item(lib, torch)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
