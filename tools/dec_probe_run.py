"""Cycle stamps of the O0 NX=4 decoder (a library built with
tools/build_variant.sh cprobe rans_chain -DFQZ5_CHAIN_PROBE): total and
full-step-loop shader cycles of the first stream of the launch, the
in-kernel clock from s_memrealtime (100 MHz), cycles per step."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/variants/libfqz5_cprobe.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch's HIP runtime first, as in tests/conftest.py)
torch.cuda.init()
from fqzcomp5_amd import lib, synth  # noqa: E402

r = synth.illumina(int(sys.argv[1]) if len(sys.argv) > 1 else 290000, seed=1)
so = lib.load()
for name, data in (("seq", r.seq.tobytes()), ("qual", r.qual.tobytes()))[:1 if "bench" in sys.argv else 2]:
    comp = lib.rans_compress(data, 0)
    back = lib.rans_uncompress(comp)
    p = (C.c_uint64 * 8)()
    so.fqz5_chain_probe_read(p)
    tot, real, ts, ns, T = p[2], p[3], p[4], p[5], p[6]
    ghz = tot / (real * 10.0) if real else 0
    print(f"{name} O0 ok={back == data} steps={T} total {tot} cyc ({tot/max(T,1):.1f}/step) "
          f"loop {ts} cyc over {ns} steps ({ts/max(ns,1):.1f}/step) clock {ghz:.3f} GHz "
          f"wall {real/100:.0f} us", flush=True)

if len(sys.argv) > 2 and sys.argv[2] == "bench":
    # the bench's -3 workload: the longest stream is job 0 of the decode launch
    sys.argv = sys.argv[:1]
    import bench
    from fqzcomp5_amd import sections as S
    reads, blocks = bench.make_blocks(1.0, seed=1, kind="illumina")
    run = S.Run(reads, blocks, torch.device("cuda", 0))
    enc_secs = run.enc_secs()
    for rep in range(2):
        res, meth_all, sizes, tried, off = S.encode_run(enc_secs, S.masks(3), S.new_state())
        so.fqz5_profile(1)
        dres = S.decode(run.dec_secs(res))
        pr = (C.c_double * 6)()
        so.fqz5_profile_read(pr)
        so.fqz5_profile(0)
        p = (C.c_uint64 * 8)()
        so.fqz5_chain_probe_read(p)
        tot, real, ts, ns, T = p[2], p[3], p[4], p[5], p[6]
        print(f"bench launch: dec {pr[3]:.1f} ms; job0 steps={T} {tot/max(T,1):.1f} cyc/step "
              f"loop {ts/max(ns,1):.1f}/step clock {tot/(real*10.0):.3f} GHz wall {real/100:.0f} us",
              flush=True)
        jt = (C.c_uint64 * (512 * 8))()
        so.fqz5_chain_jobs_read(jt)
        t0 = min(jt[8 * i] for i in range(len(dres)) if jt[8 * i])
        for i in range(len(dres)):
            a, b, cyc, k, lc, ls = jt[8 * i:8 * i + 6]
            n = k >> 32
            print(f"  job {i:2d} n={n:9d} xcc={(k >> 24) & 15} cu={(k >> 16) & 15} se={(k >> 8) & 7} "
                  f"simd={k & 3} end {(b - t0) / 100:8.0f} us ns/step {(b - a) * 10 / max(n / 4, 1):.1f} "
                  f"cyc/step {cyc / max(n / 4, 1):.1f} loop {lc / max(ls, 1):.1f} clock {cyc / max((b - a) * 10, 1):.3f} GHz")

if len(sys.argv) > 2 and sys.argv[2] == "same":
    # one stream decoded by 20 / 80 waves of one launch: per-CU spread of a
    # chain with identical data
    data = r.seq.tobytes()
    comp = lib.rans_compress(data, 0)
    cin = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    for nj in (20, 80):
        outs = [torch.empty(len(data), dtype=torch.uint8, device="cuda") for _ in range(nj)]
        jobs = [lib.RansJob(cin.data_ptr(), o.data_ptr(), len(comp), len(data), 0, 0, 0, 0) for o in outs]
        lib.uncompress_batch_dev(jobs)
        jt = (C.c_uint64 * (512 * 8))()
        so.fqz5_chain_jobs_read(jt)
        cyc = [jt[8 * i + 2] / (len(data) / 4) for i in range(nj)]
        lp = [jt[8 * i + 4] / max(jt[8 * i + 5], 1) for i in range(nj)]
        xcc = [(jt[8 * i + 3] >> 24) & 15 for i in range(nj)]
        ok = all(bytes(o.cpu().numpy()) == data for o in outs[:2])
        print(f"same stream x{nj}: ok={ok} cyc/step min {min(cyc):.1f} max {max(cyc):.1f}; "
              f"loop min {min(lp):.1f} max {max(lp):.1f}", flush=True)
        info = [jt[8 * i + 3] for i in range(nj)]
        from collections import defaultdict
        for name, f in (("simd", lambda k: k & 3), ("cu", lambda k: (k >> 16) & 15),
                        ("se", lambda k: (k >> 8) & 7), ("xcc", lambda k: (k >> 24) & 15)):
            d = defaultdict(list)
            for k, c in zip(info, lp):
                d[f(k)].append(c)
            print(f"  by {name}:", {key: (len(v), round(sum(v) / len(v), 1)) for key, v in sorted(d.items())}, flush=True)
