"""Per-job timing of one bench decode launch (a library built with
tools/build_variant.sh cprobe rans_chain -DFQZ5_CHAIN_PROBE): for the -3 or
-5 bench workload, every workgroup of the k_rans_dec launch (hedged copies
included) with its stream's size, order (O0 / O1 rows), steps and ns/step.
Usage: dec_jobs_probe.py [3|5]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FQZ5_LIB_VARIANT", os.path.join(ROOT, "tools/probe/libfqz5_cprobe.so"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets the HIP queue count before torch)
import torch  # noqa: E402
from fqzcomp5_amd import lib, sections as S, synth  # noqa: E402

level = int(sys.argv[1]) if len(sys.argv) > 1 else 5
reads = (bench.make_reads(1.0, 1, "illumina") if level == 3 else bench.make_reads(4.0, 2, "novaseq"))
blocks = synth.split_blocks(reads, bench.BLK)
run = S.Run(reads, blocks, torch.device("cuda", 0))
enc = run.enc_secs()
so = lib.load()
for rep in range(2):
    res, meth, sizes, tried, off = S.encode_run(enc, S.masks(level, full=True), S.new_state())
    so.fqz5_profile(1)
    dres = S.decode(run.dec_secs(res))
    pr = (C.c_double * 6)()
    so.fqz5_profile_read(pr)
    so.fqz5_profile(0)
print("methods per section (seq, qual):", [int(m) for m in meth[:6]], "...")
jt = (C.c_uint64 * (512 * 8))()
so.fqz5_chain_jobs_read(jt)
rows = []
for i in range(512):
    a, b, cyc, k, lc, ls, ext, inl = jt[8 * i:8 * i + 8]
    if not a:
        continue
    n = k >> 32
    o1rows, nx, mode = ext & 0xffff, (ext >> 16) & 0xff, ext >> 24
    steps = (n - (nx - 1) * (n // nx)) if o1rows else (n + nx - 1) // nx
    rows.append((b, i, n, o1rows, nx, mode, steps, lc / max(ls, 1), cyc / max(steps, 1), inl))
t0 = min(r[0] for r in rows)
print(f"launch {pr[3]:.1f} ms, {len(rows)} workgroups")
for r in sorted(rows)[-40:]:
    b, i, n, o1rows, nx, mode, steps, loopc, cps, inl = r
    print(f"wg {i:3d} n={n:9d} in={inl:9d} {'O1 rows=' + str(o1rows) if o1rows else 'O0'} nx={nx} mode={mode} "
          f"steps={steps:9d} {cps:6.1f} cyc/step (fast loop {loopc:6.1f})")
# shader clock per workgroup: its cycles over its wall time (s_memrealtime, 100 MHz)
clk = []
for i in range(512):
    a, b, cyc, k, lc, ls, ext, inl = jt[8 * i:8 * i + 8]
    if a and b > a:
        clk.append(cyc / ((b - a) * 10.0))
# placement: waves that shared a CU / a SIMD while both ran (XCC, SE, CU,
# SIMD from HW_ID, fqz5 rans_chain.hip probe word 3)
pl = []
for i in range(512):
    a, b, cyc, k, lc, ls, ext, inl = jt[8 * i:8 * i + 8]
    if a:
        pl.append((a, b, (k >> 24) & 0xf, (k >> 8) & 0x7, (k >> 16) & 0x1f, k & 3, i))
share_cu = share_simd = 0
on_shared = set()
for x in range(len(pl)):
    for y in range(x + 1, len(pl)):
        p1, p2 = pl[x], pl[y]
        if p1[0] < p2[1] and p2[0] < p1[1] and p1[2:5] == p2[2:5]:
            share_cu += 1
            if p1[5] == p2[5]:
                share_simd += 1
                on_shared.update((p1[6], p2[6]))
loop = {r[1]: r[7] for r in rows}
big = [r for r in rows if r[6] > 1000000]
for name, sel in (("sharing a SIMD", [r for r in big if r[1] in on_shared]),
                  ("alone on their SIMD", [r for r in big if r[1] not in on_shared])):
    if sel:
        print(f"long chains {name}: {len(sel)}, fast loop {sum(r[7] for r in sel)/len(sel):.1f} cyc/step")
print(f"overlapping wave pairs on one CU: {share_cu}, on one SIMD: {share_simd} "
      f"(of {len(pl)} workgroups; XCCs {sorted(set(q[2] for q in pl))})")
if clk:
    clk.sort()
    print(f"shader clock over the launch's workgroups: min {clk[0]:.3f} median {clk[len(clk)//2]:.3f} "
          f"max {clk[-1]:.3f} GHz ({len(clk)} workgroups)")
