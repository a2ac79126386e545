"""Timeline of a rocprofv3 kernel trace: the dispatches of the last `span`
seconds (or between two times), longest first within a window, as
start/end ms relative to the window start.  Usage:
  python tools/timeline.py kt_kernel_trace.csv [span_s] [min_ms]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].split("(")[0][:60], int(r["Queue_Id"]), int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)))
rows.sort()
span = float(sys.argv[2]) if len(sys.argv) > 2 else 1.7
mn = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
end = max(r[1] for r in rows)
t0 = end - int(span * 1e9)
sel = [r for r in rows if r[1] >= t0]
base = min(r[0] for r in sel)
busy = []
for s, e, n, q, g in sel:
    if (e - s) / 1e6 >= mn:
        print(f"{(s-base)/1e6:9.1f} {(e-base)/1e6:9.1f} {(e-s)/1e6:8.2f} q{q:<3} wg{g:<6} {n}")
# idle gaps (no kernel running) longer than 1 ms
iv = sorted((s, e) for s, e, *_ in sel)
cur_s, cur_e = iv[0]
gaps = []
for s, e in iv[1:]:
    if s > cur_e:
        gaps.append((cur_e, s))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
print("idle gaps > 1 ms:", [(round((a-base)/1e6, 1), round((b-a)/1e6, 1)) for a, b in gaps if b - a > 1e6])
