"""Per-kernel HBM traffic from rocprofv3 PMC passes (tools/profile.sh).

FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KB per dispatch.
MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE counts half the
bytes of a coalesced streaming read, so it is doubled; WRITE_SIZE is exact.
Usage: python tools/pmc_summary.py <prof dir> <out.json> [extra note]
"""
import csv
import json
import sys


def load(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        a = agg.setdefault(name, [0, 0.0, 0.0])
        v = float(r["Counter_Value"]) * 1024.0
        a[0] += 1
        a[1] += v
        a[2] = max(a[2], v)
    return agg


d = sys.argv[1]
fetch = load(f"{d}/fetch/fetch_counter_collection.csv")
write = load(f"{d}/write/write_counter_collection.csv")
out = {}
for k in sorted(set(fetch) | set(write)):
    fn, fb, fm = fetch.get(k, [0, 0.0, 0.0])
    wn, wb, wm = write.get(k, [0, 0.0, 0.0])
    if "fqz5::" not in k or "::k_" not in k:   # this library's kernels (templates included)
        continue
    f = 2.0 * fb / max(fn, 1)
    w = wb / max(wn, 1)
    out[k] = {"dispatches": max(fn, wn), "fetch_bytes": round(f), "write_bytes": round(w),
              "hbm_bytes_per_dispatch": round(f + w),
              # the largest dispatch of each pass (e.g. a step's main decode
              # launch beside small ones; the passes are separate runs)
              "hbm_bytes_max_dispatch": round(2.0 * fm + wm)}
json.dump({"note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, bytes per dispatch "
                   "(mean over dispatches, and of the largest dispatch); the passes run "
                   "bench.py with its defaults, so a hedged launch's copies are counted "
                   "as they ran in the timed steps" + (f"; {sys.argv[3]}" if len(sys.argv) > 3 else ""),
           "kernels": out}, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1)[:2000])
