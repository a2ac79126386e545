"""Counter values of one kernel from rocprofv3 --pmc result databases.

python tools/pmc_db.py <kernel substring> <nsym> <db> [<db> ...]
Sums each counter over the dispatches of the kernel whose name contains
the substring and prints it, with per-symbol values when nsym > 0 (the
decoder PMC runs, tools/dec_pmc.sh).  SQ_WAVE_CYCLES and the SQ wait /
active counters count in units of 4 cycles per wave on gfx950 (the SQ
samples every fourth clock), so cycle counters are also shown x4.
"""
import sqlite3
import sys

kern, nsym, dbs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
tot = {}
for db in dbs:
    c = sqlite3.connect(db)
    for name, cn, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
        if kern in name:
            tot[cn] = tot.get(cn, 0.0) + float(val)
for k in sorted(tot):
    v = tot[k]
    line = f"{k:28s} {v:16.0f}"
    if nsym:
        line += f"   per symbol {v / nsym:10.2f}"
        if "CYCLES" in k or k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE"):
            line += f"   x4 {4 * v / nsym:10.1f}"
    print(line)
