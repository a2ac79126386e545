"""Per-kernel duration summary from a rocprofv3 rocpd SQLite database
(used when the run was not asked for CSV output)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
t = {r[0].rsplit('_', 5)[0]: r[0] for r in db.execute(
    "select name from sqlite_master where type='table'")}
kd, ks = t['rocpd_kernel_dispatch'], t['rocpd_info_kernel_symbol']
rows = db.execute(f"""select s.kernel_name, count(*), sum(d.end - d.start),
    avg(d.end - d.start), min(d.end - d.start), max(d.end - d.start)
    from {kd} d join {ks} s on d.kernel_id = s.id group by s.kernel_name
    order by sum(d.end - d.start) desc""").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':60s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>9s} {'min_ms':>9s} {'max_ms':>9s} {'pct':>6s}")
for n, c, s, a, mn, mx in rows:
    print(f"{n[:60]:60s} {c:6d} {s/1e6:10.3f} {a/1e6:9.3f} {mn/1e6:9.3f} {mx/1e6:9.3f} {100*s/tot:6.2f}")
