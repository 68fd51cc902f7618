"""Per-kernel summary (calls, total / average us) of a rocprofv3 rocpd
database: python tools/rocpd_summary.py <run_results.db> [top]"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
c = sqlite3.connect(db)
q = ("select name, count(*), sum(duration)/1e3, avg(duration)/1e3 from kernels "
     "group by name order by sum(duration) desc limit ?")
print(f"{'kernel':90s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s}")
for r in c.execute(q, (top,)):
    print(f"{r[0][:90]:90s} {r[1]:6d} {r[2]:10.1f} {r[3]:9.1f}")
