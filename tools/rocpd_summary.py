"""Per-kernel summary of a rocprofv3 rocpd database (the ROCm 7 default output):
python tools/rocpd_summary.py <results.db> [name-filter] -> count / avg / total per kernel
and the mean idle gap between consecutive kernels matching the filter."""
import sqlite3
import statistics
import sys

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(end - start) / 1000.0, sum(end - start) / 1e6 from kernels "
                 "group by name order by sum(end - start) desc").fetchall()
print(f"{'kernel':60s} {'calls':>8s} {'avg_us':>10s} {'total_ms':>10s}")
for name, n, avg, tot in rows[:15]:
    print(f"{name[:60]:60s} {n:8d} {avg:10.2f} {tot:10.3f}")
if flt:
    ks = [k for k in c.execute("select name, start, end from kernels order by start") if flt in k[0]]
    gaps = [(ks[i + 1][1] - ks[i][2]) / 1000.0 for i in range(len(ks) - 1)]
    if gaps:
        print(f"{len(ks)} '{flt}' kernels: median gap {statistics.median(gaps):.2f} us, "
              f"mean gap {statistics.mean(gaps):.2f} us, span {(ks[-1][2] - ks[0][1]) / 1e6:.3f} ms")
