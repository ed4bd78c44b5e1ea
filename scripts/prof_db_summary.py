"""Per-kernel summary (calls, mean/median us, total ms) of a rocprofv3 kernel-trace database
(the default rocpd SQLite output) grouped by kernel name and grid: python prof_db_summary.py DB [N]."""
import sqlite3
import statistics
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
groups = {}
for name, gx, gy, dur in c.execute("select name, grid_x, grid_y, duration from kernels"):
    groups.setdefault((name, gx, gy), []).append(dur / 1000.0)
rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:n]
print(f"{'calls':>6} {'mean_us':>9} {'med_us':>9} {'total_ms':>9}  grid  kernel")
for (name, gx, gy), d in rows:
    print(f"{len(d):6d} {statistics.mean(d):9.2f} {statistics.median(d):9.2f} {sum(d) / 1e3:9.3f}  {gx}x{gy}  {name[:110]}")
