"""rocprofv3 sqlite output (`-d DIR -o NAME`, the default format) -> the kernel_stats.csv form of `--stats`
(Name, Calls, TotalDurationNs, AverageNs, Percentage), from the database's own top_kernels view (durations in us there).
  python tools/prof_db_stats.py <run_results.db> [out.csv]"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels "
                   "order by total_duration desc").fetchall()
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
for name, calls, tot, avg, pct in rows:
    w.writerow([name, calls, round(tot * 1e3), round(avg * 1e3, 1), round(pct, 4)])
