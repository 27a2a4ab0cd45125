"""Kernel statistics CSV (the columns of rocprofv3's kernel_stats.csv) from a rocprofv3 results.db.

rocprofv3 writes a SQLite database unless `--output-format csv` is given; this turns the database's
`kernels` view into the same summary so profiles/ holds one format.
usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rN/kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path: str) -> None:
    con = sqlite3.connect(path)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc"
    ).fetchall()
    total = sum(r[2] for r in rows)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, int(tot), f"{avg:.1f}", f"{100.0 * tot / total:.4f}", int(mn), int(mx)])


if __name__ == "__main__":
    main(sys.argv[1])
