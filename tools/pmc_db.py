"""Per-dispatch PMC counters from a rocprofv3 sqlite output (pmc_results.db, the default output format):
  python tools/pmc_db.py <db> [kernel-name substring]
One line per dispatch of the matching kernels: duration and the summed counter values."""
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else ""
cols = [r[1] for r in con.execute("pragma table_info(counters_collection)")]
rows = con.execute("select * from counters_collection").fetchall()
ix = {c: i for i, c in enumerate(cols)}
name_col = next(c for c in ("kernel_name", "name") if c in ix)
per = defaultdict(lambda: defaultdict(float))
meta = {}
for r in rows:
    if pat not in r[ix[name_col]]:
        continue
    d = r[ix["dispatch_id"]]
    per[d][r[ix["counter_name"]]] += float(r[ix["value"]])
    meta[d] = (r[ix[name_col]], (r[ix["end"]] - r[ix["start"]]) / 1e6 if "end" in ix else float("nan"))
for d in sorted(per):
    n, ms = meta[d]
    print(d, n[:60], f"dur_ms={ms:.3f}", " ".join(f"{k}={v:.5g}" for k, v in sorted(per[d].items())))
