"""Print every counter of the last self-attention dispatch in a rocprofv3 PMC output dir (tools/runs/attn_pmc2.sh)."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(lambda: defaultdict(float))
    span = {}
    for r in csv.DictReader(open(f)):
        if "attn_fwd" not in r["Kernel_Name"] or "<0" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        span[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if per:
        last = max(per)
        print(os.path.basename(f), f"dur_ms={span[last] / 1e6:.2f}",
              " ".join(f"{k}={v:.4g}" for k, v in sorted(per[last].items())))
