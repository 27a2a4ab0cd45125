"""GPU busy time vs wall span of a rocprofv3 kernel trace (csv): how much of the DiT evaluation loop the
device spends idle between kernels (launch / host gaps). Prints the busy fraction over the longest
self-attention-dense window and the largest gaps.

usage: python tools/trace_gaps.py <..._kernel_trace.csv>
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    attn = [k for k in ks if "attn_fwd_d128<0" in k[2]]
    if not attn:
        print("no self-attention launches")
        return
    # the timed region: from the first to the last self-attention launch (evaluations only)
    t0, t1 = attn[0][0], attn[-1][1]
    win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
    busy, last_end, gaps = 0, t0, []
    for s, e, n in win:
        if s > last_end:
            gaps.append((s - last_end, n))
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    span = t1 - t0
    print(f"window {span / 1e6:.1f} ms, kernels {len(win)}, busy {busy / 1e6:.1f} ms = {100 * busy / span:.2f} %")
    gaps.sort(reverse=True)
    tot_gap = sum(g for g, _ in gaps)
    print(f"gaps: {len(gaps)} totalling {tot_gap / 1e6:.2f} ms; largest:")
    for g, n in gaps[:10]:
        print(f"  {g / 1e3:9.1f} us before {n[:100]}")
    by = {}
    for s, e, n in win:
        key = n.split("(")[0][:80]
        by[key] = by.get(key, 0) + (e - s)
    print("kernel time in the window:")
    for n, t in sorted(by.items(), key=lambda x: -x[1])[:14]:
        print(f"  {100 * t / busy:6.2f} %  {t / 1e6:9.1f} ms  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
