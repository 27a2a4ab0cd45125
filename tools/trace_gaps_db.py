"""GPU busy time vs wall span of a rocprofv3 kernel trace in its default sqlite form (`-d DIR -o NAME`: the `kernels`
view): how much of a window the device spends idle between kernels (launch / host gaps). The window runs from the
first to the last launch whose name contains --anchor (default: the bf16 self-attention, so the evaluations only).

usage: python tools/trace_gaps_db.py <run_results.db> [--anchor 'attn_fwd_m16<0'] [--json out.json]
"""
import argparse
import json
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="attn_fwd_m16<0")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    ks = sorted(con.execute("select start, end, name from kernels").fetchall())
    anchor = [k for k in ks if a.anchor in k[2]]
    if not anchor:
        raise SystemExit(f"no launch named like {a.anchor!r}")
    t0, t1 = anchor[0][0], anchor[-1][1]
    win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
    busy, last_end, gaps = 0, t0, []
    for s, e, n in win:
        if s > last_end:
            gaps.append((s - last_end, n))
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    span = t1 - t0
    gaps.sort(reverse=True)
    by = {}
    for s, e, n in win:
        key = n.split("(")[0][:90]
        by[key] = by.get(key, 0) + (e - s)
    rec = {"window_ms": span / 1e6, "kernels": len(win), "busy_ms": busy / 1e6, "busy_frac": busy / span,
           "n_gaps": len(gaps), "gap_ms": sum(g for g, _ in gaps) / 1e6,
           "gaps_over_20us_ms": sum(g for g, _ in gaps if g > 20000) / 1e6,
           "largest_gaps_us": [[round(g / 1e3, 1), n[:90]] for g, n in gaps[:8]],
           "kernel_ms": [[round(t / 1e6, 2), n] for n, t in sorted(by.items(), key=lambda x: -x[1])[:16]]}
    print(json.dumps(rec, indent=1))
    if a.json:
        json.dump(rec, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
