"""Idle gaps of the main stream in the last training step of a rocprofv3 kernel trace:
    python tools/stream_gaps.py <run_kernel_trace.csv> [--marker adam] [--top 12]

The step is the span between the last two launches whose name contains ``--marker`` (the optimizer kernel ends every
step).  Prints the step's span, each stream's busy time inside it, and the main stream's largest idle gaps with the
kernels on either side and what the other streams were running meanwhile.
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adam")
    ap.add_argument("--top", type=int, default=12)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), r["Kernel_Name"]))
    rows.sort()
    ends = [e for s, e, st, k in rows if args.marker in k.lower()]
    if len(ends) < 2:
        raise SystemExit("fewer than two '%s' launches in the trace" % args.marker)
    t0, t1 = ends[-2], ends[-1]
    step = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    by = defaultdict(list)
    for r in step:
        by[r[2]].append(r)
    main_id = max(by, key=lambda k: len(by[k]))
    print("step %.3f ms, %d launches" % ((t1 - t0) / 1e6, len(step)))
    for sid, rs in sorted(by.items()):
        print("  stream %d%s: %d launches, busy %.3f ms" % (sid, " (main)" if sid == main_id else "", len(rs),
                                                           sum(e - s for s, e, _, _ in rs) / 1e6))
    m = by[main_id]
    gaps = []
    for a, b in zip(m, m[1:]):
        if b[0] > a[1]:
            gaps.append((b[0] - a[1], a, b))
    print("main idle %.3f ms in %d gaps" % (sum(g[0] for g in gaps) / 1e6, len(gaps)))
    for g, a, b in sorted(gaps, reverse=True)[:args.top]:
        side = sorted({k.split("(")[0][:40] for s, e, sid, k in step if sid != main_id and s < b[0] and e > a[1]})
        print("%7.1f us at %.3f ms  %s -> %s   | side: %s" % (g / 1e3, (a[1] - t0) / 1e6, a[3].split("(")[0][:48],
                                                             b[3].split("(")[0][:48], ", ".join(side)[:160]))


if __name__ == "__main__":
    main()
