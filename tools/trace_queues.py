"""Kernel-trace summary per (stream, hardware queue): which queue each stream's kernels ran on, over what span
(study tool, CPU; reads a rocprofv3 --kernel-trace CSV).

    python tools/trace_queues.py <run_kernel_trace.csv>
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = collections.OrderedDict()
    for r in rows:
        d = by.setdefault((r["Stream_Id"], r["Queue_Id"]), {"n": 0, "t0": int(r["Start_Timestamp"]), "t1": 0,
                                                            "names": collections.Counter()})
        d["n"] += 1
        d["t1"] = max(d["t1"], int(r["End_Timestamp"]))
        d["names"][r["Kernel_Name"][:40]] += 1
    t00 = min(int(r["Start_Timestamp"]) for r in rows)
    for (s, q), d in sorted(by.items(), key=lambda kv: kv[1]["t0"]):
        print("stream %3s queue %3s  kernels %6d  span %8.3f .. %8.3f s  %s" % (
            s, q, d["n"], (d["t0"] - t00) / 1e9, (d["t1"] - t00) / 1e9, d["names"].most_common(1)[0][0]))


if __name__ == "__main__":
    main()
