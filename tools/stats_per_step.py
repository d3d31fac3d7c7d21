"""Summarise a rocprofv3 --stats kernel_stats.csv per step:  python tools/stats_per_step.py CSV STEPS [TOP]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total %.3f ms/step" % (tot / 1e6 / steps))
for r in rows[:top]:
    print("%-100s %6s calls %8.3f ms/step %5.1f%%" % (r["Name"][:100], r["Calls"], float(r["TotalDurationNs"]) / 1e6 / steps,
                                                     100 * float(r["TotalDurationNs"]) / tot))
