"""Per-launch listing of one step from a rocprofv3 --kernel-trace CSV: the kernels between the last two launches
whose name contains MARK (default: the Adam update), with queue, start offset, duration and grid."""
import csv
import sys

path = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "adam"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = ends[-2] + 1, ends[-1] + 1
t0 = int(rows[a]["Start_Timestamp"])
busy = {}
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r["Queue_Id"]
    nm = r["Kernel_Name"].replace("void ", "").replace("vm::", "")[:78]
    grid = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * int(r["Grid_Size_Y"])
    print(f"q{q:>2} {s / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {grid:6d}  {nm}")
    busy[nm] = busy.get(nm, 0) + (e - s)
span = int(rows[b - 1]["End_Timestamp"]) - t0
print(f"step span {span / 1e3:.1f} us, {b - a} launches")
for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v / 1e3:8.1f}  {k}")
