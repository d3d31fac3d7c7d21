"""Average per-dispatch PMC values of the kernels matching a name filter (tools/pmc.sh output)."""
import csv
import glob
import os
import sys


def main():
    out, filt = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "conv3x3"
    vals = {}
    for path in sorted(glob.glob(os.path.join(out, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if filt not in k:
                continue
            kname = k.split("(")[0].replace("void ", "")
            d = vals.setdefault(kname, {})
            d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for kname, d in vals.items():
        print(kname)
        for c, v in sorted(d.items()):
            print("  %-34s %16.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
