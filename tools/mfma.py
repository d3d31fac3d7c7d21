"""Per-kernel MFMA-utilisation counters from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace ... -- python3 bench.py ...
    python tools/mfma.py --pmc DIR --out profiles/r02_mfma.json --dtype bf16 --height 1080 --width 1920 --batch 1

Per launch (averaged over a kernel's launches): SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy SIMD-cycles, all SIMDs),
SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (GPU-busy cycles summed over the 8 XCDs).  bench.py turns them into
mfma_util = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) for the dominant conv kernel.
"""

import argparse
import csv
import glob
import json
import os

COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--match", default="vm::")
    a = ap.parse_args()
    vals = {}
    for path in glob.glob(os.path.join(a.pmc, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                c = r["Counter_Name"]
                if c not in COUNTERS:
                    continue
                name = r["Kernel_Name"]
                name = (name[5:] if name.startswith("void ") else name).split("(")[0]
                if a.match not in name:
                    continue
                d = vals.setdefault(name, {}).setdefault(c, {})
                # one row per (dispatch, counter); rows of one dispatch that repeat per dimension are summed
                key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(d))
                d[key] = d.get(key, 0.0) + float(r["Counter_Value"])
    kernels = {}
    for name, d in vals.items():
        kernels[name] = {c: sum(v.values()) / len(v) for c, v in d.items()}
        kernels[name]["launches"] = max(len(v) for v in d.values())
    rec = {"config": {"dtype": a.dtype, "height": a.height, "width": a.width, "batch": a.batch},
           "method": "rocprofv3 --pmc %s --kernel-trace (one pass), per-launch averages" % " ".join(COUNTERS),
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    for k, v in sorted(kernels.items()):
        if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            print("%-70s mfma busy %.3f" % (k, v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8)))


if __name__ == "__main__":
    main()
