"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, one counter per pass).

    python tools/traffic.py --fetch DIR --write DIR --out profiles/r01_traffic.json \
        --dtype bf16 --height 1080 --width 1920 --batch 1

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE is reported in KB and on gfx950 counts exactly half the
bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE (KB) is exact for 16-B-per-lane
stores.  bytes_per_launch = mean over launches of (2*FETCH_SIZE + WRITE_SIZE) * 1024.
"""

import argparse
import csv
import glob
import json
import os


def read(d, counter):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                name = r["Kernel_Name"]
                name = name[5:] if name.startswith("void ") else name
                name = name.split("(")[0]
                out.setdefault(name, []).append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--match", default="vm::", help="only kernels whose name contains this")
    ap.add_argument("--forwards", type=int, default=3, help="forwards in the profiled run (warmup + steps)")
    ap.add_argument("--setup", default="pack_weights,fold_up2x", help="one-time kernels left out of the per-frame sum")
    a = ap.parse_args()
    fe, wr = read(a.fetch, "FETCH_SIZE"), read(a.write, "WRITE_SIZE")
    kernels = {}
    per_forward = 0.0
    setup = [k for k in a.setup.split(",") if k]
    for name in sorted(set(fe) & set(wr)):
        if a.match not in name:
            continue
        f, w = fe[name], wr[name]
        fb = 2 * 1024 * sum(f) / len(f)
        wb = 1024 * sum(w) / len(w)
        kernels[name] = {"launches": len(f), "fetch_bytes_per_launch": int(fb), "write_bytes_per_launch": int(wb),
                         "bytes_per_launch": int(fb + wb)}
        if not any(k in name for k in setup):
            per_forward += (2 * 1024 * sum(f) + 1024 * sum(w)) / a.forwards
    rec = {"config": {"dtype": a.dtype, "height": a.height, "width": a.width, "batch": a.batch},
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), "
                     "FETCH_SIZE x2 (gfx950), KB -> bytes", "forwards": a.forwards,
           "bytes_per_forward": int(per_forward), "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    for k, v in kernels.items():
        print("%-70s %4d launches  %.1f MB/launch" % (k, v["launches"], v["bytes_per_launch"] / 1e6))


if __name__ == "__main__":
    main()
