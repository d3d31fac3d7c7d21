#!/bin/bash
# GPU-box: per-layer patch-kernel config sweep + timing ablations (tools/convbench.py), one process per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-0 1 2 3 4 5 6 7 8 9 10 11 12}; do
  timeout -k 10 120 python tools/convbench.py --unet-layers --kernel 3 --patch-cfg $c --iters 20 > gpurun_out/sweep_cfg$c.log 2>&1 || { echo "cfg $c failed"; tail -5 gpurun_out/sweep_cfg$c.log; exit 1; }
done
for ab in ${ABLS:-}; do
  timeout -k 10 120 python tools/convbench.py --unet-layers --kernel 3 --ablate $ab --iters 20 > gpurun_out/sweep_abl$ab.log 2>&1 || { echo "abl $ab failed"; exit 1; }
done
python3 - <<'PY'
import glob, re, os
rows = {}; cols = []
for f in sorted(glob.glob("gpurun_out/sweep_*.log")):
    tag = os.path.basename(f)[6:-4]; cols.append(tag)
    for line in open(f):
        m = re.match(r"^(\S+)\s+\S+\s+\S+\s+([\d.]+) ms", line)
        if m: rows.setdefault(m.group(1), {})[tag] = float(m.group(2))
print("%-10s" % "layer" + "".join("%9s" % c for c in cols))
for k, v in rows.items(): print("%-10s" % k + "".join("%9.4f" % v.get(c, 0) for c in cols))
PY
