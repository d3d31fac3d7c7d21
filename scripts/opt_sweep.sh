#!/bin/bash
# GPU box: the 1080p forward (per-layer events) under each value of one vm_set_option key, interleaved rounds:
#   bash scripts/opt_sweep.sh <key> <v1> <v2> ...      (results: gpurun_out/sweep_<key>_<v>_<round>.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
KEY=$1; shift
FWD="--no-cpu-baseline --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0 --steps ${SW_STEPS:-200} --warmup 10"
for i in ${SW_ROUNDS:-1 2}; do
  for v in "$@"; do
    L=gpurun_out/sweep_${KEY}_${v}_$i.log
    timeout -k 10 240 python bench.py $FWD --layers --option $KEY=$v > $L 2>&1 || { echo "sweep $KEY=$v failed"; tail -5 $L; exit 1; }
    python3 -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print('$KEY=$v', $i, d['value'])"
  done
done
