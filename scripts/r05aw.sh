#!/bin/bash
# GPU-box: config-5 step — number of select-chain side streams (with the decoder filter-gradient stream), A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for k in 3 2 4; do
  timeout -k 10 240 python -u bench.py --only train --steps 40 --warmup 5 --train-streams $k > gpurun_out/r05aw_b.log 2>&1 || { tail -20 gpurun_out/r05aw_b.log; exit 1; }
  echo "side streams=$k: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05aw_b.log | head -1) $(grep -o '"backward": [0-9.]*' gpurun_out/r05aw_b.log | head -1)"
done
done
