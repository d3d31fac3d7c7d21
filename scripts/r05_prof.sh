#!/bin/bash
# GPU-box: the training records' final r05 profile set — bench JSON + rocprofv3 --kernel-trace --stats per record
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof5
for rec in train train_image train_chain; do
  steps=40; [ $rec = train_chain ] && steps=20
  timeout -k 10 300 python -u bench.py --only $rec --steps $steps --warmup 5 > gpurun_out/prof5/$rec.log 2>&1 || { tail -20 gpurun_out/prof5/$rec.log; exit 1; }
  tail -n 1 gpurun_out/prof5/$rec.log > gpurun_out/prof5/r05_$rec.json
  echo "$rec: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof5/r05_$rec.json | head -1)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5/rp_$rec -o run -- python bench.py --only $rec --steps 10 --warmup 3 > gpurun_out/prof5/rp_$rec.log 2>&1 || { tail -20 gpurun_out/prof5/rp_$rec.log; exit 1; }
  f=$(find gpurun_out/prof5/rp_$rec -name '*kernel_stats.csv' | head -n 1); [ -n "$f" ] && cp "$f" gpurun_out/prof5/r05_${rec}_kernel_stats.csv
done
ls gpurun_out/prof5
