#!/bin/bash
# GPU-box: padded biases refreshed by one multi-tensor copy — training tests, step timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_small_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05at_t.log 2>&1 || { tail -30 gpurun_out/r05at_t.log; exit 1; }
tail -1 gpurun_out/r05at_t.log
for rec in train train_small train; do
  timeout -k 10 240 python -u bench.py --only $rec --steps 40 --warmup 5 > gpurun_out/r05at_b.log 2>&1 || { tail -20 gpurun_out/r05at_b.log; exit 1; }
  echo "$rec: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05at_b.log | head -1) $(grep -o '"allreduce_adam_repack": [0-9.]*' gpurun_out/r05at_b.log | head -1)"
done
