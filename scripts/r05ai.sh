#!/bin/bash
# GPU-box: filter gradients on side streams (UNetImage and config-5 trainers) — tests, then same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_image_train.py tests/test_gpu_train.py -k "image or graph or step or capture or chain" -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ai_t.log 2>&1 || { tail -30 gpurun_out/r05ai_t.log; exit 1; }
tail -1 gpurun_out/r05ai_t.log
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 240 python -u bench.py --only train --steps 40 --warmup 5 --train-wgrad-stream $v > gpurun_out/r05ai_b.log 2>&1 || { tail -20 gpurun_out/r05ai_b.log; exit 1; }
  echo "train wgrad_stream=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ai_b.log | head -1) $(grep -o '"backward": [0-9.]*' gpurun_out/r05ai_b.log | head -1)"
done
done
timeout -k 10 240 python -u bench.py --only train_image --steps 40 --warmup 5 > gpurun_out/r05ai_b.log 2>&1 || { tail -20 gpurun_out/r05ai_b.log; exit 1; }
echo "train_image default: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ai_b.log | head -1)"
timeout -k 10 240 python -u bench.py --only train_chain --steps 20 --warmup 3 > gpurun_out/r05ai_c.log 2>&1 || { tail -20 gpurun_out/r05ai_c.log; exit 1; }
echo "train_chain: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ai_c.log | head -1)"
