#!/bin/bash
# GPU-box: UNetImage filter gradients on a side stream — tests, then same-box A/B (graph / eager x 0 / 1 side stream)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_image_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ah_t.log 2>&1 || { tail -30 gpurun_out/r05ah_t.log; exit 1; }
tail -1 gpurun_out/r05ah_t.log
for rep in 1 2; do
for cfg in "" "--image-streams 0" "--image-eager" "--image-eager --image-streams 0"; do
  timeout -k 10 240 python -u bench.py --only train_image --steps 40 --warmup 5 $cfg > gpurun_out/r05ah_b.log 2>&1 || { tail -20 gpurun_out/r05ah_b.log; exit 1; }
  echo "[$cfg]: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ah_b.log | head -1) $(grep -o '"backward": [0-9.]*' gpurun_out/r05ah_b.log | head -1)"
done
done
