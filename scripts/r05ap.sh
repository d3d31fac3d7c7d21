#!/bin/bash
# GPU-box: output-channel wave split for the cin <= 16 weight gradient — tests, then same-box A/B of the image step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -k "wgrad_wide" -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ap_t.log 2>&1 || { tail -30 gpurun_out/r05ap_t.log; exit 1; }
tail -1 gpurun_out/r05ap_t.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_image_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ap_t2.log 2>&1 || { tail -30 gpurun_out/r05ap_t2.log; exit 1; }
tail -1 gpurun_out/r05ap_t2.log
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 240 python -u bench.py --only train_image --steps 40 --warmup 5 --option wgrad_wide_cs=$v > gpurun_out/r05ap_b.log 2>&1 || { tail -20 gpurun_out/r05ap_b.log; exit 1; }
  echo "cs=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ap_b.log | head -1) $(grep -o '"backward": [0-9.]*' gpurun_out/r05ap_b.log | head -1)"
done
done
