#!/bin/bash
# GPU-box: flipped (data-gradient) packs 8 channels per lane — pack parity, image-train tests, same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -k "pack" tests/test_gpu_image_train.py tests/test_gpu_small_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ar_t.log 2>&1 || { tail -30 gpurun_out/r05ar_t.log; exit 1; }
tail -1 gpurun_out/r05ar_t.log
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 240 python -u bench.py --only train_image --steps 40 --warmup 5 --option pack_tiled=$v > gpurun_out/r05ar_b.log 2>&1 || { tail -20 gpurun_out/r05ar_b.log; exit 1; }
  echo "vec packs=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ar_b.log | head -1) $(grep -o '"allreduce_adam_repack": [0-9.]*' gpurun_out/r05ar_b.log | head -1)"
done
done
