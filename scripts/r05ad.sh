#!/bin/bash
# GPU-box: bf16 data gradients in the UNetImage bf16 step — kernel tests, image-train tests, A/B step time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_image_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ad_tests.log 2>&1 || { tail -30 gpurun_out/r05ad_tests.log; exit 1; }
tail -3 gpurun_out/r05ad_tests.log
for v in True; do
  timeout -k 10 240 python -u -c "
import sys, runpy
sys.path.insert(0, 'video-matting_amd')
import vmatting.image_train as it
it.ImageTrainer.bf16_dgrad = $v
sys.argv = ['bench.py', '--only', 'train_image', '--steps', '40', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r05ad_b_$v.log 2>&1 || { tail -20 gpurun_out/r05ad_b_$v.log; exit 1; }
  echo "bf16_dgrad=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ad_b_$v.log | head -1)"
done
