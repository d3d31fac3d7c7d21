#!/bin/bash
# GPU-box: UNetImage step — conv1_1's filter gradient on the caller's stream (A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_image_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ax_t.log 2>&1 || { tail -30 gpurun_out/r05ax_t.log; exit 1; }
tail -1 gpurun_out/r05ax_t.log
for rep in 1 2 3; do
for v in '("conv1_1",)' '()' '("conv1_1", "conv1_2")'; do
  timeout -k 10 240 python -u -c "
import sys, runpy
sys.path.insert(0, 'video-matting_amd')
import vmatting.image_train as it
it.ImageTrainer.main_wgrad = $v
sys.argv = ['bench.py', '--only', 'train_image', '--steps', '40', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r05ax_b.log 2>&1 || { tail -20 gpurun_out/r05ax_b.log; exit 1; }
  echo "main_wgrad=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ax_b.log | head -1)"
done
done
