#!/bin/bash
# GPU-box: exact-2x resize adjoint + work-sized relu-backward grid — tests, then same-box A/B of the image step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -k "resize_backward or relu_backward" -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05af_t1.log 2>&1 || { tail -30 gpurun_out/r05af_t1.log; exit 1; }
tail -1 gpurun_out/r05af_t1.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_image_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05af_t2.log 2>&1 || { tail -30 gpurun_out/r05af_t2.log; exit 1; }
tail -1 gpurun_out/r05af_t2.log
for cfg in "1 8" "0 0" "1 8" "0 0"; do
  set -- $cfg
  timeout -k 10 240 python -u -c "
import sys, runpy
sys.path.insert(0, 'video-matting_amd')
from vmatting import _lib
_lib.set_option('resize_bwd_2x', $1)
_lib.set_option('relu_bias_iters', $2)
sys.argv = ['bench.py', '--only', 'train_image', '--steps', '40', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r05af_b.log 2>&1 || { tail -20 gpurun_out/r05af_b.log; exit 1; }
  echo "resize2x=$1 iters=$2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05af_b.log | head -1)"
done
