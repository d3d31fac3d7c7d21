#!/bin/bash
# GPU-box: config-5 forward with the select chains queued level by level between the decoder's launches — tests, then same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -k "graph or step or chain or capture" -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05au_t.log 2>&1 || { tail -30 gpurun_out/r05au_t.log; exit 1; }
tail -1 gpurun_out/r05au_t.log
for rep in 1 2; do
for v in True False; do
  timeout -k 10 240 python -u -c "
import sys, runpy
sys.path.insert(0, 'video-matting_amd')
import vmatting.train as tr
tr.VideoTrainer.interleave_issue = $v
sys.argv = ['bench.py', '--only', 'train', '--steps', '40', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r05au_b.log 2>&1 || { tail -20 gpurun_out/r05au_b.log; exit 1; }
  echo "interleave=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05au_b.log | head -1) $(grep -o '"forward_loss": [0-9.]*' gpurun_out/r05au_b.log | head -1)"
done
done
