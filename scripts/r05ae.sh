#!/bin/bash
# GPU-box: bf16 resize-adjoint outputs in the UNetImage bf16 step — tests, step time, kernel trace of the step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05t
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -k "resize_backward" -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ae_t1.log 2>&1 || { tail -30 gpurun_out/r05ae_t1.log; exit 1; }
tail -1 gpurun_out/r05ae_t1.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_image_train.py -q --timeout 200 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05ae_t2.log 2>&1 || { tail -30 gpurun_out/r05ae_t2.log; exit 1; }
tail -1 gpurun_out/r05ae_t2.log
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --only train_image --steps 40 --warmup 5 > gpurun_out/r05ae_b$i.log 2>&1 || { tail -20 gpurun_out/r05ae_b$i.log; exit 1; }
  echo "run $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05ae_b$i.log | head -1)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05t -o trace -- python bench.py --only train_image --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r05t/bench.log 2>&1 || { tail -20 gpurun_out/r05t/bench.log; exit 1; }
ls gpurun_out/r05t
