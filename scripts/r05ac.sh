#!/bin/bash
# GPU-box: loader descriptors by value — parity, then the loader and chained records
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_loader.py tests/test_gpu_procedures.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ac_tests.log 2>&1 || { tail -40 gpurun_out/r05ac_tests.log; exit 1; }
tail -2 gpurun_out/r05ac_tests.log
timeout -k 10 200 python bench.py --only loader --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r05ac_l.log 2>&1 || { tail -5 gpurun_out/r05ac_l.log; exit 1; }
tail -1 gpurun_out/r05ac_l.log | cut -c1-400
timeout -k 10 300 python bench.py --only train_chain --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05ac_c.log 2>&1 || { tail -5 gpurun_out/r05ac_c.log; exit 1; }
tail -1 gpurun_out/r05ac_c.log | cut -c1-500
