#!/bin/bash
# round-3 GPU check: refine kernel variants, the new GPU tests, the graphed training step, per-record profiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/softmaxbench.py > gpurun_out/smx.log 2>&1; rc=$?; tail -11 gpurun_out/smx.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_temporal.py tests/test_gpu_train.py -q --timeout 120 \
    --timeout-method thread -rf > gpurun_out/pt_r03.log 2>&1; rc=$?; tail -8 gpurun_out/pt_r03.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --only train --steps 20 --warmup 3 > gpurun_out/train_graph.log 2>&1; rc=$?
tail -1 gpurun_out/train_graph.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --only train --steps 20 --warmup 3 --no-graph > gpurun_out/train_eager.log 2>&1
rc=$?; tail -1 gpurun_out/train_eager.log
[ $rc -eq 0 ] || exit $rc
SKIP="fwd mfma traffic bench" bash tools/prof_bench.sh r03a
