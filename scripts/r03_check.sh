#!/bin/bash
# round-3 GPU check: all GPU tests, refine kernel variants, folded-upconv A/B, the graphed training step,
# per-record profiles.  STEPS selects: pytest smx ab train prof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-pytest smx ab train prof}"
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has pytest; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf \
      > gpurun_out/pt_r03.log 2>&1; rc=$?; tail -12 gpurun_out/pt_r03.log
  [ $rc -le 1 ] || exit $rc
fi
if has smx; then
  timeout -k 10 120 python tools/softmaxbench.py > gpurun_out/smx.log 2>&1; rc=$?; tail -10 gpurun_out/smx.log
  [ $rc -eq 0 ] || exit $rc
fi
if has ab; then
  timeout -k 10 300 python tools/ab_unet.py ${AB:-default noskip fold_up2 fold_up2_noskip} > gpurun_out/ab.log 2>&1
  rc=$?; cat gpurun_out/ab.log | grep ms/frame
  [ $rc -eq 0 ] || exit $rc
fi
if has train; then
  timeout -k 10 300 python bench.py --only train --steps 20 --warmup 3 > gpurun_out/train_eager.log 2>&1; rc=$?
  tail -1 gpurun_out/train_eager.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --only train --steps 20 --warmup 3 --train-graph > gpurun_out/train_graph.log 2>&1
  rc=$?; tail -1 gpurun_out/train_graph.log
  [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  SKIP="${PROF_SKIP:-fwd mfma traffic bench}" bash tools/prof_bench.sh "${TAG:-r03a}" || exit $?
fi
