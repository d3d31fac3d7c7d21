#!/bin/bash
# conv3x3_rows bring-up on the GPU box: parity tests, then an interleaved same-process A/B against the patch kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "rows_kernel" --timeout 120 --timeout-method thread \
  > gpurun_out/rows_pytest.log 2>&1
rc=$?; tail -n 15 gpurun_out/rows_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/convbench.py --unet-layers --iters 20 --rounds 3 --ab rows_kernel=0,16 ${AB_ARGS} \
  > gpurun_out/rows_ab.log 2>&1
rc=$?; grep "^AB" gpurun_out/rows_ab.log; exit $rc
