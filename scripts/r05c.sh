#!/bin/bash
# round-5: capture guard, image fp32 tolerance, split6 kernel + bf16x6 forward; x6 timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 12 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf -s"
guard 600 r5c_tests.log $PT tests/test_gpu_train.py tests/test_gpu_image_train.py tests/test_gpu_split6.py -m gpu -k "nested_fork"
guard 300 r5c_x6bench.log python -u tools/x6bench.py 10
