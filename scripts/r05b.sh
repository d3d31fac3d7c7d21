#!/bin/bash
# round-5: wide wgrad f32, ImageTrainer fp32, SyncBN relaxed bound; then the nested-fork capture probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 8 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf -s"
guard 600 r5b_tests.log $PT tests/test_gpu_train.py tests/test_gpu_image_train.py tests/test_gpu_small_train.py -m gpu -k "wgrad_wide or image or syncbn_unequal"
guard 600 r5b_probe.log python -u tools/capture_probe.py --cases ${PROBE_CASES:-nested_default_single,nested_default,prio_nested_single}
