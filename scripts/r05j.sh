#!/bin/bash
# round-5: procedures tests, host profiles of the chain and the eager step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" >> "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 4 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf"
guard 600 r5j_tests.log $PT tests/test_gpu_procedures.py tests/test_gpu_train.py -m gpu -k "procedure or validation or chain_overlap"
guard 300 r5j_hp_serial.log python -u tools/chain_host_profile.py --serial
guard 300 r5j_hp_overlap.log python -u tools/chain_host_profile.py
guard 300 r5j_hp_step.log python -u tools/host_profile.py
