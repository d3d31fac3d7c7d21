#!/bin/bash
# round-5: fused object-motion warp + BGRA, batched bgra: augment tests, augment + chain bench, augment kernel profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" >> "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 3 "gpurun_out/$log" | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf"
guard 900 r5o_tests.log $PT tests/test_gpu_augment.py tests/test_gpu_train.py -m gpu -k "augment or tps or warp or config5"
grep -E "passed|failed" gpurun_out/r5o_tests.log | tail -3
guard 300 r5o_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3
grep -h '"only"' gpurun_out/r5o_chain.log | cut -c1-420
mkdir -p gpurun_out/r5o_prof
guard 300 r5o_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o_prof -o run -- python -u bench.py --only train_chain --steps 10 --warmup 3 --chain-serial
