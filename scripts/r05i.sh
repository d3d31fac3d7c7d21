#!/bin/bash
# round-5: chain overlap parity, training procedures, deform_grid draws, chain bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" >> "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 6 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf"
guard 900 r5i_tests.log $PT tests/test_gpu_train.py tests/test_gpu_procedures.py tests/test_gpu_augment.py -m gpu -k "chain_overlap or procedure or validation or tps or augment or config5"
guard 300 r5i_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3
guard 300 r5i_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3 --train-graph
guard 300 r5i_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3 --chain-serial
grep -h '"only"' gpurun_out/r5i_chain.log | cut -c1-420
for v in 0 2 0 2; do
  guard 300 r5i_wv.log python -u bench.py --only train --steps 20 --warmup 3 --option wgrad_variant=$v
done
grep -h '"only"' gpurun_out/r5i_wv.log | cut -c1-300
