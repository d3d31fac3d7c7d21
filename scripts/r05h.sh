#!/bin/bash
# round-5: conv2_1 on rows<16>, overlapped config-5 chain, chain kernel profile
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
guard 600 r5h_tests.log $PT tests/test_gpu_train.py tests/test_gpu_layers_1080p.py -m gpu -k "chain_overlap or timed_kernels or conv2_1"
guard 300 r5h_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3
guard 300 r5h_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3 --train-graph
guard 300 r5h_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3 --chain-serial
grep -h '"only"' gpurun_out/r5h_chain.log | cut -c1-600
guard 300 r5h_tl.log python -u tools/train_layers.py --steps 3 --option rows_min_cin=128
guard 300 r5h_tl.log python -u tools/train_layers.py --steps 3
grep -h " 1 24x160" gpurun_out/r5h_tl.log
OPT=rows_min_cin=64,128 AB_STEPS=100 guard 600 r5h_ab.log bash scripts/opt_ab.sh
grep -h "rows_min_cin=" gpurun_out/r5h_ab.log
mkdir -p gpurun_out/r5h_prof
guard 300 r5h_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r5h_prof -o run -- python -u bench.py --only train_chain --steps 10 --warmup 3 --train-graph
