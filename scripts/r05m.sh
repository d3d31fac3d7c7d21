#!/bin/bash
# round-5: batched augment (bit-identity tests, chain bench)
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
guard 900 r5m_tests.log $PT tests/test_gpu_augment.py tests/test_gpu_train.py tests/test_capi.py -m gpu -k "augment or tps or warp or statistics or config5 or chain_overlap or bgra or capi"
grep -E "passed|failed" gpurun_out/r5m_tests.log | tail -3
guard 300 r5m_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3
guard 300 r5m_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3 --chain-serial
guard 300 r5m_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3 --train-graph
grep -h '"only"' gpurun_out/r5m_chain.log | cut -c1-520
guard 300 r5m_aug.log python -u -c "
import sys; sys.argv=['bench.py']; import bench, torch, json
dev=torch.device('cuda',0); torch.cuda.set_device(dev)
print(json.dumps(bench.augment_bench(dev, 20, 16, cpu=False)))
"
guard 300 r5m_hp.log python -u tools/chain_host_profile.py --serial
