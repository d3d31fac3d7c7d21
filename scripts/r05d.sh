#!/bin/bash
# round-5: augment fusion + batched pipeline, loader pinned desc, chain bench, train_image record
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
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf"
guard 600 r5d_tests.log $PT tests/test_gpu_augment.py tests/test_gpu_loader.py tests/test_gpu_train.py tests/test_gpu_split6.py -m gpu -k "augment or warp or loader or compose or config5 or tps or illumination or statistics or split6 or bf16x6"
guard 300 r5d_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3
guard 300 r5d_timage.log python -u bench.py --only train_image --steps 10 --warmup 3
guard 300 r5d_aug.log python -u -c "
import sys; sys.argv=['bench.py']; import bench, torch, json
dev=torch.device('cuda',0); torch.cuda.set_device(dev)
print(json.dumps(bench.augment_bench(dev, 20, 16, cpu=False)))
"
guard 300 r5d_tlayers.log python -u tools/train_layers.py --steps 3
guard 300 r5d_x6bench.log python -u tools/x6bench.py 10
