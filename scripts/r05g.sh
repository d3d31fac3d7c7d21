#!/bin/bash
# wide wgrad A/B + fused relu/pool backward tests + UNetImage step parity and timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" >> "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 8 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
for v in base cur lb2 base cur lb2; do
  case $v in base) L=ab/lib_ww_base.so;; cur) L=video-matting_amd/vmatting/libvmatting.so;; lb2) L=ab/lib_ww_lb2.so;; esac
  echo "== $v" >> gpurun_out/r5g_ww.log
  VM_LIB_PATH=$L guard 120 r5g_ww.log python -u tools/wgradwide_bench.py 10
done
grep -E "==|total" gpurun_out/r5g_ww.log
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf -s"
guard 600 r5g_tests.log $PT tests/test_gpu_train.py tests/test_gpu_image_train.py tests/test_gpu_split6.py tests/test_gpu_augment.py -m gpu -k "relu_backward_bias or wgrad_wide or image or bf16x6_graph or bgra or augment_many or config5"
guard 300 r5g_timage.log python -u bench.py --only train_image --steps 10 --warmup 3
guard 300 r5g_x6.log python -u tools/x6bench.py 10
guard 300 r5g_chain.log python -u bench.py --only train_chain --steps 10 --warmup 3
guard 300 r5g_chain_g.log python -u bench.py --only train_chain --steps 10 --warmup 3 --train-graph
