#!/bin/bash
# wide wgrad A/B: base (32x32 wave split) vs ci16 x co64 (1 block/CU, AGPR acc) vs ci16 x co64 (2 blocks/CU, spills)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base cur lb2 base cur lb2; do
  case $v in base) L=ab/lib_ww_base.so;; cur) L=video-matting_amd/vmatting/libvmatting.so;; lb2) L=ab/lib_ww_lb2.so;; esac
  echo "== $v" >> gpurun_out/r5f_ww.log
  VM_LIB_PATH=$L timeout -k 10 120 python -u tools/wgradwide_bench.py 10 >> gpurun_out/r5f_ww.log 2>&1 || { echo "rc=$? in $v"; exit 1; }
done
grep -E "==|total" gpurun_out/r5f_ww.log
