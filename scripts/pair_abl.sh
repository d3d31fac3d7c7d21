#!/bin/bash
# pair-kernel timing ablations (pair_kernel 11 no conv1_1 MFMA, 12 no conv1_2 MFMA, 13 neither, 14 no stores, 18 no input loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
# the ablations / sweep tilings live in the study build only (make -C video-matting_amd study)
export VM_LIB_PATH=$(pwd)/video-matting_amd/study/libvmatting_study.so
[ -f "$VM_LIB_PATH" ] || { echo "missing $VM_LIB_PATH: run make -C video-matting_amd study first"; exit 1; }
mkdir -p gpurun_out
for k in 0 11 12 13 14 18 0; do
  timeout -k 10 120 python tools/pairbench.py --pair-kernel $k --iters 50 > gpurun_out/pair_$k.log 2>&1 || { tail -3 gpurun_out/pair_$k.log; exit 1; }
  echo "pair_kernel=$k $(tail -n 1 gpurun_out/pair_$k.log)"
done
