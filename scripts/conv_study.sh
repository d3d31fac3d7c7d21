#!/bin/bash
# GPU-box: patch-kernel config sweep over the UNetVideo 1080p layers + short PMC passes on two layer shapes.
#   CFGS="0 24 27" PMC_CFGS="0 27" bash scripts/conv_study.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
# the ablations / sweep tilings live in the study build only (make -C video-matting_amd study)
export VM_LIB_PATH=$(pwd)/video-matting_amd/study/libvmatting_study.so
[ -f "$VM_LIB_PATH" ] || { echo "missing $VM_LIB_PATH: run make -C video-matting_amd study first"; exit 1; }
mkdir -p gpurun_out
CFGS="${CFGS:-0}" ABLS="" timeout -k 10 900 bash scripts/sweep.sh > gpurun_out/sweep_table.txt 2>&1 || { tail -5 gpurun_out/sweep_table.txt; exit 1; }
cat gpurun_out/sweep_table.txt
for c in ${PMC_CFGS:-}; do
  for s in ${PMC_SHAPES:-540x960x256x128 270x480x512x256}; do
    PMC_SHORT=1 timeout -k 10 300 bash tools/pmc.sh "cfg${c}_$s" --shape $s --kernel 3 --patch-cfg $c --iters 10 || exit 1
  done
done
