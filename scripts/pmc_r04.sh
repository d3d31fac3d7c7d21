#!/bin/bash
# PMC passes behind DESIGN.md §8 items 4-5 (run on the GPU box): the f32 refine kernel's ablations and the narrow
# select conv, each counter set in its own rocprofv3 pass.  Output: gpurun_out/pmc_r04/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REPO=$(pwd)
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/pmc_r04
mkdir -p "$OUT"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
STUDY=$REPO/video-matting_amd/study/libvmatting_study.so
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  (cd /tmp && timeout -k 10 "$lim" "$@" > "$OUT/$log" 2>&1)
  local rc=$?
  echo "[$log] rc=$rc"; tail -n 4 "$OUT/$log"
  [ $rc -eq 0 ] || exit $rc
}
run 200 smxabl.log env VM_LIB_PATH=$STUDY python3 "$REPO/tools/smxabl.py"
export VM_LIB_PATH=$STUDY
run 120 smx_sq.log timeout -s KILL 100 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/smx_sq" -o run \
    -- python3 "$REPO/tools/smxabl.py" 0 1 2 5 6
unset VM_LIB_PATH
run 120 thin.log python3 "$REPO/tools/thinbench.py"
run 120 thin_sq.log timeout -s KILL 100 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/thin_sq" -o run \
    -- python3 "$REPO/tools/thinbench.py" --iters 10
run 120 thin_fetch.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/thin_fetch" \
    -o run -- python3 "$REPO/tools/thinbench.py" --iters 10
