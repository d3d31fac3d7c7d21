#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for one convbench shape.
#   bash tools/pmc.sh <tag> <convbench args...>
# Output: gpurun_out/pmc_<tag>/pass<N>/...counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REPO=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
PASSES=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace --output-format csv -d "$OUT/pass$i" -o run \
      -- python3 "$REPO/tools/convbench.py" "$@" > "$OUT/pass$i.log" 2>&1)
  rc=$?
  echo "[pmc $TAG pass$i] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
