#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for one convbench shape.
#   bash tools/pmc.sh <tag> <convbench args...>
# Output: gpurun_out/pmc_<tag>/pass<N>/...counter_collection.csv, summary in gpurun_out/pmc_<tag>/summary.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REPO=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
PASSES=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES"
  "TA_TA_BUSY TA_BUFFER_READ_LDS_WAVEFRONTS"
  "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES"
  "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TD_TD_BUSY"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
[ -n "$PMC_SHORT" ] && PASSES=("${PASSES[@]:0:2}")
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace --output-format csv -d "$OUT/pass$i" -o run \
      -- python3 "$REPO/tools/${PMC_TOOL:-convbench.py}" "$@" > "$OUT/pass$i.log" 2>&1)
  rc=$?
  if [ $rc -ne 0 ]; then echo "[pmc $TAG pass$i] rc=$rc"; tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
python3 "$REPO/tools/pmc_summary.py" "$OUT" "${PMC_KERNEL:-conv3x3}" | tee "$OUT/summary.txt"
