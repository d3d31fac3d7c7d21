#!/bin/bash
# SQ stall breakdown of every conv kernel of the 1080p forward (one rocprofv3 --pmc pass; run on the GPU box):
# SQ_WAIT_ANY (waves parked at s_waitcnt / s_barrier), SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_ANY, as
# fractions of SQ_WAVE_CYCLES, plus MFMA busy.  Output: gpurun_out/pmc_convs/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REPO=$(pwd)
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/pmc_convs
mkdir -p "$OUT"
FWD="--no-cpu-baseline --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0 --no-profile"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/sq" -o run \
    -- python3 "$REPO/bench.py" --steps 3 --warmup 1 $FWD "$@" > "$OUT/sq.log" 2>&1) || { echo "sq pass failed"; tail -5 "$OUT/sq.log"; exit 1; }
python3 - "$OUT/sq/run_counter_collection.csv" <<'PY'
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in rows:
    agg[r['Kernel_Name']][r['Counter_Name']] += float(r['Counter_Value']); disp[r['Kernel_Name']].add(r['Dispatch_Id'])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES']):
    if 'conv3x3' not in k and 'head' not in k:
        continue
    wc = v['SQ_WAVE_CYCLES'] or 1
    g = v['GRBM_GUI_ACTIVE'] / 8
    print("%-72s n=%3d wait_any %.3f wait_inst %.3f (lds %.3f) active %.3f mfma_busy %.3f lds_insts/launch %.0f" % (
        k[:72], len(disp[k]), v['SQ_WAIT_ANY'] / wc, v['SQ_WAIT_INST_ANY'] / wc, v['SQ_WAIT_INST_LDS'] / wc,
        v['SQ_ACTIVE_INST_ANY'] / wc, v['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g) if g else 0,
        v['SQ_INSTS_LDS'] / len(disp[k])))
PY
