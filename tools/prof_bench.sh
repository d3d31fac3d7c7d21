#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box):  bash tools/prof_bench.sh <round-tag> [bench args]
#   1. --kernel-trace --stats of the FORWARD ONLY (the headline loop + its roofline pass)  -> profiles/<tag>_kernel_stats.csv
#   2. --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (own pass)          -> profiles/<tag>_mfma.json
#   3. --pmc FETCH_SIZE, 4. --pmc WRITE_SIZE (own passes)                                 -> profiles/<tag>_traffic.json
#   5. --kernel-trace --stats of the config-3 record, one pass per (dtype, size)            -> profiles/<tag>_temporal_<dtype>_<HxW>_kernel_stats.csv
#   6. --kernel-trace --stats of the config-5 training step alone (8 x 320^2, bf16)        -> profiles/<tag>_train_kernel_stats.csv
#   7. --kernel-trace --stats of the small_train.py step alone (8 x 320^2, bf16, graphs)   -> profiles/<tag>_train_small_kernel_stats.csv
#   8. --kernel-trace --stats of train_image, train_chain, augment (batched), loader records and the split forwards
#      (f16x3 -> <tag>_x3_*, bf16x6 -> <tag>_x6_*)
#                                                                                         -> profiles/<tag>_<record>_kernel_stats.csv
#   9. the full bench (reads the profiles of 2-4)                                         -> gpurun_out/<tag>_bench.json
# SKIP="fwd mfma traffic temporal train train_small train_image train_chain augment loader x3 x6 bench" skips passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REPO=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT" "$REPO/profiles"
FWD="--no-cpu-baseline --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0"
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  (cd /tmp && timeout -k 10 "$lim" "$@" > "$OUT/$log" 2>&1)
  local rc=$?
  echo "[$log] rc=$rc"; tail -n 3 "$OUT/$log"
  [ $rc -eq 0 ] || exit $rc
}
skip() { [[ " $SKIP " == *" $1 "* ]]; }
if ! skip fwd; then
run 300 stats.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
    -- python3 "$REPO/bench.py" --steps 50 --warmup 5 $FWD "$@"
cp "$(find "$OUT/stats" -name '*kernel_stats.csv' | head -n 1)" "$REPO/profiles/${TAG}_kernel_stats.csv"
grep "^{\"metric\"" "$OUT/stats.log" | tail -n 1 > "$REPO/profiles/${TAG}_stats_bench.json"
fi
if ! skip mfma; then
run 300 mfma.log timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d "$OUT/mfma" -o run -- python3 "$REPO/bench.py" --steps 3 --warmup 1 --no-profile $FWD "$@"
python3 "$REPO/tools/mfma.py" --pmc "$OUT/mfma" --out "$REPO/profiles/${TAG}_mfma.json"
fi
if ! skip traffic; then
run 300 fetch.log timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run \
    -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-profile $FWD "$@"
run 300 write.log timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run \
    -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-profile $FWD "$@"
python3 "$REPO/tools/traffic.py" --fetch "$OUT/fetch" --write "$OUT/write" --out "$REPO/profiles/${TAG}_traffic.json" --forwards 4  # capture warm-up + 1 warmup + 2 steps
fi
if ! skip temporal; then
for dt in fp32 bf16; do
  for hw in 500x1200 1080x1920; do
    run 300 temporal_${dt}_${hw}.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/temporal_${dt}_${hw}" -o run \
        -- python3 "$REPO/bench.py" --only temporal --steps 20 --temporal-dtypes $dt --temporal-sizes $hw "$@"
    cp "$(find "$OUT/temporal_${dt}_${hw}" -name '*kernel_stats.csv' | head -n 1)" \
       "$REPO/profiles/${TAG}_temporal_${dt}_${hw}_kernel_stats.csv"
    grep "^{" "$OUT/temporal_${dt}_${hw}.log" | tail -n 1 > "$REPO/profiles/${TAG}_temporal_${dt}_${hw}.json"
  done
done
fi
if ! skip train; then
run 300 train.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train" -o run \
    -- python3 "$REPO/bench.py" --only train --steps 20 --warmup 3 "$@"  # eager: side-stream select chains
cp "$(find "$OUT/train" -name '*kernel_stats.csv' | head -n 1)" "$REPO/profiles/${TAG}_train_kernel_stats.csv"
grep "^{" "$OUT/train.log" | tail -n 1 > "$REPO/profiles/${TAG}_train.json"
fi
if ! skip train_small; then
run 300 train_small.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train_small" -o run \
    -- python3 "$REPO/bench.py" --only train_small --steps 20 --warmup 3 "$@"
cp "$(find "$OUT/train_small" -name '*kernel_stats.csv' | head -n 1)" "$REPO/profiles/${TAG}_train_small_kernel_stats.csv"
grep "^{" "$OUT/train_small.log" | tail -n 1 > "$REPO/profiles/${TAG}_train_small.json"
fi
# 9-13. (r05) the UNetImage step, the chained config-5 pipeline, the batched augment, the loader, the bf16x6 forward
for rec in train_image train_chain augment loader; do
  if ! skip $rec; then
    run 300 $rec.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$rec" -o run \
        -- python3 "$REPO/bench.py" --only $rec --steps 20 --warmup 3 "$@"
    cp "$(find "$OUT/$rec" -name '*kernel_stats.csv' | head -n 1)" "$REPO/profiles/${TAG}_${rec}_kernel_stats.csv"
    grep "^{" "$OUT/$rec.log" | tail -n 1 > "$REPO/profiles/${TAG}_${rec}.json"
  fi
done
# (r06) the split paths one at a time: f16x3 (x3) and bf16x6 (x6), each its forward alone
for sp in x3:f16x3 x6:bf16x6; do
  key=${sp%%:*}; dt=${sp##*:}
  if ! skip $key; then
    run 300 $key.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$key" -o run \
        -- python3 "$REPO/tools/x6bench.py" 10 $dt
    cp "$(find "$OUT/$key" -name '*kernel_stats.csv' | head -n 1)" "$REPO/profiles/${TAG}_${key}_kernel_stats.csv"
    grep -v "amdgpu.ids" "$OUT/$key.log" | grep -v "^[EW]20" > "$REPO/profiles/${TAG}_${key}.log" || true
  fi
done
cp "$REPO"/profiles/${TAG}_* "$REPO/gpurun_out/"
skip bench && exit 0
run 600 bench.log python3 "$REPO/bench.py" --layers "$@"
tail -n 1 "$OUT/bench.log" > "$REPO/gpurun_out/${TAG}_bench.json"
grep -E "conv #|launches" "$OUT/bench.log" > "$REPO/gpurun_out/${TAG}_bench_layers.log" || true
