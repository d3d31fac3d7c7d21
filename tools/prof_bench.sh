#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box):  bash tools/prof_bench.sh <round-tag> [bench args]
#   1. --kernel-trace --stats of a short bench run      -> profiles/<tag>_kernel_stats.csv
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (own passes) -> profiles/<tag>_traffic.json
#   4. the bench itself (reads the traffic file)         -> gpurun_out/<tag>_bench.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REPO=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT" "$REPO/profiles"
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  (cd /tmp && timeout -k 10 "$lim" "$@" > "$OUT/$log" 2>&1)
  local rc=$?
  echo "[$log] rc=$rc"; tail -n 4 "$OUT/$log"
  [ $rc -eq 0 ] || exit $rc
}
run 400 stats.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
    -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-train "$@"
cp "$(find "$OUT/stats" -name '*kernel_stats.csv' | head -n 1)" "$REPO/profiles/${TAG}_kernel_stats.csv"
run 400 fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run \
    -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-loader --no-augment --no-train --video-frames 0 "$@"
run 400 write.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run \
    -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-loader --no-augment --no-train --video-frames 0 "$@"
python3 "$REPO/tools/traffic.py" --fetch "$OUT/fetch" --write "$OUT/write" --out "$REPO/profiles/${TAG}_traffic.json" --forwards 4  # capture warm-up + 1 warmup + 2 steps
cp "$REPO/profiles/${TAG}_traffic.json" "$REPO/profiles/${TAG}_kernel_stats.csv" "$REPO/gpurun_out/"
run 600 bench.log python3 "$REPO/bench.py" --layers "$@"
tail -n 1 "$OUT/bench.log" > "$REPO/gpurun_out/${TAG}_bench.json"
