#!/bin/bash
# round-3: training tests + a serial (one-stream) rocprof of the config-5 step + the 3-stream step time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r03f}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_thin.py -q -x --timeout 200 --timeout-method thread -rf \
      > gpurun_out/pt_train.log 2>&1; rc=$?; tail -3 gpurun_out/pt_train.log
  [ $rc -eq 0 ] || exit $rc
fi
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/serial" -o run \
    -- python3 "$OLDPWD/bench.py" --only train --steps 20 --warmup 3 --train-streams 0 > "$OUT/serial.log" 2>&1) || exit $?
tail -1 "$OUT/serial.log"
cp "$(find "$OUT/serial" -name '*kernel_stats.csv' | head -n 1)" "gpurun_out/${TAG}_train_serial_kernel_stats.csv"
for v in "3 1" "0 1" "3 0" "3 1" "3 0"; do
  set -- $v
  timeout -k 10 300 python bench.py --only train --steps 30 --warmup 5 --train-streams $1 --option thin_rounds=$2 \
      > gpurun_out/train_s$1_t$2.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/train_s$1_t$2.log').read().strip().splitlines()[-1]); print('streams', $1, 'thin_rounds', $2, d['record']['ms_per_step'], d['record']['device_ms'])"
done
