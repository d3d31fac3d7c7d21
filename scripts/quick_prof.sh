#!/bin/bash
# GPU-box: parity tests, then a rocprofv3 --kernel-trace --stats bench run (summary printed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-quick}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -q -m "gpu and not slow" -x -rf > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --layers ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1)
rc=$?; [ $rc -eq 0 ] || { tail -n 20 gpurun_out/prof_$TAG.log; exit $rc; }
grep -v "^[EW]2026" gpurun_out/prof_$TAG.log | tail -n 30
python3 - "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/prof_%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print("%-70s %5s %10.1f us avg %6.2f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
