#!/bin/bash
# GPU-box check: parity tests, smoke, a short bench.  Each GPU step has its own time limit;
# a crash / abort / timeout ends the script (no further GPU work), test failures do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-pytest smoke bench}"
PYTEST_SEL="${PYTEST_SEL:-gpu and not slow}"

guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 5 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}

for s in $STEPS; do
  case $s in
    pytest) guard 900 pytest_gpu.log python -m pytest tests -q -m "$PYTEST_SEL" -rf ;;
    slow)   guard 900 pytest_slow.log python -m pytest tests -q -m "gpu and slow" -rf -s ;;
    smoke)  guard 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    convbench) guard 300 convbench.log python tools/convbench.py --unet-layers --iters 20 ${CONVBENCH_ARGS} ;;
    bench)  guard 600 bench.log python bench.py --steps "${BENCH_STEPS:-10}" --warmup 3 ${BENCH_ARGS} ;;
  esac
done
