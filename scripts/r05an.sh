#!/bin/bash
# GPU-box: the default bench line (as the driver runs it) + smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r05an_bench.log 2> gpurun_out/r05an_bench.err || { tail -20 gpurun_out/r05an_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
tail -n 1 gpurun_out/r05an_bench.log | cut -c1-400
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05an_smoke.log 2>&1 || { tail -20 gpurun_out/r05an_smoke.log; exit 1; }
tail -1 gpurun_out/r05an_smoke.log
