#!/bin/bash
# GPU-box: per-launch kernel trace of the UNetImage training step (bench shape)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05tt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05tt -o trace -- python bench.py --only train --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r05tt/bench.log 2>&1 || { tail -20 gpurun_out/r05tt/bench.log; exit 1; }
ls gpurun_out/r05tt
