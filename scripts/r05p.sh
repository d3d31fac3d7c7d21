#!/bin/bash
# GPU-box: halfskip persistent walk — parity (persistent vs streaming, 1080p layer pins), then same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "persist or rows" tests/test_gpu_layers_1080p.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p_tests.log 2>&1 || { tail -30 gpurun_out/r05p_tests.log; exit 1; }
tail -3 gpurun_out/r05p_tests.log
OPT=persist_half=0,1 AB_ROUNDS="1 2 3" bash scripts/opt_ab.sh
