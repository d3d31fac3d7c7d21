#!/bin/bash
# GPU-box: the full -m gpu suite on the final build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r05w_full.log 2>&1
rc=$?
tail -8 gpurun_out/r05w_full.log
exit $rc
