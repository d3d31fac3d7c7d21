#!/bin/bash
# round-5 first GPU check: SyncBN count fix, stream getters, graph-vs-eager at 1080p, then the capture probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 8 "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf"
guard 600 r5a_syncbn.log $PT tests/test_capi.py tests/test_gpu_small_train.py tests/test_gpu_train.py -m gpu -k "syncbn or raw_stream or ddp"
guard 400 r5a_graph1080.log $PT tests/test_gpu_layers_1080p.py -m gpu -k "graph_replay or timed_kernels or head_logits"
guard 600 r5a_wide.log $PT tests/test_gpu_train.py -m gpu -k "wgrad"
guard 900 r5a_image.log $PT tests/test_gpu_image_train.py -m gpu
guard 600 r5a_probe.log python -u tools/capture_probe.py
