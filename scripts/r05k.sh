#!/bin/bash
# round-5: LDS-DMA narrow wgrad (tests + step A/B), HIP graph branch-concurrency knobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" >> "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 3 "gpurun_out/$log" | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -rf"
guard 900 r5k_tests.log $PT tests/test_gpu_train.py -m gpu -k "wgrad or step_gradients or bf16_gradients or config5 or chain_overlap"
grep -E "passed|failed" gpurun_out/r5k_tests.log | tail -3
for v in 1 0 1 0; do
  guard 300 r5k_dma.log python -u bench.py --only train --steps 20 --warmup 3 --option wgrad_dma=$v
done
grep -h '"only"' gpurun_out/r5k_dma.log | cut -c1-330
guard 300 r5k_graph.log python -u bench.py --only train --steps 20 --warmup 3 --train-graph
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 guard 300 r5k_graph.log python -u bench.py --only train --steps 20 --warmup 3 --train-graph
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 guard 300 r5k_graph.log python -u bench.py --only train --steps 20 --warmup 3 --train-graph
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 guard 300 r5k_graph.log python -u bench.py --only train --steps 20 --warmup 3 --train-graph
grep -h '"only"' gpurun_out/r5k_graph.log | cut -c1-330
mkdir -p gpurun_out/r5k_prof
guard 300 r5k_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5k_prof -o run -- python -u bench.py --only train --steps 10 --warmup 3
