# r06: the f16x3 head on 16-row tiles vs 8 (kernel stats of the split forward, tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu > $O/r6w_tests.log 2>&1 && \
for th in 16 8; do
  (cd /tmp && VM_OPT=head_th=$th timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r6w_$th -o run \
     -- python3 $GRAFT_REPO_ROOT/tools/x6bench.py 10 f16x3 > $O/r6w_$th.log 2>&1) || exit 1
done
