# r06: the row-stationary kernel forced wherever legal (rows_kernel=16) vs auto, per layer, f16x3 and bf16
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 bf16 > $O/r6h_auto.log 2>&1 && \
VM_OPT=rows_kernel=16 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 bf16 > $O/r6h_rows16.log 2>&1 && \
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 bf16 > $O/r6h_auto2.log 2>&1
