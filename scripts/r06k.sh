# r06: patch tilings forced (patch_cfg) on the f16x3 forward: per-layer times of the 135x240 / 68x120 levels
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6k_auto.log 2>&1 && \
VM_OPT=patch_cfg=30 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6k_cfg30.log 2>&1 && \
VM_OPT=patch_cfg=19 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6k_cfg19.log 2>&1 && \
VM_OPT=patch_cfg=25 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6k_cfg25.log 2>&1
