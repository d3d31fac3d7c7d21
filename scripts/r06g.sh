# r06: grouped patch tile order (ngroup) A/B on the bf16 headline and the f16x3 forward + its bit-identity test
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_narrowin.py -m gpu -k grouped > $O/r6g_test.log 2>&1 && \
timeout -k 10 400 python -u tools/ab_unet.py default ng2 ng4 ng8 ng4_1m > $O/r6g_ab.log 2>&1 && \
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6g_x3_ng0.log 2>&1 && \
VM_OPT=ngroup=2 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6g_x3_ng2.log 2>&1 && \
VM_OPT=ngroup=4 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6g_x3_ng4.log 2>&1 && \
VM_OPT=ngroup=4,cband_bytes=1048576 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6g_x3_ng4_1m.log 2>&1
