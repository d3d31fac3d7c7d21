# r06: config-5 trainer side streams, torch pool vs probed (interleaved), after its GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_streams.py -m gpu > $O/r6s_tests.log 2>&1 && \
for k in pool probe pool probe; do timeout -k 10 200 python -u bench.py --only train --steps 40 --warmup 5 --train-side $k > $O/r6s_$k.log 2>&1 || exit 1; echo "$k $(grep -o '"ms_per_step": [0-9.]*' $O/r6s_$k.log | head -1)" >> $O/r6s_ab.txt; done
