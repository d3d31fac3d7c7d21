# r06: config-5 step against its side-stream count (select chains) and the filter-gradient stream, interleaved
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
for rep in 1 2; do
  for cfg in "3 1" "2 1" "1 1" "3 0" "4 1"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --only train --steps 40 --warmup 5 --train-streams $1 --train-wgrad-stream $2 > $O/r6t.log 2>&1 || exit 1
    echo "streams=$1 wgrad_stream=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/r6t.log | head -1)" >> $O/r6t_ab.txt
  done
done
