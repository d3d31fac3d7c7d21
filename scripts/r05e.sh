#!/bin/bash
# round-5: x6 capture fix check + timing; kernel stats of the UNetImage step and of the config-5 chain
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
REPO=$(pwd)
mkdir -p gpurun_out/r5e
guard() {  # guard <limit> <logfile> cmd...
  local lim=$1 log=$2; shift 2
  (cd /tmp && timeout -k 10 "$lim" "$@" > "$REPO/gpurun_out/$log" 2>&1)
  local rc=$?
  echo "[$log] rc=$rc"
  tail -n 6 "$REPO/gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 135 ]; then
    echo "fatal rc=$rc in $log — stopping"; exit $rc
  fi
}
guard 300 r5e_x6.log python3 -u $REPO/tools/x6bench.py 10
guard 300 r5e_timage_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/r5e/timage -o run -- python3 $REPO/bench.py --only train_image --steps 10 --warmup 2
guard 300 r5e_chain_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/r5e/chain -o run -- python3 $REPO/bench.py --only train_chain --steps 10 --warmup 2
find $REPO/gpurun_out/r5e -name '*kernel_stats.csv' | head
