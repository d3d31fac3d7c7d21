cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m "gpu and not slow" -x -rf -k "patch" > gpurun_out/pytest_patch.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_patch.log
[ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-5 7 8 9 10}; do
  timeout -k 10 120 python tools/convbench.py --unet-layers --kernel 3 --patch-cfg $c --iters 10 > gpurun_out/cb_patch$c.log 2>&1 || exit 1
done
python3 - <<'PY'
import re
import os; cfgs=[int(c) for c in os.environ.get("CFGS","5 7 8 9 10").split()]
rows={}
for c in cfgs:
    for line in open(f"gpurun_out/cb_patch{c}.log"):
        m=re.search(r"^(\S+)\s.*?([\d.]+) ms",line)
        if m: rows.setdefault(m.group(1),{})[c]=float(m.group(2))
print("%-10s"%"layer"+"".join("%8d"%c for c in cfgs))
for k,v in rows.items(): print("%-10s"%k+"".join("%8.4f"%v.get(c,0) for c in cfgs))
PY
