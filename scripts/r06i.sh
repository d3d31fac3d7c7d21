# r06: the UNetImage step inside vs outside the full bench's record sequence
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/img_interference.py > gpurun_out/r6i_img.log 2>&1
