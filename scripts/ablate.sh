cd $GRAFT_REPO_ROOT
for ab in 0 1 2 4 3 6 7; do
  echo "== ablate $ab"
  timeout -k 10 120 python tools/convbench.py --shape 270x480x256x256 --shape 1080x1920x128x64 --shape 540x960x256x128 --ablate $ab --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
done
