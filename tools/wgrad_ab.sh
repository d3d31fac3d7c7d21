#!/bin/bash
# A/B of the MFMA weight-gradient tile variants on the config-5 shapes (GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in ${VARIANTS:-1 2}; do
  echo "== wgrad_variant $v"
  WGRAD_VARIANT=$v timeout -k 10 120 python tools/wgradbench.py 10 || exit 1
done
