#!/bin/bash
# K1 speculation caps: tile statistics and same-box A/B (build_var/scap0.so vs scap1.so), then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${DIAG_VARIANTS}; do
  for cs in "var 2000000 16" "recs 2000000 48" "outer 2000000 16"; do
    SPK_CODEC_LIB=build_var/$v.so SPK_TILE_DBG=4096 timeout -k 10 200 python scripts/diag_tiles.py $cs > gpurun_out/diag_${v}.log 2>&1 || { echo "diag failed"; tail -5 gpurun_out/diag_${v}.log; exit 1; }
    echo "== $v"; cat gpurun_out/diag_${v}.log
  done
done
VARIANTS="${VARIANTS:-scap0 scap1}" CONFIGS="${CONFIGS:-c3 c4 cv}" REPS=${REPS:-2} bash scripts/ab_lib.sh || exit 1
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m "$TESTS" tests/ > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt.log; exit 1; }
  tail -2 gpurun_out/pt.log
fi
