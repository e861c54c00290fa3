#!/bin/bash
# the GPU parity suite (default lib), then the A/B of build_var/$VARIANTS over $CONFIGS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pytest_q.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
bash scripts/ab_lib.sh
