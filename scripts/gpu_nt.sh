#!/bin/bash
# nested walker change: the nested GPU parity tests, then the cm / c4 A/B of
# build_var/$VARIANTS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "monster or deep or tags or group or vnt or lists or maps or cplx or outer or wide or valreq or exp or cmpg" > gpurun_out/pytest_nt.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_nt.log; exit 1; }
tail -1 gpurun_out/pytest_nt.log
VARIANTS="${VARIANTS:-un0 un1}" CONFIGS="${CONFIGS:-cm}" REPS=${REPS:-2} bash scripts/ab_lib.sh
