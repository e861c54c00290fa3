#!/bin/bash
# GPU-box check: smoke, GPU parity tests, a short bench. Each GPU step has its
# own time limit and the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="${PYTEST_SEL:-gpu and not slow}"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 1200 python -m pytest tests -x -q -m "$PYTEST_SEL" > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
