#!/bin/bash
# Full GPU suite (smoke first), the timing prints of the bounded-time tests,
# then the driver's default bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests -q -s -m gpu -k "mispredicted or screen_defeating or long_records" > gpurun_out/pytest_timing.log 2>&1 || { echo "timing tests failed"; tail -20 gpurun_out/pytest_timing.log; exit 1; }
grep -E "MB" gpurun_out/pytest_timing.log | head
[ -n "$NO_BENCH" ] && exit 0
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default.err; exit 1; }
echo "bench took $(( $(date +%s) - start )) s"
tail -c 3000 gpurun_out/bench_default.log
