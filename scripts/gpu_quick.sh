#!/bin/bash
# Quick GPU iteration: GPU tests (not slow), then phase timings for $CONFIGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for c in ${CONFIGS:-c3 c4 c5}; do
  timeout -k 10 300 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/q_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/q_$c.log; exit 1; }
  tail -1 gpurun_out/q_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d.get('phase_ms'))"
done
