#!/bin/bash
# GPU tests (not slow) then phase / kernel timings of $CONFIGS (default c3 c4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
fi
for r in $(seq ${REPS:-1}); do
for c in ${CONFIGS:-c3 c4}; do
  timeout -k 10 300 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/q_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/q_$c.log; exit 1; }
  tail -1 gpurun_out/q_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=sorted(d['kernels'].items(), key=lambda x: -x[1]['ms_per_step'])[:3]; print('$c', d['ms_per_step'], d.get('phase_ms'), [(n.split('(')[0][-22:], round(v['ms_per_step'],4)) for n, v in k])"
done
done
