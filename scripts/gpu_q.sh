#!/bin/bash
# Quick GPU iteration: optional GPU tests, then bench phase/kernel times for $CONFIGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m "$TESTS" ${KSEL:+-k "$KSEL"} tests/ > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt.log; exit 1; }
  tail -1 gpurun_out/pt.log
fi
for c in ${CONFIGS:-c3 c4}; do
  timeout -k 10 300 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra $BENCH_ARGS > gpurun_out/q_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/q_$c.log; exit 1; }
done
for c in ${CONFIGS:-c3 c4}; do
python - $c <<'PY'
import json,sys
c=sys.argv[1]
d=json.loads(open(f'gpurun_out/q_{c}.log').read().strip().splitlines()[-1])
print(c, d.get('value'), d.get('ms_per_step'), d.get('phase_ms'))
for k,x in sorted(d.get('kernels',{}).items(), key=lambda kv:-kv[1]['ms_per_step'])[:4]:
    print('   %-28s %6.1f %8.4f %s'%(k, x['launches_per_step'], x['ms_per_step'], x.get('frac','')))
PY
done
