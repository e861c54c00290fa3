#!/bin/bash
# Round-3 GPU check: GPU tests (not slow), then quick bench lines of the
# configs in $CONFIGS (default cm c5) with $BENCH_ARGS. Each step has its own
# time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m "${TESTS:-gpu and not slow}" ${KEYS:+-k "$KEYS"} > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt.log; exit 1; }
  tail -2 gpurun_out/pt.log
fi
for c in ${CONFIGS:-cm c5}; do
  timeout -k 10 600 python bench.py --full-line --no-host-path --config $c --steps ${STEPS:-10} --warmup 2 --no-extra $BENCH_ARGS > gpurun_out/b_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/b_$c.log; exit 1; }
  python - $c <<'PY'
import json,sys
c=sys.argv[1]
d=json.loads(open(f'gpurun_out/b_{c}.log').read().strip().splitlines()[-1])
print(c, d.get('value'), d.get('ms_per_step'), d.get('phase_ms'), 'host:', d.get('host_path'), 'cpu:', (d.get('cpu_baseline') or {}).get('value'))
for k,x in sorted(d.get('kernels',{}).items(), key=lambda kv:-kv[1]['ms_per_step'])[:6]:
    print('   %-28s %6.1f %8.4f %s'%(k, x['launches_per_step'], x['ms_per_step'], x.get('frac','')))
PY
done
