#!/bin/bash
# MESSAGES nested decode change: the GPU suite, then bench cvm / c5 (kernel tables)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
for c in ${CONFIGS:-cvm}; do
  timeout -k 10 200 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/q_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/q_$c.log; exit 1; }
  tail -1 gpurun_out/q_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=sorted(d['kernels'].items(), key=lambda x: -x[1]['ms_per_step'])[:6]; print('$c', d['ms_per_step'], d.get('phase_ms'), [(n[:24], round(v['ms_per_step'],4)) for n, v in k], d['roofline']['kernel'], d['roofline']['frac'])"
done
