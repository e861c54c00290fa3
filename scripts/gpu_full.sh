#!/bin/bash
# Full-size parity (slow tests), per-config bench lines, rocprofv3 stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1; shift; local t=$1; shift
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi; }
[ -n "$SKIP_SLOW" ] || step pytest_slow 1200 python -m pytest tests -x -q -m "gpu and slow"
step probe_bw 300 python scripts/probe_bw.py
for c in ${CONFIGS:-c2 c2b c3 c4}; do
  step bench_$c 600 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline
done
rm -rf gpurun_out/prof_c2
step rocprof_c2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --full-line --no-host-path --config c2 --steps 10 --warmup 2 --no-cpu-baseline
