#!/bin/bash
# rocprofv3 kernel-trace stats for the configs in $CONFIGS (default: c2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CONFIGS:-c2}; do
  rm -rf gpurun_out/prof_$c
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/prof_$c.log 2>&1 || { echo "rocprof $c failed"; tail -20 gpurun_out/prof_$c.log; exit 1; }
  echo "== $c"; tail -1 gpurun_out/prof_$c.log | cut -c1-200
  head -12 gpurun_out/prof_$c/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
