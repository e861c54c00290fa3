#!/bin/bash
# HBM traffic of the C2 kernels from PMC counters (separate passes: FETCH_SIZE
# and WRITE_SIZE do not fit one TCC pass on gfx950), plus the host-path rate.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-c2}
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_${CFG}_$ctr
  timeout -k 10 600 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${CFG}_$ctr -o run --output-format csv -- python bench.py --full-line --no-host-path --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-extra --settle 0 > gpurun_out/pmc_${CFG}_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -20 gpurun_out/pmc_${CFG}_$ctr.log; exit 1; }
done
python scripts/pmc_summary.py $CFG > gpurun_out/pmc_${CFG}.json && cat gpurun_out/pmc_${CFG}.json
