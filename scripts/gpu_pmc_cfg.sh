#!/bin/bash
# PMC passes (one counter group per run) for the configs in $CONFIGS:
# HBM bytes (FETCH_SIZE, WRITE_SIZE) and an SQ pass (waves, cycles, stalls).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
for c in ${CONFIGS:-c3}; do
  for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    rm -rf $OUT/pmc_${c}_$tag
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/pmc_${c}_$tag -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps 2 --warmup 1 --settle 0 --no-cpu-baseline > $OUT/pmc_${c}_$tag.log 2>&1 || { echo "pmc $c $tag failed"; tail -5 $OUT/pmc_${c}_$tag.log; exit 1; }
  done
  python scripts/pmc_summary.py $c $OUT > $OUT/pmc_$c.json
done
echo ok
