#!/bin/bash
# Round evidence (one or more GPU calls: SKIP_PMC / SKIP_BENCH / PMC_CONFIGS /
# PROF_CONFIGS / PMC_DIR select the steps): HBM PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, each config on its own, --no-extra) summarised per kernel into
# $OUT/pmc_<cfg>.json; then the default bench line (C2 headline + every other
# BASELINE config in extra.configs, reading those PMC summaries, host paths);
# then rocprofv3 --kernel-trace --stats per config. Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/evidence
rm -rf $OUT && mkdir -p $OUT
step() { local name=$1; shift; local t=$1; shift
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi; }
if [ -z "$SKIP_PMC" ]; then
  for c in ${PMC_CONFIGS:-c2 c2b c3 c4 cv c5 cm}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      step pmc_${c}_$ctr 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${c}_$ctr -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps 3 --warmup 1 --settle 0 --no-cpu-baseline --no-extra
    done
    python scripts/pmc_summary.py $c $OUT > $OUT/pmc_$c.json || exit 1
    rm -rf $OUT/pmc_${c}_FETCH_SIZE $OUT/pmc_${c}_WRITE_SIZE
  done
fi
[ -n "$SKIP_BENCH" ] || step bench 900 python bench.py --pmc-dir ${PMC_DIR:-$OUT}
PROF_CONFIGS=${PROF_CONFIGS:-c2 c2b c3 c4 cv c5 cm}
[ "$PROF_CONFIGS" = none ] && PROF_CONFIGS=""
for c in $PROF_CONFIGS; do
  step prof_$c 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-extra
  cp $OUT/prof_$c/run_kernel_stats.csv $OUT/${c}_kernel_stats.csv 2>/dev/null || find $OUT/prof_$c -name "*kernel_stats.csv" -exec cp {} $OUT/${c}_kernel_stats.csv \;
  rm -rf $OUT/prof_$c
done
echo done
