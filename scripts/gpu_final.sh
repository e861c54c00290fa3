#!/bin/bash
# Round-end evidence after K1 changes: the GPU suite, PMC passes for the
# configs whose kernels changed, the default bench line (other configs' PMC
# summaries from profiles/$ROUND), rocprofv3 stats for the changed configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/evidence
rm -rf $OUT && mkdir -p $OUT
ROUND=${ROUND:-r03}
CH=${CH:-c3 c4 cv}
step() { local name=$1; shift; local t=$1; shift
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi; }
[ -n "$SKIP_TESTS" ] || step pytest_gpu 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/
for c in $CH; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step pmc_${c}_$ctr 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${c}_$ctr -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps 3 --warmup 1 --settle 0 --no-cpu-baseline --no-extra
  done
  python scripts/pmc_summary.py $c $OUT > $OUT/pmc_$c.json || exit 1
  rm -rf $OUT/pmc_${c}_FETCH_SIZE $OUT/pmc_${c}_WRITE_SIZE
done
for f in profiles/$ROUND/pmc_*.json; do
  b=$(basename $f); [ -e $OUT/$b ] || cp $f $OUT/$b
done
step bench 1000 python bench.py --pmc-dir $OUT
for c in $CH; do
  step prof_$c 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-extra
  find $OUT/prof_$c -name "*kernel_stats.csv" -exec cp {} $OUT/${c}_kernel_stats.csv \;
  rm -rf $OUT/prof_$c
done
echo done
