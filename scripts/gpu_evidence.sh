#!/bin/bash
# Round evidence in one GPU call: HBM PMC passes for the dominant kernels
# (FETCH_SIZE and WRITE_SIZE in separate runs), then bench lines for every
# config (C2 with the reference CPU baseline and the host path; traffic from
# the PMC summaries), then rocprofv3 kernel stats per config. Each GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/evidence
rm -rf $OUT && mkdir -p $OUT
step() { local name=$1; shift; local t=$1; shift
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi; }
for c in c2 c2b c3 c4; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step pmc_${c}_$ctr 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${c}_$ctr -o run --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --settle 0 --no-cpu-baseline
  done
  python scripts/pmc_summary.py $c $OUT > $OUT/pmc_$c.json || exit 1
done
step bench_c2 600 python bench.py --config c2 --host-path --pmc-json $OUT/pmc_c2.json
step bench_c2b 600 python bench.py --config c2b --steps 10 --warmup 2 --no-cpu-baseline --host-path --pmc-json $OUT/pmc_c2b.json
for c in c3 c4; do
  step bench_$c 600 python bench.py --config $c --steps 10 --warmup 2 --host-path --pmc-json $OUT/pmc_$c.json
done
step bench_c5 600 python bench.py --config c5 --steps 10 --warmup 2 --host-path
for c in ${PROF_CONFIGS:-c2 c2b c3 c4 c5}; do
  step prof_$c 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline
done
echo done
