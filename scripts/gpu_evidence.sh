#!/bin/bash
# Round evidence in one GPU call: bench lines for every config (C2 with the
# reference CPU baseline and the host path), rocprofv3 kernel stats per
# config, and the C2 HBM PMC passes. Each GPU step has its own time limit;
# the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/evidence
rm -rf $OUT && mkdir -p $OUT
step() { local name=$1; shift; local t=$1; shift
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi; }
step bench_c2 600 python bench.py --config c2 --host-path
step bench_c2b 600 python bench.py --config c2b --steps 10 --warmup 2 --no-cpu-baseline --host-path
for c in c3 c4 c5; do
  step bench_$c 600 python bench.py --config $c --steps 10 --warmup 2 --host-path
done
for c in ${PROF_CONFIGS:-c2 c2b c3 c4 c5}; do
  step prof_$c 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  step pmc_c2_$ctr 300 rocprofv3 --pmc $ctr -d $OUT/pmc_c2_$ctr -o run --output-format csv -- python bench.py --config c2 --steps 3 --warmup 1 --settle 0 --no-cpu-baseline
done
echo done
