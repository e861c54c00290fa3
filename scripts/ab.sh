#!/bin/bash
# Same-box A/B of two builds of libspk_codec.so (ab/old.so vs ab/new.so):
# alternates them $REPS times over the configs in $CONFIGS, printing the
# phase times of each run. The in-tree library is restored at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=yalantinglibs_amd/libspk_codec.so
cp $LIB ab/current.so
for r in $(seq ${REPS:-2}); do
  for v in old new; do
    cp ab/$v.so $LIB
    for c in ${CONFIGS:-c3 c4}; do
      timeout -k 10 300 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/ab_$v_$c.log; cp ab/current.so $LIB; exit 1; }
      tail -1 gpurun_out/ab_$v_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '$c', d['ms_per_step'], d.get('phase_ms'))"
    done
  done
done
cp ab/current.so $LIB
