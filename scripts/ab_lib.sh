#!/bin/bash
# Same-box A/B of builds build_var/$V.so over $CONFIGS (bench.py phase and
# top kernel times), $REPS rounds alternating the variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-old new}; do
    for c in ${CONFIGS:-c2b}; do
      SPK_CODEC_LIB=build_var/$v.so timeout -k 10 200 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/ab_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/ab_${v}_$c.log; exit 1; }
      tail -1 gpurun_out/ab_${v}_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=sorted(d['kernels'].items(), key=lambda x: -x[1]['ms_per_step'])[:3]; print('$v', '$c', d['ms_per_step'], d.get('phase_ms'), [(n[:24], v['ms_per_step']) for n, v in k])"
    done
  done
done
