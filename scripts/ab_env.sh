#!/bin/bash
# Same-box A/B of environment settings: for each "NAME=VAL ..." in $ENVS
# (";"-separated, "-" = none) the bench over $CONFIGS, $REPS rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
IFS=';' read -ra EV <<< "${ENVS:--}"
for r in $(seq ${REPS:-2}); do
  for e in "${EV[@]}"; do
    for c in ${CONFIGS:-c3 c4}; do
      tag=$(echo "$e" | tr -c 'A-Za-z0-9' '_')
      if [ "$e" = "-" ]; then ee=""; else ee="$e"; fi
      env $ee timeout -k 10 200 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/abe_${tag}_$c.log 2>&1 || { echo "bench failed ($e $c)"; tail -5 gpurun_out/abe_${tag}_$c.log; exit 1; }
      tail -1 gpurun_out/abe_${tag}_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=sorted(d['kernels'].items(), key=lambda x: -x[1]['ms_per_step'])[:4]; print('$e', '$c', d['ms_per_step'], d.get('phase_ms'), [(n[:20], round(v['ms_per_step'],4)) for n, v in k])"
    done
  done
done
