#!/bin/bash
# Same-box A/B of exported commits (build_var/bis/<commit>/, each with its
# own bench.py and codec) on one config: K1 / K4 / step times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTD=$PWD
mkdir -p gpurun_out
CFG=${CFG:-c4}
for r in 1 2; do
  for d in build_var/bis/* HEAD; do
    [ -d "$d" ] || [ "$d" = HEAD ] || continue
    [ -f "$d/bench.py" ] || [ "$d" = HEAD ] || continue
    if [ "$d" = HEAD ]; then dir=$ROOTD; extra="--full-line --no-host-path"; else dir=$ROOTD/$d; extra=""; fi
    name=$(basename $d)
    (cd $dir && timeout -k 10 120 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-extra $extra > $ROOTD/gpurun_out/bis_${name}.log 2>&1) || { echo "fail $name"; tail -3 gpurun_out/bis_${name}.log; exit 1; }
    tail -1 gpurun_out/bis_${name}.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels',{})
f=lambda p: sum(v['ms_per_step'] for n,v in k.items() if n.startswith(p))
print('$name', d['ms_per_step'], 'K1 %.4f K4 %.4f' % (f('vec_tile_spec'), f('vec_tile_emit')), d.get('phase_ms'))"
  done
done
