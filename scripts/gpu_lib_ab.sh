#!/bin/bash
# per-config kernel times for alternative builds: LIBS="default abso/x.so ..." CONFIGS="c3 c4" KERNEL=name
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-1}); do
for lib in ${LIBS:-default}; do
  for c in ${CONFIGS:-c3 c4}; do
    if [ "$lib" = default ]; then unset SPK_CODEC_LIB; else export SPK_CODEC_LIB=$lib; fi
    timeout -k 10 300 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/l_$c.log 2>&1 || { echo "bench $c $lib failed"; tail -20 gpurun_out/l_$c.log; exit 1; }
    tail -1 gpurun_out/l_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$lib', '$c', d['ms_per_step'], d.get('phase_ms'), [(n[:24], round(v['ms_per_step'],4)) for n, v in k.items() if '${KERNEL:-var_encode_write}' in n])"
  done
done
done
