#!/bin/bash
# K1 (vec_tile_spec) cost breakdown via SPK_TILE_DBG bits (outputs invalid;
# timing only): 8 = no speculative walk, 16 = no chunk-0 cross-check,
# 32 = no in-wave resolution. Needs a diagnostics build of the library
# (-DSPK_DIAG=1, scripts/build_variant.sh): a release build ignores SPK_TILE_DBG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for c in ${CONFIGS:-c3 c4}; do
  for d in ${DBGS:-0 56 48 32}; do
    SPK_TILE_DBG=$d timeout -k 10 100 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/k1_$c_$d.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/k1_$c_$d.log; exit 1; }
    tail -1 gpurun_out/k1_$c_$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$c dbg=$d', {n: v['ms_per_step'] for n, v in k.items() if 'tile_spec' in n or 'tile_emit' in n})"
  done
done
