#!/bin/bash
# A/B of the tile decoder's K1 phases on one config (SPK_TILE_DBG bits: 8 no
# speculative walk, 16 no chunk-0 cross-check, 32 no in-wave resolution;
# decode output is wrong with any bit set: timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${CFG:-cm}
for v in ${DBGS:-0 32 48 56}; do
  SPK_TILE_DBG=$v timeout -k 10 300 python bench.py --full-line --no-host-path --config $C --steps 5 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/abd_$C.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/abd_$C.log; exit 1; }
  python - $C "$v" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/abd_{sys.argv[1]}.log').read().strip().splitlines()[-1])
k=d['kernels']
print('dbg', sys.argv[2], sys.argv[1], d['phase_ms'], {n: round(v['ms_per_step'],3) for n,v in k.items() if v['ms_per_step'] > 0.05})
PY
done
