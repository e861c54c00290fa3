#!/bin/bash
# (diagnostics build only: -DSPK_DIAG=1, scripts/build_variant.sh)
# K1/K4 cost breakdown: SPK_TILE_DBG bits (8: no spec walk, 16: no chunk-0 re-screen, 32: no resolution, 64: no record stores, 128: K4 staging only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in ${DBGS:-0 8 32 40}; do
  echo "DBG=$d"; SPK_TILE_DBG=$d CONFIGS="${CONFIGS:-c3 c4}" bash scripts/gpu_q.sh | grep -E "tile_spec|tile_emit|tile_select|^c"
done
