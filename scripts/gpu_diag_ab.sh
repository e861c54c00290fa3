#!/bin/bash
# K1 statistics (SPK_TILE_DBG=4096) for $DIAG cases (case:records:param),
# then the A/B of build_var/*.so ($VARIANTS) over $CONFIGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
DIAG=${DIAG:-monster:1000000:20 var:1000000:16}
[ "$DIAG" = none ] && DIAG=""
for c in $DIAG; do
  SPK_TILE_DBG=4096 timeout -k 10 120 python scripts/diag_tiles.py ${c//:/ } || exit 1
done
[ -z "$VARIANTS" ] || bash scripts/ab_lib.sh
