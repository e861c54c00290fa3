#!/bin/bash
# C5 per-type timings (scripts/diag_c5.py) for each build_var/$V.so in $VARIANTS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARIANTS:-e0}; do
  echo "== $v"
  SPK_CODEC_LIB=build_var/$v.so timeout -k 10 120 python scripts/diag_c5.py 2>&1 | grep -E "ints|person" || exit 1
done
