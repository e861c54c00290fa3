#!/bin/bash
# A/B the build_var/*.so variants: bench kernel times per config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS}; do
  echo "== $v"
  SPK_CODEC_LIB=$PWD/build_var/$v.so CONFIGS="${CONFIGS:-c3 c4}" bash scripts/gpu_q.sh || exit 1
done
