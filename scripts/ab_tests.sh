#!/bin/bash
# the timing-printing GPU tests under each abvar/ variant (and the in-tree
# library): ab_tests.sh "pytest -k expression" variant...
k=$1; shift
mkdir -p gpurun_out/abt
for v in head "$@"; do
  lib=""; [ "$v" != head ] && lib=abvar/$v.so
  SPK_CODEC_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s \
    -k "$k" --timeout 200 --timeout-method thread > gpurun_out/abt/$v.log 2>&1 || { echo "$v failed"; exit 1; }
done
