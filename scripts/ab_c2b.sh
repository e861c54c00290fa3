#!/bin/bash
# A/B of the MESSAGES-mode fixed kernels on C2b: the in-tree library against
# abvar/ variants (scripts/build_ab.sh), alternated twice on one box.
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --config c2b --no-extra --no-cpu-baseline --no-host-path --full-line --steps 20"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/ab_c2b_head_$i.log 2>&1 || exit 1
  for v in "$@"; do
    SPK_CODEC_LIB=abvar/$v.so timeout -k 10 200 $B > gpurun_out/ab_c2b_${v}_$i.log 2>&1 || exit 1
  done
done
for f in gpurun_out/ab_c2b_*.log; do echo $f; python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print(d['ms_per_step'], {k:v['ms_per_launch'] for k,v in d['kernels'].items()})
"; done
