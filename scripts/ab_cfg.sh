#!/bin/bash
# A/B of abvar/ variants (scripts/build_ab.sh) against the in-tree library on
# the configs in $CFGS, alternated twice on one box: ab_cfg.sh variant...
set -o pipefail
mkdir -p gpurun_out/ab
for c in ${CFGS:-c3 c4}; do
  B="python bench.py --config $c --no-extra --no-cpu-baseline --no-host-path --full-line --steps 20"
  for i in 1 2; do
    timeout -k 10 200 $B > gpurun_out/ab/${c}_head_$i.log 2>&1 || exit 1
    for v in "$@"; do
      SPK_CODEC_LIB=abvar/$v.so timeout -k 10 200 $B > gpurun_out/ab/${c}_${v}_$i.log 2>&1 || exit 1
    done
  done
done
python3 scripts/ab_table.py gpurun_out/ab
