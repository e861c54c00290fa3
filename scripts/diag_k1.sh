#!/bin/bash
# K1 statistics (a -DSPK_DIAG=1 -DSPK_K1_STATS=1 -DSPK_K1_PRINT=1 variant,
# scripts/build_ab.sh): the first pick of every decode prints them.
# Usage: scripts/diag_k1.sh variant [configs...]
v=$1; shift
mkdir -p gpurun_out/diag
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=(cmpg c3)
for c in "${cfgs[@]}"; do
  SPK_TILE_DBG=4096 SPK_CODEC_LIB=abvar/$v.so timeout -k 10 200 python bench.py --config $c --no-extra \
    --no-cpu-baseline --no-host-path --steps 2 --warmup 1 > gpurun_out/diag/${c}_$v.log 2>&1 || exit 1
done
