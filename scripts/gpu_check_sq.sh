#!/bin/bash
# opt-in types on the GPU (C++ protocol test + full suite), then SQ counters of
# the decode kernels for $CONFIGS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
if [ -z "$SQ_ONLY" ]; then
bash scripts/gpu_cpp_proto.sh || exit 1
grep -q '"failures": 0' gpurun_out/proto_0.out || { echo "proto failures"; exit 1; }
NO_BENCH=1 bash scripts/gpu_round.sh || exit 1
fi
OUT=gpurun_out/sq; mkdir -p $OUT
for c in ${CONFIGS:-c3 c4}; do
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
    tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' _)
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/${c}_$tag -o run --output-format csv -- python bench.py --full-line --no-host-path --config $c --steps 2 --warmup 1 --settle 0 --no-cpu-baseline --no-extra > $OUT/${c}_$tag.log 2>&1 || { echo "pmc $c $tag failed"; tail -5 $OUT/${c}_$tag.log; exit 1; }
    python scripts/pmc_insts.py $OUT/${c}_$tag vec_tile > $OUT/${c}_$tag.txt
    rm -rf $OUT/${c}_$tag
  done
done
echo ok
