#!/bin/bash
# the C++ protocol / front-end test next to the reference, alone (its stderr kept)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for z in ${ZS:-0}; do
SPK_GPU_ZERO_ALLOC=$z timeout -k 10 300 oracle/_ref/test_gpu_protocol > gpurun_out/proto_$z.out 2> gpurun_out/proto_$z.err; rc=$?
echo "ZERO=$z rc=$rc"; tail -3 gpurun_out/proto_$z.out; grep -v "^section" gpurun_out/proto_$z.err | head -20
done
