#!/bin/bash
# The driver's default bench command (compact stdout line + detail file),
# then the gloo 2-rank rehearsal of the N>1 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default.err; exit 1; }
tail -c 5500 gpurun_out/bench_default.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('parsed ok', len(json.dumps(d)), d['value'], d['roofline']['frac'])"
[ -n "$NO_MG" ] || bash scripts/rehearse_mgpu.sh
