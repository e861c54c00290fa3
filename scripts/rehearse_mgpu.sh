#!/bin/bash
# 2 ranks on one GPU over gloo: `bench.py --gpus 2` launches its own ranks and
# exercises the N>1 line (C2 headline, C4 / C5 per-rank entries, concat_*)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --records 2000000 --steps 3 \
  --warmup 1 --settle 0 --concat-records 1000000 --extra-steps 3 > gpurun_out/mg.log 2> gpurun_out/mg.err \
  || { tail -30 gpurun_out/mg.err; exit 1; }
tail -1 gpurun_out/mg.log | python -c "import json,sys; s=sys.stdin.read(); d=json.loads(s); print(len(s), d['n_gpus'], d['value']); print(json.dumps(d.get('extra'))); print(json.dumps(d.get('concat')))"
