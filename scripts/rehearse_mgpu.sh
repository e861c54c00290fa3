#!/bin/bash
# 2 ranks on one GPU over gloo: exercises bench.py's N>1 path incl. concat_*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --records 2000000 --steps 3 --warmup 1 \
  --settle 0 --concat-records 1000000 > gpurun_out/mg.log 2>&1 || { tail -30 gpurun_out/mg.log; exit 1; }
tail -1 gpurun_out/mg.log | python -c "import json,sys; s=sys.stdin.read(); d=json.loads(s); print(len(s), d['value']); print(json.dumps(d.get('concat')))"
