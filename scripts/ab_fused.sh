set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "SPK_FUSED=0" "SPK_FUSED=1" "SPK_FUSED=1 SPK_TILE_DBG=1024" "SPK_FUSED=1 SPK_TILE_DBG=2048" "SPK_FUSED=1 SPK_TILE_DBG=3072"; do
  for c in c3 c4; do
    env $v timeout -k 10 300 python bench.py --full-line --no-host-path --config $c --steps 10 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/ab_$c.log 2>&1 || { echo "fail $v $c"; tail -5 gpurun_out/ab_$c.log; exit 1; }
    python - $c "$v" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/ab_{sys.argv[1]}.log').read().strip().splitlines()[-1])
k=d['kernels']
print(sys.argv[2], sys.argv[1], 'decode', d['phase_ms'].get('decode'), {n: round(v['ms_per_step'],4) for n,v in k.items() if 'tile' in n or 'big' in n})
PY
  done
done
