"""Summarise scripts/ab_cfg.sh logs: per config and variant, ms/step and the
per-launch time of every kernel (mean over the repeats)."""
import collections
import json
import os
import sys

d = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(os.listdir(d)):
    if not f.endswith(".log"):
        continue
    cfg, var = f[:-4].split("_", 1)
    var = var.rsplit("_", 1)[0]
    for line in open(os.path.join(d, f)):
        if line.startswith("{"):
            rows[(cfg, var)].append(json.loads(line))
for (cfg, var), ls in sorted(rows.items()):
    ms = sum(x["ms_per_step"] for x in ls) / len(ls)
    ks = collections.defaultdict(float)
    for x in ls:
        for k, v in x["kernels"].items():
            ks[k] += v["ms_per_step"] / len(ls)
    top = sorted(ks.items(), key=lambda kv: -kv[1])[:5]
    print(f"{cfg:5s} {var:10s} {ms:8.4f} ms/step  " +
          "  ".join(f"{k.split('<')[0][:18]}={v:.4f}" for k, v in top))
