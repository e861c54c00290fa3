"""Which path decodes a compatible-member VECTOR message: the tile passes
(launch_compat_tiles) or the one-lane walk behind them. Prints the per-kernel
times of one decode per case (the walk's kernels leave at once when the tile
passes were clean) and checks the round trip."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import spk_helpers as H  # noqa: E402
from yalantinglibs_amd import _capi as C  # noqa: E402
from yalantinglibs_amd import synth  # noqa: E402
from test_gpu_parity import codec_for, to_dev  # noqa: E402

C.load_codec()
for case, n, param in [("cmp", 5000, 48), ("cmpg", 3000, 16), ("cmpnew", 20000, 8),
                       ("cmp", 200000, 16), ("cmpg", 200000, 16)]:
    cd = codec_for(case)
    L, recs, heaps = synth.make_batch(case, n, 0xC0FFEE + n, param)
    out, _ = cd.serialize(to_dev(cd, recs, heaps), C.SPK_MODE_VECTOR)
    cd.deserialize(out, C.SPK_MODE_VECTOR)  # (warm-up)
    torch.cuda.synchronize()
    C.trace_reset()
    C.trace_enable(True)
    res, back, _ = cd.deserialize(out, C.SPK_MODE_VECTOR)
    torch.cuda.synchronize()
    tr = C.trace_read()
    C.trace_enable(False)
    ok = (res.errc == 0 and res.count == n and
          back.recs[:n].cpu().numpy().tobytes() == np.ascontiguousarray(recs).view(np.uint8).tobytes())
    tot = sum(ms for _, ms in tr.values())
    top = sorted(((ms, k.split("(")[0][-28:]) for k, (l, ms) in tr.items()), reverse=True)[:6]
    serial = [round(ms, 4) for k, (l, ms) in tr.items() if "nest_vec_serial" in k]
    print(case, n, "ok" if ok else "MISMATCH", "wire", out.numel(), "total ms", round(tot, 4),
          "nest_vec_serial", serial, [(round(a, 4), b) for a, b in top], flush=True)
