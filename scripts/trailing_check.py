"""VECTOR decode of a message followed by other bytes: the reference decodes
the message and reports consume_len = its length (struct_pack.hpp:343-357)."""
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
rng = np.random.default_rng(5)
for case, n, param in [("recs", 5000, 48), ("outer", 3000, 16), ("monster", 300, 20)]:
    cd = codec_for(case)
    L, recs, heaps = synth.make_batch(case, n, 0xC0FFEE + n, param)
    out, _ = cd.serialize(to_dev(cd, recs, heaps), C.SPK_MODE_VECTOR)
    m = out.cpu().numpy().tobytes()
    for tail_kind in ["zeros", "random", "copy"]:
        for tl in [7, 5000, 100000]:
            tail = (bytes(tl) if tail_kind == "zeros" else
                    bytes(rng.integers(0, 256, tl, dtype=np.uint8)) if tail_kind == "random" else
                    (m * (tl // len(m) + 1))[:tl])
            buf = torch.from_numpy(np.frombuffer(m + tail, np.uint8).copy()).cuda()
            res, back, _ = cd.deserialize(buf, C.SPK_MODE_VECTOR)
            ok = (res.errc == 0 and res.count == n and res.consumed == len(m) and
                  back.recs[:n].cpu().numpy().tobytes() ==
                  np.ascontiguousarray(recs).view(np.uint8).tobytes())
            print(case, tail_kind, tl, "ok" if ok else f"BAD errc={res.errc} count={res.count} "
                  f"consumed={res.consumed} len={len(m)}", flush=True)
