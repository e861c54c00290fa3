import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np, torch
import spk_helpers as H
from yalantinglibs_amd import _capi as C, struct_pack as SP, synth, layout as LY
for case in ("fv", "fv32", "fve", "var"):
    cd = SP.Codec(LY.case_layout(case))
    for n in (3, 100, 5000):
        _, recs, heaps = synth.make_batch(case, n, 0x2E80, 8)
        recs = np.zeros_like(recs); heaps = [np.zeros_like(h) for h in heaps]
        exp, _, _ = H.oracle_encode(cd.L, C.SPK_MODE_VECTOR, recs, heaps)
        w = torch.from_numpy(np.frombuffer(exp, np.uint8).copy()).cuda()
        res, back, _ = cd.deserialize(w, C.SPK_MODE_VECTOR)
        got = back.recs.cpu().numpy().reshape(-1)
        want = np.ascontiguousarray(recs).view(np.uint8).reshape(-1)
        d = np.nonzero(got != want)[0]
        print(case, n, "errc", res.errc, "count", res.count, "ndiff", len(d),
              "offs mod stride", sorted(set((d % cd.L.stride).tolist()))[:16], "vals", sorted(set(got[d].tolist()))[:8], flush=True)
