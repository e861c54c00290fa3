"""Diagnostic: vector-decode re-verification worklist sizes (VCtl.wl_n) for
C3/C4 at full size, read back from the codec workspace after one decode."""
import struct
import sys

import torch

sys.path.insert(0, ".")
from yalantinglibs_amd import layout as LY
from yalantinglibs_amd import struct_pack as SP

for case, n, p, seed in (("recs", 10_000_000, 48, 0x5EED0003), ("outer", 10_000_000, 16, 0x5EED0004)):
    cd = SP.Codec(LY.case_layout(case))
    b = SP.synth_batch(cd, case, n, seed, p)
    wire, _ = cd.serialize(b)
    elems = [int(h.numel()) // sp.elem.size for h, sp in zip(b.heaps, cd.L.dev.spans)]
    dec = cd.alloc_batch(n, elems)
    cd.deserialize_to(dec, wire)
    torch.cuda.synchronize()
    ctl = cd._ws[2048:2048 + 128].cpu().numpy().tobytes()
    nch = struct.unpack_from("<Q", ctl, 16)[0]
    wl = struct.unpack_from("<7I", ctl, 72)
    unver, term, ovf = struct.unpack_from("<III", ctl, 60)
    print(case, "chunks", nch, "wl_n", wl, "n_unver", unver, flush=True)
