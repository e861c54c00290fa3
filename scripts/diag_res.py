"""K1 resolution statistics from an -DSPK_RESDBG=1 build (SPK_CODEC_LIB):
tiles whose lanes re-walked, total rounds, lanes that missed (diagnostic)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from yalantinglibs_amd import layout as LY, struct_pack as SP

for case, n, param in (("recs", 10_000_000, 48), ("outer", 10_000_000, 16)):
    cd = SP.Codec(LY.case_layout(case), device="cuda:0")
    b = SP.synth_batch(cd, case, n, 0x5EED0003 if case == "recs" else 0x5EED0004, param)
    wire, _ = cd.serialize(b, SP.MODE_VECTOR)
    out = cd.alloc_batch(n, [int(h.numel()) // sp.elem.size for h, sp in zip(b.heaps, cd.L.dev.spans)])
    cd.deserialize_to(out, wire, SP.MODE_VECTOR)
    r = cd.result()
    torch.cuda.synchronize()
    ws = cd._ws[:4096].cpu().numpy()
    f = np.frombuffer(ws[2048 + 1280:2048 + 1280 + 400].tobytes(), np.uint64)
    # FCtl: broken[4], unresolved, seq, njobs, term_tile, term_pos, end_pos, total,
    # htot[8], entry0, nglob, range|last, stot[8], nlist[4]
    broken, seq = f[0:4], f[5]
    nlist = f[4 + 1 + 1 + 1 + 1 + 1 + 1 + 1 + 8 + 1 + 1 + 1 + 8:][:4]
    ntiles = wire.numel() // 16384 + 1
    print(case, "tiles", ntiles, "errc", r.errc, "tiles needing rounds", int(broken[3]),
          "rounds", int(nlist[3]), "missed lanes", int(seq), "repaired", r.tiles_repaired, flush=True)
