"""K1 statistics of the tile decoder on a synthetic VECTOR message
(SPK_TILE_DBG=4096, in a codec built with -DSPK_K1_STATS=1): speculative candidate walks, their failures, lanes whose
speculative start was wrong, resolution rounds and re-walks, chunk-0
cross-checks; tiles re-walked by the select passes.

    SPK_TILE_DBG=4096 python scripts/diag_tiles.py monster 1000000 20
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from yalantinglibs_amd import synth, struct_pack as SP  # noqa: E402
from yalantinglibs_amd import _capi as C  # noqa: E402
from yalantinglibs_amd import layout as LY  # noqa: E402
from yalantinglibs_amd import schema as S  # noqa: E402

WS_FCTL = 2048 + 1280


def main():
    case, n, param = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    cd = SP.Codec(LY.case_layout(case, S.DEFAULT))  # default sp_config
    _, recs, heaps = synth.make_batch(case, n, 0xD1A6, param)
    r = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).reshape(n, cd.L.stride)
                         .copy()).cuda()
    hs = [torch.from_numpy(np.ascontiguousarray(h).view(np.uint8).copy()).cuda() for h in heaps]
    out, _ = cd.serialize(SP.RecordBatch(cd.L, r, hs), C.SPK_MODE_VECTOR)
    res, back, _ = cd.deserialize(out, C.SPK_MODE_VECTOR)
    torch.cuda.synchronize()
    ws = cd._ws.cpu().numpy()
    # FCtl: broken[4], unresolved, seq, njobs, term_tile, term_pos, end_pos, total,
    # htot[8], entry0, nglob, range/last, stot[8], nlist[4], diag[8]
    words = np.frombuffer(ws[WS_FCTL:WS_FCTL + 8 * 64].tobytes(), dtype=np.uint64)
    diag = words[34:42]
    ntiles = (out.numel() + 16383) // 16384
    names = ["round-lanes (x64)", "re-walks", "spec walks", "spec off-grid", "wrong spec lanes",
             "chunk0 cross-checks", "max tile cycles", "sum tile cycles"]
    print(f"{case} n={n} wire={out.numel() / 1e6:.1f} MB tiles={ntiles} errc={res.errc} "
          f"repaired={res.tiles_repaired} sequential={res.tiles_sequential}")
    for k, nm in enumerate(names):
        print(f"  {nm:20s} {int(diag[k]):12d}  per tile {int(diag[k]) / ntiles:9.2f}")


if __name__ == "__main__":
    main()
