"""K1 statistics (diagnostics build: SPK_CODEC_LIB=build_var/diag.so, built
with -DSPK_DIAG=1 -DSPK_K1_STATS=1; SPK_TILE_DBG=4096) on Var records whose
strings are random bytes, 0-2 B then 100-3000 B every 7th (tail=mixed), all
long (long) or from the first record on (uniform)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from yalantinglibs_amd import synth, struct_pack as SP  # noqa: E402
from yalantinglibs_amd import _capi as C  # noqa: E402
from yalantinglibs_amd import layout as LY  # noqa: E402
from yalantinglibs_amd import schema as S  # noqa: E402

WS_FCTL = 2048 + 1280


def main():
    tail = sys.argv[1] if len(sys.argv) > 1 else "mixed"
    case = sys.argv[2] if len(sys.argv) > 2 else "var"
    cd = SP.Codec(LY.case_layout(case, S.DEFAULT))
    rng = np.random.default_rng(29)
    n = 30000
    lens = rng.integers(0, 3, n)
    if tail == "long":
        lens[64:] = rng.integers(100, 3000, n - 64)
    elif tail == "mixed":
        lens[64::7] = rng.integers(100, 3000, len(lens[64::7]))
    else:
        lens[:] = rng.integers(100, 3000, n)
    _, recs, _ = synth.make_batch(case, n, 0x5EED000C, 16)
    fld = "s" if case == "var" else "name"
    recs[f"{fld}.n"] = lens
    recs[f"{fld}.off"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    heaps = [rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)]
    r = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).reshape(n, cd.L.stride)
                         .copy()).cuda()
    hs = [torch.from_numpy(h.copy()).cuda() for h in heaps]
    out, _ = cd.serialize(SP.RecordBatch(cd.L, r, hs), C.SPK_MODE_VECTOR)
    res, back, _ = cd.deserialize(out, C.SPK_MODE_VECTOR)
    torch.cuda.synchronize()
    ws = cd._ws.cpu().numpy()
    words = np.frombuffer(ws[WS_FCTL:WS_FCTL + 8 * 64].tobytes(), dtype=np.uint64)
    diag = words[34:42]
    ntiles = (out.numel() + 16383) // 16384
    names = ["round-lanes (x64)", "re-walks", "spec walks", "spec off-grid", "wrong spec lanes",
             "chunk0 cross-checks", "max tile cycles", "sum tile cycles"]
    print(f"{case} {tail}: {out.numel() / 1e6:.1f} MB, {ntiles} tiles, errc {res.errc}, "
          f"repaired {res.tiles_repaired}")
    for nm, v in zip(names, diag):
        print(f"  {nm:22s} {int(v):>14d}  per tile {int(v) / ntiles:12.1f}")


if __name__ == "__main__":
    main()
