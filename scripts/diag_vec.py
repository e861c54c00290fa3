"""Diagnostics for the speculative vector decode: unverified chunk count and
a few (E_{c-1}, P_c) pairs that failed to meet."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from yalantinglibs_amd import layout as LY, struct_pack as SP, _capi as C

case, n, param = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
seed = {"recs": 0x5EED0003, "outer": 0x5EED0004}[case]
cd = SP.Codec(LY.case_layout(case))
b = SP.synth_batch(cd, case, n, seed, param)
wire, _ = cd.serialize(b, SP.MODE_VECTOR)
elems = [int(h.numel()) // sp.elem.size for h, sp in zip(b.heaps, cd.L.dev.spans)]
dec = cd.alloc_batch(n, elems)
cd.deserialize_to(dec, wire, SP.MODE_VECTOR)
torch.cuda.synchronize()
ws = cd._ws.cpu().numpy()
ctl = ws[2048:2048 + 80]
p0, nn, nch = [int(x) for x in np.frombuffer(ctl[:24].tobytes(), np.uint64)]
w, errc, lp, nunv, term, ovf = [int(x) for x in np.frombuffer(ctl[48:72].tobytes(), np.uint32)]
print(f"p0={p0} n={nn} nchunks={nch} w={w} errc={errc} lp={lp} n_unver={nunv} term={term} overflow={ovf}")
# layout offsets (mirror vec_ws_layout)
S, EXT = 2048, 16
nchc = wire.numel() // S + 2
off = 4096
def take(nb):
    global off
    o = off; off += (nb + 255) & ~255; return o
oP = take(nchc * lp * 2); oPn = take(nchc * 4); oE = take(nchc * EXT * 4); oEn = take(nchc * 4)
ofl = take(nchc * 4); oT = take(nchc * 8); ocnt = take(nchc * 4); obase = take(nchc * 8); ounv = take(nchc * 4)
Pn = ws[oPn:oPn + nch * 4].view(np.uint32)
En = ws[oEn:oEn + nch * 4].view(np.uint32)
fl = ws[ofl:ofl + nch * 4].view(np.uint32)
unv = np.sort(ws[ounv:ounv + nunv * 4].view(np.uint32))
print("Pn stats", Pn.min(), Pn.mean(), Pn.max(), "En zero:", int((En == 0).sum()), "flags hist", np.bincount(fl)[:8])
print("first unverified:", unv[:20])
for c in unv[:3]:
    c = int(c)
    P = ws[oP + c * lp * 2: oP + (c * lp + Pn[c]) * 2].view(np.uint16).astype(np.int64) + c * S
    E = ws[oE + (c - 1) * EXT * 4: oE + ((c - 1) * EXT + En[c - 1]) * 4].view(np.uint32).astype(np.int64) + (c - 1) * S
    print("chunk", c, "E_prev", E[:16].tolist())
    print("        P", P[:20].tolist())
