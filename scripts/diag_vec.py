"""Diagnostics for the speculative vector decode (mirrors vec_ws_layout in
spk_var.hip): how often a chunk's speculative walk misses the true path."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from yalantinglibs_amd import layout as LY, struct_pack as SP

S, EXT = int(sys.argv[4]) if len(sys.argv) > 4 else 256, int(sys.argv[5]) if len(sys.argv) > 5 else 4
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
wl = np.frombuffer(ws[2048 + 72:2048 + 72 + 9 * 4].tobytes(), np.uint32)
print("worklist per round:", wl.tolist())
print(f"p0={p0} n={nn} nchunks={nch} w={w} errc={errc} lp={lp} n_unver={nunv} term={term} overflow={ovf}")
nchc = wire.numel() // S + 2
off = 4096
def take(nb):
    global off
    o = off; off += (nb + 255) & ~255; return o
oP = take(nchc * lp * 2); oPn = take(nchc * 4); oE = take(nchc * EXT * 4); oEn = take(nchc * 4)
ofl = take(nchc * 4); oT = take(nchc * 8); ocnt = take(nchc * 4); obase = take(nchc * 8)
ounv = take(2 * nchc * 4); oex = take(nchc * 8); oused = take(nchc * 8)
Pn = ws[oPn:oPn + nch * 4].view(np.uint32)
En = ws[oEn:oEn + nch * 4].view(np.uint32)
fl = ws[ofl:ofl + nch * 4].view(np.uint32)
P = ws[oP:oP + nch * lp * 2].view(np.uint16).reshape(nch, lp).astype(np.int64)
E = ws[oE:oE + nch * EXT * 4].view(np.uint32).reshape(nch, EXT).astype(np.int64)
used = ws[oused:oused + nch * 8].view(np.uint64)
cs = p0 + np.arange(nch, dtype=np.int64) * S
specentry = np.where(En[:-1] > 0, cs[:-1] + E[:-1, 0], -1)
first = np.where(Pn[1:] > 0, cs[1:] + P[1:, 0], -2)
print("Pn mean", Pn.mean(), "empty P:", int((Pn == 0).sum()), "flags hist", np.bincount(fl)[:8])
miss = first != specentry
print(f"round-0 P[0]!=E_prev[0]: {int(miss.sum())} of {nch-1} ({100*miss.mean():.2f}%)")
truth = used[1:].astype(np.int64)
wrongE = specentry != truth
print(f"chunks whose spec entry was wrong (re-walked): {int(wrongE.sum())}")
bad = np.nonzero(miss)[0][:5] + 1
for c in bad:
    print("chunk", c, "cs", cs[c], "used", int(used[c]), "E_prev", (cs[c-1] + E[c-1, :En[c-1]]).tolist(), "P", (cs[c] + P[c, :Pn[c]]).tolist())
# chunks left for the sequential fixup (final worklist, parity kRounds & 1 = 0)
olist = ounv
fin = ws[olist:olist + int(wl[-1]) * 4].view(np.uint32)
exitp = ws[oex:oex + nch * 8].view(np.uint64)
print("fixup list:", fin.tolist())
for c in sorted(fin.tolist())[:6]:
    print("  chunk", c, "cs", cs[c], "used", int(used[c]), "exit_prev", int(exitp[c-1]), "exit", int(exitp[c]),
          "En_prev", int(En[c-1]), "E_prev", (cs[c-1] + E[c-1, :En[c-1]]).tolist(), "P", (cs[c] + P[c, :Pn[c]]).tolist(), "flags", int(fl[c]))
