"""Decode one golden fixture and print the decode result and the per-chunk
state of the speculative vector decode (layout mirrors vec_ws_layout)."""
import json, sys
import numpy as np
import torch
sys.path.insert(0, ".")
from yalantinglibs_amd import layout as LY, struct_pack as SP, _capi as C

name = sys.argv[1] if len(sys.argv) > 1 else "recs_A_n300_p48_default"
S, EXT = 256, 4
ent = {e["name"]: e for e in json.load(open("tests/golden/manifest.json"))}[name]
wire_b = open("tests/golden/" + ent["file"], "rb").read()
cd = SP.Codec(LY.case_layout(ent["case"]), device="cuda:0")
wire = torch.from_numpy(np.frombuffer(wire_b, np.uint8).copy()).cuda()
res, back, _ = cd.deserialize(wire, SP.MODE_VECTOR)
print("res errc", res.errc, "count", res.count, "consumed", res.consumed, "len", len(wire_b),
      "heap_used", list(res.heap_used)[:2], "n", ent["n"])
ws = cd._ws.cpu().numpy()
ctl = ws[2048:2048 + 128]
p0, nn, nch, dl, endp, tot = [int(x) for x in np.frombuffer(ctl[:48].tobytes(), np.uint64)]
w, errc, lp, nunv, term, ovf = [int(x) for x in np.frombuffer(ctl[48:72].tobytes(), np.uint32)]
print(f"p0={p0} n={nn} nch={nch} data_len={dl} end_pos={endp} total={tot} w={w} errc={errc} lp={lp} term={term} ovf={ovf}")
nchc = len(wire_b) // S + 2
ns = len(cd.L.dev.spans)
off = 4096
def take(nb):
    global off
    o = off; off += (nb + 255) & ~255; return o
oP = take(nchc * lp * 2); oPn = take(nchc * 4); oE = take(nchc * EXT * 4); oEn = take(nchc * 4)
ofl = take(nchc * 4); oT = take(nchc * 8); ocnt = take(nchc * 4); obase = take(nchc * 8)
owl = take(2 * nchc * 4); oex = take(nchc * 8); oused = take(nchc * 8); odirty = take(2 * nchc * 4)
omj = take(nchc * 4); opsum = take(ns * nchc * 8); ohs = take(ns * nchc * 8); ohb = take(ns * nchc * 8)
oscan = take((nchc // 4096 + 2) * 8); otot = take(16 * 8)
g = lambda o, dt, cnt: np.frombuffer(ws[o:o + cnt * np.dtype(dt).itemsize].tobytes(), dt)
print("cnt ", g(ocnt, np.uint32, nch).tolist())
print("base", g(obase, np.uint64, nch).tolist())
print("psum", g(opsum, np.uint64, nch).tolist())
print("hs  ", g(ohs, np.uint64, nch).tolist())
print("hb  ", g(ohb, np.uint64, nch).tolist())
print("mj  ", [(int(x) >> 16, int(x) & 0xFFFF) for x in g(omj, np.uint32, nch)])
print("flags", g(ofl, np.uint32, nch).tolist())
print("tot", g(otot, np.uint64, 4).tolist())
