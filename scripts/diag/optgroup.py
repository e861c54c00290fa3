"""Diagnose the VECTOR decode of optional groups into garbage-filled outputs:
records {int32; optional<string>; optional<Inner>; optional<vector<int32>>;
optional<RecS>} (the C++ unique_ptr test's shape) vs the oracle, field by field."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np, torch
import spk_helpers as H
from yalantinglibs_amd import _capi as C, struct_pack as SP, schema as S, synth, layout as LY
UP = S.Struct("UP", [("id", S.int32), ("s", S.Optional(S.String())), ("p", S.Optional(synth.Inner)),
                     ("v", S.Optional(S.Vector(S.int32))), ("r", S.Optional(synth.RecS))])
L = LY.make_layout(UP)
cd = SP.Codec(L)
rng = np.random.default_rng(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
recs = np.zeros(n, L.dev.dtype)
recs["id"] = rng.integers(-1000, 1000, n)
heaps = [[], [], [], []]
offs = [0, 0, 0, 0]
def put(k, arr, field_n, field_off, i, esz):
    recs[field_n][i] = len(arr) // esz
    recs[field_off][i] = offs[k]
    offs[k] += len(arr) // esz
    heaps[k].append(arr)
for i in range(n):
    if i % 3:
        recs["s.has"][i] = 1
        put(0, rng.integers(97, 120, i % 17).astype(np.uint8).tobytes(), "s.value.n", "s.value.off", i, 1)
    if i % 2:
        put(1, np.array([i, 0], np.int32).tobytes(), "p.n", "p.off", i, 8)
    if i % 5 != 1:
        recs["v.has"][i] = 1
        put(2, np.full(i % 9, i, np.int32).tobytes(), "v.value.n", "v.value.off", i, 4)
    if i % 4 == 0:
        recs["r.has"][i] = 1
        recs["r.value.id"][i] = i
        recs["r.value.v"][i] = i * 0.5
        put(3, rng.integers(97, 120, i % 20).astype(np.uint8).tobytes(), "r.value.name.n", "r.value.name.off", i, 1)
hp = [np.frombuffer(b"".join(h) or b"\0", np.uint8).copy() for h in heaps]
exp, _, _ = H.oracle_encode(L, C.SPK_MODE_VECTOR, recs, hp)
w = torch.from_numpy(np.frombuffer(exp, np.uint8).copy()).cuda()
for fill in (0, 0xAB):
    out = cd.alloc_batch(n + 10, [len(h) // max(1, sp.elem.size) + 8 for h, sp in zip(hp, L.dev.spans)])
    out.recs.fill_(fill)
    for h in out.heaps:
        h.fill_(fill)
    cd.deserialize_to(out, w, C.SPK_MODE_VECTOR)
    res = cd.result()
    got = out.recs[:n].cpu().numpy().view(L.dev.dtype).reshape(-1)
    print("fill", hex(fill), "errc", res.errc, "count", res.count, "consumed", res.consumed, len(exp),
          "repaired", res.tiles_repaired, "seq", res.tiles_sequential)
    bad = {}
    for f in L.dev.dtype.names:
        head = f.split(".")[0]
        if head in ("s", "v", "r") and not f.endswith(".has"):
            mask = recs[head + ".has"] != 0
        elif head == "p":
            mask = np.ones(n, bool) if f == "p.n" else recs["p.n"] != 0
        else:
            mask = np.ones(n, bool)
        diff = np.nonzero((got[f] != recs[f]) & mask)[0]
        if len(diff):
            bad[f] = (len(diff), diff[:8].tolist(), got[f][diff[:4]].tolist(), recs[f][diff[:4]].tolist())
    print("  bad fields:", bad if bad else "none")
