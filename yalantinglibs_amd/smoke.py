"""One small invocation of the hot path on cuda:0, checked against the
reference's own bytes (tests/golden fixtures) and the CPU oracle."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import _capi as C
from . import layout as LY
from . import struct_pack as SP
from . import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _fixture(name):
    with open(os.path.join(GOLD, "manifest.json")) as f:
        ent = {e["name"]: e for e in json.load(f)}[name]
    with open(os.path.join(GOLD, ent["file"]), "rb") as f:
        return ent, f.read()


def _check_case(name):
    ent, wire = _fixture(name)
    cd = SP.Codec(LY.case_layout(ent["case"]), device="cuda:0")
    _, recs, heaps = synth.make_batch(ent["case"], ent["n"], ent["seed"], ent["param"])
    dev = torch.device("cuda:0")
    r = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8)
                         .reshape(ent["n"], cd.L.stride).copy()).to(dev)
    hs = [torch.from_numpy(h.view(np.uint8).copy()).to(dev) for h in heaps]
    out, _ = cd.serialize(SP.RecordBatch(cd.L, r, hs), SP.MODE_VECTOR)
    got = out.cpu().numpy().tobytes()
    assert got == wire, f"{name}: encode differs from the reference fixture"
    # the oracle agrees too (checker only)
    o = C.load_oracle()
    assert o is not None
    res, back, _ = cd.deserialize(out, SP.MODE_VECTOR)
    assert res.errc == 0 and res.count == ent["n"] and res.consumed == len(wire)
    assert back.recs.cpu().numpy().tobytes() == r.cpu().numpy().tobytes()
    for k, h in enumerate(hs):
        assert torch.equal(back.heaps[k][:h.numel()], h)
    return len(wire)


def run():
    assert torch.cuda.is_available(), "smoke() needs a GPU"
    C.load_codec()
    n1 = _check_case("rec64_A_n1000_p0_default")
    n2 = _check_case("recs_A_n300_p48_default")
    n3 = _check_case("outer_A_n100_p16_default")
    torch.cuda.synchronize()
    print(json.dumps({"smoke": "ok", "bytes": [n1, n2, n3]}))
