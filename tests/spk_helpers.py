"""Shared test helpers: golden fixtures and the CPU oracle (checker only)."""
from __future__ import annotations

import ctypes as ct
import hashlib
import json
import os

import numpy as np

from yalantinglibs_amd import _capi as C
from yalantinglibs_amd import layout as LY
from yalantinglibs_amd import schema as S
from yalantinglibs_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

CONF = {"default": S.DEFAULT, "typeinfo": S.ENABLE_TYPE_INFO,
        "nometa": S.DISABLE_ALL_META_INFO}


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def errs():
    with open(os.path.join(GOLDEN, "errs.json")) as f:
        return json.load(f)


def read_fixture(ent):
    with open(os.path.join(GOLDEN, ent["file"]), "rb") as f:
        wire = f.read()
    lens = None
    if ent["mode"] == "B":
        with open(os.path.join(GOLDEN, ent["name"] + ".lens"), "rb") as f:
            lens = np.frombuffer(f.read(), dtype=np.uint64)
    return wire, lens


def sha256(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def layout_for(ent):
    return LY.case_layout(ent["case"], CONF[ent["conf"]])


def mode_of(ent):
    return C.SPK_MODE_VECTOR if ent["mode"] == "A" else C.SPK_MODE_MESSAGES


def batch_for(ent):
    return synth.make_batch(ent["case"], ent["n"], ent["seed"], ent["param"])


def _ptr(a):
    return ct.c_void_p(a.ctypes.data) if a is not None and a.size else ct.c_void_p(0)


# ---- oracle wrappers (CPU checker) -----------------------------------------
def oracle_encode(L, mode, recs, heaps):
    o = C.load_oracle()
    n = len(recs)
    plan = C.spk_plan_t()
    hp = (ct.c_void_p * max(len(heaps), 1))(*[h.ctypes.data for h in heaps])
    rc = o.spko_plan(L.ptr, mode, n, _ptr(recs), hp, ct.byref(plan))
    assert rc == 0, rc
    out = np.zeros(max(plan.total_bytes, 1), np.uint8)
    offs = np.zeros(n + 1, np.uint64)
    written = ct.c_uint64(0)
    rc = o.spko_encode(L.ptr, mode, n, _ptr(recs), hp, _ptr(out), out.size,
                       _ptr(offs), ct.byref(written))
    assert rc == 0, rc
    return out[:plan.total_bytes].tobytes(), offs, plan


def oracle_decode(L, mode, wire: bytes, offsets=None, n_msgs=0, rec_cap=None,
                  heap_caps=None):
    o = C.load_oracle()
    w = np.frombuffer(wire, np.uint8) if len(wire) else np.zeros(1, np.uint8)
    if rec_cap is None:
        rec_cap = max(len(wire), 1) if mode == C.SPK_MODE_VECTOR else max(n_msgs, 1)
    recs = np.zeros(rec_cap, L.dev.dtype)
    heaps, caps = [], []
    wcaps = S.heap_caps_for_wire(L.dev, len(wire), rec_cap)
    for sp, wc in zip(L.dev.spans, wcaps):
        cap = heap_caps or max(wc, len(wire) // max(sp.elem.size, 1) + 1)
        heaps.append(np.zeros(cap * sp.elem.size, np.uint8))
        caps.append(cap)
    hp = (ct.c_void_p * max(len(heaps), 1))(*[h.ctypes.data for h in heaps])
    hc = (ct.c_uint64 * max(len(caps), 1))(*caps)
    res = C.spk_dresult_t()
    errc = np.zeros(max(n_msgs, 1), np.int32)
    offs = offsets if offsets is not None else np.zeros(1, np.uint64)
    rc = o.spko_decode(L.ptr, mode, _ptr(w), len(wire), _ptr(offs), n_msgs,
                       _ptr(recs), rec_cap, hp, hc, ct.byref(res), _ptr(errc))
    assert rc == 0, rc
    return res, recs, heaps, errc


def lens_to_offsets(lens):
    offs = np.zeros(len(lens) + 1, np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64))
    return offs


def records_equal(L, a, b, heaps_a, heaps_b, heap_used=None):
    """Compare decoded records/heaps with the synth inputs (canonical heap).
    heap_used: elements in use per heap (the decode result); needed for the
    heaps of ARRAY elements, whose counts are not in the top-level records."""
    if L.dev.trivial:
        return a.tobytes() == b.tobytes()
    ok = a.tobytes() == b.tobytes()
    for k, sp in enumerate(L.dev.spans):
        if heap_used is not None:
            n = int(heap_used[k])
        else:
            n = int(a[sp.path + ".n"].astype(np.uint64).sum())
        used = n * sp.elem.size
        ok = ok and heaps_a[k][:used].tobytes() == heaps_b[k][:used].tobytes()
        ok = ok and len(heaps_b[k]) == used
    return ok


# ---- associative containers: the reference's insertion semantics ------------
def _assoc_key(L, k, sub_rec, heaps, elem_bytes):
    """Sort key of one element of top-level span k (a map's pair: its first;
    a set: the element): signed integers by value, strings bytewise."""
    sp = L.dev.spans[k]
    t = sp.elem
    key_t = getattr(getattr(L.rtype, "fields", None) and
                    dict(L.rtype.fields).get(sp.path), "key", None)
    kt = key_t if key_t is not None else getattr(dict(L.rtype.fields).get(sp.path), "elem", None)
    if sp.sub is None:  # trivially serializable element bytes: the key's bytes first
        return int.from_bytes(elem_bytes[:kt.size], "little", signed=kt.npdt[1] == "i")
    name = "first" if sp.kind.endswith("map") else "value"
    if isinstance(kt, S.String):
        kk = [q for q, s2 in enumerate(L.dev.spans) if s2.path == f"{sp.path}[].{name}"][0]
        n, o = int(sub_rec[name + ".n"]), int(sub_rec[name + ".off"])
        return bytes(heaps[kk][o:o + n])
    return int(sub_rec[name])


def normalize_assoc(L, recs, heaps):
    """What the reference's decode builds from a map / set on the wire
    (unpacker.hpp:983-1122): a map / set keeps the first of repeated keys
    (try_emplace / emplace), a multi container all of them, and iteration is
    in key order (equal keys in insertion order). Our decode keeps the wire
    order (the record model); this re-orders each top-level ordered
    associative container's elements the same way so that re-encoding gives
    the reference's canonical bytes. Returns new (recs, heaps)."""
    recs = recs.copy()
    heaps = [np.array(h, np.uint8, copy=True) for h in heaps]
    for k, sp in enumerate(L.dev.spans):
        if not sp.kind or "[]" in sp.path:
            continue
        assert sp.kind in ("map", "multimap", "set", "multiset"), sp.kind
        esz = sp.elem.size
        out = bytearray()
        for i in range(len(recs)):
            n, o = int(recs[i][sp.path + ".n"]), int(recs[i][sp.path + ".off"])
            elems = [bytes(heaps[k][(o + j) * esz:(o + j + 1) * esz]) for j in range(n)]
            subs = ([np.frombuffer(e, sp.sub.dtype)[0] for e in elems] if sp.sub is not None
                    else [None] * n)
            keys = [_assoc_key(L, k, sr, heaps, e) for sr, e in zip(subs, elems)]
            order = sorted(range(n), key=lambda j: keys[j])  # stable
            if not sp.kind.startswith("multi"):
                seen, keep = set(), []
                for j in range(n):  # the first of repeated keys stays
                    if keys[j] not in seen:
                        seen.add(keys[j])
                        keep.append(j)
                order = sorted(keep, key=lambda j: keys[j])
            recs[sp.path + ".n"][i] = len(order)
            recs[sp.path + ".off"][i] = len(out) // esz
            out += b"".join(elems[j] for j in order)
        heaps[k] = np.frombuffer(bytes(out), np.uint8).copy() if out else np.zeros(0, np.uint8)
    return recs, heaps


def has_assoc(L):
    return any(sp.kind and "[]" not in sp.path for sp in L.dev.spans)
