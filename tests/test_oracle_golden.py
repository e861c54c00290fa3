"""CPU: pin the oracle and the host type model against the REFERENCE's bytes.

Fixtures in tests/golden/ were produced by oracle/_ref/golden_gen, compiled
from the unmodified reference headers (tests/golden/make_golden.py). This
suite establishes that our CPU restatement (oracle/spk_oracle.c) and type
model (yalantinglibs_amd/schema.py) reproduce them, so that the GPU parity
tests may use the oracle as the checker at sizes/inputs the fixtures do not
cover.
"""
import numpy as np
import pytest

import spk_helpers as H
from yalantinglibs_amd import _capi as C
from yalantinglibs_amd import schema as S
from yalantinglibs_amd import synth

KAT_TYPES = {
    "Rec64": synth.Rec64, "vector<Rec64>": S.Vector(synth.Rec64),
    "RecS": synth.RecS, "vector<RecS>": S.Vector(synth.RecS),
    "Inner": synth.Inner, "Outer": synth.Outer, "vector<Outer>": S.Vector(synth.Outer),
    "Pad": synth.Pad, "vector<Pad>": S.Vector(synth.Pad),
    "Mixed": synth.Mixed, "vector<Mixed>": S.Vector(synth.Mixed),
    "rect<int>": synth.RectInt, "vector<rect<int>>": S.Vector(synth.RectInt),
    "rpc::point": synth.Point, "rpc::rect": synth.RpcRect,
    "vector<rpc::rect>": S.Vector(synth.RpcRect),
    "person": synth.Person, "vector<person>": S.Vector(synth.Person),
    "vector<int32_t>": S.Vector(S.int32), "string": S.String(), "int32_t": S.int32,
    "req_header": synth.ReqHeader, "resp_header": synth.RespHeader,
    "monostate": S.Monostate(), "array<int16_t,3>": S.Array(S.int16, 3),
    "vector<string>": S.Vector(S.String()),
    "ResponseCode": synth.ResponseCode, "AliMessage": synth.AliMessage,
    "ValidateRequest": synth.ValidateRequest, "vector<ValidateRequest>": S.Vector(synth.ValidateRequest),
    "Exp": synth.Exp, "vector<Exp>": S.Vector(synth.Exp),
    "expected<void,int32_t>": S.Expected(S.Monostate(), S.int32), "CmpG": synth.CmpG,
    "Vec3": synth.Vec3, "Weapon": synth.Weapon, "Monster": synth.Monster,
    "vector<Monster>": S.Vector(synth.Monster), "rect2<int32_t>": synth.Rect2,
    "Lists": synth.Lists, "Maps": synth.Maps, "vector<Maps>": S.Vector(synth.Maps),
    "map<int32_t,string>": S.Map(S.int32, S.String()),
    "unordered_multimap<int32_t,int32_t>": S.Map(S.int32, S.int32, multi=True, ordered=False),
    "pair<string,person>": S.Pair(S.String(), synth.CPerson),
    "complicated_object": synth.Cplx,
    "bitset<64>": S.Bitset(64), "bitset<128>": S.Bitset(128),
    "u16string": S.String(elem=S.char16), "u32string": S.String(elem=S.char32),
    "wstring": S.String(elem=S.wchar), "WideT": synth.WideT, "vector<WideT>": S.Vector(synth.WideT),
    "Wide": synth.Wide, "vector<Wide>": S.Vector(synth.Wide),
}


@pytest.mark.parametrize("name", sorted(KAT_TYPES))
def test_type_literal_and_code(name):
    k = H.kat()[name]
    t = KAT_TYPES[name]
    assert t.root_literal().hex() == k["literal"]
    assert t.code() == k["code"]


def test_tuple_and_fundamentals_codes():
    k = H.kat()
    assert S.get_type_code(S.int32, S.int32, S.int16) == k["<int32_t,int32_t,int16_t>"]["code"]
    fs = [S.uint8, S.uint16, S.uint32, S.uint64, S.int8, S.int16, S.int64,
          S.boolean, S.char, S.float32, S.float64]
    assert S.get_type_literal(*fs).hex() == k["fundamentals"]["literal"]
    fs = [S.int128, S.uint128, S.wchar, S.char16, S.char32]
    assert S.get_type_literal(*fs).hex() == k["wide fundamentals"]["literal"]
    assert S.get_type_code(*fs) == k["wide fundamentals"]["code"]


def test_size_literal():
    # get_size_literal (type_calculate.hpp:26-97)
    assert S.size_literal(0) == bytes([129])
    assert S.size_literal(126) == bytes([255])
    assert S.size_literal(127) == bytes([1, 130])
    assert S.size_literal(127 * 127) == bytes([1, 1, 130])


SMALL = [e for e in H.manifest() if "file" in e]
MEDIUM = [e for e in H.manifest() if "file" not in e and e["size_class"] == "small"]


@pytest.mark.parametrize("ent", SMALL, ids=[e["name"] for e in SMALL])
def test_oracle_encode_matches_reference(ent):
    L = H.layout_for(ent)
    wire, lens = H.read_fixture(ent)
    _, recs, heaps = H.batch_for(ent)
    got, offs, plan = H.oracle_encode(L, H.mode_of(ent), recs, heaps)
    assert len(got) == ent["wire_len"] == len(wire)
    assert got == wire
    if lens is not None:
        assert np.array_equal(np.diff(offs), lens)


@pytest.mark.parametrize("ent", SMALL, ids=[e["name"] for e in SMALL])
def test_oracle_decode_roundtrip_reference(ent):
    L = H.layout_for(ent)
    wire, lens = H.read_fixture(ent)
    _, recs, heaps = H.batch_for(ent)
    if ent["mode"] == "A":
        res, out, oh, _ = H.oracle_decode(L, C.SPK_MODE_VECTOR, wire)
        assert res.errc == 0
        assert res.count == ent["n"]
        assert res.consumed == len(wire)
    else:
        offs = H.lens_to_offsets(lens)
        res, out, oh, errc = H.oracle_decode(L, C.SPK_MODE_MESSAGES, wire, offs, ent["n"])
        assert res.errc == 0 and res.count == ent["n"]
        assert (errc[:ent["n"]] == 0).all()
    assert H.records_equal(L, out[:ent["n"]], recs, oh, heaps, res.heap_used)


@pytest.mark.parametrize("ent", MEDIUM, ids=[e["name"] for e in MEDIUM])
def test_oracle_encode_digest_medium(ent):
    L = H.layout_for(ent)
    _, recs, heaps = H.batch_for(ent)
    got, offs, _ = H.oracle_encode(L, H.mode_of(ent), recs, heaps)
    assert len(got) == ent["wire_len"]
    assert H.sha256(got) == ent["sha256"]
    if ent["mode"] == "B":
        assert H.sha256(np.diff(offs).astype(np.uint64).tobytes()) == ent["lens_sha256"]


ERRS = H.errs()


@pytest.mark.parametrize("base", ERRS, ids=[f"{b['case']}_{b['mode']}_{b['n']}_{b['conf']}"
                                            for b in ERRS])
def test_oracle_error_parity(base):
    """errc / consume_len / decoded value of mutated buffers == reference."""
    ent = dict(base)
    L = H.layout_for(ent)
    wire0 = bytes.fromhex(base["base"])
    mode = H.mode_of(ent)
    bad = []
    for t in base["tests"]:
        buf = bytearray(wire0)
        toks = t["mut"].split()
        i = 0
        while i < len(toks):
            if toks[i] == "trunc":
                del buf[int(toks[i + 1]):]
                i += 2
            else:
                p, v = int(toks[i + 1]), int(toks[i + 2])
                if p < len(buf):
                    buf[p] = v
                i += 3
        buf = bytes(buf)
        if mode == C.SPK_MODE_VECTOR:
            res, out, oh, _ = H.oracle_decode(L, mode, buf)
            e, consumed, cnt = res.errc, res.consumed, res.count
        else:
            offs = np.array([0, len(buf)], np.uint64)
            res, out, oh, errc = H.oracle_decode(L, mode, buf, offs, 1)
            e, consumed, cnt = int(errc[0]), res.consumed, 1
        if e != t["errc"] or (e == 0 and consumed != t["consume"]):
            bad.append((t["mut"], e, t["errc"], consumed, t["consume"]))
            continue
        if e == 0:
            o2, oh2 = out[:cnt], oh
            if H.has_assoc(L):  # the reference's map / set from the decoded sequence
                o2, oh2 = H.normalize_assoc(L, o2, oh2)
            re, _, _ = H.oracle_encode(L, mode, o2, oh2)
            if H.sha256(re) != t["reenc_sha256"]:
                bad.append((t["mut"], "reenc"))
    assert not bad, bad[:10]


# ---- varint edge values (LEB128 / zigzag KATs, varint.hpp:194-330) ----------
VARP_EDGE = [  # (x: var_int64_t, y: var_uint32_t, expected LEB128 bytes of x, of y)
    (-(1 << 63), 0xFFFFFFFF, "ff" * 9 + "01", "ffffffff0f"),
    ((1 << 63) - 1, 0, "fe" + "ff" * 8 + "01", "00"),
    (-1, 127, "01", "7f"),
    (0, 128, "00", "8001"),
    (63, 16383, "7e", "ff7f"),
    (-64, 16384, "7f", "808001"),
    (64, 1 << 28, "8001", "8080808001"),
]


def varp_edge_records():
    from yalantinglibs_amd import layout as LY
    L = LY.case_layout("varp")
    recs = np.zeros(len(VARP_EDGE), L.dev.dtype)
    recs["id"] = np.arange(len(VARP_EDGE), dtype=np.int32) - 3
    recs["x"] = [e[0] for e in VARP_EDGE]
    recs["y"] = [e[1] for e in VARP_EDGE]
    return L, recs


def varp_edge_wire(L):
    head = (L.c.fmt_one.code & ~1).to_bytes(4, "little")  # no container: no meta byte
    return [head + int(i - 3).to_bytes(4, "little", signed=True) + bytes.fromhex(xb)
            + bytes.fromhex(yb) for i, (_, _, xb, yb) in enumerate(VARP_EDGE)]


def test_oracle_varint_edge_values():
    L, recs = varp_edge_records()
    wire, offs, _ = H.oracle_encode(L, C.SPK_MODE_MESSAGES, recs, [])
    msgs = varp_edge_wire(L)
    assert wire == b"".join(msgs)
    assert list(np.diff(offs.astype(np.int64))) == [len(m) for m in msgs]
    res, back, _, ec = H.oracle_decode(L, C.SPK_MODE_MESSAGES, wire, offs, len(msgs))
    assert res.errc == 0 and (ec == 0).all()
    assert back[:len(msgs)].tobytes() == recs.tobytes()


def test_reference_binary_goldens_are_our_fixtures():
    """The reference's own goldens (src/struct_pack/tests/binary_data/
    test_cross_platform*.dat, checked by test_cross_platform.cpp:25-52) are
    byte for byte the complicated_object fixtures our generator writes, so
    every fixture test below covers them."""
    import os
    g = H.GOLDEN
    for ref, mine in (("ref_test_cross_platform.dat", "cplx_B_n1_p0_typeinfo.bin"),
                      ("ref_test_cross_platform_without_debug_info.dat",
                       "cplx_B_n1_p0_default.bin")):
        with open(os.path.join(g, ref), "rb") as f, open(os.path.join(g, mine), "rb") as f2:
            assert f.read() == f2.read()


@pytest.mark.parametrize("ref,conf", [("ref_test_cross_platform.dat", "typeinfo"),
                                      ("ref_test_cross_platform_without_debug_info.dat",
                                       "default")])
def test_oracle_decodes_reference_binary_goldens(ref, conf):
    """test_cross_platform.cpp:25-52 restated: deserialize<complicated_object>
    of the reference's file == create_complicated_object(), and back to the
    same bytes."""
    import os
    from yalantinglibs_amd import layout as LY
    with open(os.path.join(H.GOLDEN, ref), "rb") as f:
        wire = f.read()
    L = LY.case_layout("cplx", H.CONF[conf])
    _, recs, heaps = synth.make_batch("cplx", 1, 0, 0)
    res, out, oh, errc = H.oracle_decode(L, C.SPK_MODE_MESSAGES, wire,
                                         np.array([0, len(wire)], np.uint64), 1)
    assert res.errc == 0 and errc[0] == 0 and res.consumed == len(wire)
    assert H.records_equal(L, out[:1], recs, oh, heaps, res.heap_used)
    back, _, _ = H.oracle_encode(L, C.SPK_MODE_MESSAGES, out[:1], oh)
    assert back == wire


@pytest.mark.parametrize("case", sorted(synth.CASE_TYPES))
def test_min_record_wire_bytes_is_a_lower_bound(case):
    """schema.min_record_wire_bytes bounds a decode's record capacity: no
    record of the type takes fewer wire bytes, checked on all-zero records
    (empty containers, zero varints: the smallest encodings) through the
    pinned oracle. For rect2<int32_t> (four fast varints) it is the 1-byte
    bitset (packer.hpp:193-212)."""
    from yalantinglibs_amd import layout as LY
    L = LY.case_layout(case)
    n = 64
    _, recs, heaps = synth.make_batch(case, n, 0x2E80, 4)
    recs = np.zeros(recs.shape, recs.dtype)  # (zeros_like leaves padding bytes unset)
    heaps = [np.zeros_like(h) for h in heaps]
    try:
        wire_n, _, _ = H.oracle_encode(L, C.SPK_MODE_VECTOR, recs, heaps)
    except AssertionError:
        pytest.skip("all-zero records are not encodable for this case (e.g. a variant index)")
    wire_1, _, _ = H.oracle_encode(L, C.SPK_MODE_VECTOR, recs[:1], [h[:0] for h in heaps])
    per_rec = (len(wire_n) - len(wire_1)) / (n - 1)
    assert per_rec >= S.min_record_wire_bytes(L.dev), (per_rec, S.min_record_wire_bytes(L.dev))
    if case == "rect2":
        assert S.min_record_wire_bytes(L.dev) == 1
