"""CPU: the C-ABI library loads, exports every symbol include/spk_codec.h
declares, and validates descriptors (no device work without a GPU)."""
import ctypes as ct
import os
import re

import pytest

import spk_helpers as H
from yalantinglibs_amd import _capi as C
from yalantinglibs_amd import layout as LY
from yalantinglibs_amd import schema as S
from yalantinglibs_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "spk_codec.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(spk_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = C.load_codec()
    syms = header_symbols()
    assert set(syms) == set(C.CODEC_SYMBOLS)
    for s in syms:
        assert hasattr(lib, s), s


def test_abi_and_messages():
    lib = C.load_codec()
    assert lib.spk_abi_version() == C.SPK_ABI_VERSION
    assert lib.spk_errc_message(1) == b"no buffer space"
    assert lib.spk_errc_message(2) == b"invalid argument"
    assert lib.spk_errc_message(3) == b"hash conflict"


def test_struct_sizes_match_header():
    assert ct.sizeof(C.spk_op) == 16
    assert ct.sizeof(C.spk_msgfmt) == 16 + C.SPK_MAX_LITERAL
    assert ct.sizeof(C.spk_plan_t) == 40
    assert ct.sizeof(C.spk_dresult_t) == 32 + 8 * C.SPK_MAX_SPANS


@pytest.mark.parametrize("case", sorted(synth.CASE_TYPES))
def test_layout_check_accepts_configs(case):
    lib = C.load_codec()
    L = LY.case_layout(case)
    assert lib.spk_layout_check(L.ptr) == 0
    assert lib.spk_workspace_bytes(L.ptr, C.SPK_MODE_VECTOR, 1000, 1 << 20) > 0


def test_layout_check_rejects_malformed():
    lib = C.load_codec()
    L = LY.case_layout("recs")
    L.c.abi = 99
    assert lib.spk_layout_check(L.ptr) == C.SPK_E_LAYOUT
    L = LY.case_layout("recs")
    L.c.ops[1].rec_off = 3  # misaligned count
    assert lib.spk_layout_check(L.ptr) == C.SPK_E_LAYOUT
    L = LY.case_layout("rec64")
    L.c.ops[0].size = 60  # trivial layout must copy the whole record
    assert lib.spk_layout_check(L.ptr) == C.SPK_E_LAYOUT


def test_layout_check_varint_ops():
    lib = C.load_codec()
    L = LY.case_layout("var")
    vi = [i for i in range(L.c.n_ops) if L.c.ops[i].kind == C.SPK_OP_VARINT]
    assert len(vi) == 4 and L.c.ops[vi[0]].aux == C.SPK_VARINT_ZIGZAG
    assert [L.c.ops[i].aux for i in vi] == [1, 0, 1, 0]  # var_int32, var_uint64, var_int64, var_uint32
    for field, bad in (("size", 2), ("size", 16), ("rec_off", 2), ("aux", 4)):
        L = LY.case_layout("var")
        setattr(L.c.ops[vi[0]], field, bad)
        assert lib.spk_layout_check(L.ptr) == C.SPK_E_LAYOUT, (field, bad)
    # varints alone (no span / option) make a valid non-trivial record
    assert lib.spk_layout_check(LY.case_layout("varp").ptr) == 0
    # ... also with only 4-byte neighbours: {int32; var_uint32_t; int32} has
    # no 8-byte member, its device stride still rounds up to 8 (12 -> 16)
    t = S.Struct("V4", [("a", S.int32), ("b", S.var_uint32), ("c", S.int32)])
    L4 = LY.make_layout(t)
    assert L4.stride == 16 and lib.spk_layout_check(L4.ptr) == 0


def test_layout_check_compat_ops():
    """compatible<T, ver> members: one SPK_OP_COMPAT per member with its
    version rank in kind >> 8; top-level only, the hash head required, and no
    body / sharded entry point (the version passes trail the whole message)."""
    lib = C.load_codec()
    L = LY.case_layout("cmpnew")
    ks = [L.c.ops[i].kind for i in range(L.c.n_ops) if (L.c.ops[i].kind & 0xFF) == C.SPK_OP_COMPAT]
    assert [k >> 8 for k in ks] == [0, 1, 0, 2]  # 20210101, 20240101, 20210101, 20250101
    assert lib.spk_layout_check(L.ptr) == 0
    for field, bad in (("rec_off", 2), ("aux", 4), ("size", 0), ("kind", C.SPK_OP_COMPAT | 1 << 16)):
        Lb = LY.case_layout("cmp")
        setattr(Lb.c.ops[1], field, bad)
        assert lib.spk_layout_check(Lb.ptr) == C.SPK_E_LAYOUT, (field, bad)
    Lb = LY.case_layout("cmp")
    Lb.c.fmt_one.flags &= ~C.SPK_MF_HASH_HEAD
    assert lib.spk_layout_check(Lb.ptr) == C.SPK_E_LAYOUT
    with pytest.raises(ValueError):  # DISABLE_ALL_META_INFO: a static_assert in the reference
        LY.case_layout("cmp", S.DISABLE_ALL_META_INFO)
    # inside a container element: outside the flat model (host) / E_LAYOUT (C ABI)
    with pytest.raises(NotImplementedError):
        LY.make_layout(S.Struct("W", [("v", S.Vector(synth.Cmp))]))
    Lt = LY.case_layout("tags")
    el = next(i for i in range(Lt.c.n_ops) if Lt.c.ops[i].kind == C.SPK_OP_ARRAY)
    Lt.c.ops[el + 1].kind = C.SPK_OP_COMPAT
    Lt.c.ops[el + 1].aux = 8
    assert lib.spk_layout_check(Lt.ptr) == C.SPK_E_LAYOUT
    # trivially serializable apart from the compatible member (packer.hpp:422-431)
    with pytest.raises(NotImplementedError):
        LY.make_layout(S.Struct("T", [("a", S.int32), ("c", S.Compatible(S.int32, 1))]))
    vb = (ct.c_uint8 * 64)()
    assert lib.spk_vector_header(L.ptr, 3, 1, vb, 64) == C.SPK_E_LAYOUT
    assert lib.spk_encode_body(L.ptr, 0, None, None, 1, vb, 64, vb, 1 << 20, None) == C.SPK_E_LAYOUT
    assert lib.spk_decode_body(L.ptr, vb, 0, 1, 0, None, 0, None, None, vb, vb, 1 << 20,
                               None) == C.SPK_E_LAYOUT


def test_layout_check_fast_varint_ops():
    """USE_FAST_VARINT: one SPK_OP_FVAR per varint member of the top-level
    record (signed flag for var_int* / int*); ENCODING_WITH_VARINT alone turns
    plain ints into VARINT ops (int32_t sign-extended, no zigzag)."""
    lib = C.load_codec()
    L = LY.case_layout("fve")
    fv = [(L.c.ops[i].kind, L.c.ops[i].size, L.c.ops[i].aux) for i in range(L.c.n_ops)
          if L.c.ops[i].kind == C.SPK_OP_FVAR]
    assert fv == [(9, 4, 1), (9, 8, 0), (9, 8, 1), (9, 4, 0)]  # int32, uint64, int64, uint32
    assert lib.spk_layout_check(L.ptr) == 0
    i0 = next(i for i in range(L.c.n_ops) if L.c.ops[i].kind == C.SPK_OP_FVAR)
    for field, bad in (("size", 2), ("rec_off", 2), ("aux", 2)):
        Lb = LY.case_layout("fve")
        setattr(Lb.c.ops[i0], field, bad)
        assert lib.spk_layout_check(Lb.ptr) == C.SPK_E_LAYOUT, (field, bad)
    Le = LY.case_layout("ev")
    vi = [(Le.c.ops[i].size, Le.c.ops[i].aux) for i in range(Le.c.n_ops)
          if Le.c.ops[i].kind == C.SPK_OP_VARINT]
    assert vi == [(4, C.SPK_VARINT_SEXT), (8, 0), (8, 0), (4, 0)]
    Lb = LY.case_layout("ev")
    k = next(i for i in range(Lb.c.n_ops) if Lb.c.ops[i].kind == C.SPK_OP_VARINT)
    Lb.c.ops[k].aux = C.SPK_VARINT_SEXT | C.SPK_VARINT_ZIGZAG
    assert lib.spk_layout_check(Lb.ptr) == C.SPK_E_LAYOUT
    with pytest.raises(NotImplementedError):  # the tag on a nested struct
        LY.make_layout(S.Struct("W", [("k", S.int32), ("v", synth.FV)]))


def test_encode_rejects_bad_args_without_device_work():
    lib = C.load_codec()
    L = LY.case_layout("rec64")
    rc = lib.spk_encode(L.ptr, 7, 10, None, None, None, None, 0, None, None, 0, None)
    assert rc == C.SPK_E_ARG
    rc = lib.spk_plan(L.ptr, C.SPK_MODE_VECTOR, 10, None, None, None, 0, None)
    assert rc == C.SPK_E_ARG


def test_oracle_is_separate_library():
    # the product library never links the CPU restatement
    with open(C.CODEC_PATH, "rb") as f:
        blob = f.read()
    assert b"spko_" not in blob


@pytest.mark.parametrize("name", ["recs_A_n300_p48_default", "tags_A_n30_p300_default",
                                  "rec64_A_n1000_p0_nometa", "outer_A_n1000_p16_default"])
def test_parse_vector_header_host(name):
    """spk_parse_vector_header (host) on reference fixtures: record count,
    width and header length; truncated / corrupted heads give the errc."""
    ent = next(e for e in H.manifest() if e["name"] == name)
    wire, _ = H.read_fixture(ent)
    L = H.layout_for(ent)
    lib = C.load_codec()
    n, w, hl = ct.c_uint64(), ct.c_uint32(), ct.c_uint32()
    buf = (ct.c_uint8 * len(wire)).from_buffer_copy(wire)
    assert lib.spk_parse_vector_header(L.ptr, buf, len(wire), ct.byref(n), ct.byref(w),
                                       ct.byref(hl)) == 0
    assert n.value == ent["n"]
    plan = C.spk_plan_t()
    _, recs, heaps = H.batch_for(ent)
    o = C.load_oracle()
    hp = (ct.c_void_p * max(len(heaps), 1))(*[h.ctypes.data for h in heaps])
    assert o.spko_plan(L.ptr, C.SPK_MODE_VECTOR, len(recs), H._ptr(recs), hp, ct.byref(plan)) == 0
    assert w.value == plan.width and hl.value == plan.header_bytes
    assert lib.spk_parse_vector_header(L.ptr, buf, hl.value - 1, ct.byref(n), ct.byref(w),
                                       ct.byref(hl)) == C.ERRC_NO_BUFFER_SPACE
    if ent["conf"] != "nometa":
        bad = bytearray(wire)
        bad[1] ^= 0x40
        bb = (ct.c_uint8 * len(bad)).from_buffer_copy(bytes(bad))
        assert lib.spk_parse_vector_header(L.ptr, bb, len(bad), ct.byref(n), ct.byref(w),
                                           ct.byref(hl)) == C.ERRC_INVALID_BUFFER
