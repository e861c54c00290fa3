"""Seeded synthetic record batches (numpy, host side).

Restates the generator of oracle/ref/types.hpp (used by the golden
generator compiled against the reference) so tests can rebuild the exact
inputs behind each fixture; the device restatement is spk_synth in
yalantinglibs_amd/csrc/spk_codec.hip (used at full size on the GPU box).
Outputs are in device-record form (schema.flatten): a structured array of
records plus one heap per span member.
"""
from __future__ import annotations

import numpy as np

from . import schema as S

GOLD = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def rnd(seed, i, k):
    i = np.asarray(i, dtype=np.uint64)
    k = np.asarray(k, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.asarray(seed, dtype=np.uint64) + (i * np.uint64(64) + k + np.uint64(1)) * GOLD
    return mix64(x)


def rf(r):
    return (np.asarray(r, np.uint64).astype(np.uint32).view(np.int32)
            .astype(np.float32) / np.float32(65536.0))


def rd(r):
    return (np.asarray(r, np.uint64).astype(np.uint32).view(np.int32)
            .astype(np.float64) / 65536.0)


def i32(r):
    return np.asarray(r, np.uint64).astype(np.uint32).view(np.int32)


# ---- record types of the BASELINE configs (oracle/ref/types.hpp) --------
Rec64 = S.Struct("Rec64", [("i0", S.int32), ("i1", S.int32), ("i2", S.int32),
                           ("i3", S.int32), ("f0", S.float32), ("f1", S.float32),
                           ("f2", S.float32), ("f3", S.float32),
                           ("d0", S.float64), ("d1", S.float64),
                           ("d2", S.float64), ("d3", S.float64)])
RecS = S.Struct("RecS", [("id", S.int32), ("name", S.String()), ("v", S.float64)])
Inner = S.Struct("Inner", [("x", S.int32), ("y", S.float32)])
Outer = S.Struct("Outer", [("key", S.int64), ("items", S.Vector(Inner))])
Pad = S.Struct("Pad", [("a", S.int8), ("b", S.int32), ("c", S.int16)])
Mixed = S.Struct("Mixed", [("p", Pad), ("k", S.int64), ("arr", S.Array(S.int16, 3)),
                           ("s", S.String()), ("v", S.Vector(S.int32))])
RectInt = S.Struct("rect<int>", [("x", S.int32), ("y", S.int32), ("width", S.int32),
                                 ("height", S.int32)],
                   config=S.DISABLE_ALL_META_INFO)
Point = S.Struct("point", [("x", S.float64), ("y", S.float64)])
RpcRect = S.Struct("rect", [("p1", Point), ("p2", Point)])
Person = S.Struct("person", [("id", S.int32), ("name", S.String()), ("age", S.int32),
                             ("salary", S.float64)])
Ints = S.Vector(S.int32)
ReqHeader = S.Struct("req_header", [("magic", S.uint8), ("version", S.uint8),
                                    ("serialize_type", S.uint8), ("msg_type", S.uint8),
                                    ("seq_num", S.uint32), ("function_id", S.uint32),
                                    ("length", S.uint32), ("attach_length", S.uint32)])
RespHeader = S.Struct("resp_header", [("magic", S.uint8), ("version", S.uint8),
                                      ("err_code", S.uint8), ("msg_type", S.uint8),
                                      ("seq_num", S.uint32), ("length", S.uint32),
                                      ("attach_length", S.uint32)])

Opt = S.Struct("Opt", [("id", S.int32), ("score", S.Optional(S.float64)),
                       ("tag", S.String()), ("pad", S.Optional(Pad))])
OptP = S.Struct("OptP", [("k", S.int64), ("a", S.Optional(S.int32)),
                         ("b", S.Optional(Point))])

Var = S.Struct("Var", [("a", S.var_int32), ("s", S.String()), ("b", S.var_uint64),
                       ("d", S.float64), ("c", S.var_int64), ("e", S.var_uint32)])
VarP = S.Struct("VarP", [("id", S.int32), ("x", S.var_int64), ("y", S.var_uint32)])

# containers of non-trivially-serializable elements (SPK_OP_ARRAY)
Tags = S.Struct("Tags", [("id", S.int32), ("tags", S.Vector(S.String())), ("w", S.float64)])
Group = S.Struct("Group", [("gid", S.int64), ("members", S.Vector(RecS)),
                           ("label", S.String())])
Deep = S.Struct("Deep", [("k", S.uint16), ("m", S.Vector(S.Vector(S.String())))])

Vnt = S.Struct("Vnt", [("id", S.int32),
                       ("v", S.Variant(S.int32, S.float64, S.String(), Inner)),
                       ("w", S.Variant(S.Monostate(), S.Vector(S.int32))),
                       ("list", S.Vector(S.Variant(S.int64, S.String())))])

# struct_pack::compatible members (types.hpp Cmp / CmpOld / CmpNew: one type
# code, three writer versions)
Cmp = S.Struct("Cmp", [("id", S.int32), ("a", S.Compatible(S.int64, 20210101)),
                       ("name", S.String()), ("c", S.Compatible(S.float64, 20240101)),
                       ("b", S.Compatible(S.int16, 20210101))])
CmpOld = S.Struct("CmpOld", [("id", S.int32), ("name", S.String())])
CmpNew = S.Struct("CmpNew", Cmp.fields + [("d", S.Compatible(S.int32, 20250101))])

# sp_config varint encodings (types.hpp FV / FVE / FV32 / EV)
FV = S.Struct("FV", [("a", S.var_int32), ("s", S.String()), ("b", S.var_uint64),
                     ("d", S.float64), ("c", S.var_int64), ("e", S.var_uint32)],
              config=S.USE_FAST_VARINT)
FVE = S.Struct("FVE", [("a", S.int32), ("s", S.String()), ("b", S.uint64), ("d", S.float64),
                       ("c", S.int64), ("e", S.uint32), ("f", S.int16)],
               config=S.ENCODING_WITH_VARINT | S.USE_FAST_VARINT)
FV32 = S.Struct("FV32", [("a", S.var_uint32), ("x", S.int16), ("b", S.var_int32)],
                config=S.USE_FAST_VARINT)
EV = S.Struct("EV", [("a", S.int32), ("s", S.String()), ("b", S.uint64), ("c", S.int64),
                     ("e", S.uint32)], config=S.ENCODING_WITH_VARINT)

# alignment overrides (types.hpp; ref alignment.hpp, tests/test_alignas.cpp)
Al8 = S.Struct("Al8", [("a", S.char), ("b", S.int16)], alignas=8)
AlA = S.Struct("AlA", [("a", S.char), ("b", S.int16)], alignas=4)
AlB = S.Struct("AlB", [("a", S.char), ("b", S.int32)], alignas=8)
AlOuter = S.Struct("AlOuter", [("a", AlA), ("b", AlB)], alignas=16)
Packed = S.Struct("Packed", [("a", S.char), ("b", S.int32), ("c", S.int16)], pack=1)
AlRec = S.Struct("AlRec", [("o", AlOuter), ("s", S.String()), ("p", Packed), ("e", Al8)])

# optional / expected / compatible of values that are not trivially
# serializable (SPK_OP_OPTGROUP / SPK_OP_CGROUP): the coro_rpc benchmark's
# request type (ref src/coro_rpc/benchmark/api/ValidateRequest.h) and types.hpp
ResponseCode = S.Struct("ResponseCode", [("retcode", S.int32),
                                         ("error_message", S.Optional(S.String()))])
AliMessage = S.Struct("AliMessage", [
    ("message_type", S.int32), ("session_no", S.Optional(S.String())),
    ("tint_flag", S.Optional(S.boolean)), ("source_entity", S.Optional(S.uint32)),
    ("dest_entity", S.Optional(S.uint32)), ("client_ip", S.Optional(S.String())),
    ("rc", S.Optional(ResponseCode)), ("version", S.Optional(S.int32))])
ValidateRequest = S.Struct("ValidateRequest", [
    ("msg", AliMessage), ("job_id", S.Optional(S.int32)),
    ("query_keys", S.Vector(S.String())), ("clean", S.Optional(S.boolean))])
Exp = S.Struct("Exp", [("id", S.int32), ("r", S.Expected(S.String(), S.int32)),
                       ("q", S.Expected(Inner, S.String())),
                       ("l", S.Optional(S.Vector(S.String()))),
                       ("e", S.Expected(S.int64, ResponseCode))])
CmpG = S.Struct("CmpG", [("id", S.int32), ("note", S.Compatible(S.String(), 20230101)),
                         ("name", S.String()),
                         ("ints", S.Compatible(S.Vector(S.int32), 20230101)),
                         ("in", S.Compatible(Inner, 20240101)),
                         ("rc", S.Compatible(ResponseCode, 20240101))])

# the reference benchmark's shapes (ref src/struct_pack/benchmark/data_def.hpp)
Vec3 = S.Struct("Vec3", [("x", S.float32), ("y", S.float32), ("z", S.float32)])
Weapon = S.Struct("Weapon", [("name", S.String()), ("damage", S.int16)])
Monster = S.Struct("Monster", [("pos", Vec3), ("mana", S.int16), ("hp", S.int16),
                               ("name", S.String()), ("inventory", S.String()),
                               ("color", S.uint8),  # enum Color : uint8_t
                               ("weapons", S.Vector(Weapon)), ("equipped", Weapon),
                               ("path", S.Vector(Vec3))])
Rect2 = S.Struct("rect2<int32_t>", [("x", S.int32), ("y", S.int32), ("width", S.int32),
                                    ("height", S.int32)],
                 config=S.DISABLE_ALL_META_INFO | S.USE_FAST_VARINT | S.ENCODING_WITH_VARINT)

# the other container kinds (types.hpp Lists / Maps) and the reference's
# complicated_object (ref src/struct_pack/tests/test_struct.hpp:17-103)
Lists = S.Struct("Lists", [("id", S.int32), ("names", S.List(S.String())),
                           ("vals", S.List(S.int32, "std::deque")), ("pts", S.List(Inner))])
Maps = S.Struct("Maps", [("id", S.int32), ("m", S.Map(S.int32, S.String())),
                         ("s", S.Set(S.String())), ("mm", S.Map(S.int64, Inner, multi=True)),
                         ("ms", S.Set(S.int32, multi=True)), ("mr", S.Map(S.String(), RecS))])
CPerson = S.Struct("person", [("age", S.int32), ("name", S.String())])
TrivialOne = S.Struct("trivial_one", [("a", S.int32), ("b", S.float64), ("c", S.float32)])
Cplx = S.Struct("complicated_object", [
    ("color", S.int32), ("a", S.int32), ("b", S.String()), ("c", S.Vector(CPerson)),
    ("d", S.List(S.String())), ("e", S.List(S.int32, "std::deque")),
    ("f", S.Map(S.int32, CPerson)), ("g", S.Map(S.int32, CPerson, multi=True)),
    ("h", S.Set(S.String())), ("i", S.Set(S.int32, multi=True)),
    ("j", S.Map(S.int32, CPerson, ordered=False)),
    ("k", S.Map(S.int32, S.int32, multi=True, ordered=False)),
    ("m", S.Array(CPerson, 2)), ("n", S.Array(CPerson, 2)), ("o", S.Pair(S.String(), CPerson)),
    ("p", S.Vector(S.Array(TrivialOne, 2)))])
# the reference's opt-in types (types.hpp WideT / Wide: 128-bit integers,
# std::bitset, wchar_t, char16_t / char32_t strings)
WideT = S.Struct("WideT", [("a", S.int128), ("bits", S.Bitset(64)), ("c32", S.char32),
                           ("wc", S.wchar), ("c16", S.char16), ("b", S.uint128)])
Wide = S.Struct("Wide", [("id", S.int32), ("a", S.String(elem=S.char16)), ("big", S.int128),
                         ("b", S.String(elem=S.char32)), ("bits", S.Bitset(128)),
                         ("c", S.String(elem=S.wchar)), ("ubig", S.uint128), ("wc", S.wchar),
                         ("c16", S.char16), ("t", WideT)])

CASE_TYPES = {"rec64": Rec64, "recs": RecS, "outer": Outer, "pad": Pad,
              "mixed": Mixed, "rect": RectInt, "rpcrect": RpcRect,
              "person": Person, "ints": Ints, "opt": Opt, "optp": OptP,
              "var": Var, "varp": VarP, "tags": Tags, "group": Group, "deep": Deep,
              "vnt": Vnt, "cmp": Cmp, "cmpold": CmpOld, "cmpnew": CmpNew, "fv": FV, "fve": FVE,
              "fv32": FV32, "ev": EV, "al8": Al8, "alout": AlOuter, "packed": Packed, "alrec": AlRec,
              "valreq": ValidateRequest, "exp": Exp, "cmpg": CmpG, "monster": Monster,
              "rect2": Rect2, "lists": Lists, "maps": Maps, "cplx": Cplx,
              "widet": WideT, "wide": Wide}
# vector<rect<int>> / vector<rect2<int32_t>> have their own ADL set_sp_config
# (benchmark data_def.hpp:69-72,90-94)
VECTOR_CONFIG = {"rect": S.DISABLE_ALL_META_INFO, "rect2": S.DISABLE_ALL_META_INFO}


def _chars(seed, idx, lens, raw=False):
    """make_chars: char j of record i from word 2 + (j>>3)%56 ('a'..'z', or
    the byte itself when raw)."""
    total = int(lens.sum())
    rec = np.repeat(idx, lens)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if len(lens) else np.zeros(0, np.int64)
    j = np.arange(total, dtype=np.uint64) - np.repeat(starts, lens).astype(np.uint64)
    w = rnd(seed, rec, np.uint64(2) + (j >> np.uint64(3)) % np.uint64(56))
    b = (w >> ((j & np.uint64(7)) * np.uint64(8))) & np.uint64(0xFF)
    if raw:
        return b.astype(np.uint8)
    return (np.uint64(ord("a")) + b % np.uint64(26)).astype(np.uint8)


def recs_lens(seed, idx, param):
    """Lengths of make_chars (types.hpp chars_len): a plain param < 65536 is
    U[0, param]; otherwise maxlen in bits 0-15, minlen in bits 16-30, bit 31
    = raw bytes."""
    if param < 0x10000:
        return (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
    mx, mn = param & 0xFFFF, (param >> 16) & 0x7FFF
    return (np.uint64(mn) + rnd(seed, idx, 1) % np.uint64(mx - mn + 1)).astype(np.int64)


def _seg(cnt):
    """(owner index, index within the owner) of every element of lists with
    counts `cnt`."""
    cnt = np.asarray(cnt, np.int64)
    owner = np.repeat(np.arange(len(cnt)), cnt)
    j = np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(_excl(cnt), cnt)
    return owner, j.astype(np.uint64)


def _tag_strings(h):
    """tag_chars(h) of types.hpp for every word in h: (lengths, chars)."""
    h = np.asarray(h, np.uint64)
    lens = (h % np.uint64(13)).astype(np.int64)
    owner, k = _seg(lens)
    with np.errstate(over="ignore"):
        w = mix64(h[owner] + (k >> np.uint64(3)))
    b = (w >> ((k & np.uint64(7)) * np.uint64(8))) & np.uint64(0xFF)
    return lens, (np.uint64(ord("a")) + b % np.uint64(26)).astype(np.uint8)


def _elem_word(seed, i, j):
    """elem_word(seed, i, j) of types.hpp."""
    return mix64(rnd(seed, i, np.uint64(2) + np.asarray(j, np.uint64) % np.uint64(56))
                 ^ np.asarray(j, np.uint64))


def _str_records(sub, lens):
    """element records of a std::string element layout (value.n / value.off)."""
    e = np.zeros(len(lens), dtype=sub.dtype)
    e["value.n"] = lens
    e["value.off"] = _excl(lens)
    return e


def _excl(cnt):
    return np.concatenate([[0], np.cumsum(cnt)[:-1]]) if len(cnt) else np.zeros(0, np.int64)


def _pad_raw(w):
    """fill(Pad&): a = w & 0xFF, b = w >> 8, c = w >> 40, zero padding."""
    m = len(w)
    raw = np.zeros((m, 12), np.uint8)
    raw[:, 0] = (w & np.uint64(0xFF)).astype(np.uint8)
    raw[:, 4:8] = (w >> np.uint64(8)).astype(np.uint32)[:, None].view(np.uint8).reshape(m, 4)
    raw[:, 8:10] = (w >> np.uint64(40)).astype(np.uint16)[:, None].view(np.uint8).reshape(m, 2)
    return raw


def make_batch(case: str, n: int, seed: int, param: int = 48):
    """Return (layout, records ndarray, [heaps]) for n records of `case`."""
    t = CASE_TYPES[case]
    L = S.flatten(t)
    recs = np.zeros(n, dtype=L.dtype)
    idx = np.arange(n, dtype=np.uint64)
    heaps = []
    if case == "rec64":
        raw = np.zeros((n, 64), np.uint8)
        v = raw.view(np.int32).reshape(n, 16)
        for k in range(4):
            v[:, k] = i32(rnd(seed, idx, k))
        raw.view(np.float32).reshape(n, 16)[:, 4:8] = np.stack(
            [rf(rnd(seed, idx, 4 + k)) for k in range(4)], 1)
        raw.view(np.float64).reshape(n, 8)[:, 4:8] = np.stack(
            [rd(rnd(seed, idx, 8 + k)) for k in range(4)], 1)
        recs = raw.view(L.dtype).reshape(n)
    elif case == "recs":
        lens = recs_lens(seed, idx, param)
        recs["id"] = i32(rnd(seed, idx, 0))
        recs["name.n"] = lens
        recs["name.off"] = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n else []
        recs["v"] = rd(rnd(seed, idx, 60))
        heaps.append(_chars(seed, idx, lens, raw=param >= 0x80000000))
    elif case == "outer":
        cnt = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["key"] = rnd(seed, idx, 0).view(np.int64)
        recs["items.n"] = cnt
        recs["items.off"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else []
        rec = np.repeat(idx, cnt)
        starts = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else np.zeros(0, np.int64)
        j = (np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(starts, cnt)).astype(np.uint64)
        w = rnd(seed, rec, np.uint64(2) + j % np.uint64(62))
        w2 = mix64(w ^ j)
        inner = np.zeros((len(j), 8), np.uint8)
        inner.view(np.int32).reshape(-1, 2)[:, 0] = i32(w2)
        inner.view(np.float32).reshape(-1, 2)[:, 1] = rf(w2 >> np.uint64(32))
        heaps.append(inner.reshape(-1))
    elif case == "pad":
        w = rnd(seed, idx, 0)
        raw = np.zeros((n, 12), np.uint8)
        raw[:, 0] = (w & np.uint64(0xFF)).astype(np.uint8)
        raw[:, 4:8] = (w >> np.uint64(8)).astype(np.uint32)[:, None].view(np.uint8).reshape(n, 4)
        raw[:, 8:10] = (w >> np.uint64(40)).astype(np.uint16)[:, None].view(np.uint8).reshape(n, 2)
        recs = raw.view(L.dtype).reshape(n)
    elif case == "mixed":
        w = rnd(seed, idx, 0)
        praw = np.zeros((n, 12), np.uint8)
        praw[:, 0] = (w & np.uint64(0xFF)).astype(np.uint8)
        praw[:, 4:8] = (w >> np.uint64(8)).astype(np.uint32)[:, None].view(np.uint8).reshape(n, 4)
        praw[:, 8:10] = (w >> np.uint64(40)).astype(np.uint16)[:, None].view(np.uint8).reshape(n, 2)
        recs["p"] = praw.view("V12").reshape(n)
        recs["k"] = rnd(seed, idx, 58).view(np.int64)
        a = rnd(seed, idx, 59)
        arr = np.stack([(a >> np.uint64(s)).astype(np.uint16) for s in (0, 16, 32)], 1)
        recs["arr"] = arr.view("V6").reshape(n)
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["s.n"] = lens
        recs["s.off"] = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n else []
        heaps.append(_chars(seed, idx, lens))
        cnt = (rnd(seed, idx, 61) % np.uint64(param + 1)).astype(np.int64)
        recs["v.n"] = cnt
        recs["v.off"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else []
        rec = np.repeat(idx, cnt)
        starts = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else np.zeros(0, np.int64)
        j = (np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(starts, cnt)).astype(np.uint64)
        with np.errstate(over="ignore"):
            vals = mix64(rnd(seed, rec, 62) + j)
        heaps.append(i32(vals).view(np.uint8))
    elif case == "rect":
        raw = np.tile(np.array([1, 0, 11, 1], np.int32), (n, 1))
        recs = raw.view(np.uint8).reshape(n, 16).view(L.dtype).reshape(n)
    elif case == "rpcrect":
        raw = np.stack([rd(rnd(seed, idx, k)) for k in range(4)], 1) if n else np.zeros((0, 4))
        recs = raw.astype(np.float64).view(np.uint8).reshape(n, 32).view(L.dtype).reshape(n)
    elif case == "person":
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["id"] = i32(rnd(seed, idx, 0))
        recs["name.n"] = lens
        recs["name.off"] = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n else []
        recs["age"] = (rnd(seed, idx, 60) % np.uint64(100)).astype(np.int32)
        recs["salary"] = rd(rnd(seed, idx, 61))
        heaps.append(_chars(seed, idx, lens))
    elif case == "ints":
        cnt = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["value.n"] = cnt
        recs["value.off"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else []
        rec = np.repeat(idx, cnt)
        starts = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else np.zeros(0, np.int64)
        j = (np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(starts, cnt)).astype(np.uint64)
        with np.errstate(over="ignore"):
            vals = mix64(rnd(seed, rec, 2) + j)
        heaps.append(i32(vals).view(np.uint8))
    elif case == "opt":  # fill(Opt&): optional members (types.hpp)
        bits = rnd(seed, idx, 3)
        recs["id"] = i32(rnd(seed, idx, 0))
        has_s = (bits & np.uint64(1)).astype(np.int64)
        recs["score.n"] = has_s
        recs["score.off"] = _excl(has_s)
        heaps.append(rd(rnd(seed, idx[has_s == 1], 60)).astype("<f8").view(np.uint8))
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["tag.n"] = lens
        recs["tag.off"] = _excl(lens)
        heaps.append(_chars(seed, idx, lens))
        has_p = ((bits >> np.uint64(1)) & np.uint64(1)).astype(np.int64)
        recs["pad.n"] = has_p
        recs["pad.off"] = _excl(has_p)
        heaps.append(_pad_raw(rnd(seed, idx[has_p == 1], 0)).reshape(-1))
    elif case == "optp":  # fill(OptP&)
        bits = rnd(seed, idx, 3)
        recs["k"] = rnd(seed, idx, 0).view(np.int64)
        has_a = (bits & np.uint64(1)).astype(np.int64)
        recs["a.n"] = has_a
        recs["a.off"] = _excl(has_a)
        heaps.append(i32(rnd(seed, idx[has_a == 1], 4)).view(np.uint8))
        has_b = ((bits >> np.uint64(2)) & np.uint64(1)).astype(np.int64)
        recs["b.n"] = has_b
        recs["b.off"] = _excl(has_b)
        sel = idx[has_b == 1]
        pts = np.stack([rd(rnd(seed, sel, 5)), rd(rnd(seed, sel, 6))], 1) if len(sel) \
            else np.zeros((0, 2))
        heaps.append(pts.astype("<f8").view(np.uint8).reshape(-1))
    elif case == "var":  # fill(Var&): varint members (types.hpp)
        r0 = rnd(seed, idx, 0)
        a = _spread(r0) & np.uint64(0xFFFFFFFF)
        a = np.where(r0 & np.uint64(1), ~a & np.uint64(0xFFFFFFFF), a)
        recs["a"] = a.astype(np.uint32).view(np.int32)
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["s.n"] = lens
        recs["s.off"] = _excl(lens)
        heaps.append(_chars(seed, idx, lens))
        recs["b"] = _spread(rnd(seed, idx, 3))
        recs["d"] = rd(rnd(seed, idx, 60))
        r4 = rnd(seed, idx, 4)
        c = _spread(r4)
        recs["c"] = np.where(r4 & np.uint64(1), ~c, c).view(np.int64)
        recs["e"] = (_spread(rnd(seed, idx, 5)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    elif case == "varp":  # fill(VarP&)
        recs["id"] = i32(rnd(seed, idx, 0))
        r1 = rnd(seed, idx, 1)
        x = _spread(r1)
        recs["x"] = np.where(r1 & np.uint64(1), ~x, x).view(np.int64)
        recs["y"] = (_spread(rnd(seed, idx, 2)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    elif case == "tags":  # fill(Tags&)
        recs["id"] = i32(rnd(seed, idx, 0))
        cnt = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["tags.n"] = cnt
        recs["tags.off"] = _excl(cnt)
        recs["w"] = rd(rnd(seed, idx, 60))
        owner, j = _seg(cnt)
        lens, chars = _tag_strings(_elem_word(seed, idx[owner], j))
        heaps.append(_str_records(L.spans[0].sub, lens).view(np.uint8))
        heaps.append(chars)
    elif case == "group":  # fill(Group&): member j = make_recs(mix64(seed + i), j, 20)
        recs["gid"] = rnd(seed, idx, 0).view(np.int64)
        cnt = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["members.n"] = cnt
        recs["members.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        with np.errstate(over="ignore"):
            s2 = mix64(np.uint64(seed) + idx[owner])
        m = np.zeros(len(j), dtype=L.spans[0].sub.dtype)
        m["id"] = i32(rnd(s2, j, 0))
        mlen = (rnd(s2, j, 1) % np.uint64(21)).astype(np.int64)
        m["name.n"] = mlen
        m["name.off"] = _excl(mlen)
        m["v"] = rd(rnd(s2, j, 60))
        mo, c = _seg(mlen)
        w = rnd(s2[mo], j[mo], np.uint64(2) + (c >> np.uint64(3)) % np.uint64(56))
        b = (w >> ((c & np.uint64(7)) * np.uint64(8))) & np.uint64(0xFF)
        heaps.append(m.view(np.uint8))
        heaps.append((np.uint64(ord("a")) + b % np.uint64(26)).astype(np.uint8))
        lens = (rnd(seed, idx, 1) % np.uint64(13)).astype(np.int64)
        recs["label.n"] = lens
        recs["label.off"] = _excl(lens)
        heaps.append(_chars(seed, idx, lens))
    elif case == "deep":  # fill(Deep&): list j of record i has h % 5 strings
        recs["k"] = rnd(seed, idx, 0).astype(np.uint16)
        cnt = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["m.n"] = cnt
        recs["m.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        h = _elem_word(seed, idx[owner], j)
        m = (h % np.uint64(5)).astype(np.int64)
        lists = np.zeros(len(j), dtype=L.spans[0].sub.dtype)
        lists["value.n"] = m
        lists["value.off"] = _excl(m)
        lo, q = _seg(m)
        with np.errstate(over="ignore"):
            lens, chars = _tag_strings(mix64(h[lo] + q + np.uint64(1)))
        heaps.append(lists.view(np.uint8))
        heaps.append(_str_records(L.spans[1].sub, lens).view(np.uint8))
        heaps.append(chars)
    elif case in ("al8", "alout", "packed", "alrec"):  # fill(Al8& / AlOuter& / Packed& / AlRec&)
        def al8_raw(r):
            raw = np.zeros((n, 8), np.uint8)
            raw[:, 0] = (r & np.uint64(0xFF)).astype(np.uint8)
            raw[:, 2:4] = (r >> np.uint64(8)).astype(np.uint16)[:, None].view(np.uint8).reshape(n, 2)
            return raw

        def alout_raw(r):
            raw = np.zeros((n, 16), np.uint8)
            raw[:, 0] = (r & np.uint64(0xFF)).astype(np.uint8)
            raw[:, 2:4] = (r >> np.uint64(8)).astype(np.uint16)[:, None].view(np.uint8).reshape(n, 2)
            raw[:, 8] = ((r >> np.uint64(24)) & np.uint64(0xFF)).astype(np.uint8)
            raw[:, 12:16] = (r >> np.uint64(32)).astype(np.uint32)[:, None].view(np.uint8).reshape(n, 4)
            return raw

        def packed_raw(r):
            raw = np.zeros((n, 7), np.uint8)
            raw[:, 0] = (r & np.uint64(0xFF)).astype(np.uint8)
            raw[:, 1:5] = (r >> np.uint64(8)).astype(np.uint32)[:, None].view(np.uint8).reshape(n, 4)
            raw[:, 5:7] = (r >> np.uint64(40)).astype(np.uint16)[:, None].view(np.uint8).reshape(n, 2)
            return raw
        if case == "al8":
            recs = al8_raw(rnd(seed, idx, 0)).view(L.dtype).reshape(n)
        elif case == "alout":
            recs = alout_raw(rnd(seed, idx, 1)).view(L.dtype).reshape(n)
        elif case == "packed":
            recs = packed_raw(rnd(seed, idx, 2)).view(L.dtype).reshape(n)
        else:
            recs["o"] = alout_raw(rnd(seed, idx, 1)).view("V16").reshape(n)
            lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
            recs["s.n"] = lens
            recs["s.off"] = _excl(lens)
            heaps.append(_chars(seed, idx, lens))
            recs["p"] = packed_raw(rnd(seed, idx, 2)).view("V7").reshape(n)
            recs["e"] = al8_raw(rnd(seed, idx, 0)).view("V8").reshape(n)
    elif case in ("fv", "fve", "fv32", "ev"):  # FvGen of types.hpp
        r7 = rnd(seed, idx, 7)
        sh = r7 >> np.uint64(58)
        z = r7 & np.uint64(0xFFFFFFFF)

        def u(j):
            return np.where((z >> np.uint64(j)) & np.uint64(1), np.uint64(0),
                            rnd(seed, idx, j) >> sh).astype(np.uint64)

        def sg(j):
            x = u(j)
            neg = rnd(seed, idx, j) & np.uint64(1)
            return np.where((z >> np.uint64(j)) & np.uint64(1), np.uint64(0),
                            np.where(neg, ~x, x)).astype(np.uint64)
        if case == "fv32":
            recs["a"] = (u(0) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            recs["x"] = rnd(seed, idx, 5).astype(np.uint16).view(np.int16)
            recs["b"] = (sg(1) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
        else:
            recs["a"] = (sg(0) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
            lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
            recs["s.n"] = lens
            recs["s.off"] = _excl(lens)
            heaps.append(_chars(seed, idx, lens))
            recs["b"] = u(2)
            if case != "ev":
                recs["d"] = rd(rnd(seed, idx, 60))
            recs["c"] = sg(3).view(np.int64)
            recs["e"] = (u(4) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            if case == "fve":
                recs["f"] = rnd(seed, idx, 5).astype(np.uint16).view(np.int16)
    elif case in ("cmp", "cmpold", "cmpnew"):  # fill(Cmp& / CmpOld& / CmpNew&)
        recs["id"] = i32(rnd(seed, idx, 0))
        m = rnd(seed, idx, 6)

        def compat(field, bit, vals):
            has = ((m >> np.uint64(bit)) & np.uint64(1)).astype(np.int64)
            recs[field + ".n"] = has
            recs[field + ".off"] = _excl(has)
            heaps.append(np.ascontiguousarray(vals[has == 1]).view(np.uint8))
        if case != "cmpold":
            compat("a", 0, rnd(seed, idx, 2).view(np.int64))
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["name.n"] = lens
        recs["name.off"] = _excl(lens)
        heaps.append(_chars(seed, idx, lens))
        if case != "cmpold":
            compat("c", 1, rd(rnd(seed, idx, 3)).astype("<f8"))
            compat("b", 2, rnd(seed, idx, 4).astype(np.uint16).view(np.int16))
        if case == "cmpnew":
            compat("d", 3, i32(rnd(seed, idx, 5)))
    elif case == "vnt":  # fill(Vnt&)
        recs["id"] = i32(rnd(seed, idx, 0))
        a = (rnd(seed, idx, 1) % np.uint64(4)).astype(np.int64)
        recs["v.index"] = a
        recs["v.0"] = np.where(a == 0, i32(rnd(seed, idx, 2)), 0)
        recs["v.1"] = np.where(a == 1, rd(rnd(seed, idx, 3)), 0.0)
        lens = np.where(a == 2, (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64), 0)
        recs["v.2.n"] = lens
        recs["v.2.off"] = np.where(a == 2, _excl(lens), 0)
        inner = np.zeros((n, 8), np.uint8)
        sel = a == 3
        inner.view(np.int32).reshape(-1, 2)[:, 0] = np.where(sel, i32(rnd(seed, idx, 4)), 0)
        inner.view(np.float32).reshape(-1, 2)[:, 1] = np.where(sel, rf(rnd(seed, idx, 5)), 0)
        recs["v.3"] = inner.view("V8").reshape(n)
        heaps.append(_chars(seed, idx, lens))
        has_w = (rnd(seed, idx, 6) & np.uint64(1)).astype(np.int64)
        recs["w.index"] = has_w
        cnt = np.where(has_w == 1, (rnd(seed, idx, 7) % np.uint64(param + 1)).astype(np.int64), 0)
        recs["w.1.n"] = cnt
        recs["w.1.off"] = np.where(has_w == 1, _excl(cnt), 0)
        owner, j = _seg(cnt)
        with np.errstate(over="ignore"):
            vals = mix64(rnd(seed, idx[owner], 8) + j)
        heaps.append(i32(vals).view(np.uint8))
        m = (rnd(seed, idx, 9) % np.uint64(5)).astype(np.int64)
        recs["list.n"] = m
        recs["list.off"] = _excl(m)
        lo, q = _seg(m)
        h = _elem_word(seed, idx[lo], q)
        sub = L.spans[2].sub
        el = np.zeros(len(q), dtype=sub.dtype)
        isstr = (h & np.uint64(1)).astype(np.int64)
        el["value.index"] = isstr
        el["value.0"] = np.where(isstr == 0, (h >> np.uint64(1)).view(np.int64), 0)
        slen, chars = _tag_strings((h >> np.uint64(1))[isstr == 1])
        sl = np.zeros(len(q), np.int64)
        sl[isstr == 1] = slen
        el["value.1.n"] = sl
        el["value.1.off"] = np.where(isstr == 1, _excl(sl), 0)
        heaps.append(el.view(np.uint8))
        heaps.append(chars)
    elif case in ("valreq", "exp", "cmpg", "monster", "rect2"):
        recs, heaps = _make_groups(case, L, recs, idx, seed, param)
    elif case == "lists":  # fill(Lists&)
        recs["id"] = i32(rnd(seed, idx, 0))
        cnt = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["names.n"] = cnt
        recs["names.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        lens, chars = _tag_strings(_elem_word(seed, idx[owner], j))
        heaps.append(_str_records(L.spans[0].sub, lens).view(np.uint8))
        heaps.append(chars)
        r3 = rnd(seed, idx, 3)
        cnt = ((r3 >> np.uint64(8)) % np.uint64(7)).astype(np.int64)
        recs["vals.n"] = cnt
        recs["vals.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        with np.errstate(over="ignore"):
            heaps.append(i32(mix64(rnd(seed, idx[owner], 4) + j)).view(np.uint8))
        cnt = (r3 % np.uint64(5)).astype(np.int64)
        recs["pts.n"] = cnt
        recs["pts.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        with np.errstate(over="ignore"):
            w = mix64(rnd(seed, idx[owner], 5) + j)
        pts = np.zeros((len(w), 2), np.int32)
        pts[:, 0] = i32(w)
        pts.view(np.float32)[:, 1] = rf(w >> np.uint64(32))
        heaps.append(pts.view(np.uint8).reshape(-1))
    elif case == "maps":
        recs, heaps = _make_maps(L, recs, idx, seed)
    elif case == "cplx":
        recs, heaps = _make_cplx(L, recs, n)
    elif case == "widet":
        recs = _widet_raw(seed, idx).view(L.dtype).reshape(n)
    elif case == "wide":  # fill(Wide&)
        recs["id"] = i32(rnd(seed, idx, 0))
        for f, kl, kw, dt in (("a", 1, 2, np.uint16), ("b", 5, 6, np.uint32), ("c", 8, 9, np.uint32)):
            lens = (rnd(seed, idx, kl) % np.uint64(param + 1)).astype(np.int64)
            recs[f + ".n"] = lens
            recs[f + ".off"] = _excl(lens)
            owner, j = _seg(lens)
            with np.errstate(over="ignore"):
                w = mix64(rnd(seed, idx[owner], kw) + j)
            heaps.append(w.astype(dt).view(np.uint8).reshape(-1))
        recs["big"] = _u128_raw(rnd(seed, idx, 3), rnd(seed, idx, 4)).view("V16").reshape(n)
        recs["bits"] = _u128_raw(rnd(seed, idx, 7), rnd(seed, idx, 27)).view("V16").reshape(n)
        recs["ubig"] = _u128_raw(rnd(seed, idx, 10), rnd(seed, idx, 11)).view("V16").reshape(n)
        r = rnd(seed, idx, 12)
        recs["wc"] = i32(r)
        recs["c16"] = (r >> np.uint64(32)).astype(np.uint16)
        recs["t"] = _widet_raw(seed, idx).view("V64").reshape(n)
    else:
        raise KeyError(case)
    return L, recs, heaps


def _u128_raw(hi, lo):
    """(hi << 64) | lo as 16 little-endian bytes per row."""
    return np.ascontiguousarray(np.stack([np.asarray(lo, np.uint64), np.asarray(hi, np.uint64)],
                                         1)).view(np.uint8).reshape(-1, 16)


def _widet_raw(seed, idx):
    """fill(WideT&): a (16 B), bits (8), c32, wc, c16, zero padding, b (16) at 48."""
    raw = np.zeros((len(idx), 64), np.uint8)
    raw[:, 0:16] = _u128_raw(rnd(seed, idx, 20), rnd(seed, idx, 21))
    raw[:, 16:24] = rnd(seed, idx, 22)[:, None].view(np.uint8).reshape(-1, 8)
    r = rnd(seed, idx, 23)
    raw[:, 24:32] = r[:, None].view(np.uint8).reshape(-1, 8)  # c32 = low word, wc = high
    raw[:, 32:34] = rnd(seed, idx, 24).astype(np.uint16)[:, None].view(np.uint8).reshape(-1, 2)
    raw[:, 48:64] = _u128_raw(rnd(seed, idx, 25), rnd(seed, idx, 26))
    return raw


def _opt_span(recs, path, has, lens):
    """An optional / expected / compatible group holding a string at `path`:
    the string's count and offset are set only where the group is present
    (the decoder leaves an absent group's fields alone)."""
    lens = np.where(has, lens, 0).astype(np.int64)
    recs[path + ".n"] = lens
    recs[path + ".off"] = np.where(has, _excl(lens), 0)
    return lens


def _opt_heap(recs, path, has, vals):
    """A trivially serializable optional (SPK_OP_OPTION): count 0/1 and the
    offset of the value among the present ones (absent ones too)."""
    has = has.astype(np.int64)
    recs[path + ".n"] = has
    recs[path + ".off"] = _excl(has)
    return np.ascontiguousarray(vals[has == 1]).view(np.uint8).reshape(-1)


def _tag_heap(h, mask):
    """Chars of tag_chars(h) where mask (lengths h % 13, else 0)."""
    lens, chars = _tag_strings(h)
    keep = np.repeat(mask, lens)
    return np.where(mask, lens, 0).astype(np.int64), chars[keep]


def _make_groups(case, L, recs, idx, seed, param):
    n = len(idx)
    heaps = []
    bit = lambda w, k: ((w >> np.uint64(k)) & np.uint64(1)).astype(bool)  # noqa: E731
    if case == "valreq":  # fill(ValidateRequest&)
        b = rnd(seed, idx, 3)
        recs["msg.message_type"] = i32(rnd(seed, idx, 0))
        has = bit(b, 0)
        recs["msg.session_no.has"] = has
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        lens = _opt_span(recs, "msg.session_no.value", has, lens)
        heaps.append(_chars(seed, idx, lens))
        heaps.append(_opt_heap(recs, "msg.tint_flag", bit(b, 1),
                               (rnd(seed, idx, 4) & np.uint64(1)).astype(np.uint8)))
        heaps.append(_opt_heap(recs, "msg.source_entity", bit(b, 2),
                               rnd(seed, idx, 5).astype(np.uint32)))
        heaps.append(_opt_heap(recs, "msg.dest_entity", bit(b, 3),
                               rnd(seed, idx, 6).astype(np.uint32)))
        has = bit(b, 4)
        recs["msg.client_ip.has"] = has
        lens, chars = _tag_heap(rnd(seed, idx, 7), has)
        _opt_span(recs, "msg.client_ip.value", has, lens)
        heaps.append(chars)
        has = bit(b, 5)
        recs["msg.rc.has"] = has
        recs["msg.rc.value.retcode"] = np.where(has, i32(rnd(seed, idx, 8)), 0)
        he = has & bit(b, 6)
        recs["msg.rc.value.error_message.has"] = he
        lens, chars = _tag_heap(rnd(seed, idx, 9), he)
        _opt_span(recs, "msg.rc.value.error_message.value", he, lens)
        heaps.append(chars)
        heaps.append(_opt_heap(recs, "msg.version", bit(b, 7), i32(rnd(seed, idx, 10))))
        heaps.append(_opt_heap(recs, "job_id", bit(b, 8), i32(rnd(seed, idx, 11))))
        cnt = ((b >> np.uint64(16)) % np.uint64(5)).astype(np.int64)
        recs["query_keys.n"] = cnt
        recs["query_keys.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        lens, chars = _tag_strings(_elem_word(seed, idx[owner], j))
        heaps.append(_str_records(L.spans[8].sub, lens).view(np.uint8))
        heaps.append(chars)
        heaps.append(_opt_heap(recs, "clean", bit(b, 9),
                               ((rnd(seed, idx, 12) >> np.uint64(1)) & np.uint64(1)).astype(np.uint8)))
    elif case == "exp":  # fill(Exp&)
        b = rnd(seed, idx, 3)
        recs["id"] = i32(rnd(seed, idx, 0))
        has = bit(b, 0)
        recs["r.has"] = has
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        lens = _opt_span(recs, "r.value", has, lens)
        heaps.append(_chars(seed, idx, lens))
        recs["r.error"] = np.where(has, 0, i32(rnd(seed, idx, 4)))
        has = bit(b, 1)
        recs["q.has"] = has
        inner = np.zeros((n, 8), np.uint8)
        inner.view(np.int32).reshape(-1, 2)[:, 0] = np.where(has, i32(rnd(seed, idx, 5)), 0)
        inner.view(np.float32).reshape(-1, 2)[:, 1] = np.where(has, rf(rnd(seed, idx, 6)), 0)
        recs["q.value"] = inner.view("V8").reshape(n)
        lens, chars = _tag_heap(rnd(seed, idx, 7), ~has)
        _opt_span(recs, "q.error", ~has, lens)
        heaps.append(chars)
        has = bit(b, 2)
        recs["l.has"] = has
        cnt = np.where(has, ((b >> np.uint64(16)) % np.uint64(4)).astype(np.int64), 0)
        recs["l.value.n"] = cnt
        recs["l.value.off"] = np.where(has, _excl(cnt), 0)
        owner, j = _seg(cnt)
        lens, chars = _tag_strings(_elem_word(seed, idx[owner], j))
        heaps.append(_str_records(L.spans[2].sub, lens).view(np.uint8))
        heaps.append(chars)
        has = bit(b, 3)
        recs["e.has"] = has
        recs["e.value"] = np.where(has, rnd(seed, idx, 8).view(np.int64), 0)
        recs["e.error.retcode"] = np.where(has, 0, i32(rnd(seed, idx, 9)))
        he = ~has & bit(b, 4)
        recs["e.error.error_message.has"] = he
        lens, chars = _tag_heap(rnd(seed, idx, 10), he)
        _opt_span(recs, "e.error.error_message.value", he, lens)
        heaps.append(chars)
    elif case == "cmpg":  # fill(CmpG&)
        m = rnd(seed, idx, 6)
        recs["id"] = i32(rnd(seed, idx, 0))
        has = bit(m, 0)
        recs["note.has"] = has
        lens, chars = _tag_heap(rnd(seed, idx, 2), has)
        _opt_span(recs, "note.value", has, lens)
        heaps.append(chars)
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["name.n"] = lens
        recs["name.off"] = _excl(lens)
        heaps.append(_chars(seed, idx, lens))
        has = bit(m, 1)
        recs["ints.has"] = has
        cnt = _opt_span(recs, "ints.value", has, ((m >> np.uint64(8)) % np.uint64(6)).astype(np.int64))
        owner, j = _seg(cnt)
        with np.errstate(over="ignore"):
            vals = mix64(rnd(seed, idx[owner], 3) + j)
        heaps.append(i32(vals).view(np.uint8))
        has = bit(m, 2).astype(np.int64)
        recs["in.n"] = has
        recs["in.off"] = _excl(has)
        sel = idx[has == 1]
        inner = np.zeros((len(sel), 8), np.uint8)
        inner.view(np.int32).reshape(-1, 2)[:, 0] = i32(rnd(seed, sel, 4))
        inner.view(np.float32).reshape(-1, 2)[:, 1] = rf(rnd(seed, sel, 5))
        heaps.append(inner.reshape(-1))
        has = bit(m, 3)
        recs["rc.has"] = has
        recs["rc.value.retcode"] = np.where(has, i32(rnd(seed, idx, 7)), 0)
        he = has & bit(m, 4)
        recs["rc.value.error_message.has"] = he
        lens, chars = _tag_heap(rnd(seed, idx, 8), he)
        _opt_span(recs, "rc.value.error_message.value", he, lens)
        heaps.append(chars)
    elif case == "monster":  # fill(Monster&)
        pos = np.zeros((n, 12), np.uint8)
        pv = pos.view(np.float32).reshape(n, 3)
        for k in range(3):
            pv[:, k] = rf(rnd(seed, idx, 4 + k))
        recs["pos"] = pos.view("V12").reshape(n)
        r7, r9, r10 = rnd(seed, idx, 7), rnd(seed, idx, 9), rnd(seed, idx, 10)
        recs["mana"] = r7.astype(np.uint16).view(np.int16)
        recs["hp"] = (r7 >> np.uint64(16)).astype(np.uint16).view(np.int16)
        lens = (rnd(seed, idx, 1) % np.uint64(param + 1)).astype(np.int64)
        recs["name.n"] = lens
        recs["name.off"] = _excl(lens)
        heaps.append(_chars(seed, idx, lens))
        lens, chars = _tag_strings(rnd(seed, idx, 8))
        recs["inventory.n"] = lens
        recs["inventory.off"] = _excl(lens)
        heaps.append(chars)
        recs["color"] = (r9 % np.uint64(3)).astype(np.uint8)
        cnt = ((r9 >> np.uint64(8)) % np.uint64(5)).astype(np.int64)
        recs["weapons.n"] = cnt
        recs["weapons.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        h = _elem_word(seed, idx[owner], j)
        wl, wc = _tag_strings(h)
        el = np.zeros(len(h), dtype=L.spans[2].sub.dtype)
        el["name.n"] = wl
        el["name.off"] = _excl(wl)
        el["damage"] = (h >> np.uint64(32)).astype(np.uint16).view(np.int16)
        heaps.append(el.view(np.uint8))
        heaps.append(wc)
        lens, chars = _tag_strings(r10)
        recs["equipped.name.n"] = lens
        recs["equipped.name.off"] = _excl(lens)
        heaps.append(chars)
        recs["equipped.damage"] = (r10 >> np.uint64(40)).astype(np.uint16).view(np.int16)
        cnt = ((r9 >> np.uint64(16)) % np.uint64(9)).astype(np.int64)
        recs["path.n"] = cnt
        recs["path.off"] = _excl(cnt)
        owner, j = _seg(cnt)
        with np.errstate(over="ignore"):
            w = mix64(rnd(seed, idx[owner], 11) + j)
        v = np.zeros((len(w), 3), np.float32)
        v[:, 0] = rf(w)
        v[:, 1] = rf(w >> np.uint64(32))
        v[:, 2] = rf(mix64(w))
        heaps.append(v.view(np.uint8).reshape(-1))
    elif case == "rect2":  # fill(rect2<int32_t>&): FvGen of types.hpp
        r7 = rnd(seed, idx, 7)
        sh = r7 >> np.uint64(58)
        z = r7 & np.uint64(0xFFFFFFFF)
        for k, f in enumerate(("x", "y", "width", "height")):
            x = np.where((z >> np.uint64(k)) & np.uint64(1), np.uint64(0), rnd(seed, idx, k) >> sh)
            neg = rnd(seed, idx, k) & np.uint64(1)
            v = np.where((z >> np.uint64(k)) & np.uint64(1), np.uint64(0), np.where(neg, ~x, x))
            recs[f] = (v.astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
    return recs, heaps


def _spread(w):
    """spread() of types.hpp: magnitudes from 0 to 64 bits."""
    return w >> ((w >> np.uint64(58)) & np.uint64(63))


# ---- per-record builders (associative containers and fixed objects) --------
def _u64(x):
    return int(np.uint64(x))


def _mix(z):
    return int(mix64(np.uint64(z & 0xFFFFFFFFFFFFFFFF)))


def _rnd1(seed, i, k):
    return int(rnd(seed, np.uint64(i), np.uint64(k)))


def _tag1(h):
    """tag_chars(h) of types.hpp for one word."""
    h &= 0xFFFFFFFFFFFFFFFF
    return bytes(ord("a") + ((_mix(h + (k >> 3)) >> ((k & 7) * 8)) & 0xFF) % 26
                 for k in range(h % 13))


def _s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


class _Heaps:
    """Device heaps built element by element (canonical: record order)."""

    def __init__(self, L):
        self.L = L
        self.h = [bytearray() for _ in L.spans]

    def put(self, k, data: bytes):
        """append to heap k; returns the element offset"""
        off = len(self.h[k]) // self.L.spans[k].elem.size
        self.h[k] += data
        return off

    def string(self, k, s: bytes):
        return len(s), self.put(k, s)

    def out(self):
        return [np.frombuffer(bytes(b), np.uint8).copy() for b in self.h]


def _elem_records(sub, rows):
    """element records of an ARRAY from per-element {field: value} dicts"""
    e = np.zeros(len(rows), dtype=sub.dtype)
    for j, r in enumerate(rows):
        for f, v in r.items():
            e[f][j] = v
    return e.view(np.uint8).tobytes()


def _make_maps(L, recs, idx, seed):
    """fill(Maps&) of types.hpp with the containers' own order and key rules:
    map / set keep the first of repeated keys, multimap / multiset all (equal
    keys in insertion order), all sorted by key (std::less: signed integers,
    strings bytewise)."""
    H = _Heaps(L)
    sp = {s.path: k for k, s in enumerate(L.spans)}
    for i in map(int, idx):
        recs["id"][i] = _s32(_rnd1(seed, i, 0))
        b = _rnd1(seed, i, 3)
        m = {}
        for j in range(b % 5):
            h = int(_elem_word(seed, np.uint64(i), np.uint64(j)))
            m.setdefault((h % 7) - 3, _tag1(h >> 8))
        rows = []
        for key in sorted(m):
            ln, off = H.string(sp["m[].second"], m[key])
            rows.append({"first": key, "second.n": ln, "second.off": off})
        recs["m.n"][i] = len(rows)
        recs["m.off"][i] = H.put(sp["m"], _elem_records(L.spans[sp["m"]].sub, rows))
        ss = sorted({_tag1(_mix(_rnd1(seed, i, 20) + j) % 5) for j in range((b >> 8) % 5)})
        rows = []
        for v in ss:
            ln, off = H.string(sp["s[].value"], v)
            rows.append({"value.n": ln, "value.off": off})
        recs["s.n"][i] = len(rows)
        recs["s.off"][i] = H.put(sp["s"], _elem_records(L.spans[sp["s"]].sub, rows))
        mm = []
        for j in range((b >> 16) % 4):
            w = _mix(_rnd1(seed, i, 22) + j)
            mm.append(((_mix(_rnd1(seed, i, 21) + j) % 3) - 1,
                       np.array([_s32(w)], "<i4").tobytes() +
                       rf(np.uint64(w >> 32)).astype("<f4").tobytes()))
        mm.sort(key=lambda kv: kv[0])  # stable: equal keys keep insertion order
        recs["mm.n"][i] = len(mm)
        recs["mm.off"][i] = H.put(sp["mm"], b"".join(np.array([k], "<i8").tobytes() + v
                                                    for k, v in mm))
        ms = sorted((_mix(_rnd1(seed, i, 23) + j) % 7) - 3 for j in range((b >> 24) % 6))
        recs["ms.n"][i] = len(ms)
        recs["ms.off"][i] = H.put(sp["ms"], np.array(ms, "<i4").tobytes())
        mr = {}
        for j in range((b >> 32) % 3):
            mr.setdefault(_tag1(_mix(_rnd1(seed, i, 24) + j) % 4 + 1), j)
        rows = []
        s2 = _mix(seed + i)
        for key in sorted(mr):
            j = mr[key]
            kl, ko = H.string(sp["mr[].first"], key)
            nm = bytes(_chars(np.uint64(s2), np.array([j], np.uint64),
                              np.array([_rnd1(s2, j, 1) % 11], np.int64)))
            nl, no = H.string(sp["mr[].second.name"], nm)
            rows.append({"first.n": kl, "first.off": ko, "second.id": _s32(_rnd1(s2, j, 0)),
                         "second.name.n": nl, "second.name.off": no,
                         "second.v": float(rd(np.uint64(_rnd1(s2, j, 60))))})
        recs["mr.n"][i] = len(rows)
        recs["mr.off"][i] = H.put(sp["mr"], _elem_records(L.spans[sp["mr"]].sub, rows))
    return recs, H.out()


def _make_cplx(L, recs, n):
    """create_complicated_object() (ref src/struct_pack/tests/test_struct.hpp:
    82-103) in every record; padding bytes zero."""
    H = _Heaps(L)
    sp = {s.path: k for k, s in enumerate(L.spans)}

    def person_rows(ps, path):
        rows = []
        for age, name in ps:
            ln, off = H.string(sp[path], name)
            rows.append({"age": age, "name.n": ln, "name.off": off})
        return rows

    def pair_rows(kvs, path):
        rows = []
        for k, (age, name) in kvs:
            ln, off = H.string(sp[path], name)
            rows.append({"first": k, "second.age": age, "second.name.n": ln, "second.name.off": off})
        return rows

    def arr(field, rows, k):
        recs[field + ".n"][i] = len(rows)
        recs[field + ".off"][i] = H.put(sp[field], _elem_records(L.spans[k].sub, rows))

    def span(field, data: bytes):
        esz = L.spans[sp[field]].elem.size
        recs[field + ".n"][i] = len(data) // esz
        recs[field + ".off"][i] = H.put(sp[field], data)

    def string(field, s):
        recs[field + ".n"][i], recs[field + ".off"][i] = H.string(sp[field], s)

    for i in range(n):
        recs["color"][i] = 0  # Color::red
        recs["a"][i] = 42
        string("b", b"hello")
        arr("c", person_rows([(20, b"tom"), (22, b"jerry")], "c[].name"), sp["c"])
        rows = []
        for s_ in (b"hello", b"world"):
            ln, off = H.string(sp["d[].value"], s_)
            rows.append({"value.n": ln, "value.off": off})
        arr("d", rows, sp["d"])
        span("e", np.array([1, 2], "<i4").tobytes())
        arr("f", pair_rows([(1, (20, b"tom"))], "f[].second.name"), sp["f"])
        arr("g", pair_rows([(1, (20, b"tom")), (1, (22, b"jerry"))], "g[].second.name"), sp["g"])
        rows = []
        for s_ in (b"aa", b"bb"):
            ln, off = H.string(sp["h[].value"], s_)
            rows.append({"value.n": ln, "value.off": off})
        arr("h", rows, sp["h"])
        span("i", np.array([1, 2], "<i4").tobytes())
        arr("j", pair_rows([(1, (20, b"tom"))], "j[].second.name"), sp["j"])
        span("k", np.array([1, 2], "<i4").tobytes())
        for f, ps in (("m", [(20, b"tom"), (22, b"jerry")]), ("n", [(15, b"tom"), (31, b"jerry")])):
            for q, (age, name) in enumerate(ps):
                recs[f"{f}[{q}].age"][i] = age
                string(f"{f}[{q}].name", name)
        string("o.first", b"aa")
        recs["o.second.age"][i] = 20
        string("o.second.name", b"tom")
        t = np.zeros(4, dtype=np.dtype({"names": ["a", "b", "c"], "formats": ["<i4", "<f8", "<f4"],
                                        "offsets": [0, 8, 16], "itemsize": 24}))
        t["a"] = [1232114, 12315, 4, 1123115]
        t["b"] = [1.7, 1.4, 0.7, 11111.4]
        t["c"] = np.array([2.4, 2.6, 1.4, 2213321.6], np.float32)
        span("p", t.tobytes())
    return recs, H.out()
