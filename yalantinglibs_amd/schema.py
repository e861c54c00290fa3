"""Host-side type model for struct_pack records (Python mirror of the C++20
reflection in include/ylt/struct_pack_gpu/reflect.hpp).

Computes, exactly as the reference does at compile time:
  * the type literal  — get_type_literal (ref include/ylt/struct_pack/
    type_calculate.hpp:194-373) with type_id codes of type_id.hpp:25-81 and
    get_size_literal (type_calculate.hpp:26-97);
  * the type code     — MD5Hash32Constexpr(literal) & 0xFFFFFFFE
    (type_calculate.hpp:507-516, md5_constexpr.hpp:315-331);
  * is_trivial_serializable (ref reflection.hpp:851-922), alignment literals
    (alignment.hpp:90-122) and check_if_has_container
    (type_calculate.hpp:793-857);
  * the sp_config resolution that decides hash head / type literal
    (type_calculate.hpp:158-172, 744-891);
and flattens a record type into the spk_layout descriptor of
include/spk_codec.h (COPY / SPAN / OPTION ops over a "device record").
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Optional as Optional_
from typing import List, Optional, Sequence, Tuple

import numpy as np

# ---- sp_config (ref reflection.hpp:53-60) ---------------------------------
DEFAULT = 0
DISABLE_TYPE_INFO = 0b1
ENABLE_TYPE_INFO = 0b10
DISABLE_ALL_META_INFO = 0b11

# ---- type_id (ref type_id.hpp:25-81) --------------------------------------
TID_INT32, TID_UINT32, TID_INT64, TID_UINT64 = 1, 2, 3, 4
TID_INT8, TID_UINT8, TID_INT16, TID_UINT16 = 5, 6, 7, 8
TID_INT128, TID_UINT128 = 9, 10
TID_BOOL, TID_CHAR8, TID_CHAR16, TID_CHAR32, TID_WCHAR = 11, 12, 13, 14, 15
TID_FLOAT32, TID_FLOAT64 = 17, 18
TID_VINT32, TID_VINT64, TID_VUINT32, TID_VUINT64 = 20, 21, 22, 23
TID_STRING, TID_ARRAY, TID_MAP, TID_SET, TID_CONTAINER = 128, 129, 130, 131, 132
TID_OPTIONAL, TID_VARIANT, TID_EXPECTED, TID_BITSET = 133, 134, 135, 136
TID_MONOSTATE = 250
TID_STRUCT = 253
TID_END = 255


def size_literal(n: int) -> bytes:
    """get_size_literal<n>() (ref type_calculate.hpp:26-97): base-127
    little-endian digits +1, the most significant digit +129."""
    out = []
    while n >= 127:
        out.append(n % 127 + 1)
        n //= 127
    out.append(n + 129)
    return bytes(out)


def md5_hash32(data: bytes) -> int:
    """MD5Hash32Constexpr (ref md5_constexpr.hpp:315-331): SwapEndian(a) of
    the MD5 state == the first four digest bytes read big-endian."""
    return int.from_bytes(hashlib.md5(data).digest()[:4], "big")


class SpType:
    name: str = "?"

    def literal(self) -> bytes:  # get_type_literal<T>
        raise NotImplementedError

    @property
    def trivial(self) -> bool:  # is_trivial_serializable<T>
        return False

    @property
    def has_container(self) -> bool:  # check_if_has_container<T>
        return False

    # C layout (only meaningful for trivially serializable types)
    size: int = 0
    align: int = 1
    config: int = DEFAULT  # per-type sp_config (set_sp_config ADL)

    def root_literal(self) -> bytes:  # get_types_literal<T, get_types<T>...>
        return self.literal()

    def code(self) -> int:  # get_type_code<T>()
        return md5_hash32(self.root_literal()) & 0xFFFFFFFE

    def __repr__(self):
        return self.name


class Fund(SpType):
    """Fundamental / enum member (get_integral_type, type_id.hpp:130-280)."""

    def __init__(self, name: str, tid: int, size: int, npdt: str):
        self.name, self.tid, self.size, self.npdt = name, tid, size, npdt
        self.align = size
        self.config = DEFAULT

    def literal(self):
        return bytes([self.tid])

    @property
    def trivial(self):
        return True


int8 = Fund("int8_t", TID_INT8, 1, "<i1")
uint8 = Fund("uint8_t", TID_UINT8, 1, "<u1")
int16 = Fund("int16_t", TID_INT16, 2, "<i2")
uint16 = Fund("uint16_t", TID_UINT16, 2, "<u2")
int32 = Fund("int32_t", TID_INT32, 4, "<i4")
uint32 = Fund("uint32_t", TID_UINT32, 4, "<u4")
int64 = Fund("int64_t", TID_INT64, 8, "<i8")
uint64 = Fund("uint64_t", TID_UINT64, 8, "<u8")
boolean = Fund("bool", TID_BOOL, 1, "<u1")
char = Fund("char", TID_CHAR8, 1, "<u1")
float32 = Fund("float", TID_FLOAT32, 4, "<f4")
float64 = Fund("double", TID_FLOAT64, 8, "<f8")
char16 = Fund("char16_t", TID_CHAR16, 2, "<u2")
char32 = Fund("char32_t", TID_CHAR32, 4, "<u4")
# the reference's opt-in types (type_id.hpp:37-44,168-172,190-197): wchar_t
# under STRUCT_PACK_ENABLE_UNPORTABLE_TYPE (4 bytes, Linux), __int128 /
# unsigned __int128 under STRUCT_PACK_ENABLE_INT128 (16 bytes, alignment 16;
# raw bytes in the device record)
wchar = Fund("wchar_t", TID_WCHAR, 4, "<i4")
int128 = Fund("__int128", TID_INT128, 16, "V16")
uint128 = Fund("unsigned __int128", TID_UINT128, 16, "V16")


class Bitset(Fund):
    """std::bitset<N> (bitset_t, STRUCT_PACK_ENABLE_UNPORTABLE_TYPE;
    reflection.hpp:558-591): only bitsets whose object is exactly (N + 7) / 8
    bytes (libstdc++: whole 64-bit words), written raw (packer.hpp:268-270);
    literal bitset_t + size literal of N (type_calculate.hpp:264-268)."""

    def __init__(self, nbits: int):
        size = (nbits + 7) // 8
        if size % 8:
            raise ValueError("std::bitset<N> is a struct_pack bitset only when "
                             "(N + 7) / 8 == sizeof: N in (64k - 8, 64k]")
        super().__init__(f"std::bitset<{nbits}>", TID_BITSET, size, f"V{size}")
        self.nbits = nbits
        self.align = 8

    def literal(self):
        return bytes([TID_BITSET]) + size_literal(self.nbits)


class VarInt(SpType):
    """struct_pack::var_int32_t / var_int64_t (sint<T>, zigzag) and
    var_uint32_t / var_uint64_t (varint<T>) (ref varint.hpp:352-355): held
    as a plain integer in the device record, LEB128 on the wire. Not
    trivially serializable (reflection.hpp:872), so a struct holding one is
    written member by member."""

    def __init__(self, name: str, tid: int, size: int, npdt: str, zigzag: bool):
        self.name, self.tid, self.size, self.npdt = name, tid, size, npdt
        self.align = size
        self.zigzag = zigzag
        self.config = DEFAULT

    def literal(self):
        return bytes([self.tid])


var_int32 = VarInt("var_int32_t", TID_VINT32, 4, "<i4", True)
var_int64 = VarInt("var_int64_t", TID_VINT64, 8, "<i8", True)
var_uint32 = VarInt("var_uint32_t", TID_VUINT32, 4, "<u4", False)
var_uint64 = VarInt("var_uint64_t", TID_VUINT64, 8, "<u8", False)

# sp_config bits of a record type (reflection.hpp:53-60)
ENCODING_WITH_VARINT, USE_FAST_VARINT = 0b100, 0b1000
_PLAIN_VAR = {TID_INT32: TID_VINT32, TID_UINT32: TID_VUINT32, TID_INT64: TID_VINT64,
              TID_UINT64: TID_VUINT64}


def varint_tid(t: SpType, tag: int):
    """get_varint_type<T, parent_tag> (type_id.hpp:83-125): the type id of a
    varint member under its struct's sp_config tag, or None (reflection.hpp:
    843: with ENCODING_WITH_VARINT plain (u)int32/64 are varints too);
    USE_FAST_VARINT selects the fast_v* ids."""
    if isinstance(t, VarInt):
        tid = t.tid
    elif isinstance(t, Fund) and tag & ENCODING_WITH_VARINT and t.tid in _PLAIN_VAR:
        tid = _PLAIN_VAR[t.tid]
    else:
        return None
    return tid + 4 if tag & USE_FAST_VARINT else tid


class Monostate(SpType):
    name = "std::monostate"
    size = 1
    align = 1

    def literal(self):
        return bytes([TID_MONOSTATE])

    @property
    def trivial(self):
        return True


class Vector(SpType):
    """std::vector<T> (container_t) — also std::span<T> (same bytes)."""

    def __init__(self, elem: SpType, config: int = DEFAULT):
        self.elem = elem
        self.config = config
        self.name = f"std::vector<{elem.name}>"

    def literal(self):
        return bytes([TID_CONTAINER]) + self.elem.literal()

    @property
    def has_container(self):
        return True


class List(Vector):
    """std::list<T> / std::deque<T>: container_t like std::vector, the same
    literal and bytes (type_id.hpp:334-336); decode appends in wire order."""

    def __init__(self, elem: SpType, name: str = "std::list"):
        super().__init__(elem)
        self.name = f"{name}<{elem.name}>"


class Set(Vector):
    """std::set / multiset / unordered_set / unordered_multiset
    (set_container_t): [count:w] then the keys in the container's iteration
    order; literal set_container_t + literal(key) (type_calculate.hpp:280-283).
    The record model keeps the elements in wire order: the reference inserts
    them in that order (unpacker.hpp:1097-1122, emplace: a repeated key of a
    set is dropped), so a host set built by inserting the array equals its."""

    def __init__(self, key: SpType, multi: bool = False, ordered: bool = True):
        super().__init__(key)
        self.multi, self.ordered = multi, ordered
        kind = ("std::multiset" if multi else "std::set") if ordered else \
            ("std::unordered_multiset" if multi else "std::unordered_set")
        self.name = f"{kind}<{key.name}>"
        self.kind = ("multi" if multi else "") + ("set" if ordered else "uset")

    def literal(self):
        return bytes([TID_SET]) + self.elem.literal()


class Map(Vector):
    """std::map / multimap / unordered_map / unordered_multimap
    (map_container_t): [count:w] then each std::pair<const K, V> in the
    container's iteration order, written as a struct (first, second: raw
    sizeof(pair) when both are trivially serializable, packer.hpp:411-421);
    literal map_container_t + literal(K) + literal(V) (type_calculate.hpp:
    284-290). The record model keeps the pairs in wire order: the reference
    decodes them in that order with try_emplace (map: a repeated key keeps
    the first value) / emplace (multimap) (unpacker.hpp:983-1095), so a host
    map built that way from the array equals its."""

    def __init__(self, key: SpType, value: SpType, multi: bool = False, ordered: bool = True):
        super().__init__(Struct("std::pair", [("first", key), ("second", value)]))
        self.key, self.value = key, value
        self.multi, self.ordered = multi, ordered
        kind = ("std::multimap" if multi else "std::map") if ordered else \
            ("std::unordered_multimap" if multi else "std::unordered_map")
        self.name = f"{kind}<{key.name},{value.name}>"
        self.kind = ("multi" if multi else "") + ("map" if ordered else "umap")

    def literal(self):
        return bytes([TID_MAP]) + self.key.literal() + self.value.literal()


def Pair(first: SpType, second: SpType) -> "Struct":
    """std::pair<A, B>: a struct of first and second (type_id.hpp:360,
    type_calculate.hpp:918-920), trivially serializable when both are."""
    return Struct("std::pair", [("first", first), ("second", second)])


class String(SpType):
    """std::string / std::string_view (string_t of char); elem = char16 /
    char32 / wchar for std::u16string / u32string / wstring (string_t + the
    char type's id, type_calculate.hpp:274-278; elements raw on the wire)."""

    def __init__(self, config: int = DEFAULT, elem: SpType = None):
        self.config = config
        self.elem = elem or char
        self.name = {TID_CHAR16: "std::u16string", TID_CHAR32: "std::u32string",
                     TID_WCHAR: "std::wstring"}.get(self.elem.tid, "std::string")

    def literal(self):
        return bytes([TID_STRING, self.elem.tid])

    @property
    def has_container(self):
        return True


class Optional(SpType):
    """std::optional<T> (optional_t): wire [has_value:1][T if present]
    (ref packer.hpp:382-388, unpacker.hpp:1251-1275); its literal is
    optional_t + literal(T) (type_calculate.hpp:273-278); a container only if
    T holds one (type_calculate.hpp:846-849)."""

    def __init__(self, elem: SpType):
        self.elem = elem
        self.name = f"std::optional<{elem.name}>"
        self.config = DEFAULT

    def literal(self):
        return bytes([TID_OPTIONAL]) + self.elem.literal()

    @property
    def has_container(self):
        return self.elem.has_container


class Expected(SpType):
    """struct_pack::expected<T, E> (tl / std::expected; expected_t): wire
    [has_value:1] then T if present else E (ref packer.hpp:400-410; decode
    unpacker.hpp:1251-1277 drops the value's / error's errc); literal
    expected_t + literal(T) + literal(E) (type_calculate.hpp:291-297); T may be
    Monostate() for expected<void, E>. Never trivially serializable
    (reflection.hpp:903-905). Device record: u32 has_value, then T's fields
    and E's fields side by side (SPK_OP_OPTGROUP with two groups)."""

    def __init__(self, value: SpType, error: SpType):
        self.value, self.error = value, error
        self.name = f"struct_pack::expected<{value.name},{error.name}>"
        self.config = DEFAULT

    def literal(self):
        return bytes([TID_EXPECTED]) + self.value.literal() + self.error.literal()

    @property
    def has_container(self):
        return self.value.has_container or self.error.has_container


class Compatible(SpType):
    """struct_pack::compatible<T, version> (compatible_t, ref compatible.hpp:
    21-154): an optional written after the main pass, in the version pass of
    its version (packer.hpp:66-78,453-461); not in the type literal nor the
    hash (type_calculate.hpp:298-303); the message gets a total-length field
    (calculate_size.hpp:457-470). Only a member of the top-level record with a
    trivially serializable T is in the flat record model."""

    def __init__(self, elem: SpType, version: int = 0):
        # (a U that is not trivially serializable is an SPK_OP_CGROUP: its
        # ops inline in the record, [has][U] in the version pass)
        self.elem, self.version = elem, version
        self.name = f"struct_pack::compatible<{elem.name},{version}>"
        self.config = DEFAULT

    def literal(self):
        return b""

    @property
    def has_container(self):
        return self.elem.has_container


def has_compatible(t: SpType) -> bool:
    """serialize_static_config<T>::has_compatible (type_calculate.hpp:746)."""
    if isinstance(t, Compatible):
        return True
    if isinstance(t, Struct):
        return any(has_compatible(ft) for _, ft in t.fields)
    if isinstance(t, (Vector, Optional)):
        return has_compatible(t.elem)
    if isinstance(t, Expected):
        return has_compatible(t.value) or has_compatible(t.error)
    return False


class Variant(SpType):
    """std::variant<A, B, ...> (variant_t): wire [index:1][active
    alternative] (ref packer.hpp:389-398; decode: an index past the last
    alternative is invalid_buffer, unpacker.hpp:1278-1292); literal
    variant_t + the alternatives' literals + end (type_calculate.hpp:245-253);
    a container if any alternative holds one (type_calculate.hpp:785-815).
    Device record: the u32 active index, then every alternative's fields side
    by side (a decode writes only the active one's)."""

    def __init__(self, *alts: SpType):
        assert 0 < len(alts) < 256
        self.alts = alts
        self.name = "std::variant<" + ",".join(a.name for a in alts) + ">"
        self.config = DEFAULT

    def literal(self):
        return bytes([TID_VARIANT]) + b"".join(a.literal() for a in self.alts) + bytes([TID_END])

    @property
    def has_container(self):
        return any(a.has_container for a in self.alts)


class Array(SpType):
    """std::array<T, n> / T[n] (array_t): no length prefix on the wire."""

    def __init__(self, elem: SpType, n: int):
        assert n > 0
        self.elem, self.n = elem, n
        self.name = f"std::array<{elem.name},{n}>"
        self.size = elem.size * n
        self.align = elem.align
        self.config = DEFAULT

    def literal(self):
        return bytes([TID_ARRAY]) + self.elem.literal() + size_literal(self.n)

    @property
    def trivial(self):
        return self.elem.trivial

    @property
    def has_container(self):
        return self.elem.has_container


class Struct(SpType):
    """An aggregate: members in declaration order (visit_members)."""

    def __init__(self, name: str, fields: Sequence[Tuple[str, SpType]],
                 config: int = DEFAULT, alignas: int = 0, pack: int = 0):
        """alignas: alignas(N) on the struct; pack: #pragma pack(N) together
        with the user override struct_pack::pack_alignment_v<T> = N
        (ref alignment.hpp:72-122; tests/test_alignas.cpp)."""
        self.name = name
        self.fields = list(fields)
        self.config = config
        self._alignas = alignas
        self._pack = pack
        # C layout
        off = 0
        al = 1
        self.offsets = []
        for _, t in self.fields:
            a = min(t.align, pack) if pack else t.align
            off = (off + a - 1) // a * a
            self.offsets.append(off)
            off += t.size
            al = max(al, a)
        if alignas:
            al = max(al, alignas)
        self.align = al
        self.size = (off + al - 1) // al * al if self.fields else 1

    @property
    def trivial(self):
        return all(t.trivial and varint_tid(t, self.config) is None for _, t in self.fields)

    @property
    def trivial_ignoring_compatible(self):
        """is_trivial_serializable<T, true> (reflection.hpp:851-921)."""
        return all(isinstance(t, Compatible) or t.trivial for _, t in self.fields)

    @property
    def has_container(self):
        return any(t.has_container for _, t in self.fields)

    def literal(self):
        body = b"".join(bytes([varint_tid(t, self.config)]) if varint_tid(t, self.config)
                        else t.literal() for _, t in self.fields)
        if self.trivial:
            # pack_alignment_v (max member alignment_v) and alignment_v
            # (alignof) literals: type_calculate.hpp:232-239, alignment.hpp
            pack = self._pack or max((t.align for _, t in self.fields), default=1)
            return (bytes([TID_STRUCT]) + body + size_literal(pack) +
                    size_literal(self.align) + bytes([TID_END]))
        return bytes([TID_STRUCT]) + body + bytes([TID_END])


class Tuple(SpType):
    """serialize(a, b, ...) packs std::tuple<A, B, ...> (never trivial)."""

    def __init__(self, *elems: SpType):
        self.elems = elems
        self.name = "std::tuple<" + ",".join(e.name for e in elems) + ">"
        self.config = DEFAULT

    def literal(self):
        return (bytes([TID_STRUCT]) + b"".join(e.literal() for e in self.elems)
                + bytes([TID_END]))

    @property
    def has_container(self):
        return any(e.has_container for e in self.elems)


def get_type_code(*types: SpType) -> int:
    """struct_pack::get_type_code<Args...>() (ref struct_pack.hpp:75-92)."""
    t = types[0] if len(types) == 1 else Tuple(*types)
    return t.code()


def get_type_literal(*types: SpType) -> bytes:
    t = types[0] if len(types) == 1 else Tuple(*types)
    return t.root_literal()


# ---- config resolution (ref type_calculate.hpp:744-891) ------------------
def resolve_flags(msg: SpType, conf: int = DEFAULT, debug: bool = False) -> int:
    """SPK_MF_* flags for message type `msg` serialized with call-site
    sp_config `conf`. `debug` models a build without NDEBUG
    (serialize_static_config::has_type_literal, type_calculate.hpp:744-752)."""
    from . import _capi as C
    c = conf & 0b11
    if c == DEFAULT:
        c = msg.config & 0b11
    disable_head = c == DISABLE_ALL_META_INFO
    if disable_head and has_compatible(msg):  # a static_assert in the reference
        raise ValueError("compatible members need the hash head "
                         "(type_calculate.hpp:868-876)")
    if c == DEFAULT:
        type_lit = debug
    else:
        type_lit = c == ENABLE_TYPE_INFO
    flags = 0
    if not disable_head:
        flags |= C.SPK_MF_HASH_HEAD
        if type_lit:
            flags |= C.SPK_MF_TYPE_LITERAL
    if msg.has_container:
        flags |= C.SPK_MF_HAS_CONTAINER
    return flags


# ---- flattening into the device-record descriptor ------------------------
@dataclass
class SpanField:
    path: str
    elem: SpType
    count_off: int
    off_off: int
    sub: "Optional_[DeviceLayout]" = None  # ARRAY: the element record layout
    kind: str = ""  # "map" / "multimap" / "umap" / "set" / ...: an associative container


class ElemRecord(SpType):
    """The device record of a container element that is not trivially
    serializable (an SPK_OP_ARRAY heap holds these)."""

    def __init__(self, layout: "DeviceLayout"):
        self.layout = layout
        self.name = f"record<{layout.rtype.name}>"
        self.size = layout.stride
        self.align = 8
        self.config = DEFAULT


@dataclass
class DeviceLayout:
    """The flattened record: COPY / SPAN ops plus a numpy dtype of the
    device record (what spk_codec kernels read and write)."""
    rtype: SpType
    stride: int
    ops: List[Tuple[int, int, int, int]]  # (kind, rec_off, size, aux)
    spans: List[SpanField]
    np_fields: List[Tuple[str, str, int]]  # (name, dtype, offset)
    trivial: bool

    @property
    def dtype(self) -> np.dtype:
        if self.trivial:
            return np.dtype((np.void, self.stride))
        names = [n for n, _, _ in self.np_fields]
        fmts = [f for _, f, _ in self.np_fields]
        offs = [o for _, _, o in self.np_fields]
        return np.dtype({"names": names, "formats": fmts, "offsets": offs,
                         "itemsize": self.stride})


def _np_format(t: SpType) -> str:
    if isinstance(t, Fund):
        return t.npdt
    return f"V{t.size}"


def flatten(rtype: SpType) -> DeviceLayout:
    """Flatten a record type (ref packer.hpp:411-448 decides per member:
    trivially serializable → raw sizeof bytes incl. padding; container of
    trivially serializable → [count][raw elements])."""
    from . import _capi as C
    if rtype.trivial:
        return DeviceLayout(rtype, rtype.size, [(C.SPK_OP_COPY, 0, rtype.size, 0)],
                            [], [("raw", f"V{rtype.size}", 0)], True)
    if isinstance(rtype, Struct) and has_compatible(rtype) and rtype.trivial_ignoring_compatible:
        # packer.hpp:422-431 writes such a struct field by field WITH padding
        raise NotImplementedError(f"{rtype.name}: trivially serializable apart from "
                                  "compatible members is outside the flat record model")
    versions = sorted({ft.version for _, ft in getattr(rtype, "fields", [])
                       if isinstance(ft, Compatible)})
    ops: List[Tuple[int, int, int, int]] = []
    spans: List[SpanField] = []
    npf: List[Tuple[str, str, int]] = []
    cur = [0, 1]  # offset, max align

    def place(size: int, align: int) -> int:
        off = (cur[0] + align - 1) // align * align
        cur[0] = off + size
        cur[1] = max(cur[1], align)
        return off

    def visit(t: SpType, path: str):
        if t.trivial:
            off = place(t.size, t.align)
            ops.append((C.SPK_OP_COPY, off, t.size, 0))
            npf.append((path, _np_format(t), off))
        elif isinstance(t, (String, Vector)) and not t.elem.trivial:
            # container of non-trivially-serializable elements: SPK_OP_ARRAY
            # over the element's own flattened layout (packer.hpp:365-367)
            if has_compatible(t.elem):
                raise NotImplementedError(f"{path}: compatible members inside container "
                                          "elements are outside the flat record model")
            sub = flatten(t.elem)
            coff = place(4, 4)
            ooff = place(8, 8)
            ops.append((C.SPK_OP_ARRAY, coff, sub.stride, ooff))
            spans.append(SpanField(path, ElemRecord(sub), coff, ooff, sub,
                                   getattr(t, "kind", "")))
            npf.append((path + ".n", "<u4", coff))
            npf.append((path + ".off", "<u8", ooff))
            for op in (sub.ops if not sub.trivial else [(C.SPK_OP_COPY, 0, sub.stride, 0)]):
                ops.append(op)
            ops.append((C.SPK_OP_END, 0, 0, 0))
            for sp in sub.spans:
                spans.append(SpanField(f"{path}[].{sp.path}", sp.elem, sp.count_off, sp.off_off,
                                       sp.sub))
        elif isinstance(t, (String, Vector)):
            coff = place(4, 4)
            ooff = place(8, 8)
            ops.append((C.SPK_OP_SPAN, coff, t.elem.size, ooff))
            spans.append(SpanField(path, t.elem, coff, ooff, None, getattr(t, "kind", "")))
            npf.append((path + ".n", "<u4", coff))
            npf.append((path + ".off", "<u8", ooff))
        elif isinstance(t, Optional) and not t.elem.trivial:
            # SPK_OP_OPTGROUP: u32 has_value, U's fields inline (packer.hpp:
            # 382-388; unpacker.hpp:1251-1275 drops U's errc)
            ioff = place(4, 4)
            ops.append((C.SPK_OP_OPTGROUP, ioff, 1, 0))
            npf.append((path + ".has", "<u4", ioff))
            visit(t.elem, path + ".value")
            ops.append((C.SPK_OP_END, 0, 0, 0))
        elif isinstance(t, Expected):
            ioff = place(4, 4)
            ops.append((C.SPK_OP_OPTGROUP, ioff, 2, 0))
            npf.append((path + ".has", "<u4", ioff))
            if not isinstance(t.value, Monostate):
                visit(t.value, path + ".value")
            ops.append((C.SPK_OP_END, 0, 0, 0))
            if not isinstance(t.error, Monostate):
                visit(t.error, path + ".error")
            ops.append((C.SPK_OP_END, 0, 0, 0))
        elif isinstance(t, Optional):
            coff = place(4, 4)
            ooff = place(8, 8)
            ops.append((C.SPK_OP_OPTION, coff, t.elem.size, ooff))
            spans.append(SpanField(path, t.elem, coff, ooff))
            npf.append((path + ".n", "<u4", coff))
            npf.append((path + ".off", "<u8", ooff))
        elif isinstance(t, Compatible) and not t.elem.trivial:
            if path.count(".") or path.count("["):
                raise NotImplementedError(
                    f"{path}: compatible<{t.elem.name}> is only in the record model "
                    "as a member of the top-level record")
            ioff = place(4, 4)
            rank = versions.index(t.version)
            ops.append((C.SPK_OP_CGROUP | (rank << 8), ioff, 1, 0))
            npf.append((path + ".has", "<u4", ioff))
            visit(t.elem, path + ".value")
            ops.append((C.SPK_OP_END, 0, 0, 0))
        elif isinstance(t, Compatible):
            if path.count(".") or path.count("["):
                raise NotImplementedError(
                    f"{path}: compatible<{t.elem.name}> is only in the record model "
                    "as a member of the top-level record")
            coff = place(4, 4)
            ooff = place(8, 8)
            rank = versions.index(t.version)
            ops.append((C.SPK_OP_COMPAT | (rank << 8), coff, t.elem.size, ooff))
            spans.append(SpanField(path, t.elem, coff, ooff))
            npf.append((path + ".n", "<u4", coff))
            npf.append((path + ".off", "<u8", ooff))
        elif isinstance(t, Variant):
            ioff = place(4, 4)
            ops.append((C.SPK_OP_VARIANT, ioff, len(t.alts), 0))
            npf.append((path + ".index", "<u4", ioff))
            for a, alt in enumerate(t.alts):
                if not isinstance(alt, Monostate):
                    visit(alt, f"{path}.{a}")
                ops.append((C.SPK_OP_END, 0, 0, 0))
        elif isinstance(t, VarInt):
            off = place(t.size, t.size)
            ops.append((C.SPK_OP_VARINT, off, t.size,
                        C.SPK_VARINT_ZIGZAG if t.zigzag else 0))
            npf.append((path, t.npdt, off))
        elif isinstance(t, Struct) and t.config & (ENCODING_WITH_VARINT | USE_FAST_VARINT):
            if path:
                raise NotImplementedError(f"{path}: varint sp_config bits are only in the "
                                          "flat record model on the top-level record")
            for fname, ft in t.fields:
                tid = varint_tid(ft, t.config)
                if tid is None:
                    visit(ft, fname)
                    continue
                off = place(ft.size, ft.size)
                npf.append((fname, ft.npdt, off))
                signed = tid in (TID_VINT32, TID_VINT64, TID_VINT32 + 4, TID_VINT64 + 4)
                if t.config & USE_FAST_VARINT:  # the record's fast-varint group
                    ops.append((C.SPK_OP_FVAR, off, ft.size, C.SPK_FVAR_SIGNED if signed else 0))
                elif isinstance(ft, VarInt):
                    ops.append((C.SPK_OP_VARINT, off, ft.size,
                                C.SPK_VARINT_ZIGZAG if ft.zigzag else 0))
                else:  # plain (u)int under ENCODING_WITH_VARINT: v = t, no zigzag
                    ops.append((C.SPK_OP_VARINT, off, ft.size,
                                C.SPK_VARINT_SEXT if (signed and ft.size == 4) else 0))
        elif isinstance(t, Struct):
            for fname, ft in t.fields:
                visit(ft, f"{path}.{fname}" if path else fname)
        elif isinstance(t, Array):
            for i in range(t.n):
                visit(t.elem, f"{path}[{i}]")
        else:
            raise NotImplementedError(f"{path}: {t.name} not in flat model")

    visit(rtype, "" if isinstance(rtype, Struct) else "value")
    if len(spans) > C.SPK_MAX_SPANS:
        raise NotImplementedError("too many variable-length members")
    if (sum(op[0] == C.SPK_OP_VARINT for op in ops) > C.SPK_MAX_VARINTS or
            sum(op[0] == C.SPK_OP_FVAR for op in ops) > C.SPK_MAX_VARINTS):
        raise NotImplementedError("too many varint members")
    if len(ops) > C.SPK_MAX_OPS:
        raise NotImplementedError("too many layout ops")
    # merge COPY runs contiguous in the record (always contiguous on the wire);
    # never across an ARRAY's element ops (they address another record)
    merged: List[Tuple[int, int, int, int]] = []
    depth, last_depth = 0, -1
    for op in ops:
        if (merged and op[0] == C.SPK_OP_COPY and merged[-1][0] == C.SPK_OP_COPY
                and last_depth == depth and merged[-1][1] + merged[-1][2] == op[1]):
            k, o, s, a = merged[-1]
            merged[-1] = (k, o, s + op[2], a)
        else:
            merged.append(op)
        last_depth = depth
        if op[0] == C.SPK_OP_ARRAY:
            depth += 1
            last_depth = -1
        elif op[0] == C.SPK_OP_END:
            depth -= 1
            last_depth = -1
    # non-trivial device records are 8-byte aligned (the kernels read span
    # offsets as u64; spk_layout_check rejects other strides), also when the
    # record has only 4-byte members and varints
    align = max(cur[1], 8)
    stride = (cur[0] + align - 1) // align * align
    return DeviceLayout(rtype, stride, merged, spans, npf, False)


def _walk_levels(dev: DeviceLayout):
    """(op, ARRAY nesting, group nesting) for every op but the ENDs: the
    ops of an ARRAY element repeat per element; the ops of a VARIANT /
    OPTGROUP / CGROUP group sit in the same record, present or not."""
    from . import _capi as C
    stack = []  # [kind, ENDs still to close]
    for op in dev.ops:
        k = op[0] & 0xFF
        arr = sum(1 for s in stack if s[0] == C.SPK_OP_ARRAY)
        grp = len(stack) - arr
        if k == C.SPK_OP_END:
            stack[-1][1] -= 1
            if stack[-1][1] == 0:
                stack.pop()
            continue
        yield op, arr, grp
        if k == C.SPK_OP_ARRAY:
            stack.append([k, 1])
        elif k in (C.SPK_OP_VARIANT, C.SPK_OP_OPTGROUP, C.SPK_OP_CGROUP):
            stack.append([k, op[2]])


def min_record_wire_bytes(dev: DeviceLayout) -> int:
    """Fewest wire bytes one top-level record can take (each container count
    >= 1 byte; an absent optional / a variant's index 1 byte; compatible
    members none: an older writer has none; the record's fast-varint group
    only its bitset of ceil((n + 2) / 8) bytes, since zero members take no
    bytes, packer.hpp:193-212): bounds a decode's record capacity by the
    wire length."""
    from . import _capi as C
    total = 0
    n_fvar = 0
    for (k, _, sz, _), arr, grp in _walk_levels(dev):
        k &= 0xFF
        if arr or grp or k in (C.SPK_OP_COMPAT, C.SPK_OP_CGROUP):
            continue
        if k == C.SPK_OP_FVAR:
            n_fvar += 1
            continue
        total += sz if k == C.SPK_OP_COPY else 1
    if n_fvar:
        total += (n_fvar + 2 + 7) // 8
    return max(total, 1)


def heap_caps_for_wire(dev: DeviceLayout, wire_len: int, rec_cap: int) -> List[int]:
    """Per-heap element capacities no decode of `wire_len` bytes can exceed:
    a SPAN's elements take their size in wire bytes; an ARRAY element and an
    OPTION inside an ARRAY element at least one byte; an OPTION / compatible
    member of the top-level record one per record."""
    from . import _capi as C
    caps = []
    for (k, _, sz, _), arr, grp in _walk_levels(dev):
        k &= 0xFF
        if k == C.SPK_OP_SPAN:
            caps.append(wire_len // max(sz, 1) + 1)
        elif k == C.SPK_OP_OPTION:
            caps.append(rec_cap if arr == 0 else wire_len + 1)
        elif k == C.SPK_OP_COMPAT:
            caps.append(rec_cap)
        elif k == C.SPK_OP_ARRAY:
            caps.append(wire_len + 1)
    return caps
