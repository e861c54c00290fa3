// layout.hpp — host C++20 reflection -> spk_layout descriptor, and the
// host-object <-> device-record marshalling used when a batch starts or ends
// in host memory (coro_rpc socket buffers).
//
// Device record of a record type T:
//   * T trivially serializable (reference reflection.hpp:851-922): the device
//     record IS T, byte for byte (padding included) — one COPY op.
//   * otherwise members are flattened in declaration order (reference
//     packer.hpp:432-447): trivially serializable members become COPY ops at
//     a C-like offset of the device record; std::string / std::vector<U>
//     (U trivially serializable) become a SPAN op {u32 count; u64 element
//     offset into that member's heap}; std::optional<U> (U trivially
//     serializable) an OPTION op with the same fields and a count of 0/1.
//     Nested non-trivial aggregates are flattened inline.
// This is the same flattening as yalantinglibs_amd/schema.py:flatten, so
// Python and C++ front ends produce identical descriptors.
#pragma once
#include <cstring>
#include <new>
#include <stdexcept>
#include <variant>
#include <vector>

#include "../../spk_codec.h"
#include "type_code.hpp"

namespace struct_pack::gpu {
namespace detail {

struct layout_builder {
  spk_layout L{};
  uint32_t off = 0, align = 1, spans = 0, vars = 0, fvars = 0;
  uint32_t depth = 0;           // record nesting (1: members of the top-level record)
  bool element = false;         // building a container element's record
  uint64_t vers[SPK_MAX_OPS];   // sorted distinct compatible versions of the record
  uint32_t n_vers = 0;
  uint32_t place(uint32_t size, uint32_t al) {
    off = (off + al - 1) / al * al;
    const uint32_t o = off;
    off += size;
    if (al > align) align = al;
    return o;
  }
  void push(const spk_op &o) {
    if (L.n_ops >= SPK_MAX_OPS) throw std::length_error("struct_pack: too many layout ops");
    L.ops[L.n_ops++] = o;
  }
  void copy(uint32_t size, uint32_t al) {
    const uint32_t o = place(size, al);
    if (L.n_ops && L.ops[L.n_ops - 1].kind == SPK_OP_COPY &&
        L.ops[L.n_ops - 1].rec_off + L.ops[L.n_ops - 1].size == o) {
      L.ops[L.n_ops - 1].size += size;  // merge runs contiguous in the record
      return;
    }
    push(spk_op{SPK_OP_COPY, o, size, 0});
  }
  void count_var(uint32_t &n) {
    if (++n > SPK_MAX_VARINTS) throw std::length_error("struct_pack: too many varint members");
  }
  void varint(uint32_t size, uint32_t aux) {
    const uint32_t o = place(size, size);
    count_var(vars);
    push(spk_op{SPK_OP_VARINT, o, size, aux});
  }
  void fvar(uint32_t size, uint32_t aux) {
    const uint32_t o = place(size, size);
    count_var(fvars);
    push(spk_op{SPK_OP_FVAR, o, size, aux});
  }
  void span(uint32_t esz, uint32_t kind = SPK_OP_SPAN) {
    const uint32_t c = place(4, 4), a = place(8, 8);
    if (++spans > SPK_MAX_SPANS)
      throw std::length_error("struct_pack: too many variable-length members");
    push(spk_op{kind, c, esz, a});
  }
  uint32_t index(uint32_t kind, uint32_t groups) {  // VARIANT / OPTGROUP / CGROUP head
    const uint32_t o = place(4, 4);
    push(spk_op{kind, o, groups, 0});
    return o;
  }
  void end() { push(spk_op{SPK_OP_END, 0, 0, 0}); }
};

template <typename T>
void flatten_into(layout_builder &b);

// a container of non-trivially-serializable elements E (packer.hpp:365-367):
// SPK_OP_ARRAY {count, element stride, element offset} over E's own
// flattened record, closed by END; E's heaps follow the ARRAY's
template <typename E>
void flatten_array(layout_builder &b) {
  layout_builder sb;
  sb.element = true;
  flatten_into<E>(sb);
  const uint32_t al = sb.align < 8 ? 8 : sb.align;
  const uint32_t stride = (sb.off + al - 1) / al * al;
  const uint32_t c = b.place(4, 4), a = b.place(8, 8);
  if ((b.spans += 1 + sb.spans) > SPK_MAX_SPANS)
    throw std::length_error("struct_pack: too many variable-length members");
  b.vars += sb.vars;
  b.fvars += sb.fvars;
  if (b.vars > SPK_MAX_VARINTS || b.fvars > SPK_MAX_VARINTS)
    throw std::length_error("struct_pack: too many varint members");
  b.push(spk_op{SPK_OP_ARRAY, c, stride, a});
  for (uint32_t i = 0; i < sb.L.n_ops; ++i) b.push(sb.L.ops[i]);
  b.end();
}

template <typename A>
void flatten_alternative(layout_builder &b) {
  if constexpr (!is_monostate_v<A>) flatten_into<A>(b);  // monostate: an empty group
  b.end();
}
template <typename... A>
void flatten_variant(layout_builder &b, std::variant<A...> *) {
  // std::variant (packer.hpp:389-398): u32 index, every alternative's fields
  // side by side, one END-closed group each
  b.index(SPK_OP_VARIANT, sizeof...(A));
  (flatten_alternative<A>(b), ...);
}

// the members of a record whose sp_config makes members varints (top-level
// record only, like the Python mirror): FVAR ops under USE_FAST_VARINT,
// VARINT ops otherwise (packer.hpp:152-235, varint.hpp:249-259)
template <typename F, uint64_t cfg>
void flatten_config_member(layout_builder &b) {
  constexpr uint8_t tid = varint_tid<F, cfg>();
  if constexpr (tid == 0) {
    flatten_into<F>(b);
  } else {
    using V = std::conditional_t<is_varint_v<F>, typename varint_traits<F>::value_type, F>;
    constexpr uint8_t base = (cfg & kCfgUseFastVarint) ? tid - 4 : tid;
    constexpr bool is_signed = base == TID_VINT32 || base == TID_VINT64;
    if constexpr ((cfg & kCfgUseFastVarint) != 0) {
      b.fvar(sizeof(V), is_signed ? SPK_FVAR_SIGNED : 0u);
    } else if constexpr (is_varint_v<F>) {
      b.varint(sizeof(V), varint_traits<F>::zigzag ? SPK_VARINT_ZIGZAG : 0u);
    } else {  // plain (u)int under ENCODING_WITH_VARINT: v = t, no zigzag
      b.varint(sizeof(V), (is_signed && sizeof(V) == 4) ? SPK_VARINT_SEXT : 0u);
    }
  }
}
template <typename M, uint64_t cfg, std::size_t... I>
void flatten_config_members(layout_builder &b, std::index_sequence<I...>) {
  (flatten_config_member<std::tuple_element_t<I, M>, cfg>(b), ...);
}

template <typename T>
void flatten_into(layout_builder &b) {
  if constexpr (is_trivially_serializable<T>()) {
    b.copy(sizeof(T), alignof(T));
  } else if constexpr (is_trivial_view_v<T>) {  // T's bytes (packer.hpp:243-245)
    using E = typename trivial_view_traits<T>::value_type;
    b.copy(sizeof(E), alignof(E));
  } else if constexpr (is_varint_v<T>) {
    b.varint(sizeof(typename varint_traits<T>::value_type),
             varint_traits<T>::zigzag ? SPK_VARINT_ZIGZAG : 0u);
  } else if constexpr (is_string_v<T>) {
    b.span(sizeof(string_char_t<T>));
  } else if constexpr (is_container_v<T>) {
    using E = elem_t<T>;
    if constexpr (is_trivially_serializable<E>())
      b.span(sizeof(E));
    else
      flatten_array<E>(b);
  } else if constexpr (is_std_optional<T>::value) {
    using E = opt_value_t<T>;
    if constexpr (is_trivially_serializable<E>()) {
      b.span(sizeof(E), SPK_OP_OPTION);
    } else {  // SPK_OP_OPTGROUP: u32 has_value, E's fields inline (packer.hpp:382-388)
      b.index(SPK_OP_OPTGROUP, 1);
      flatten_into<E>(b);
      b.end();
    }
  } else if constexpr (is_compat_v<T>) {
    using E = remove_cvref_t<typename T::value_type>;
    if (b.depth != 1 || b.element)
      throw std::logic_error("MI355X codec: compatible members only at the top level");
    uint32_t rank = 0;
    while (b.vers[rank] != compat_traits<T>::version) ++rank;
    if constexpr (is_trivially_serializable<E>()) {
      b.span(sizeof(E), SPK_OP_COMPAT | rank << 8);
    } else {  // SPK_OP_CGROUP: [has][E] in its version pass, E's fields inline
      b.index(SPK_OP_CGROUP | rank << 8, 1);
      flatten_into<E>(b);
      b.end();
    }
  } else if constexpr (is_std_variant<T>::value) {
    flatten_variant(b, static_cast<T *>(nullptr));
  } else if constexpr (is_std_array<T>::value) {
    for (std::size_t i = 0; i < std::tuple_size_v<T>; ++i)
      flatten_into<typename T::value_type>(b);
  } else {
    static_assert(is_record_v<T>, "MI355X codec: member type outside the record model");
    using M = members_tuple_t<T>;
    constexpr uint64_t cfg = type_config<T>() & kCfgVarintBits;
    ++b.depth;
    if constexpr (cfg != 0) {
      if (b.depth != 1 || b.element)
        throw std::logic_error(
            "MI355X codec: varint sp_config bits only on the top-level record");
      flatten_config_members<M, cfg>(b, std::make_index_sequence<std::tuple_size_v<M>>{});
    } else {
      [&]<std::size_t... I>(std::index_sequence<I...>) {
        (flatten_into<std::tuple_element_t<I, M>>(b), ...);
      }(std::make_index_sequence<std::tuple_size_v<M>>{});
    }
    --b.depth;
  }
}

// the sorted distinct versions of T's compatible members (type_calculate.hpp:
// 531-556: the order of the version passes)
template <typename F>
void add_version(layout_builder &b) {
  if constexpr (is_compat_v<F>) {
    constexpr uint64_t v = compat_traits<F>::version;
    uint32_t j = 0;
    while (j < b.n_vers && b.vers[j] < v) ++j;
    if (j < b.n_vers && b.vers[j] == v) return;
    for (uint32_t k = b.n_vers; k > j; --k) b.vers[k] = b.vers[k - 1];
    b.vers[j] = v;
    ++b.n_vers;
  }
}
template <typename M, std::size_t... I>
void add_versions(layout_builder &b, std::index_sequence<I...>) {
  (add_version<std::tuple_element_t<I, M>>(b), ...);
}
template <typename T>
void collect_versions(layout_builder &b) {
  if constexpr (is_record_v<T> && !is_trivially_serializable<T>()) {
    using M = members_tuple_t<T>;
    add_versions<M>(b, std::make_index_sequence<std::tuple_size_v<M>>{});
  }
}

inline void fill_fmt(spk_msgfmt &f, uint32_t code, uint32_t flags, const lit_t &lit) {
  f.code = code;
  f.flags = flags;
  f.literal_len = static_cast<uint32_t>(lit.n);
  for (std::size_t i = 0; i < lit.n && i < SPK_MAX_LITERAL; ++i) f.literal[i] = lit.d[i];
}

// sp_config resolution (type_calculate.hpp:744-891): call-site conf first,
// then the message type's own config; DEFAULT -> type literal iff !NDEBUG.
template <typename Msg, uint64_t conf>
constexpr uint32_t msg_flags() {
  uint64_t c = conf & 0b11;
  if (c == sp_config::DEFAULT) c = type_config<Msg>() & 0b11;
  const bool no_head = c == sp_config::DISABLE_ALL_META_INFO;
#ifdef NDEBUG
  constexpr bool debug_literal = false;
#else
  constexpr bool debug_literal = true;
#endif
  const bool lit = c == sp_config::DEFAULT ? debug_literal : c == sp_config::ENABLE_TYPE_INFO;
  uint32_t f = 0;
  if (!no_head) {
    f |= SPK_MF_HASH_HEAD;
    if (lit) f |= SPK_MF_TYPE_LITERAL;
  }
  if (has_container<Msg>()) f |= SPK_MF_HAS_CONTAINER;
  return f;
}

}  // namespace detail

namespace detail {
// the message type whose code and header a record type's one-record
// messages carry: boxed<M> -> M, else the record itself
template <typename T>
struct message_type {
  using type = T;
};
template <typename M>
struct message_type<boxed<M>> {
  using type = M;
};
template <typename T>
using message_type_t = typename message_type<T>::type;
}  // namespace detail

// Descriptor of record type T for the batch codec (cacheable, immutable).
template <typename T, uint64_t conf = sp_config::DEFAULT>
spk_layout make_spk_layout() {
  using namespace detail;
  layout_builder b;
  b.L.abi = SPK_ABI_VERSION;
  collect_versions<T>(b);
  flatten_into<T>(b);
  if constexpr (is_trivially_serializable<T>()) {
    b.L.flags = SPK_LAYOUT_TRIVIAL;
    b.L.rec_stride = sizeof(T);
  } else {
    // non-trivial device records are 8-byte aligned (the kernels read span
    // offsets as u64): a record of 4-byte members and varints rounds up too
    const uint32_t al = b.align < 8 ? 8 : b.align;
    b.L.rec_stride = (b.off + al - 1) / al * al;
    // a record that is not trivially serializable but has fixed-size members
    // only (std::tuple<int, bool>, a YLT_REFL type of plain members): its
    // wire is the members' bytes back to back (packer.hpp:432-447), so its
    // device record is that packed form, one COPY -- the marshalling writes
    // a COPY op's bytes in sequence -- and it takes the trivial kernels
    bool fixed = true;
    uint32_t bytes = 0;
    for (uint32_t i = 0; i < b.L.n_ops; ++i) {
      fixed = fixed && b.L.ops[i].kind == SPK_OP_COPY;
      bytes += b.L.ops[i].size;
    }
    if (fixed && bytes) {
      b.L.n_ops = 1;
      b.L.ops[0] = spk_op{SPK_OP_COPY, 0, bytes, 0};
      b.L.flags = SPK_LAYOUT_TRIVIAL;
      b.L.rec_stride = bytes;
    }
  }
  using M = message_type_t<T>;
  fill_fmt(b.L.fmt_vector, get_type_code<std::vector<M>>(),
           msg_flags<std::vector<M>, conf>(), get_type_literal<std::vector<M>>());
  fill_fmt(b.L.fmt_one, get_type_code<M>(), msg_flags<M, conf>(), get_type_literal<M>());
  return b.L;
}

namespace detail {

// ---- walking a descriptor -------------------------------------------------
// ops that own a heap, numbered in op order at every level (SPAN / OPTION /
// COMPAT: the member's values; ARRAY: the element records)
inline bool op_has_heap(const spk_op &o) {
  const uint32_t k = SPK_OP_KIND(o.kind);
  return k == SPK_OP_SPAN || k == SPK_OP_OPTION || k == SPK_OP_COMPAT || k == SPK_OP_ARRAY;
}
// END-closed groups an op opens
inline uint32_t op_groups(const spk_op &o) {
  const uint32_t k = SPK_OP_KIND(o.kind);
  if (k == SPK_OP_ARRAY || k == SPK_OP_CGROUP) return 1;
  if (k == SPK_OP_VARIANT || k == SPK_OP_OPTGROUP) return o.size;
  return 0;
}
// i = the first op of a group: the op after its END; heaps inside added to nh
inline uint32_t skip_group(const spk_layout *L, uint32_t i, uint32_t &nh) {
  while (SPK_OP_KIND(L->ops[i].kind) != SPK_OP_END) {
    nh += op_has_heap(L->ops[i]) ? 1u : 0u;
    const uint32_t g = op_groups(L->ops[i]);
    ++i;
    for (uint32_t j = 0; j < g; ++j) i = skip_group(L, i, nh);
  }
  return i + 1;
}

// Per-heap element capacities no decode of `wire_len` bytes into at most
// `rec_cap` records can exceed (the Python mirror's heap_caps_for_wire): a
// SPAN element takes its size in wire bytes, an ARRAY element and an OPTION
// inside one at least a byte, an OPTION / COMPAT of the top-level record one
// per record. Also: the fewest wire bytes one record takes.
inline std::vector<uint64_t> heap_caps_for_wire(const spk_layout &L, uint64_t wire_len,
                                                uint64_t rec_cap) {
  std::vector<uint64_t> caps;
  uint32_t stack[SPK_MAX_OPS][2];  // [is ARRAY, ENDs still to close]
  uint32_t sp = 0;
  for (uint32_t i = 0; i < L.n_ops; ++i) {
    const spk_op &o = L.ops[i];
    const uint32_t k = SPK_OP_KIND(o.kind);
    if (k == SPK_OP_END) {
      if (--stack[sp - 1][1] == 0) --sp;
      continue;
    }
    uint32_t arr = 0;
    for (uint32_t j = 0; j < sp; ++j) arr += stack[j][0];
    if (k == SPK_OP_SPAN) caps.push_back(wire_len / (o.size ? o.size : 1) + 1);
    else if (k == SPK_OP_OPTION) caps.push_back(arr == 0 ? rec_cap : wire_len + 1);
    else if (k == SPK_OP_COMPAT) caps.push_back(rec_cap);
    else if (k == SPK_OP_ARRAY) caps.push_back(wire_len + 1);
    if (op_groups(o)) {
      stack[sp][0] = k == SPK_OP_ARRAY;
      stack[sp][1] = op_groups(o);
      ++sp;
    }
  }
  return caps;
}
// Fewest wire bytes of one top-level record: a container count or an
// optional / variant tag >= 1 byte, compatible members none, and the
// record's fast-varint group only its bitset of ceil((n + 2) / 8) bytes (zero
// members take no bytes, packer.hpp:193-212). A true lower bound, so the
// record capacity wire_len / min + 1 holds every decodable message.
inline uint64_t min_record_wire_bytes(const spk_layout &L) {
  uint64_t total = 0, n_fvar = 0;
  uint32_t stack[SPK_MAX_OPS], sp = 0;  // groups (and ARRAY elements) open
  for (uint32_t i = 0; i < L.n_ops; ++i) {
    const spk_op &o = L.ops[i];
    const uint32_t k = SPK_OP_KIND(o.kind);
    if (k == SPK_OP_END) {
      if (--stack[sp - 1] == 0) --sp;
      continue;
    }
    if (!sp && k == SPK_OP_FVAR) ++n_fvar;
    else if (!sp && k != SPK_OP_COMPAT && k != SPK_OP_CGROUP)
      total += k == SPK_OP_COPY ? o.size : 1;
    if (op_groups(o)) stack[sp++] = op_groups(o);
  }
  if (n_fvar) total += (n_fvar + 2 + 7) / 8;
  return total ? total : 1;
}

// ---- host object <-> device record ----------------------------------------
struct marshal_state {
  const spk_layout *L;
  uint8_t *rec;                                   // current device record
  uint32_t op = 0, within = 0;                    // walking the op list
  std::vector<std::vector<uint8_t>> *heaps;       // one per heap
  uint32_t span = 0;                              // next heap
};

inline void put_copy(marshal_state &s, const void *src, uint32_t size) {
  // COPY ops may merge several members: advance through the current op
  const spk_op &op = s.L->ops[s.op];
  std::memcpy(s.rec + op.rec_off + s.within, src, size);
  s.within += size;
  if (s.within == op.size) {
    ++s.op;
    s.within = 0;
  }
}
inline void put_u32(uint8_t *rec, uint32_t off, uint32_t v) { std::memcpy(rec + off, &v, 4); }
inline void put_u64(uint8_t *rec, uint32_t off, uint64_t v) { std::memcpy(rec + off, &v, 8); }

template <typename T>
void to_device(const T &v, marshal_state &s);

// a trivially serializable element's bytes (a map's pair built in zeroed
// storage, so padding bytes are zero)
template <typename E, typename X>
void append_raw(std::vector<uint8_t> &heap, const X &x) {
  if constexpr (is_std_pair<E>::value) {
    alignas(E) unsigned char buf[sizeof(E)] = {};
    E *p = ::new (static_cast<void *>(buf)) E(x.first, x.second);
    const auto *b = reinterpret_cast<const uint8_t *>(p);
    heap.insert(heap.end(), b, b + sizeof(E));
    p->~E();
  } else {
    const auto *b = reinterpret_cast<const uint8_t *>(&x);
    heap.insert(heap.end(), b, b + sizeof(E));
  }
}

// the ops after a group head (OPTGROUP / CGROUP / an ARRAY element): value v
// marshalled into record `rec`; the state then continues after the group
template <typename V>
void put_group(const V *v, marshal_state &s, uint8_t *rec) {
  const uint32_t first = s.op + 1, h0 = s.span;
  uint32_t nh = 0;
  const uint32_t next = skip_group(s.L, first, nh);
  if (v) {
    marshal_state g{s.L, rec, first, 0, s.heaps, h0};
    to_device(*v, g);
  }
  s.op = next;
  s.span = h0 + nh;
}

template <std::size_t I, typename Var>
void put_alternative(const Var &v, marshal_state &s, uint32_t first, uint32_t h0) {
  if constexpr (I < std::variant_size_v<Var>) {
    if (v.index() == I) {
      if constexpr (!is_monostate_v<std::variant_alternative_t<I, Var>>) {
        marshal_state g{s.L, s.rec, first, 0, s.heaps, h0};
        to_device(std::get<I>(v), g);
      }
      return;
    }
    uint32_t nh = 0;
    const uint32_t nxt = skip_group(s.L, first, nh);
    put_alternative<I + 1>(v, s, nxt, h0 + nh);
  }
}

template <typename T>
void to_device(const T &v, marshal_state &s) {
  if constexpr (is_trivially_serializable<T>()) {
    put_copy(s, &v, sizeof(T));
  } else if constexpr (is_trivial_view_v<T>) {
    put_copy(s, &v.get(), sizeof(typename trivial_view_traits<T>::value_type));
  } else if constexpr (is_varint_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    const typename varint_traits<T>::value_type x = v;
    std::memcpy(s.rec + op.rec_off, &x, op.size);
  } else if constexpr (is_string_v<T> || is_container_v<T>) {
    using E = std::conditional_t<is_string_v<T>, string_char_t<T>, elem_t<T>>;
    const spk_op &op = s.L->ops[s.op];
    const uint32_t h = s.span;
    const uint32_t cnt = static_cast<uint32_t>(v.size());
    const uint64_t base = (*s.heaps)[h].size();
    put_u32(s.rec, op.rec_off, cnt);
    put_u64(s.rec, op.aux, base / op.size);
    if constexpr (is_trivially_serializable<E>()) {  // SPAN: the raw elements
      auto &heap = (*s.heaps)[h];
      if constexpr (is_string_v<T> || is_contiguous_v<T>) {
        const auto *p = reinterpret_cast<const uint8_t *>(v.data());
        heap.insert(heap.end(), p, p + static_cast<std::size_t>(cnt) * op.size);
      } else {
        for (const auto &e : v) append_raw<E>(heap, e);
      }
      ++s.op;
      ++s.span;
    } else {  // ARRAY: element records in heap h, their heaps after it
      (*s.heaps)[h].resize(base + static_cast<std::size_t>(cnt) * op.size, 0);
      const uint32_t first = s.op + 1;
      uint32_t nh = 0;
      const uint32_t next = skip_group(s.L, first, nh);
      std::size_t j = 0;
      for (const auto &e : v) {
        uint8_t *rec = (*s.heaps)[h].data() + base + j++ * op.size;  // other heaps grow only
        marshal_state g{s.L, rec, first, 0, s.heaps, h + 1};
        if constexpr (is_map_v<T>) {
          const E pe(e.first, e.second);
          to_device(pe, g);
        } else {
          to_device(e, g);
        }
      }
      s.op = next;
      s.span = h + 1 + nh;
    }
  } else if constexpr (is_std_optional<T>::value || is_compat_v<T>) {
    using E = opt_value_t<T>;
    const spk_op &op = s.L->ops[s.op];
    const uint32_t cnt = opt_has(v) ? 1u : 0u;
    if constexpr (is_trivially_serializable<E>()) {  // OPTION / COMPAT: heap value
      auto &heap = (*s.heaps)[s.span++];
      ++s.op;
      put_u32(s.rec, op.rec_off, cnt);
      put_u64(s.rec, op.aux, heap.size() / op.size);
      if (cnt) append_raw<E>(heap, *v);
    } else {  // OPTGROUP / CGROUP: has_value, the value's fields inline
      put_u32(s.rec, op.rec_off, cnt);
      put_group<E>(cnt ? &*v : nullptr, s, s.rec);
    }
  } else if constexpr (is_std_variant<T>::value) {
    const spk_op &op = s.L->ops[s.op];
    put_u32(s.rec, op.rec_off, static_cast<uint32_t>(v.index()));
    put_alternative<0>(v, s, s.op + 1, s.span);
    uint32_t i = s.op + 1, nh = 0;
    for (uint32_t g = 0; g < op.size; ++g) i = skip_group(s.L, i, nh);
    s.op = i;
    s.span += nh;
  } else if constexpr (is_std_array<T>::value) {
    for (const auto &e : v) to_device(e, s);
  } else {
    constexpr uint64_t cfg = type_config<T>() & kCfgVarintBits;
    std::apply(
        [&](const auto &...m) {
          (
              [&](const auto &x) {
                using F = remove_cvref_t<decltype(x)>;
                if constexpr (cfg != 0 && !is_varint_v<F> && varint_tid<F, cfg>() != 0) {
                  const spk_op &op = s.L->ops[s.op++];  // a plain integer as a varint
                  std::memcpy(s.rec + op.rec_off, &x, sizeof(F));
                } else {
                  to_device(x, s);
                }
              }(m),
              ...);
        },
        tie_members(v));
  }
}

struct unmarshal_state {
  const spk_layout *L;
  const uint8_t *rec;
  uint32_t op = 0, within = 0;
  const uint8_t *const *heaps;
  uint32_t span = 0;
};

inline void get_copy(unmarshal_state &s, void *dst, uint32_t size) {
  const spk_op &op = s.L->ops[s.op];
  std::memcpy(dst, s.rec + op.rec_off + s.within, size);
  s.within += size;
  if (s.within == op.size) {
    ++s.op;
    s.within = 0;
  }
}
inline uint32_t get_u32(const uint8_t *rec, uint32_t off) {
  uint32_t v;
  std::memcpy(&v, rec + off, 4);
  return v;
}
inline uint64_t get_u64(const uint8_t *rec, uint32_t off) {
  uint64_t v;
  std::memcpy(&v, rec + off, 8);
  return v;
}

template <typename T>
void from_device(T &v, unmarshal_state &s);

// insert a decoded element the way the reference's decoder does (unpacker.hpp:
// 983-1226): push_back for sequences, emplace for sets / multisets, try_emplace
// for maps (a repeated key keeps the first value), emplace for multimaps
template <typename T, typename E>
void add_element(T &c, E &&e) {
  if constexpr (is_map_v<T>)
    c.emplace(std::move(e.first), std::move(e.second));
  else if constexpr (is_set_v<T>)
    c.emplace(std::move(e));
  else
    c.push_back(std::move(e));
}

template <std::size_t I, typename Var>
void get_alternative(Var &v, unmarshal_state &s, uint32_t idx, uint32_t first, uint32_t h0) {
  if constexpr (I < std::variant_size_v<Var>) {
    if (idx == I) {
      auto &a = v.template emplace<I>();
      if constexpr (!is_monostate_v<std::variant_alternative_t<I, Var>>) {
        unmarshal_state g{s.L, s.rec, first, 0, s.heaps, h0};
        from_device(a, g);
      }
      return;
    }
    uint32_t nh = 0;
    const uint32_t nxt = skip_group(s.L, first, nh);
    get_alternative<I + 1>(v, s, idx, nxt, h0 + nh);
  }
}

template <typename T>
void from_device(T &v, unmarshal_state &s) {
  if constexpr (is_trivially_serializable<T>()) {
    get_copy(s, &v, sizeof(T));
  } else if constexpr (is_trivial_view_v<T>) {
    // the view points into the decoded host record (kept by the codec until
    // this thread's next decode of the type; the reference's view points
    // into its input buffer, unpacker.hpp:787-800)
    using E = typename trivial_view_traits<T>::value_type;
    const spk_op &op = s.L->ops[s.op];
    v.set(*reinterpret_cast<const E *>(s.rec + op.rec_off + s.within));
    s.within += sizeof(E);
    if (s.within == op.size) {
      ++s.op;
      s.within = 0;
    }
  } else if constexpr (is_varint_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    typename varint_traits<T>::value_type x;
    std::memcpy(&x, s.rec + op.rec_off, op.size);
    v = x;
  } else if constexpr (is_string_v<T> || is_container_v<T>) {
    using E = std::conditional_t<is_string_v<T>, string_char_t<T>, elem_t<T>>;
    const spk_op &op = s.L->ops[s.op];
    const uint32_t h = s.span;
    const uint32_t cnt = get_u32(s.rec, op.rec_off);
    const uint64_t eoff = get_u64(s.rec, op.aux);
    const uint8_t *src = s.heaps[h] + eoff * op.size;
    if constexpr (is_trivially_serializable<E>()) {
      if constexpr (is_string_view_v<T> || is_std_span<T>::value) {
        // views alias the decoded heap (the reference's views alias the input)
        v = T(reinterpret_cast<typename T::const_pointer>(src), cnt);
      } else if constexpr (is_string_v<T> || is_contiguous_v<T>) {
        v.resize(cnt);
        if (cnt) std::memcpy(v.data(), src, static_cast<std::size_t>(cnt) * op.size);
      } else {
        v.clear();
        for (uint32_t j = 0; j < cnt; ++j) {
          E e;
          std::memcpy(static_cast<void *>(&e), src + static_cast<std::size_t>(j) * op.size,
                      sizeof(E));
          add_element(v, std::move(e));
        }
      }
      ++s.op;
      ++s.span;
    } else {
      const uint32_t first = s.op + 1;
      uint32_t nh = 0;
      const uint32_t next = skip_group(s.L, first, nh);
      if constexpr (is_contiguous_v<T>) v.resize(cnt);
      else v.clear();
      for (uint32_t j = 0; j < cnt; ++j) {
        unmarshal_state g{s.L, src + static_cast<std::size_t>(j) * op.size, first, 0, s.heaps,
                          h + 1};
        if constexpr (is_contiguous_v<T>) {
          from_device(v[j], g);
        } else {
          E e{};
          from_device(e, g);
          add_element(v, std::move(e));
        }
      }
      s.op = next;
      s.span = h + 1 + nh;
    }
  } else if constexpr (is_std_optional<T>::value || is_compat_v<T>) {
    using E = opt_value_t<T>;
    const spk_op &op = s.L->ops[s.op];
    const uint32_t cnt = get_u32(s.rec, op.rec_off);
    if constexpr (is_trivially_serializable<E>()) {
      const uint8_t *heap = s.heaps[s.span++];
      ++s.op;
      if (cnt) {
        opt_emplace(v);
        std::memcpy(static_cast<void *>(&*v), heap + get_u64(s.rec, op.aux) * op.size, op.size);
      } else {
        v.reset();
      }
    } else {
      const uint32_t first = s.op + 1, h0 = s.span;
      uint32_t nh = 0;
      const uint32_t next = skip_group(s.L, first, nh);
      if (cnt) {
        opt_emplace(v);
        unmarshal_state g{s.L, s.rec, first, 0, s.heaps, h0};
        from_device(*v, g);
      } else {
        v.reset();
      }
      s.op = next;
      s.span = h0 + nh;
    }
  } else if constexpr (is_std_variant<T>::value) {
    const spk_op &op = s.L->ops[s.op];
    get_alternative<0>(v, s, get_u32(s.rec, op.rec_off), s.op + 1, s.span);
    uint32_t i = s.op + 1, nh = 0;
    for (uint32_t g = 0; g < op.size; ++g) i = skip_group(s.L, i, nh);
    s.op = i;
    s.span += nh;
  } else if constexpr (is_std_array<T>::value) {
    for (auto &e : v) from_device(e, s);
  } else {
    constexpr uint64_t cfg = type_config<T>() & kCfgVarintBits;
    std::apply(
        [&](auto &...m) {
          (
              [&](auto &x) {
                using F = remove_cvref_t<decltype(x)>;
                if constexpr (cfg != 0 && !is_varint_v<F> && varint_tid<F, cfg>() != 0) {
                  const spk_op &op = s.L->ops[s.op++];
                  std::memcpy(&x, s.rec + op.rec_off, sizeof(F));
                } else {
                  from_device(x, s);
                }
              }(m),
              ...);
        },
        tie_members(v));
  }
}

}  // namespace detail
}  // namespace struct_pack::gpu
