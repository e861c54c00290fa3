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
#include <stdexcept>
#include <vector>

#include "../../spk_codec.h"
#include "type_code.hpp"

namespace struct_pack::gpu {
namespace detail {

struct layout_builder {
  spk_layout L{};
  uint32_t off = 0, align = 1, spans = 0, vars = 0;
  uint32_t depth = 0;           // record nesting (1: members of the top-level record)
  uint64_t vers[SPK_MAX_OPS];   // sorted distinct compatible versions of the record
  uint32_t n_vers = 0;
  uint32_t place(uint32_t size, uint32_t al) {
    off = (off + al - 1) / al * al;
    const uint32_t o = off;
    off += size;
    if (al > align) align = al;
    return o;
  }
  void copy(uint32_t size, uint32_t al) {
    const uint32_t o = place(size, al);
    if (L.n_ops && L.ops[L.n_ops - 1].kind == SPK_OP_COPY &&
        L.ops[L.n_ops - 1].rec_off + L.ops[L.n_ops - 1].size == o) {
      L.ops[L.n_ops - 1].size += size;  // merge runs contiguous in the record
      return;
    }
    if (L.n_ops >= SPK_MAX_OPS) throw std::length_error("struct_pack: too many members");
    L.ops[L.n_ops++] = spk_op{SPK_OP_COPY, o, size, 0};
  }
  void varint(uint32_t size, uint32_t zigzag) {
    const uint32_t o = place(size, size);
    if (L.n_ops >= SPK_MAX_OPS || ++vars > SPK_MAX_VARINTS)
      throw std::length_error("struct_pack: too many varint members");
    L.ops[L.n_ops++] = spk_op{SPK_OP_VARINT, o, size, zigzag ? SPK_VARINT_ZIGZAG : 0u};
  }
  void span(uint32_t esz, uint32_t kind = SPK_OP_SPAN) {
    const uint32_t c = place(4, 4), a = place(8, 8);
    if (L.n_ops >= SPK_MAX_OPS || spans >= SPK_MAX_SPANS)
      throw std::length_error("struct_pack: too many variable-length members");
    L.ops[L.n_ops++] = spk_op{kind, c, esz, a};
    ++spans;
  }
};

template <typename T>
void flatten_into(layout_builder &b) {
  if constexpr (is_trivially_serializable<T>()) {
    b.copy(sizeof(T), alignof(T));
  } else if constexpr (is_varint_v<T>) {
    b.varint(sizeof(typename varint_traits<T>::value_type), varint_traits<T>::zigzag);
  } else if constexpr (is_string_v<T>) {
    b.span(1);
  } else if constexpr (is_container_v<T>) {
    using E = remove_cvref_t<typename T::value_type>;
    static_assert(is_trivially_serializable<E>(),
                  "MI355X codec: containers of non-trivially-serializable elements are "
                  "outside the flat record model");
    b.span(sizeof(E));
  } else if constexpr (is_std_optional<T>::value) {
    using E = remove_cvref_t<typename T::value_type>;
    static_assert(is_trivially_serializable<E>(),
                  "MI355X codec: optional of a non-trivially-serializable value is "
                  "outside the flat record model");
    b.span(sizeof(E), SPK_OP_OPTION);
  } else if constexpr (is_compat_v<T>) {
    using E = remove_cvref_t<typename T::value_type>;
    static_assert(is_trivially_serializable<E>(),
                  "MI355X codec: compatible of a non-trivially-serializable value is "
                  "outside the flat record model");
    if (b.depth != 1)
      throw std::logic_error("MI355X codec: compatible members only at the top level");
    uint32_t rank = 0;
    while (b.vers[rank] != compat_traits<T>::version) ++rank;
    b.span(sizeof(E), SPK_OP_COMPAT | rank << 8);
  } else if constexpr (is_std_array<T>::value) {
    for (std::size_t i = 0; i < std::tuple_size_v<T>; ++i)
      flatten_into<typename T::value_type>(b);
  } else {
    using M = members_tuple_t<T>;
    ++b.depth;
    [&]<std::size_t... I>(std::index_sequence<I...>) {
      (flatten_into<std::tuple_element_t<I, M>>(b), ...);
    }(std::make_index_sequence<std::tuple_size_v<M>>{});
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

// Descriptor of record type T for the batch codec (cacheable, immutable).
template <typename T, uint64_t conf = sp_config::DEFAULT>
spk_layout make_spk_layout() {
  using namespace detail;
  static_assert((type_config<T>() & (sp_config::ENCODING_WITH_VARINT | sp_config::USE_FAST_VARINT)) == 0,
                "MI355X codec C++ front end: records with ENCODING_WITH_VARINT / USE_FAST_VARINT "
                "are described through the C ABI (SPK_OP_FVAR, SPK_VARINT_SEXT) by the Python "
                "mirror; this front end does not flatten them yet");
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
  }
  fill_fmt(b.L.fmt_vector, get_type_code<std::vector<T>>(),
           msg_flags<std::vector<T>, conf>(), get_type_literal<std::vector<T>>());
  fill_fmt(b.L.fmt_one, get_type_code<T>(), msg_flags<T, conf>(), get_type_literal<T>());
  return b.L;
}

namespace detail {

// ---- host object <-> device record ----------------------------------------
struct marshal_state {
  const spk_layout *L;
  uint8_t *rec;                                   // current device record
  uint32_t op = 0, within = 0;                    // walking the op list
  std::vector<std::vector<uint8_t>> *heaps;       // one per span
  uint32_t span = 0;
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

template <typename T>
void to_device(const T &v, marshal_state &s) {
  if constexpr (is_trivially_serializable<T>()) {
    put_copy(s, &v, sizeof(T));
  } else if constexpr (is_varint_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    const typename varint_traits<T>::value_type x = v;
    std::memcpy(s.rec + op.rec_off, &x, op.size);
  } else if constexpr (is_string_v<T> || is_container_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    auto &heap = (*s.heaps)[s.span++];
    const uint32_t cnt = static_cast<uint32_t>(v.size());
    const uint64_t eoff = heap.size() / op.size;
    std::memcpy(s.rec + op.rec_off, &cnt, 4);
    std::memcpy(s.rec + op.aux, &eoff, 8);
    const auto *p = reinterpret_cast<const uint8_t *>(v.data());
    heap.insert(heap.end(), p, p + static_cast<std::size_t>(cnt) * op.size);
  } else if constexpr (is_std_optional<T>::value || is_compat_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    auto &heap = (*s.heaps)[s.span++];
    const uint32_t cnt = v.has_value() ? 1u : 0u;
    const uint64_t eoff = heap.size() / op.size;
    std::memcpy(s.rec + op.rec_off, &cnt, 4);
    std::memcpy(s.rec + op.aux, &eoff, 8);
    if (cnt) {
      const auto *p = reinterpret_cast<const uint8_t *>(&*v);
      heap.insert(heap.end(), p, p + op.size);
    }
  } else if constexpr (is_std_array<T>::value) {
    for (const auto &e : v) to_device(e, s);
  } else {
    std::apply([&](const auto &...m) { (to_device(m, s), ...); }, tie_members(v));
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

template <typename T>
void from_device(T &v, unmarshal_state &s) {
  if constexpr (is_trivially_serializable<T>()) {
    get_copy(s, &v, sizeof(T));
  } else if constexpr (is_varint_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    typename varint_traits<T>::value_type x;
    std::memcpy(&x, s.rec + op.rec_off, op.size);
    v = x;
  } else if constexpr (is_string_v<T> || is_container_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    const uint8_t *heap = s.heaps[s.span++];
    uint32_t cnt;
    uint64_t eoff;
    std::memcpy(&cnt, s.rec + op.rec_off, 4);
    std::memcpy(&eoff, s.rec + op.aux, 8);
    const uint8_t *src = heap + eoff * op.size;
    if constexpr (std::is_same_v<T, std::string_view> || is_std_span<T>::value) {
      // views alias the decoded heap (the reference's views alias the input)
      v = T(reinterpret_cast<typename T::const_pointer>(src), cnt);
    } else {
      v.resize(cnt);
      if (cnt) std::memcpy(v.data(), src, static_cast<std::size_t>(cnt) * op.size);
    }
  } else if constexpr (is_std_optional<T>::value || is_compat_v<T>) {
    const spk_op &op = s.L->ops[s.op++];
    const uint8_t *heap = s.heaps[s.span++];
    uint32_t cnt;
    uint64_t eoff;
    std::memcpy(&cnt, s.rec + op.rec_off, 4);
    std::memcpy(&eoff, s.rec + op.aux, 8);
    if (cnt) {
      v.emplace();
      std::memcpy(static_cast<void *>(&*v), heap + eoff * op.size, op.size);
    } else {
      v.reset();
    }
  } else if constexpr (is_std_array<T>::value) {
    for (auto &e : v) from_device(e, s);
  } else {
    std::apply([&](auto &...m) { (from_device(m, s), ...); }, tie_members(v));
  }
}

}  // namespace detail
}  // namespace struct_pack::gpu
