// type_code.hpp — compile-time type literal and 32-bit type code of the
// MI355X struct_pack front end (our own implementation of the reference's
// wire contract):
//   type_id bytes           ref include/ylt/struct_pack/type_id.hpp:25-81
//   get_type_literal         ref type_calculate.hpp:194-373
//   get_size_literal         ref type_calculate.hpp:26-97
//   code = MD5_32 & ~1       ref type_calculate.hpp:507-516, md5_constexpr.hpp
//   is_trivial_serializable  ref reflection.hpp:851-922
//   check_if_has_container   ref type_calculate.hpp:793-857
//   pack / alignment literal ref alignment.hpp:23-122 (user overrides
//                            struct_pack::pack_alignment_v / alignment_v)
// The MD5 below is a straightforward constexpr RFC 1321 implementation.
#pragma once
#include <array>
#include <cstdint>

#include "reflect.hpp"

namespace struct_pack::gpu {
namespace detail {

// ---- fixed-capacity constexpr byte string ----------------------------------
struct lit_t {
  std::array<uint8_t, 256> d{};
  std::size_t n = 0;
  constexpr void push(uint8_t b) { d[n++] = b; }
  constexpr void append(const lit_t &o) {
    for (std::size_t i = 0; i < o.n; ++i) d[n++] = o.d[i];
  }
};

enum : uint8_t {
  TID_INT32 = 1, TID_UINT32 = 2, TID_INT64 = 3, TID_UINT64 = 4, TID_INT8 = 5,
  TID_UINT8 = 6, TID_INT16 = 7, TID_UINT16 = 8, TID_INT128 = 9, TID_UINT128 = 10,
  TID_BOOL = 11, TID_CHAR8 = 12, TID_CHAR16 = 13, TID_CHAR32 = 14, TID_WCHAR = 15,
  TID_FLOAT32 = 17, TID_FLOAT64 = 18,
  TID_VINT32 = 20, TID_VINT64 = 21, TID_VUINT32 = 22, TID_VUINT64 = 23,
  TID_STRING = 128, TID_ARRAY = 129, TID_MAP = 130, TID_SET = 131, TID_CONTAINER = 132,
  TID_OPTIONAL = 133, TID_VARIANT = 134, TID_BITSET = 136, TID_MONOSTATE = 250, TID_STRUCT = 253, TID_END = 255
};

// sp_config bits of a record that turn members into varints (reflection.hpp:
// 53-60, 843): ENCODING_WITH_VARINT makes plain (u)int32/64 members varints,
// USE_FAST_VARINT writes the record's varints as one fast-varint group
inline constexpr uint64_t kCfgEncodingWithVarint = 0b100, kCfgUseFastVarint = 0b1000;
inline constexpr uint64_t kCfgVarintBits = kCfgEncodingWithVarint | kCfgUseFastVarint;

// a plain integer member that ENCODING_WITH_VARINT turns into a varint
template <typename T>
constexpr bool is_plain_varint_v = std::is_same_v<T, int32_t> || std::is_same_v<T, uint32_t> ||
                                   std::is_same_v<T, int64_t> || std::is_same_v<T, uint64_t>;

// get_varint_type<T, parent_tag> (type_id.hpp:83-125): the type id of member
// T under its record's config `cfg`, or 0 when it is not a varint there;
// USE_FAST_VARINT selects the fast_v* ids (varint id + 4)
template <typename T, uint64_t cfg>
constexpr uint8_t varint_tid() {
  uint8_t t = 0;
  if constexpr (is_varint_v<T>) {
    using V = typename varint_traits<T>::value_type;
    constexpr bool zz = varint_traits<T>::zigzag;
    t = sizeof(V) == 4 ? (zz ? TID_VINT32 : TID_VUINT32) : (zz ? TID_VINT64 : TID_VUINT64);
  } else if constexpr ((cfg & kCfgEncodingWithVarint) && is_plain_varint_v<T>) {
    t = sizeof(T) == 4 ? (std::is_signed_v<T> ? TID_VINT32 : TID_VUINT32)
                       : (std::is_signed_v<T> ? TID_VINT64 : TID_VUINT64);
  }
  if (t && (cfg & kCfgUseFastVarint)) t += 4;
  return t;
}

// the reference's opt-in types (type_id.hpp:168-172,190-197, 317-320): the
// same macros switch them on here
#ifdef STRUCT_PACK_ENABLE_UNPORTABLE_TYPE
inline constexpr bool kUnportableTypes = true;
#else
inline constexpr bool kUnportableTypes = false;
#endif
#if defined(STRUCT_PACK_ENABLE_INT128) && (defined(__GNUC__) || defined(__clang__))
inline constexpr bool kInt128Types = true;
#else
inline constexpr bool kInt128Types = false;
#endif
template <typename T>
inline constexpr bool dependent_false_v = false;

template <typename T>
constexpr uint8_t fundamental_id() {
  if constexpr (is_int128_v<T>) {
    static_assert(kInt128Types || dependent_false_v<T>,
                  "128-bit integers need STRUCT_PACK_ENABLE_INT128 (as in the reference)");
    return std::is_same_v<T, __int128> ? TID_INT128 : TID_UINT128;
  } else if constexpr (std::is_same_v<T, wchar_t>) {
    static_assert(kUnportableTypes || dependent_false_v<T>,
                  "wchar_t needs STRUCT_PACK_ENABLE_UNPORTABLE_TYPE (as in the reference)");
    return TID_WCHAR;
  } else if constexpr (std::is_enum_v<T>) {
    return fundamental_id<std::underlying_type_t<T>>();
  } else if constexpr (std::is_same_v<T, bool>) {
    return TID_BOOL;
  } else if constexpr (std::is_same_v<T, char> || std::is_same_v<T, char8_t>) {
    return TID_CHAR8;  // char is saved as unsigned (type_id.hpp:160-166)
  } else if constexpr (std::is_same_v<T, char16_t>) {
    return TID_CHAR16;
  } else if constexpr (std::is_same_v<T, char32_t>) {
    return TID_CHAR32;
  } else if constexpr (std::is_floating_point_v<T>) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "long double unsupported");
    return sizeof(T) == 4 ? TID_FLOAT32 : TID_FLOAT64;
  } else {
    static_assert(std::is_integral_v<T>);
    if constexpr (std::is_signed_v<T>)
      return sizeof(T) == 1 ? TID_INT8 : sizeof(T) == 2 ? TID_INT16
                                       : sizeof(T) == 4 ? TID_INT32 : TID_INT64;
    else
      return sizeof(T) == 1 ? TID_UINT8 : sizeof(T) == 2 ? TID_UINT16
                                        : sizeof(T) == 4 ? TID_UINT32 : TID_UINT64;
  }
}

constexpr lit_t size_literal(std::size_t n) {
  lit_t l;
  while (n >= 127) {
    l.push(static_cast<uint8_t>(n % 127 + 1));
    n /= 127;
  }
  l.push(static_cast<uint8_t>(n + 129));
  return l;
}

template <typename T>
constexpr bool is_trivially_serializable();

template <typename Tup, uint64_t cfg, std::size_t... I>
constexpr bool all_trivial(std::index_sequence<I...>) {
  return ((is_trivially_serializable<std::tuple_element_t<I, Tup>>() &&
           varint_tid<std::tuple_element_t<I, Tup>, cfg>() == 0) &&
          ...);
}

template <typename T>
constexpr bool is_trivially_serializable() {
  if constexpr (is_fundamental_v<T> || is_monostate_v<T>) {
    return true;
  } else if constexpr (is_bitset_v<T>) {  // reflection.hpp:878
    return true;
  } else if constexpr (is_std_array<T>::value) {
    return is_trivially_serializable<typename T::value_type>();
  } else if constexpr (is_string_v<T> || is_container_v<T> || is_std_optional<T>::value ||
                       is_varint_v<T> || is_compat_v<T> || is_std_variant<T>::value) {
    return false;  // reflection.hpp:872-876,899-905
  } else if constexpr (is_ylt_refl_v<T>) {
    return false;  // user_defined_refl: member by member (reflection.hpp:896-898)
  } else if constexpr (is_trivial_view_v<T>) {
    return false;  // its record goes member by member (reflection.hpp:875-877)
  } else if constexpr (is_std_tuple<T>::value) {
    return false;  // std::tuple: member by member (reflection.hpp:893-895)
  } else {
    static_assert(is_record_v<T>, "unsupported member type");
    using M = members_tuple_t<T>;
    return all_trivial<M, type_config<T>() & kCfgVarintBits>(
        std::make_index_sequence<std::tuple_size_v<M>>{});
  }
}

template <typename V>
struct variant_any_container;

template <typename T>
constexpr bool has_container();
template <typename Tup, std::size_t... I>
constexpr bool any_container(std::index_sequence<I...>) {
  return (has_container<std::tuple_element_t<I, Tup>>() || ...);
}
template <typename T>
constexpr bool has_container() {
  if constexpr (is_string_v<T> || is_container_v<T>)
    return true;
  else if constexpr (is_std_variant<T>::value)  // type_calculate.hpp:785-815
    return variant_any_container<T>::value;
  else if constexpr (is_std_array<T>::value || is_std_optional<T>::value || is_compat_v<T>)
    return has_container<opt_value_t<T>>();  // type_calculate.hpp:846-849
  else if constexpr (is_record_v<T>) {
    using M = members_tuple_t<T>;
    return any_container<M>(std::make_index_sequence<std::tuple_size_v<M>>{});
  } else
    return false;
}

template <typename... A>
struct variant_any_container<std::variant<A...>> {
  static constexpr bool value = (has_container<A>() || ...);
};

// max over the members' alignment (alignment.hpp:33-41,63-71)
template <typename T>
constexpr std::size_t alignment_of();
template <typename M, std::size_t... I>
constexpr std::size_t max_member_alignment(std::index_sequence<I...>) {
  std::size_t a = 0;
  ((a = alignment_of<std::tuple_element_t<I, M>>() > a ? alignment_of<std::tuple_element_t<I, M>>()
                                                        : a),
   ...);
  return a;
}

// pack_alignment_v (alignment.hpp:72-88): the user's struct_pack::
// pack_alignment_v<T> when set (#pragma pack), else the largest member
// alignment
template <typename T>
constexpr std::size_t pack_alignment_of() {
  constexpr std::size_t user = user_pack_alignment<T>;
  static_assert(user == 0 || user == 1 || user == 2 || user == 4 || user == 8 || user == 16,
                "struct_pack::pack_alignment_v must be 0, 1, 2, 4, 8 or 16");
  if constexpr (user != 0) {
    return user;
  } else {
    using M = members_tuple_t<T>;
    return max_member_alignment<M>(std::make_index_sequence<std::tuple_size_v<M>>{});
  }
}

// alignment_v (alignment.hpp:90-122): the user's struct_pack::alignment_v<T>
// when set (it must equal alignof for a trivially serializable type);
// otherwise alignof for trivially serializable / non-record types and, for a
// non-trivial record, the user's pack alignment or the largest member
// alignment
template <typename T>
constexpr std::size_t alignment_of() {
  if constexpr (is_record_v<T>) {
    constexpr std::size_t user = user_alignment<T>;
    if constexpr (user != 0) {
      static_assert((user & (user - 1)) == 0, "alignment should be power of 2");
      if constexpr (is_trivially_serializable<T>())
        static_assert(user == alignof(T), "struct_pack::alignment_v must equal alignof(T)");
      return user;
    } else if constexpr (is_trivially_serializable<T>()) {
      return alignof(T);
    } else if constexpr (user_pack_alignment<T> != 0) {
      return user_pack_alignment<T>;
    } else {
      using M = members_tuple_t<T>;
      return max_member_alignment<M>(std::make_index_sequence<std::tuple_size_v<M>>{});
    }
  } else {
    return alignof(T);
  }
}

template <typename T>
constexpr lit_t type_literal();

// a member's literal under its record's config: a varint there is its type id
template <typename F, uint64_t cfg>
constexpr lit_t member_literal() {
  if constexpr (varint_tid<F, cfg>() != 0) {
    lit_t l;
    l.push(varint_tid<F, cfg>());
    return l;
  } else {
    return type_literal<F>();
  }
}
template <typename Tup, uint64_t cfg, std::size_t... I>
constexpr void append_members(lit_t &l, std::index_sequence<I...>) {
  (l.append(member_literal<std::tuple_element_t<I, Tup>, cfg>()), ...);
}
template <typename... A>
constexpr void append_alternatives(lit_t &l, std::variant<A...> *) {
  (l.append(type_literal<A>()), ...);
}

template <typename T>
constexpr lit_t type_literal() {
  lit_t l;
  if constexpr (is_trivial_view_v<T>) {  // T's literal (type_calculate.hpp:196-198)
    l.append(type_literal<typename trivial_view_traits<T>::value_type>());
  } else if constexpr (is_fundamental_v<T>) {
    l.push(fundamental_id<T>());
  } else if constexpr (is_string_v<T>) {  // string_t + the char type's id
    l.push(TID_STRING);
    l.push(fundamental_id<string_char_t<T>>());
  } else if constexpr (is_bitset_v<T>) {  // bitset_t + its bit count (type_calculate.hpp:264-268)
    static_assert(kUnportableTypes || dependent_false_v<T>,
                  "std::bitset needs STRUCT_PACK_ENABLE_UNPORTABLE_TYPE (as in the reference)");
    l.push(TID_BITSET);
    l.append(size_literal(bitset_traits<T>::bits));
  } else if constexpr (is_map_v<T>) {  // type_calculate.hpp:284-290
    l.push(TID_MAP);
    l.append(type_literal<remove_cvref_t<typename T::key_type>>());
    l.append(type_literal<remove_cvref_t<typename T::mapped_type>>());
  } else if constexpr (is_set_v<T>) {  // type_calculate.hpp:280-283
    l.push(TID_SET);
    l.append(type_literal<remove_cvref_t<typename T::key_type>>());
  } else if constexpr (is_container_v<T>) {
    l.push(TID_CONTAINER);
    l.append(type_literal<remove_cvref_t<typename T::value_type>>());
  } else if constexpr (is_std_variant<T>::value) {  // type_calculate.hpp:245-253
    l.push(TID_VARIANT);
    append_alternatives(l, static_cast<T *>(nullptr));
    l.push(TID_END);
  } else if constexpr (is_monostate_v<T>) {
    l.push(TID_MONOSTATE);
  } else if constexpr (is_varint_v<T>) {  // get_varint_type (type_id.hpp:84-125)
    using V = typename varint_traits<T>::value_type;
    constexpr bool zz = varint_traits<T>::zigzag;
    l.push(sizeof(V) == 4 ? (zz ? TID_VINT32 : TID_VUINT32) : (zz ? TID_VINT64 : TID_VUINT64));
  } else if constexpr (is_compat_v<T>) {  // not in the literal (type_calculate.hpp:298-303)
  } else if constexpr (is_std_optional<T>::value) {  // type_calculate.hpp:269-278
    l.push(TID_OPTIONAL);
    l.append(type_literal<opt_value_t<T>>());
  } else if constexpr (is_std_array<T>::value) {
    l.push(TID_ARRAY);
    l.append(type_literal<typename T::value_type>());
    l.append(size_literal(std::tuple_size_v<T>));
  } else {
    static_assert(is_record_v<T>, "unsupported type");
    using M = members_tuple_t<T>;
    l.push(TID_STRUCT);
    append_members<M, type_config<T>() & kCfgVarintBits>(
        l, std::make_index_sequence<std::tuple_size_v<M>>{});
    if constexpr (is_trivially_serializable<T>()) {  // type_calculate.hpp:229-239
      static_assert(pack_alignment_of<T>() <= alignment_of<T>(),
                    "If you add #pragma pack to a struct, please specify "
                    "struct_pack::pack_alignment_v<T>.");
      l.append(size_literal(pack_alignment_of<T>()));
      l.append(size_literal(alignment_of<T>()));
    }
    l.push(TID_END);
  }
  return l;
}

// ---- constexpr MD5 (RFC 1321) ------------------------------------------------
constexpr uint32_t md5_rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

constexpr std::array<uint8_t, 16> md5(const uint8_t *msg, std::size_t len) {
  constexpr uint32_t K[64] = {
      0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
      0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
      0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
      0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
      0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
      0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
      0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
      0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
      0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
      0xeb86d391};
  constexpr int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                         5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                         4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                         6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
  uint32_t a0 = 0x67452301, b0 = 0xefcdab89, c0 = 0x98badcfe, d0 = 0x10325476;
  const std::size_t total = ((len + 8) / 64 + 1) * 64;
  for (std::size_t blk = 0; blk < total; blk += 64) {
    uint32_t M[16] = {};
    for (int i = 0; i < 64; ++i) {
      const std::size_t idx = blk + i;
      uint8_t b = 0;
      if (idx < len)
        b = msg[idx];
      else if (idx == len)
        b = 0x80;
      else if (idx >= total - 8)
        b = static_cast<uint8_t>((static_cast<uint64_t>(len) * 8) >> (8 * (idx - (total - 8))));
      M[i / 4] |= static_cast<uint32_t>(b) << (8 * (i % 4));
    }
    uint32_t A = a0, B = b0, C = c0, D = d0;
    for (int i = 0; i < 64; ++i) {
      uint32_t F;
      int g;
      if (i < 16) { F = (B & C) | (~B & D); g = i; }
      else if (i < 32) { F = (D & B) | (~D & C); g = (5 * i + 1) % 16; }
      else if (i < 48) { F = B ^ C ^ D; g = (3 * i + 5) % 16; }
      else { F = C ^ (B | ~D); g = (7 * i) % 16; }
      F = F + A + K[i] + M[g];
      A = D;
      D = C;
      C = B;
      B = B + md5_rotl(F, R[i]);
    }
    a0 += A; b0 += B; c0 += C; d0 += D;
  }
  std::array<uint8_t, 16> out{};
  const uint32_t h[4] = {a0, b0, c0, d0};
  for (int i = 0; i < 16; ++i) out[i] = static_cast<uint8_t>(h[i / 4] >> (8 * (i % 4)));
  return out;
}

// MD5Hash32Constexpr: the first four digest bytes read big-endian
constexpr uint32_t md5_hash32(const lit_t &l) {
  const auto d = md5(l.d.data(), l.n);
  return (static_cast<uint32_t>(d[0]) << 24) | (static_cast<uint32_t>(d[1]) << 16) |
         (static_cast<uint32_t>(d[2]) << 8) | static_cast<uint32_t>(d[3]);
}

}  // namespace detail

// Public: get_type_literal / get_type_code of one type (struct_pack.hpp:75-110)
template <typename T>
constexpr auto get_type_literal() {
  return detail::type_literal<detail::remove_cvref_t<T>>();
}
template <typename T>
constexpr uint32_t get_type_code() {
  return detail::md5_hash32(get_type_literal<T>()) & 0xFFFFFFFEu;
}

}  // namespace struct_pack::gpu
