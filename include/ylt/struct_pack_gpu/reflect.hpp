// reflect.hpp — compile-time reflection for the MI355X struct_pack front end
// (our own implementation; behaviour follows the reference's ylt::reflection,
// member_count.hpp:158-209 / member_ptr.hpp:95-137): aggregates by
// brace-initialisation member counting and structured bindings; non-aggregate
// types (or a chosen member list) through YLT_REFL(Type, member...), whose
// members are whatever refl_object_to_tuple ties (data members or accessor
// calls, user_reflect_macro.hpp:27-57).
//
// Supported members: fundamentals, enums, std::string / std::string_view,
// std::vector<T> / std::span<T> / std::list<T> / std::deque<T>, the set and
// map containers (ordered / unordered, multi or not), std::array<T, N>,
// std::optional<T>, std::variant<...>, std::pair<A, B>, the varint types,
// struct_pack::compatible<T, v>, and nested records. (C arrays inside
// aggregates defeat brace-init counting -- use std::array.)
#pragma once
#include <array>
#include <bitset>
#include <cstddef>
#include <deque>
#include <list>
#include <map>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <variant>
#include <cstdint>
#include <memory>
#include <optional>
#include <span>
#include <string>
#include <string_view>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

#include "config.hpp"

namespace struct_pack::gpu::detail {

template <typename T>
using remove_cvref_t = std::remove_cv_t<std::remove_reference_t<T>>;

template <typename T> struct is_std_vector : std::false_type {};
template <typename T, typename A> struct is_std_vector<std::vector<T, A>> : std::true_type {};
template <typename T> struct is_std_span : std::false_type {};
template <typename T, std::size_t E> struct is_std_span<std::span<T, E>> : std::bool_constant<E == std::dynamic_extent> {};
// optional-like members: std::optional<T> and a non-polymorphic
// std::unique_ptr<T> share the type literal (optional_t, type_id.hpp:337-346)
// and the wire [has_value][T] (packer.hpp:271-283,382-388)
template <typename T> struct is_std_optional : std::false_type {};
template <typename T> struct is_std_optional<std::optional<T>> : std::true_type {};
template <typename T, typename D> struct is_std_optional<std::unique_ptr<T, D>> : std::true_type {
  static_assert(!std::is_polymorphic_v<T>,
                "struct_pack::gpu: polymorphic std::unique_ptr<Base> members are not supported");
};
template <typename T> struct is_std_unique_ptr : std::false_type {};
template <typename T, typename D> struct is_std_unique_ptr<std::unique_ptr<T, D>> : std::true_type {};
// the value type of an optional-like / array / compatible / container type
template <typename T, bool = is_std_unique_ptr<T>::value>
struct opt_value {
  using type = std::remove_cv_t<std::remove_reference_t<typename T::value_type>>;
};
template <typename T>
struct opt_value<T, true> {
  using type = std::remove_cv_t<typename T::element_type>;
};
template <typename T>
using opt_value_t = typename opt_value<T>::type;
template <typename T>
bool opt_has(const T &v) {
  return static_cast<bool>(v);
}
template <typename T>
void opt_emplace(T &v) {
  if constexpr (is_std_unique_ptr<T>::value)
    v = std::make_unique<typename T::element_type>();
  else
    v.emplace();
}
template <typename T> struct is_std_array : std::false_type {};
template <typename T, std::size_t N> struct is_std_array<std::array<T, N>> : std::true_type {};

template <typename T> struct is_std_list : std::false_type {};  // list / deque: container_t
template <typename T, typename A> struct is_std_list<std::list<T, A>> : std::true_type {};
template <typename T, typename A> struct is_std_list<std::deque<T, A>> : std::true_type {};
template <typename T> struct is_std_variant : std::false_type {};
template <typename... A> struct is_std_variant<std::variant<A...>> : std::true_type {};
template <typename T> struct is_std_pair : std::false_type {};
template <typename A, typename B> struct is_std_pair<std::pair<A, B>> : std::true_type {};
// std::tuple: a struct of its elements, never trivially serializable
// (reflection.hpp:893-895); the message type of a multi-argument call
// (get_args_type, reflection.hpp:64-67)
template <typename T> struct is_std_tuple : std::false_type {};
template <typename... A> struct is_std_tuple<std::tuple<A...>> : std::true_type {};

// A message whose type is not a record (std::string, a container of
// non-record elements, an optional, a variant, ...) is encoded as the one
// member of boxed<M>: the same payload bytes, under M's own type code
// (layout.hpp message_type_t); the front end boxes and unboxes it.
template <typename M>
struct boxed {
  M v;
};
template <typename T> struct is_boxed : std::false_type {};
template <typename M> struct is_boxed<boxed<M>> : std::true_type {};

// set_container_t (type_id.hpp: set, multiset, unordered_set, unordered_multiset)
template <typename T> struct set_traits : std::false_type {};
template <typename K, typename C, typename A>
struct set_traits<std::set<K, C, A>> : std::true_type { static constexpr bool multi = false; };
template <typename K, typename C, typename A>
struct set_traits<std::multiset<K, C, A>> : std::true_type { static constexpr bool multi = true; };
template <typename K, typename H, typename E, typename A>
struct set_traits<std::unordered_set<K, H, E, A>> : std::true_type {
  static constexpr bool multi = false;
};
template <typename K, typename H, typename E, typename A>
struct set_traits<std::unordered_multiset<K, H, E, A>> : std::true_type {
  static constexpr bool multi = true;
};
// map_container_t (map, multimap, unordered_map, unordered_multimap)
template <typename T> struct map_traits : std::false_type {};
template <typename K, typename V, typename C, typename A>
struct map_traits<std::map<K, V, C, A>> : std::true_type { static constexpr bool multi = false; };
template <typename K, typename V, typename C, typename A>
struct map_traits<std::multimap<K, V, C, A>> : std::true_type {
  static constexpr bool multi = true;
};
template <typename K, typename V, typename H, typename E, typename A>
struct map_traits<std::unordered_map<K, V, H, E, A>> : std::true_type {
  static constexpr bool multi = false;
};
template <typename K, typename V, typename H, typename E, typename A>
struct map_traits<std::unordered_multimap<K, V, H, E, A>> : std::true_type {
  static constexpr bool multi = true;
};

// string_t (type_id.hpp:160-187, reflection.hpp:350-360): std::basic_string /
// basic_string_view of char, char8_t, char16_t, char32_t and wchar_t (the last
// only under STRUCT_PACK_ENABLE_UNPORTABLE_TYPE, checked by its type id)
template <typename C>
constexpr bool is_char_v = std::is_same_v<C, char> || std::is_same_v<C, char8_t> ||
                           std::is_same_v<C, char16_t> || std::is_same_v<C, char32_t> ||
                           std::is_same_v<C, wchar_t>;
template <typename T> struct string_traits : std::false_type {
  static constexpr bool view = false;
};
template <typename C, typename Tr, typename A>
struct string_traits<std::basic_string<C, Tr, A>> : std::bool_constant<is_char_v<C>> {
  using char_type = C;
  static constexpr bool view = false;
};
template <typename C, typename Tr>
struct string_traits<std::basic_string_view<C, Tr>> : std::bool_constant<is_char_v<C>> {
  using char_type = C;
  static constexpr bool view = true;
};
template <typename T>
constexpr bool is_string_v = string_traits<T>::value;
template <typename T>
constexpr bool is_string_view_v = string_traits<T>::value && string_traits<T>::view;
// the element of a string_t (char for anything else: never used there)
template <typename T, bool = is_string_v<T>>
struct string_char { using type = char; };
template <typename T>
struct string_char<T, true> { using type = typename string_traits<T>::char_type; };
template <typename T>
using string_char_t = typename string_char<T>::type;
// 128-bit integers (type_id.hpp:190-197: int128_t / uint128_t under
// STRUCT_PACK_ENABLE_INT128, gcc / clang): fundamentals of 16 bytes
template <typename T>
constexpr bool is_int128_v = std::is_same_v<T, __int128> || std::is_same_v<T, unsigned __int128>;
// bitset_t (reflection.hpp:558-591, under STRUCT_PACK_ENABLE_UNPORTABLE_TYPE):
// std::bitset<N> whose object is exactly its (N + 7) / 8 bytes, written raw
template <typename T> struct bitset_traits : std::false_type {};
template <std::size_t N>
struct bitset_traits<std::bitset<N>> : std::bool_constant<(N + 7) / 8 == sizeof(std::bitset<N>)> {
  static constexpr std::size_t bits = N;
};
template <typename T>
constexpr bool is_bitset_v = bitset_traits<T>::value;
template <typename T>
constexpr bool is_set_v = set_traits<T>::value;
template <typename T>
constexpr bool is_map_v = map_traits<T>::value;
// contiguous containers (memcpy of trivially serializable elements)
template <typename T>
constexpr bool is_contiguous_v = is_std_vector<T>::value || is_std_span<T>::value;
// every [count][elements] container (string_t aside)
template <typename T>
constexpr bool is_container_v =
    is_contiguous_v<T> || is_std_list<T>::value || is_set_v<T> || is_map_v<T>;
template <typename T>
constexpr bool is_monostate_v = std::is_same_v<T, std::monostate>;
template <typename T>
constexpr bool is_fundamental_v = std::is_arithmetic_v<T> || std::is_enum_v<T> || is_int128_v<T>;
template <typename T>
constexpr bool is_varint_v = varint_traits<T>::value;
template <typename T>
constexpr bool is_compat_v = compat_traits<T>::value;
template <typename T>
constexpr bool is_trivial_view_v = trivial_view_traits<T>::value;
template <typename T>
constexpr bool is_aggregate_record_v = std::is_aggregate_v<T> && std::is_class_v<T> &&
                                       !is_std_array<T>::value && !is_string_v<T> &&
                                       !is_container_v<T> && !is_std_optional<T>::value &&
                                       !is_varint_v<T> && !is_compat_v<T> && !is_ylt_refl_v<T> &&
                                       !is_monostate_v<T>;
// records: aggregates, YLT_REFL types, std::pair (a struct of first,
// second: type_id.hpp, the element of a map container) and std::tuple
template <typename T>
constexpr bool is_record_v = is_aggregate_record_v<T> || (std::is_class_v<T> && is_ylt_refl_v<T>) ||
                             is_std_pair<T>::value || is_std_tuple<T>::value;

// element type of a container as its device record holds it (a map's
// pair<const K, V> as pair<K, V>)
template <typename T, bool = is_map_v<T>>
struct elem_of {
  using type = remove_cvref_t<typename T::value_type>;
};
template <typename T>
struct elem_of<T, true> {
  using type = std::pair<remove_cvref_t<typename T::key_type>, typename T::mapped_type>;
};
template <typename T>
using elem_t = typename elem_of<T>::type;

// ---- aggregate member count (brace-init probing) ----------------------------
struct any_init {
  template <typename T>
  operator T() const noexcept;  // unevaluated only (never defined)
};

template <typename T, std::size_t... I>
constexpr bool brace_constructible(std::index_sequence<I...>) {
  return requires { T{((void)I, any_init{})...}; };
}

template <typename T, std::size_t N = 0>
constexpr std::size_t members_count_impl() {
  if constexpr (N > 40) {
    return N;  // give up (static_assert below)
  } else if constexpr (brace_constructible<T>(std::make_index_sequence<N + 1>{})) {
    return members_count_impl<T, N + 1>();
  } else {
    return N;
  }
}

template <typename T>
constexpr std::size_t members_count_v = members_count_impl<T>();

// ---- tie members: refl_object_to_tuple for YLT_REFL types, structured
// bindings for aggregates ------------------------------------------------------
#define SPK_TIE_CASE(N, ...)                   \
  else if constexpr (n == N) {                 \
    auto &&[__VA_ARGS__] = obj;                \
    return std::forward_as_tuple(__VA_ARGS__); \
  }

template <typename T>
constexpr auto tie_aggregate(T &obj) {
  using U = remove_cvref_t<T>;
  constexpr std::size_t n = members_count_v<U>;
  static_assert(n <= 24, "struct_pack MI355X front end: at most 24 members per aggregate");
  if constexpr (n == 0) {
    return std::tuple<>{};
  }
  SPK_TIE_CASE(1, a0)
  SPK_TIE_CASE(2, a0, a1)
  SPK_TIE_CASE(3, a0, a1, a2)
  SPK_TIE_CASE(4, a0, a1, a2, a3)
  SPK_TIE_CASE(5, a0, a1, a2, a3, a4)
  SPK_TIE_CASE(6, a0, a1, a2, a3, a4, a5)
  SPK_TIE_CASE(7, a0, a1, a2, a3, a4, a5, a6)
  SPK_TIE_CASE(8, a0, a1, a2, a3, a4, a5, a6, a7)
  SPK_TIE_CASE(9, a0, a1, a2, a3, a4, a5, a6, a7, a8)
  SPK_TIE_CASE(10, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9)
  SPK_TIE_CASE(11, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10)
  SPK_TIE_CASE(12, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11)
  SPK_TIE_CASE(13, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12)
  SPK_TIE_CASE(14, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13)
  SPK_TIE_CASE(15, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14)
  SPK_TIE_CASE(16, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15)
  SPK_TIE_CASE(17, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16)
  SPK_TIE_CASE(18, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17)
  SPK_TIE_CASE(19, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17, a18)
  SPK_TIE_CASE(20, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17, a18, a19)
  SPK_TIE_CASE(21, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17, a18, a19, a20)
  SPK_TIE_CASE(22, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17, a18, a19, a20, a21)
  SPK_TIE_CASE(23, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17, a18, a19, a20, a21, a22)
  SPK_TIE_CASE(24, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13, a14, a15, a16,
               a17, a18, a19, a20, a21, a22, a23)
}
#undef SPK_TIE_CASE

template <typename T, std::size_t... I>
constexpr auto tie_tuple(T &obj, std::index_sequence<I...>) {
  return std::forward_as_tuple(std::get<I>(obj)...);
}

template <typename T>
constexpr auto tie_members(T &obj) {
  if constexpr (is_std_pair<remove_cvref_t<T>>::value)
    return std::forward_as_tuple(obj.first, obj.second);
  else if constexpr (is_std_tuple<remove_cvref_t<T>>::value)
    return tie_tuple(obj, std::make_index_sequence<std::tuple_size_v<remove_cvref_t<T>>>{});
  else if constexpr (is_boxed<remove_cvref_t<T>>::value)
    return std::forward_as_tuple(obj.v);
  else if constexpr (is_ylt_refl_v<remove_cvref_t<T>>)
    return refl_tuple(obj);
  else
    return tie_aggregate(obj);
}

// member types as a tuple of values (for compile-time walks; no lambda in
// the unevaluated operand, which g++ 11 does not survive)
template <typename Tup>
struct decay_tuple;
template <typename... A>
struct decay_tuple<std::tuple<A...>> {
  using type = std::tuple<remove_cvref_t<A>...>;
};
template <typename T>
using members_tuple_t = typename decay_tuple<decltype(tie_members(std::declval<T &>()))>::type;

// ---- per-type sp_config: ADL set_sp_config(T*) or T::struct_pack_config
// (ref type_calculate.hpp:158-172) -----------------------------------------
template <typename T>
concept adl_config = requires { set_sp_config(static_cast<T *>(nullptr)); };
template <typename T>
concept member_config = requires { T::struct_pack_config; };

template <typename T>
constexpr uint64_t type_config() {
  if constexpr (adl_config<T>)
    return static_cast<uint64_t>(set_sp_config(static_cast<T *>(nullptr)));
  else if constexpr (member_config<T>)
    return static_cast<uint64_t>(T::struct_pack_config);
  else
    return sp_config::DEFAULT;
}

}  // namespace struct_pack::gpu::detail
