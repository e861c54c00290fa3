// config.hpp — the struct_pack vocabulary the MI355X front end is written
// against: errc / err_code, sp_config, the varint member types, the
// alignment customisation points, expected<T> and YLT_REFL.
//
// Two ways to build, decided per translation unit:
//   * next to the reference (the drop-in case): when the reference header
//     <ylt/struct_pack.hpp> is on the include path it is included here and
//     its own types are used -- struct_pack::errc, err_code, sp_config,
//     var_int32_t ..., pack_alignment_v / alignment_v, set_sp_config, YLT_REFL
//     -- so user types written for the reference need no change and the GPU
//     path can sit beside the CPU one (coro_rpc's struct_pack_gpu_protocol).
//     Nothing is declared in namespace struct_pack by this front end then:
//     it lives in struct_pack::gpu.
//   * standalone (no reference on the include path, e.g. the GPU box, or
//     SPK_GPU_STANDALONE defined): the same names are declared here with the
//     reference's meaning (ref include/ylt/struct_pack/error_code.hpp:21-64,
//     reflection.hpp:53-60, varint.hpp:79-185,352-355, alignment.hpp:90-122,
//     reflection/user_reflect_macro.hpp:27-57), so the same user code compiles.
#pragma once
#include <cstddef>
#include <cstdint>
#include <optional>
#include <string_view>
#include <tuple>
#include <type_traits>
#include <utility>

#if !defined(SPK_GPU_STANDALONE) && __has_include(<ylt/struct_pack.hpp>)
#include <ylt/struct_pack.hpp>
#define SPK_GPU_WITH_REFERENCE 1
#else
#define SPK_GPU_WITH_REFERENCE 0
#endif

#if !SPK_GPU_WITH_REFERENCE
namespace struct_pack {

// error_code.hpp:21-64 (operator bool is implicit there too)
enum class errc {
  ok = 0,
  no_buffer_space,
  invalid_buffer,
  hash_conflict,
  invalid_width_of_container_length,
};

struct err_code {
  errc ec;
  constexpr err_code() noexcept : ec(errc::ok) {}
  constexpr err_code(errc e) noexcept : ec(e) {}
  constexpr err_code &operator=(errc e) noexcept {
    ec = e;
    return *this;
  }
  constexpr operator errc() const noexcept { return ec; }
  constexpr operator bool() const noexcept { return ec != errc::ok; }
  constexpr int val() const noexcept { return static_cast<int>(ec); }
  constexpr std::string_view message() const noexcept {
    switch (ec) {
      case errc::ok: return "ok";
      case errc::no_buffer_space: return "no buffer space";
      case errc::invalid_buffer: return "invalid argument";
      case errc::hash_conflict: return "hash conflict";
      case errc::invalid_width_of_container_length:
        return "invalid width of container length";
    }
    return "(unrecognized error)";
  }
};

// reflection.hpp:53-60
enum sp_config : uint64_t {
  DEFAULT = 0,
  DISABLE_TYPE_INFO = 0b1,
  ENABLE_TYPE_INFO = 0b10,
  DISABLE_ALL_META_INFO = 0b11,
  ENCODING_WITH_VARINT = 0b100,
  USE_FAST_VARINT = 0b1000
};

// user customisation points of the type hash (alignment.hpp:74,95-99)
template <typename T>
constexpr std::size_t pack_alignment_v = 0;
template <typename T>
constexpr std::size_t alignment_v = 0;

namespace detail {
// varint<T> (LEB128) and sint<T> (zigzag + LEB128), varint.hpp:79-185
template <typename T>
class varint {
 public:
  using value_type = T;
  varint() noexcept = default;
  varint(T t) noexcept : val(t) {}
  [[nodiscard]] operator T() const noexcept { return val; }
  varint &operator=(T t) noexcept {
    val = t;
    return *this;
  }
  [[nodiscard]] bool operator==(const varint &o) const noexcept { return val == o.val; }
  [[nodiscard]] bool operator==(T t) const noexcept { return val == t; }
  [[nodiscard]] bool operator<(const varint &o) const noexcept { return val < o.val; }
  const T &get() const noexcept { return val; }
  T &get() noexcept { return val; }

 private:
  T val{};
};
template <typename T>
class sint : public varint<T> {
 public:
  using varint<T>::varint;
};
}  // namespace detail
using var_int32_t = detail::sint<int32_t>;
using var_int64_t = detail::sint<int64_t>;
using var_uint32_t = detail::varint<uint32_t>;
using var_uint64_t = detail::varint<uint64_t>;

// compatible.hpp:21-154: an optional member that is written after the main
// pass, in the pass of its version (forward / backward compatible fields)
template <typename T, uint64_t version = 0>
struct compatible : public std::optional<T> {
  constexpr compatible() = default;
  constexpr compatible(const compatible &) = default;
  constexpr compatible(compatible &&) = default;
  constexpr compatible(std::optional<T> &&o) : std::optional<T>(std::move(o)) {}
  constexpr compatible(const std::optional<T> &o) : std::optional<T>(o) {}
  using std::optional<T>::optional;
  constexpr compatible &operator=(const compatible &) = default;
  constexpr compatible &operator=(compatible &&) = default;
  static constexpr uint64_t version_number = version;
};
template <typename T, uint64_t v1, uint64_t v2>
inline bool operator==(const compatible<T, v1> &a, const compatible<T, v2> &b) {
  return static_cast<bool>(a) == static_cast<bool>(b) && (!a || *a == *b);
}

// trivial_view.hpp:79-102: a view of a trivially serializable T, equal to T
// in the type system and on the wire
template <typename T, typename = void>
struct trivial_view {
 private:
  const T *ref;

 public:
  trivial_view(const T *t) : ref(t) {}
  trivial_view(const T &t) : ref(&t) {}
  trivial_view(const trivial_view &) = default;
  trivial_view() : ref(nullptr) {}
  trivial_view &operator=(const trivial_view &) = default;
  using value_type = T;
  void set(const T &obj) { ref = &obj; }
  const T &get() const { return *ref; }
  const T *operator->() const { return ref; }
};

}  // namespace struct_pack

// ---- YLT_REFL(Type, member...) ---------------------------------------------
// Non-aggregate / selected-member reflection (user_reflect_macro.hpp:27-57):
// usable at namespace scope next to the type or inside the class. The
// reference treats such a type as never trivially serializable
// (reflection.hpp:896-898): members written one by one, no padding.
#ifndef YLT_REFL
#define SPK_REFL_CAT_(a, b) a##b
#define SPK_REFL_CAT(a, b) SPK_REFL_CAT_(a, b)
#define SPK_REFL_N_(_1, _2, _3, _4, _5, _6, _7, _8, _9, _10, _11, _12, _13, _14, _15, _16, \
                    _17, _18, _19, _20, _21, _22, _23, _24, N, ...)                        \
  N
#define SPK_REFL_N(...)                                                                    \
  SPK_REFL_N_(__VA_ARGS__, 24, 23, 22, 21, 20, 19, 18, 17, 16, 15, 14, 13, 12, 11, 10, 9, 8, \
              7, 6, 5, 4, 3, 2, 1)
#define SPK_REFL_M1(t, a) t.a
#define SPK_REFL_M2(t, a, ...) t.a, SPK_REFL_M1(t, __VA_ARGS__)
#define SPK_REFL_M3(t, a, ...) t.a, SPK_REFL_M2(t, __VA_ARGS__)
#define SPK_REFL_M4(t, a, ...) t.a, SPK_REFL_M3(t, __VA_ARGS__)
#define SPK_REFL_M5(t, a, ...) t.a, SPK_REFL_M4(t, __VA_ARGS__)
#define SPK_REFL_M6(t, a, ...) t.a, SPK_REFL_M5(t, __VA_ARGS__)
#define SPK_REFL_M7(t, a, ...) t.a, SPK_REFL_M6(t, __VA_ARGS__)
#define SPK_REFL_M8(t, a, ...) t.a, SPK_REFL_M7(t, __VA_ARGS__)
#define SPK_REFL_M9(t, a, ...) t.a, SPK_REFL_M8(t, __VA_ARGS__)
#define SPK_REFL_M10(t, a, ...) t.a, SPK_REFL_M9(t, __VA_ARGS__)
#define SPK_REFL_M11(t, a, ...) t.a, SPK_REFL_M10(t, __VA_ARGS__)
#define SPK_REFL_M12(t, a, ...) t.a, SPK_REFL_M11(t, __VA_ARGS__)
#define SPK_REFL_M13(t, a, ...) t.a, SPK_REFL_M12(t, __VA_ARGS__)
#define SPK_REFL_M14(t, a, ...) t.a, SPK_REFL_M13(t, __VA_ARGS__)
#define SPK_REFL_M15(t, a, ...) t.a, SPK_REFL_M14(t, __VA_ARGS__)
#define SPK_REFL_M16(t, a, ...) t.a, SPK_REFL_M15(t, __VA_ARGS__)
#define SPK_REFL_M17(t, a, ...) t.a, SPK_REFL_M16(t, __VA_ARGS__)
#define SPK_REFL_M18(t, a, ...) t.a, SPK_REFL_M17(t, __VA_ARGS__)
#define SPK_REFL_M19(t, a, ...) t.a, SPK_REFL_M18(t, __VA_ARGS__)
#define SPK_REFL_M20(t, a, ...) t.a, SPK_REFL_M19(t, __VA_ARGS__)
#define SPK_REFL_M21(t, a, ...) t.a, SPK_REFL_M20(t, __VA_ARGS__)
#define SPK_REFL_M22(t, a, ...) t.a, SPK_REFL_M21(t, __VA_ARGS__)
#define SPK_REFL_M23(t, a, ...) t.a, SPK_REFL_M22(t, __VA_ARGS__)
#define SPK_REFL_M24(t, a, ...) t.a, SPK_REFL_M23(t, __VA_ARGS__)
#define SPK_REFL_MEMBERS(t, ...) \
  SPK_REFL_CAT(SPK_REFL_M, SPK_REFL_N(__VA_ARGS__))(t, __VA_ARGS__)
#define YLT_REFL(STRUCT, ...)                                                         \
  [[maybe_unused]] inline static auto refl_object_to_tuple(STRUCT &t) {              \
    return std::tie(SPK_REFL_MEMBERS(t, __VA_ARGS__));                               \
  }                                                                                  \
  [[maybe_unused]] inline static auto refl_object_to_tuple(const STRUCT &t) {        \
    return std::tie(SPK_REFL_MEMBERS(t, __VA_ARGS__));                               \
  }
#endif
#endif  // !SPK_GPU_WITH_REFERENCE

namespace struct_pack::gpu {

// ---- expected<T> of the decode API -------------------------------------------
#if SPK_GPU_WITH_REFERENCE
template <typename T>
using expected = struct_pack::expected<T, struct_pack::err_code>;
template <typename T>
inline expected<T> make_unexpected(err_code e) {
  return struct_pack::unexpected<struct_pack::err_code>{e};
}
#else
// the subset of expected<T, err_code> the reference's callers use
template <typename T>
class expected {
 public:
  expected() : v_(std::in_place) {}
  expected(T v) : v_(std::move(v)) {}
  bool has_value() const noexcept { return v_.has_value(); }
  explicit operator bool() const noexcept { return has_value(); }
  T &value() & { return v_.value(); }
  const T &value() const & { return v_.value(); }
  T &&value() && { return std::move(v_.value()); }
  T &operator*() { return *v_; }
  const T &operator*() const { return *v_; }
  T *operator->() { return &*v_; }
  const T *operator->() const { return &*v_; }
  err_code error() const noexcept { return e_; }
  template <typename U>
  friend expected<U> make_unexpected(err_code e);

 private:
  std::optional<T> v_;
  err_code e_{};
};
template <typename T>
inline expected<T> make_unexpected(err_code e) {
  expected<T> r;
  r.v_.reset();
  r.e_ = e;
  return r;
}
#endif

namespace detail {

// ---- varint member traits (both builds name the types struct_pack::detail::
// varint<T> / sint<T>, varint.hpp:79-185,352-355) -----------------------------
template <typename T>
struct varint_traits : std::false_type {};
template <typename T>
struct varint_traits<struct_pack::detail::varint<T>> : std::true_type {
  using value_type = T;
  static constexpr bool zigzag = false;
};
template <typename T>
struct varint_traits<struct_pack::detail::sint<T>> : std::true_type {
  using value_type = T;
  static constexpr bool zigzag = true;
};

// ---- trivial_view<T> members (trivial_view.hpp:79-102) ----------------------
template <typename T>
struct trivial_view_traits : std::false_type {};
template <typename T, typename E>
struct trivial_view_traits<struct_pack::trivial_view<T, E>> : std::true_type {
  using value_type = T;
};

// ---- compatible<T, version> members (compatible.hpp:21-154) ------------------
template <typename T>
struct compat_traits : std::false_type {};
template <typename T, uint64_t V>
struct compat_traits<struct_pack::compatible<T, V>> : std::true_type {
  using value_type = T;
  static constexpr uint64_t version = V;
};

// ---- YLT_REFL detection: refl_object_to_tuple found by ADL (macro at
// namespace scope) or as a static member (macro inside the class) -------------
template <typename T>
concept ylt_refl_out = requires(T &t) { refl_object_to_tuple(t); };
template <typename T>
concept ylt_refl_in = requires(T &t) { T::refl_object_to_tuple(t); };
template <typename T>
constexpr bool is_ylt_refl_v = ylt_refl_out<T> || ylt_refl_in<T>;

template <typename T>
constexpr auto refl_tuple(T &t) {
  using U = std::remove_cv_t<T>;
  if constexpr (ylt_refl_in<U>)
    return U::refl_object_to_tuple(t);
  else
    return refl_object_to_tuple(t);
}

// ---- user alignment overrides (alignment.hpp:90-122) --------------------------
template <typename T>
constexpr std::size_t user_pack_alignment = struct_pack::pack_alignment_v<T>;
template <typename T>
constexpr std::size_t user_alignment = struct_pack::alignment_v<T>;

}  // namespace detail
}  // namespace struct_pack::gpu
