// walk.hpp — host-side extent walker over the struct_pack wire format.
//
// The device decoder needs a message's bytes in one buffer. Two reference
// entry points do not hand it one:
//   * deserialize_to(T&, Reader&) / get_field(Reader&) read from any reader_t
//     (read / ignore / tellg, reference reflection.hpp:110-114), field by
//     field, e.g. the reference's detail::memory_reader (unpacker.hpp:46-76)
//     or a socket-like reader that cannot seek;
//   * get_field<T, I> reads members 0..I only (unpacker.hpp:446-470,
//     1554-1592): the members before I are skipped one by one, each result
//     overwriting the last, and nothing after member I is read.
// walk_one<T> restates the reference's skip mode (deserialize_one<...,
// NotSkip = false>, unpacker.hpp:780-1420) over a cursor: the same reads in
// the same order, the same errc and the same dropped errc (optional /
// variant / unique_ptr values), but no values kept. The front end uses it to
// pull exactly one message's bytes out of a reader (pull_cursor), and to
// find member I of a get_field (mem_cursor). Values are decoded on the GPU.
#pragma once
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "layout.hpp"

namespace struct_pack::gpu::detail {

// ---- cursors -----------------------------------------------------------------
// A buffer in host memory with the reference memory_reader's rules
// (unpacker.hpp:46-76): a read or ignore that does not fit fails and
// consumes nothing.
struct mem_cursor {
  const char *d;
  std::size_t n;
  std::size_t pos = 0;
  bool read(void *dst, std::size_t k) {
    if (n - pos < k) return false;
    std::memcpy(dst, d + pos, k);
    pos += k;
    return true;
  }
  bool ignore(std::size_t k) {
    if (n - pos < k) return false;
    pos += k;
    return true;
  }
  std::size_t tell() const { return pos; }
};

// readers that report a short read through gcount (the std::istream family)
template <typename R>
concept counted_reader = requires(R &r) { r.gcount(); };

// bytes delivered by one read of a reader_t: an istream's partial read per
// gcount, any other reader (bool read) all or nothing
template <typename Reader>
std::size_t reader_read(Reader &r, char *p, std::size_t n) {
  if constexpr (counted_reader<Reader>) {
    r.read(p, static_cast<std::streamsize>(n));
    return static_cast<std::size_t>(r.gcount());
  } else {
    return r.read(p, n) ? n : 0;
  }
}

// Pulls the bytes the walk reads out of a reader into `buf`. Large runs are
// read in 1 MiB steps, as the reference reads a container from a reader
// without check() (unpacker.hpp:1166-1195), so a corrupted count never
// allocates more than the reader holds plus one step. After a short read the
// reader is dry: the partial bytes are dropped (the reference's read failed,
// it never used them) and every later read fails.
template <typename Reader>
struct pull_cursor {
  static constexpr std::size_t kStep = std::size_t(1) << 20;
  Reader &r;
  std::vector<char> &buf;
  bool dry = false;
  bool pull(std::size_t k) {
    if (dry) return false;
    while (k) {
      const std::size_t step = k < kStep ? k : kStep;
      const std::size_t at = buf.size();
      buf.resize(at + step);
      const std::size_t got = reader_read(r, buf.data() + at, step);
      if (got < step) {
        buf.resize(at);
        dry = true;
        return false;
      }
      k -= step;
    }
    return true;
  }
  bool read(void *dst, std::size_t k) {
    const std::size_t at = buf.size();
    if (!pull(k)) return false;
    std::memcpy(dst, buf.data() + at, k);
    return true;
  }
  bool ignore(std::size_t k) { return pull(k); }
  std::size_t tell() const { return buf.size(); }
};

// After a short read: every byte the reader can still deliver. A reader whose
// failed read consumed nothing (memory_reader) still holds the rest, and the
// reference's later reads see it; one whose failed read consumed the rest (an
// istream, a socket) delivers nothing more. Either way `buf` then holds
// exactly what the reference's read sequence could have read, so decoding
// it as a buffer in memory reproduces the reference's result.
template <typename Reader>
void drain(Reader &r, std::vector<char> &buf) {
  std::size_t step = std::size_t(1) << 16;
  while (step) {
    const std::size_t at = buf.size();
    buf.resize(at + step);
    const std::size_t got = reader_read(r, buf.data() + at, step);
    buf.resize(at + got);
    if (got == step) continue;
    if (counted_reader<Reader> || got) break;  // an istream ends at its first short read
    step /= 2;                                 // all-or-nothing: try less
  }
}

// ---- skip mode of the reference's deserialize_one -----------------------------
template <typename T, uint64_t tag = 0, typename Cur>
errc walk_one(Cur &c, uint32_t w);

template <typename Cur>
bool walk_count(Cur &c, uint32_t w, uint64_t &n) {
  unsigned char b[8] = {};
  if (!c.read(b, w)) return false;  // low_bytes_read_wrapper<w> (endian_wrapper.hpp:201-271)
  n = 0;
  for (uint32_t i = 0; i < w; ++i) n |= static_cast<uint64_t>(b[i]) << (8 * i);
  return true;
}

// count * size bytes of trivially serializable elements (unpacker.hpp:
// 1127-1132, 1199: the overflow check, then ignore)
template <typename Cur>
errc walk_bytes(Cur &c, uint64_t count, std::size_t size) {
  if (size > 1 && count > std::numeric_limits<std::size_t>::max() / size)
    return errc::no_buffer_space;
  return c.ignore(static_cast<std::size_t>(count * size)) ? errc{} : errc::no_buffer_space;
}

// LEB128 (varint.hpp:278-295): byte by byte, a 10th continuation byte is
// invalid_buffer
template <typename Cur>
errc walk_varint(Cur &c) {
  for (int i = 0; i < 10; ++i) {
    unsigned char b;
    if (!c.read(&b, 1)) return errc::no_buffer_space;
    if (!(b & 0x80u)) return {};
  }
  return errc::invalid_buffer;
}

template <typename T>
constexpr bool fixed_member_v = is_fundamental_v<T> || is_bitset_v<T>;

// members of a record whose config `cfg` makes some of them varints
template <typename M, uint64_t cfg, std::size_t... I>
constexpr std::size_t count_cfg_varints(std::index_sequence<I...>) {
  return ((varint_tid<std::tuple_element_t<I, M>, cfg>() != 0 ? 1u : 0u) + ... + 0u);
}
template <typename F>
constexpr std::size_t varint_value_size() {
  if constexpr (is_varint_v<F>)
    return sizeof(typename varint_traits<F>::value_type);
  else
    return sizeof(F);
}
template <typename M, uint64_t cfg, std::size_t... I>
constexpr bool has_64bit_cfg_varint(std::index_sequence<I...>) {
  return ((varint_tid<std::tuple_element_t<I, M>, cfg>() != 0 &&
           varint_value_size<std::tuple_element_t<I, M>>() == 8) ||
          ...);
}

// the fast-varint group of a record (unpacker.hpp:688-747): bitset + width
// code, then the non-zero members at min(2^code, size) bytes each
template <typename M, uint64_t cfg, typename Cur>
errc walk_fast_varints(Cur &c) {
  constexpr auto seq = std::make_index_sequence<std::tuple_size_v<M>>{};
  constexpr std::size_t cnt = count_cfg_varints<M, cfg>(seq);
  if constexpr (cnt == 0) {
    return {};
  } else {
    constexpr std::size_t bytes = (cnt + 2 + 7) / 8;
    unsigned char vec[bytes];
    if (!c.read(vec, bytes)) return errc::no_buffer_space;
    auto bit = [&](std::size_t i) { return (vec[i / 8] >> (i % 8)) & 1u; };
    const unsigned code = bit(cnt) + 2 * bit(cnt + 1);
    if (code == 3 && !has_64bit_cfg_varint<M, cfg>(seq)) return errc::invalid_buffer;
    const std::size_t width = std::size_t(1) << code;
    errc e{};
    std::size_t i = 0;
    [&]<std::size_t... J>(std::index_sequence<J...>) {
      auto one = [&](auto tagv) {
        using F = typename decltype(tagv)::type;
        if constexpr (varint_tid<F, cfg>() != 0) {
          const std::size_t idx = i++;
          if (!bit(idx)) return true;
          const std::size_t real = width < varint_value_size<F>() ? width : varint_value_size<F>();
          if (!c.ignore(real)) {
            e = errc::no_buffer_space;
            return false;
          }
        }
        return true;
      };
      (one(std::type_identity<std::tuple_element_t<J, M>>{}) && ...);
    }(seq);
    return e;
  }
}

template <std::size_t I, typename Var, typename Cur>
errc walk_alternative(Cur &c, uint32_t w, std::size_t idx) {
  if constexpr (I < std::variant_size_v<Var>) {
    if (idx == I) {
      using A = std::variant_alternative_t<I, Var>;
      if constexpr (!is_monostate_v<A>) (void)walk_one<A>(c, w);  // errc dropped (unpacker.hpp:476-490)
      return {};
    }
    return walk_alternative<I + 1, Var>(c, w, idx);
  } else {
    return {};
  }
}

// a record's members in order, stopping at the first error (deserialize_many,
// unpacker.hpp:621-630)
template <typename T, typename Cur>
errc walk_members(Cur &c, uint32_t w) {
  using M = members_tuple_t<T>;
  constexpr uint64_t cfg = type_config<T>() & kCfgVarintBits;
  if constexpr ((cfg & kCfgUseFastVarint) != 0) {
    if (errc e = walk_fast_varints<M, cfg>(c); e != errc{}) return e;
  }
  errc e{};
  [&]<std::size_t... J>(std::index_sequence<J...>) {
    ((e = walk_one<std::tuple_element_t<J, M>, cfg>(c, w), e == errc{}) && ...);
  }(std::make_index_sequence<std::tuple_size_v<M>>{});
  return e;
}

template <typename T, uint64_t tag, typename Cur>
errc walk_one(Cur &c, uint32_t w) {
  if constexpr (is_trivial_view_v<T>) {
    return c.ignore(sizeof(typename trivial_view_traits<T>::value_type)) ? errc{}
                                                                       : errc::no_buffer_space;
  } else if constexpr (is_compat_v<T> || is_monostate_v<T>) {
    return {};  // compatible: its version pass (unpacker.hpp:804-806)
  } else if constexpr (varint_tid<T, tag>() != 0) {
    if constexpr ((tag & kCfgUseFastVarint) != 0)
      return {};  // read with the record's fast-varint group
    else
      return walk_varint(c);
  } else if constexpr (fixed_member_v<T>) {
    return c.ignore(sizeof(T)) ? errc{} : errc::no_buffer_space;
  } else if constexpr (is_std_optional<T>::value) {  // optional / unique_ptr
    unsigned char has;
    if (!c.read(&has, 1)) return errc::no_buffer_space;
    if (has) (void)walk_one<opt_value_t<T>>(c, w);  // errc dropped (unpacker.hpp:856-880,1251-1277)
    return {};
  } else if constexpr (is_std_variant<T>::value) {
    unsigned char idx;
    if (!c.read(&idx, 1)) return errc::no_buffer_space;
    if (idx >= std::variant_size_v<T>) return errc::invalid_buffer;
    return walk_alternative<0, T>(c, w, idx);
  } else if constexpr (is_std_array<T>::value) {
    if constexpr (is_trivially_serializable<T>()) {
      return c.ignore(sizeof(T)) ? errc{} : errc::no_buffer_space;
    } else {
      for (std::size_t i = 0; i < std::tuple_size_v<T>; ++i)
        if (errc e = walk_one<typename T::value_type>(c, w); e != errc{}) return e;
      return {};
    }
  } else if constexpr (is_string_v<T> || is_container_v<T>) {
    uint64_t n;
    if (!walk_count(c, w, n)) return errc::no_buffer_space;
    if (n == 0) return {};
    if constexpr (is_string_v<T>) {
      return walk_bytes(c, n, sizeof(string_char_t<T>));
    } else {
      using E = elem_t<T>;
      // contiguous containers of trivially serializable elements, and set /
      // map containers of them in skip mode: one ignore (unpacker.hpp:
      // 984-995, 1097-1107, 1126-1200); anything else element by element
      if constexpr (is_trivially_serializable<E>() &&
                    (is_contiguous_v<T> || is_set_v<T> || is_map_v<T>)) {
        return walk_bytes(c, n, sizeof(E));
      } else {
        for (uint64_t i = 0; i < n; ++i)
          if (errc e = walk_one<E>(c, w); e != errc{}) return e;
        return {};
      }
    }
  } else if constexpr (is_record_v<T>) {
    if constexpr (is_trivially_serializable<T>())
      return c.ignore(sizeof(T)) ? errc{} : errc::no_buffer_space;
    else
      return walk_members<T>(c, w);
  } else {
    static_assert(dependent_false_v<T>, "struct_pack::gpu: type outside the record model");
    return {};
  }
}

// ---- message header --------------------------------------------------------
// deserialize_metainfo's reads (unpacker.hpp:548-619) for message format f:
// the width `w` and the compatible-data length (0: none) of the message.
// Stops at a head that is not f's (invalid_buffer); the literal is read, not
// compared (the decode of the pulled bytes compares it).
struct header_info {
  uint32_t w = 1;
  uint64_t data_len = 0;
};
template <typename Cur>
errc walk_header(Cur &c, const spk_msgfmt &f, header_info &h) {
  unsigned char meta = 0;
  if (!(f.flags & SPK_MF_HASH_HEAD)) {
    if (f.flags & SPK_MF_HAS_CONTAINER) {
      if (!c.read(&meta, 1)) return errc::no_buffer_space;
      h.w = 1u << ((meta >> 3) & 3u);
    }
    return {};
  }
  unsigned char hd[4];
  if (!c.read(hd, 4)) return errc::no_buffer_space;
  const uint32_t head = hd[0] | hd[1] << 8 | hd[2] << 16 | static_cast<uint32_t>(hd[3]) << 24;
  if (head / 2 != f.code / 2) return errc::invalid_buffer;
  if (!(head & 1u)) return {};
  if (!c.read(&meta, 1)) return errc::no_buffer_space;
  if (const unsigned cl = meta & 3u) {
    uint64_t len;
    if (!walk_count(c, 1u << cl, len)) return errc::no_buffer_space;
    h.data_len = len;
  }
  if (meta & 4u)
    if (!c.ignore(f.literal_len + 1)) return errc::no_buffer_space;
  h.w = 1u << ((meta >> 3) & 3u);
  return {};
}

// ---- compatible members: the version passes (unpacker.hpp:292-366) ---------------
template <typename F>
constexpr uint64_t compat_version() {
  if constexpr (is_compat_v<F>)
    return compat_traits<F>::version;
  else
    return std::numeric_limits<uint64_t>::max();
}
template <typename M, std::size_t... I>
constexpr std::size_t compat_count(std::index_sequence<I...>) {
  return (std::size_t{is_compat_v<std::tuple_element_t<I, M>>} + ... + 0u);
}
template <typename T>
constexpr bool record_has_compat() {
  if constexpr (is_record_v<T> && !is_trivially_serializable<T>()) {
    using M = members_tuple_t<T>;
    return compat_count<M>(std::make_index_sequence<std::tuple_size_v<M>>{}) > 0;
  } else {
    return false;
  }
}
// the sorted distinct versions of T's compatible members
template <typename T>
std::vector<uint64_t> compat_versions() {
  std::vector<uint64_t> v;
  if constexpr (record_has_compat<T>()) {
    using M = members_tuple_t<T>;
    [&]<std::size_t... J>(std::index_sequence<J...>) {
      auto add = [&](uint64_t x) {
        if (x == std::numeric_limits<uint64_t>::max()) return;
        auto it = v.begin();
        while (it != v.end() && *it < x) ++it;
        if (it == v.end() || *it != x) v.insert(it, x);
      };
      (add(compat_version<std::tuple_element_t<J, M>>()), ...);
    }(std::make_index_sequence<std::tuple_size_v<M>>{});
  }
  return v;
}

// one compatible member in its version pass, skip mode (unpacker.hpp:
// 1354-1376): at or past the data length the pass ends (`past`, not an
// error once the passes are over)
template <typename F, typename Cur>
errc walk_compat_member(Cur &c, uint32_t w, uint64_t data_len, bool &past) {
  if (c.tell() >= data_len) {
    past = true;
    return errc::no_buffer_space;
  }
  unsigned char has;
  if (!c.read(&has, 1)) return errc::no_buffer_space;
  if (has) (void)walk_one<typename compat_traits<F>::value_type>(c, w);  // errc dropped
  return {};
}

// the version passes of a whole record message (deserialize_compatibles,
// unpacker.hpp:292-366): each pass reads that version's members in order and
// stops at the first error; the passes stop at the first failing one
template <typename T, typename Cur>
errc walk_versions(Cur &c, uint32_t w, uint64_t data_len, bool &past) {
  using M = members_tuple_t<T>;
  errc e{};
  for (uint64_t v : compat_versions<T>()) {
    [&]<std::size_t... J>(std::index_sequence<J...>) {
      auto one = [&](auto tagv) {
        using F = typename decltype(tagv)::type;
        if constexpr (is_compat_v<F>) {
          if (compat_traits<F>::version == v) e = walk_compat_member<F>(c, w, data_len, past);
        }
        return e == errc{};
      };
      (one(std::type_identity<std::tuple_element_t<J, M>>{}) && ...);
    }(std::make_index_sequence<std::tuple_size_v<M>>{});
    if (e != errc{}) break;
  }
  return e;
}

// the version passes of a vector<R> message (deserialize_compatibles over
// the container, unpacker.hpp:1397-1404): each pass visits R's members of
// that version in every one of the n records, in record order
template <typename R, typename Cur>
errc walk_versions_vec(Cur &c, uint32_t w, uint64_t n, uint64_t data_len, bool &past) {
  using M = members_tuple_t<R>;
  errc e{};
  for (uint64_t v : compat_versions<R>()) {
    for (uint64_t i = 0; i < n && e == errc{}; ++i) {
      [&]<std::size_t... J>(std::index_sequence<J...>) {
        auto one = [&](auto tagv) {
          using F = typename decltype(tagv)::type;
          if constexpr (is_compat_v<F>) {
            if (compat_traits<F>::version == v) e = walk_compat_member<F>(c, w, data_len, past);
          }
          return e == errc{};
        };
        (one(std::type_identity<std::tuple_element_t<J, M>>{}) && ...);
      }(std::make_index_sequence<std::tuple_size_v<M>>{});
    }
    if (e != errc{}) break;
  }
  return e;
}


// ---- views alias the input (unpacker.hpp:787-800, 1135-1145) ---------------
// std::string_view / std::span / trivial_view members decoded by the
// reference point into the buffer it read. The device decode writes their
// bytes into host staging; rebase_views walks the decoded value and the wire
// side by side (both are the same message, already decoded without error) and
// points every view at its bytes in the caller's buffer instead, so a view
// lives exactly as long as that buffer (coro_rpc keeps a request's buffer
// alive for the handler).
template <typename T>
constexpr bool has_views();
template <typename M, std::size_t... I>
constexpr bool any_views(std::index_sequence<I...>) {
  return (has_views<std::tuple_element_t<I, M>>() || ...);
}
template <typename V>
struct variant_views;
template <typename... A>
struct variant_views<std::variant<A...>> {
  static constexpr bool value = (has_views<A>() || ...);
};
template <typename T>
constexpr bool has_views() {
  if constexpr (is_trivial_view_v<T> || is_string_view_v<T> || is_std_span<T>::value) {
    return true;
  } else if constexpr (is_string_v<T> || is_fundamental_v<T> || is_varint_v<T> ||
                       is_bitset_v<T> || is_monostate_v<T>) {
    return false;
  } else if constexpr (is_container_v<T>) {
    return has_views<elem_t<T>>();
  } else if constexpr (is_std_optional<T>::value || is_compat_v<T>) {
    return has_views<opt_value_t<T>>();
  } else if constexpr (is_std_variant<T>::value) {
    return variant_views<T>::value;
  } else if constexpr (is_std_array<T>::value) {
    return has_views<typename T::value_type>();
  } else if constexpr (is_record_v<T>) {
    using M = members_tuple_t<T>;
    return any_views<M>(std::make_index_sequence<std::tuple_size_v<M>>{});
  } else {
    return false;
  }
}

template <typename T, uint64_t tag = 0>
void rebase_views(T &v, mem_cursor &c, uint32_t w);

template <typename T>
void rebase_members(T &v, mem_cursor &c, uint32_t w) {
  constexpr uint64_t cfg = type_config<T>() & kCfgVarintBits;
  using M = members_tuple_t<T>;
  if constexpr ((cfg & kCfgUseFastVarint) != 0) (void)walk_fast_varints<M, cfg>(c);
  auto tied = tie_members(v);
  [&]<std::size_t... J>(std::index_sequence<J...>) {
    (rebase_views<std::tuple_element_t<J, M>, cfg>(
         const_cast<std::tuple_element_t<J, M> &>(std::get<J>(tied)), c, w),
     ...);
  }(std::make_index_sequence<std::tuple_size_v<M>>{});
}

template <typename T, uint64_t tag>
void rebase_views(T &v, mem_cursor &c, uint32_t w) {
  if constexpr (!has_views<T>()) {
    (void)walk_one<T, tag>(c, w);
  } else if constexpr (is_trivial_view_v<T>) {
    using E = typename trivial_view_traits<T>::value_type;
    v = T(reinterpret_cast<const E *>(c.d + c.pos));
    c.pos += sizeof(E);
  } else if constexpr (is_string_view_v<T> || is_std_span<T>::value) {
    using E = std::remove_cv_t<typename T::value_type>;
    uint64_t n = 0;
    (void)walk_count(c, w, n);
    v = T(reinterpret_cast<const E *>(c.d + c.pos), static_cast<std::size_t>(n));
    c.pos += static_cast<std::size_t>(n) * sizeof(E);
  } else if constexpr (is_container_v<T>) {
    uint64_t n = 0;
    (void)walk_count(c, w, n);
    for (auto &e : v) {  // a map's pair<const K, V>: both parts
      if constexpr (is_map_v<T>) {
        rebase_views(const_cast<remove_cvref_t<decltype(e.first)> &>(e.first), c, w);
        rebase_views(e.second, c, w);
      } else {
        rebase_views(const_cast<remove_cvref_t<decltype(e)> &>(e), c, w);
      }
    }
  } else if constexpr (is_std_optional<T>::value) {
    ++c.pos;  // has_value
    if (v) rebase_views(*v, c, w);
  } else if constexpr (is_std_variant<T>::value) {
    ++c.pos;  // index
    std::visit([&](auto &a) { rebase_views(a, c, w); }, v);
  } else if constexpr (is_std_array<T>::value) {
    for (auto &e : v) rebase_views(e, c, w);
  } else if constexpr (is_compat_v<T>) {
    static_assert(dependent_false_v<T>, "views inside compatible members are not supported");
  } else {
    rebase_members(v, c, w);
  }
}

}  // namespace struct_pack::gpu::detail
