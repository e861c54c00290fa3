// struct_pack_gpu.hpp — MI355X-native struct_pack front end (our
// implementation), namespace struct_pack::gpu.
//
// Keeps the reference's entry-point names, argument order, argument meaning
// and error values (reference include/ylt/struct_pack.hpp:75-658,
// error_code.hpp:21-64) and produces the reference's wire bytes exactly. The
// byte work runs in the gfx950 HIP kernels of libspk_codec.so behind the C
// ABI of include/spk_codec.h; this header reflects types, builds the layout
// descriptor, stages host objects and calls the ABI. There is no CPU codec
// and no HIP header here: device memory, copies and streams also go through
// the C ABI, so any C++20 compiler can build a caller.
//
// It compiles next to the reference header (then struct_pack::errc,
// sp_config, var_int32_t ... ARE the reference's, see config.hpp) or alone.
//
//   get_type_code<T>() / get_type_literal<T>()          compile time
//   get_needed_size(t)                                   size pass (device)
//   serialize(t) / serialize<Buffer>(t) / serialize<conf, Buffer>(t)
//   serialize_to(buffer|writer, t) / serialize_to(char*, serialize_buffer_size, t)
//   serialize_to_with_offset(buffer, offset, t) / serialize_with_offset(offset, t)
//   deserialize_to(t, view|data,size [, consume_len])
//   deserialize_to_with_offset(t, view|data,size, offset)
//   deserialize<T>(view|data,size [, consume_len]) / deserialize<conf, T>(...)
//   get_field<T, I>(view|data,size)
//       t = std::vector<R> (or std::span<R> to serialize): one message of
//           records, SPK_MODE_VECTOR; t = R: one record message
//           (SPK_MODE_MESSAGES with one message)
//   serialize_messages / deserialize_messages           coro_rpc payload batches
//   serialize_frames / deserialize_frames               ... in coro_rpc's framing
//   device::codec<R>                                     device-resident batches
//
// Build: <c++20 compiler> -I include ... -L yalantinglibs_amd -lspk_codec
#pragma once
#include <cstdlib>
#include <cstring>
#include <ios>
#include <memory>
#include <span>
#include <stdexcept>
#include <string>
#include <string_view>
#include <type_traits>
#include <vector>

#include "../spk_codec.h"
#include "struct_pack_gpu/layout.hpp"
#include "struct_pack_gpu/walk.hpp"

namespace struct_pack::gpu {

// Device / ABI failures (not wire errors: those come back as errc, never as
// exceptions, like the reference's decoder)
class spk_error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// serialize_buffer_size (calculate_size.hpp:391-405): message length and
// metainfo byte of a planned message
struct serialize_buffer_size {
  std::size_t len_ = 0;
  unsigned char metainfo_ = 0;
  constexpr std::size_t size() const { return len_; }
  constexpr unsigned char metainfo() const { return metainfo_; }
  constexpr operator std::size_t() const { return len_; }
};

namespace detail {

// ---- what the batch model covers (compile-time, SFINAE-friendly) -----------
template <typename T>
constexpr bool supported();
template <typename M, std::size_t... I>
constexpr bool all_supported(std::index_sequence<I...>) {
  return (supported<std::tuple_element_t<I, M>>() && ...);
}
template <typename V>
struct variant_supported;
template <typename... A>
struct variant_supported<std::variant<A...>> {
  static constexpr bool value = ((is_monostate_v<A> || supported<A>()) && ...);
};
template <typename T>
constexpr bool supported() {
  if constexpr (is_fundamental_v<T> || is_string_v<T> || is_varint_v<T> || is_bitset_v<T>) {
    return true;
  } else if constexpr (is_trivial_view_v<T>) {
    return is_trivially_serializable<typename trivial_view_traits<T>::value_type>();
  } else if constexpr (is_container_v<T>) {
    return supported<elem_t<T>>();
  } else if constexpr (is_std_optional<T>::value || is_compat_v<T>) {
    return supported<opt_value_t<T>>();
  } else if constexpr (is_std_variant<T>::value) {
    return variant_supported<T>::value;
  } else if constexpr (is_std_array<T>::value) {
    return supported<typename T::value_type>();
  } else if constexpr (is_record_v<T>) {
    using M = members_tuple_t<T>;
    return all_supported<M>(std::make_index_sequence<std::tuple_size_v<M>>{});
  } else {
    return false;
  }
}
// a record type the batch codec encodes as the element of a message
template <typename R>
constexpr bool record_supported() {
  if constexpr (is_record_v<R> || is_fundamental_v<R> || is_std_array<R>::value)
    return supported<R>();
  else
    return false;
}

// the argument of serialize / deserialize_to:
//  * std::vector<R> / std::span<R> of records R: a VECTOR message;
//  * a record R (aggregate, YLT_REFL type, std::pair, std::tuple -- the
//    message of a multi-argument call --, fundamental, std::array): one
//    MESSAGES message of R;
//  * any other supported type M (std::string, a container of non-records, an
//    optional, a variant, a map ...): one message of the record boxed<M>,
//    whose payload bytes are M's, under M's type code (boxed = true);
//  * std::monostate (the reply of a void handler, struct_pack_protocol.hpp:
//    34-36): a message without payload, its header alone (empty = true).
template <typename T, bool = record_supported<T>()>
struct msg_traits_of {
  static constexpr bool vector = false, record = true, boxed = false, empty = false;
  using rec = T;
};
template <typename T>
struct msg_traits_of<T, false> {
  static constexpr bool empty = is_monostate_v<T>;
  static constexpr bool vector = false, record = empty || (supported<T>() && !is_compat_v<T>),
                        boxed = !empty;
  using rec = detail::boxed<T>;
};
template <typename T>
struct msg_traits : msg_traits_of<T> {};
template <typename R, typename A>
struct msg_traits<std::vector<R, A>> : msg_traits_of<std::vector<R, A>> {
  static constexpr bool vector = record_supported<R>(),
                        record = !vector && msg_traits_of<std::vector<R, A>>::record,
                        boxed = !vector;
  using rec = std::conditional_t<vector, R, detail::boxed<std::vector<R, A>>>;
};
template <typename R, std::size_t E>
struct msg_traits<std::span<R, E>> {
  static constexpr bool vector = E == std::dynamic_extent && record_supported<remove_cvref_t<R>>(),
                        record = false, boxed = false, empty = false;
  using rec = remove_cvref_t<R>;
};

}  // namespace detail

// true when the GPU front end handles `T` as a whole message
template <typename T>
constexpr bool is_gpu_message_v =
    detail::msg_traits<detail::remove_cvref_t<T>>::vector ||
    detail::msg_traits<detail::remove_cvref_t<T>>::record;
// true for a batch message: std::vector<R> / std::span<R> of records
template <typename T>
constexpr bool is_gpu_batch_v = detail::msg_traits<detail::remove_cvref_t<T>>::vector;

namespace device {

inline void check(int rc, const char *what) {
  if (rc != SPK_OK) throw spk_error(std::string("struct_pack::gpu: ") + what + " failed (" +
                                    std::to_string(rc) + ")");
}

// RAII device allocation (spk_device_alloc)
class buffer {
 public:
  buffer() = default;
  explicit buffer(std::size_t n) { resize(n); }
  buffer(const buffer &) = delete;
  buffer &operator=(const buffer &) = delete;
  buffer(buffer &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr, o.n_ = 0; }
  buffer &operator=(buffer &&o) noexcept {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    return *this;
  }
  ~buffer() {
    if (p_) (void)spk_device_free(p_);
  }
  void resize(std::size_t n) {  // grows only; contents not preserved
    if (n <= n_ && p_) return;
    if (p_) check(spk_device_free(p_), "spk_device_free");
    p_ = nullptr;
    n_ = 0;
    check(spk_device_alloc(&p_, n ? n : 1), "spk_device_alloc");
    n_ = n;
  }
  void *data() const { return p_; }
  std::size_t size() const { return n_; }

 private:
  void *p_ = nullptr;
  std::size_t n_ = 0;
};

// RAII pinned host allocation (spk_host_alloc_pinned), grows only
class pinned {
 public:
  pinned() = default;
  pinned(const pinned &) = delete;
  pinned &operator=(const pinned &) = delete;
  ~pinned() {
    if (p_) (void)spk_host_free_pinned(p_);
  }
  void resize(std::size_t n) {  // contents not preserved
    if (n <= n_ && p_) return;
    if (p_) check(spk_host_free_pinned(p_), "spk_host_free_pinned");
    p_ = nullptr;
    n_ = 0;
    check(spk_host_alloc_pinned(&p_, n ? n : 1), "spk_host_alloc_pinned");
    n_ = n;
  }
  uint8_t *data() const { return static_cast<uint8_t *>(p_); }

 private:
  void *p_ = nullptr;
  std::size_t n_ = 0;
};

inline void copy(void *dst, const void *src, std::size_t n, int kind, void *s) {
  check(spk_copy_async(dst, src, n, kind, s), "spk_copy_async");
}
inline void sync(void *s) { check(spk_stream_sync(s), "spk_stream_sync"); }


// A batch of R in device memory: device records + one heap per span.
template <typename R>
struct batch {
  buffer recs;
  std::vector<buffer> heaps;
  std::vector<uint64_t> heap_elems;
  std::size_t n = 0;
};

template <typename R, uint64_t conf = sp_config::DEFAULT>
class codec {
 public:
  explicit codec(void *stream = nullptr) : s_(stream) {}

  static const spk_layout &layout() {
    static const spk_layout L = [] {
      spk_layout l = make_spk_layout<R, conf>();
      check(spk_layout_check(&l), "spk_layout_check");
      return l;
    }();
    return L;
  }
  static constexpr bool trivial = detail::is_trivially_serializable<R>();

  // ---- staging (host <-> device) -----------------------------------------
  // X = R, or M for R = boxed<M> (the message marshalled as boxed<M>'s one
  // member, without a copy: a std::unique_ptr message cannot be copied)
  template <typename X = R>
  batch<R> upload(const X *v, std::size_t n) {
    const spk_layout &L = layout();
    batch<R> b;
    b.n = n;
    b.recs.resize(n * L.rec_stride);
    if constexpr (trivial && std::is_same_v<X, R>) {
      copy(b.recs.data(), v, n * sizeof(R), SPK_COPY_H2D, s_);
      sync(s_);
    } else {
      std::vector<uint8_t> recs(n * L.rec_stride, 0);
      std::vector<std::vector<uint8_t>> heaps(n_spans());
      for (std::size_t i = 0; i < n; ++i) {
        detail::marshal_state st{&L, recs.data() + i * L.rec_stride, 0, 0, &heaps, 0};
        detail::to_device(v[i], st);
      }
      copy(b.recs.data(), recs.data(), recs.size(), SPK_COPY_H2D, s_);
      for (uint32_t k = 0; k < n_spans(); ++k) {
        b.heaps.emplace_back(heaps[k].size());
        b.heap_elems.push_back(heaps[k].size() / span_elem(k));
        copy(b.heaps[k].data(), heaps[k].data(), heaps[k].size(), SPK_COPY_H2D, s_);
      }
      sync(s_);  // host staging buffers die here
    }
    return b;
  }

  // ok(i) selects the records to materialise (failed messages stay default);
  // X = R, or M for R = boxed<M>
  template <typename X = R, typename Pred = std::nullptr_t>
  void download(const batch<R> &b, std::size_t n, X *out, Pred ok = nullptr) {
    const spk_layout &L = layout();
    if constexpr (trivial && std::is_same_v<X, R>) {
      copy(out, b.recs.data(), n * sizeof(R), SPK_COPY_D2H, s_);
      sync(s_);
    } else {
      // kept in the codec: string_view / span / trivial_view members of the
      // decoded objects alias these host records and heaps, valid until this
      // thread's next decode of R; the decode entry points that take the
      // wire from the caller then point them into the caller's buffer
      // (rebase_views), as the reference's views alias its input
      // (unpacker.hpp:787-800,1135-1145)
      std::vector<uint8_t> &recs = view_recs_;
      recs.assign(n * L.rec_stride, 0);
      std::vector<std::vector<uint8_t>> &heaps = view_heaps_;
      heaps.assign(n_spans(), {});
      copy(recs.data(), b.recs.data(), recs.size(), SPK_COPY_D2H, s_);
      std::vector<const uint8_t *> hp(n_spans());
      for (uint32_t k = 0; k < n_spans(); ++k) {
        heaps[k].resize(b.heap_elems[k] * span_elem(k));
        copy(heaps[k].data(), b.heaps[k].data(), heaps[k].size(), SPK_COPY_D2H, s_);
        hp[k] = heaps[k].data();
      }
      sync(s_);
      for (std::size_t i = 0; i < n; ++i) {
        if constexpr (!std::is_same_v<Pred, std::nullptr_t>)
          if (!ok(i)) continue;
        detail::unmarshal_state st{&L, recs.data() + i * L.rec_stride, 0, 0, hp.data(), 0};
        detail::from_device(out[i], st);
      }
    }
  }

  // ---- one small message per call (the coro_rpc seam) ---------------------
  // A per-thread device arena and a pinned staging buffer with the same
  // layout, both reused across calls (grown, never freed per call): the
  // records and heaps go to the device in ONE copy, plan + encode (or the
  // decode) run stream-ordered in the arena, the plan / result and the
  // output come back in ONE copy, and the call syncs once. No allocation
  // after the first call of a size. Calls larger than kSmallBytes take the
  // batch path (upload / plan / encode / download).
  static constexpr std::size_t kSmallBytes = std::size_t(1) << 20;
  static constexpr std::size_t al(std::size_t x) { return (x + 255) & ~std::size_t(255); }

  // Marshal n values into the encode scratch (records + one vector per heap).
  template <typename X = R>
  std::size_t marshal(const X *v, std::size_t n) {
    const spk_layout &L = layout();
    mrecs_.assign(n * L.rec_stride, 0);
    mheaps_.resize(n_spans());
    for (auto &h : mheaps_) h.clear();
    if constexpr (trivial && std::is_same_v<X, R>) {
      if (n) std::memcpy(mrecs_.data(), v, n * sizeof(R));
    } else {
      for (std::size_t i = 0; i < n; ++i) {
        detail::marshal_state st{&L, mrecs_.data() + i * L.rec_stride, 0, 0, &mheaps_, 0};
        detail::to_device(v[i], st);
      }
    }
    std::size_t b = mrecs_.size();
    for (auto &h : mheaps_) b += h.size();
    return b;
  }

  // serialize n values as one message (VECTOR) or one record message
  // (MESSAGES, n == 1): returns false (nothing done) when the call is not
  // small; otherwise sink(bytes, len) gets the message.
  template <typename X, typename Sink>
  bool encode_small(const X *v, std::size_t n, int mode, Sink &&sink) {
    const spk_layout &L = layout();
    const std::size_t in_bytes = marshal(v, n);
    if (in_bytes > kSmallBytes) return false;
    // arena: [plan 256][out cap][offsets 256][records][heap 0]...[heap k]
    // (the first two come back in one D2H, the rest goes over in one H2D)
    const std::size_t out_cap = al(2 * in_bytes + 16 * n + 4096);
    const std::size_t o_out = 256, o_offs = o_out + out_cap, o_recs = o_offs + 256;
    std::size_t end = al(o_recs + mrecs_.size());
    std::vector<std::size_t> o_heap(n_spans());
    for (uint32_t k = 0; k < n_spans(); ++k) {
      o_heap[k] = end;
      end = al(end + mheaps_[k].size());
    }
    arena_.resize(end);
    pin_.resize(end);
    uint8_t *hp = pin_.data(), *dp = static_cast<uint8_t *>(arena_.data());
    if (!mrecs_.empty()) std::memcpy(hp + o_recs, mrecs_.data(), mrecs_.size());
    std::vector<const void *> dheaps(n_spans() ? n_spans() : 1, nullptr);
    for (uint32_t k = 0; k < n_spans(); ++k) {
      if (!mheaps_[k].empty()) std::memcpy(hp + o_heap[k], mheaps_[k].data(), mheaps_[k].size());
      dheaps[k] = dp + o_heap[k];
    }
    if (end > o_recs) copy(dp + o_recs, hp + o_recs, end - o_recs, SPK_COPY_H2D, s_);
    ws_.resize(spk_workspace_bytes(&L, mode, n, 0));
    spk_plan_t *d_plan = reinterpret_cast<spk_plan_t *>(dp);
    uint64_t *d_offs = mode == SPK_MODE_MESSAGES ? reinterpret_cast<uint64_t *>(dp + o_offs) : nullptr;
    // (plan + write: one launch for a small flat variable-size message)
    check(spk_plan_encode(&L, mode, n, dp + o_recs, dheaps.data(), d_plan, dp + o_out, out_cap,
                          d_offs, ws_.data(), ws_.size(), s_), "spk_plan_encode");
    copy(hp, dp, o_out + out_cap, SPK_COPY_D2H, s_);
    sync(s_);
    spk_plan_t p;
    std::memcpy(&p, hp, sizeof p);
    last_plan_ = p;
    if (p.total_bytes <= out_cap) {
      sink(reinterpret_cast<const char *>(hp + o_out), static_cast<std::size_t>(p.total_bytes));
      return true;
    }
    // (a bound that did not hold: encode again into an exact buffer; the
    // plan and workspace in the arena are still this message's)
    buffer big(p.total_bytes);
    check(spk_encode(&L, mode, n, dp + o_recs, dheaps.data(), d_plan, big.data(), p.total_bytes,
                     d_offs, ws_.data(), ws_.size(), s_), "spk_encode");
    std::vector<char> tmp(p.total_bytes);
    copy(tmp.data(), big.data(), tmp.size(), SPK_COPY_D2H, s_);
    sync(s_);
    sink(tmp.data(), tmp.size());
    return true;
  }
  const spk_plan_t &last_plan() const { return last_plan_; }

  // decode one message of `size` bytes (VECTOR into at most cap records, or
  // one MESSAGES record): false when the call is not small; otherwise r is
  // the result and, when r.errc == 0, the records / heaps are in the host
  // view buffers (view_recs_ / view_heaps_) for unmarshal().
  bool decode_small(const char *data, std::size_t size, int mode, std::size_t cap,
                    spk_dresult_t &r) {
    const spk_layout &L = layout();
    const std::vector<uint64_t> caps = detail::heap_caps_for_wire(L, size, cap);
    // arena: [result 256][errc 256][records][heap 0]...[heap k] | [offsets 256][wire]
    const std::size_t o_errc = 256, o_recs = 512;
    std::size_t end = al(o_recs + cap * L.rec_stride);
    std::vector<std::size_t> o_heap(n_spans());
    for (uint32_t k = 0; k < n_spans(); ++k) {
      o_heap[k] = end;
      end = al(end + caps[k] * span_elem(k));
    }
    const std::size_t back = end, o_offs = end, o_wire = end + 256;
    end = al(o_wire + size + 16);
    if (back > kSmallBytes || size > kSmallBytes) return false;
    arena_.resize(end);
    pin_.resize(end);
    uint8_t *hp = pin_.data(), *dp = static_cast<uint8_t *>(arena_.data());
    const uint64_t o[2] = {0, size};
    std::memcpy(hp + o_offs, o, sizeof o);
    if (size) std::memcpy(hp + o_wire, data, size);
    copy(dp + o_offs, hp + o_offs, o_wire + size - o_offs, SPK_COPY_H2D, s_);
    ws_.resize(spk_workspace_bytes(&L, mode, mode == SPK_MODE_VECTOR ? cap : 1, size));
    std::vector<void *> dheaps(n_spans() ? n_spans() : 1, nullptr);
    for (uint32_t k = 0; k < n_spans(); ++k) dheaps[k] = dp + o_heap[k];
    spk_dresult_t *d_res = reinterpret_cast<spk_dresult_t *>(dp);
    int32_t *d_errc = mode == SPK_MODE_MESSAGES ? reinterpret_cast<int32_t *>(dp + o_errc) : nullptr;
    check(spk_decode(&L, mode, dp + o_wire, size,
                     mode == SPK_MODE_MESSAGES ? reinterpret_cast<const uint64_t *>(dp + o_offs)
                                               : nullptr,
                     mode == SPK_MODE_MESSAGES ? 1 : 0, dp + o_recs, cap, dheaps.data(),
                     caps.data(), d_res, d_errc, ws_.data(), ws_.size(), s_), "spk_decode");
    copy(hp, dp, back, SPK_COPY_D2H, s_);
    sync(s_);
    std::memcpy(&r, hp, sizeof r);
    if (mode == SPK_MODE_MESSAGES) std::memcpy(&r.errc, hp + o_errc, sizeof r.errc);
    if (r.errc) return true;
    const std::size_t nrec = mode == SPK_MODE_VECTOR ? r.count : 1;
    view_recs_.assign(hp + o_recs, hp + o_recs + nrec * L.rec_stride);
    view_heaps_.resize(n_spans());
    for (uint32_t k = 0; k < n_spans(); ++k)
      view_heaps_[k].assign(hp + o_heap[k], hp + o_heap[k] + r.heap_used[k] * span_elem(k));
    return true;
  }

  // the n records held in the host view buffers -> out (decode_small)
  template <typename X = R>
  void unmarshal(std::size_t n, X *out) {
    const spk_layout &L = layout();
    if constexpr (trivial && std::is_same_v<X, R>) {
      if (n) std::memcpy(static_cast<void *>(out), view_recs_.data(), n * sizeof(R));
    } else {
      std::vector<const uint8_t *> hp(n_spans());
      for (uint32_t k = 0; k < n_spans(); ++k) hp[k] = view_heaps_[k].data();
      for (std::size_t i = 0; i < n; ++i) {
        detail::unmarshal_state st{&L, view_recs_.data() + i * L.rec_stride, 0, 0, hp.data(), 0};
        detail::from_device(out[i], st);
      }
    }
  }

  // ---- device-resident codec ----------------------------------------------
  spk_plan_t plan(const batch<R> &b, int mode) {
    ws_.resize(spk_workspace_bytes(&layout(), mode, b.n, 0));
    plan_.resize(sizeof(spk_plan_t));
    std::vector<const void *> hp = heap_ptrs(b);
    check(spk_plan_ex(&layout(), mode, b.n, b.recs.data(), hp.data(), (spk_plan_t *)plan_.data(),
                      ws_.data(), ws_.size(), s_),
          "spk_plan_ex");
    spk_plan_t p{};
    copy(&p, plan_.data(), sizeof(p), SPK_COPY_D2H, s_);
    sync(s_);
    return p;
  }

  // after plan(): write into d_out (device). Stream-ordered, no sync.
  void encode(const batch<R> &b, int mode, void *d_out, std::size_t cap,
              uint64_t *d_offsets = nullptr) {
    std::vector<const void *> hp = heap_ptrs(b);
    check(spk_encode(&layout(), mode, b.n, b.recs.data(), hp.data(),
                     (const spk_plan_t *)plan_.data(), d_out, cap, d_offsets, ws_.data(),
                     ws_.size(), s_), "spk_encode");
  }

  // after plan(SPK_MODE_MESSAGES): n framed messages [prefix][serialize(rec)]
  void encode_framed(const batch<R> &b, const spk_frame &f, void *d_out, std::size_t cap,
                     uint64_t *d_offsets = nullptr) {
    std::vector<const void *> hp = heap_ptrs(b);
    check(spk_encode_framed(&layout(), b.n, b.recs.data(), hp.data(),
                            (const spk_plan_t *)plan_.data(), &f, d_out, cap, d_offsets,
                            ws_.data(), ws_.size(), s_), "spk_encode_framed");
  }

  // after plan(SPK_MODE_MESSAGES): framed messages whose seq_num is the u32 at
  // d_seq_src[d_seq_offsets[i] + seq_src_off] (responses echoing the routed
  // requests, coro_rpc_protocol.hpp:191-201)
  void encode_framed_echo(const batch<R> &b, const spk_frame &f, const void *d_seq_src,
                          const uint64_t *d_seq_offsets, uint32_t seq_src_off, void *d_out,
                          std::size_t cap, uint64_t *d_offsets = nullptr) {
    std::vector<const void *> hp = heap_ptrs(b);
    check(spk_encode_framed_echo(&layout(), b.n, b.recs.data(), hp.data(),
                                 (const spk_plan_t *)plan_.data(), &f, d_seq_src, d_seq_offsets,
                                 seq_src_off, d_out, cap, d_offsets, ws_.data(), ws_.size(), s_),
          "spk_encode_framed_echo");
  }

  // decode frames that need not be adjacent: message i = d_wire[d_begins[i] +
  // prefix, d_ends[i]) (one function id's lists from a frame_router)
  spk_dresult_t decode_frames(batch<R> &out, const void *d_wire, std::size_t len,
                              const uint64_t *d_begins, const uint64_t *d_ends, std::size_t n,
                              uint32_t prefix, int32_t *d_errc = nullptr) {
    ws_.resize(spk_workspace_bytes(&layout(), SPK_MODE_MESSAGES, n, len));
    res_.resize(sizeof(spk_dresult_t));
    std::vector<void *> hp(n_spans() ? n_spans() : 1, nullptr);
    std::vector<uint64_t> caps(n_spans() ? n_spans() : 1, 0);
    for (uint32_t k = 0; k < n_spans(); ++k) {
      hp[k] = out.heaps[k].data();
      caps[k] = out.heap_elems[k];
    }
    check(spk_decode_frames(&layout(), d_wire, len, d_begins, d_ends, n, prefix, out.recs.data(),
                            out.n, hp.data(), caps.data(), (spk_dresult_t *)res_.data(), d_errc,
                            ws_.data(), ws_.size(), s_), "spk_decode_frames");
    spk_dresult_t r{};
    copy(&r, res_.data(), sizeof(r), SPK_COPY_D2H, s_);
    sync(s_);
    return r;
  }

  // decode into `out` (capacities from out.n / out.heap_elems); `prefix` =
  // frame bytes before each message (MESSAGES mode only)
  spk_dresult_t decode(batch<R> &out, const void *d_wire, std::size_t len, int mode,
                       const uint64_t *d_offsets = nullptr, std::size_t n_msgs = 0,
                       int32_t *d_errc = nullptr, uint32_t prefix = 0) {
    const uint64_t nrec = mode == SPK_MODE_VECTOR ? out.n : n_msgs;
    ws_.resize(spk_workspace_bytes(&layout(), mode, nrec, len));
    res_.resize(sizeof(spk_dresult_t));
    std::vector<void *> hp(n_spans() ? n_spans() : 1, nullptr);
    std::vector<uint64_t> caps(n_spans() ? n_spans() : 1, 0);
    for (uint32_t k = 0; k < n_spans(); ++k) {
      hp[k] = out.heaps[k].data();
      caps[k] = out.heap_elems[k];
    }
    if (prefix)
      check(spk_decode_framed(&layout(), d_wire, len, d_offsets, n_msgs, prefix, out.recs.data(),
                              out.n, hp.data(), caps.data(), (spk_dresult_t *)res_.data(), d_errc,
                              ws_.data(), ws_.size(), s_), "spk_decode_framed");
    else
      check(spk_decode(&layout(), mode, d_wire, len, d_offsets, n_msgs, out.recs.data(), out.n,
                       hp.data(), caps.data(), (spk_dresult_t *)res_.data(), d_errc, ws_.data(),
                       ws_.size(), s_), "spk_decode");
    spk_dresult_t r{};
    copy(&r, res_.data(), sizeof(r), SPK_COPY_D2H, s_);
    sync(s_);
    return r;
  }

  // after plan(SPK_MODE_VECTOR): the records' bytes only, every container
  // count at `width` bytes (spk_encode_body; struct_pack::write,
  // user_helper.hpp:16-30). Stream-ordered, no sync.
  void encode_body(const batch<R> &b, uint32_t width, void *d_out, std::size_t cap) {
    std::vector<const void *> hp = heap_ptrs(b);
    check(spk_encode_body(&layout(), b.n, b.recs.data(), hp.data(), width, d_out, cap,
                          ws_.data(), ws_.size(), s_), "spk_encode_body");
  }
  // exactly n records from a body at `width` (spk_decode_body; struct_pack::
  // read, user_helper.hpp:31-64); result->consumed = body bytes used
  spk_dresult_t decode_body(batch<R> &out, const void *d_body, std::size_t len, uint32_t width,
                            std::size_t n) {
    ws_.resize(spk_workspace_bytes(&layout(), SPK_MODE_VECTOR, out.n, len));
    res_.resize(sizeof(spk_dresult_t));
    std::vector<void *> hp(n_spans() ? n_spans() : 1, nullptr);
    std::vector<uint64_t> caps(n_spans() ? n_spans() : 1, 0);
    for (uint32_t k = 0; k < n_spans(); ++k) {
      hp[k] = out.heaps[k].data();
      caps[k] = out.heap_elems[k];
    }
    check(spk_decode_body(&layout(), d_body, len, width, n, out.recs.data(), out.n, hp.data(),
                          caps.data(), (spk_dresult_t *)res_.data(), ws_.data(), ws_.size(), s_),
          "spk_decode_body");
    spk_dresult_t r{};
    copy(&r, res_.data(), sizeof(r), SPK_COPY_D2H, s_);
    sync(s_);
    return r;
  }

  // a batch able to hold the decode of a `len`-byte wire buffer into at most
  // max_records records: every heap can hold the whole wire
  batch<R> alloc_for_wire(std::size_t len, std::size_t max_records) {
    batch<R> b;
    b.n = max_records;
    b.recs.resize(max_records * layout().rec_stride);
    const std::vector<uint64_t> caps = detail::heap_caps_for_wire(layout(), len, max_records);
    for (uint32_t k = 0; k < n_spans(); ++k) {
      b.heap_elems.push_back(caps[k]);
      b.heaps.emplace_back(caps[k] * span_elem(k));
    }
    if (const char *z = std::getenv("SPK_GPU_ZERO_ALLOC"); z && z[0] == '1') {  // (diagnostic)
      auto zero = [&](buffer &x, std::size_t nb) {
        std::vector<uint8_t> h(nb, z[1] == 'g' ? 0xAB : 0);
        copy(x.data(), h.data(), nb, SPK_COPY_H2D, s_);
        sync(s_);
      };
      zero(b.recs, max_records * layout().rec_stride);
      for (uint32_t k = 0; k < n_spans(); ++k) zero(b.heaps[k], caps[k] * span_elem(k));
    }
    return b;
  }

  // heaps: SPAN / OPTION / COMPAT values and ARRAY element records, in op
  // order at every level (COPY, VARINT and group heads live in the record)
  static uint32_t n_spans() {
    uint32_t k = 0;
    for (uint32_t i = 0; i < layout().n_ops; ++i) k += has_heap(layout().ops[i]);
    return k;
  }
  static bool has_heap(const spk_op &o) { return detail::op_has_heap(o); }
  // bytes per heap element (an ARRAY's: its element record stride)
  static uint32_t span_elem(uint32_t k) {
    for (uint32_t i = 0, s = 0; i < layout().n_ops; ++i)
      if (has_heap(layout().ops[i]) && s++ == k) return layout().ops[i].size;
    return 1;
  }
  // fewest wire bytes a record can take: a bound on the records in a buffer
  static std::size_t min_record_wire() { return detail::min_record_wire_bytes(layout()); }
  void *stream() const { return s_; }

 private:
  std::vector<const void *> heap_ptrs(const batch<R> &b) const {
    std::vector<const void *> hp(n_spans() ? n_spans() : 1, nullptr);
    for (uint32_t k = 0; k < n_spans(); ++k) hp[k] = b.heaps[k].data();
    return hp;
  }
  void *s_;
  buffer ws_, plan_, res_;
  std::vector<std::vector<uint8_t>> view_heaps_;
  std::vector<uint8_t> view_recs_;
  // small-call state (encode_small / decode_small)
  buffer arena_;
  pinned pin_;
  std::vector<uint8_t> mrecs_;
  std::vector<std::vector<uint8_t>> mheaps_;
  spk_plan_t last_plan_{};
};

// A connection's request frames in arrival order, function ids interleaved:
// the handler lookup of the reference server (router.hpp:226-240) for the
// whole batch. After route(), list k (function_ids[k]; the last list: ids in
// no handler map) holds its frames' bounds and arrival indices, in arrival
// order, for codec<Args>::decode_frames and encode_framed_echo.
class frame_router {
 public:
  frame_router(std::vector<uint32_t> function_ids, std::size_t capacity, void *stream = nullptr)
      : ids_(std::move(function_ids)), cap_(capacity), s_(stream) {
    const std::size_t lists = ids_.size() + 1;
    for (std::size_t k = 0; k < lists; ++k) {
      beg_.emplace_back((capacity ? capacity : 1) * 8);
      end_.emplace_back((capacity ? capacity : 1) * 8);
      idx_.emplace_back((capacity ? capacity : 1) * 8);
    }
    counts_.resize(lists * 8);
    ws_.resize(spk_route_workspace_bytes(capacity, (uint32_t)ids_.size()));
  }
  // frame i = d_wire[d_offsets[i], d_offsets[i+1]); returns the list sizes
  std::vector<uint64_t> route(const void *d_wire, std::size_t len, const uint64_t *d_offsets,
                              std::size_t n) {
    if (n > cap_) throw spk_error("struct_pack::gpu::frame_router: more frames than capacity");
    std::vector<uint64_t *> b, e, x;
    for (std::size_t k = 0; k <= ids_.size(); ++k) {
      b.push_back((uint64_t *)beg_[k].data());
      e.push_back((uint64_t *)end_[k].data());
      x.push_back((uint64_t *)idx_[k].data());
    }
    check(spk_route_frames(d_wire, len, d_offsets, n, rpc_key_off, ids_.data(),
                           (uint32_t)ids_.size(), b.data(), e.data(), x.data(),
                           (uint64_t *)counts_.data(), ws_.data(), ws_.size(), s_),
          "spk_route_frames");
    std::vector<uint64_t> c(ids_.size() + 1);
    copy(c.data(), counts_.data(), c.size() * 8, SPK_COPY_D2H, s_);
    sync(s_);
    return c;
  }
  const uint64_t *begins(std::size_t k) const { return (const uint64_t *)beg_[k].data(); }
  const uint64_t *ends(std::size_t k) const { return (const uint64_t *)end_[k].data(); }
  const uint64_t *index(std::size_t k) const { return (const uint64_t *)idx_[k].data(); }
  static constexpr uint32_t rpc_key_off = 8;  // req_header.function_id

 private:
  std::vector<uint32_t> ids_;
  std::size_t cap_;
  void *s_;
  std::vector<buffer> beg_, end_, idx_;
  buffer counts_, ws_;
};

// The calling thread's own non-blocking stream for the front end's per-call
// codecs (call_codec: serialize / deserialize of one message take host data
// and sync before they return, so no caller work on other streams is ordered
// against it). On the legacy null stream each copy and launch paid its
// implicit device-wide ordering (small calls ~7 % slower).
struct thread_stream_holder {
  void *s = nullptr;
  thread_stream_holder() { check(spk_stream_create(&s), "spk_stream_create"); }
  ~thread_stream_holder() {
    if (s) (void)spk_stream_destroy(s);
  }
};
inline void *thread_stream() {
  thread_local thread_stream_holder h;
  return h.s;
}

// the thread's codec of R on the null stream (callers may order their own
// null-stream work after its stream-ordered calls)
template <typename R, uint64_t conf>
codec<R, conf> &thread_codec() {
  thread_local codec<R, conf> c;
  return c;
}
// the thread's codec of R for whole calls of the front end (staged_message,
// decode_one_dev): its own stream, synced inside every call
template <typename R, uint64_t conf>
codec<R, conf> &call_codec() {
  thread_local codec<R, conf> c(thread_stream());
  return c;
}

}  // namespace device

namespace detail {

template <typename T>
concept byte_view = requires(const T &v) {
  v.data();
  v.size();
} && sizeof(*std::declval<const T &>().data()) == 1;

template <typename T>
concept resizable_buffer = requires(T &b, std::size_t n) {
  b.resize(n);
  b.data();
  b.size();
} && sizeof(*std::declval<T &>().data()) == 1;

template <typename T>
concept byte_writer = requires(T &w, const char *p, std::size_t n) { w.write(p, n); };

// One planned message of `t` staged on the device (plan + encode); the bytes
// stay in `out` until copied to the caller.
// the descriptor of a payload-free message type (std::monostate): only its
// header shape (fmt_one) is used, by spk_message_header / _parse_
template <typename M, uint64_t conf>
const spk_layout &empty_message_layout() {
  static const spk_layout L = [] {
    spk_layout l = make_spk_layout<boxed<M>, conf>();
    device::check(spk_layout_check(&l), "spk_layout_check");
    return l;
  }();
  return L;
}

template <uint64_t conf, typename T>
struct staged_message {
  using tr = msg_traits<remove_cvref_t<T>>;
  using R = typename tr::rec;
  device::buffer out, offs;
  spk_plan_t plan{};
  std::size_t len = 0;
  uint8_t hdr[4 + 1 + SPK_MAX_LITERAL + 1] = {};  // tr::empty: the whole message

  std::vector<char> host;  // the message, when the small-call path made it
  bool on_host = false;

  explicit staged_message(const T &t) {
    if constexpr (tr::empty) {
      const int n = spk_message_header(&empty_message_layout<remove_cvref_t<T>, conf>(), 1, hdr,
                                       sizeof hdr);
      if (n < 0) device::check(n, "spk_message_header");
      len = static_cast<std::size_t>(n);
    } else {
      // small messages: one H2D, plan + encode in the codec's arena, one D2H
      auto &c = device::call_codec<R, conf>();
      auto sink = [&](const char *p, std::size_t k) {
        host.assign(p, p + k);
        len = k;
        plan = c.last_plan();
      };
      if constexpr (tr::vector)
        on_host = c.encode_small(t.data(), t.size(), SPK_MODE_VECTOR, sink);
      else
        on_host = c.encode_small(&t, 1, SPK_MODE_MESSAGES, sink);
      if (!on_host) stage_on_device(t);
    }
  }
  void stage_on_device(const T &t) {
    if constexpr (tr::empty) {
    } else if constexpr (tr::vector) {
      auto &c = device::call_codec<R, conf>();
      auto b = c.upload(t.data(), t.size());
      plan = c.plan(b, SPK_MODE_VECTOR);
      len = plan.total_bytes;
      out.resize(len);
      c.encode(b, SPK_MODE_VECTOR, out.data(), out.size());
    } else {
      auto &c = device::call_codec<R, conf>();
      auto b = c.upload(&t, 1);  // (boxed<M>: t is its one member)
      plan = c.plan(b, SPK_MODE_MESSAGES);
      len = plan.total_bytes;
      out.resize(len);
      offs.resize(2 * sizeof(uint64_t));
      c.encode(b, SPK_MODE_MESSAGES, out.data(), out.size(), (uint64_t *)offs.data());
    }
  }
  void copy_to(void *dst) {
    if constexpr (tr::empty) {
      std::memcpy(dst, hdr, len);
    } else if (on_host) {
      if (len) std::memcpy(dst, host.data(), len);
    } else {
      auto &c = device::call_codec<R, conf>();
      device::copy(dst, out.data(), len, SPK_COPY_D2H, c.stream());
      device::sync(c.stream());
    }
  }
};

template <typename T>
constexpr void check_message_type() {
  static_assert(is_gpu_message_v<T>,
                "struct_pack::gpu handles one std::vector<R> / std::span<R> of records or one "
                "record R whose members are fundamentals, enums, std::array, std::string, "
                "sequence / set / map containers, optionals, variants, compatibles, varints "
                "and nested records; use the reference's CPU struct_pack for anything else");
}

template <uint64_t conf, typename T>
err_code decode_one_dev(T &t, const char *data, std::size_t size, std::size_t &consume_len);

// decode of one message into t: VECTOR for std::vector<R>, one MESSAGES
// message for a record. errc / consume_len as the reference
// (struct_pack.hpp:326-357); `t` is left unchanged on an error.
template <uint64_t conf, typename T>
err_code decode_one(T &t, const char *data, std::size_t size, std::size_t &consume_len) {
  check_message_type<T>();
  using tr = msg_traits<T>;
  using R = typename tr::rec;
  static_assert(!std::is_same_v<T, std::span<R>>, "deserialize into std::vector<R>");
  consume_len = 0;
  if constexpr (tr::empty) {  // the header is the whole message
    uint32_t w = 0, hl = 0;
    const int32_t e = spk_parse_message_header(&empty_message_layout<T, conf>(), data, size, &w,
                                               &hl);
    if (e < 0) device::check(e, "spk_parse_message_header");
    if (e) return static_cast<errc>(e);
    consume_len = hl;
    return {};
  } else {
    return decode_one_dev<conf>(t, data, size, consume_len);
  }
}

template <uint64_t conf, typename T>
err_code decode_one_dev(T &t, const char *data, std::size_t size, std::size_t &consume_len) {
  using tr = msg_traits<T>;
  using R = typename tr::rec;
  auto &c = device::call_codec<R, conf>();
  std::size_t cap = tr::vector ? size / c.min_record_wire() + 1 : 1;
  // small messages: one H2D, the decode in the codec's arena, one D2H
  for (spk_dresult_t r;;) {
    if (!c.decode_small(data, size, tr::vector ? SPK_MODE_VECTOR : SPK_MODE_MESSAGES, cap, r))
      break;  // not small: the batch path below
    if (r.errc == SPK_ERRC_CAPACITY) {
      cap = cap * 2 + 1;
      continue;
    }
    if (r.errc) return static_cast<errc>(r.errc);
    if constexpr (tr::vector) {
      T out(r.count);
      c.unmarshal(r.count, out.data());
      t = std::move(out);
    } else {
      c.unmarshal(1, &t);  // (boxed<M>: t is its one member)
    }
    if constexpr (has_views<T>()) {  // views alias `data`, as the reference's do
      mem_cursor mc{data, size};
      header_info h;
      (void)walk_header(mc, tr::vector ? c.layout().fmt_vector : c.layout().fmt_one, h);
      rebase_views(t, mc, h.w);
    }
    consume_len = r.consumed;
    return {};
  }
  device::buffer wire(size + 16);
  device::copy(wire.data(), data, size, SPK_COPY_H2D, c.stream());
  for (;;) {
    // the capacities bound every decodable message (min_record_wire is a
    // lower bound on a record's wire bytes, fast-varint groups counted as
    // their bitset; no heap exceeds the wire); the loop only guards that
    // invariant and never surfaces a non-reference errc
    auto b = c.alloc_for_wire(size, cap);
    spk_dresult_t r;
    if constexpr (tr::vector) {
      r = c.decode(b, wire.data(), size, SPK_MODE_VECTOR);
    } else {
      device::buffer offs(2 * sizeof(uint64_t)), ec(sizeof(int32_t));
      const uint64_t o[2] = {0, size};
      device::copy(offs.data(), o, sizeof o, SPK_COPY_H2D, c.stream());
      r = c.decode(b, wire.data(), size, SPK_MODE_MESSAGES, (const uint64_t *)offs.data(), 1,
                   (int32_t *)ec.data());
      int32_t e = 0;
      device::copy(&e, ec.data(), sizeof e, SPK_COPY_D2H, c.stream());
      device::sync(c.stream());
      r.errc = e;
    }
    if (r.errc == SPK_ERRC_CAPACITY) {
      cap = cap * 2 + 1;
      continue;
    }
    if (r.errc) return static_cast<errc>(r.errc);
    for (uint32_t k = 0; k < c.n_spans(); ++k) b.heap_elems[k] = r.heap_used[k];
    if constexpr (tr::vector) {
      T out(r.count);
      c.download(b, r.count, out.data());
      t = std::move(out);
    } else {
      c.download(b, 1, &t);  // (boxed<M>: t is its one member)
    }
    if constexpr (has_views<T>()) {  // views alias `data`, as the reference's do
      mem_cursor mc{data, size};
      header_info h;
      (void)walk_header(mc, tr::vector ? c.layout().fmt_vector : c.layout().fmt_one, h);
      rebase_views(t, mc, h.w);
    }
    consume_len = r.consumed;
    return {};
  }
}

}  // namespace detail

// ===========================================================================
// Reference-named entry points (host data in, host bytes out)
// ===========================================================================

namespace detail {
template <uint64_t conf, typename T>
serialize_buffer_size needed_size_dev(const T &t);
}  // namespace detail

// get_needed_size (struct_pack.hpp:131-135)
template <uint64_t conf = sp_config::DEFAULT, typename T>
serialize_buffer_size get_needed_size(const T &t) {
  detail::check_message_type<T>();
  using tr = detail::msg_traits<detail::remove_cvref_t<T>>;
  serialize_buffer_size r;
  if constexpr (tr::empty) {  // header only, no metainfo byte (no container)
    detail::staged_message<conf, T> m(t);
    r.len_ = m.len;
    r.metainfo_ = m.len > 4 ? m.hdr[4] : 0;
    return r;
  } else {
    return detail::needed_size_dev<conf>(t);
  }
}

namespace detail {
template <uint64_t conf, typename T>
serialize_buffer_size needed_size_dev(const T &t) {
  using tr = detail::msg_traits<detail::remove_cvref_t<T>>;
  using R = typename tr::rec;
  serialize_buffer_size r;
  auto &c = device::thread_codec<R, conf>();
  spk_plan_t p;
  if constexpr (tr::vector) {
    auto b = c.upload(t.data(), t.size());
    p = c.plan(b, SPK_MODE_VECTOR);
  } else {
    auto b = c.upload(&t, 1);
    p = c.plan(b, SPK_MODE_MESSAGES);
  }
  r.len_ = p.total_bytes;
  if constexpr (tr::vector) {
    r.metainfo_ = static_cast<unsigned char>(p.has_meta ? p.metainfo : 0);
  } else {  // one message: its header shape at the record's own width
    const spk_msgfmt &f = c.layout().fmt_one;
    const bool head = f.flags & SPK_MF_HASH_HEAD, lit = head && (f.flags & SPK_MF_TYPE_LITERAL);
    const bool cont = f.flags & SPK_MF_HAS_CONTAINER;
    const uint32_t w = cont ? p.width : 1;
    const bool meta = lit || (!head && cont) || w > 1;
    const unsigned char wb = w == 1 ? 0 : w == 2 ? 0x08 : w == 4 ? 0x10 : 0x18;
    r.metainfo_ = meta ? static_cast<unsigned char>(wb | (lit ? 0x04 : 0)) : 0;
  }
  return r;
}
}  // namespace detail

// serialize_to(Buffer& | Writer&, t): appends to a byte buffer or writes to
// a writer (struct_pack.hpp:137-159)
template <uint64_t conf = sp_config::DEFAULT, typename Writer, typename T>
void serialize_to(Writer &writer, const T &t) {
  detail::check_message_type<T>();
  detail::staged_message<conf, T> m(t);
  if constexpr (detail::resizable_buffer<Writer>) {
    const std::size_t old = writer.size();
    writer.resize(old + m.len);
    m.copy_to(writer.data() + old);
  } else {
    static_assert(detail::byte_writer<Writer>,
                  "serialize_to needs a contiguous byte buffer or a writer with "
                  "write(const char*, size_t)");
    std::vector<char> tmp(m.len);
    m.copy_to(tmp.data());
    writer.write(tmp.data(), tmp.size());
  }
}

// serialize_to(char*, serialize_buffer_size, t): the caller sized the buffer
// with get_needed_size (struct_pack.hpp:161-167)
template <uint64_t conf = sp_config::DEFAULT, typename T>
void serialize_to(char *buffer, serialize_buffer_size info, const T &t) {
  detail::check_message_type<T>();
  detail::staged_message<conf, T> m(t);
  if (m.len != info.size())
    throw spk_error("struct_pack::gpu::serialize_to: serialize_buffer_size does not match t");
  m.copy_to(buffer);
}
#if SPK_GPU_WITH_REFERENCE
// ... with the size object of the reference's own get_needed_size
template <uint64_t conf = sp_config::DEFAULT, typename T>
void serialize_to(char *buffer, struct_pack::serialize_buffer_size info, const T &t) {
  serialize_buffer_size s;
  s.len_ = info.size();
  s.metainfo_ = info.metainfo();
  serialize_to<conf>(buffer, s, t);
}
#endif

// serialize_to_with_offset(buffer, offset, t): `offset` bytes reserved
// before the message, e.g. coro_rpc's req_header (struct_pack.hpp:169-189)
template <uint64_t conf = sp_config::DEFAULT, typename Buffer, typename T>
void serialize_to_with_offset(Buffer &buffer, std::size_t offset, const T &t) {
  detail::check_message_type<T>();
  static_assert(detail::resizable_buffer<Buffer>, "a contiguous byte buffer");
  detail::staged_message<conf, T> m(t);
  const std::size_t old = buffer.size();
  buffer.resize(old + offset + m.len);
  m.copy_to(buffer.data() + old + offset);
}

// serialize<Buffer>(t) and serialize<conf, Buffer>(t) (struct_pack.hpp:191-262)
template <typename Buffer = std::vector<char>, typename T>
  requires detail::resizable_buffer<Buffer>
[[nodiscard]] Buffer serialize(const T &t) {
  Buffer b;
  serialize_to<sp_config::DEFAULT>(b, t);
  return b;
}
template <uint64_t conf, typename Buffer = std::vector<char>, typename T>
  requires detail::resizable_buffer<Buffer>
[[nodiscard]] Buffer serialize(const T &t) {
  Buffer b;
  serialize_to<conf>(b, t);
  return b;
}
template <typename Buffer = std::vector<char>, typename T>
  requires detail::resizable_buffer<Buffer>
[[nodiscard]] Buffer serialize_with_offset(std::size_t offset, const T &t) {
  Buffer b;
  serialize_to_with_offset<sp_config::DEFAULT>(b, offset, t);
  return b;
}
template <uint64_t conf, typename Buffer = std::vector<char>, typename T>
  requires detail::resizable_buffer<Buffer>
[[nodiscard]] Buffer serialize_with_offset(std::size_t offset, const T &t) {
  Buffer b;
  serialize_to_with_offset<conf>(b, offset, t);
  return b;
}

// deserialize_to (struct_pack.hpp:266-357): errc as the reference; with
// consume_len the message end (or the compatible-data length if larger), 0 on
// an error
template <uint64_t conf = sp_config::DEFAULT, typename T>
[[nodiscard]] err_code deserialize_to(T &t, const char *data, std::size_t size,
                                      std::size_t &consume_len) {
  return detail::decode_one<conf>(t, data, size, consume_len);
}
template <uint64_t conf = sp_config::DEFAULT, typename T>
[[nodiscard]] err_code deserialize_to(T &t, const char *data, std::size_t size) {
  std::size_t consumed;
  return detail::decode_one<conf>(t, data, size, consumed);
}
template <uint64_t conf = sp_config::DEFAULT, typename T, detail::byte_view View>
[[nodiscard]] err_code deserialize_to(T &t, const View &v) {
  std::size_t consumed;
  return detail::decode_one<conf>(t, reinterpret_cast<const char *>(v.data()), v.size(),
                                  consumed);
}
template <uint64_t conf = sp_config::DEFAULT, typename T, detail::byte_view View>
[[nodiscard]] err_code deserialize_to(T &t, const View &v, std::size_t &consume_len) {
  return detail::decode_one<conf>(t, reinterpret_cast<const char *>(v.data()), v.size(),
                                  consume_len);
}

// deserialize_to_with_offset: decode at data + offset, advance offset by the
// bytes consumed (struct_pack.hpp:359-385)
template <uint64_t conf = sp_config::DEFAULT, typename T>
[[nodiscard]] err_code deserialize_to_with_offset(T &t, const char *data, std::size_t size,
                                                  std::size_t &offset) {
  std::size_t sz;
  auto e = detail::decode_one<conf>(t, data + offset, size - offset, sz);
  offset += sz;
  return e;
}
template <uint64_t conf = sp_config::DEFAULT, typename T, detail::byte_view View>
[[nodiscard]] err_code deserialize_to_with_offset(T &t, const View &v, std::size_t &offset) {
  return deserialize_to_with_offset<conf>(t, reinterpret_cast<const char *>(v.data()), v.size(),
                                          offset);
}

// deserialize<T>(...) and deserialize<conf, T>(...) -> expected<T, err_code>
// (struct_pack.hpp:387-533; one message type)
template <typename T, detail::byte_view View>
[[nodiscard]] expected<T> deserialize(const View &v) {
  T t{};
  if (auto e = deserialize_to(t, v)) return make_unexpected<T>(e);
  return t;
}
template <typename T>
[[nodiscard]] expected<T> deserialize(const char *data, std::size_t size) {
  T t{};
  if (auto e = deserialize_to(t, data, size)) return make_unexpected<T>(e);
  return t;
}
template <typename T, detail::byte_view View>
[[nodiscard]] expected<T> deserialize(const View &v, std::size_t &consume_len) {
  T t{};
  if (auto e = deserialize_to(t, v, consume_len)) return make_unexpected<T>(e);
  return t;
}
template <typename T>
[[nodiscard]] expected<T> deserialize(const char *data, std::size_t size,
                                      std::size_t &consume_len) {
  T t{};
  if (auto e = deserialize_to(t, data, size, consume_len)) return make_unexpected<T>(e);
  return t;
}
template <uint64_t conf, typename T, detail::byte_view View>
[[nodiscard]] expected<T> deserialize(const View &v) {
  T t{};
  if (auto e = deserialize_to<conf>(t, v)) return make_unexpected<T>(e);
  return t;
}
template <uint64_t conf, typename T>
[[nodiscard]] expected<T> deserialize(const char *data, std::size_t size) {
  T t{};
  if (auto e = deserialize_to<conf>(t, data, size)) return make_unexpected<T>(e);
  return t;
}
template <uint64_t conf, typename T, detail::byte_view View>
[[nodiscard]] expected<T> deserialize(const View &v, std::size_t &consume_len) {
  T t{};
  if (auto e = deserialize_to<conf>(t, v, consume_len)) return make_unexpected<T>(e);
  return t;
}

// ---- user helpers: struct_pack::write / read / get_write_size --------------
// (user_helper.hpp:16-85) The payload bytes of t (or of t[0..len)) without
// header, container counts at size_width bytes: the body of a VECTOR message
// at that width, so the device codec writes and reads it
// (spk_encode_body / spk_decode_body). Used by sp_serialize_to /
// sp_deserialize_to of user-defined types (test_user_defined_type.cpp:55-120).
namespace detail {
template <typename T>
using helper_rec_t = std::conditional_t<record_supported<T>(), T, boxed<T>>;

template <std::size_t W, uint64_t conf, typename T>
struct staged_body {
  using R = helper_rec_t<T>;
  device::buffer out;
  std::size_t len = 0;
  staged_body(const T *t, std::size_t n) {
    static_assert(W == 1 || W == 2 || W == 4 || W == 8, "size_width must be 1, 2, 4 or 8");
    auto &c = device::thread_codec<R, conf>();
    auto b = c.upload(t, n);  // (boxed<T>: each t[i] is its one member)
    const spk_plan_t p = c.plan(b, SPK_MODE_VECTOR);
    if (c.layout().flags & SPK_LAYOUT_TRIVIAL) {
      len = n * c.layout().rec_stride;
    } else {
      const uint64_t fields = p.width ? (p.total_bytes - p.header_bytes - p.var_bytes) / p.width : 0;
      len = p.var_bytes + fields * W;
    }
    out.resize(len);
    c.encode_body(b, W, out.data(), len);
  }
  void copy_to(void *dst) {
    auto &c = device::thread_codec<R, conf>();
    device::copy(dst, out.data(), len, SPK_COPY_D2H, c.stream());
    device::sync(c.stream());
  }
};

// read n records of T from a body in host memory; consumed = body bytes used
template <std::size_t W, uint64_t conf, typename T>
err_code decode_body_host(T *t, std::size_t n, const char *data, std::size_t size,
                          std::size_t &consumed) {
  using R = helper_rec_t<T>;
  auto &c = device::thread_codec<R, conf>();
  consumed = 0;
  device::buffer wire(size + 16);
  device::copy(wire.data(), data, size, SPK_COPY_H2D, c.stream());
  auto b = c.alloc_for_wire(size, n);
  spk_dresult_t r = c.decode_body(b, wire.data(), size, W, n);
  if (r.errc == SPK_ERRC_CAPACITY)  // heaps hold the whole wire: unreachable
    throw std::logic_error("struct_pack::gpu: decode capacity invariant broken");
  if (r.errc) return static_cast<errc>(r.errc);
  for (uint32_t k = 0; k < c.n_spans(); ++k) b.heap_elems[k] = r.heap_used[k];
  c.download(b, n, t);  // (boxed<T>: each t[i] is its one member)
  if constexpr (has_views<T>()) {  // views alias `data`
    mem_cursor mc{data, size};
    for (std::size_t i = 0; i < n; ++i) rebase_views(t[i], mc, static_cast<uint32_t>(W));
  }
  consumed = r.consumed;
  return {};
}
}  // namespace detail

template <std::size_t size_width = sizeof(uint64_t), typename Writer, typename T>
void write(Writer &writer, const T *t, std::size_t len) {
  static_assert(is_gpu_message_v<T>, "struct_pack::gpu::write: type outside the record model");
  detail::staged_body<size_width, sp_config::DEFAULT, T> m(t, len);
  std::vector<char> tmp(m.len);
  if (m.len) m.copy_to(tmp.data());
  writer.write(tmp.data(), tmp.size());
}
template <std::size_t size_width = sizeof(uint64_t), typename Writer, typename T>
void write(Writer &writer, const T &t) {
  write<size_width>(writer, &t, 1);
}
template <std::size_t size_width = sizeof(uint64_t), typename T>
std::size_t get_write_size(const T *t, std::size_t len) {
  return detail::staged_body<size_width, sp_config::DEFAULT, T>(t, len).len;
}
template <std::size_t size_width = sizeof(uint64_t), typename T>
std::size_t get_write_size(const T &t) {
  return get_write_size<size_width>(&t, 1);
}
// read from a byte view (advancing `pos`) or a reader (below); ifSkip:
// consume without keeping the values
template <std::size_t size_width = sizeof(uint64_t), bool ifSkip = false, typename T>
err_code read_from(const char *data, std::size_t size, std::size_t &pos, T *t, std::size_t len) {
  std::size_t used = 0;
  err_code e;
  if constexpr (ifSkip) {
    std::vector<T> sink(len);
    e = detail::decode_body_host<size_width, sp_config::DEFAULT>(sink.data(), len, data + pos,
                                                                  size - pos, used);
  } else {
    e = detail::decode_body_host<size_width, sp_config::DEFAULT>(t, len, data + pos, size - pos,
                                                                  used);
  }
  pos += used;
  return e;
}
// ---- get_field<T, I> (struct_pack.hpp:565-658) -------------------------------
// The reference reads members 0..I of a T message and stops: the members
// before I in skip mode, each result overwriting the previous one (the
// &&-fold of for_each only stops at member I, unpacker.hpp:1554-1592), then
// member I into `dst`; a T with compatible members also runs the version
// passes over members 0..I (deserialize_compatible_fields, unpacker.hpp:
// 367-444). So on a buffer cut after member I the field still comes back.
// Here the header is parsed on the host (spk_parse_message_header), members
// 0..I-1 are skipped by the host walker (walk.hpp) and member I is decoded on
// the device as a one-record body at the message's width (spk_decode_body).
// The members of a trivially serializable T are walked one by one too, with
// no padding, like the reference's get_field_impl.
template <typename T, std::size_t I>
using field_t = std::tuple_element_t<I, detail::members_tuple_t<T>>;

namespace detail {
template <uint64_t conf, typename F>
err_code decode_field(F &dst, const char *data, std::size_t size, uint32_t w, std::size_t &used) {
  switch (w) {
    case 1: return decode_body_host<1, conf>(&dst, 1, data, size, used);
    case 2: return decode_body_host<2, conf>(&dst, 1, data, size, used);
    case 4: return decode_body_host<4, conf>(&dst, 1, data, size, used);
    default: return decode_body_host<8, conf>(&dst, 1, data, size, used);
  }
}

// get_field's reads over cursor `c`, after the header: main pass over members
// 0..I (member I by main(c)), then, for a T with compatible members, the
// version passes over members 0..I (member I by in_pass(c, past) when it is a
// compatible member of that version). Returns the reference's errc.
template <typename T, std::size_t I, typename Cur, typename Main, typename InPass>
errc get_field_walk(Cur &c, uint32_t w, uint64_t data_len, Main &&main, InPass &&in_pass) {
  using M = members_tuple_t<T>;
  static_assert(I < std::tuple_size_v<M>, "get_field: member index out of range");
  using F = std::tuple_element_t<I, M>;
  errc code{};
  [&]<std::size_t... J>(std::index_sequence<J...>) {
    ((code = walk_one<std::tuple_element_t<J, M>>(c, w)), ...);
  }(std::make_index_sequence<I>{});
  if constexpr (is_compat_v<F>)
    code = {};  // a compatible member is read in its version pass
  else
    code = main(c);
  if constexpr (record_has_compat<T>()) {
    if (code != errc{}) return code;
    bool past = false;
    for (uint64_t v : compat_versions<T>()) {
      errc pc{};
      [&]<std::size_t... J>(std::index_sequence<J...>) {
        auto one = [&](auto jc, auto tagv) {
          using G = typename decltype(tagv)::type;
          constexpr std::size_t j = decltype(jc)::value;
          pc = {};
          if constexpr (is_compat_v<G>) {
            if (compat_traits<G>::version == v) {
              if constexpr (j < I)
                pc = walk_compat_member<G>(c, w, data_len, past);
              else
                pc = in_pass(c, past);
            }
          }
        };
        (one(std::integral_constant<std::size_t, J>{},
             std::type_identity<std::tuple_element_t<J, M>>{}),
         ...);
      }(std::make_index_sequence<I + 1>{});
      code = pc;
      if (code != errc{}) break;
    }
    if (past) code = {};  // the buffer ended before a version: not an error
  }
  return code;
}

template <typename T, std::size_t I, uint64_t conf>
err_code get_field_mem(field_t<T, I> &dst, const char *data, std::size_t size) {
  static_assert(is_record_v<T>, "get_field reads a member of a record message");
  using F = field_t<T, I>;
  const spk_layout &L = device::codec<typename msg_traits<T>::rec, conf>::layout();
  uint32_t w = 0, hl = 0;
  const int32_t he = spk_parse_message_header(&L, data, size, &w, &hl);
  if (he < 0) device::check(he, "spk_parse_message_header");
  if (he) return static_cast<errc>(he);
  mem_cursor c{data, size};
  header_info h;
  (void)walk_header(c, L.fmt_one, h);  // the header parsed above: positions c, data length
  auto main = [&](mem_cursor &cc) -> errc {
    if constexpr (!is_compat_v<F>) {
      std::size_t used = 0;
      const err_code e =
          decode_field<sp_config::DEFAULT>(dst, cc.d + cc.pos, cc.n - cc.pos, w, used);
      cc.pos += used;
      return e;
    } else {
      return (void)cc, errc{};
    }
  };
  auto in_pass = [&](mem_cursor &cc, bool &past) -> errc {
    if constexpr (is_compat_v<F>) {
      if (cc.tell() >= h.data_len) {
        past = true;
        return errc::no_buffer_space;
      }
      // [has][U] decoded as an optional<U>: the value's errc is dropped like
      // the reference's (unpacker.hpp:1354-1376)
      std::optional<typename compat_traits<F>::value_type> o;
      std::size_t used = 0;
      const err_code e = decode_field<sp_config::DEFAULT>(o, cc.d + cc.pos, cc.n - cc.pos, w, used);
      if (e) return e;
      cc.pos += used;
      if (o) dst = F{std::move(*o)};
      return {};
    } else {
      (void)cc, (void)past;
      return {};
    }
  };
  return get_field_walk<T, I>(c, w, h.data_len, main, in_pass);
}
}  // namespace detail

template <typename T, std::size_t I, uint64_t conf = sp_config::DEFAULT, typename Field>
[[nodiscard]] err_code get_field_to(Field &dst, const char *data, std::size_t size) {
  static_assert(std::is_same_v<Field, field_t<T, I>>,
                "The dst's type is not correct. It should be as same as the T's Ith field's type");
  return detail::get_field_mem<T, I, conf>(dst, data, size);
}
template <typename T, std::size_t I, uint64_t conf = sp_config::DEFAULT, typename Field,
          detail::byte_view View>
[[nodiscard]] err_code get_field_to(Field &dst, const View &v) {
  return gpu::get_field_to<T, I, conf>(dst, reinterpret_cast<const char *>(v.data()), v.size());
}
template <typename T, std::size_t I, uint64_t conf = sp_config::DEFAULT>
[[nodiscard]] expected<field_t<T, I>> get_field(const char *data, std::size_t size) {
  field_t<T, I> f{};
  if (auto e = gpu::get_field_to<T, I, conf>(f, data, size)) return make_unexpected<field_t<T, I>>(e);
  return expected<field_t<T, I>>(std::move(f));
}
template <typename T, std::size_t I, uint64_t conf = sp_config::DEFAULT, detail::byte_view View>
[[nodiscard]] expected<field_t<T, I>> get_field(const View &v) {
  return gpu::get_field<T, I, conf>(reinterpret_cast<const char *>(v.data()), v.size());
}

// ---- readers (struct_pack.hpp:289-323, 415-533, 595-612, 660-676) -----------
// Any reader_t of the reference (read / ignore / tellg, reflection.hpp:
// 110-114): std::istream, the reference's detail::memory_reader, a socket-like
// reader that cannot seek. The host walker (walk.hpp) reads exactly the
// message's bytes through read() -- the reads the reference's decoder would
// make, in the same order -- and the device decodes them. On success the
// reader is left right after the message (after the compatible-data length,
// struct_pack.hpp:302-312), as the reference leaves it. After a short read the
// walker takes whatever the reader still delivers, so the decode sees what
// the reference's reads could have seen and returns its errc; the reader is
// then left at its end (the reference leaves it where its last read stopped).
namespace detail {
template <typename R>
concept reader_t = requires(R &r, char *p, std::size_t n) {
  r.read(p, n);
  r.ignore(n);
  r.tellg();
};

// one message of type T (one std::vector<R>, one record, a boxed message or
// a header-only one) out of a reader
template <uint64_t conf, typename T, typename Reader>
std::vector<char> pull_message(Reader &rd) {
  using tr = msg_traits<T>;
  std::vector<char> buf;
  pull_cursor<Reader> c{rd, buf};
  header_info h;
  errc e{};
  if constexpr (tr::empty) {
    e = walk_header(c, empty_message_layout<T, conf>().fmt_one, h);
  } else {
    const spk_layout &L = device::codec<typename tr::rec, conf>::layout();
    e = walk_header(c, tr::vector ? L.fmt_vector : L.fmt_one, h);
    if constexpr (tr::vector && record_has_compat<typename tr::rec>()) {
      // a vector of records with compatible members: the main pass over its
      // n records, then the version passes over them
      using R = typename tr::rec;
      uint64_t n = 0;
      if (e == errc{}) e = walk_count(c, h.w, n) ? errc{} : errc::no_buffer_space;
      for (uint64_t i = 0; i < n && e == errc{}; ++i) e = walk_one<R>(c, h.w);
      if (e == errc{}) {
        bool past = false;
        (void)walk_versions_vec<R>(c, h.w, n, h.data_len, past);
      }
    } else {
      if (e == errc{}) e = walk_one<T>(c, h.w);
      if constexpr (record_has_compat<T>()) {
        if (e == errc{}) {
          bool past = false;
          (void)walk_versions<T>(c, h.w, h.data_len, past);
        }
      }
    }
    // a message with compatible members ends at its data length at the
    // earliest: the reader skips what a newer writer added
    // (struct_pack.hpp:302-312)
    if (e == errc{} && !c.dry && c.tell() < h.data_len) (void)c.ignore(h.data_len - c.tell());
  }
  if (c.dry) drain(rd, buf);
  return buf;
}
}  // namespace detail

template <uint64_t conf = sp_config::DEFAULT, typename T, typename Reader>
  requires detail::reader_t<Reader>
[[nodiscard]] err_code deserialize_to(T &t, Reader &reader) {
  detail::check_message_type<T>();
  static_assert(!detail::has_views<T>(),
                "string_view / span / trivial_view members alias the buffer they are decoded "
                "from: decode them from a buffer, not a reader");
  const std::vector<char> buf = detail::pull_message<conf, T>(reader);
  std::size_t consumed;
  return detail::decode_one<conf>(t, buf.data(), buf.size(), consumed);
}
template <typename T, typename Reader>
  requires detail::reader_t<Reader>
[[nodiscard]] expected<T> deserialize(Reader &reader) {
  T t{};
  if (auto e = deserialize_to(t, reader)) return make_unexpected<T>(e);
  return t;
}
template <uint64_t conf, typename T, typename Reader>
  requires detail::reader_t<Reader>
[[nodiscard]] expected<T> deserialize(Reader &reader) {
  T t{};
  if (auto e = deserialize_to<conf>(t, reader)) return make_unexpected<T>(e);
  return t;
}

// get_field from a reader: header and members 0..I (and their version
// passes) pulled through the walker, then get_field over those bytes
template <typename T, std::size_t I, uint64_t conf = sp_config::DEFAULT, typename Field,
          typename Reader>
  requires detail::reader_t<Reader>
[[nodiscard]] err_code get_field_to(Field &dst, Reader &reader) {
  static_assert(std::is_same_v<Field, field_t<T, I>>,
                "The dst's type is not correct. It should be as same as the T's Ith field's type");
  static_assert(!detail::has_views<Field>(),
                "a view member aliases the buffer it is decoded from: get it from a buffer");
  using namespace detail;
  const spk_layout &L = device::codec<typename msg_traits<T>::rec, conf>::layout();
  std::vector<char> buf;
  pull_cursor<Reader> c{reader, buf};
  header_info h;
  if (walk_header(c, L.fmt_one, h) == errc{}) {
    using F = field_t<T, I>;
    (void)get_field_walk<T, I>(
        c, h.w, h.data_len, [&](pull_cursor<Reader> &cc) { return walk_one<F>(cc, h.w); },
        [&](pull_cursor<Reader> &cc, bool &past) -> errc {
          if constexpr (is_compat_v<F>)
            return walk_compat_member<F>(cc, h.w, h.data_len, past);
          else
            return (void)cc, (void)past, errc{};
        });
  }
  if (c.dry) drain(reader, buf);
  return get_field_mem<T, I, conf>(dst, buf.data(), buf.size());
}
template <typename T, std::size_t I, uint64_t conf = sp_config::DEFAULT, typename Reader>
  requires detail::reader_t<Reader>
[[nodiscard]] expected<field_t<T, I>> get_field(Reader &reader) {
  field_t<T, I> f{};
  if (auto e = gpu::get_field_to<T, I, conf>(f, reader)) return make_unexpected<field_t<T, I>>(e);
  return expected<field_t<T, I>>(std::move(f));
}

// struct_pack::read over a reader (user_helper.hpp:31-64): len records of T
// at size_width, pulled by the walker, decoded as a body on the device
template <std::size_t size_width = sizeof(uint64_t), bool ifSkip = false, typename Reader,
          typename T>
  requires detail::reader_t<Reader>
err_code read(Reader &reader, T *t, std::size_t len) {
  using namespace detail;
  static_assert(!has_views<T>(), "views alias their buffer: read them from a buffer");
  std::vector<char> buf;
  pull_cursor<Reader> c{reader, buf};
  if constexpr (is_trivially_serializable<T>()) {
    (void)c.ignore(sizeof(T) * len);
  } else {
    for (std::size_t i = 0; i < len; ++i)
      if (walk_one<T>(c, size_width) != errc{}) break;
  }
  if (c.dry) drain(reader, buf);
  std::size_t pos = 0;
  return read_from<size_width, ifSkip>(buf.data(), buf.size(), pos, t, len);
}
template <std::size_t size_width = sizeof(uint64_t), bool ifSkip = false, typename Reader,
          typename T>
  requires detail::reader_t<Reader>
err_code read(Reader &reader, T &t) {
  return read<size_width, ifSkip>(reader, &t, 1);
}

// ---- coro_rpc payload batches: n independent serialize(R) messages --------
template <uint64_t conf = sp_config::DEFAULT, typename R>
std::vector<char> serialize_messages(const std::vector<R> &v, std::vector<uint64_t> &offsets) {
  auto &c = device::thread_codec<R, conf>();
  auto b = c.upload(v.data(), v.size());
  spk_plan_t p = c.plan(b, SPK_MODE_MESSAGES);
  device::buffer out(p.total_bytes), offs((v.size() + 1) * sizeof(uint64_t));
  c.encode(b, SPK_MODE_MESSAGES, out.data(), out.size(), (uint64_t *)offs.data());
  std::vector<char> bytes(p.total_bytes);
  offsets.resize(v.size() + 1);
  device::copy(bytes.data(), out.data(), bytes.size(), SPK_COPY_D2H, c.stream());
  device::copy(offsets.data(), offs.data(), offsets.size() * 8, SPK_COPY_D2H, c.stream());
  device::sync(c.stream());
  return bytes;
}

// decodes message i = data[offsets[i] + prefix, offsets[i+1]) into out[i];
// returns per-message errc
template <uint64_t conf = sp_config::DEFAULT, typename R>
std::vector<err_code> deserialize_messages(std::vector<R> &out, const char *data,
                                           std::size_t size,
                                           const std::vector<uint64_t> &offsets,
                                           uint32_t prefix = 0) {
  auto &c = device::thread_codec<R, conf>();
  const std::size_t n = offsets.empty() ? 0 : offsets.size() - 1;
  device::buffer wire(size + 16), offs(offsets.size() * 8 + 8), ec(n * 4 + 4);
  device::copy(wire.data(), data, size, SPK_COPY_H2D, c.stream());
  device::copy(offs.data(), offsets.data(), offsets.size() * 8, SPK_COPY_H2D, c.stream());
  auto b = c.alloc_for_wire(size, n);
  spk_dresult_t r = c.decode(b, wire.data(), size, SPK_MODE_MESSAGES, (uint64_t *)offs.data(), n,
                             (int32_t *)ec.data(), prefix);
  if (r.errc == SPK_ERRC_CAPACITY)  // heaps hold the whole wire: unreachable
    throw std::logic_error("struct_pack::gpu: decode capacity invariant broken");
  std::vector<int32_t> e(n);
  device::copy(e.data(), ec.data(), n * 4, SPK_COPY_D2H, c.stream());
  for (uint32_t k = 0; k < c.n_spans(); ++k) b.heap_elems[k] = r.heap_used[k];
  device::sync(c.stream());
  out.assign(n, R{});
  c.download(b, n, out.data(), [&](std::size_t i) { return e[i] == 0; });
  std::vector<err_code> res(n);
  for (std::size_t i = 0; i < n; ++i) res[i] = static_cast<errc>(e[i]);
  return res;
}

// ---- coro_rpc framing ------------------------------------------------------
// coro_rpc puts a 20-byte req_header before every request payload and a
// 16-byte resp_header before every response (ref coro_rpc_protocol.hpp:60-79;
// written with DISABLE_ALL_META_INFO = the raw struct bytes, client
// coro_rpc_client.hpp:1285-1335, server coro_rpc_protocol.hpp:191-240).
namespace rpc_frame {
inline constexpr uint8_t magic_number = 21;  // coro_rpc_protocol.hpp:250
inline constexpr uint32_t req_head_len = 20, resp_head_len = 16;

// requests of function `function_id`; message i carries seq_num = seq_base + i
inline spk_frame request(uint32_t function_id, uint32_t seq_base = 0,
                         uint32_t attach_length = 0) {
  spk_frame f{};
  f.prefix_len = req_head_len;
  f.seq_off = 4;
  f.len_off = 12;
  f.seq_base = seq_base;
  f.tmpl[0] = magic_number;  // version, serialize_type, msg_type = 0
  for (int k = 0; k < 4; ++k) {
    f.tmpl[8 + k] = (uint8_t)(function_id >> (8 * k));
    f.tmpl[16 + k] = (uint8_t)(attach_length >> (8 * k));
  }
  return f;
}

// responses echoing seq_num = seq_base + i
inline spk_frame response(uint32_t seq_base = 0, uint8_t err_code = 0) {
  spk_frame f{};
  f.prefix_len = resp_head_len;
  f.seq_off = 4;
  f.len_off = 8;
  f.seq_base = seq_base;
  f.tmpl[0] = magic_number;
  f.tmpl[2] = err_code;
  return f;
}
}  // namespace rpc_frame

// n framed messages [frame prefix][serialize(v[i])]; offsets = frame starts
template <uint64_t conf = sp_config::DEFAULT, typename R>
std::vector<char> serialize_frames(const std::vector<R> &v, const spk_frame &f,
                                   std::vector<uint64_t> &offsets) {
  auto &c = device::thread_codec<R, conf>();
  auto b = c.upload(v.data(), v.size());
  spk_plan_t p = c.plan(b, SPK_MODE_MESSAGES);
  const std::size_t total = p.total_bytes + v.size() * (std::size_t)f.prefix_len;
  device::buffer out(total), offs((v.size() + 1) * sizeof(uint64_t));
  c.encode_framed(b, f, out.data(), out.size(), (uint64_t *)offs.data());
  std::vector<char> bytes(total);
  offsets.resize(v.size() + 1);
  device::copy(bytes.data(), out.data(), bytes.size(), SPK_COPY_D2H, c.stream());
  device::copy(offsets.data(), offs.data(), offsets.size() * 8, SPK_COPY_D2H, c.stream());
  device::sync(c.stream());
  return bytes;
}

// frames data[offsets[i], offsets[i+1]) with a prefix_len-byte header each
template <uint64_t conf = sp_config::DEFAULT, typename R>
std::vector<err_code> deserialize_frames(std::vector<R> &out, const char *data, std::size_t size,
                                         const std::vector<uint64_t> &offsets,
                                         uint32_t prefix_len) {
  return deserialize_messages<conf>(out, data, size, offsets, prefix_len);
}

#if SPK_GPU_WITH_REFERENCE
// next to the reference our constexpr type hash must be the reference's:
// checked at compile time for every message type the GPU path sees
template <typename T>
constexpr bool hash_matches_reference() {
  return get_type_code<T>() == struct_pack::get_type_code<T>();
}
#endif

}  // namespace struct_pack::gpu
