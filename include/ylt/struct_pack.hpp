// struct_pack.hpp — MI355X-native struct_pack front end (our implementation).
//
// Keeps the reference's entry-point names, argument meaning and error values
// (reference include/ylt/struct_pack.hpp:75-727, error_code.hpp:21-64) for
// batches of records, and produces the reference's wire bytes exactly. The
// byte work runs in the gfx950 HIP kernels of libspk_codec.so behind the C
// ABI of include/spk_codec.h; this header only reflects types, builds the
// descriptor, stages host objects and calls the ABI. There is no CPU codec.
//
//   get_type_code<T>() / get_type_literal<T>()        compile time
//   get_needed_size(const std::vector<T>&)             size pass (device)
//   serialize(const std::vector<T>&) / serialize_to(buf, ...)
//   deserialize_to(std::vector<T>&, const char*, size_t[, size_t& consume])
//   deserialize<std::vector<T>>(const char*, size_t)  -> result<T>
//   serialize_messages / deserialize_messages         coro_rpc payload batches
//   serialize_frames / deserialize_frames             ... in coro_rpc's framing
//                                                      ([req|resp header][payload])
//   device::codec<T>                                   device-resident batches
//
// Build: hipcc -std=c++20 -I include ... -L yalantinglibs_amd -lspk_codec
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "spk_codec.h"
#include "struct_pack/spk_layout.hpp"

namespace struct_pack {

// ---- error model (error_code.hpp:21-64) ------------------------------------
enum class errc {
  ok = 0,
  no_buffer_space,
  invalid_buffer,
  hash_conflict,
  invalid_width_of_container_length,
};

struct err_code {
  errc ec = errc::ok;
  constexpr err_code() noexcept = default;
  constexpr err_code(errc e) noexcept : ec(e) {}
  constexpr operator errc() const noexcept { return ec; }
  constexpr explicit operator bool() const noexcept { return ec != errc::ok; }
  constexpr int val() const noexcept { return static_cast<int>(ec); }
  std::string_view message() const noexcept {
    return spk_errc_message(static_cast<int32_t>(ec));
  }
};

// expected<T, err_code> stand-in (the reference returns tl::expected)
template <typename T>
class result {
 public:
  result(T v) : v_(std::move(v)) {}
  result(err_code e) : e_(e) {}
  bool has_value() const noexcept { return v_.has_value(); }
  explicit operator bool() const noexcept { return has_value(); }
  T &value() { return v_.value(); }
  const T &value() const { return v_.value(); }
  T &operator*() { return *v_; }
  err_code error() const noexcept { return e_; }

 private:
  std::optional<T> v_;
  err_code e_{};
};

// serialize_buffer_size (calculate_size.hpp:391-405)
struct serialize_buffer_size {
  std::size_t len_ = 0;
  unsigned char metainfo_ = 0;
  constexpr std::size_t size() const { return len_; }
  constexpr unsigned char metainfo() const { return metainfo_; }
  constexpr operator std::size_t() const { return len_; }
};

class spk_error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

namespace device {

inline void check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw spk_error(std::string(what) + ": " + hipGetErrorString(e));
}
inline void check_spk(int rc, const char *what) {
  if (rc != SPK_OK) throw spk_error(std::string(what) + " failed (" + std::to_string(rc) + ")");
}

// RAII device allocation
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
    if (p_) (void)hipFree(p_);
  }
  void resize(std::size_t n) {  // grows only; contents not preserved
    if (n <= n_) return;
    if (p_) check(hipFree(p_), "hipFree");
    p_ = nullptr;
    check(hipMalloc(&p_, n ? n : 1), "hipMalloc");
    n_ = n;
  }
  void *data() const { return p_; }
  std::size_t size() const { return n_; }

 private:
  void *p_ = nullptr;
  std::size_t n_ = 0;
};

// A batch of T in device memory: device records + one heap per span.
template <typename T>
struct batch {
  buffer recs;
  std::vector<buffer> heaps;
  std::vector<uint64_t> heap_elems;
  std::size_t n = 0;
};

template <typename T, uint64_t conf = sp_config::DEFAULT>
class codec {
 public:
  explicit codec(hipStream_t s = nullptr) : s_(s) {}

  static const spk_layout &layout() {
    static const spk_layout L = [] {
      spk_layout l = make_spk_layout<T, conf>();
      check_spk(spk_layout_check(&l), "spk_layout_check");
      return l;
    }();
    return L;
  }
  static constexpr bool trivial = spk_detail::is_trivially_serializable<T>();

  // ---- staging (host <-> device) -----------------------------------------
  batch<T> upload(const T *v, std::size_t n) {
    const spk_layout &L = layout();
    batch<T> b;
    b.n = n;
    b.recs.resize(n * L.rec_stride);
    if constexpr (trivial) {
      if (n) check(hipMemcpyAsync(b.recs.data(), v, n * sizeof(T), hipMemcpyHostToDevice, s_),
                   "H2D");
    } else {
      std::vector<uint8_t> recs(n * L.rec_stride, 0);
      std::vector<std::vector<uint8_t>> heaps(n_spans());
      for (std::size_t i = 0; i < n; ++i) {
        spk_detail::marshal_state st{&L, recs.data() + i * L.rec_stride, 0, 0, &heaps, 0};
        spk_detail::to_device(v[i], st);
      }
      if (n) check(hipMemcpyAsync(b.recs.data(), recs.data(), recs.size(),
                                  hipMemcpyHostToDevice, s_), "H2D");
      for (uint32_t k = 0; k < n_spans(); ++k) {
        b.heaps.emplace_back(heaps[k].size());
        b.heap_elems.push_back(heaps[k].size() / span_elem(k));
        if (!heaps[k].empty())
          check(hipMemcpyAsync(b.heaps[k].data(), heaps[k].data(), heaps[k].size(),
                               hipMemcpyHostToDevice, s_), "H2D");
      }
      check(hipStreamSynchronize(s_), "sync");  // host staging buffers die here
    }
    return b;
  }

  // ok(i) selects the records to materialise (failed messages stay default)
  template <typename Pred = std::nullptr_t>
  void download(const batch<T> &b, std::size_t n, T *out, Pred ok = nullptr) {
    const spk_layout &L = layout();
    if constexpr (trivial) {
      if (n) check(hipMemcpyAsync(out, b.recs.data(), n * sizeof(T), hipMemcpyDeviceToHost, s_),
                   "D2H");
      check(hipStreamSynchronize(s_), "sync");
    } else {
      std::vector<uint8_t> recs(n * L.rec_stride);
      // kept in the codec: string_view / span members of the decoded objects
      // alias these host heaps, valid until this thread's next decode of T
      // (the reference's views alias its input buffer, unpacker.hpp:1135-1145)
      std::vector<std::vector<uint8_t>> &heaps = view_heaps_;
      heaps.assign(n_spans(), {});
      if (n) check(hipMemcpyAsync(recs.data(), b.recs.data(), recs.size(),
                                  hipMemcpyDeviceToHost, s_), "D2H");
      std::vector<const uint8_t *> hp(n_spans());
      for (uint32_t k = 0; k < n_spans(); ++k) {
        heaps[k].resize(b.heap_elems[k] * span_elem(k));
        if (!heaps[k].empty())
          check(hipMemcpyAsync(heaps[k].data(), b.heaps[k].data(), heaps[k].size(),
                               hipMemcpyDeviceToHost, s_), "D2H");
        hp[k] = heaps[k].data();
      }
      check(hipStreamSynchronize(s_), "sync");
      for (std::size_t i = 0; i < n; ++i) {
        if constexpr (!std::is_same_v<Pred, std::nullptr_t>)
          if (!ok(i)) continue;
        spk_detail::unmarshal_state st{&L, recs.data() + i * L.rec_stride, 0, 0, hp.data(), 0};
        spk_detail::from_device(out[i], st);
      }
    }
  }

  // ---- device-resident codec ----------------------------------------------
  spk_plan_t plan(const batch<T> &b, int mode) {
    ws_.resize(spk_workspace_bytes(&layout(), mode, b.n, 0));
    plan_.resize(sizeof(spk_plan_t));
    check_spk(spk_plan(&layout(), mode, b.n, b.recs.data(), (spk_plan_t *)plan_.data(),
                       ws_.data(), ws_.size(), s_), "spk_plan");
    spk_plan_t p{};
    check(hipMemcpyAsync(&p, plan_.data(), sizeof(p), hipMemcpyDeviceToHost, s_), "D2H");
    check(hipStreamSynchronize(s_), "sync");
    return p;
  }

  // after plan(): write into d_out (device). Stream-ordered, no sync.
  void encode(const batch<T> &b, int mode, void *d_out, std::size_t cap,
              uint64_t *d_offsets = nullptr) {
    std::vector<const void *> hp(n_spans() ? n_spans() : 1, nullptr);
    for (uint32_t k = 0; k < n_spans(); ++k) hp[k] = b.heaps[k].data();
    check_spk(spk_encode(&layout(), mode, b.n, b.recs.data(), hp.data(),
                         (const spk_plan_t *)plan_.data(), d_out, cap, d_offsets, ws_.data(),
                         ws_.size(), s_), "spk_encode");
  }

  // after plan(SPK_MODE_MESSAGES): n framed messages [prefix][serialize(rec)]
  void encode_framed(const batch<T> &b, const spk_frame &f, void *d_out, std::size_t cap,
                     uint64_t *d_offsets = nullptr) {
    std::vector<const void *> hp(n_spans() ? n_spans() : 1, nullptr);
    for (uint32_t k = 0; k < n_spans(); ++k) hp[k] = b.heaps[k].data();
    check_spk(spk_encode_framed(&layout(), b.n, b.recs.data(), hp.data(),
                                (const spk_plan_t *)plan_.data(), &f, d_out, cap, d_offsets,
                                ws_.data(), ws_.size(), s_), "spk_encode_framed");
  }

  // decode into `out` (capacities from out.n / out.heap_elems); `prefix` =
  // frame bytes before each message (MESSAGES mode only)
  spk_dresult_t decode(batch<T> &out, const void *d_wire, std::size_t len, int mode,
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
      check_spk(spk_decode_framed(&layout(), d_wire, len, d_offsets, n_msgs, prefix,
                                  out.recs.data(), out.n, hp.data(), caps.data(),
                                  (spk_dresult_t *)res_.data(), d_errc, ws_.data(), ws_.size(),
                                  s_), "spk_decode_framed");
    else
      check_spk(spk_decode(&layout(), mode, d_wire, len, d_offsets, n_msgs, out.recs.data(),
                           out.n, hp.data(), caps.data(), (spk_dresult_t *)res_.data(), d_errc,
                           ws_.data(), ws_.size(), s_), "spk_decode");
    spk_dresult_t r{};
    check(hipMemcpyAsync(&r, res_.data(), sizeof(r), hipMemcpyDeviceToHost, s_), "D2H");
    check(hipStreamSynchronize(s_), "sync");
    return r;
  }

  // a batch able to hold the decode of a `len`-byte wire buffer
  batch<T> alloc_for_wire(std::size_t len, std::size_t max_records) {
    batch<T> b;
    b.n = max_records;
    b.recs.resize(max_records * layout().rec_stride);
    for (uint32_t k = 0; k < n_spans(); ++k) {
      // an OPTION holds at most one value per record, readable or not
      b.heap_elems.push_back(span_is_option(k) ? max_records : len / span_elem(k) + 1);
      b.heaps.emplace_back(b.heap_elems.back() * span_elem(k));
    }
    return b;
  }

  static uint32_t n_spans() {
    uint32_t k = 0;
    for (uint32_t i = 0; i < layout().n_ops; ++i) k += has_heap(layout().ops[i]);
    return k;
  }
  // SPAN + OPTION members: one heap each (COPY and VARINT live in the record)
  static bool has_heap(const spk_op &o) {
    return o.kind == SPK_OP_SPAN || o.kind == SPK_OP_OPTION;
  }
  static uint32_t span_elem(uint32_t k) {
    for (uint32_t i = 0, s = 0; i < layout().n_ops; ++i)
      if (has_heap(layout().ops[i]) && s++ == k) return layout().ops[i].size;
    return 1;
  }
  static bool span_is_option(uint32_t k) {
    for (uint32_t i = 0, s = 0; i < layout().n_ops; ++i)
      if (has_heap(layout().ops[i]) && s++ == k)
        return layout().ops[i].kind == SPK_OP_OPTION;
    return false;
  }
  static std::size_t min_record_wire() {
    std::size_t m = 0;
    for (uint32_t i = 0; i < layout().n_ops; ++i)
      m += layout().ops[i].kind == SPK_OP_COPY ? layout().ops[i].size : 1;
    return m ? m : 1;
  }
  hipStream_t stream() const { return s_; }

 private:
  hipStream_t s_;
  buffer ws_, plan_, res_;
  std::vector<std::vector<uint8_t>> view_heaps_;
};

template <typename T, uint64_t conf>
codec<T, conf> &thread_codec() {
  thread_local codec<T, conf> c;
  return c;
}

}  // namespace device

// ===========================================================================
// Reference-named entry points (host data in, host bytes out)
// ===========================================================================
template <uint64_t conf = sp_config::DEFAULT, typename T>
serialize_buffer_size get_needed_size(const std::vector<T> &v) {
  auto &c = device::thread_codec<T, conf>();
  auto b = c.upload(v.data(), v.size());
  spk_plan_t p = c.plan(b, SPK_MODE_VECTOR);
  serialize_buffer_size r;
  r.len_ = p.total_bytes;
  r.metainfo_ = static_cast<unsigned char>(p.has_meta ? p.metainfo : 0);
  return r;
}

// serialize_to(Buffer&, const std::vector<T>&): appends (struct_pack.hpp:137-159)
template <uint64_t conf = sp_config::DEFAULT, typename Buffer, typename T>
void serialize_to(Buffer &buffer, const std::vector<T> &v) {
  auto &c = device::thread_codec<T, conf>();
  auto b = c.upload(v.data(), v.size());
  spk_plan_t p = c.plan(b, SPK_MODE_VECTOR);
  device::buffer out(p.total_bytes);
  c.encode(b, SPK_MODE_VECTOR, out.data(), out.size());
  const std::size_t old = buffer.size();
  buffer.resize(old + p.total_bytes);
  device::check(hipMemcpyAsync(buffer.data() + old, out.data(), p.total_bytes,
                               hipMemcpyDeviceToHost, c.stream()), "D2H");
  device::check(hipStreamSynchronize(c.stream()), "sync");
}

// serialize<Buffer>(v) and serialize<conf, Buffer>(v), as the reference's two
// overloads (struct_pack.hpp:191-207, 228-244)
template <typename Buffer = std::vector<char>, typename T>
Buffer serialize(const std::vector<T> &v) {
  Buffer b;
  serialize_to<sp_config::DEFAULT>(b, v);
  return b;
}
template <uint64_t conf, typename Buffer = std::vector<char>, typename T>
Buffer serialize(const std::vector<T> &v) {
  Buffer b;
  serialize_to<conf>(b, v);
  return b;
}

// deserialize_to(std::vector<T>&, data, size, consume_len) (struct_pack.hpp:343-357)
template <uint64_t conf = sp_config::DEFAULT, typename T>
err_code deserialize_to(std::vector<T> &out, const char *data, std::size_t size,
                        std::size_t &consume_len) {
  auto &c = device::thread_codec<T, conf>();
  device::buffer wire(size + 16);
  if (size)
    device::check(hipMemcpyAsync(wire.data(), data, size, hipMemcpyHostToDevice, c.stream()),
                  "H2D");
  const std::size_t cap = size / c.min_record_wire() + 1;
  auto b = c.alloc_for_wire(size, cap);
  spk_dresult_t r = c.decode(b, wire.data(), size, SPK_MODE_VECTOR);
  consume_len = 0;
  if (r.errc == SPK_ERRC_CAPACITY) throw spk_error("struct_pack: decode capacity exceeded");
  if (r.errc) return static_cast<errc>(r.errc);
  for (uint32_t k = 0; k < c.n_spans(); ++k) b.heap_elems[k] = r.heap_used[k];
  out.resize(r.count);
  c.download(b, r.count, out.data());
  consume_len = r.consumed;
  return {};
}

template <uint64_t conf = sp_config::DEFAULT, typename T>
err_code deserialize_to(std::vector<T> &out, const char *data, std::size_t size) {
  std::size_t consumed;
  return deserialize_to<conf>(out, data, size, consumed);
}

template <uint64_t conf = sp_config::DEFAULT, typename T, typename View>
  requires requires(const View &v) { v.data(); v.size(); }
err_code deserialize_to(std::vector<T> &out, const View &v) {
  return deserialize_to<conf>(out, reinterpret_cast<const char *>(v.data()), v.size());
}

template <typename Vec, uint64_t conf = sp_config::DEFAULT>
result<Vec> deserialize(const char *data, std::size_t size) {
  Vec v;
  err_code e = deserialize_to<conf>(v, data, size);
  if (e) return e;
  return v;
}

// ---- coro_rpc payload batches: n independent serialize(T) messages --------
template <uint64_t conf = sp_config::DEFAULT, typename T>
std::vector<char> serialize_messages(const std::vector<T> &v, std::vector<uint64_t> &offsets) {
  auto &c = device::thread_codec<T, conf>();
  auto b = c.upload(v.data(), v.size());
  spk_plan_t p = c.plan(b, SPK_MODE_MESSAGES);
  device::buffer out(p.total_bytes), offs((v.size() + 1) * sizeof(uint64_t));
  c.encode(b, SPK_MODE_MESSAGES, out.data(), out.size(), (uint64_t *)offs.data());
  std::vector<char> bytes(p.total_bytes);
  offsets.resize(v.size() + 1);
  device::check(hipMemcpyAsync(bytes.data(), out.data(), bytes.size(), hipMemcpyDeviceToHost,
                               c.stream()), "D2H");
  device::check(hipMemcpyAsync(offsets.data(), offs.data(), offsets.size() * 8,
                               hipMemcpyDeviceToHost, c.stream()), "D2H");
  device::check(hipStreamSynchronize(c.stream()), "sync");
  return bytes;
}

// decodes message i = data[offsets[i] + prefix, offsets[i+1]) into out[i];
// returns per-message errc
template <uint64_t conf = sp_config::DEFAULT, typename T>
std::vector<err_code> deserialize_messages(std::vector<T> &out, const char *data,
                                           std::size_t size,
                                           const std::vector<uint64_t> &offsets,
                                           uint32_t prefix = 0) {
  auto &c = device::thread_codec<T, conf>();
  const std::size_t n = offsets.empty() ? 0 : offsets.size() - 1;
  device::buffer wire(size + 16), offs(offsets.size() * 8 + 8), ec(n * 4 + 4);
  device::check(hipMemcpyAsync(wire.data(), data, size, hipMemcpyHostToDevice, c.stream()), "H2D");
  device::check(hipMemcpyAsync(offs.data(), offsets.data(), offsets.size() * 8,
                               hipMemcpyHostToDevice, c.stream()), "H2D");
  auto b = c.alloc_for_wire(size, n);
  spk_dresult_t r = c.decode(b, wire.data(), size, SPK_MODE_MESSAGES, (uint64_t *)offs.data(), n,
                             (int32_t *)ec.data(), prefix);
  if (r.errc == SPK_ERRC_CAPACITY) throw spk_error("struct_pack: decode capacity exceeded");
  std::vector<int32_t> e(n);
  device::check(hipMemcpyAsync(e.data(), ec.data(), n * 4, hipMemcpyDeviceToHost, c.stream()),
                "D2H");
  for (uint32_t k = 0; k < c.n_spans(); ++k) b.heap_elems[k] = r.heap_used[k];
  device::check(hipStreamSynchronize(c.stream()), "sync");
  out.assign(n, T{});
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
template <uint64_t conf = sp_config::DEFAULT, typename T>
std::vector<char> serialize_frames(const std::vector<T> &v, const spk_frame &f,
                                   std::vector<uint64_t> &offsets) {
  auto &c = device::thread_codec<T, conf>();
  auto b = c.upload(v.data(), v.size());
  spk_plan_t p = c.plan(b, SPK_MODE_MESSAGES);
  const std::size_t total = p.total_bytes + v.size() * (std::size_t)f.prefix_len;
  device::buffer out(total), offs((v.size() + 1) * sizeof(uint64_t));
  c.encode_framed(b, f, out.data(), out.size(), (uint64_t *)offs.data());
  std::vector<char> bytes(total);
  offsets.resize(v.size() + 1);
  device::check(hipMemcpyAsync(bytes.data(), out.data(), bytes.size(), hipMemcpyDeviceToHost,
                               c.stream()), "D2H");
  device::check(hipMemcpyAsync(offsets.data(), offs.data(), offsets.size() * 8,
                               hipMemcpyDeviceToHost, c.stream()), "D2H");
  device::check(hipStreamSynchronize(c.stream()), "sync");
  return bytes;
}

// frames data[offsets[i], offsets[i+1]) with a prefix_len-byte header each
template <uint64_t conf = sp_config::DEFAULT, typename T>
std::vector<err_code> deserialize_frames(std::vector<T> &out, const char *data, std::size_t size,
                                         const std::vector<uint64_t> &offsets,
                                         uint32_t prefix_len) {
  return deserialize_messages<conf>(out, data, size, offsets, prefix_len);
}

}  // namespace struct_pack
