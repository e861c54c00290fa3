// get_field<T, I> and reader_t decoding of struct_pack::gpu against the
// reference, in one process (built next to the reference headers into
// oracle/_ref/test_reader_field).
//
//   test_reader_field cpu   the host walker alone (no GPU): the bytes it
//                           pulls out of the reference's memory_reader and
//                           out of a forward-only reader for every message
//                           and every cut of it, against the reference's own
//                           reader positions (deserialize_to(T&, Reader&),
//                           get_field_to(Field&, Reader&));
//   test_reader_field       GPU: get_field / get_field_to on every fixture
//                           cut at every byte (long messages: every byte of
//                           the first 96, then a stride) == the reference's
//                           errc and field; deserialize_to(t, reader) and
//                           get_field(reader) over memory_reader and a
//                           forward-only reader == the reference's errc,
//                           value and reader position.
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include <ylt/struct_pack.hpp>
#include <ylt/struct_pack_gpu.hpp>

#include "../../oracle/ref/types.hpp"

static_assert(SPK_GPU_WITH_REFERENCE, "build with the reference on the include path");

static int g_fail = 0, g_checks = 0;
static const char *g_what = "";
#define CHECK(c)                                                                              \
  do {                                                                                        \
    ++g_checks;                                                                               \
    if (!(c)) {                                                                               \
      if (++g_fail < 40) std::fprintf(stderr, "%s:%d: %s: CHECK(%s) failed\n", __FILE__, __LINE__, \
                                      g_what, #c);                                            \
    }                                                                                         \
  } while (0)

// a forward-only reader whose short read consumes the rest (a closed socket)
struct fwd_reader {
  const char *p, *end;
  bool read(char *dst, std::size_t n) {
    if (static_cast<std::size_t>(end - p) < n) {
      p = end;
      return false;
    }
    std::memcpy(dst, p, n);
    p += n;
    return true;
  }
  bool ignore(std::size_t n) {
    if (static_cast<std::size_t>(end - p) < n) {
      p = end;
      return false;
    }
    p += n;
    return true;
  }
  std::size_t tellg() { return reinterpret_cast<std::size_t>(p); }
};
using mem_reader = struct_pack::detail::memory_reader;

template <typename X>
std::string bytes_of(const X &x) {
  if constexpr (struct_pack::gpu::detail::is_compat_v<X>) {
    if (!x.has_value()) return "<none>";
    return struct_pack::serialize<std::string>(*x);
  } else {
    return struct_pack::serialize<std::string>(x);
  }
}

// the cuts of a message: every length for the first 96 bytes, then a stride
static std::vector<std::size_t> cuts(std::size_t n) {
  std::vector<std::size_t> c;
  const std::size_t step = n <= 256 ? 1 : (n - 96) / 96 + 1;
  for (std::size_t k = 0; k <= n; k += (k < 96 ? 1 : step)) c.push_back(k);
  if (c.back() != n) c.push_back(n);
  return c;
}

namespace spk_gold {
inline void fill(rpcb::person &p, uint64_t seed, uint64_t i, uint32_t maxlen) {
  p = make_person(seed, i, maxlen);
}
inline void fill(RecS &r, uint64_t seed, uint64_t i, uint32_t maxlen) { r = make_recs(seed, i, maxlen); }
inline void fill(Outer &o, uint64_t seed, uint64_t i, uint32_t maxn) { o = make_outer(seed, i, maxn); }
inline void fill(Rec64 &r, uint64_t seed, uint64_t i, uint32_t) { r = make_rec64(seed, i); }
}  // namespace spk_gold

// ---- CPU: the walker's bytes against the reference's reader positions ------
template <typename T>
void cpu_message(const std::string &buf, const char *what) {
  g_what = what;
  namespace d = struct_pack::gpu::detail;
  for (std::size_t k : cuts(buf.size())) {
    const std::string cut = buf.substr(0, k);
    // memory_reader: the reference's reads then its position
    T ref{};
    mem_reader rr{cut.data(), cut.data() + cut.size()};
    const auto re = struct_pack::deserialize_to(ref, rr);
    const std::size_t rpos = static_cast<std::size_t>(rr.now - cut.data());
    mem_reader gr{cut.data(), cut.data() + cut.size()};
    const std::vector<char> got = d::pull_message<struct_pack::sp_config::DEFAULT, T>(gr);
    const std::size_t gpos = static_cast<std::size_t>(gr.now - cut.data());
    CHECK(std::string(got.begin(), got.end()) == cut.substr(0, gpos));
    // a whole message: exactly its bytes; a cut one: everything the reader
    // holds, unless the walk stopped at bad data first
    if (k == buf.size()) CHECK(!re && gpos == rpos);
    if (re) CHECK(gpos == k || re == struct_pack::errc::invalid_buffer ||
                  re == struct_pack::errc::hash_conflict);
    if (re && !(gpos == k || re == struct_pack::errc::invalid_buffer ||
                re == struct_pack::errc::hash_conflict) && g_fail < 10)
      std::fprintf(stderr, "  cut %zu of %zu: ref errc %d at %zu, walker pulled %zu\n", k,
                   buf.size(), (int)re.val(), rpos, gpos);
    // forward-only reader: a short read ends it; the bytes pulled are those
    // before the failed read, and on success the reader is where the
    // reference leaves the same kind of reader
    T ref2{};
    fwd_reader fr0{cut.data(), cut.data() + cut.size()};
    const auto re2 = struct_pack::deserialize_to(ref2, fr0);
    fwd_reader fr{cut.data(), cut.data() + cut.size()};
    const std::vector<char> got2 = d::pull_message<struct_pack::sp_config::DEFAULT, T>(fr);
    CHECK(std::string(got2.begin(), got2.end()) == cut.substr(0, got2.size()));
    if (!re2) CHECK(fr.p == fr0.p);
  }
}

// the walker's get_field pull (header + members 0..I, + version passes) ==
// the reference's memory_reader position after its get_field_to
template <typename T, std::size_t I>
void cpu_field(const std::string &buf) {
  namespace d = struct_pack::gpu::detail;
  using F = struct_pack::gpu::field_t<T, I>;
  F rf{};
  mem_reader rr{buf.data(), buf.data() + buf.size()};
  const auto re = struct_pack::get_field_to<T, I>(rf, rr);
  const std::size_t rpos = static_cast<std::size_t>(rr.now - buf.data());
  const spk_layout &L =
      struct_pack::gpu::device::codec<typename d::msg_traits<T>::rec>::layout();
  std::vector<char> pulled;
  mem_reader gr{buf.data(), buf.data() + buf.size()};
  d::pull_cursor<mem_reader> c{gr, pulled};
  d::header_info h;
  if (d::walk_header(c, L.fmt_one, h) == struct_pack::errc{})
    (void)d::get_field_walk<T, I>(
        c, h.w, h.data_len, [&](auto &cc) { return d::walk_one<F>(cc, h.w); },
        [&](auto &cc, bool &past) -> struct_pack::errc {
          if constexpr (d::is_compat_v<F>)
            return d::walk_compat_member<F>(cc, h.w, h.data_len, past);
          else
            return (void)cc, (void)past, struct_pack::errc{};
        });
  // the walk ran dry (a member before I did not fit, the reference carried
  // on with the next one): then everything the reader holds is taken
  if (c.dry) d::drain(gr, pulled);
  if (!re) CHECK(pulled.size() == (c.dry ? buf.size() : rpos));
}

// ---- GPU: get_field on every cut, readers ------------------------------------
template <typename T, std::size_t I>
void gpu_field(const std::string &buf) {
  using F = struct_pack::gpu::field_t<T, I>;
  for (std::size_t k : cuts(buf.size())) {
    auto r = struct_pack::get_field<T, I>(buf.data(), k);
    auto g = struct_pack::gpu::get_field<T, I>(buf.data(), k);
    CHECK(r.has_value() == g.has_value());
    if (r.has_value() != g.has_value()) {
      std::fprintf(stderr, "  member %zu cut %zu of %zu: ref %d gpu %d\n", I, k, buf.size(),
                   r.has_value() ? 0 : (int)r.error(), g.has_value() ? 0 : (int)g.error());
      continue;
    }
    if (r.has_value())
      CHECK(bytes_of(r.value()) == bytes_of(g.value()));
    else
      CHECK(r.error().val() == g.error().val());
    F a{}, b{};
    const auto ea = struct_pack::get_field_to<T, I>(a, buf.data(), k);
    const auto eb = struct_pack::gpu::get_field_to<T, I>(b, buf.data(), k);
    CHECK(ea.val() == eb.val());
    if (!ea && !eb) CHECK(bytes_of(a) == bytes_of(b));
  }
  // from readers (test_stream.cpp:91-138): the whole message and a few cuts
  for (std::size_t k : {buf.size(), buf.size() / 2, buf.size() > 3 ? buf.size() - 3 : 0}) {
    mem_reader rr{buf.data(), buf.data() + k}, gr{buf.data(), buf.data() + k};
    auto r = struct_pack::get_field<T, I>(rr);
    auto g = struct_pack::gpu::get_field<T, I>(gr);
    CHECK(r.has_value() == g.has_value());
    if (r.has_value() && g.has_value()) {
      CHECK(bytes_of(r.value()) == bytes_of(g.value()));
      // the reference's position, or the reader's end when an earlier
      // member did not fit and the rest was drained (struct_pack_gpu.hpp)
      CHECK(rr.now == gr.now || gr.now == buf.data() + k);
      if (rr.now != gr.now && gr.now != buf.data() + k)
        std::fprintf(stderr, "  get_field<%zu>(reader) cut %zu of %zu: ref at %zd, gpu at %zd\n", I,
                     k, buf.size(), rr.now - buf.data(), gr.now - buf.data());
    }
    if (!r.has_value() && !g.has_value()) CHECK(r.error().val() == g.error().val());
  }
}

template <typename T, typename Reader>
void gpu_reader_one(const std::string &cut) {
  T ref{}, got{};
  Reader rr{cut.data(), cut.data() + cut.size()}, gr{cut.data(), cut.data() + cut.size()};
  const auto re = struct_pack::deserialize_to(ref, rr);
  const auto ge = struct_pack::gpu::deserialize_to(got, gr);
  CHECK(re.val() == ge.val());
  if (re.val() != ge.val())
    std::fprintf(stderr, "  %s %s cut %zu: ref %d gpu %d\n", g_what,
                 std::is_same_v<Reader, fwd_reader> ? "fwd" : "mem", cut.size(), (int)re.val(),
                 (int)ge.val());
  if (!re && !ge) {
    CHECK(bytes_of(ref) == bytes_of(got));
    const std::size_t end = reinterpret_cast<std::size_t>(cut.data() + cut.size());
    CHECK(rr.tellg() == gr.tellg() || gr.tellg() == end);
    if (rr.tellg() != gr.tellg() && gr.tellg() != end)
      std::fprintf(stderr, "  %s deserialize_to(reader) cut %zu: ref at %zu, gpu at %zu\n",
                   std::is_same_v<Reader, fwd_reader> ? "fwd" : "mem", cut.size(),
                   rr.tellg() - (std::size_t)cut.data(), gr.tellg() - (std::size_t)cut.data());
  }
}

template <typename T>
void gpu_message(const std::string &buf, const char *what) {
  g_what = what;
  for (std::size_t k : cuts(buf.size())) {
    const std::string cut = buf.substr(0, k);
    gpu_reader_one<T, mem_reader>(cut);
    gpu_reader_one<T, fwd_reader>(cut);
  }
  // two messages back to back: the reader is left at the second
  std::string two = buf + buf;
  mem_reader r{two.data(), two.data() + two.size()};
  T a{}, b{};
  CHECK(!struct_pack::gpu::deserialize_to(a, r));
  CHECK(r.now == two.data() + buf.size());
  CHECK(!struct_pack::gpu::deserialize_to(b, r) && r.now == two.data() + two.size());
  CHECK(bytes_of(a) == buf && bytes_of(b) == buf);
}

template <typename T, std::size_t... I>
void fields(bool gpu, const std::string &buf, std::index_sequence<I...>) {
  if (gpu)
    (gpu_field<T, I>(buf), ...);
  else
    (cpu_field<T, I>(buf), ...);
}

static const char *g_only = nullptr;
template <typename T>
void type_case(bool gpu, const char *what, uint64_t seed, uint32_t param, int nvals = 3) {
  if (g_only && std::strcmp(g_only, what) != 0) return;
  g_what = what;
  using M = struct_pack::gpu::detail::members_tuple_t<T>;
  for (int i = 0; i < nvals; ++i) {
    T v{};
    spk_gold::fill(v, seed, static_cast<uint64_t>(i) * 7 + 1, param);
    const std::string one = struct_pack::serialize<std::string>(v);
    if (gpu) CHECK(struct_pack::gpu::serialize<std::string>(v) == one);
    fields<T>(gpu, one, std::make_index_sequence<std::tuple_size_v<M>>{});
    if (gpu)
      gpu_message<T>(one, what);
    else
      cpu_message<T>(one, what);
  }
  std::vector<T> vs(40);
  for (std::size_t i = 0; i < vs.size(); ++i) spk_gold::fill(vs[i], seed, i + 100, param);
  const std::string many = struct_pack::serialize<std::string>(vs);
  if (gpu)
    gpu_message<std::vector<T>>(many, what);
  else
    cpu_message<std::vector<T>>(many, what);
}

int main(int argc, char **argv) {
  const bool gpu = !(argc > 1 && std::strcmp(argv[1], "cpu") == 0);
  if (argc > 2) g_only = argv[2];
  // the reference's own case (test_serialize.cpp get_field): person cut
  // short still yields member 1
  if (gpu) {
    g_what = "person{7,Betty,24,1.5}";
    const rpcb::person p{7, "Betty", 24, 1.5};
    const std::string b = struct_pack::serialize<std::string>(p);
    for (std::size_t k : {std::size_t(18), std::size_t(20)}) {
      auto r = struct_pack::get_field<rpcb::person, 1>(b.data(), k);
      auto g = struct_pack::gpu::get_field<rpcb::person, 1>(b.data(), k);
      CHECK(r.has_value() && g.has_value() && g.value() == "Betty");
      CHECK(!struct_pack::gpu::deserialize<rpcb::person>(b.data(), k).has_value());
    }
  }
  type_case<rpcb::person>(gpu, "person", 0x5EED0008, 24);
  type_case<RecS>(gpu, "recs", 0x5EED0003, 30);
  type_case<Outer>(gpu, "outer", 0x5EED0004, 6);
  type_case<Rec64>(gpu, "rec64", 0x5EED0002, 0);
  type_case<Pad>(gpu, "pad", 0x5EED0005, 0);
  type_case<Mixed>(gpu, "mixed", 0x5EED0006, 12);
  type_case<Opt>(gpu, "opt", 0x5EED0007, 12);
  type_case<OptP>(gpu, "optp", 0x5EED0009, 0);
  type_case<Var>(gpu, "var", 0x5EED000A, 12);
  type_case<VarP>(gpu, "varp", 0x5EED000B, 0);
  type_case<Tags>(gpu, "tags", 0x5EED000E, 4);
  type_case<Group>(gpu, "group", 0x5EED000F, 3);
  type_case<Deep>(gpu, "deep", 0x5EED0010, 3);
  type_case<Vnt>(gpu, "vnt", 0x5EED0011, 6);
  type_case<Cmp>(gpu, "cmp", 0x5EED0012, 8);
  type_case<CmpG>(gpu, "cmpg", 0x5EED001D, 6);
  type_case<FV>(gpu, "fv", 0x5EED0013, 8);
  type_case<FVE>(gpu, "fve", 0x5EED0014, 8);
  type_case<FV32>(gpu, "fv32", 0x5EED0015, 0);
  type_case<EV>(gpu, "ev", 0x5EED0016, 8);
  type_case<ValidateRequest>(gpu, "valreq", 0x5EED001B, 6);
  type_case<Monster>(gpu, "monster", 0x5EED001E, 6);
  type_case<rect2<int32_t>>(gpu, "rect2", 0x5EED001F, 0);
  type_case<Lists>(gpu, "lists", 0x5EED0020, 4);
  type_case<Maps>(gpu, "maps", 0x5EED0021, 0);
  type_case<AlRec>(gpu, "alrec", 0x5EED0019, 8);
  type_case<Wide>(gpu, "wide", 0x5EED0023, 6);
  std::printf("{\"checks\": %d, \"failures\": %d}\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
