// GPU: coro_rpc's serialize-protocol seam with the MI355X codec behind it.
//
// Built NEXT TO THE REFERENCE (-I /root/reference/include ...): the reference's
// coro_rpc handler executor (rpc_execute.hpp:56-179) runs a batch handler with
// struct_pack_gpu_protocol as its serialize protocol, and every byte is
// compared with the reference's own struct_pack_protocol on the same values
// (computed in this process by the reference's CPU struct_pack) and with the
// committed reference-built fixtures. Also checks that the front end's type
// codes equal the reference's at compile time. The binary is built by
// __graft_entry__.build() into oracle/_ref/ (it contains reference code) and
// run by tests/test_gpu_cpp.py on the GPU box.
#include <csignal>
#include <cstdio>
#include <execinfo.h>
#include <unistd.h>
#include <cstring>
#include <fstream>
#include <sstream>
#include <array>
#include <chrono>
#include <memory>
#include <iterator>
#include <map>
#include <optional>
#include <variant>
#include <string>
#include <type_traits>
#include <vector>

#include <ylt/coro_rpc/impl/protocol/coro_rpc_protocol.hpp>
#include <ylt/coro_rpc/impl/protocol/struct_pack_gpu_protocol.hpp>
#include <ylt/coro_rpc/impl/rpc_execute.hpp>

#include "../../oracle/ref/types.hpp"

static_assert(SPK_GPU_WITH_REFERENCE, "build with the reference on the include path");

using coro_rpc::protocol::struct_pack_gpu_protocol;
using coro_rpc::protocol::struct_pack_protocol;
using rpc_protocol = coro_rpc::protocol::coro_rpc_protocol;

static int g_fail = 0, g_checks = 0, g_section = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    ++g_checks;                                                                  \
    if (!(c)) {                                                                  \
      ++g_fail;                                                                  \
      std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
    }                                                                            \
  } while (0)

// our constexpr type hash == the reference's, for every type the tests use
template <typename... T>
constexpr bool all_match() {
  return (struct_pack::gpu::hash_matches_reference<T>() && ...);
}
static_assert(all_match<Rec64, RecS, Inner, Outer, Pad, Mixed, Opt, OptP, Var, VarP,
                        rpcb::point, rpcb::rect, rpcb::person, rect<int>>());
// alignment overrides (alignas, nested alignas, #pragma pack + pack_alignment_v)
static_assert(all_match<Al8, AlOuter, Packed, AlRec, std::vector<AlRec>, std::vector<Packed>>());
static_assert(all_match<std::vector<Rec64>, std::vector<RecS>, std::vector<Outer>,
                        std::vector<Mixed>, std::vector<Opt>, std::vector<Var>,
                        std::vector<rpcb::person>, std::vector<rect<int>>>());

// nested layouts: containers of non-trivial elements, variants, optional /
// compatible values that are not trivially serializable, the varint sp_config
// bits and the set / map / list containers
static_assert(all_match<Tags, Group, Deep, Vnt, CmpG, FV, FVE, FV32, EV, ResponseCode, AliMessage,
                        ValidateRequest, Vec3, Weapon, Monster, rect2<int32_t>, Lists, Maps>());
static_assert(all_match<std::vector<Tags>, std::vector<Vnt>, std::vector<ValidateRequest>,
                        std::vector<Monster>, std::vector<rect2<int32_t>>, std::vector<Maps>,
                        std::vector<Lists>, std::vector<FV>>());
static_assert(struct_pack::gpu::is_gpu_batch_v<std::vector<Monster>> &&
              struct_pack::gpu::is_gpu_batch_v<std::vector<Tags>> &&
              struct_pack::gpu::is_gpu_batch_v<std::vector<rect2<int32_t>>> &&
              struct_pack::gpu::is_gpu_batch_v<std::vector<ValidateRequest>> &&
              struct_pack::gpu::is_gpu_batch_v<std::vector<Maps>>);

static std::string golden(const std::string &name) {
  std::ifstream f(std::string(SPK_GOLDEN_DIR) + "/" + name, std::ios::binary);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

bool operator==(const RecS &a, const RecS &b) { return a.id == b.id && a.name == b.name && a.v == b.v; }
bool operator==(const Inner &a, const Inner &b) { return a.x == b.x && a.y == b.y; }
bool operator==(const Outer &a, const Outer &b) { return a.key == b.key && a.items == b.items; }
namespace rpcb {
bool operator==(const person &a, const person &b) {
  return a.id == b.id && a.name == b.name && a.age == b.age && a.salary == b.salary;
}
}  // namespace rpcb

// ---- handlers: what a coro_rpc service registers ------------------------------
std::vector<RecS> echo_recs(std::vector<RecS> v) { return v; }
std::vector<Outer> reverse_outer(std::vector<Outer> v) {
  std::reverse(v.begin(), v.end());
  return v;
}
int count_people(std::vector<rpcb::person> v) { return (int)v.size(); }  // batch in, int out
std::string greet(rpcb::person p, int times) {  // two arguments: a std::tuple message
  std::string s;
  for (int i = 0; i < times; ++i) s += p.name;
  return s;
}
// the ordinary single-call shapes of a coro_rpc service
rpcb::person echo_person(rpcb::person p) { return p; }
rpcb::rect echo_rect(rpcb::rect r) { return r; }
std::string echo_str(std::string s) { return s; }
int add(int a, int b) { return a + b; }
static int g_pinged = 0;
void ping() { ++g_pinged; }                        // no arguments, void reply
void note(std::string s) { g_pinged += (int)s.size(); }  // void reply
std::vector<int> iota_n(int n) {
  std::vector<int> v(n);
  for (int i = 0; i < n; ++i) v[i] = i * 7 - 3;
  return v;
}
std::vector<std::string> split_name(rpcb::person p, std::string sep) {
  return {p.name, sep, std::to_string(p.age)};
}
std::optional<rpcb::person> maybe(int id, std::optional<std::string> name) {
  if (!name) return std::nullopt;
  return rpcb::person{id, *name, 3, 4.5};
}
std::map<int, std::string> to_map(std::vector<std::string> v) {
  std::map<int, std::string> m;
  for (std::size_t i = 0; i < v.size(); ++i) m[(int)i] = v[i];
  return m;
}
std::variant<int, std::string> pick(bool s, int x) {
  if (s) return std::to_string(x);
  return x;
}
std::pair<int, double> pair_of(int a, double b) { return {a, b}; }

// the reference benchmark's services (src/struct_pack/benchmark/data_def.hpp,
// src/coro_rpc/benchmark/api/ValidateRequest.h)
std::vector<Monster> echo_monsters(std::vector<Monster> v) { return v; }
std::vector<rect2<int32_t>> grow_rects(std::vector<rect2<int32_t>> v) {
  for (auto &r : v) r.width += 1;
  return v;
}
int validate(std::vector<ValidateRequest> v) {
  int ok = 0;
  for (auto &r : v) ok += r.job_id.has_value() && !r.query_keys.empty();
  return ok;
}
std::vector<Maps> echo_maps(std::vector<Maps> v) { return v; }
std::vector<Tags> echo_tags(std::vector<Tags> v) { return v; }
std::vector<Vnt> echo_vnt(std::vector<Vnt> v) { return v; }

// unique_ptr members (optional-like: packer.hpp:271-283), trivial_view
// members (trivial_view.hpp:79-102) and the same record without the view
struct UPtrRec {
  int32_t id;
  std::unique_ptr<std::string> s;
  std::unique_ptr<Inner> p;
  std::unique_ptr<std::vector<int32_t>> v;
  std::unique_ptr<RecS> r;
};
struct ViewData {
  std::array<int32_t, 6> a;
  double d;
};
struct ViewRec {
  std::string name;
  struct_pack::trivial_view<ViewData> data;
  int32_t k;
};
struct PlainRec {
  std::string name;
  ViewData data;
  int32_t k;
};
static_assert(struct_pack::gpu::hash_matches_reference<UPtrRec>() &&
              struct_pack::gpu::hash_matches_reference<std::vector<UPtrRec>>() &&
              struct_pack::gpu::hash_matches_reference<ViewRec>() &&
              struct_pack::gpu::hash_matches_reference<std::tuple<rpcb::person, int>>() &&
              struct_pack::gpu::hash_matches_reference<std::unique_ptr<Inner>>());
static_assert(struct_pack::get_type_code<ViewRec>() == struct_pack::get_type_code<PlainRec>());

// a writer for the user helpers (struct_pack::write needs write(const char*, size_t))
struct str_writer {
  std::string buf;
  void write(const char *p, std::size_t n) { buf.append(p, n); }
};

// the executor as coro_rpc's router calls it (router.hpp:155-163)
template <auto func, typename Proto>
std::pair<coro_rpc::err_code, std::string> run(std::string_view args) {
  coro_rpc::rpc_context<rpc_protocol> ctx;  // handlers above take no context
  return coro_rpc::internal::execute<rpc_protocol, Proto, func>(args, ctx);
}

template <auto func, typename Arg>
void same_as_reference(const Arg &arg, const char *what) {
  // the request payload a coro_rpc client sends (rpc_execute / client pack:
  // one argument -> serialize(arg))
  const std::string req = struct_pack::serialize<std::string>(arg);
  auto ref = run<func, struct_pack_protocol>(req);
  auto gpu = run<func, struct_pack_gpu_protocol>(req);
  CHECK(!ref.first && !gpu.first);
  CHECK(ref.second == gpu.second);
  if (ref.second != gpu.second) std::fprintf(stderr, "  mismatch in %s\n", what);
}

// a call with any number of arguments, packed as the reference client packs
// them (serialize_to_with_offset(buffer, offset, args...), coro_rpc_client.hpp:
// 1398-1410: several arguments are one std::tuple message)
template <auto func, typename... Args>
void call_same_as_reference(const char *what, const Args &...args) {
  std::string req;  // no arguments: no payload (the executor decodes nothing)
  if constexpr (sizeof...(Args) > 0) struct_pack::serialize_to(req, args...);
  auto ref = run<func, struct_pack_protocol>(req);
  auto gpu = run<func, struct_pack_gpu_protocol>(req);
  CHECK(!ref.first && !gpu.first);
  CHECK(ref.second == gpu.second);
  if (ref.first.val() != gpu.first.val() || ref.second != gpu.second)
    std::fprintf(stderr, "  mismatch in %s (%zu vs %zu bytes)\n", what, ref.second.size(),
                 gpu.second.size());
}

static void on_fault(int sig) {  // a host fault: where (stderr), then die
  void *bt[64];
  const int n = backtrace(bt, 64);
  std::fprintf(stderr, "signal %d, section %d\n", sig, g_section);
  backtrace_symbols_fd(bt, n, 2);
  _exit(128 + sig);
}

int main() {
  std::signal(SIGSEGV, on_fault);
  std::signal(SIGABRT, on_fault);
  using namespace spk_gold;
  // (no size thresholds: every payload of every handler below goes through
  // struct_pack::gpu, compared with the reference's struct_pack_protocol)
  const uint64_t S3 = 0x5EED0003, S4 = 0x5EED0004, S8 = 0x5EED0008;

  g_section = 1;
  std::fprintf(stderr, "section 1\n");
  // 1. the protocol statics against the reference protocol and fixtures
  {
    std::vector<RecS> v(300);
    for (uint64_t i = 0; i < v.size(); ++i) v[i] = make_recs(S3, i, 48);
    const std::string want = golden("recs_A_n300_p48_default.bin");
    CHECK(!want.empty());
    const std::string g = struct_pack_gpu_protocol::serialize(v);
    CHECK(g == want);
    CHECK(g == struct_pack_protocol::serialize(v));
    std::tuple<std::vector<RecS>> args;
    CHECK(struct_pack_gpu_protocol::deserialize_to(args, want));
    CHECK(std::get<0>(args) == v);
    // a corrupted head: the protocol reports failure like the reference's
    std::string bad = want;
    bad[0] ^= 0x10;
    std::tuple<std::vector<RecS>> args2;
    CHECK(!struct_pack_gpu_protocol::deserialize_to(args2, bad));
    CHECK(!struct_pack_protocol::deserialize_to(args2, bad));
    // truncated: no_buffer_space on both
    std::tuple<std::vector<RecS>> args3;
    CHECK(!struct_pack_gpu_protocol::deserialize_to(args3, std::string_view(want).substr(0, want.size() - 3)));
  }
  {
    std::vector<Outer> v(1000);
    for (uint64_t i = 0; i < v.size(); ++i) v[i] = make_outer(S4, i, 16);
    const std::string want = golden("outer_A_n1000_p16_default.bin");
    CHECK(struct_pack_gpu_protocol::serialize(v) == want);
    std::tuple<std::vector<Outer>> args;
    CHECK(struct_pack_gpu_protocol::deserialize_to(args, want));
    CHECK(std::get<0>(args) == v);
  }
  g_section = 2;
  std::fprintf(stderr, "section 2\n");
  // 2. the reference's handler executor with the GPU protocol
  {
    std::vector<RecS> v(5000);
    for (uint64_t i = 0; i < v.size(); ++i) v[i] = make_recs(S3, i, 48);
    same_as_reference<echo_recs>(v, "echo_recs");
    std::vector<Outer> o(3000);
    for (uint64_t i = 0; i < o.size(); ++i) o[i] = make_outer(S4, i, 16);
    same_as_reference<reverse_outer>(o, "reverse_outer");
    std::vector<rpcb::person> p(700);
    for (uint64_t i = 0; i < p.size(); ++i) p[i] = make_person(S8, i, 64);
    same_as_reference<count_people>(p, "count_people");
    // an empty batch and a one-record batch
    same_as_reference<echo_recs>(std::vector<RecS>{}, "echo_recs(empty)");
    same_as_reference<echo_recs>(std::vector<RecS>{make_recs(S3, 7, 48)}, "echo_recs(1)");
    // two arguments: one std::tuple<person, int> message, through the GPU
    call_same_as_reference<greet>("greet", make_person(S8, 1, 10), 3);
    const std::string req =
        struct_pack::serialize<std::string>(std::make_tuple(make_person(S8, 1, 10), 3));
    std::string packed;
    struct_pack::serialize_to(packed, make_person(S8, 1, 10), 3);
    CHECK(req == packed);  // serialize(a, b) == serialize(std::tuple{a, b})
    std::tuple<rpcb::person, int> targs;
    CHECK(struct_pack_gpu_protocol::deserialize_to(targs, req));
    CHECK(std::get<0>(targs) == make_person(S8, 1, 10) && std::get<1>(targs) == 3);
    CHECK((struct_pack::gpu::get_type_code<std::tuple<rpcb::person, int>>() ==
           struct_pack::get_type_code<rpcb::person, int>()));
    // a malformed request: coro_rpc's invalid_rpc_arguments on both paths
    std::string bad = struct_pack::serialize<std::string>(v);
    bad.resize(bad.size() / 2);
    auto rb = run<echo_recs, struct_pack_protocol>(bad);
    auto gb = run<echo_recs, struct_pack_gpu_protocol>(bad);
    CHECK(rb.first && gb.first && rb.first.val() == gb.first.val());
  }
  g_section = 21;
  std::fprintf(stderr, "section 2b\n");
  // 2b. handlers over nested record types (C++ front end: ARRAY / VARIANT /
  // OPTGROUP / FVAR layouts and map / set containers)
  {
    auto make = [](auto tag, std::size_t n, uint64_t seed, uint32_t p) {
      std::vector<typename decltype(tag)::type> v(n);
      for (uint64_t i = 0; i < n; ++i) fill(v[i], seed, i, p);
      return v;
    };
    same_as_reference<echo_monsters>(make(std::type_identity<Monster>{}, 2000, 0x5EED001E, 20),
                                     "echo_monsters");
    same_as_reference<grow_rects>(make(std::type_identity<rect2<int32_t>>{}, 3000, 0x5EED001F, 0),
                                  "grow_rects");
    same_as_reference<validate>(
        make(std::type_identity<ValidateRequest>{}, 1500, 0x5EED001B, 16), "validate");
    same_as_reference<echo_maps>(make(std::type_identity<Maps>{}, 500, 0x5EED0021, 0),
                                 "echo_maps");
    same_as_reference<echo_tags>(make(std::type_identity<Tags>{}, 1000, 0x5EED000E, 6),
                                 "echo_tags");
    same_as_reference<echo_vnt>(make(std::type_identity<Vnt>{}, 1000, 0x5EED0011, 6), "echo_vnt");
    same_as_reference<echo_monsters>(std::vector<Monster>{}, "echo_monsters(empty)");
  }
  g_section = 22;
  std::fprintf(stderr, "section 2c\n");
  // 2c. every call shape at default settings: single records, strings, ints,
  // several arguments (std::tuple messages), no arguments, void replies,
  // containers of non-records, optionals, maps, variants, pairs as replies
  {
    call_same_as_reference<echo_person>("echo_person", make_person(S8, 5, 40));
    call_same_as_reference<echo_rect>("echo_rect", rpcb::rect{{1, 2}, {3, 4}});
    call_same_as_reference<echo_str>("echo_str", std::string("hello, coro_rpc"));
    call_same_as_reference<echo_str>("echo_str(empty)", std::string());
    call_same_as_reference<echo_str>("echo_str(300)", std::string(300, 'x'));
    call_same_as_reference<add>("add", 40, 2);
    call_same_as_reference<ping>("ping");
    call_same_as_reference<note>("note", std::string("abc"));
    call_same_as_reference<iota_n>("iota_n", 1000);
    call_same_as_reference<iota_n>("iota_n(0)", 0);
    call_same_as_reference<split_name>("split_name", make_person(S8, 9, 20), std::string("/"));
    call_same_as_reference<maybe>("maybe", 7, std::optional<std::string>("bob"));
    call_same_as_reference<maybe>("maybe(null)", 7, std::optional<std::string>());
    call_same_as_reference<to_map>("to_map", std::vector<std::string>{"a", "bb", "ccc"});
    call_same_as_reference<pick>("pick(s)", true, 77);
    call_same_as_reference<pick>("pick(i)", false, 77);
    call_same_as_reference<pair_of>("pair_of", 3, 2.5);
    call_same_as_reference<count_people>("count_people(1)",
                                         std::vector<rpcb::person>{make_person(S8, 2, 30)});
    // a malformed two-argument request: invalid_rpc_arguments on both paths
    std::string req;
    struct_pack::serialize_to(req, make_person(S8, 1, 10), 3);
    req.resize(req.size() - 2);
    auto rb = run<greet, struct_pack_protocol>(req);
    auto gb = run<greet, struct_pack_gpu_protocol>(req);
    CHECK(rb.first && gb.first && rb.first.val() == gb.first.val());
    // a request of another type: hash_conflict -> invalid arguments on both
    const std::string other = struct_pack::serialize<std::string>(std::string("x"));
    auto ro = run<add, struct_pack_protocol>(other);
    auto go = run<add, struct_pack_gpu_protocol>(other);
    CHECK(ro.first && go.first && ro.first.val() == go.first.val());
  }
  g_section = 3;
  std::fprintf(stderr, "section 3\n");
  // 3. the front end's single-record and reference-order entry points next to
  // the reference: identical bytes for one record message, deserialize<conf, T>
  {
    const rpcb::person p = make_person(S8, 3, 64);
    const auto want = struct_pack::serialize<std::string>(p);
    CHECK(struct_pack::gpu::serialize<std::string>(p) == want);
    auto sz = struct_pack::gpu::get_needed_size(p);
    auto rsz = struct_pack::get_needed_size(p);
    CHECK(sz.size() == rsz.size() && sz.metainfo() == rsz.metainfo());
    std::string buf(sz.size(), '\0');
    struct_pack::gpu::serialize_to(buf.data(), sz, p);
    CHECK(buf == want);
    std::string buf2(rsz.size(), '\0');
    struct_pack::gpu::serialize_to(buf2.data(), rsz, p);  // the reference's size object
    CHECK(buf2 == want);
    auto r = struct_pack::gpu::deserialize<struct_pack::sp_config::DEFAULT, rpcb::person>(want);
    CHECK(r.has_value() && r.value() == p);
    auto f = struct_pack::gpu::get_field<rpcb::person, 1>(want);
    auto rf = struct_pack::get_field<rpcb::person, 1>(want);
    CHECK(f.has_value() && rf.has_value() && f.value() == rf.value());
    std::string off;
    struct_pack::gpu::serialize_to_with_offset(off, 20, p);
    std::string roff;
    struct_pack::serialize_to_with_offset(roff, 20, p);
    CHECK(off.size() == roff.size() && off.substr(20) == roff.substr(20));
  }
  g_section = 4;
  std::fprintf(stderr, "section 4\n");
  // 4. stream readers / writers (the reference's test_stream.cpp shapes): a
  // file of alternating messages written by the reference is read back by
  // struct_pack::gpu::deserialize(ifstream) and the other way round; the two
  // files are byte for byte equal; a cut file is no_buffer_space on both
  {
    const std::string f_ref = "/tmp/spk_stream_ref.bin", f_gpu = "/tmp/spk_stream_gpu.bin";
    std::vector<rpcb::person> ps;
    std::vector<ValidateRequest> vs;  // optionals: the whole-remainder read
    std::vector<std::vector<RecS>> bs;
    for (int i = 0; i < 20; ++i) {
      ps.push_back(make_person(S8, i, 16 + i));
      ValidateRequest v{};
      fill(v, 0x5EED001B, i, 8);
      vs.push_back(v);
      std::vector<RecS> b(50 + 100 * i);
      for (uint64_t j = 0; j < b.size(); ++j) b[j] = make_recs(S3, j + i, 48);
      bs.push_back(b);
    }
    {
      std::ofstream r(f_ref, std::ios::binary), g(f_gpu, std::ios::binary);
      for (int i = 0; i < 20; ++i) {
        struct_pack::serialize_to(r, ps[i]);
        struct_pack::serialize_to(r, vs[i]);
        struct_pack::serialize_to(r, bs[i]);
        struct_pack::gpu::serialize_to(g, ps[i]);
        struct_pack::gpu::serialize_to(g, vs[i]);
        struct_pack::gpu::serialize_to(g, bs[i]);
      }
    }
    std::ifstream a(f_ref, std::ios::binary), b(f_gpu, std::ios::binary);
    const std::string ra((std::istreambuf_iterator<char>(a)), std::istreambuf_iterator<char>());
    const std::string gb((std::istreambuf_iterator<char>(b)), std::istreambuf_iterator<char>());
    CHECK(!ra.empty() && ra == gb);
    std::ifstream gi(f_ref, std::ios::binary), ri(f_gpu, std::ios::binary);
    bool all = true;
    for (int i = 0; i < 20; ++i) {
      auto p = struct_pack::gpu::deserialize<rpcb::person>(gi);
      auto v = struct_pack::gpu::deserialize<ValidateRequest>(gi);
      std::vector<RecS> rb;
      auto e = struct_pack::gpu::deserialize_to(rb, gi);
      all = all && p.has_value() && p.value() == ps[i] && v.has_value() &&
            struct_pack::serialize<std::string>(v.value()) ==
                struct_pack::serialize<std::string>(vs[i]) &&
            !e && rb == bs[i];
      auto rp = struct_pack::deserialize<rpcb::person>(ri);
      auto rv = struct_pack::deserialize<ValidateRequest>(ri);
      auto rr = struct_pack::deserialize<std::vector<RecS>>(ri);
      all = all && rp.has_value() && rp.value() == ps[i] && rv.has_value() && rr.has_value() &&
            rr.value() == bs[i];
    }
    CHECK(all);
    CHECK(static_cast<std::size_t>(gi.tellg()) == ra.size());
    // get_field from a stream (test_stream.cpp:91-138)
    std::ifstream gf(f_ref, std::ios::binary);
    auto name = struct_pack::gpu::get_field<rpcb::person, 1>(gf);
    CHECK(name.has_value() && name.value() == ps[0].name);
    std::string name2;
    std::ifstream gf2(f_ref, std::ios::binary);
    auto fe = struct_pack::gpu::get_field_to<rpcb::person, 1>(name2, gf2);
    CHECK(!fe && name2 == ps[0].name);
    // a file cut short (test_stream.cpp:206-224): no_buffer_space on both
    {
      std::vector<std::string> data = {"Hello", "Hi", "Hey", "Hoo"};
      auto buf = struct_pack::serialize<std::string>(data);
      buf.resize(buf.size() - 5);
      std::ofstream(f_ref, std::ios::binary).write(buf.data(), buf.size());
      std::ifstream x(f_ref, std::ios::binary), y(f_ref, std::ios::binary);
      std::vector<std::string> d1, d2;
      auto e1 = struct_pack::deserialize_to(d1, x);
      auto e2 = struct_pack::gpu::deserialize_to(d2, y);
      CHECK(e1 == struct_pack::errc::no_buffer_space && e2 == struct_pack::errc::no_buffer_space);
    }
    // a 2 MiB string cut to 16 bytes and to 2 MiB - 10000 (test_stream.cpp:226-261)
    for (std::size_t cut : {std::size_t(16), std::size_t(2 * 1024 * 1024 - 10000)}) {
      auto buf = struct_pack::serialize<std::string>(std::string(2 * 1024 * 1024, 'A'));
      buf.resize(cut);
      std::ofstream(f_ref, std::ios::binary).write(buf.data(), buf.size());
      std::ifstream y(f_ref, std::ios::binary);
      std::string d;
      CHECK(struct_pack::gpu::deserialize_to(d, y) == struct_pack::errc::no_buffer_space);
    }
    // the whole 2 MiB string message and one record after it
    {
      std::ofstream o(f_gpu, std::ios::binary);
      struct_pack::serialize_to(o, std::string(2 * 1024 * 1024 + 5, 'B'));
      struct_pack::serialize_to(o, ps[3]);
    }
    std::ifstream y(f_gpu, std::ios::binary);
    std::string big;
    CHECK(!struct_pack::gpu::deserialize_to(big, y) && big == std::string(2 * 1024 * 1024 + 5, 'B'));
    auto p3 = struct_pack::gpu::deserialize<rpcb::person>(y);
    CHECK(p3.has_value() && p3.value() == ps[3]);
    std::remove(f_ref.c_str());
    std::remove(f_gpu.c_str());
  }
  g_section = 5;
  std::fprintf(stderr, "section 5\n");
  // 5. unique_ptr and trivial_view members, next to the reference
  {
    auto mk = [&](int i) {
      UPtrRec u;
      u.id = i * 3 - 7;
      if (i % 3) u.s = std::make_unique<std::string>(std::string(i % 17, (char)('a' + i % 26)));
      if (i % 2) u.p = std::make_unique<Inner>(Inner{i, 0.5f * i});
      if (i % 5 != 1) u.v = std::make_unique<std::vector<int32_t>>(std::vector<int32_t>(i % 9, i));
      if (i % 4 == 0) u.r = std::make_unique<RecS>(make_recs(S3, i, 20));
      return u;
    };
    auto same = [](const UPtrRec &a, const UPtrRec &b) {
      auto eq = [](const auto &x, const auto &y) { return (!x && !y) || (x && y && *x == *y); };
      return a.id == b.id && eq(a.s, b.s) && eq(a.p, b.p) && eq(a.v, b.v) && eq(a.r, b.r);
    };
    bool ok = true;
    for (int i = 0; i < 12; ++i) {
      const UPtrRec u = mk(i);
      const auto want = struct_pack::serialize<std::string>(u);
      ok = ok && struct_pack::gpu::serialize<std::string>(u) == want;
      auto back = struct_pack::gpu::deserialize<UPtrRec>(want);
      ok = ok && back.has_value() && same(back.value(), u);
    }
    CHECK(ok);
    std::vector<UPtrRec> batch;
    for (int i = 0; i < 3000; ++i) batch.push_back(mk(i));
    const auto want = struct_pack::serialize<std::string>(batch);
    CHECK(struct_pack::gpu::serialize<std::string>(batch) == want);
    std::vector<UPtrRec> back;
    CHECK(!struct_pack::gpu::deserialize_to(back, want) && back.size() == batch.size());
    bool all = back.size() == batch.size();
    for (std::size_t i = 0; all && i < back.size(); ++i) all = same(back[i], batch[i]);
    CHECK(all);
    // a truncated message: the reference's errc
    std::vector<UPtrRec> b2;
    auto cut = std::string_view(want).substr(0, want.size() - 5);
    auto e1 = struct_pack::gpu::deserialize_to(b2, cut);
    std::vector<UPtrRec> b3;
    auto e2 = struct_pack::deserialize_to(b3, cut);
    CHECK(e1.val() == e2.val());
    // a unique_ptr as the whole message
    auto up = std::make_unique<Inner>(Inner{4, 2.5f});
    CHECK(struct_pack::gpu::serialize<std::string>(up) == struct_pack::serialize<std::string>(up));
  }
  {
    ViewData d{{1, 2, 3, 4, 5, 6}, 7.5};
    ViewRec v{"viewed", d, 42};
    PlainRec pl{"viewed", d, 42};
    const auto want = struct_pack::serialize<std::string>(v);
    CHECK(want == struct_pack::serialize<std::string>(pl));
    CHECK(struct_pack::gpu::serialize<std::string>(v) == want);
    auto back = struct_pack::gpu::deserialize<ViewRec>(want);
    CHECK(back.has_value() && back->name == "viewed" && back->k == 42 &&
          back->data.get().a == d.a && back->data.get().d == d.d);
    auto plain = struct_pack::gpu::deserialize<PlainRec>(want);  // the same bytes as T
    CHECK(plain.has_value() && plain->data.a == d.a);
  }
  g_section = 6;
  std::fprintf(stderr, "section 6\n");
  // 6. user helpers (user_helper.hpp:16-85) next to the reference's
  {
    str_writer rw, gw;
    const std::string name = "a user-defined type";
    const std::vector<int32_t> vals = {1, -2, 3, 40000};
    const std::vector<std::string> strs = {"x", "", "yy"};
    std::vector<RecS> rs;
    for (int i = 0; i < 500; ++i) rs.push_back(make_recs(S3, i, 30));
    const std::array<Inner, 3> in = {Inner{1, 1.f}, Inner{2, 2.f}, Inner{3, 3.f}};
    struct_pack::write(rw, name);
    struct_pack::write(rw, vals);
    struct_pack::write<4>(rw, strs);
    struct_pack::write(rw, in.data(), in.size());
    struct_pack::write(rw, rs.data(), rs.size());
    struct_pack::gpu::write(gw, name);
    struct_pack::gpu::write(gw, vals);
    struct_pack::gpu::write<4>(gw, strs);
    struct_pack::gpu::write(gw, in.data(), in.size());
    struct_pack::gpu::write(gw, rs.data(), rs.size());
    CHECK(!rw.buf.empty() && gw.buf == rw.buf);
    CHECK(struct_pack::gpu::get_write_size(name) == struct_pack::get_write_size(name));
    CHECK(struct_pack::gpu::get_write_size<4>(strs) == struct_pack::get_write_size<4>(strs));
    CHECK(struct_pack::gpu::get_write_size(rs.data(), rs.size()) ==
          struct_pack::get_write_size(rs.data(), rs.size()));
    std::istringstream is(rw.buf);
    std::string n2;
    std::vector<int32_t> v2;
    std::vector<std::string> s2;
    std::array<Inner, 3> i2{};
    std::vector<RecS> r2(rs.size());
    CHECK(!struct_pack::gpu::read(is, n2) && n2 == name);
    CHECK(!struct_pack::gpu::read(is, v2) && v2 == vals);
    CHECK(!struct_pack::gpu::read<4>(is, s2) && s2 == strs);
    CHECK(!struct_pack::gpu::read(is, i2.data(), i2.size()) && i2 == in);
    CHECK(!struct_pack::gpu::read(is, r2.data(), r2.size()) && r2 == rs);
    CHECK(static_cast<std::size_t>(is.tellg()) == rw.buf.size());
    std::istringstream cut(rw.buf.substr(0, 5));
    std::string n3;
    CHECK(struct_pack::gpu::read(cut, n3) == struct_pack::errc::no_buffer_space);
  }
  g_section = 7;
  std::fprintf(stderr, "section 7\n");
  // 7. the opt-in types (__int128, std::bitset, wchar_t, u16string / u32string /
  // wstring; this binary is built with the reference's macros for them)
  {
    std::vector<Wide> ws(2500);
    for (std::size_t i = 0; i < ws.size(); ++i) spk_gold::fill(ws[i], 0x5EED0023, i, 24);
    const auto want = struct_pack::serialize<std::string>(ws);
    CHECK(struct_pack::gpu::serialize<std::string>(ws) == want);
    std::vector<Wide> back;
    CHECK(!struct_pack::gpu::deserialize_to(back, want) && back.size() == ws.size());
    CHECK(struct_pack::serialize<std::string>(back) == want);  // every member came back
    bool ok = back.size() == ws.size();
    for (std::size_t i = 0; ok && i < ws.size(); ++i)
      ok = back[i].a == ws[i].a && back[i].c == ws[i].c && back[i].big == ws[i].big &&
           back[i].bits == ws[i].bits && back[i].t.b == ws[i].t.b;
    CHECK(ok);
    Wide one;
    spk_gold::fill(one, 7, 3, 40);
    const auto w1 = struct_pack::serialize<std::string>(one);
    CHECK(struct_pack::gpu::serialize<std::string>(one) == w1);
    auto b1 = struct_pack::gpu::deserialize<Wide>(w1);
    CHECK(b1.has_value() && struct_pack::serialize<std::string>(b1.value()) == w1);
    std::vector<WideT> ts(4000);
    for (std::size_t i = 0; i < ts.size(); ++i) spk_gold::fill(ts[i], 0x5EED0022, i, 0);
    const auto wt = struct_pack::serialize<std::string>(ts);
    CHECK(struct_pack::gpu::serialize<std::string>(ts) == wt);
    std::vector<WideT> tb;
    CHECK(!struct_pack::gpu::deserialize_to(tb, wt) && struct_pack::serialize<std::string>(tb) == wt);
    const std::u32string u = U"wide \U0001F600 chars";
    CHECK(struct_pack::gpu::serialize<std::string>(u) == struct_pack::serialize<std::string>(u));
    auto ub = struct_pack::gpu::deserialize<std::u32string>(struct_pack::serialize<std::string>(u));
    CHECK(ub.has_value() && ub.value() == u);
  }
  g_section = 8;
  std::fprintf(stderr, "section 8\n");
  // 8. view arguments alias the request buffer (the reference's views point
  // into the buffer coro_rpc keeps alive for the call, unpacker.hpp:1135-1145):
  // a handler holding a std::string_view across a second decode of the same
  // type on this thread (a suspended coroutine handler) still sees its bytes
  {
    struct VArg {
      int32_t id;
      std::string_view name;
      std::vector<std::string_view> tags;
    };
    const std::string r1 = struct_pack::serialize<std::string>(
        VArg{1, "first request", {"a", "bb"}});
    const std::string r2 = struct_pack::serialize<std::string>(
        VArg{2, "second, longer request", {"ccc", "dddd", "e"}});
    std::tuple<VArg> a1, a2;
    CHECK(struct_pack_gpu_protocol::deserialize_to(a1, r1));
    CHECK(struct_pack_gpu_protocol::deserialize_to(a2, r2));  // same type, same thread
    const VArg &v1 = std::get<0>(a1), &v2 = std::get<0>(a2);
    CHECK(v1.id == 1 && v1.name == "first request" && v1.tags.size() == 2 &&
          v1.tags[0] == "a" && v1.tags[1] == "bb");
    CHECK(v2.id == 2 && v2.name == "second, longer request" && v2.tags.size() == 3 &&
          v2.tags[2] == "e");
    CHECK(v1.name.data() >= r1.data() && v1.name.data() + v1.name.size() <= r1.data() + r1.size());
    CHECK(v2.tags[1].data() >= r2.data() && v2.tags[1].data() < r2.data() + r2.size());
    // the same from the front end: a view of a vector message aliases the input
    std::vector<VArg> many;
    for (int i = 0; i < 300; ++i) many.push_back(VArg{i, i % 2 ? "odd" : "even", {"x"}});
    const std::string rm = struct_pack::serialize<std::string>(many);
    std::vector<VArg> back;
    CHECK(!struct_pack::gpu::deserialize_to(back, rm) && back.size() == many.size());
    bool ok = back.size() == many.size();
    for (std::size_t i = 0; ok && i < back.size(); ++i)
      ok = back[i].id == (int)i && back[i].name == many[i].name && back[i].tags[0] == "x" &&
           back[i].name.data() >= rm.data() && back[i].name.data() < rm.data() + rm.size();
    CHECK(ok);
    auto f = struct_pack::gpu::get_field<VArg, 1>(r2);
    CHECK(f.has_value() && f.value() == "second, longer request" && f.value().data() > r2.data() &&
          f.value().data() < r2.data() + r2.size());
  }
  // 9. small-call latency of the protocol (no size threshold: every payload
  // takes the GPU): add(int, int) and echo_person through the reference's
  // executor, per call, next to the reference's CPU protocol
  {
    auto time_calls = [](auto fn, int n) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; ++i) fn();
      return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                 .count() / n;
    };
    std::string req;
    struct_pack::serialize_to(req, 40, 2);
    const std::string preq = struct_pack::serialize<std::string>(make_person(S8, 5, 40));
    const int n = 300;
    (void)run<add, struct_pack_gpu_protocol>(req);  // warm the codec and the device
    (void)run<echo_person, struct_pack_gpu_protocol>(preq);
    const double g_add = time_calls([&] { (void)run<add, struct_pack_gpu_protocol>(req); }, n);
    const double r_add = time_calls([&] { (void)run<add, struct_pack_protocol>(req); }, n);
    const double g_p = time_calls([&] { (void)run<echo_person, struct_pack_gpu_protocol>(preq); }, n);
    const double r_p = time_calls([&] { (void)run<echo_person, struct_pack_protocol>(preq); }, n);
    std::fprintf(stderr,
                 "small-call latency (us per call): add gpu %.1f ref %.2f; echo_person gpu %.1f "
                 "ref %.2f\n", g_add, r_add, g_p, r_p);
    std::printf("{\"small_call_us\": {\"add_gpu\": %.2f, \"add_ref\": %.3f, "
                "\"echo_person_gpu\": %.2f, \"echo_person_ref\": %.3f}}\n",
                g_add, r_add, g_p, r_p);
  }
  std::printf("{\"checks\": %d, \"failures\": %d}\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
