// GPU: the C++20 front end end-to-end through the HIP codec, checked against
// the REFERENCE's own bytes (tests/golden/*.bin written by golden_gen built
// from /root/reference). Reads like the reference's doctest suites
// (src/struct_pack/tests/test_serialize.cpp): serialize -> compare bytes,
// deserialize -> compare objects, truncated / corrupted buffers -> errc.
#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <variant>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "ylt/struct_pack_gpu.hpp"
#include "../../oracle/ref/types.hpp"

// the GPU front end's names; compiled both standalone and next to the
// reference header (then errc / sp_config / var_int*_t are the reference's)
using namespace struct_pack::gpu;
using struct_pack::errc;
using struct_pack::sp_config;
static int g_fail = 0, g_checks = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    ++g_checks;                                                         \
    if (!(c)) {                                                         \
      ++g_fail;                                                         \
      std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
    }                                                                   \
  } while (0)

static std::string golden(const std::string &name) {
  std::ifstream f(std::string(SPK_GOLDEN_DIR) + "/" + name, std::ios::binary);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
static std::vector<uint64_t> golden_lens(const std::string &name) {
  std::string b = golden(name);
  std::vector<uint64_t> v(b.size() / 8);
  std::memcpy(v.data(), b.data(), b.size());
  return v;
}

bool operator==(const Rec64 &a, const Rec64 &b) { return std::memcmp(&a, &b, sizeof a) == 0; }
bool operator==(const RecS &a, const RecS &b) { return a.id == b.id && a.name == b.name && a.v == b.v; }
bool operator==(const Inner &a, const Inner &b) { return a.x == b.x && a.y == b.y; }
bool operator==(const Outer &a, const Outer &b) { return a.key == b.key && a.items == b.items; }
bool operator==(const Pad &a, const Pad &b) { return a.a == b.a && a.b == b.b && a.c == b.c; }
bool operator==(const Opt &a, const Opt &b) {
  return a.id == b.id && a.score == b.score && a.tag == b.tag && a.pad == b.pad;
}
namespace rpcb {
bool operator==(const point &a, const point &b) { return a.x == b.x && a.y == b.y; }
bool operator==(const rect &a, const rect &b) { return std::memcmp(&a, &b, sizeof a) == 0; }
bool operator==(const person &a, const person &b) {
  return a.id == b.id && a.name == b.name && a.age == b.age && a.salary == b.salary;
}
}  // namespace rpcb
bool operator==(const OptP &a, const OptP &b) { return a.k == b.k && a.a == b.a && a.b == b.b; }
bool operator==(const Var &a, const Var &b) {
  return a.a == b.a && a.s == b.s && a.b == b.b && a.d == b.d && a.c == b.c && a.e == b.e;
}
bool operator==(const VarP &a, const VarP &b) { return a.id == b.id && a.x == b.x && a.y == b.y; }

// structural equality through the front end's own reflection (records,
// containers, optionals, variants, compatibles), for the record types with
// no operator==
template <typename T>
static bool same(const T &a, const T &b) {
  namespace d = struct_pack::gpu::detail;
  using U = d::remove_cvref_t<T>;
  if constexpr (d::is_fundamental_v<U> || d::is_string_v<U> || d::is_monostate_v<U>) {
    return a == b;
  } else if constexpr (d::is_varint_v<U>) {
    return typename d::varint_traits<U>::value_type(a) == typename d::varint_traits<U>::value_type(b);
  } else if constexpr (d::is_std_optional<U>::value || d::is_compat_v<U>) {
    return a.has_value() == b.has_value() && (!a.has_value() || same(*a, *b));
  } else if constexpr (d::is_std_variant<U>::value) {
    return a.index() == b.index() &&
           std::visit([&](const auto &x) {
             return same(x, *std::get_if<d::remove_cvref_t<decltype(x)>>(&b));
           }, a);
  } else if constexpr (d::is_container_v<U> || d::is_std_array<U>::value) {
    if (a.size() != b.size()) return false;
    auto i = a.begin();
    auto j = b.begin();
    for (; i != a.end(); ++i, ++j)
      if (!same(*i, *j)) return false;
    return true;
  } else if constexpr (d::is_std_pair<U>::value) {
    return same(a.first, b.first) && same(a.second, b.second);
  } else {
    auto ta = d::tie_members(const_cast<U &>(a));
    auto tb = d::tie_members(const_cast<U &>(b));
    return [&]<std::size_t... I>(std::index_sequence<I...>) {
      return (same(std::get<I>(ta), std::get<I>(tb)) && ...);
    }(std::make_index_sequence<std::tuple_size_v<decltype(ta)>>{});
  }
}

// A vector message of a nested record type (ARRAY / VARIANT / OPTGROUP /
// CGROUP / FVAR layouts and the other container kinds) through the C++ front
// end: bytes == the reference's, decode == the records, and a truncated
// buffer / broken hash reported as the reference does. trunc / hash: whether
// the type's last member and head make those errc deterministic.
template <typename T, typename Gen>
static void roundtrip_nested(const char *fixture, std::size_t n, Gen gen, bool trunc = true,
                             bool hash = true) {
  std::vector<T> v(n);
  for (std::size_t i = 0; i < n; ++i) gen(v[i], i);
  const std::string want = golden(fixture);
  CHECK(!want.empty());
  auto sz = get_needed_size(v);
  CHECK(sz.size() == want.size());
  auto bytes = serialize<sp_config::DEFAULT, std::string>(v);
  CHECK(bytes == want);
  if (bytes != want) std::fprintf(stderr, "  %s: bytes differ (%zu vs %zu)\n", fixture,
                                  bytes.size(), want.size());
  std::vector<T> back;
  std::size_t consumed = 0;
  auto ec = deserialize_to(back, want.data(), want.size(), consumed);
  CHECK(!ec);
  CHECK(consumed == want.size());
  bool eq = back.size() == v.size();
  for (std::size_t i = 0; eq && i < n; ++i) eq = same(back[i], v[i]);
  CHECK(eq);
  if (!eq) std::fprintf(stderr, "  %s: decoded records differ\n", fixture);
  // the decoded objects re-encode to the same bytes
  CHECK((serialize<sp_config::DEFAULT, std::string>(back) == want));
  if (trunc && n) {
    std::vector<T> t;
    CHECK(deserialize_to(t, want.data(), want.size() - 1).ec == errc::no_buffer_space);
  }
  if (hash && n) {
    std::string bad = want;
    bad[1] ^= 0x40;
    std::vector<T> t2;
    CHECK(deserialize_to(t2, bad.data(), bad.size()).ec == errc::invalid_buffer);
  }
}

// check_trunc: a record type whose last member may be an optional value is
// exempt from the "one byte short -> no_buffer_space" check: the reference
// drops the value read's errc (unpacker.hpp:1271-1273; errs.json pins it)
template <typename T, typename Gen, bool check_trunc = true>
static void roundtrip_vector(const char *fixture, std::size_t n, Gen gen) {
  std::vector<T> v(n);
  for (std::size_t i = 0; i < n; ++i) gen(v[i], i);
  const std::string want = golden(fixture);
  CHECK(!want.empty());
  auto sz = get_needed_size(v);
  CHECK(sz.size() == want.size());
  auto bytes = serialize<sp_config::DEFAULT, std::string>(v);
  CHECK(bytes == want);
  std::vector<T> back;
  std::size_t consumed = 0;
  auto ec = deserialize_to(back, want.data(), want.size(), consumed);
  CHECK(!ec);
  CHECK(consumed == want.size());
  CHECK(back == v);
  // truncation: the reference reports no_buffer_space (test_serialize.cpp:816-845)
  if (check_trunc && want.size() > 5) {
    std::vector<T> t;
    auto e2 = deserialize_to(t, want.data(), want.size() - 1);
    CHECK(e2.ec == errc::no_buffer_space);
  }
  // hash mismatch -> invalid_buffer (test_serialize.cpp:529-547)
  std::string bad = want;
  bad[1] ^= 0x40;
  std::vector<T> t2;
  CHECK(deserialize_to(t2, bad.data(), bad.size()).ec == errc::invalid_buffer);
  auto r = deserialize<std::vector<T>>(want.data(), want.size());
  CHECK(r.has_value() && r.value() == v);
}

template <typename T, typename Gen>
static void roundtrip_messages(const char *fixture, const char *lens, std::size_t n, Gen gen) {
  std::vector<T> v(n);
  for (std::size_t i = 0; i < n; ++i) gen(v[i], i);
  const std::string want = golden(fixture);
  std::vector<uint64_t> offs;
  auto bytes = serialize_messages(v, offs);
  CHECK(std::string(bytes.begin(), bytes.end()) == want);
  auto l = golden_lens(lens);
  CHECK(offs.size() == n + 1);
  for (std::size_t i = 0; i < n && i < l.size(); ++i) CHECK(offs[i + 1] - offs[i] == l[i]);
  std::vector<T> back;
  auto errs = deserialize_messages(back, want.data(), want.size(), offs);
  bool all_ok = true;
  for (auto &e : errs) all_ok &= !e;
  CHECK(all_ok);
  CHECK(back == v);
}

// coro_rpc framing, against frames built by golden_gen the way coro_rpc does
template <typename T, typename Gen>
static void roundtrip_frames(const char *fixture, const char *lens, std::size_t n, bool req,
                             uint32_t fid, uint32_t seq, Gen gen) {
  std::vector<T> v(n);
  for (std::size_t i = 0; i < n; ++i) gen(v[i], i);
  const std::string want = golden(fixture);
  CHECK(!want.empty());
  const spk_frame f = req ? rpc_frame::request(fid, seq) : rpc_frame::response(seq);
  std::vector<uint64_t> offs;
  auto bytes = serialize_frames(v, f, offs);
  CHECK(std::string(bytes.begin(), bytes.end()) == want);
  auto l = golden_lens(lens);
  CHECK(offs.size() == n + 1);
  for (std::size_t i = 0; i < n && i < l.size(); ++i) CHECK(offs[i + 1] - offs[i] == l[i]);
  std::vector<T> back;
  auto errs = deserialize_frames(back, want.data(), want.size(), offs, f.prefix_len);
  bool all_ok = true;
  for (auto &e : errs) all_ok &= !e;
  CHECK(all_ok);
  CHECK(back == v);
}

static uint32_t fid_of(const char *name);

// A mixed batch in arrival order: reference-built request frames of rect and
// person interleaved (plus one frame of an unregistered id), routed by
// function id on the GPU, each type decoded where its frames lie, and the
// responses encoded with their requests' seq_num == the reference-built
// response frames.
template <typename T>
static std::vector<std::string> split_frames(const char *fixture, const char *lens) {
  const std::string w = golden(fixture);
  auto l = golden_lens(lens);
  std::vector<std::string> f;
  std::size_t p = 0;
  for (auto x : l) {
    f.push_back(w.substr(p, x));
    p += x;
  }
  return f;
}
static void routed_mixed_batch() {
  using namespace spk_gold;
  using rect_t = rpcb::rect;
  using person_t = rpcb::person;
  auto fr = split_frames<rect_t>("frames_rpcrect_req_n100_p0.bin", "frames_rpcrect_req_n100_p0.lens");
  auto fp = split_frames<person_t>("frames_person_req_n120_p48.bin",
                                   "frames_person_req_n120_p48.lens");
  CHECK(fr.size() == 100 && fp.size() == 120);
  std::string wire;
  std::vector<uint64_t> offs{0};
  std::vector<int> who;  // 0 rect, 1 person, 2 unknown id
  std::size_t ir = 0, ip = 0;
  for (std::size_t j = 0; ir < fr.size() || ip < fp.size(); ++j) {
    std::string f;
    if (j == 57) {
      f = fp[0];
      f[8] = 0x7F;  // an id no handler has
      who.push_back(2);
    } else if (ip >= fp.size() || (ir < fr.size() && (j * 7) % 11 < 5)) {
      f = fr[ir++];
      who.push_back(0);
    } else {
      f = fp[ip++];
      who.push_back(1);
    }
    wire += f;
    offs.push_back(wire.size());
  }
  const std::size_t n = who.size();
  void *s = nullptr;
  device::buffer dw(wire.size() + 16), doffs(offs.size() * 8);
  device::copy(dw.data(), wire.data(), wire.size(), SPK_COPY_H2D, s);
  device::copy(doffs.data(), offs.data(), offs.size() * 8, SPK_COPY_H2D, s);
  device::frame_router rt({fid_of("echo_rect"), fid_of("echo_person")}, n, s);
  auto counts = rt.route(dw.data(), wire.size(), (const uint64_t *)doffs.data(), n);
  CHECK(counts.size() == 3 && counts[0] == 100 && counts[1] == 120 && counts[2] == 1);
  // arrival order within each id (the stable partition)
  std::vector<uint64_t> idx(n);
  device::copy(idx.data(), rt.index(1), counts[1] * 8, SPK_COPY_D2H, s);
  device::sync(s);
  std::vector<uint64_t> want;
  for (std::size_t i = 0; i < n; ++i)
    if (who[i] == 1) want.push_back(i);
  CHECK(std::equal(want.begin(), want.end(), idx.begin()));
  auto check_type = [&](auto tag, std::size_t k, const char *resp_fixture, auto gen) {
    using T = typename decltype(tag)::type;
    auto &c = device::thread_codec<T, sp_config::DEFAULT>();
    auto b = c.alloc_for_wire(wire.size(), counts[k]);
    spk_dresult_t r = c.decode_frames(b, dw.data(), wire.size(), rt.begins(k), rt.ends(k),
                                      counts[k], rpc_frame::req_head_len);
    CHECK(r.errc == 0 && r.count == counts[k]);
    for (uint32_t q = 0; q < c.n_spans(); ++q) b.heap_elems[q] = r.heap_used[q];
    std::vector<T> got(counts[k]);
    c.download(b, counts[k], got.data());
    bool same = true;
    for (std::size_t i = 0; i < got.size(); ++i) same &= got[i] == gen(i);
    CHECK(same);
    // responses: the echo encode writes each request's seq_num
    b.n = counts[k];
    spk_plan_t p = c.plan(b, SPK_MODE_MESSAGES);
    const spk_frame f = rpc_frame::response(0);
    const std::size_t total = p.total_bytes + counts[k] * f.prefix_len;
    device::buffer out(total + 16);
    c.encode_framed_echo(b, f, dw.data(), rt.begins(k), 4, out.data(), out.size());
    std::string bytes(total, '\0');
    device::copy(bytes.data(), out.data(), total, SPK_COPY_D2H, s);
    device::sync(s);
    CHECK(bytes == golden(resp_fixture));
  };
  const uint64_t S7 = 0x5EED0007, S8 = 0x5EED0008;
  check_type(std::type_identity<rect_t>{}, 0, "frames_rpcrect_resp_n100_p0.bin",
             [&](std::size_t i) { return make_rpc_rect(S7, i); });
  check_type(std::type_identity<person_t>{}, 1, "frames_person_resp_n120_p48.bin",
             [&](std::size_t i) { return make_person(S8, i, 48); });
}

static uint32_t fid_of(const char *name) {  // frames.json function_id (MD5Hash32 of the name)
  std::ifstream f(std::string(SPK_GOLDEN_DIR) + "/frames.json");
  std::string js((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  auto p = js.find(std::string("\"function\": \"") + name + "\"");
  if (p == std::string::npos) return 0;
  p = js.find("\"function_id\": ", p);
  return (uint32_t)std::strtoul(js.c_str() + p + 15, nullptr, 10);
}

int main() {
  using namespace spk_gold;
  const uint64_t S2 = 0x5EED0002, S3 = 0x5EED0003, S4 = 0x5EED0004, S8 = 0x5EED0008;
  roundtrip_vector<Rec64>("rec64_A_n1000_p0_default.bin", 1000,
                          [&](Rec64 &o, uint64_t i) { o = make_rec64(S2, i); });
  roundtrip_vector<Rec64>("rec64_A_n255_p0_default.bin", 255,
                          [&](Rec64 &o, uint64_t i) { o = make_rec64(S2, i); });
  roundtrip_vector<RecS>("recs_A_n300_p48_default.bin", 300,
                         [&](RecS &o, uint64_t i) { o = make_recs(S3, i, 48); });
  roundtrip_vector<RecS>("recs_A_n40_p300_default.bin", 40,
                         [&](RecS &o, uint64_t i) { o = make_recs(S3, i, 300); });
  roundtrip_vector<Outer>("outer_A_n1000_p16_default.bin", 1000,
                          [&](Outer &o, uint64_t i) { o = make_outer(S4, i, 16); });
  roundtrip_vector<rpcb::person>("person_A_n100_p64_default.bin", 100,
                                 [&](rpcb::person &o, uint64_t i) { o = make_person(S8, i, 64); });
  // C1: benchmark rect<int> with ADL DISABLE_ALL_META_INFO (16,003 B)
  {
    std::vector<rect<int>> v(1000);
    auto bytes = serialize<sp_config::DEFAULT, std::string>(v);
    CHECK(bytes == golden("rect_A_n1000_p0_default.bin"));
    CHECK(bytes.size() == 16003);
    // the reference's other overloads: serialize<Buffer>(v), serialize(v)
    CHECK(serialize<std::string>(v) == bytes);
    const std::vector<char> vc = serialize(v);
    CHECK(std::string(vc.begin(), vc.end()) == bytes);
  }
  roundtrip_messages<RecS>("recs_B_n500_p300_default.bin", "recs_B_n500_p300_default.lens", 500,
                           [&](RecS &o, uint64_t i) { o = make_recs(S3, i, 300); });
  roundtrip_messages<Rec64>("rec64_B_n300_p0_default.bin", "rec64_B_n300_p0_default.lens", 300,
                            [&](Rec64 &o, uint64_t i) { o = make_rec64(S2, i); });
  const uint64_t S7 = 0x5EED0007, S9 = 0x5EED0009;
  roundtrip_frames<rpcb::rect>("frames_rpcrect_req_n100_p0.bin", "frames_rpcrect_req_n100_p0.lens",
                               100, true, fid_of("echo_rect"), 1,
                               [&](rpcb::rect &o, uint64_t i) { o = make_rpc_rect(S7, i); });
  roundtrip_frames<rpcb::person>("frames_person_resp_n120_p48.bin",
                                 "frames_person_resp_n120_p48.lens", 120, false, 0, 7,
                                 [&](rpcb::person &o, uint64_t i) { o = make_person(S8, i, 48); });
  roundtrip_frames<rpcb::person>("frames_person_req_n120_p48.bin",
                                 "frames_person_req_n120_p48.lens", 120, true,
                                 fid_of("echo_person"), 7,
                                 [&](rpcb::person &o, uint64_t i) { o = make_person(S8, i, 48); });
  CHECK(fid_of("array_1K_int") != 0);
  // std::optional members (SPK_OP_OPTION)
  const uint64_t SA = 0x5EED000A, SB = 0x5EED000B;
  auto gen_opt = [&](uint32_t p) { return [=](Opt &o, uint64_t i) { fill(o, SA, i, p); }; };
  auto gen_optp = [&](OptP &o, uint64_t i) { fill(o, SB, i, 0); };
  roundtrip_vector<Opt, decltype(gen_opt(16)), false>("opt_A_n300_p16_default.bin", 300,
                                                      gen_opt(16));
  roundtrip_vector<OptP, decltype(gen_optp), false>("optp_A_n300_p0_default.bin", 300, gen_optp);
  roundtrip_messages<Opt>("opt_B_n200_p300_default.bin", "opt_B_n200_p300_default.lens", 200,
                          gen_opt(300));
  roundtrip_messages<OptP>("optp_B_n200_p0_default.bin", "optp_B_n200_p0_default.lens", 200,
                           gen_optp);
  // varint members (SPK_OP_VARINT)
  const uint64_t SC = 0x5EED000C, SD = 0x5EED000D;
  auto gen_var = [&](uint32_t p) { return [=](Var &o, uint64_t i) { fill(o, SC, i, p); }; };
  auto gen_varp = [&](VarP &o, uint64_t i) { fill(o, SD, i, 0); };
  roundtrip_vector<Var>("var_A_n300_p16_default.bin", 300, gen_var(16));
  roundtrip_vector<VarP>("varp_A_n300_p0_default.bin", 300, gen_varp);
  roundtrip_messages<Var>("var_B_n200_p300_default.bin", "var_B_n200_p300_default.lens", 200,
                          gen_var(300));
  roundtrip_messages<VarP>("varp_B_n200_p0_default.bin", "varp_B_n200_p0_default.lens", 200,
                           gen_varp);
  routed_mixed_batch();
  // nested layouts through the C++ front end (make_spk_layout flattens ARRAY,
  // VARIANT, OPTGROUP, CGROUP, FVAR and the set / map / list containers)
  auto gen = [](uint64_t seed, uint32_t p) {
    return [=](auto &o, uint64_t i) { fill(o, seed, i, p); };
  };
  roundtrip_nested<Tags>("tags_A_n200_p6_default.bin", 200, gen(0x5EED000E, 6));
  roundtrip_nested<Tags>("tags_A_n30_p300_default.bin", 30, gen(0x5EED000E, 300));
  roundtrip_nested<Group>("group_A_n100_p5_default.bin", 100, gen(0x5EED000F, 5));
  roundtrip_nested<Deep>("deep_A_n100_p4_default.bin", 100, gen(0x5EED0010, 4));
  roundtrip_nested<Vnt>("vnt_A_n200_p6_default.bin", 200, gen(0x5EED0011, 6), false);
  roundtrip_nested<FV>("fv_A_n300_p8_default.bin", 300, gen(0x5EED0017, 8));
  roundtrip_nested<FVE>("fve_A_n300_p8_default.bin", 300, gen(0x5EED0018, 8));
  roundtrip_nested<FV32>("fv32_A_n300_p0_default.bin", 300, gen(0x5EED0019, 0));
  roundtrip_nested<EV>("ev_A_n300_p8_default.bin", 300, gen(0x5EED001A, 8));
  roundtrip_nested<ValidateRequest>("valreq_A_n300_p16_default.bin", 300, gen(0x5EED001B, 16),
                                    false);
  roundtrip_nested<CmpG>("cmpg_A_n200_p8_default.bin", 200, gen(0x5EED001D, 8), false);
  roundtrip_nested<Monster>("monster_A_n300_p20_default.bin", 300, gen(0x5EED001E, 20));
  roundtrip_nested<Monster>("monster_A_n40_p300_default.bin", 40, gen(0x5EED001E, 300));
  // vector<rect2<int32_t>>: DISABLE_ALL_META_INFO, no hash to break
  roundtrip_nested<rect2<int32_t>>("rect2_A_n300_p0_default.bin", 300, gen(0x5EED001F, 0), true,
                                   false);
  roundtrip_nested<Lists>("lists_A_n200_p6_default.bin", 200, gen(0x5EED0020, 6));
  roundtrip_nested<Maps>("maps_A_n200_p0_default.bin", 200, gen(0x5EED0021, 0));
  std::printf("{\"checks\": %d, \"failures\": %d}\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
