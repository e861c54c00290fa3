// Record types and the seeded input generator shared by the golden generator
// (golden_gen.cpp) and the reference CPU baseline (ref_bench.cpp).
//
// TEST INFRASTRUCTURE ONLY. These translation units are compiled against the
// read-only reference headers under /root/reference/include (see
// oracle/Makefile); their binaries land in oracle/_ref/ and are never linked
// into the product library.
//
// The generator formula is restated bit-for-bit in
//   * yalantinglibs_amd/csrc/spk_synth.hip (device generator used at full size)
//   * yalantinglibs_amd/synth.py (numpy, small sizes)
// so that the GPU box can regenerate the exact same inputs from a seed.
#pragma once
#include <array>
#include <bitset>
#include <cstdint>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <optional>
#include <set>
#include <unordered_map>
#include <string>
#include <variant>
#include <vector>

// ---- varint members: LEB128, zigzag for var_int* --
struct Var {  // a varint first: no count field to screen candidates on
  struct_pack::var_int32_t a;
  std::string s;
  struct_pack::var_uint64_t b;
  double d;
  struct_pack::var_int64_t c;
  struct_pack::var_uint32_t e;
};

// varints and fixed members only: no container, no span
struct VarP {
  int32_t id;
  struct_pack::var_int64_t x;
  struct_pack::var_uint32_t y;
};

namespace spk_gold {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
// counter-based: word k (0..63) of record i
inline uint64_t rnd(uint64_t seed, uint64_t i, uint64_t k) {
  return mix64(seed + (i * 64 + k + 1) * 0x9E3779B97F4A7C15ULL);
}
inline float rf(uint64_t r) { return (float)(int32_t)(uint32_t)r / 65536.0f; }
inline double rd(uint64_t r) { return (double)(int32_t)(uint32_t)r / 65536.0; }

}  // namespace spk_gold

// ---- C2: 64-byte fixed-width POD ---------------------------------------
struct Rec64 {
  int32_t i0, i1, i2, i3;
  float f0, f1, f2, f3;
  double d0, d1, d2, d3;
};
static_assert(sizeof(Rec64) == 64);

// ---- C3: one std::string field -----------------------------------------
struct RecS {
  int32_t id;
  std::string name;
  double v;
};

// ---- C4: nested vector of trivially-copyable inner records -------------
struct Inner {
  int32_t x;
  float y;
};
struct Outer {
  int64_t key;
  std::vector<Inner> items;
};

// ---- padding / mixed-member coverage -----------------------------------
struct Pad {  // trivially serializable, 12 bytes with 3+0+2 padding bytes
  int8_t a;
  int32_t b;
  int16_t c;
};
struct Mixed {  // non-trivial: raw Pad (with padding), raw array, two spans
  Pad p;
  int64_t k;
  std::array<int16_t, 3> arr;
  std::string s;
  std::vector<int32_t> v;
};

// ---- optional members: [has_value:1][value?] -----
struct Opt {  // optional first member (no screening byte for the walker)
  int32_t id;
  std::optional<double> score;
  std::string tag;
  std::optional<Pad> pad;  // trivially serializable value incl. padding
};

// ---- C1: src/struct_pack/benchmark/data_def.hpp rect<int> --------------
template <typename T>
struct rect {
  T x = 1;
  T y = 0;
  T width = 11;
  T height = 1;
};
inline constexpr struct_pack::sp_config set_sp_config(rect<int> *) {
  return struct_pack::DISABLE_ALL_META_INFO;
}
inline constexpr struct_pack::sp_config set_sp_config(
    std::vector<rect<int>> *) {
  return struct_pack::DISABLE_ALL_META_INFO;
}

// ---- C5: coro_rpc benchmark payload shapes ------------------------------
namespace rpcb {
struct point {
  double x, y;
};
struct rect {
  point p1, p2;
};
struct person {  // src/struct_pack/benchmark/data_def.hpp person
  int32_t id;
  std::string name;
  int age;
  double salary;
};
// coro_rpc req_header (include/ylt/coro_rpc/impl/protocol/coro_rpc_protocol.hpp:60-68)
struct req_header {
  uint8_t magic;
  uint8_t version;
  uint8_t serialize_type;
  uint8_t msg_type;
  uint32_t seq_num;
  uint32_t function_id;
  uint32_t length;
  uint32_t attach_length;
};
struct resp_header {
  uint8_t magic;
  uint8_t version;
  uint8_t err_code;
  uint8_t msg_type;
  uint32_t seq_num;
  uint32_t length;
  uint32_t attach_length;
};
}  // namespace rpcb

// only optional members: no container, so no metainfo byte per message
struct OptP {
  int64_t k;
  std::optional<int32_t> a;
  std::optional<rpcb::point> b;
};

// ---- containers of non-trivially-serializable elements (SPK_OP_ARRAY) ----
struct Tags {  // vector<string>
  int32_t id;
  std::vector<std::string> tags;
  double w;
};
struct Group {  // vector<struct with a string>, then a string
  int64_t gid;
  std::vector<RecS> members;
  std::string label;
};
struct Deep {  // two nesting levels: vector<vector<string>>
  uint16_t k;
  std::vector<std::vector<std::string>> m;
};

// ---- alignment overrides (ref alignment.hpp:72-122, tests/test_alignas.cpp) --
struct alignas(8) Al8 {  // alignas on a trivially serializable struct: 8 B
  char a;
  short b;
};
struct alignas(4) AlA {
  char a;
  short b;
};
struct alignas(8) AlB {
  char a;
  int b;
};
struct alignas(16) AlOuter {  // nesting: pack_alignment 8, alignment 16
  AlA a;
  AlB b;
};
#pragma pack(push, 1)
struct Packed {  // #pragma pack(1) + struct_pack::pack_alignment_v = 1
  char a;
  int32_t b;
  int16_t c;
};
#pragma pack(pop)
template <>
constexpr inline std::size_t struct_pack::pack_alignment_v<Packed> = 1;
struct AlRec {  // non-trivial record holding aligned / packed members verbatim
  AlOuter o;
  std::string s;
  Packed p;
  Al8 e;
};

// ---- std::variant members (SPK_OP_VARIANT) ----------------------------
struct Vnt {
  int32_t id;
  std::variant<int32_t, double, std::string, Inner> v;
  std::variant<std::monostate, std::vector<int32_t>> w;
  std::vector<std::variant<int64_t, std::string>> list;
};

// ---- struct_pack::compatible<T, version> members (SPK_OP_COMPAT) --------
// Cmp is the record; CmpOld is an older writer without the compatible members
// and CmpNew a newer one with an extra version: all three share one type
// code (compatible members are not in the literal).
struct Cmp {
  int32_t id;
  struct_pack::compatible<int64_t, 20210101> a;
  std::string name;
  struct_pack::compatible<double, 20240101> c;
  struct_pack::compatible<int16_t, 20210101> b;
};
struct CmpOld {
  int32_t id;
  std::string name;
};
struct CmpNew {
  int32_t id;
  struct_pack::compatible<int64_t, 20210101> a;
  std::string name;
  struct_pack::compatible<double, 20240101> c;
  struct_pack::compatible<int16_t, 20210101> b;
  struct_pack::compatible<int32_t, 20250101> d;
};
// ---- sp_config varint encodings of the record (reflection.hpp:53-60) ------
// USE_FAST_VARINT: [bitset: non-zero flags + 2 width bits][non-zero varints at
// one width] before the other members (packer.hpp:200-235);
// ENCODING_WITH_VARINT: plain int32/64 and uint32/64 members are varints
// (reflection.hpp:843), LEB128 without zigzag.
struct FV {
  struct_pack::var_int32_t a;
  std::string s;
  struct_pack::var_uint64_t b;
  double d;
  struct_pack::var_int64_t c;
  struct_pack::var_uint32_t e;
};
constexpr struct_pack::sp_config set_sp_config(FV *) {
  return struct_pack::sp_config::USE_FAST_VARINT;
}
struct FVE {
  int32_t a;
  std::string s;
  uint64_t b;
  double d;
  int64_t c;
  uint32_t e;
  int16_t f;
};
constexpr struct_pack::sp_config set_sp_config(FVE *) {
  return static_cast<struct_pack::sp_config>(struct_pack::sp_config::ENCODING_WITH_VARINT |
                                             struct_pack::sp_config::USE_FAST_VARINT);
}
struct FV32 {  // 32-bit varints only: width code 3 is invalid_buffer on decode
  struct_pack::var_uint32_t a;
  int16_t x;
  struct_pack::var_int32_t b;
};
constexpr struct_pack::sp_config set_sp_config(FV32 *) {
  return struct_pack::sp_config::USE_FAST_VARINT;
}
struct EV {
  int32_t a;
  std::string s;
  uint64_t b;
  int64_t c;
  uint32_t e;
};
constexpr struct_pack::sp_config set_sp_config(EV *) {
  return struct_pack::sp_config::ENCODING_WITH_VARINT;
}

// ---- std::optional / expected / compatible of values that are not trivially
// serializable (SPK_OP_OPTGROUP / SPK_OP_CGROUP) ---------------------------
// the coro_rpc benchmark's request type, member for member as declared in
// src/coro_rpc/benchmark/api/ValidateRequest.h
struct ResponseCode {
  int32_t retcode;
  std::optional<std::string> error_message;
};
struct AliMessage {
  int32_t message_type;
  std::optional<std::string> session_no;
  std::optional<bool> tint_flag;
  std::optional<uint32_t> source_entity;
  std::optional<uint32_t> dest_entity;
  std::optional<std::string> client_ip;
  std::optional<ResponseCode> rc;
  std::optional<int32_t> version;
};
struct ValidateRequest {
  AliMessage msg;
  std::optional<int32_t> job_id;
  std::vector<std::string> query_keys;
  std::optional<bool> clean;
};
// struct_pack::expected<T, E> members (packer.hpp:400-410); the standalone
// C++ front end (no reference on the include path) has no expected<T, E>
#if !defined(SPK_GPU_WITH_REFERENCE) || SPK_GPU_WITH_REFERENCE
#define SPK_TYPES_HAVE_EXPECTED 1
struct Exp {
  int32_t id;
  struct_pack::expected<std::string, int32_t> r;
  struct_pack::expected<Inner, std::string> q;
  std::optional<std::vector<std::string>> l;
  struct_pack::expected<int64_t, ResponseCode> e;
};
#endif
// compatible<U, ver> with U not trivially serializable, beside a trivial one
struct CmpG {
  int32_t id;
  struct_pack::compatible<std::string, 20230101> note;
  std::string name;
  struct_pack::compatible<std::vector<int32_t>, 20230101> ints;
  struct_pack::compatible<Inner, 20240101> in;
  struct_pack::compatible<ResponseCode, 20240101> rc;
};

// ---- the reference benchmark's shapes (src/struct_pack/benchmark/data_def.hpp)
enum Color : uint8_t { Red, Green, Blue };
struct Vec3 {
  float x, y, z;
};
struct Weapon {
  std::string name;
  int16_t damage;
};
struct Monster {
  Vec3 pos;
  int16_t mana;
  int16_t hp;
  std::string name;
  std::string inventory;
  Color color;
  std::vector<Weapon> weapons;
  Weapon equipped;
  std::vector<Vec3> path;
};
template <typename T>
struct rect2 {
  T x, y, width, height;
};
inline constexpr struct_pack::sp_config set_sp_config(rect2<int32_t> *) {
  return struct_pack::sp_config{struct_pack::sp_config::DISABLE_ALL_META_INFO |
                                struct_pack::sp_config::USE_FAST_VARINT |
                                struct_pack::sp_config::ENCODING_WITH_VARINT};
}
inline constexpr struct_pack::sp_config set_sp_config(std::vector<rect2<int32_t>> *) {
  return struct_pack::sp_config{struct_pack::DISABLE_ALL_META_INFO};
}

// ---- the other container kinds (reflection.hpp:328-350): list / deque are
// container_t like vector; set_container_t / map_container_t hold their keys /
// pairs in the container's order ----------------------------------------------
struct Lists {
  int32_t id;
  std::list<std::string> names;
  std::deque<int32_t> vals;
  std::list<Inner> pts;
};
struct Maps {
  int32_t id;
  std::map<int32_t, std::string> m;
  std::set<std::string> s;
  std::multimap<int64_t, Inner> mm;  // pair<const int64_t, Inner>: 16 raw bytes
  std::multiset<int32_t> ms;
  std::map<std::string, RecS> mr;
};

// A mirror of complicated_object (src/struct_pack/tests/test_struct.hpp:17-103),
// the type of the reference's own binary goldens (tests/binary_data/
// test_cross_platform*.dat): same member types in the same order, so the same
// type literal, code and bytes.
namespace cpx {
struct person {
  int age;
  std::string name;
};
enum class Color { red, black, white };
struct trivial_one {
  int a;
  double b;
  float c;
};
struct complicated_object {
  Color color;
  int a;
  std::string b;
  std::vector<person> c;
  std::list<std::string> d;
  std::deque<int> e;
  std::map<int, person> f;
  std::multimap<int, person> g;
  std::set<std::string> h;
  std::multiset<int> i;
  std::unordered_map<int, person> j;
  std::unordered_multimap<int, int> k;
  std::array<person, 2> m;
  person n[2];
  std::pair<std::string, person> o;
  std::vector<std::array<trivial_one, 2>> p;
};
}  // namespace cpx

// ---- the reference's opt-in types (built with STRUCT_PACK_ENABLE_INT128 and
// STRUCT_PACK_ENABLE_UNPORTABLE_TYPE, as its own tests are): 128-bit
// integers, std::bitset, wchar_t, and the char16_t / char32_t strings
struct WideT {  // trivially serializable: raw bytes with padding
  __int128 a;
  std::bitset<64> bits;
  char32_t c32;
  wchar_t wc;
  char16_t c16;
  unsigned __int128 b;
};
struct Wide {
  int32_t id;
  std::u16string a;
  __int128 big;
  std::u32string b;
  std::bitset<128> bits;
  std::wstring c;
  unsigned __int128 ubig;
  wchar_t wc;
  char16_t c16;
  WideT t;
};

template <typename T>
constexpr bool kHasCompat = false;
template <>
inline constexpr bool kHasCompat<Cmp> = true;
template <>
inline constexpr bool kHasCompat<CmpNew> = true;
template <>
inline constexpr bool kHasCompat<CmpG> = true;

namespace spk_gold {

inline Rec64 make_rec64(uint64_t seed, uint64_t i) {
  Rec64 r;
  r.i0 = (int32_t)(uint32_t)rnd(seed, i, 0);
  r.i1 = (int32_t)(uint32_t)rnd(seed, i, 1);
  r.i2 = (int32_t)(uint32_t)rnd(seed, i, 2);
  r.i3 = (int32_t)(uint32_t)rnd(seed, i, 3);
  r.f0 = rf(rnd(seed, i, 4));
  r.f1 = rf(rnd(seed, i, 5));
  r.f2 = rf(rnd(seed, i, 6));
  r.f3 = rf(rnd(seed, i, 7));
  r.d0 = rd(rnd(seed, i, 8));
  r.d1 = rd(rnd(seed, i, 9));
  r.d2 = rd(rnd(seed, i, 10));
  r.d3 = rd(rnd(seed, i, 11));
  return r;
}

// string of record i: length rnd(i,1) % (maxlen+1); char j from word 2+j/8
// param: maxlen in bits 0-15, minlen in bits 16-30 (length U[minlen,
// maxlen]), bit 31: any byte value instead of 'a'..'z' (bench c3r / c3l:
// binary std::string payloads); a plain maxlen < 65536 is the original U[0, maxlen]
inline uint32_t chars_len(uint64_t seed, uint64_t i, uint32_t param) {
  const uint32_t mx = param & 0xFFFFu, mn = (param >> 16) & 0x7FFFu;
  return mn + (uint32_t)(rnd(seed, i, 1) % (uint64_t)(mx - mn + 1));
}
inline std::string make_chars(uint64_t seed, uint64_t i, uint32_t param) {
  const uint32_t len = param < 0x10000u ? (uint32_t)(rnd(seed, i, 1) % (uint64_t)(param + 1))
                                        : chars_len(seed, i, param);
  const bool raw = (param >> 31) != 0;
  std::string s(len, '\0');
  for (uint32_t j = 0; j < len; ++j) {
    uint64_t w = rnd(seed, i, 2 + (j >> 3) % 56);  // words 2..57, recycled
    const uint32_t b = (uint32_t)((w >> ((j & 7) * 8)) & 0xFF);
    s[j] = (char)(raw ? b : 'a' + b % 26);
  }
  return s;
}

inline RecS make_recs(uint64_t seed, uint64_t i, uint32_t maxlen) {
  RecS r;
  r.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  r.name = make_chars(seed, i, maxlen);
  r.v = rd(rnd(seed, i, 60));
  return r;
}

inline Outer make_outer(uint64_t seed, uint64_t i, uint32_t maxn) {
  Outer o;
  o.key = (int64_t)rnd(seed, i, 0);
  uint32_t n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(maxn + 1));
  o.items.resize(n);
  for (uint32_t j = 0; j < n; ++j) {
    uint64_t w = rnd(seed, i, 2 + j % 62);
    uint64_t w2 = mix64(w ^ (uint64_t)j);
    o.items[j].x = (int32_t)(uint32_t)w2;
    o.items[j].y = rf(w2 >> 32);
  }
  return o;
}

// Generators fill objects IN PLACE (T& out): padding bytes of trivially
// serializable structs travel verbatim on the wire, so they must stay the
// zeros of value-initialisation (a by-value copy may leave them garbage).
inline void fill(Pad &p, uint64_t seed, uint64_t i, uint32_t) {
  std::memset((void *)&p, 0, sizeof(p));
  uint64_t w = rnd(seed, i, 0);
  p.a = (int8_t)(w & 0xFF);
  p.b = (int32_t)(uint32_t)(w >> 8);
  p.c = (int16_t)(w >> 40);
}

inline void fill(Mixed &m, uint64_t seed, uint64_t i, uint32_t maxlen) {
  fill(m.p, seed, i, 0);
  m.k = (int64_t)rnd(seed, i, 58);
  uint64_t a = rnd(seed, i, 59);
  m.arr = {(int16_t)a, (int16_t)(a >> 16), (int16_t)(a >> 32)};
  m.s = make_chars(seed, i, maxlen);
  uint32_t n = (uint32_t)(rnd(seed, i, 61) % (uint64_t)(maxlen + 1));
  m.v.resize(n);
  for (uint32_t j = 0; j < n; ++j)
    m.v[j] = (int32_t)(uint32_t)mix64(rnd(seed, i, 62) + j);
}

inline void fill(Opt &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  const uint64_t bits = rnd(seed, i, 3);
  if (bits & 1) o.score = rd(rnd(seed, i, 60));
  o.tag = make_chars(seed, i, maxlen);
  if (bits & 2) {
    o.pad.emplace();
    fill(*o.pad, seed, i, 0);
  }
}

inline void fill(OptP &o, uint64_t seed, uint64_t i, uint32_t) {
  o.k = (int64_t)rnd(seed, i, 0);
  const uint64_t bits = rnd(seed, i, 3);
  if (bits & 1) o.a = (int32_t)(uint32_t)rnd(seed, i, 4);
  if (bits & 4) o.b = rpcb::point{rd(rnd(seed, i, 5)), rd(rnd(seed, i, 6))};
}

// magnitudes from 0 to 64 bits, so every LEB128 length 1..10 occurs
inline uint64_t spread(uint64_t w) { return w >> ((w >> 58) & 63); }

inline void fill(Var &v, uint64_t seed, uint64_t i, uint32_t maxlen) {
  const uint64_t r0 = rnd(seed, i, 0), r3 = rnd(seed, i, 3), r4 = rnd(seed, i, 4),
                 r5 = rnd(seed, i, 5);
  const uint32_t a = (uint32_t)spread(r0);
  v.a = (int32_t)((r0 & 1) ? ~a : a);
  v.s = make_chars(seed, i, maxlen);
  v.b = spread(r3);
  v.d = rd(rnd(seed, i, 60));
  const uint64_t c = spread(r4);
  v.c = (int64_t)((r4 & 1) ? ~c : c);
  v.e = (uint32_t)spread(r5);
}

inline void fill(VarP &v, uint64_t seed, uint64_t i, uint32_t) {
  const uint64_t r0 = rnd(seed, i, 0), r1 = rnd(seed, i, 1), r2 = rnd(seed, i, 2);
  v.id = (int32_t)(uint32_t)r0;
  const uint64_t x = spread(r1);
  v.x = (int64_t)((r1 & 1) ? ~x : x);
  v.y = (uint32_t)spread(r2);
}

inline rpcb::rect make_rpc_rect(uint64_t seed, uint64_t i) {
  return rpcb::rect{{rd(rnd(seed, i, 0)), rd(rnd(seed, i, 1))},
                    {rd(rnd(seed, i, 2)), rd(rnd(seed, i, 3))}};
}

inline rpcb::person make_person(uint64_t seed, uint64_t i, uint32_t maxlen) {
  rpcb::person p;
  p.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  p.name = make_chars(seed, i, maxlen);
  p.age = (int32_t)(rnd(seed, i, 60) % 100);
  p.salary = rd(rnd(seed, i, 61));
  return p;
}

inline std::vector<int32_t> make_ints(uint64_t seed, uint64_t i,
                                      uint32_t maxn) {
  uint32_t n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(maxn + 1));
  std::vector<int32_t> v(n);
  for (uint32_t j = 0; j < n; ++j)
    v[j] = (int32_t)(uint32_t)mix64(rnd(seed, i, 2) + j);
  return v;
}

// element j of a record's list: a short string from word h (len h % 13)
inline std::string tag_chars(uint64_t h) {
  std::string s((size_t)(h % 13), '\0');
  for (size_t k = 0; k < s.size(); ++k) {
    uint64_t w = mix64(h + (k >> 3));
    s[k] = (char)('a' + ((w >> ((k & 7) * 8)) & 0xFF) % 26);
  }
  return s;
}
inline uint64_t elem_word(uint64_t seed, uint64_t i, uint64_t j) {
  return mix64(rnd(seed, i, 2 + j % 56) ^ j);
}

inline void fill(Tags &t, uint64_t seed, uint64_t i, uint32_t maxn) {
  t.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  const uint32_t n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(maxn + 1));
  t.tags.resize(n);
  for (uint32_t j = 0; j < n; ++j) t.tags[j] = tag_chars(elem_word(seed, i, j));
  t.w = rd(rnd(seed, i, 60));
}

inline void fill(Group &g, uint64_t seed, uint64_t i, uint32_t maxn) {
  g.gid = (int64_t)rnd(seed, i, 0);
  const uint32_t n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(maxn + 1));
  const uint64_t s2 = mix64(seed + i);  // member j = RecS j of seed s2
  g.members.resize(n);
  for (uint32_t j = 0; j < n; ++j) g.members[j] = make_recs(s2, j, 20);
  g.label = make_chars(seed, i, 12);
}

inline void fill(Deep &d, uint64_t seed, uint64_t i, uint32_t maxn) {
  d.k = (uint16_t)rnd(seed, i, 0);
  const uint32_t n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(maxn + 1));
  d.m.resize(n);
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t h = elem_word(seed, i, j);
    d.m[j].resize((size_t)(h % 5));
    for (size_t q = 0; q < d.m[j].size(); ++q) d.m[j][q] = tag_chars(mix64(h + q + 1));
  }
}

inline void fill(Vnt &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  switch (rnd(seed, i, 1) % 4) {
    case 0: o.v = (int32_t)(uint32_t)rnd(seed, i, 2); break;
    case 1: o.v = rd(rnd(seed, i, 3)); break;
    case 2: o.v = make_chars(seed, i, maxlen); break;
    default: o.v = Inner{(int32_t)(uint32_t)rnd(seed, i, 4), rf(rnd(seed, i, 5))};
  }
  if (rnd(seed, i, 6) & 1) {
    std::vector<int32_t> v((size_t)(rnd(seed, i, 7) % (uint64_t)(maxlen + 1)));
    for (size_t j = 0; j < v.size(); ++j) v[j] = (int32_t)(uint32_t)mix64(rnd(seed, i, 8) + j);
    o.w = std::move(v);
  }
  const uint64_t n = rnd(seed, i, 9) % 5;
  o.list.clear();
  for (uint64_t j = 0; j < n; ++j) {
    const uint64_t h = elem_word(seed, i, j);
    if (h & 1)
      o.list.emplace_back(tag_chars(h >> 1));
    else
      o.list.emplace_back((int64_t)(h >> 1));
  }
}

// varint values with one magnitude per record (64 - sh bits), member j zero
// when bit j of z is set, signed ones negated (~x) on bit 0 of their word
struct FvGen {
  uint64_t seed, i;
  uint32_t sh, z;
  FvGen(uint64_t s, uint64_t i_) : seed(s), i(i_) {
    const uint64_t r7 = rnd(s, i_, 7);
    sh = (uint32_t)(r7 >> 58);
    z = (uint32_t)r7;
  }
  uint64_t u(uint32_t j) const { return ((z >> j) & 1) ? 0 : rnd(seed, i, j) >> sh; }
  uint64_t sg(uint32_t j) const {
    const uint64_t x = u(j);
    return ((z >> j) & 1) ? 0 : (rnd(seed, i, j) & 1) ? ~x : x;
  }
};
template <typename F>
inline void fill_fv(F &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  const FvGen g(seed, i);
  o.a = (int32_t)(uint32_t)g.sg(0);
  o.s = make_chars(seed, i, maxlen);
  o.b = g.u(2);
  o.d = rd(rnd(seed, i, 60));
  o.c = (int64_t)g.sg(3);
  o.e = (uint32_t)g.u(4);
}
inline void fill(FV &o, uint64_t seed, uint64_t i, uint32_t maxlen) { fill_fv(o, seed, i, maxlen); }
inline void fill(FVE &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  fill_fv(o, seed, i, maxlen);
  o.f = (int16_t)rnd(seed, i, 5);
}
inline void fill(FV32 &o, uint64_t seed, uint64_t i, uint32_t) {
  const FvGen g(seed, i);
  o.a = (uint32_t)g.u(0);
  o.x = (int16_t)rnd(seed, i, 5);
  o.b = (int32_t)(uint32_t)g.sg(1);
}
inline void fill(EV &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  const FvGen g(seed, i);
  o.a = (int32_t)(uint32_t)g.sg(0);
  o.s = make_chars(seed, i, maxlen);
  o.b = g.u(2);
  o.c = (int64_t)g.sg(3);
  o.e = (uint32_t)g.u(4);
}

template <typename C>
inline void fill_cmp(C &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  const uint64_t m = rnd(seed, i, 6);
  if (m & 1) o.a = (int64_t)rnd(seed, i, 2);
  o.name = make_chars(seed, i, maxlen);
  if (m & 2) o.c = rd(rnd(seed, i, 3));
  if (m & 4) o.b = (int16_t)rnd(seed, i, 4);
}
inline void fill(Cmp &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  fill_cmp(o, seed, i, maxlen);
}
inline void fill(CmpNew &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  fill_cmp(o, seed, i, maxlen);
  if (rnd(seed, i, 6) & 8) o.d = (int32_t)(uint32_t)rnd(seed, i, 5);
}
inline void fill(CmpOld &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  o.name = make_chars(seed, i, maxlen);
}

inline void fill(Al8 &o, uint64_t seed, uint64_t i, uint32_t) {
  std::memset((void *)&o, 0, sizeof(o));
  const uint64_t r = rnd(seed, i, 0);
  o.a = (char)r;
  o.b = (short)(r >> 8);
}
inline void fill(AlOuter &o, uint64_t seed, uint64_t i, uint32_t) {
  std::memset((void *)&o, 0, sizeof(o));
  const uint64_t r = rnd(seed, i, 1);
  o.a.a = (char)r;
  o.a.b = (short)(r >> 8);
  o.b.a = (char)(r >> 24);
  o.b.b = (int)(r >> 32);
}
inline void fill(Packed &o, uint64_t seed, uint64_t i, uint32_t) {
  std::memset((void *)&o, 0, sizeof(o));
  const uint64_t r = rnd(seed, i, 2);
  o.a = (char)r;
  o.b = (int32_t)(r >> 8);
  o.c = (int16_t)(r >> 40);
}
inline void fill(AlRec &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  fill(o.o, seed, i, 0);
  o.s = make_chars(seed, i, maxlen);
  fill(o.p, seed, i, 0);
  fill(o.e, seed, i, 0);
}

inline void fill(Lists &o, uint64_t seed, uint64_t i, uint32_t maxn) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  const uint32_t n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(maxn + 1));
  for (uint32_t j = 0; j < n; ++j) o.names.push_back(tag_chars(elem_word(seed, i, j)));
  const uint64_t r3 = rnd(seed, i, 3);
  for (uint32_t j = 0; j < (uint32_t)((r3 >> 8) % 7); ++j)
    o.vals.push_back((int32_t)(uint32_t)mix64(rnd(seed, i, 4) + j));
  for (uint32_t j = 0; j < (uint32_t)(r3 % 5); ++j) {
    const uint64_t w = mix64(rnd(seed, i, 5) + j);
    o.pts.push_back(Inner{(int32_t)(uint32_t)w, rf(w >> 32)});
  }
}

// keys drawn from small ranges, so maps and sets see repeated keys (a map /
// set keeps the first, a multimap / multiset all of them)
inline void fill(Maps &o, uint64_t seed, uint64_t i, uint32_t) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  const uint64_t b = rnd(seed, i, 3);
  for (uint32_t j = 0; j < (uint32_t)(b % 5); ++j) {
    const uint64_t h = elem_word(seed, i, j);
    o.m.emplace((int32_t)(h % 7) - 3, tag_chars(h >> 8));
  }
  for (uint32_t j = 0; j < (uint32_t)((b >> 8) % 5); ++j)
    o.s.insert(tag_chars(mix64(rnd(seed, i, 20) + j) % 5));
  for (uint32_t j = 0; j < (uint32_t)((b >> 16) % 4); ++j) {
    const uint64_t w = mix64(rnd(seed, i, 22) + j);
    o.mm.emplace((int64_t)(mix64(rnd(seed, i, 21) + j) % 3) - 1,
                 Inner{(int32_t)(uint32_t)w, rf(w >> 32)});
  }
  for (uint32_t j = 0; j < (uint32_t)((b >> 24) % 6); ++j)
    o.ms.insert((int32_t)(mix64(rnd(seed, i, 23) + j) % 7) - 3);
  for (uint32_t j = 0; j < (uint32_t)((b >> 32) % 3); ++j)
    o.mr.emplace(tag_chars(mix64(rnd(seed, i, 24) + j) % 4 + 1), make_recs(mix64(seed + i), j, 10));
}

// create_complicated_object() (test_struct.hpp:82-103), padding bytes zero
inline void fill(cpx::complicated_object &x, uint64_t, uint64_t, uint32_t) {
  using cpx::person;
  x.color = cpx::Color::red;
  x.a = 42;
  x.b = "hello";
  x.c = {{20, "tom"}, {22, "jerry"}};
  x.d = {"hello", "world"};
  x.e = {1, 2};
  x.f = {{1, {20, "tom"}}};
  x.g = {{1, {20, "tom"}}, {1, {22, "jerry"}}};
  x.h = {"aa", "bb"};
  x.i = {1, 2};
  x.j = {{1, {20, "tom"}}};
  x.k = {{1, 2}};
  x.m = {person{20, "tom"}, {22, "jerry"}};
  x.n[0] = person{15, "tom"};
  x.n[1] = person{31, "jerry"};
  x.o = std::make_pair(std::string("aa"), person{20, "tom"});
  const double bs[4] = {1.7, 1.4, 0.7, 11111.4};
  const float cs[4] = {2.4f, 2.6f, 1.4f, 2213321.6f};
  const int as[4] = {1232114, 12315, 4, 1123115};
  x.p.resize(2);
  std::memset((void *)x.p.data(), 0, 2 * sizeof(x.p[0]));
  for (int q = 0; q < 4; ++q) {
    cpx::trivial_one &t = x.p[q / 2][q % 2];
    t.a = as[q];
    t.b = bs[q];
    t.c = cs[q];
  }
}

inline void fill(ValidateRequest &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  const uint64_t b = rnd(seed, i, 3);
  AliMessage &m = o.msg;
  m.message_type = (int32_t)(uint32_t)rnd(seed, i, 0);
  if (b & 1) m.session_no = make_chars(seed, i, maxlen);
  if (b & 2) m.tint_flag = (rnd(seed, i, 4) & 1) != 0;
  if (b & 4) m.source_entity = (uint32_t)rnd(seed, i, 5);
  if (b & 8) m.dest_entity = (uint32_t)rnd(seed, i, 6);
  if (b & 16) m.client_ip = tag_chars(rnd(seed, i, 7));
  if (b & 32) {
    m.rc.emplace();
    m.rc->retcode = (int32_t)(uint32_t)rnd(seed, i, 8);
    if (b & 64) m.rc->error_message = tag_chars(rnd(seed, i, 9));
  }
  if (b & 128) m.version = (int32_t)(uint32_t)rnd(seed, i, 10);
  if (b & 256) o.job_id = (int32_t)(uint32_t)rnd(seed, i, 11);
  const uint32_t n = (uint32_t)((b >> 16) % 5);
  o.query_keys.resize(n);
  for (uint32_t j = 0; j < n; ++j) o.query_keys[j] = tag_chars(elem_word(seed, i, j));
  if (b & 512) o.clean = ((rnd(seed, i, 12) >> 1) & 1) != 0;
}

#ifdef SPK_TYPES_HAVE_EXPECTED
inline void fill(Exp &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  const uint64_t b = rnd(seed, i, 3);
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  if (b & 1)
    o.r = make_chars(seed, i, maxlen);
  else
    o.r = struct_pack::unexpected<int32_t>((int32_t)(uint32_t)rnd(seed, i, 4));
  if (b & 2)
    o.q = Inner{(int32_t)(uint32_t)rnd(seed, i, 5), rf(rnd(seed, i, 6))};
  else
    o.q = struct_pack::unexpected<std::string>(tag_chars(rnd(seed, i, 7)));
  if (b & 4) {
    o.l.emplace();
    const uint32_t n = (uint32_t)((b >> 16) % 4);
    for (uint32_t j = 0; j < n; ++j) o.l->push_back(tag_chars(elem_word(seed, i, j)));
  }
  if (b & 8) {
    o.e = (int64_t)rnd(seed, i, 8);
  } else {
    ResponseCode rc{(int32_t)(uint32_t)rnd(seed, i, 9), std::nullopt};
    if (b & 16) rc.error_message = tag_chars(rnd(seed, i, 10));
    o.e = struct_pack::unexpected<ResponseCode>(rc);
  }
}
#endif

inline void fill(CmpG &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  const uint64_t m = rnd(seed, i, 6);
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  if (m & 1) o.note = tag_chars(rnd(seed, i, 2));
  o.name = make_chars(seed, i, maxlen);
  if (m & 2) {
    std::vector<int32_t> v((size_t)((m >> 8) % 6));
    for (size_t j = 0; j < v.size(); ++j) v[j] = (int32_t)(uint32_t)mix64(rnd(seed, i, 3) + j);
    o.ints = std::move(v);
  }
  if (m & 4) o.in = Inner{(int32_t)(uint32_t)rnd(seed, i, 4), rf(rnd(seed, i, 5))};
  if (m & 8) {
    ResponseCode rc{(int32_t)(uint32_t)rnd(seed, i, 7), std::nullopt};
    if (m & 16) rc.error_message = tag_chars(rnd(seed, i, 8));
    o.rc = rc;
  }
}

inline void fill(Monster &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  o.pos = Vec3{rf(rnd(seed, i, 4)), rf(rnd(seed, i, 5)), rf(rnd(seed, i, 6))};
  const uint64_t r7 = rnd(seed, i, 7), r9 = rnd(seed, i, 9), r10 = rnd(seed, i, 10);
  o.mana = (int16_t)r7;
  o.hp = (int16_t)(r7 >> 16);
  o.name = make_chars(seed, i, maxlen);
  o.inventory = tag_chars(rnd(seed, i, 8));
  o.color = (Color)(r9 % 3);
  o.weapons.resize((size_t)((r9 >> 8) % 5));
  for (size_t j = 0; j < o.weapons.size(); ++j) {
    const uint64_t h = elem_word(seed, i, j);
    o.weapons[j] = Weapon{tag_chars(h), (int16_t)(h >> 32)};
  }
  o.equipped = Weapon{tag_chars(r10), (int16_t)(r10 >> 40)};
  o.path.resize((size_t)((r9 >> 16) % 9));
  for (size_t j = 0; j < o.path.size(); ++j) {
    const uint64_t w = mix64(rnd(seed, i, 11) + j);
    o.path[j] = Vec3{rf(w), rf(w >> 32), rf(mix64(w))};
  }
}

inline void fill(rect2<int32_t> &o, uint64_t seed, uint64_t i, uint32_t) {
  const FvGen g(seed, i);
  o.x = (int32_t)(uint32_t)g.sg(0);
  o.y = (int32_t)(uint32_t)g.sg(1);
  o.width = (int32_t)(uint32_t)g.sg(2);
  o.height = (int32_t)(uint32_t)g.sg(3);
}

inline unsigned __int128 u128(uint64_t hi, uint64_t lo) {
  return ((unsigned __int128)hi << 64) | lo;
}
inline void fill(WideT &o, uint64_t seed, uint64_t i, uint32_t) {
  std::memset((void *)&o, 0, sizeof(o));
  o.a = (__int128)u128(rnd(seed, i, 20), rnd(seed, i, 21));
  o.bits = std::bitset<64>(rnd(seed, i, 22));
  const uint64_t r = rnd(seed, i, 23);
  o.c32 = (char32_t)(uint32_t)r;
  o.wc = (wchar_t)(int32_t)(uint32_t)(r >> 32);
  o.c16 = (char16_t)rnd(seed, i, 24);
  o.b = u128(rnd(seed, i, 25), rnd(seed, i, 26));
}
// element j of a wide string: the low bytes of mix64(word k + j)
inline void fill(Wide &o, uint64_t seed, uint64_t i, uint32_t maxlen) {
  o.id = (int32_t)(uint32_t)rnd(seed, i, 0);
  o.a.resize((size_t)(rnd(seed, i, 1) % (maxlen + 1ull)));
  for (size_t j = 0; j < o.a.size(); ++j) o.a[j] = (char16_t)mix64(rnd(seed, i, 2) + j);
  o.big = (__int128)u128(rnd(seed, i, 3), rnd(seed, i, 4));
  o.b.resize((size_t)(rnd(seed, i, 5) % (maxlen + 1ull)));
  for (size_t j = 0; j < o.b.size(); ++j) o.b[j] = (char32_t)(uint32_t)mix64(rnd(seed, i, 6) + j);
  o.bits = (std::bitset<128>(rnd(seed, i, 7)) << 64) | std::bitset<128>(rnd(seed, i, 27));
  o.c.resize((size_t)(rnd(seed, i, 8) % (maxlen + 1ull)));
  for (size_t j = 0; j < o.c.size(); ++j)
    o.c[j] = (wchar_t)(int32_t)(uint32_t)mix64(rnd(seed, i, 9) + j);
  o.ubig = u128(rnd(seed, i, 10), rnd(seed, i, 11));
  const uint64_t r = rnd(seed, i, 12);
  o.wc = (wchar_t)(int32_t)(uint32_t)r;
  o.c16 = (char16_t)(r >> 32);
  fill(o.t, seed, i, 0);
}

}  // namespace spk_gold
