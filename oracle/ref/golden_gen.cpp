// Golden-vector generator built against the REFERENCE struct_pack headers
// (/root/reference/include, read-only). TEST INFRASTRUCTURE ONLY: the binary
// lives in oracle/_ref/ and is driven by tests/golden/make_golden.py, which
// commits small fixtures + SHA-256 digests under tests/golden/.
//
// Subcommands
//   kat                                  type literals / type codes (JSON)
//   emit <case> <n> <seed> <param> <conf> <wire_out> [<lens_out>]
//        mode "A" cases serialize one std::vector<T> message,
//        mode "B" cases serialize n independent T messages back to back and
//        write the per-message byte lengths (u64 LE) to <lens_out>.
//   frames <case> <n> <seed> <param> <req|resp> <function_id> <seq_base>
//          <wire_out> <lens_out>
//        coro_rpc framing of n messages, built the way coro_rpc does it:
//        serialize_to_with_offset(buf, REQ_HEAD_LEN, arg) then the header
//        struct serialized with DISABLE_ALL_META_INFO into the reserved bytes
//        (coro_rpc_client.hpp:1285-1335); responses = resp_header bytes +
//        serialize(ret) (coro_rpc_protocol.hpp:191-240)
//   errs <case> <n> <seed> <param> <conf> <mutations> <wire_in>
//        decode every mutation of <wire_in> with the reference deserialize_to
//        and print errc / consume_len / canonical re-encoding digest (JSON).
#include <ylt/struct_pack.hpp>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "types.hpp"

using namespace spk_gold;
using struct_pack::sp_config;

static void hexlit(std::ostream &os, const char *p, size_t n) {
  os << "\"";
  static const char *hx = "0123456789abcdef";
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = (unsigned char)p[i];
    os << hx[c >> 4] << hx[c & 15];
  }
  os << "\"";
}

template <typename... T>
static void kat_one(std::ostream &os, const char *name, bool &first) {
  constexpr auto lit = struct_pack::get_type_literal<T...>();
  uint32_t code = struct_pack::get_type_code<T...>();
  if (!first) os << ",\n";
  first = false;
  os << "  \"" << name << "\": {\"code\": " << code << ", \"literal\": ";
  hexlit(os, lit.data(), lit.size());
  os << "}";
}

static int cmd_kat() {
  std::ostringstream os;
  bool first = true;
  os << "{\n";
  kat_one<Rec64>(os, "Rec64", first);
  kat_one<std::vector<Rec64>>(os, "vector<Rec64>", first);
  kat_one<RecS>(os, "RecS", first);
  kat_one<std::vector<RecS>>(os, "vector<RecS>", first);
  kat_one<Inner>(os, "Inner", first);
  kat_one<Outer>(os, "Outer", first);
  kat_one<std::vector<Outer>>(os, "vector<Outer>", first);
  kat_one<Pad>(os, "Pad", first);
  kat_one<std::vector<Pad>>(os, "vector<Pad>", first);
  kat_one<Mixed>(os, "Mixed", first);
  kat_one<std::vector<Mixed>>(os, "vector<Mixed>", first);
  kat_one<rect<int>>(os, "rect<int>", first);
  kat_one<std::vector<rect<int>>>(os, "vector<rect<int>>", first);
  kat_one<rpcb::point>(os, "rpc::point", first);
  kat_one<rpcb::rect>(os, "rpc::rect", first);
  kat_one<std::vector<rpcb::rect>>(os, "vector<rpc::rect>", first);
  kat_one<rpcb::person>(os, "person", first);
  kat_one<std::vector<rpcb::person>>(os, "vector<person>", first);
  kat_one<std::vector<int32_t>>(os, "vector<int32_t>", first);
  kat_one<std::string>(os, "string", first);
  kat_one<int32_t>(os, "int32_t", first);
  kat_one<int32_t, int32_t, int16_t>(os, "<int32_t,int32_t,int16_t>", first);
  kat_one<rpcb::req_header>(os, "req_header", first);
  kat_one<rpcb::resp_header>(os, "resp_header", first);
  kat_one<std::monostate>(os, "monostate", first);
  kat_one<Opt>(os, "Opt", first);
  kat_one<std::vector<Opt>>(os, "vector<Opt>", first);
  kat_one<OptP>(os, "OptP", first);
  kat_one<std::vector<OptP>>(os, "vector<OptP>", first);
  kat_one<std::optional<int32_t>>(os, "optional<int32_t>", first);
  kat_one<Var>(os, "Var", first);
  kat_one<std::vector<Var>>(os, "vector<Var>", first);
  kat_one<VarP>(os, "VarP", first);
  kat_one<std::vector<VarP>>(os, "vector<VarP>", first);
  kat_one<struct_pack::var_int32_t, struct_pack::var_int64_t, struct_pack::var_uint32_t,
          struct_pack::var_uint64_t>(os, "varints", first);
  kat_one<std::array<int16_t, 3>>(os, "array<int16_t,3>", first);
  kat_one<std::vector<std::string>>(os, "vector<string>", first);
  kat_one<Tags>(os, "Tags", first);
  kat_one<std::vector<Tags>>(os, "vector<Tags>", first);
  kat_one<Group>(os, "Group", first);
  kat_one<std::vector<Group>>(os, "vector<Group>", first);
  kat_one<Deep>(os, "Deep", first);
  kat_one<Vnt>(os, "Vnt", first);
  kat_one<Al8>(os, "Al8", first);
  kat_one<AlOuter>(os, "AlOuter", first);
  kat_one<Packed>(os, "Packed", first);
  kat_one<AlRec>(os, "AlRec", first);
  kat_one<std::vector<AlRec>>(os, "vector<AlRec>", first);
  kat_one<std::vector<Vnt>>(os, "vector<Vnt>", first);
  kat_one<std::variant<int32_t, std::string>>(os, "variant<int32_t,string>", first);
  kat_one<std::vector<Deep>>(os, "vector<Deep>", first);
  kat_one<Cmp>(os, "Cmp", first);
  kat_one<std::vector<Cmp>>(os, "vector<Cmp>", first);
  kat_one<CmpOld>(os, "CmpOld", first);
  kat_one<CmpNew>(os, "CmpNew", first);
  kat_one<FV>(os, "FV", first);
  kat_one<std::vector<FV>>(os, "vector<FV>", first);
  kat_one<FVE>(os, "FVE", first);
  kat_one<FV32>(os, "FV32", first);
  kat_one<EV>(os, "EV", first);
  kat_one<std::vector<EV>>(os, "vector<EV>", first);
  kat_one<ResponseCode>(os, "ResponseCode", first);
  kat_one<AliMessage>(os, "AliMessage", first);
  kat_one<ValidateRequest>(os, "ValidateRequest", first);
  kat_one<std::vector<ValidateRequest>>(os, "vector<ValidateRequest>", first);
  kat_one<Exp>(os, "Exp", first);
  kat_one<std::vector<Exp>>(os, "vector<Exp>", first);
  kat_one<struct_pack::expected<void, int32_t>>(os, "expected<void,int32_t>", first);
  kat_one<CmpG>(os, "CmpG", first);
  kat_one<Vec3>(os, "Vec3", first);
  kat_one<Weapon>(os, "Weapon", first);
  kat_one<Monster>(os, "Monster", first);
  kat_one<std::vector<Monster>>(os, "vector<Monster>", first);
  kat_one<rect2<int32_t>>(os, "rect2<int32_t>", first);
  kat_one<std::vector<rect2<int32_t>>>(os, "vector<rect2<int32_t>>", first);
  kat_one<Lists>(os, "Lists", first);
  kat_one<Maps>(os, "Maps", first);
  kat_one<std::vector<Maps>>(os, "vector<Maps>", first);
  kat_one<std::map<int32_t, std::string>>(os, "map<int32_t,string>", first);
  kat_one<std::unordered_multimap<int32_t, int32_t>>(os, "unordered_multimap<int32_t,int32_t>", first);
  kat_one<std::pair<std::string, cpx::person>>(os, "pair<string,person>", first);
  kat_one<cpx::complicated_object>(os, "complicated_object", first);
  kat_one<uint8_t, uint16_t, uint32_t, uint64_t, int8_t, int16_t, int64_t,
          bool, char, float, double>(os, "fundamentals", first);
  kat_one<__int128, unsigned __int128, wchar_t, char16_t, char32_t>(os, "wide fundamentals",
                                                                   first);
  kat_one<std::bitset<64>>(os, "bitset<64>", first);
  kat_one<std::bitset<128>>(os, "bitset<128>", first);
  kat_one<std::u16string>(os, "u16string", first);
  kat_one<std::u32string>(os, "u32string", first);
  kat_one<std::wstring>(os, "wstring", first);
  kat_one<WideT>(os, "WideT", first);
  kat_one<std::vector<WideT>>(os, "vector<WideT>", first);
  kat_one<Wide>(os, "Wide", first);
  kat_one<std::vector<Wide>>(os, "vector<Wide>", first);
  os << "\n}\n";
  std::cout << os.str();
  return 0;
}

// ---------------------------------------------------------------------------
struct Args {
  std::string kase;
  uint64_t n, seed;
  uint32_t param;
  std::string conf;
};

template <typename T>
struct elem_of {
  using type = T;
};
template <typename T>
struct elem_of<std::vector<T>> {
  using type = T;
};
// DISABLE_ALL_META_INFO is a compile error with compatible members
// (type_calculate.hpp:868-876): such cases fall back to the default config
template <uint64_t conf, typename T>
static constexpr uint64_t conf_for() {
  if constexpr (conf == sp_config::DISABLE_ALL_META_INFO &&
                kHasCompat<typename elem_of<T>::type>)
    return sp_config::DEFAULT;
  else
    return conf;
}

template <uint64_t conf, typename T>
static void ser_append(std::string &out, const T &v) {
  struct_pack::serialize_to<conf_for<conf, T>()>(out, v);
}

template <typename T, typename Gen>
static void emit_typed(const Args &a, Gen gen, std::string &wire,
                       std::vector<uint64_t> &lens, bool modeB) {
  if (!modeB) {
    std::vector<T> v(a.n);  // value-initialised: zero padding
    for (uint64_t i = 0; i < a.n; ++i) gen(v[i], i);
    if (a.conf == "typeinfo")
      ser_append<sp_config::ENABLE_TYPE_INFO>(wire, v);
    else if (a.conf == "nometa")
      ser_append<sp_config::DISABLE_ALL_META_INFO>(wire, v);
    else
      ser_append<sp_config::DEFAULT>(wire, v);
    lens.push_back(wire.size());
  }
  else {
    for (uint64_t i = 0; i < a.n; ++i) {
      T v{};
      gen(v, i);
      size_t before = wire.size();
      if (a.conf == "typeinfo")
        ser_append<sp_config::ENABLE_TYPE_INFO>(wire, v);
      else if (a.conf == "nometa")
        ser_append<sp_config::DISABLE_ALL_META_INFO>(wire, v);
      else
        ser_append<sp_config::DEFAULT>(wire, v);
      lens.push_back(wire.size() - before);
    }
  }
}

// dispatch on the case name; calls f.template operator()<T>(gen)
template <typename F>
static bool with_case(const Args &a, F &&f) {
  const std::string &k = a.kase;
  uint64_t s = a.seed;
  uint32_t p = a.param;
  if (k == "rec64")
    return f.template operator()<Rec64>([=](Rec64 &o, uint64_t i) { o = make_rec64(s, i); });
  if (k == "recs")
    return f.template operator()<RecS>([=](RecS &o, uint64_t i) { o = make_recs(s, i, p); });
  if (k == "outer")
    return f.template operator()<Outer>([=](Outer &o, uint64_t i) { o = make_outer(s, i, p); });
  if (k == "pad")
    return f.template operator()<Pad>([=](Pad &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "mixed")
    return f.template operator()<Mixed>([=](Mixed &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "opt")
    return f.template operator()<Opt>([=](Opt &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "optp")
    return f.template operator()<OptP>([=](OptP &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "var")
    return f.template operator()<Var>([=](Var &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "varp")
    return f.template operator()<VarP>([=](VarP &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "tags")
    return f.template operator()<Tags>([=](Tags &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "group")
    return f.template operator()<Group>([=](Group &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "al8")
    return f.template operator()<Al8>([=](Al8 &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "alout")
    return f.template operator()<AlOuter>([=](AlOuter &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "packed")
    return f.template operator()<Packed>([=](Packed &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "alrec")
    return f.template operator()<AlRec>([=](AlRec &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "vnt")
    return f.template operator()<Vnt>([=](Vnt &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "cmp")
    return f.template operator()<Cmp>([=](Cmp &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "cmpold")
    return f.template operator()<CmpOld>([=](CmpOld &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "cmpnew")
    return f.template operator()<CmpNew>([=](CmpNew &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "fv")
    return f.template operator()<FV>([=](FV &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "fve")
    return f.template operator()<FVE>([=](FVE &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "fv32")
    return f.template operator()<FV32>([=](FV32 &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "ev")
    return f.template operator()<EV>([=](EV &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "deep")
    return f.template operator()<Deep>([=](Deep &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "lists")
    return f.template operator()<Lists>([=](Lists &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "maps")
    return f.template operator()<Maps>([=](Maps &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "cplx")
    return f.template operator()<cpx::complicated_object>(
        [=](cpx::complicated_object &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "valreq")
    return f.template operator()<ValidateRequest>([=](ValidateRequest &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "exp")
    return f.template operator()<Exp>([=](Exp &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "cmpg")
    return f.template operator()<CmpG>([=](CmpG &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "monster")
    return f.template operator()<Monster>([=](Monster &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "widet")
    return f.template operator()<WideT>([=](WideT &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "wide")
    return f.template operator()<Wide>([=](Wide &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "rect2")
    return f.template operator()<rect2<int32_t>>([=](rect2<int32_t> &o, uint64_t i) { fill(o, s, i, p); });
  if (k == "rect")  // C1: benchmark rect<int> default values
    return f.template operator()<rect<int>>([=](rect<int> &o, uint64_t) { o = rect<int>{}; });
  if (k == "rpcrect")
    return f.template operator()<rpcb::rect>([=](rpcb::rect &o, uint64_t i) { o = make_rpc_rect(s, i); });
  if (k == "person")
    return f.template operator()<rpcb::person>([=](rpcb::person &o, uint64_t i) { o = make_person(s, i, p); });
  if (k == "ints")  // messages of std::vector<int32_t>
    return f.template operator()<std::vector<int32_t>>(
        [=](std::vector<int32_t> &o, uint64_t i) { o = make_ints(s, i, p); });
  return false;
}

static bool write_file(const std::string &path, const void *p, size_t n) {
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) return false;
  size_t w = n ? fwrite(p, 1, n, f) : 0;
  fclose(f);
  return w == n;
}

static int cmd_emit(const Args &a, bool modeB, const std::string &wire_out,
                    const std::string &lens_out) {
  std::string wire;
  std::vector<uint64_t> lens;
  bool ok = with_case(a, [&]<typename T>(auto gen) {
    emit_typed<T>(a, gen, wire, lens, modeB);
    return true;
  });
  if (!ok) {
    std::cerr << "unknown case " << a.kase << "\n";
    return 2;
  }
  if (!write_file(wire_out, wire.data(), wire.size())) return 3;
  if (!lens_out.empty() &&
      !write_file(lens_out, lens.data(), lens.size() * sizeof(uint64_t)))
    return 3;
  std::cout << wire.size() << "\n";
  return 0;
}

// ---------------------------------------------------------------------------
static int cmd_frames(const Args &a, bool req, uint32_t fid, uint32_t seq_base,
                      const std::string &wire_out, const std::string &lens_out) {
  std::string wire;
  std::vector<uint64_t> lens;
  bool ok = with_case(a, [&]<typename T>(auto gen) {
    for (uint64_t i = 0; i < a.n; ++i) {
      T v{};
      gen(v, i);
      std::string buf;
      if (req) {
        constexpr size_t off = sizeof(rpcb::req_header);  // REQ_HEAD_LEN = 20
        struct_pack::serialize_to_with_offset(buf, off, v);
        rpcb::req_header h{};
        h.magic = 21;  // coro_rpc_protocol::magic_number
        h.function_id = fid;
        h.seq_num = seq_base + (uint32_t)i;
        h.length = (uint32_t)(buf.size() - off);
        auto hl = struct_pack::get_needed_size<sp_config::DISABLE_ALL_META_INFO>(h);
        struct_pack::serialize_to<sp_config::DISABLE_ALL_META_INFO>(buf.data(), hl, h);
      }
      else {
        std::string body;
        struct_pack::serialize_to(body, v);
        rpcb::resp_header h{};
        h.magic = 21;
        h.seq_num = seq_base + (uint32_t)i;
        h.length = (uint32_t)body.size();
        struct_pack::serialize_to<sp_config::DISABLE_ALL_META_INFO>(buf, h);
        buf += body;
      }
      wire += buf;
      lens.push_back(buf.size());
    }
    return true;
  });
  if (!ok) return 2;
  if (!write_file(wire_out, wire.data(), wire.size())) return 3;
  if (!write_file(lens_out, lens.data(), lens.size() * sizeof(uint64_t))) return 3;
  std::cout << wire.size() << "\n";
  return 0;
}

// ---------------------------------------------------------------------------
// Negative / mutation tests: mutation list file has lines
//   trunc <len>            keep the first <len> bytes
//   set <pos> <byte>       overwrite one byte
// Output: one JSON object per line {errc, consume, reenc_hex|null}
template <uint64_t conf0, typename T>
static void decode_report(const std::string &buf, std::ostream &os) {
  constexpr uint64_t conf = conf_for<conf0, T>();
  T obj{};
  size_t consume = 0;
  auto ec = struct_pack::deserialize_to<conf>(obj, buf.data(), buf.size(),
                                              consume);
  os << "{\"errc\": " << (int)ec.ec << ", \"consume\": " << consume
     << ", \"reenc\": ";
  if (!ec) {
    std::string re;
    struct_pack::serialize_to<conf>(re, obj);
    hexlit(os, re.data(), re.size());
  }
  else {
    os << "null";
  }
  os << "}\n";
}

static int cmd_errs(const Args &a, bool modeB, const std::string &muts,
                    const std::string &wire_in) {
  std::ifstream wf(wire_in, std::ios::binary);
  std::string wire((std::istreambuf_iterator<char>(wf)),
                   std::istreambuf_iterator<char>());
  std::ifstream mf(muts);
  std::string line;
  std::ostringstream os;
  while (std::getline(mf, line)) {
    if (line.empty()) continue;
    std::istringstream ls(line);
    std::string op;
    ls >> op;
    std::string buf = wire;
    while (!op.empty()) {
      if (op == "trunc") {
        size_t n;
        ls >> n;
        buf.resize(std::min(n, buf.size()));
      }
      else if (op == "set") {
        size_t pos;
        unsigned v;
        ls >> pos >> v;
        if (pos < buf.size()) buf[pos] = (char)v;
      }
      op.clear();
      ls >> op;
    }
    with_case(a, [&]<typename T>(auto) {
      using M = std::conditional_t<true, T, void>;
      if (!modeB) {
        if (a.conf == "typeinfo")
          decode_report<sp_config::ENABLE_TYPE_INFO, std::vector<M>>(buf, os);
        else if (a.conf == "nometa")
          decode_report<sp_config::DISABLE_ALL_META_INFO, std::vector<M>>(buf, os);
        else
          decode_report<sp_config::DEFAULT, std::vector<M>>(buf, os);
      }
      else {
        if (a.conf == "typeinfo")
          decode_report<sp_config::ENABLE_TYPE_INFO, M>(buf, os);
        else if (a.conf == "nometa")
          decode_report<sp_config::DISABLE_ALL_META_INFO, M>(buf, os);
        else
          decode_report<sp_config::DEFAULT, M>(buf, os);
      }
      return true;
    });
  }
  std::cout << os.str();
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    std::cerr << "usage: golden_gen kat | emit ... | errs ...\n";
    return 2;
  }
  std::string cmd = argv[1];
  if (cmd == "kat") return cmd_kat();
  if (cmd == "frames" && argc >= 11) {
    Args a;
    std::string kase = argv[2];
    a.kase = kase.substr(0, kase.size() - 2);
    a.n = strtoull(argv[3], nullptr, 0);
    a.seed = strtoull(argv[4], nullptr, 0);
    a.param = (uint32_t)strtoul(argv[5], nullptr, 0);
    a.conf = "default";
    return cmd_frames(a, std::string(argv[6]) == "req",
                      (uint32_t)strtoul(argv[7], nullptr, 0),
                      (uint32_t)strtoul(argv[8], nullptr, 0), argv[9], argv[10]);
  }
  if ((cmd == "emit" || cmd == "errs") && argc >= 8) {
    Args a;
    std::string kase = argv[2];
    bool modeB = kase.size() > 2 && kase.substr(kase.size() - 2) == "_B";
    a.kase = kase.substr(0, kase.size() - 2);  // strip _A / _B
    a.n = strtoull(argv[3], nullptr, 0);
    a.seed = strtoull(argv[4], nullptr, 0);
    a.param = (uint32_t)strtoul(argv[5], nullptr, 0);
    a.conf = argv[6];
    if (cmd == "emit")
      return cmd_emit(a, modeB, argv[7], argc > 8 ? argv[8] : "");
    if (argc >= 9) return cmd_errs(a, modeB, argv[7], argv[8]);
  }
  std::cerr << "bad arguments\n";
  return 2;
}
