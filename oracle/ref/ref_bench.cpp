// CPU baseline: the REFERENCE header-only struct_pack (compiled from the
// unmodified /root/reference/include with -O3 -DNDEBUG -DSTRUCT_PACK_OPTIMIZE,
// as src/struct_pack/benchmark/CMakeLists.txt:20 builds its benchmark),
// timed on the host's cores. TEST/BENCH INFRASTRUCTURE ONLY: bench.py runs
// the prebuilt oracle/_ref/ref_bench as its cpu_baseline leg.
//
//   ref_bench <case> <n> <seed> <param> <threads> <reps>
//
// Every thread owns a contiguous slice of the n records (SURVEY.md §8d
// "mode A": each slice is its own std::vector<T> message), with the output
// string pre-reserved and pre-faulted and the decode target pre-sized, then
// runs serialize_to / deserialize_to `reps` times. Prints one JSON line with
// the best (min) wall time per phase over the reps.
#include <ylt/struct_pack.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "types.hpp"

using namespace spk_gold;
using clk = std::chrono::steady_clock;

template <typename T, typename Gen>
static int run(const char *name, uint64_t n, int threads, int reps, Gen gen) {
  struct Slice {
    std::vector<T> in, out;
    std::string wire;
  };
  std::vector<Slice> sl(threads);
  uint64_t in_bytes = 0;
  for (int t = 0; t < threads; ++t) {
    uint64_t a = n * t / threads, b = n * (t + 1) / threads;
    sl[t].in.resize(b - a);
    for (uint64_t i = a; i < b; ++i) gen(sl[t].in[i - a], i);
    auto sz = struct_pack::get_needed_size(sl[t].in).size();
    sl[t].wire.reserve(sz);
    sl[t].wire.assign(sz, '\0');  // pre-fault
    sl[t].wire.clear();
    sl[t].out.resize(b - a);      // pre-sized destination
  }
  double best_enc = 1e30, best_dec = 1e30;
  uint64_t wire_bytes = 0;
  for (int r = 0; r < reps; ++r) {
    std::vector<std::thread> th;
    std::atomic<int> go{0};
    // encode
    auto t0 = clk::now();
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        sl[t].wire.clear();
        struct_pack::serialize_to(sl[t].wire, sl[t].in);
      });
    for (auto &x : th) x.join();
    auto t1 = clk::now();
    th.clear();
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        auto ec = struct_pack::deserialize_to(sl[t].out, sl[t].wire);
        if (ec) std::abort();
      });
    for (auto &x : th) x.join();
    auto t2 = clk::now();
    best_enc = std::min(best_enc, std::chrono::duration<double>(t1 - t0).count());
    best_dec = std::min(best_dec, std::chrono::duration<double>(t2 - t1).count());
    wire_bytes = 0;
    for (auto &s : sl) wire_bytes += s.wire.size();
    (void)go;
  }
  printf("{\"case\": \"%s\", \"n\": %llu, \"threads\": %d, \"reps\": %d, "
         "\"encode_s\": %.6f, \"decode_s\": %.6f, \"wire_bytes\": %llu}\n",
         name, (unsigned long long)n, threads, reps, best_enc, best_dec,
         (unsigned long long)wire_bytes);
  return 0;
}

// ---- C5: coro_rpc server step over framed requests ------------------------
// Request frames are built the way coro_rpc_client::prepare_buffer does
// (serialize_to_with_offset + DISABLE_ALL_META_INFO req_header); the timed
// server step decodes every frame's argument (deserialize_to, as
// rpc_execute.hpp:83) and frames the echo response as prepare_response does
// (resp_header + serialize(ret), coro_rpc_protocol.hpp:191-240).
template <typename T, typename Gen>
struct C5Type {
  std::vector<std::string> req;  // per thread: concatenated request frames
  std::vector<std::vector<uint64_t>> offs;
  std::vector<std::vector<T>> args;
  std::vector<std::string> resp;
  uint64_t n = 0;
  Gen gen;
  explicit C5Type(Gen g) : gen(g) {}
  void build(uint64_t n_, int threads, uint32_t fid) {
    n = n_;
    req.resize(threads);
    offs.resize(threads);
    args.resize(threads);
    resp.resize(threads);
    for (int t = 0; t < threads; ++t) {
      uint64_t a = n * t / threads, b = n * (t + 1) / threads;
      offs[t].push_back(0);
      for (uint64_t i = a; i < b; ++i) {
        T v{};
        gen(v, i);
        std::string buf;
        struct_pack::serialize_to_with_offset(buf, sizeof(rpcb::req_header), v);
        rpcb::req_header h{};
        h.magic = 21;
        h.function_id = fid;
        h.seq_num = (uint32_t)i;
        h.length = (uint32_t)(buf.size() - sizeof(rpcb::req_header));
        auto hl = struct_pack::get_needed_size<
            struct_pack::sp_config::DISABLE_ALL_META_INFO>(h);
        struct_pack::serialize_to<struct_pack::sp_config::DISABLE_ALL_META_INFO>(
            buf.data(), hl, h);
        req[t] += buf;
        offs[t].push_back(req[t].size());
      }
      args[t].resize(b - a);
      resp[t].reserve(req[t].size());
      resp[t].assign(req[t].size(), '\0');  // pre-fault
      resp[t].clear();
    }
  }
  void decode(int t) {
    const std::string &r = req[t];
    for (size_t k = 0; k + 1 < offs[t].size(); ++k) {
      const char *p = r.data() + offs[t][k] + sizeof(rpcb::req_header);
      size_t len = offs[t][k + 1] - offs[t][k] - sizeof(rpcb::req_header);
      if (struct_pack::deserialize_to(args[t][k], p, len)) std::abort();
    }
  }
  void encode(int t) {
    std::string &o = resp[t];
    o.clear();
    for (size_t k = 0; k < args[t].size(); ++k) {
      rpcb::resp_header h{};
      h.magic = 21;
      h.seq_num = (uint32_t)k;
      h.length = (uint32_t)struct_pack::get_needed_size(args[t][k]).size();
      struct_pack::serialize_to<struct_pack::sp_config::DISABLE_ALL_META_INFO>(o, h);
      struct_pack::serialize_to(o, args[t][k]);
    }
  }
};

static int run_c5(uint64_t n, int threads, int reps) {
  const uint64_t s1 = 0x5EED0007, s2 = 0x5EED0008, s3 = 0x5EED0009;
  auto g1 = [=](rpcb::rect &o, uint64_t i) { o = make_rpc_rect(s1, i); };
  auto g2 = [=](rpcb::person &o, uint64_t i) { o = make_person(s2, i, 48); };
  auto g3 = [=](std::vector<int32_t> &o, uint64_t i) { o = make_ints(s3, i, 2000); };
  C5Type<rpcb::rect, decltype(g1)> a(g1);
  C5Type<rpcb::person, decltype(g2)> b(g2);
  C5Type<std::vector<int32_t>, decltype(g3)> c(g3);
  a.build(n / 3, threads, 1);
  b.build(n / 3, threads, 2);
  c.build(n / 3, threads, 3);
  double best_enc = 1e30, best_dec = 1e30;
  uint64_t wire = 0;
  for (int r = 0; r < reps; ++r) {
    std::vector<std::thread> th;
    auto t0 = clk::now();
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] { a.decode(t); b.decode(t); c.decode(t); });
    for (auto &x : th) x.join();
    auto t1 = clk::now();
    th.clear();
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] { a.encode(t); b.encode(t); c.encode(t); });
    for (auto &x : th) x.join();
    auto t2 = clk::now();
    best_dec = std::min(best_dec, std::chrono::duration<double>(t1 - t0).count());
    best_enc = std::min(best_enc, std::chrono::duration<double>(t2 - t1).count());
  }
  for (int t = 0; t < threads; ++t)
    wire += a.req[t].size() + b.req[t].size() + c.req[t].size();
  printf("{\"case\": \"c5\", \"n\": %llu, \"threads\": %d, \"reps\": %d, "
         "\"encode_s\": %.6f, \"decode_s\": %.6f, \"wire_bytes\": %llu}\n",
         (unsigned long long)(n / 3 * 3), threads, reps, best_enc, best_dec,
         (unsigned long long)wire);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: ref_bench <case> <n> <seed> <param> <threads> <reps>\n");
    return 2;
  }
  std::string k = argv[1];
  uint64_t n = strtoull(argv[2], nullptr, 0), s = strtoull(argv[3], nullptr, 0);
  uint32_t p = (uint32_t)strtoul(argv[4], nullptr, 0);
  int threads = atoi(argv[5]), reps = atoi(argv[6]);
  if (threads < 1) threads = 1;
  if (k == "c5") return run_c5(n, threads, reps);
  if (k == "rec64")
    return run<Rec64>("rec64", n, threads, reps,
                      [=](Rec64 &o, uint64_t i) { o = make_rec64(s, i); });
  if (k == "recs")
    return run<RecS>("recs", n, threads, reps,
                     [=](RecS &o, uint64_t i) { o = make_recs(s, i, p); });
  if (k == "outer")
    return run<Outer>("outer", n, threads, reps,
                      [=](Outer &o, uint64_t i) { o = make_outer(s, i, p); });
  if (k == "var")
    return run<Var>("var", n, threads, reps, [=](Var &o, uint64_t i) { fill(o, s, i, p); });
  fprintf(stderr, "unknown case\n");
  return 2;
}
