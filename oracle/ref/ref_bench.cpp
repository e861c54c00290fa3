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
  if (k == "rec64")
    return run<Rec64>("rec64", n, threads, reps,
                      [=](Rec64 &o, uint64_t i) { o = make_rec64(s, i); });
  if (k == "recs")
    return run<RecS>("recs", n, threads, reps,
                     [=](RecS &o, uint64_t i) { o = make_recs(s, i, p); });
  if (k == "outer")
    return run<Outer>("outer", n, threads, reps,
                      [=](Outer &o, uint64_t i) { o = make_outer(s, i, p); });
  fprintf(stderr, "unknown case\n");
  return 2;
}
