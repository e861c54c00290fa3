// C2 timing outside torch: the library's spk_plan/spk_encode/spk_decode on
// hipMalloc'ed buffers vs the same copy done by a hand kernel, to separate
// kernel cost from harness effects. Probe only (not shipped).
#include <cstdio>
#include <cstdint>
#include "ylt/struct_pack.hpp"
#include "../../oracle/ref/types.hpp"

int main(int argc, char **argv) {
  const uint64_t n = 100000000ull;
  const spk_layout L = struct_pack::make_spk_layout<std::vector<Rec64>::value_type>();
  void *recs, *wire, *dec, *ws, *plan, *res;
  size_t wsb = spk_workspace_bytes(&L, SPK_MODE_VECTOR, n, n * 64 + 64);
  hipMalloc(&recs, n * 64); hipMalloc(&wire, n * 64 + 64); hipMalloc(&dec, n * 64);
  hipMalloc(&ws, wsb); hipMalloc(&plan, 64); hipMalloc(&res, 256);
  spk_synth(SPK_SYNTH_REC64, 0x5EED0002, 0, n, 0, recs, nullptr, nullptr, nullptr);
  hipMemset(wire, 0, n * 64 + 64); hipMemset(dec, 0, n * 64);
  hipDeviceSynchronize();
  auto step = [&](int what) {
    if (what & 1) {
      spk_plan(&L, SPK_MODE_VECTOR, n, recs, (spk_plan_t *)plan, ws, wsb, nullptr);
      spk_encode(&L, SPK_MODE_VECTOR, n, recs, nullptr, (spk_plan_t *)plan, wire, n * 64 + 64,
                 nullptr, ws, wsb, nullptr);
    }
    if (what & 2)
      { int rc = spk_decode(&L, SPK_MODE_VECTOR, wire, n * 64 + 9, nullptr, 0, dec, n, nullptr, nullptr,
                 (spk_dresult_t *)res, nullptr, ws, wsb, nullptr); if (rc) printf("decode rc %d\n", rc); }
  };
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep)
    for (int what : {1, 2, 3}) {
      for (int i = 0; i < 3; ++i) step(what);
      hipEventRecord(a);
      for (int i = 0; i < 20; ++i) step(what);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("rep %d %s: %.3f ms per step\n", rep, what == 1 ? "encode" : what == 2 ? "decode" : "enc+dec", ms / 20);
    }
  return 0;
}
