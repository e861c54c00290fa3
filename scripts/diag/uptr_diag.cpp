// diagnostic: which device record bytes of a VECTOR decode differ between a
// zero-filled and a 0xAB-filled output (fields the decoder leaves unwritten)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include <ylt/struct_pack_gpu.hpp>
using namespace struct_pack::gpu;
struct RecS { int32_t id; std::string name; double v; };
struct Inner { int32_t x; float y; };
struct UPtrRec { int32_t id; std::unique_ptr<std::string> s; std::unique_ptr<Inner> p; std::unique_ptr<std::vector<int32_t>> v; std::unique_ptr<RecS> r; };
int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 3000;
  std::vector<UPtrRec> batch;
  for (int i = 0; i < N; ++i) {
    UPtrRec u;
    u.id = i * 3 - 7;
    if (i % 3) u.s = std::make_unique<std::string>(std::string(i % 17, (char)('a' + i % 26)));
    if (i % 2) u.p = std::make_unique<Inner>(Inner{i, 0.5f * i});
    if (i % 5 != 1) u.v = std::make_unique<std::vector<int32_t>>(std::vector<int32_t>(i % 9, i));
    if (i % 4 == 0) u.r = std::make_unique<RecS>(RecS{i, std::string(i % 20, 'q'), 0.25 * i});
    batch.push_back(std::move(u));
  }
  const std::string wire = serialize<std::string>(batch);
  auto &c = device::thread_codec<UPtrRec, 0>();
  const auto &L = c.layout();
  device::buffer dw(wire.size() + 16);
  device::copy(dw.data(), wire.data(), wire.size(), SPK_COPY_H2D, c.stream());
  std::vector<uint8_t> out[2];
  std::size_t cap = wire.size() / c.min_record_wire() + 1;
  for (int f = 0; f < 2; ++f) {
    auto b = c.alloc_for_wire(wire.size(), cap);
    std::vector<uint8_t> fill(cap * L.rec_stride, f ? 0xAB : 0);
    device::copy(b.recs.data(), fill.data(), fill.size(), SPK_COPY_H2D, c.stream());
    for (uint32_t k = 0; k < c.n_spans(); ++k) {
      std::vector<uint8_t> hf(b.heap_elems[k] * c.span_elem(k), f ? 0xAB : 0);
      device::copy(b.heaps[k].data(), hf.data(), hf.size(), SPK_COPY_H2D, c.stream());
    }
    device::sync(c.stream());
    spk_dresult_t r = c.decode(b, dw.data(), wire.size(), SPK_MODE_VECTOR);
    std::printf("fill %d errc %d count %lu consumed %lu/%zu repaired %u seq %u cap %zu\n", f, r.errc,
                (unsigned long)r.count, (unsigned long)r.consumed, wire.size(), r.tiles_repaired,
                r.tiles_sequential, cap);
    for (uint32_t k = 0; k < c.n_spans(); ++k) std::printf("  heap %u used %lu cap %lu\n", k, (unsigned long)r.heap_used[k], (unsigned long)b.heap_elems[k]);
    out[f].resize(N * L.rec_stride);
    device::copy(out[f].data(), b.recs.data(), out[f].size(), SPK_COPY_D2H, c.stream());
    device::sync(c.stream());
  }
  int shown = 0, ndiff = 0;
  for (int i = 0; i < N; ++i)
    for (uint32_t o = 0; o < L.rec_stride; ++o)
      if (out[0][i * L.rec_stride + o] != out[1][i * L.rec_stride + o]) {
        ++ndiff;
        if (shown++ < 40) std::printf("rec %d off %u: %02x vs %02x\n", i, o, out[0][i * L.rec_stride + o], out[1][i * L.rec_stride + o]);
      }
  std::printf("differing bytes: %d\n", ndiff);
  // relevant fields vs the batch (fill 1)
  int bad = 0;
  auto u32 = [&](int i, int o) { uint32_t v; std::memcpy(&v, &out[1][i * L.rec_stride + o], 4); return v; };
  auto u64 = [&](int i, int o) { uint64_t v; std::memcpy(&v, &out[1][i * L.rec_stride + o], 8); return v; };
  for (int i = 0; i < N && bad < 20; ++i) {
    const auto &u = batch[i];
    bool ok = u32(i, 4) == (u.s ? 1u : 0u) && u32(i, 24) == (u.p ? 1u : 0u) && u32(i, 40) == (u.v ? 1u : 0u) && u32(i, 56) == (u.r ? 1u : 0u);
    if (ok && u.s) ok = u32(i, 8) == u.s->size();
    if (ok && u.v) ok = u32(i, 44) == u.v->size();
    if (ok && u.r) ok = u32(i, 64) == u.r->name.size();
    if (!ok) { ++bad; std::printf("rec %d: has %u %u %u %u  s.n %u v.n %u r.n %u r.off %lu\n", i, u32(i,4), u32(i,24), u32(i,40), u32(i,56), u32(i,8), u32(i,44), u32(i,64), (unsigned long)u64(i,72)); }
  }
  std::printf("bad records: %d\n", bad);
}
