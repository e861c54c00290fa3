// spk_synth.hip — device restatement of the seeded record generator of
// oracle/ref/types.hpp (used by the golden generator built against the
// reference), so the GPU box regenerates bit-identical inputs for the
// full-size BASELINE configs and compares digests. Bench/test support only;
// it is exported through the same C ABI for convenience.
#include "spk_internal.hpp"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t i, uint64_t k) {
  return mix64(seed + (i * 64 + k + 1) * 0x9E3779B97F4A7C15ULL);
}
__device__ __forceinline__ float rf(uint64_t r) {
  return (float)(int32_t)(uint32_t)r / 65536.0f;
}
__device__ __forceinline__ double rd(uint64_t r) {
  return (double)(int32_t)(uint32_t)r / 65536.0;
}

struct Rec64 {
  int32_t i[4];
  float f[4];
  double d[4];
};
struct RecSDev {  // schema.flatten(RecS): id, name.n, name.off, v
  int32_t id;
  uint32_t n;
  uint64_t off;
  double v;
};
struct OuterDev {  // schema.flatten(Outer): key, items.n, items.off
  int64_t key;
  uint32_t n;
  uint32_t pad;
  uint64_t off;
};

__global__ void synth_rec64(uint64_t seed, uint64_t first, uint64_t n, Rec64 *out) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t;
    Rec64 r;
    for (int k = 0; k < 4; ++k) r.i[k] = (int32_t)(uint32_t)rnd(seed, i, k);
    for (int k = 0; k < 4; ++k) r.f[k] = rf(rnd(seed, i, 4 + k));
    for (int k = 0; k < 4; ++k) r.d[k] = rd(rnd(seed, i, 8 + k));
    out[t] = r;
  }
}

// RECS lengths (types.hpp chars_len): a plain param < 65536 is U[0, param];
// otherwise maxlen in bits 0-15, minlen in bits 16-30, bit 31 = raw bytes
__device__ __forceinline__ uint32_t recs_len(uint64_t seed, uint64_t i, uint32_t param) {
  if (param < 0x10000u) return (uint32_t)(rnd(seed, i, 1) % (uint64_t)(param + 1));
  const uint32_t mx = param & 0xFFFFu, mn = (param >> 16) & 0x7FFFu;
  return mn + (uint32_t)(rnd(seed, i, 1) % (uint64_t)(mx - mn + 1));
}

__global__ void synth_counts(int kind, uint64_t seed, uint64_t first, uint64_t n,
                             uint32_t param, uint64_t *cnt) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs)
    cnt[t] = kind == SPK_SYNTH_RECS ? recs_len(seed, first + t, param)
                                    : rnd(seed, first + t, 1) % (uint64_t)(param + 1);
}

__global__ void synth_recs(uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                           RecSDev *out, uint8_t *heap, const uint64_t *hoff) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t;
    RecSDev r;
    r.id = (int32_t)(uint32_t)rnd(seed, i, 0);
    r.n = recs_len(seed, i, param);
    r.off = hoff[t];
    r.v = rd(rnd(seed, i, 60));
    out[t] = r;
    uint8_t *dst = heap + r.off;
    const bool raw = (param >> 31) != 0;
    for (uint32_t j = 0; j < r.n; ++j) {
      const uint64_t w = rnd(seed, i, 2 + (j >> 3) % 56);
      const uint32_t b = (uint32_t)((w >> ((j & 7) * 8)) & 0xFF);
      dst[j] = (uint8_t)(raw ? b : 'a' + b % 26);
    }
  }
}

__global__ void synth_outer(uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                            OuterDev *out, uint8_t *heap, const uint64_t *hoff) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t;
    OuterDev o;
    o.key = (int64_t)rnd(seed, i, 0);
    o.n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(param + 1));
    o.pad = 0;
    o.off = hoff[t];
    out[t] = o;
    int32_t *dst = reinterpret_cast<int32_t *>(heap + o.off * 8);
    for (uint32_t j = 0; j < o.n; ++j) {
      const uint64_t w = rnd(seed, i, 2 + j % 62);
      const uint64_t w2 = mix64(w ^ (uint64_t)j);
      dst[2 * j] = (int32_t)(uint32_t)w2;
      const float y = rf(w2 >> 32);
      dst[2 * j + 1] = __float_as_int(y);
    }
  }
}

// ---- C5 coro_rpc payload shapes (types.hpp rpcb::rect / person, make_ints)
struct PersonDev {  // schema.flatten(person): id, name.n, name.off, age, salary
  int32_t id;
  uint32_t n;
  uint64_t off;
  int32_t age;
  uint32_t pad;
  double salary;
};
struct IntsDev {  // schema.flatten(std::vector<int32_t>): value.n, value.off
  uint32_t n;
  uint32_t pad;
  uint64_t off;
};

__global__ void synth_rpcrect(uint64_t seed, uint64_t first, uint64_t n, double *out) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs)
    for (int k = 0; k < 4; ++k) out[4 * t + k] = rd(rnd(seed, first + t, k));
}

__global__ void synth_person(uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                             PersonDev *out, uint8_t *heap, const uint64_t *hoff) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t;
    PersonDev r;
    r.id = (int32_t)(uint32_t)rnd(seed, i, 0);
    r.n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(param + 1));
    r.off = hoff[t];
    r.age = (int32_t)(rnd(seed, i, 60) % 100);
    r.pad = 0;
    r.salary = rd(rnd(seed, i, 61));
    out[t] = r;
    uint8_t *dst = heap + r.off;
    for (uint32_t j = 0; j < r.n; ++j) {
      const uint64_t w = rnd(seed, i, 2 + (j >> 3) % 56);
      dst[j] = (uint8_t)('a' + ((w >> ((j & 7) * 8)) & 0xFF) % 26);
    }
  }
}

__global__ void synth_ints(uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                           IntsDev *out, uint8_t *heap, const uint64_t *hoff) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t;
    IntsDev r;
    r.n = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(param + 1));
    r.pad = 0;
    r.off = hoff[t];
    out[t] = r;
    int32_t *dst = reinterpret_cast<int32_t *>(heap + r.off * 4);
    const uint64_t base = rnd(seed, i, 2);
    for (uint32_t j = 0; j < r.n; ++j) dst[j] = (int32_t)(uint32_t)mix64(base + j);
  }
}

// ---- the reference benchmark's Monster (types.hpp fill(Monster&)) -----------
// schema.flatten(Monster): 96-byte record, six heaps (name, inventory, weapon
// element records, weapon names, equipped.name, path); Weapon element record
// {u32 name.n, u64 name.off, i16 damage} = 24 bytes
constexpr int kMonHeaps = 6;
__device__ __forceinline__ uint32_t tag_len(uint64_t h) { return (uint32_t)(h % 13); }
__device__ __forceinline__ void tag_fill(uint8_t *d, uint64_t h) {
  for (uint32_t k = 0; k < tag_len(h); ++k) {
    const uint64_t w = mix64(h + (k >> 3));
    d[k] = (uint8_t)('a' + ((w >> ((k & 7) * 8)) & 0xFF) % 26);
  }
}
__device__ __forceinline__ uint64_t elem_word(uint64_t seed, uint64_t i, uint64_t j) {
  return mix64(rnd(seed, i, 2 + j % 56) ^ j);
}
// counts per record: [0] name chars, [1] inventory chars, [2] weapons,
// [3] weapon-name chars, [4] equipped.name chars, [5] path points
__global__ void synth_monster_counts(uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                                     uint64_t *cnt) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t, r9 = rnd(seed, i, 9);
    const uint32_t nw = (uint32_t)((r9 >> 8) % 5);
    uint64_t wl = 0;
    for (uint32_t j = 0; j < nw; ++j) wl += tag_len(elem_word(seed, i, j));
    cnt[t] = rnd(seed, i, 1) % (uint64_t)(param + 1);
    cnt[n + t] = tag_len(rnd(seed, i, 8));
    cnt[2 * n + t] = nw;
    cnt[3 * n + t] = wl;
    cnt[4 * n + t] = tag_len(rnd(seed, i, 10));
    cnt[5 * n + t] = (r9 >> 16) % 9;
  }
}
struct MonHeaps {
  uint8_t *h[kMonHeaps];
};
__global__ void synth_monster(uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                              uint8_t *recs, MonHeaps H, const uint64_t *off) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gs) {
    const uint64_t i = first + t;
    uint8_t *r = recs + t * 96;
    for (int q = 0; q < 12; ++q) reinterpret_cast<uint64_t *>(r)[q] = 0;
    float *pos = reinterpret_cast<float *>(r);
    for (int k = 0; k < 3; ++k) pos[k] = rf(rnd(seed, i, 4 + k));
    const uint64_t r7 = rnd(seed, i, 7), r9 = rnd(seed, i, 9), r10 = rnd(seed, i, 10);
    *reinterpret_cast<int16_t *>(r + 12) = (int16_t)r7;
    *reinterpret_cast<int16_t *>(r + 14) = (int16_t)(r7 >> 16);
    // name: make_chars (words 2.. of the record)
    const uint32_t nl = (uint32_t)(rnd(seed, i, 1) % (uint64_t)(param + 1));
    *reinterpret_cast<uint32_t *>(r + 16) = nl;
    *reinterpret_cast<uint64_t *>(r + 24) = off[t];
    for (uint32_t j = 0; j < nl; ++j) {
      const uint64_t w = rnd(seed, i, 2 + (j >> 3) % 56);
      H.h[0][off[t] + j] = (uint8_t)('a' + ((w >> ((j & 7) * 8)) & 0xFF) % 26);
    }
    const uint64_t r8 = rnd(seed, i, 8);
    *reinterpret_cast<uint32_t *>(r + 32) = tag_len(r8);
    *reinterpret_cast<uint64_t *>(r + 40) = off[n + t];
    tag_fill(H.h[1] + off[n + t], r8);
    r[48] = (uint8_t)(r9 % 3);
    const uint32_t nw = (uint32_t)((r9 >> 8) % 5);
    *reinterpret_cast<uint32_t *>(r + 52) = nw;
    *reinterpret_cast<uint64_t *>(r + 56) = off[2 * n + t];
    uint64_t wo = off[3 * n + t];
    for (uint32_t j = 0; j < nw; ++j) {
      const uint64_t h = elem_word(seed, i, j);
      uint8_t *e = H.h[2] + (off[2 * n + t] + j) * 24;
      for (int q = 0; q < 3; ++q) reinterpret_cast<uint64_t *>(e)[q] = 0;
      *reinterpret_cast<uint32_t *>(e) = tag_len(h);
      *reinterpret_cast<uint64_t *>(e + 8) = wo;
      *reinterpret_cast<int16_t *>(e + 16) = (int16_t)(h >> 32);
      tag_fill(H.h[3] + wo, h);
      wo += tag_len(h);
    }
    *reinterpret_cast<uint32_t *>(r + 64) = tag_len(r10);
    *reinterpret_cast<uint64_t *>(r + 72) = off[4 * n + t];
    tag_fill(H.h[4] + off[4 * n + t], r10);
    *reinterpret_cast<int16_t *>(r + 80) = (int16_t)(r10 >> 40);
    const uint32_t np = (uint32_t)((r9 >> 16) % 9);
    *reinterpret_cast<uint32_t *>(r + 84) = np;
    *reinterpret_cast<uint64_t *>(r + 88) = off[5 * n + t];
    float *pt = reinterpret_cast<float *>(H.h[5] + off[5 * n + t] * 12);
    for (uint32_t j = 0; j < np; ++j) {
      const uint64_t w = mix64(rnd(seed, i, 11) + j);
      pt[3 * j] = rf(w);
      pt[3 * j + 1] = rf(w >> 32);
      pt[3 * j + 2] = rf(mix64(w));
    }
  }
}

unsigned grid_of(uint64_t n) {
  uint64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (unsigned)(b ? b : 1);
}

}  // namespace

extern "C" int spk_synth_counts(int kind, uint64_t seed, uint64_t first, uint64_t n,
                                uint32_t param, uint64_t *d_counts, void *stream) {
  if (!d_counts || (kind != SPK_SYNTH_RECS && kind != SPK_SYNTH_OUTER &&
                    kind != SPK_SYNTH_PERSON && kind != SPK_SYNTH_INTS))
    return SPK_E_ARG;
  SPK_LAUNCH(synth_counts, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, kind,
                     seed, first, n, param, d_counts);
  return hipGetLastError() == hipSuccess ? SPK_OK : SPK_E_HIP;
}

extern "C" int spk_synth(int kind, uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                         void *d_recs, void *d_heap, const uint64_t *d_heap_offsets,
                         void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!d_recs && n) return SPK_E_ARG;
  switch (kind) {
    case SPK_SYNTH_REC64:
      SPK_LAUNCH(synth_rec64, dim3(grid_of(n)), dim3(256), 0, s, seed, first, n,
                         (Rec64 *)d_recs);
      break;
    case SPK_SYNTH_RECS:
      if (!d_heap_offsets) return SPK_E_ARG;
      SPK_LAUNCH(synth_recs, dim3(grid_of(n)), dim3(256), 0, s, seed, first, n, param,
                         (RecSDev *)d_recs, (uint8_t *)d_heap, d_heap_offsets);
      break;
    case SPK_SYNTH_OUTER:
      if (!d_heap_offsets) return SPK_E_ARG;
      SPK_LAUNCH(synth_outer, dim3(grid_of(n)), dim3(256), 0, s, seed, first, n, param,
                         (OuterDev *)d_recs, (uint8_t *)d_heap, d_heap_offsets);
      break;
    case SPK_SYNTH_RPCRECT:
      SPK_LAUNCH(synth_rpcrect, dim3(grid_of(n)), dim3(256), 0, s, seed, first, n,
                         (double *)d_recs);
      break;
    case SPK_SYNTH_PERSON:
      if (!d_heap_offsets) return SPK_E_ARG;
      SPK_LAUNCH(synth_person, dim3(grid_of(n)), dim3(256), 0, s, seed, first, n,
                         param, (PersonDev *)d_recs, (uint8_t *)d_heap, d_heap_offsets);
      break;
    case SPK_SYNTH_INTS:
      if (!d_heap_offsets) return SPK_E_ARG;
      SPK_LAUNCH(synth_ints, dim3(grid_of(n)), dim3(256), 0, s, seed, first, n, param,
                         (IntsDev *)d_recs, (uint8_t *)d_heap, d_heap_offsets);
      break;
    default:
      return SPK_E_ARG;
  }
  return hipGetLastError() == hipSuccess ? SPK_OK : SPK_E_HIP;
}

// multi-heap kinds (SPK_SYNTH_MONSTER): d_counts / d_heap_offsets are
// [heaps][n] columns (elements per record; exclusive prefix sums of them)
extern "C" int spk_synth_counts_ex(int kind, uint64_t seed, uint64_t first, uint64_t n,
                                   uint32_t param, uint64_t *d_counts, void *stream) {
  if (kind != SPK_SYNTH_MONSTER || !d_counts) return SPK_E_ARG;
  SPK_LAUNCH(synth_monster_counts, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, seed,
             first, n, param, d_counts);
  return hipGetLastError() == hipSuccess ? SPK_OK : SPK_E_HIP;
}

extern "C" int spk_synth_ex(int kind, uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                            void *d_recs, void *const *d_heaps, const uint64_t *d_heap_offsets,
                            void *stream) {
  if (kind != SPK_SYNTH_MONSTER || (n && (!d_recs || !d_heaps || !d_heap_offsets)))
    return SPK_E_ARG;
  MonHeaps H;
  for (int k = 0; k < kMonHeaps; ++k) H.h[k] = (uint8_t *)(d_heaps ? d_heaps[k] : nullptr);
  SPK_LAUNCH(synth_monster, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, seed, first, n,
             param, (uint8_t *)d_recs, H, d_heap_offsets);
  return hipGetLastError() == hipSuccess ? SPK_OK : SPK_E_HIP;
}
