// Micro-benchmark: variants of the speculative chunk walk of the vector
// decode on a C3-shaped wire ([id:4][n:4][n bytes][f64], n in [0,48]).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 spec_probe.hip -o spec_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u v4u_una __attribute__((aligned(1)));
typedef uint32_t u32_una __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

constexpr uint32_t kPlaus = 4096;
constexpr uint32_t kExt = 4;

struct Out {
  uint16_t *P;
  uint32_t *Pn, *E, *En;
  unsigned long long *ctr;  // [0] tries [1] steps
};

__device__ __forceinline__ uint32_t rd_lds(const lds_u32 *d, uint32_t o) {
  const uint32_t sh = o & 3, i = o >> 2;
  return __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
}

// VAR 0: LDS region, P/E stores; 1: LDS, no stores; 2: global reads, stores;
// 3: LDS region, 32-bit offsets, stores; S = chunk bytes
template <int VAR, int S, int WAVES, int CTR>
__global__ __launch_bounds__(64 * WAVES) void spec(const uint8_t *__restrict__ wire, uint64_t len,
                                                   uint64_t p0, uint64_t nch, Out o, uint32_t lp) {
  constexpr uint32_t kRegionVec = (64 * S + 512) / 16;
  __shared__ v4u reg_s[WAVES][kRegionVec + 1];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t ch0 = ((uint64_t)blockIdx.x * WAVES + wv) * 64;
  if (ch0 >= nch) return;
  const uint64_t rs = p0 + ch0 * S;
  const uint64_t wend = rs + kRegionVec * 16 < len ? rs + kRegionVec * 16 : len;
  v4u *reg = reg_s[wv];
  if (VAR != 2 && VAR != 6 && VAR != 9) {
    for (uint32_t v = lane; v < kRegionVec; v += 64) {
      const uint64_t g = rs + 16ull * v;
      v4u val = {0u, 0u, 0u, 0u};
      if (g + 16 <= len) val = *reinterpret_cast<const v4u_una *>(wire + g);
      reg[v] = val;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const lds_u32 *d = (const lds_u32 *)reg;
  const uint64_t ch = ch0 + lane;
  const bool live = ch < nch;
  if (!CTR && !live) return;
  const uint64_t cs = p0 + (live ? ch : ch0) * S;
  const uint64_t ce = cs + S < len ? cs + S : len;
  uint16_t *Pl = o.P + ch * lp;
  uint32_t *El = o.E + ch * kExt;
  uint32_t np = 0, ne = 0;
  uint32_t tries = 0, steps = 0;
  auto cnt_at = [&](uint64_t x) -> uint32_t {
    if (VAR != 2 && VAR != 6 && VAR != 9 && x + 4 <= wend) return rd_lds(d, (uint32_t)(x - rs));
    return *reinterpret_cast<const u32_una *>(wire + x);
  };
  const uint32_t ntries = ch == 0 ? 1 : S;
  if (!live) {
  } else if (VAR < 4) {
  for (uint32_t t = 0; t < ntries; ++t) {
    uint64_t x = cs + t;
    if (x >= ce) break;
    ++tries;
    np = ne = 0;
    bool ok = true;
    for (;;) {
      if (x >= ce && ne == kExt) break;
      ++steps;
      uint64_t L = 0;
      if (x + 8 <= len) {
        const uint64_t c = cnt_at(x + 4);
        const uint64_t e = x + 8 + c + 8;
        L = e <= len ? e - x : 0;
      }
      if (ch != 0 && ((L == 0 && x < len) || L > kPlaus)) { ok = false; break; }
      if (VAR != 1) {
        if (x < ce) { if (np < lp) Pl[np] = (uint16_t)(x - cs); ++np; }
        else El[ne++] = (uint32_t)(x - cs);
      } else {
        if (x < ce) ++np; else ++ne;
      }
      if (!L) break;
      x += L;
    }
    if (ok) break;
  }
  } else if (VAR >= 8) {
    // flattened + 8-wide first-count prefilter while searching
    uint32_t t = 0;
    uint64_t x = cs;
    bool searching = ch != 0;
    bool done = cs >= ce;
    tries = 0;
    while (!done) {
      ++steps;
      if (searching) {
        // counts at cs+t+4+k, k=0..7: bytes [cs+t+4, cs+t+15)
        const uint64_t b0 = cs + t + 4;
        uint32_t m = 0;
        if (b0 + 16 <= wend && VAR == 8) {
          const uint32_t o0 = (uint32_t)(b0 - rs);
          const uint32_t i = o0 >> 2, sh = o0 & 3;
          const uint32_t d0 = d[i], d1 = d[i + 1], d2 = d[i + 2], d3 = d[i + 3];
          const uint32_t wd[3] = {__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                                  __builtin_amdgcn_alignbyte(d3, d2, sh)};
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t c = __builtin_amdgcn_alignbyte(wd[(k >> 2) + 1], wd[k >> 2], k & 3);
            m |= (c <= kPlaus - 16 ? 1u : 0u) << k;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint64_t xx = b0 + k;
            uint32_t c = ~0u;
            if (xx + 4 <= len) c = cnt_at(xx);
            m |= (c <= kPlaus - 16 ? 1u : 0u) << k;
          }
        }
        // candidates past the chunk end are not allowed
        const uint64_t rem = ce - (cs + t);
        if (rem < 8) m &= (1u << rem) - 1;
        if (!m) {
          t += 8;
          tries += 8;
          if (t >= ntries || cs + t >= ce) done = true;
          continue;
        }
        const uint32_t k = __builtin_ctz(m);
        t += k;
        tries += k + 1;
        x = cs + t;
        np = ne = 0;
        searching = false;
      }
      uint64_t L = 0;
      if (x + 8 <= len) {
        const uint64_t c = cnt_at(x + 4);
        const uint64_t e = x + 8 + c + 8;
        L = e <= len ? e - x : 0;
      }
      if (ch != 0 && ((L == 0 && x < len) || L > kPlaus)) {
        ++t;
        searching = true;
        if (t >= ntries || cs + t >= ce) done = true;
        continue;
      }
      if (x < ce) { if (np < lp) Pl[np] = (uint16_t)(x - cs); ++np; }
      else El[ne++] = (uint32_t)(x - cs);
      if (!L) break;
      x += L;
      if (x >= ce && ne == kExt) done = true;
    }
  } else {
    // flattened: one record step per iteration for every lane
    uint32_t t = 0;
    uint64_t x = cs;
    tries = 1;
    bool done = cs >= ce;
    while (!done) {
      ++steps;
      uint64_t L = 0;
      if (x + 8 <= len) {
        const uint64_t c = cnt_at(x + 4);
        const uint64_t e = x + 8 + c + 8;
        L = e <= len ? e - x : 0;
      }
      if (ch != 0 && ((L == 0 && x < len) || L > kPlaus)) {
        ++t;
        x = cs + t;
        np = ne = 0;
        ++tries;
        if (t >= ntries || x >= ce) { done = true; }
        continue;
      }
      if (x < ce) { if (np < lp) Pl[np] = (uint16_t)(x - cs); ++np; }
      else El[ne++] = (uint32_t)(x - cs);
      if (!L) break;
      x += L;
      if (x >= ce && ne == kExt) done = true;
    }
  }
  if (live) {
    o.Pn[ch] = np;
    o.En[ch] = ne;
  }
  if (CTR) {
    unsigned long long a = tries, b = steps;
    for (int k = 32; k > 0; k >>= 1) { a += __shfl_xor(a, k); b += __shfl_xor(b, k); }
    if (lane == 0) { atomicAdd(&o.ctr[0], a); atomicAdd(&o.ctr[1], b); }
  }
}

template <int VAR, int S, int WAVES>
int run(const char *name, const uint8_t *dw, uint64_t len, uint64_t p0, Out o) {
  const uint64_t nch = (len - p0 + S - 1) / S;
  const uint32_t lp = S / 16 + 2;
  const unsigned grid = (unsigned)((nch + 64 * WAVES - 1) / (64 * WAVES));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipMemset(o.ctr, 0, 16));
  hipLaunchKernelGGL((spec<VAR, S, WAVES, 1>), dim3(grid), dim3(64 * WAVES), 0, 0, dw, len, p0, nch, o, lp);
  CK(hipDeviceSynchronize());
  unsigned long long ctr[2];
  CK(hipMemcpy(ctr, o.ctr, 16, hipMemcpyDeviceToHost));
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((spec<VAR, S, WAVES, 0>), dim3(grid), dim3(64 * WAVES), 0, 0, dw, len, p0, nch, o, lp);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("%-28s S=%4d waves=%d chunks=%9llu  %8.3f ms  tries/chunk=%.2f steps/chunk=%.2f\n", name, S,
         WAVES, (unsigned long long)nch, ms / reps, (double)ctr[0] / nch, (double)ctr[1] / nch);
  return 0;
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ull;
  std::vector<uint8_t> h;
  h.reserve(n * 41 + 64);
  for (int i = 0; i < 9; ++i) h.push_back(0);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t id = (uint32_t)rnd();
    const uint32_t len = (uint32_t)(rnd() % 49);
    uint8_t b[8];
    memcpy(b, &id, 4);
    h.insert(h.end(), b, b + 4);
    memcpy(b, &len, 4);
    h.insert(h.end(), b, b + 4);
    for (uint32_t j = 0; j < len; ++j) h.push_back((uint8_t)('a' + rnd() % 26));
    const uint64_t v = rnd();
    memcpy(b, &v, 8);
    h.insert(h.end(), b, b + 8);
  }
  const uint64_t len = h.size();
  printf("wire %llu bytes, %llu records\n", (unsigned long long)len, (unsigned long long)n);
  uint8_t *dw;
  CK(hipMalloc(&dw, len + 64));
  CK(hipMemcpy(dw, h.data(), len, hipMemcpyHostToDevice));
  Out o;
  const uint64_t maxch = len / 64 + 2;
  CK(hipMalloc(&o.P, maxch * 8 * 2));
  CK(hipMalloc(&o.Pn, maxch * 4));
  CK(hipMalloc(&o.E, maxch * kExt * 4));
  CK(hipMalloc(&o.En, maxch * 4));
  CK(hipMalloc(&o.ctr, 16));
  const uint64_t p0 = 9;
  run<4, 256, 2>("flat lds", dw, len, p0, o);
  run<6, 256, 4>("flat global", dw, len, p0, o);
  run<6, 1024, 4>("flat global", dw, len, p0, o);
  run<8, 256, 2>("prefilter lds", dw, len, p0, o);
  run<9, 256, 4>("prefilter global", dw, len, p0, o);
  run<8, 128, 4>("prefilter lds", dw, len, p0, o);
  run<9, 512, 4>("prefilter global", dw, len, p0, o);
  run<9, 1024, 4>("prefilter global", dw, len, p0, o);
  run<9, 2048, 4>("prefilter global", dw, len, p0, o);
  return 0;
}
