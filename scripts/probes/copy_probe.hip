// Micro-benchmark: variants of the shifted stream copy behind C2.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u v4u_u __attribute__((aligned(1)));

__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t r) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * r));
}
template <int R> __device__ __forceinline__ v4u f16(const v4u &a, const v4u &b) {
  if constexpr (R == 0) return a; else {
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  constexpr int q = R >> 2, r = R & 3; v4u o;
  if constexpr (r == 0) { o.x = w[q]; o.y = w[q+1]; o.z = w[q+2]; o.w = w[q+3]; }
  else { o.x = funnel(w[q], w[q+1], r); o.y = funnel(w[q+1], w[q+2], r); o.z = funnel(w[q+2], w[q+3], r); o.w = funnel(w[q+3], w[q+4], r);} return o; }
}
__device__ __forceinline__ v4u shfl_next(const v4u &v, uint32_t lane) {
  const int addr = (int)(((lane + 1) & 63) << 2); v4u o;
  o.x = __builtin_amdgcn_ds_bpermute(addr, (int)v.x); o.y = __builtin_amdgcn_ds_bpermute(addr, (int)v.y);
  o.z = __builtin_amdgcn_ds_bpermute(addr, (int)v.z); o.w = __builtin_amdgcn_ds_bpermute(addr, (int)v.w); return o; }
__device__ __forceinline__ v4u rl0(const v4u &v) { v4u o;
  o.x = __builtin_amdgcn_readlane((int)v.x, 0); o.y = __builtin_amdgcn_readlane((int)v.y, 0);
  o.z = __builtin_amdgcn_readlane((int)v.z, 0); o.w = __builtin_amdgcn_readlane((int)v.w, 0); return o; }

template <class T> __device__ __forceinline__ T ld(const T* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }
template <class T> __device__ __forceinline__ void st(T v, T* p, bool nt) { if (nt) __builtin_nontemporal_store(v, p); else *p = v; }

// variant 0: funnel + bpermute; 1: unaligned loads; 2: pure aligned copy
template <int VAR, int U, int NTL, int NTS, int R>
__global__ __launch_bounds__(256) void k(v4u* __restrict__ dst, const uint8_t* __restrict__ srcb, uint64_t nk) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint64_t tile = 64ull * U;
  const v4u* src = (const v4u*)srcb;  // aligned base
  for (uint64_t t0 = wid * tile; t0 + tile <= nk; t0 += nw * tile) {
    if constexpr (VAR == 1) {
      v4u c[U];
#pragma unroll
      for (int j = 0; j < U; ++j) c[j] = NTL ? __builtin_nontemporal_load((const v4u_u*)(srcb + 16 * (t0 + j * 64 + lane) + R)) : *(const v4u_u*)(srcb + 16 * (t0 + j * 64 + lane) + R);
#pragma unroll
      for (int j = 0; j < U; ++j) st(c[j], &dst[t0 + j * 64 + lane], NTS);
    } else {
      v4u c[U];
#pragma unroll
      for (int j = 0; j < U; ++j) c[j] = ld(&src[t0 + j * 64 + lane], NTL);
      if constexpr (VAR == 2 || R == 0) {
#pragma unroll
        for (int j = 0; j < U; ++j) st(c[j], &dst[t0 + j * 64 + lane], NTS);
      } else {
        const v4u extra = src[t0 + tile];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const v4u l0 = (j + 1 < U) ? rl0(c[j + 1]) : extra;
          const v4u nb = shfl_next(c[j], lane);
          const v4u nx = lane == 63 ? l0 : nb;
          st(f16<R>(c[j], nx), &dst[t0 + j * 64 + lane], NTS);
        }
      }
    }
  }
}

template <int VAR, int U, int NTL, int NTS, int R>
void run(const char* name, v4u* d, const uint8_t* s, uint64_t nk, int blocks) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  k<VAR, U, NTL, NTS, R><<<blocks, 256>>>(d, s, nk);
  hipDeviceSynchronize();
  const int reps = 10;
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) k<VAR, U, NTL, NTS, R><<<blocks, 256>>>(d, s, nk);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= reps;
  printf("%-34s blocks=%6d  %.3f ms  %.1f GB/s\n", name, blocks, ms, 2.0 * nk * 16 / ms / 1e6);
}

int main() {
  const uint64_t bytes = 6400000000ull;
  uint8_t *s, *d;
  hipMalloc(&s, bytes + 4096); hipMalloc(&d, bytes + 4096);
  hipMemset(s, 1, bytes + 4096); hipMemset(d, 0, bytes + 4096);
  const uint64_t nk = bytes / 16 - 1024;
  const uint64_t full8 = nk / (64 * 8) / 4, full16 = nk / (64 * 16) / 4;
  for (int blocks : {32768}) {
    run<1, 16, 0, 0, 7>("unaligned R7 U16 dst+16 (warm)", (v4u*)(d + 16), s, nk, blocks);
    run<1, 16, 0, 0, 7>("unaligned R7 U16 dst+16", (v4u*)(d + 16), s, nk, blocks);
    run<1, 16, 1, 0, 7>("unaligned R7 U16 dst+16 ntload", (v4u*)(d + 16), s, nk, blocks);
    run<1, 16, 0, 1, 7>("unaligned R7 U16 dst+16 ntstore", (v4u*)(d + 16), s, nk, blocks);
    run<1, 16, 1, 1, 7>("unaligned R7 U16 dst+16 nt both", (v4u*)(d + 16), s, nk, blocks);
    run<2, 16, 0, 0, 0>("pure copy U16 dst+16", (v4u*)(d + 16), s, nk, blocks);
    run<2, 16, 0, 1, 0>("pure copy U16 dst+16 ntstore", (v4u*)(d + 16), s, nk, blocks);
    run<2, 16, 1, 1, 0>("pure copy U16 dst+16 nt both", (v4u*)(d + 16), s, nk, blocks);
    run<1, 16, 0, 0, 7>("unaligned R7 U16 dst+16 (again)", (v4u*)(d + 16), s, nk, blocks);
  }
  return 0;
}
