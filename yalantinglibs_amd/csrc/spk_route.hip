// spk_route.hip — routing a mixed-type batch of coro_rpc request frames by
// function id, in arrival order (include/spk_codec.h: spk_route_frames).
//
// The reference server handles one frame at a time: it reads the 20-byte
// req_header (coro_rpc_protocol.hpp:60-79), takes function_id
// (coro_rpc_protocol.hpp:95) and looks the handler up in its map
// (router.hpp:226-240), which fixes the argument types the payload is
// deserialized into. Here a batch of frames is split per function id at
// once: a stable partition (arrival order kept within each key), so that
// each type's frames are decoded by one launch (spk_decode_frames) and the
// result lines up with a sequential dispatch of the same frames.
//
// Three kernels, no atomics: per block a histogram of keys (wave ballots),
// one block scans the histograms per key, and the scatter recomputes each
// frame's rank among the block's frames of its key by the same ballots.
#include "spk_internal.hpp"

namespace {

constexpr uint32_t kRT = 256;                  // frames per block (one per lane)
constexpr uint32_t kRW = kRT / 64;             // waves per block
constexpr uint32_t kRK = SPK_MAX_ROUTES + 1;   // keys + "unrouted"

struct RouteArgs {
  uint64_t n, wire_len;
  uint32_t key_off, nk;  // nk = n_keys (list nk = unrouted)
  uint32_t keys[SPK_MAX_ROUTES];
  uint32_t chk;          // header check on (spk_route_hdr)
  spk_route_hdr h;
  uint64_t *beg[kRK];
  uint64_t *end[kRK];
  uint64_t *idx[kRK];
};

__device__ __forceinline__ uint32_t ld_u32le(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// the reference server's header checks (coro_rpc_protocol.hpp:98-117) and
// the frame size they imply: head + length + attach_length
__device__ __forceinline__ bool header_ok(const RouteArgs &a, const uint8_t *f, uint64_t size) {
  const spk_route_hdr &h = a.h;
  if (size < h.head_len) return false;
  if (h.magic >= 0 && f[0] != (uint32_t)h.magic) return false;
  if (h.max_version >= 0 && f[1] > (uint32_t)h.max_version) return false;
  if (h.serialize_type >= 0 && f[2] != (uint32_t)h.serialize_type) return false;
  uint64_t want = (uint64_t)h.head_len + ld_u32le(f + h.len_off);
  if (h.attach_off != SPK_FRAME_NONE) want += ld_u32le(f + h.attach_off);
  return want == size;
}

// key slot of frame i: 0..nk-1, or nk when the key is unknown / unreadable
// (or, with the header check, the frame is not one the server would dispatch)
__device__ __forceinline__ uint32_t frame_slot(const RouteArgs &a, const uint8_t *wire,
                                               const uint64_t *offs, uint64_t i) {
  const uint64_t b = offs[i], e = offs[i + 1];
  if (e < b || e > a.wire_len || e - b < (uint64_t)a.key_off + 4) return a.nk;
  if (a.chk && !header_ok(a, wire + b, e - b)) return a.nk;
  const uint32_t key = ld_u32le(wire + b + a.key_off);
  for (uint32_t k = 0; k < a.nk; ++k)
    if (a.keys[k] == key) return k;
  return a.nk;
}

// per block: frames per key slot -> bcnt[slot][block]; slots -> tslot[i]
__global__ __launch_bounds__(kRT) void route_count(RouteArgs a, const uint8_t *__restrict__ wire,
                                                   const uint64_t *__restrict__ offs,
                                                   uint8_t *__restrict__ tslot,
                                                   uint64_t *__restrict__ bcnt) {
  __shared__ uint32_t wc[kRW][kRK];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t i = (uint64_t)blockIdx.x * kRT + threadIdx.x;
  const uint32_t t = i < a.n ? frame_slot(a, wire, offs, i) : kRK;  // kRK: no frame
  if (i < a.n) tslot[i] = (uint8_t)t;
  for (uint32_t k = 0; k <= a.nk; ++k) {
    const uint64_t m = __ballot(t == k);
    if (lane == 0) wc[wv][k] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (threadIdx.x <= a.nk) {
    uint64_t s = 0;
    for (uint32_t w = 0; w < kRW; ++w) s += wc[w][threadIdx.x];
    bcnt[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
  }
}

// inclusive wave64 prefix sum on the DPP network (row_shr 1/2/4/8, then
// row_bcast 15 / 31)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK,
                                                             0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL,
                                                             ROW_MASK, 0xf, false);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t incl_scan64(uint64_t v) {
  v += dpp64<0x111, 0xf>(v);
  v += dpp64<0x112, 0xf>(v);
  v += dpp64<0x114, 0xf>(v);
  v += dpp64<0x118, 0xf>(v);
  v += dpp64<0x142, 0xa>(v);
  v += dpp64<0x143, 0xc>(v);
  return v;
}

// one block: per slot, exclusive prefix over blocks (in place) and the total.
// Thread j owns a run of consecutive blocks (summed serially), so each slot
// takes one block-wide scan however many routing blocks there are.
constexpr uint32_t kScanT = 1024;
__global__ __launch_bounds__(kScanT) void route_scan(uint64_t nblocks, uint32_t nk,
                                                     uint64_t *__restrict__ bcnt,
                                                     uint64_t *__restrict__ counts) {
  __shared__ uint64_t sh[kScanT / 64];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t per = (nblocks + kScanT - 1) / kScanT;
  const uint64_t b0 = (uint64_t)threadIdx.x * per;
  const uint64_t b1 = b0 + per < nblocks ? b0 + per : nblocks;
  for (uint32_t k = 0; k <= nk; ++k) {
    uint64_t run = 0;
    uint64_t *col = bcnt + (uint64_t)k * nblocks;
    for (uint64_t b = b0; b < b1; ++b) run += col[b];
    const uint64_t inc = incl_scan64(run);
    if (lane == 63) sh[wv] = inc;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
    for (uint32_t w = 0; w < kScanT / 64; ++w) {
      if (w < wv) wbase += sh[w];
      tot += sh[w];
    }
    __syncthreads();
    uint64_t x = wbase + inc - run;  // exclusive prefix of this thread's run
    for (uint64_t b = b0; b < b1; ++b) {
      const uint64_t c = col[b];
      col[b] = x;
      x += c;
    }
    if (threadIdx.x == 0) counts[k] = tot;
  }
}

__global__ __launch_bounds__(kRT) void route_scatter(RouteArgs a,
                                                     const uint8_t *__restrict__ wire,
                                                     const uint64_t *__restrict__ offs,
                                                     const uint8_t *__restrict__ tslot,
                                                     const uint64_t *__restrict__ bcnt) {
  __shared__ uint32_t wc[kRW][kRK];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t i = (uint64_t)blockIdx.x * kRT + threadIdx.x;
  const uint32_t t = i < a.n ? tslot[i] : kRK;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t rank = 0;
  for (uint32_t k = 0; k <= a.nk; ++k) {
    const uint64_t m = __ballot(t == k);
    if (t == k) rank = (uint32_t)__popcll(m & below);
    if (lane == 0) wc[wv][k] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (t >= kRK || !a.beg[t]) return;
  uint64_t pos = bcnt[(uint64_t)t * gridDim.x + blockIdx.x] + rank;
  for (uint32_t w = 0; w < wv; ++w) pos += wc[w][t];
  const uint64_t b = offs[i];
  a.beg[t][pos] = b;
  if (a.end[t]) {
    uint64_t e = offs[i + 1];
    // checked frames: the message ends before the attachment
    if (a.chk && t < a.nk) e = b + a.h.head_len + ld_u32le(wire + b + a.h.len_off);
    a.end[t][pos] = e;
  }
  if (a.idx[t]) a.idx[t][pos] = i;
}

__global__ void copy_frame_field(uint8_t *__restrict__ dst, const uint64_t *__restrict__ doffs,
                                 uint32_t doff, const uint8_t *__restrict__ src,
                                 const uint64_t *__restrict__ soffs, uint32_t soff,
                                 uint32_t bytes, uint64_t n) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
    const uint8_t *s = src + soffs[i] + soff;
    uint8_t *d = dst + doffs[i] + doff;
    for (uint32_t b = 0; b < bytes; ++b) d[b] = s[b];
  }
}

uint64_t route_blocks(uint64_t n) { return (n + kRT - 1) / kRT; }

}  // namespace

extern "C" size_t spk_route_workspace_bytes(uint64_t n_frames, uint32_t n_keys) {
  (void)n_keys;
  const uint64_t nb = route_blocks(n_frames);
  return (size_t)(((n_frames + 255) & ~255ull) + nb * kRK * 8 + 256);
}

extern "C" int spk_route_frames_checked(const void *d_wire, uint64_t wire_len,
                                        const uint64_t *d_frame_offsets, uint64_t n_frames,
                                        uint32_t key_off, const uint32_t *h_keys,
                                        uint32_t n_keys, const spk_route_hdr *hdr,
                                        uint64_t *const *d_begins, uint64_t *const *d_ends,
                                        uint64_t *const *d_index, uint64_t *d_counts,
                                        void *d_ws, size_t ws_bytes, void *stream) {
  if (n_keys > SPK_MAX_ROUTES || (n_keys && !h_keys) || !d_counts || !d_begins) return SPK_E_ARG;
  if (hdr && (hdr->head_len < 4 || hdr->len_off > hdr->head_len - 4 ||
              (hdr->attach_off != SPK_FRAME_NONE && hdr->attach_off > hdr->head_len - 4) ||
              key_off > hdr->head_len - 4))
    return SPK_E_ARG;
  if (n_frames && (!d_frame_offsets || !d_wire || !d_ws)) return SPK_E_ARG;
  if (ws_bytes < spk_route_workspace_bytes(n_frames, n_keys)) return SPK_E_WORKSPACE;
  for (uint32_t k = 0; k < n_keys; ++k) {
    if (!d_begins[k]) return SPK_E_ARG;
    for (uint32_t j = 0; j < k; ++j)
      if (h_keys[j] == h_keys[k]) return SPK_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  RouteArgs a = {};
  a.n = n_frames;
  a.wire_len = wire_len;
  a.key_off = key_off;
  a.nk = n_keys;
  a.chk = hdr ? 1u : 0u;
  if (hdr) a.h = *hdr;
  for (uint32_t k = 0; k < n_keys; ++k) a.keys[k] = h_keys[k];
  for (uint32_t k = 0; k <= n_keys; ++k) {
    a.beg[k] = d_begins[k];
    a.end[k] = d_ends ? d_ends[k] : nullptr;
    a.idx[k] = d_index ? d_index[k] : nullptr;
  }
  if (!n_frames) {
    return hipMemsetAsync(d_counts, 0, (n_keys + 1) * sizeof(uint64_t), s) == hipSuccess
               ? SPK_OK
               : SPK_E_HIP;
  }
  const uint64_t nb = route_blocks(n_frames);
  uint8_t *tslot = (uint8_t *)d_ws;
  uint64_t *bcnt = reinterpret_cast<uint64_t *>((uint8_t *)d_ws + ((n_frames + 255) & ~255ull));
  const uint8_t *wire = (const uint8_t *)d_wire;
  SPK_LAUNCH(route_count, dim3((unsigned)nb), dim3(kRT), 0, s, a, wire, d_frame_offsets, tslot,
             bcnt);
  SPK_LAUNCH(route_scan, dim3(1), dim3(kScanT), 0, s, nb, n_keys, bcnt, d_counts);
  SPK_LAUNCH(route_scatter, dim3((unsigned)nb), dim3(kRT), 0, s, a, wire, d_frame_offsets,
             (const uint8_t *)tslot, (const uint64_t *)bcnt);
  return hipGetLastError() == hipSuccess ? SPK_OK : SPK_E_HIP;
}

extern "C" int spk_route_frames(const void *d_wire, uint64_t wire_len,
                                const uint64_t *d_frame_offsets, uint64_t n_frames,
                                uint32_t key_off, const uint32_t *h_keys, uint32_t n_keys,
                                uint64_t *const *d_begins, uint64_t *const *d_ends,
                                uint64_t *const *d_index, uint64_t *d_counts, void *d_ws,
                                size_t ws_bytes, void *stream) {
  return spk_route_frames_checked(d_wire, wire_len, d_frame_offsets, n_frames, key_off, h_keys,
                                  n_keys, nullptr, d_begins, d_ends, d_index, d_counts, d_ws,
                                  ws_bytes, stream);
}

extern "C" int spk_copy_frame_field(void *d_dst, const uint64_t *d_dst_offsets, uint32_t dst_off,
                                    const void *d_src, const uint64_t *d_src_offsets,
                                    uint32_t src_off, uint32_t bytes, uint64_t n, void *stream) {
  if (bytes == 0 || bytes > 8) return SPK_E_ARG;
  if (!n) return SPK_OK;
  if (!d_dst || !d_dst_offsets || !d_src || !d_src_offsets) return SPK_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  uint64_t g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  SPK_LAUNCH(copy_frame_field, dim3((unsigned)g), dim3(256), 0, s, (uint8_t *)d_dst,
             d_dst_offsets, dst_off, (const uint8_t *)d_src, d_src_offsets, src_off, bytes, n);
  return hipGetLastError() == hipSuccess ? SPK_OK : SPK_E_HIP;
}
