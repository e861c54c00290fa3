// spk_fixed.hip — gfx950 kernels for trivially-serializable records
// (is_trivial_serializable<T>: one raw sizeof(T) copy per record, incl.
// padding — ref packer.hpp:411-421, unpacker.hpp:1127-1156,1293-1312).
//
// SPK_MODE_VECTOR: the message is [header][count:w][n*stride raw bytes], so
// encode and decode are byte-shifted stream copies between a 16-B aligned
// buffer and one displaced by the header length h (9 bytes for C2). The
// copy writes whole aligned 16-B chunks (global_store_dwordx4, 1 KiB per
// wave-instruction) and reads each one with a single byte-aligned
// global_load_dwordx4 (gfx950 runs in unaligned-access mode): every HBM byte
// is read once and written once, no cross-lane shuffles. Measured on MI355X
// (scripts/probes/stream_probe.hip, gpurun_out logs in profiles/r06/): 32
// chunks in flight per lane (512 B, a 32 KiB wave-tile) with non-temporal
// loads AND stores and one wave-tile per wave (exact grid) run at 6.15-6.17
// TB/s where the round-5 form (16 chunks, default policy, 32 Ki blocks) runs
// at 5.64-5.66 on the same box (+9 %); nt on either side alone, or nt at 16
// chunks, does not pay. An LDS-DMA ring (global_load_lds_dwordx4 into a
// per-wave 2-4 slot ring, ds_read_b128, aligned stores; with and without nt)
// measured 4-10 % SLOWER than the register form, and hipMemcpyAsync D2D
// slower still (4.4-5.0 TB/s).
// The shift is data-dependent on decode (width/meta/type-literal of the
// incoming header): the kernel reads it from a device-side CopyJob written by
// the header kernel, so no host round trip is needed.
//
// SPK_MODE_MESSAGES: n independent [header][record] messages (coro_rpc
// payloads): blocks of R messages staged through LDS so that both the
// record stream and the wire stream move as aligned 16-B chunks
// (fixed_msg_encode_lds / fixed_msg_decode_lds); a plain dword/byte gather
// remains for records too large to stage.
#include "spk_internal.hpp"

namespace spk {

// ---------------------------------------------------------------------------
// copy job: dst[dst_off + i] = src[src_off + i], i < nbytes; optionally
// prefixed by hdr_len header bytes taken from `hdr` written at dst[dst_off -
// hdr_len ...]. Lives in device memory so that decode can derive it from the
// incoming header without a host round trip.
struct CopyJob {
  uint64_t dst_off;
  uint64_t src_off;
  uint64_t nbytes;
  uint64_t hdr_len;  // header bytes written before dst_off (encode)
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

typedef v4u v4u_unaligned __attribute__((aligned(1)));

constexpr int kCopyThreads = 256;
constexpr int kCopyUnroll = 32;
constexpr uint64_t kTile = 64ull * kCopyUnroll;  // chunks per wave-tile

// dst chunk k (k in [0, nk)) = 16 source bytes at sp + 16k (any alignment)
__device__ __forceinline__ void shift_body(v4u *__restrict__ dst,
                                           const uint8_t *__restrict__ sp, uint64_t nk) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = (uint64_t)blockIdx.x * (kCopyThreads / 64) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (kCopyThreads / 64);
  for (uint64_t t0 = wid * kTile; t0 < nk; t0 += nw * kTile) {
    if (t0 + kTile <= nk) {
      v4u c[kCopyUnroll];
#pragma unroll
      for (int j = 0; j < kCopyUnroll; ++j)
        c[j] = __builtin_nontemporal_load(
            reinterpret_cast<const v4u_unaligned *>(sp + 16 * (t0 + j * 64 + lane)));
      // Keep all kCopyUnroll loads in flight before the first store: after
      // inlining, the compiler no longer proves dst and sp disjoint and
      // would otherwise interleave load/store pairs (2 loads in flight,
      // ~12 % slower: scripts/probes/c2_probe.cpp vs copy_probe.hip).
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < kCopyUnroll; ++j) __builtin_nontemporal_store(c[j], &dst[t0 + j * 64 + lane]);
    } else {
      for (uint64_t k = t0 + lane; k < nk; k += 64)
        dst[k] = *reinterpret_cast<const v4u_unaligned *>(sp + 16 * k);
    }
  }
}

// One launch covers: header bytes, the byte-wise head/tail of the range, and
// the aligned interior. `job` may be written by a preceding kernel.
__global__ __launch_bounds__(kCopyThreads) void shift_copy_kernel(
    uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
    const CopyJob *__restrict__ job, const uint8_t *__restrict__ hdr) {
  const uint64_t dst_off = job->dst_off, src_off = job->src_off, nb = job->nbytes;
  const uint64_t hdr_len = job->hdr_len;
  uint8_t *d = dst + dst_off;
  const uint8_t *s = src + src_off;
  const uint64_t dmis = (uint64_t)d & 15;
  // interior: aligned dst chunks fully inside [d, d+nb)
  uint64_t head = dmis ? 16 - dmis : 0;
  if (head > nb) head = nb;
  const uint64_t body = (nb - head) & ~15ull;
  const uint64_t tail_start = head + body;
  if (blockIdx.x == 0) {
    for (uint64_t i = threadIdx.x; i < hdr_len; i += blockDim.x)
      dst[dst_off - hdr_len + i] = hdr[i];
    for (uint64_t i = threadIdx.x; i < head; i += blockDim.x) d[i] = s[i];
    for (uint64_t i = tail_start + threadIdx.x; i < nb; i += blockDim.x) d[i] = s[i];
  }
  if (body == 0) return;
  shift_body(reinterpret_cast<v4u *>(d + head), s + head, body >> 4);
}

__global__ __launch_bounds__(kCopyThreads) void shift_copy_kernel(
    uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
    const CopyJob *__restrict__ job, const uint8_t *__restrict__ hdr);
static unsigned copy_grid(uint64_t max_bytes) {
  uint64_t tiles = (max_bytes / 16 + kTile - 1) / kTile;
  uint64_t blocks = (tiles + (kCopyThreads / 64) - 1) / (kCopyThreads / 64);
  // one wave-tile per wave (exact grid; 48,828 blocks for C2's 6.4 GB) — the
  // probe's best point; grid-stride only past 2^20 blocks (> 128 GiB)
  if (blocks > (1u << 20)) blocks = 1u << 20;
  if (blocks < 1) blocks = 1;
  return (unsigned)blocks;
}

// ---------------------------------------------------------------------------
// Plan for trivial records: O(1), written by a 1-thread kernel so the whole
// encode stays stream-ordered and graph-capturable.
struct FixedPlanArgs {
  spk_msgfmt fmt;  // message format (vector or one)
  uint64_t n;
  const uint64_t *dn;  // MESSAGES: device count (min(*dn, n)) or null
  uint32_t stride;
  int mode;
};

__global__ void fixed_plan_kernel(FixedPlanArgs a, spk_plan_t *plan, uint8_t *ws) {
  if (threadIdx.x != 0) return;
  spk_plan_t p;
  if (a.mode == SPK_MODE_VECTOR) {
    const uint32_t w = width_of(a.n);  // max_size = n (calculate_size.hpp:79)
    const HdrShape h = hdr_shape(a.fmt.flags, a.fmt.literal_len, w);
    uint8_t *hb = ws + kWsHdrVec;
    uint32_t len = write_hdr(hb, a.fmt, w);
    for (uint32_t i = 0; i < w; ++i) hb[len + i] = (uint8_t)(a.n >> (8 * i));
    CopyJob *job = reinterpret_cast<CopyJob *>(ws + kWsCtl);
    job->hdr_len = len + w;
    job->dst_off = len + w;
    job->src_off = 0;
    job->nbytes = a.n * a.stride;
    p.total_bytes = len + w + a.n * a.stride;
    p.max_count = a.n;
    p.var_bytes = a.n * a.stride;
    p.width = w;
    p.header_bytes = len + w;
    p.metainfo = h.meta;
    p.has_meta = h.has_meta;
  } else {
    const HdrShape h = hdr_shape(a.fmt.flags, a.fmt.literal_len, 1);
    write_hdr(ws + kWsHdrMsg, a.fmt, 1);
    const uint64_t n = dev_count(a.n, a.dn);
    p.total_bytes = n * (h.len + a.stride);
    p.max_count = 0;
    p.var_bytes = n * a.stride;
    p.width = 1;
    p.header_bytes = h.len;
    p.metainfo = h.meta;
    p.has_meta = h.has_meta;
  }
  *plan = p;
}

hipError_t launch_fixed_plan(const spk_layout *L, int mode, uint64_t n,
                             spk_plan_t *d_plan, void *d_ws, hipStream_t s,
                             const uint64_t *d_n) {
  FixedPlanArgs a;
  a.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  a.n = n;
  a.dn = d_n;
  a.stride = L->rec_stride;
  a.mode = mode;
  SPK_LAUNCH(fixed_plan_kernel, dim3(1), dim3(64), 0, s, a, d_plan,
                     (uint8_t *)d_ws);
  return hipGetLastError();
}

hipError_t launch_fixed_encode_vector(const spk_layout *L, uint64_t n,
                                      const void *d_recs, void *d_out,
                                      const void *d_ws, hipStream_t s) {
  const uint8_t *ws = (const uint8_t *)d_ws;
  const uint64_t max_bytes = n * (uint64_t)L->rec_stride;
  SPK_LAUNCH(shift_copy_kernel, dim3(copy_grid(max_bytes)), dim3(kCopyThreads),
                     0, s, (uint8_t *)d_out, (const uint8_t *)d_recs,
                     reinterpret_cast<const CopyJob *>(ws + kWsCtl), ws + kWsHdrVec);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// SPK_MODE_VECTOR decode: parse + validate the header on one wave (the
// reference's deserialize_metainfo, unpacker.hpp:548-619, then the
// trivially-copyable container branch :904-982,1127-1156), publish a CopyJob,
// then the same shift_copy moves the payload. The result is written before
// the copy; the copy length is 0 unless the header and length check passed.
struct FixedDecArgs {
  spk_msgfmt fmt;
  uint64_t wire_len;
  uint64_t rec_cap;
  uint32_t stride;
  uint32_t body_w;   // spk_decode_body: no header, body_n records at this width
  uint64_t body_n;
};

__global__ void fixed_decode_hdr_kernel(FixedDecArgs a, const uint8_t *wire,
                                        CopyJob *job, spk_dresult_t *res) {
  if (threadIdx.x != 0) return;
  uint64_t pos = 0, data_len = 0;
  uint32_t w = a.body_w;
  int32_t e = a.body_w ? SPK_ERRC_OK : parse_hdr(a.fmt, wire, a.wire_len, &pos, &w, &data_len);
  uint64_t n = 0;
  if (!e) {
    if (!a.body_w && a.wire_len < pos + w) {
      e = SPK_ERRC_NO_BUFFER_SPACE;
    } else {
      n = a.body_w ? a.body_n : ld_le(wire + pos, w);
      pos += a.body_w ? 0 : w;
      // overflow guard + check(mem_sz) (unpacker.hpp:1128-1149)
      if (n > ~0ull / a.stride || a.wire_len - pos < n * a.stride)
        e = SPK_ERRC_NO_BUFFER_SPACE;
    }
  }
  spk_dresult_t r = {};
  r.errc = e;
  r.width = w;
  job->hdr_len = 0;
  job->dst_off = 0;
  job->src_off = pos;
  job->nbytes = 0;
  if (!e) {
    r.count = n;
    const uint64_t end = pos + n * a.stride;
    r.consumed = end > data_len ? end : data_len;
    if (n > a.rec_cap)
      r.errc = SPK_ERRC_CAPACITY;
    else
      job->nbytes = n * a.stride;
  }
  *res = r;
}

hipError_t launch_fixed_decode_vector(const spk_layout *L, const void *d_wire,
                                         uint64_t wire_len, void *d_recs,
                                         uint64_t rec_cap, spk_dresult_t *d_res,
                                         void *d_ws, hipStream_t s, uint32_t body_w,
                                         uint64_t body_n) {
  FixedDecArgs a;
  a.body_w = body_w;
  a.body_n = body_n;
  a.fmt = L->fmt_vector;
  a.wire_len = wire_len;
  a.rec_cap = rec_cap;
  a.stride = L->rec_stride;
  CopyJob *job = reinterpret_cast<CopyJob *>((uint8_t *)d_ws + kWsCtl);
  SPK_LAUNCH(fixed_decode_hdr_kernel, dim3(1), dim3(64), 0, s, a,
                     (const uint8_t *)d_wire, job, d_res);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  uint64_t max_bytes = rec_cap * (uint64_t)L->rec_stride;
  if (max_bytes > wire_len) max_bytes = wire_len;
  SPK_LAUNCH(shift_copy_kernel, dim3(copy_grid(max_bytes)), dim3(kCopyThreads),
                     0, s, (uint8_t *)d_recs, (const uint8_t *)d_wire,
                     (const CopyJob *)job, (const uint8_t *)nullptr);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// SPK_MODE_MESSAGES, trivial records: message i = [hdr (H bytes)][record].
constexpr uint32_t kMsgHdrMax = 320;  // frame prefix (<= 64) + struct_pack header

struct MsgEncArgs {
  uint64_t n;
  const uint64_t *dn;  // device count (min(*dn, n)) or null
  uint32_t stride;    // bytes
  uint32_t hlen;      // header bytes (frame prefix + struct_pack header)
  uint32_t seq_off;   // frame sequence field (u32 LE = seq_base + i) or ~0u
  uint32_t seq_base;
  SeqEcho echo;
  uint8_t hdr[kMsgHdrMax];
};

// byte r (< hlen) of message i's header: the template, with the frame's
// sequence number field patched in
__device__ __forceinline__ uint8_t msg_hdr_byte(const uint8_t *hdr, uint32_t r, uint64_t i,
                                                uint32_t seq_off, uint32_t seq_base,
                                                const SeqEcho &echo) {
  const uint32_t q = r - seq_off;
  return r >= seq_off && q < 4 ? (uint8_t)(seq_value(echo, seq_base, i) >> (8 * q)) : hdr[r];
}

// dword gather: out dword d -> message i = d / Mw, word r = d % Mw
__global__ __launch_bounds__(256) void fixed_msg_encode_w4(
    MsgEncArgs a, const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
    uint64_t *__restrict__ offs) {
  const uint64_t N = dev_count(a.n, a.dn);
  const uint32_t Hw = a.hlen >> 2, Sw = a.stride >> 2, Mw = Hw + Sw;
  const uint64_t total_w = N * Mw;
  const uint64_t nchunks = (total_w + 3) >> 2;
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
       c += gstride) {
    const uint64_t d0 = c << 2;
    uint64_t i = d0 / Mw;
    uint32_t r = (uint32_t)(d0 - i * Mw);
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (r < Hw) {
        uint32_t h;
        __builtin_memcpy(&h, a.hdr + 4 * r, 4);
        // (i == n: the padding past the last message; an echo has no entry)
        v[j] = 4 * r == a.seq_off && i < N ? seq_value(a.echo, a.seq_base, i) : h;
      } else {
        v[j] = (d0 + j < total_w) ? in[i * Sw + (r - Hw)] : 0u;
      }
      if (++r == Mw) {
        r = 0;
        ++i;
      }
    }
    if (d0 + 4 <= total_w) {
      *reinterpret_cast<uint4 *>(out + d0) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
      for (int j = 0; j < 4; ++j)
        if (d0 + j < total_w) out[d0 + j] = v[j];
    }
  }
  if (offs) {
    const uint64_t M = (uint64_t)Mw * 4;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= N;
         i += gstride)
      offs[i] = i * M;
  }
}

// byte gather (header or stride not dword multiples)
__global__ __launch_bounds__(256) void fixed_msg_encode_b1(
    MsgEncArgs a, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
    uint64_t *__restrict__ offs) {
  const uint64_t N = dev_count(a.n, a.dn);
  const uint64_t M = (uint64_t)a.hlen + a.stride;
  const uint64_t total = N * M;
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < total;
       b += gstride) {
    const uint64_t i = b / M;
    const uint32_t r = (uint32_t)(b - i * M);
    out[b] = r < a.hlen ? msg_hdr_byte(a.hdr, r, i, a.seq_off, a.seq_base, a.echo)
                        : in[i * a.stride + (r - a.hlen)];
  }
  if (offs)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= N;
         i += gstride)
      offs[i] = i * M;
}

static unsigned elem_grid(uint64_t items, unsigned threads = 256) {
  uint64_t b = (items + threads - 1) / threads;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

// ---------------------------------------------------------------------------
// LDS-staged message batches. A block owns R consecutive messages (R a
// multiple of 16, so every block's record range and — when the header is a
// dword multiple — its wire range start on 64-B boundaries):
//   encode: the block's R*S record bytes are staged in LDS with 16-B loads,
//           then each lane assembles one aligned 16-B wire chunk from the
//           header (LDS) and the staged records and stores it: reads and
//           writes are both contiguous streams, one HBM pass each;
//   decode: the block's wire span is staged the same way, every lane parses
//           its message header from LDS (parse_hdr), and the records are
//           written as aligned 16-B chunks assembled with v_alignbyte from
//           the staged bytes (payloads start at any byte offset).
// Spans that do not fit the staging buffer (malformed offsets) fall back to
// global loads inside the same kernel, so results never depend on the path.
#ifndef SPK_MSG_THREADS
#define SPK_MSG_THREADS 256
#endif
constexpr int kMsgThreads = SPK_MSG_THREADS;
constexpr uint32_t kMsgStageMax = 32768;  // staging bytes per block
constexpr uint32_t kStagePer = 5;  // 16-B staging loads in flight per lane (decode)

struct MsgLdsArgs {
  spk_msgfmt fmt;   // decode only
  uint64_t n;
  const uint64_t *dn;  // device count (min(*dn, n)) or null
  uint64_t wire_len;
  uint64_t rec_cap;
  uint32_t stride;  // S (multiple of 4)
  uint32_t hlen;    // H (encode header bytes)
  uint32_t R;       // messages per block
  uint32_t cap;     // staging bytes (decode)
  uint32_t fixed_M; // implicit message stride when offsets == nullptr
  uint32_t prefix;  // decode: frame bytes before each message
  uint32_t seq_off; // encode: frame sequence field or ~0u
  uint32_t seq_base;
  SeqEcho echo;     // encode: seq_num echoed from request frames
  const uint64_t *ends;  // decode: message i ends at ends[i] (null: offs[i + 1])
  spk_plan_t *plan_out;  // encode: block 0 stores plan_val there (spk_plan_encode)
  spk_plan_t plan_val;
  uint8_t hdr[kMsgHdrMax];
};

__device__ __forceinline__ uint32_t lds_u32_at(const uint8_t *lds, uint32_t pos) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(lds + (pos & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], pos & 3u);  // shift in bytes
}

__device__ __forceinline__ uint32_t g_u32_at(const uint8_t *p) {
  return *reinterpret_cast<const uint32_t __attribute__((aligned(1))) *>(p);
}

// MESSAGES mode: non-temporal staging loads and record / wire stores (C2b
// A/B on one box: encode 2.556 -> 2.47 ms, decode 2.89 -> 2.85 ms). (A
// software-pipelined decode — the next group's staging loads in registers
// while this group is parsed and stored — measured 25 % SLOWER: 2.81 ->
// 3.65 ms, same box, profiles/r06/ab_c2b.txt.)
#ifndef SPK_MSG_NT
#define SPK_MSG_NT 1
#endif
__device__ __forceinline__ v4u msg_ld16(const uint8_t *p) {
  const v4u_unaligned *q = reinterpret_cast<const v4u_unaligned *>(p);
  if (SPK_MSG_NT) return __builtin_nontemporal_load(q);
  return *q;
}
__device__ __forceinline__ void msg_st16(uint8_t *p, const v4u &v) {
  if (SPK_MSG_NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(p));
  else *reinterpret_cast<v4u *>(p) = v;
}

template <bool DW>
__global__ __launch_bounds__(kMsgThreads) void fixed_msg_encode_lds(
    MsgLdsArgs a, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
    uint64_t *__restrict__ offs) {
  const uint64_t N = dev_count(a.n, a.dn);
  extern __shared__ v4u smem_v4[];
  uint8_t *hdr = reinterpret_cast<uint8_t *>(smem_v4);
  uint8_t *inl = hdr + kMsgHdrMax;
  const uint32_t tid = threadIdx.x;
  const uint32_t S = a.stride, H = a.hlen, M = H + S;
  const uint64_t first = (uint64_t)blockIdx.x * a.R;
  if (offs && blockIdx.x == gridDim.x - 1 && tid == 0) offs[N] = N * M;
  if (a.plan_out && blockIdx.x == 0 && tid == 0) *a.plan_out = a.plan_val;
  if (first >= N) return;
  const uint32_t nR = (uint32_t)((N - first) < a.R ? (N - first) : a.R);
  for (uint32_t k = tid; k < H; k += kMsgThreads) hdr[k] = a.hdr[k];
  const uint8_t *src = in + first * S;
  const uint32_t bin = nR * S;  // multiple of 4
  // kStagePer 16-B loads in flight per lane before their LDS writes
  for (uint32_t c0 = 0; c0 < bin / 16; c0 += kStagePer * kMsgThreads) {
    v4u val[kStagePer];
#pragma unroll
    for (uint32_t k = 0; k < kStagePer; ++k) {
      const uint32_t c = c0 + tid + k * kMsgThreads;
      if (c < bin / 16) val[k] = msg_ld16(src + 16 * c);
    }
#pragma unroll
    for (uint32_t k = 0; k < kStagePer; ++k) {
      const uint32_t c = c0 + tid + k * kMsgThreads;
      if (c < bin / 16) reinterpret_cast<v4u *>(inl)[c] = val[k];
    }
  }
  for (uint32_t d = (bin / 16) * 4 + tid; d < bin / 4; d += kMsgThreads)
    reinterpret_cast<uint32_t *>(inl)[d] = reinterpret_cast<const uint32_t *>(src)[d];
  if (offs)
    for (uint32_t k = tid; k < nR; k += kMsgThreads) offs[first + k] = (first + k) * M;
  __syncthreads();
  uint8_t *dst = out + first * M;
  const uint32_t bout = nR * M;
  if constexpr (DW) {
    const uint32_t Mw = M / 4, Hw = H / 4, Sw = S / 4, nq = bout / 4;
    const uint32_t seq_w = a.seq_off / 4;  // dword-aligned (host-checked) or huge
    const uint32_t *hw = reinterpret_cast<const uint32_t *>(hdr);
    const uint32_t *iw = reinterpret_cast<const uint32_t *>(inl);
    for (uint32_t t = tid; 4 * t < nq; t += kMsgThreads) {
      const uint32_t q0 = 4 * t;
      uint32_t i = q0 / Mw, r = q0 - i * Mw;
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = r < Hw ? (r == seq_w && i < nR ? seq_value(a.echo, a.seq_base, first + i) : hw[r])
                      : iw[i * Sw + (r - Hw)];
        if (++r == Mw) {
          r = 0;
          ++i;
        }
      }
      if (q0 + 4 <= nq) {
        v4u o = {v[0], v[1], v[2], v[3]};
        msg_st16(dst + 16 * t, o);
      } else {
        for (uint32_t k = 0; q0 + k < nq; ++k)
          reinterpret_cast<uint32_t *>(dst)[q0 + k] = v[k];
      }
    }
  } else {
    for (uint32_t j = tid; j < bout; j += kMsgThreads) {
      const uint32_t i = j / M, r = j - i * M;
      dst[j] = r < H ? msg_hdr_byte(hdr, r, first + i, a.seq_off, a.seq_base, a.echo)
                     : inl[i * S + (r - H)];
    }
  }
}

__global__ __launch_bounds__(kMsgThreads) void fixed_msg_decode_lds(
    MsgLdsArgs a, const uint8_t *__restrict__ wire, const uint64_t *__restrict__ offs,
    int32_t *__restrict__ errc, spk_dresult_t *__restrict__ res, uint8_t *__restrict__ out,
    uint64_t *__restrict__ part) {
  const uint64_t N = dev_count(a.n, a.dn);
  extern __shared__ v4u smem_v4[];
  uint8_t *stage = reinterpret_cast<uint8_t *>(smem_v4);
  __shared__ uint64_t s_lo[kMsgThreads / 64], s_hi[kMsgThreads / 64];
  __shared__ uint64_t s_pay[kMsgThreads];  // payload position (staged: LDS offset)
  const uint32_t tid = threadIdx.x;
  const uint32_t S = a.stride;
  const uint64_t ngroups = (N + a.R - 1) / a.R;
  // one block (a small call's messages): it resets and writes the result
  // itself, no memset and no msg_sum_partials launch
  const bool solo = gridDim.x == 1 && part == nullptr;
  if (solo) {
    if (tid == 0) *res = spk_dresult_t{};
    __syncthreads();
  }
  // more frames than the caller's n_max: the excess is not decoded
  if (a.dn && blockIdx.x == 0 && tid == 0 && *a.dn > a.n) atomicExch(&res->errc, SPK_ERRC_CAPACITY);
  // ok / consumed accumulate over the block's groups: one atomic per wave at
  // the end (same-address atomics per group would serialise in L2)
  unsigned long long ok = 0, consumed = 0;
  bool cap_hit = false;
  // message bounds of this lane in group g (prefetched one group ahead)
  auto bounds = [&](uint64_t g, uint64_t &b, uint64_t &e) {
    const uint64_t i = g * a.R + tid;
    if (g >= ngroups || tid >= a.R || i >= N) return;
    b = offs ? offs[i] : i * a.fixed_M;
    e = offs ? (a.ends ? a.ends[i] : offs[i + 1]) : (i + 1) * a.fixed_M;
  };
  uint64_t b_nx = 0, e_nx = 0;
  bounds(blockIdx.x, b_nx, e_nx);
  for (uint64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint64_t first = g * a.R;
    const uint32_t nR = (uint32_t)((N - first) < a.R ? (N - first) : a.R);
    uint64_t b = b_nx, e = e_nx;
    b_nx = e_nx = 0;
    bounds(g + gridDim.x, b_nx, e_nx);
    bool inr = false;
    if (tid < nR) {
      inr = e >= b && e <= a.wire_len && e - b >= a.prefix;
      b += a.prefix;  // the struct_pack message starts after the frame prefix
    }
    // block min of starts / max of ends over in-range messages
    uint64_t mn = inr ? b : ~0ull, mx = inr ? e : 0;
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t on = __shfl_xor(mn, o), ox = __shfl_xor(mx, o);
      mn = on < mn ? on : mn;
      mx = ox > mx ? ox : mx;
    }
    if ((tid & 63) == 0) {
      s_lo[tid >> 6] = mn;
      s_hi[tid >> 6] = mx;
    }
    __syncthreads();
    uint64_t blo = s_lo[0], hi = s_hi[0];
    for (int k = 1; k < kMsgThreads / 64; ++k) {
      blo = s_lo[k] < blo ? s_lo[k] : blo;
      hi = s_hi[k] > hi ? s_hi[k] : hi;
    }
    const uint64_t lo = blo & ~15ull;
    const bool staged = blo != ~0ull && hi - lo <= a.cap;
    if (staged) {
      const uint32_t nb = (uint32_t)(hi - lo);
      const uint64_t full = (a.wire_len - lo) / 16;  // 16-B chunks inside the wire
      const uint32_t nc = (nb + 15) / 16;
      if (nc <= full) {
        // each lane issues kStagePer 16-B loads before its LDS writes (a
        // load / store loop waits one load latency per 4 KiB); one round
        // covers 256 68-B messages
        for (uint32_t c0 = 0; c0 < nc; c0 += kStagePer * kMsgThreads) {
          v4u val[kStagePer];
#pragma unroll
          for (uint32_t k = 0; k < kStagePer; ++k) {
            const uint32_t c = c0 + tid + k * kMsgThreads;
            if (c < nc) val[k] = msg_ld16(wire + lo + 16 * (uint64_t)c);
          }
#pragma unroll
          for (uint32_t k = 0; k < kStagePer; ++k) {
            const uint32_t c = c0 + tid + k * kMsgThreads;
            if (c < nc) reinterpret_cast<v4u *>(stage)[c] = val[k];
          }
        }
      } else {
        for (uint32_t c = tid; 16 * c < nb; c += kMsgThreads) {
          if (c < full) {
            reinterpret_cast<v4u *>(stage)[c] =
                *reinterpret_cast<const v4u_unaligned *>(wire + lo + 16 * (uint64_t)c);
          } else {
            for (uint32_t k = 0; k < 16 && 16 * c + k < nb; ++k)
              stage[16 * c + k] = wire[lo + 16 * (uint64_t)c + k];
          }
        }
      }
    }
    __syncthreads();
    if (tid < nR) {
      const uint64_t i = first + tid;
      int32_t ec = SPK_ERRC_OK;
      uint64_t pos = 0, dl = 0;
      uint32_t w = 1;
      if (!inr) {
        ec = SPK_ERRC_NO_BUFFER_SPACE;
      } else {
        const uint8_t *p = staged ? stage + (b - lo) : wire + b;
        ec = parse_hdr(a.fmt, p, e - b, &pos, &w, &dl);
        if (!ec && e - b - pos < S) ec = SPK_ERRC_NO_BUFFER_SPACE;
      }
      if (!ec && i >= a.rec_cap) {
        ec = SPK_ERRC_CAPACITY;
        cap_hit = true;
      }
      if (errc) errc[i] = ec;
      s_pay[tid] = ec ? ~0ull : (staged ? b - lo : b) + pos;
      if (!ec) {
        ++ok;
        const uint64_t used = pos + S;
        consumed += used > dl ? used : dl;
      }
    }
    __syncthreads();
    if (first < a.rec_cap) {
      const uint32_t nW = (uint32_t)((a.rec_cap - first) < nR ? (a.rec_cap - first) : nR);
      const uint32_t Sw = S / 4, nd = nW * Sw;
      uint8_t *dst = out + first * S;
      for (uint32_t t = tid; 4 * t < nd; t += kMsgThreads) {
        const uint32_t d0 = 4 * t;
        uint32_t i = d0 / Sw, j = d0 - i * Sw;
        uint32_t v[4];
        uint32_t valid = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (d0 + k < nd) {
            const uint64_t p = s_pay[i];
            if (p != ~0ull) {
              v[k] = staged ? lds_u32_at(stage, (uint32_t)p + 4 * j)
                            : g_u32_at(wire + p + 4 * j);
              valid |= 1u << k;
            }
          }
          if (++j == Sw) {
            j = 0;
            ++i;
          }
        }
        if (valid == 0xF) {
          v4u o = {v[0], v[1], v[2], v[3]};
          msg_st16(dst + 16 * t, o);
        } else {
          for (int k = 0; k < 4; ++k)
            if (valid & (1u << k)) reinterpret_cast<uint32_t *>(dst)[d0 + k] = v[k];
        }
      }
    }
    __syncthreads();  // stage / s_pay are reused by the next group
  }
  // per-block partials (summed by msg_sum_partials): same-address atomics
  // from thousands of blocks would serialise in L2
  for (int o = 32; o > 0; o >>= 1) {
    ok += __shfl_down(ok, o);
    consumed += __shfl_down(consumed, o);
  }
  if ((tid & 63) == 0) {
    s_lo[tid >> 6] = ok;
    s_hi[tid >> 6] = consumed;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t o = 0, c = 0;
    for (int k = 0; k < kMsgThreads / 64; ++k) {
      o += s_lo[k];
      c += s_hi[k];
    }
    if (solo) {
      res->count = o;
      res->consumed = c;
    } else {
      part[2 * blockIdx.x] = o;
      part[2 * blockIdx.x + 1] = c;
    }
  }
  if (__any(cap_hit) && (tid & 63) == 0) atomicExch(&res->errc, SPK_ERRC_CAPACITY);
}

__global__ __launch_bounds__(1024) void msg_sum_partials(const uint64_t *__restrict__ part,
                                                         uint32_t nblocks,
                                                         spk_dresult_t *__restrict__ res) {
  __shared__ uint64_t sh[2][1024 / 64];
  uint64_t o = 0, c = 0;
  for (uint32_t b = threadIdx.x; b < nblocks; b += blockDim.x) {
    o += part[2 * b];
    c += part[2 * b + 1];
  }
  for (int k = 32; k > 0; k >>= 1) {
    o += __shfl_down(o, k);
    c += __shfl_down(c, k);
  }
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = o;
    sh[1][threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < blockDim.x / 64; ++k) {
      o += sh[0][k];
      c += sh[1][k];
    }
    res->count = o;
    res->consumed = c;
  }
}

// A grid-stride kernel's grid: the blocks the device holds at once (occupancy
// x CUs), at most `want` and `fixed_cap`. A fixed cap (4096) left a second, partial round of
// blocks once the first had run: each block strides over the same number of
// groups, so a grid of 1.8 resident rounds took two full ones.
#ifndef SPK_RESIDENT_GRID
#define SPK_RESIDENT_GRID 1
#endif
template <typename K>
static uint64_t resident_grid(K kernel, int threads, size_t shm, uint64_t want, uint64_t fixed_cap) {
  if (!SPK_RESIDENT_GRID) return want < fixed_cap ? want : fixed_cap;
  static int ncu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 0;
    return v;
  }();
  int nb = 0;
  if (!ncu || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, shm) != hipSuccess ||
      nb <= 0)
    return want < fixed_cap ? want : fixed_cap;
  uint64_t cap = (uint64_t)nb * (uint64_t)ncu;
  if (cap > fixed_cap) cap = fixed_cap;  // (the workspace holds fixed_cap blocks' partials)
  return want < cap ? want : cap;
}

// messages per block for the LDS-staged kernels: a multiple of 16 whose
// staging (R messages of M bytes, + alignment slack) fits kMsgStageMax; 0 if
// a single group of 16 does not fit (very large records: global path)
static uint32_t msg_block_R(uint32_t M) {
  uint32_t R = (kMsgStageMax - 64) / M;
  if (R > (uint32_t)kMsgThreads) R = kMsgThreads;
  return R & ~15u;
}

// frame prefix + struct_pack header of one message into hdr; returns the
// length. The frame's length field is constant for trivial records.
static uint32_t msg_header(const spk_layout *L, const spk_frame *F, uint8_t *hdr,
                           uint32_t *seq_off, uint32_t *seq_base) {
  uint32_t P = 0;
  *seq_off = ~0u;
  *seq_base = 0;
  if (F) {
    P = F->prefix_len;
    for (uint32_t k = 0; k < P; ++k) hdr[k] = F->tmpl[k];
  }
  const uint32_t H = write_hdr(hdr + P, L->fmt_one, 1);
  if (F) {
    const uint32_t len = H + L->rec_stride;
    if (F->len_off != SPK_FRAME_NONE)
      for (int k = 0; k < 4; ++k) hdr[F->len_off + k] = (uint8_t)(len >> (8 * k));
    if (F->seq_off != SPK_FRAME_NONE) {
      *seq_off = F->seq_off;
      *seq_base = F->seq_base;
    }
  }
  return P + H;
}

// spk_plan_encode, trivially copyable records, MESSAGES: the plan is known on
// the host (fixed_plan_kernel's), so the encode kernel's block 0 stores it --
// one launch instead of two for a small call's message
hipError_t launch_fixed_plan_encode_messages(const spk_layout *L, uint64_t n,
                                             const void *d_recs, void *d_out,
                                             uint64_t *d_offsets, spk_plan_t *d_plan,
                                             void *d_ws, hipStream_t s) {
  const HdrShape h = hdr_shape(L->fmt_one.flags, L->fmt_one.literal_len, 1);
  spk_plan_t p = {};
  p.total_bytes = n * (h.len + (uint64_t)L->rec_stride);
  p.max_count = 0;
  p.var_bytes = n * (uint64_t)L->rec_stride;
  p.width = 1;
  p.header_bytes = h.len;
  p.metainfo = h.meta;
  p.has_meta = h.has_meta;
  hipError_t e = launch_fixed_encode_messages(L, n, d_recs, d_out, d_offsets, nullptr, s,
                                              nullptr, nullptr, d_plan, &p);
  if (e == hipErrorNotSupported)  // (not the LDS kernel: plan, then encode)
    if ((e = launch_fixed_plan(L, SPK_MODE_MESSAGES, n, d_plan, d_ws, s)) == hipSuccess)
      e = launch_fixed_encode_messages(L, n, d_recs, d_out, d_offsets, nullptr, s, nullptr,
                                       nullptr);
  return e;
}

hipError_t launch_fixed_encode_messages(const spk_layout *L, uint64_t n,
                                        const void *d_recs, void *d_out,
                                        uint64_t *d_offsets, const spk_frame *F,
                                        hipStream_t s, const SeqEcho *echo,
                                        const uint64_t *d_n, spk_plan_t *d_plan_out,
                                        const spk_plan_t *plan_val) {
  {
    MsgLdsArgs b = {};
    if (d_plan_out) {
      b.plan_out = d_plan_out;
      b.plan_val = *plan_val;
    }
    if (echo) b.echo = *echo;
    b.n = n;
    b.dn = d_n;
    b.stride = L->rec_stride;
    b.hlen = msg_header(L, F, b.hdr, &b.seq_off, &b.seq_base);
    const uint32_t M = b.hlen + b.stride;
    b.R = msg_block_R(M);
    const bool dw = (b.hlen % 4 == 0) && (b.seq_off == ~0u || b.seq_off % 4 == 0) &&
                    ((uintptr_t)d_out % 16 == 0);
    // the LDS kernels move records in dwords: a packed stride (e.g. 7 B,
    // #pragma pack) takes the byte kernels below
    if (b.R && (uintptr_t)d_recs % 4 == 0 && b.stride % 4 == 0) {
      const uint64_t blocks = n ? (n + b.R - 1) / b.R : 1;
      const size_t lds = kMsgHdrMax + (size_t)b.R * b.stride + 16;
      if (dw)
        SPK_LAUNCH(fixed_msg_encode_lds<true>, dim3((unsigned)blocks),
                           dim3(kMsgThreads), lds, s, b, (const uint8_t *)d_recs,
                           (uint8_t *)d_out, d_offsets);
      else
        SPK_LAUNCH(fixed_msg_encode_lds<false>, dim3((unsigned)blocks),
                           dim3(kMsgThreads), lds, s, b, (const uint8_t *)d_recs,
                           (uint8_t *)d_out, d_offsets);
      return hipGetLastError();
    }
  }
  if (d_plan_out) return hipErrorNotSupported;  // (the caller plans separately)
  MsgEncArgs a = {};
  if (echo) a.echo = *echo;
  a.n = n;
  a.dn = d_n;
  a.stride = L->rec_stride;
  a.hlen = msg_header(L, F, a.hdr, &a.seq_off, &a.seq_base);
  const bool w4 = (a.hlen % 4 == 0) && (a.stride % 4 == 0) &&
                  (a.seq_off == ~0u || a.seq_off % 4 == 0) &&
                  ((uintptr_t)d_recs % 4 == 0) && ((uintptr_t)d_out % 16 == 0);
  if (w4) {
    const uint64_t chunks = (n * ((a.hlen + a.stride) / 4) + 3) / 4;
    SPK_LAUNCH(fixed_msg_encode_w4, dim3(elem_grid(chunks > n ? chunks : n + 1)),
                       dim3(256), 0, s, a, (const uint32_t *)d_recs, (uint32_t *)d_out,
                       d_offsets);
  } else {
    SPK_LAUNCH(fixed_msg_encode_b1, dim3(elem_grid(n * (a.hlen + a.stride) + 1)),
                       dim3(256), 0, s, a, (const uint8_t *)d_recs, (uint8_t *)d_out,
                       d_offsets);
  }
  return hipGetLastError();
}

// Decode: one thread per message parses the header (parse_hdr), then the
// record bytes are moved by a dword/byte gather over output records.
struct MsgDecArgs {
  spk_msgfmt fmt;
  uint64_t n;
  const uint64_t *dn;  // device count (min(*dn, n)) or null
  uint64_t wire_len;
  uint64_t rec_cap;
  uint32_t stride;
  uint32_t fixed_M;  // implicit message stride when offsets == nullptr
  uint32_t prefix;   // frame bytes before each message
  const uint64_t *ends;  // message i ends at ends[i] (null: offs[i + 1])
};

__global__ __launch_bounds__(256) void fixed_msg_parse(
    MsgDecArgs a, const uint8_t *__restrict__ wire, const uint64_t *__restrict__ offs,
    uint64_t *__restrict__ payload, int32_t *__restrict__ errc,
    spk_dresult_t *__restrict__ res) {
  const uint64_t N = dev_count(a.n, a.dn);
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long ok = 0, consumed = 0;
  if (a.dn && blockIdx.x == 0 && threadIdx.x == 0 && *a.dn > a.n)
    atomicExch(&res->errc, SPK_ERRC_CAPACITY);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N;
       i += gstride) {
    uint64_t b = offs ? offs[i] : i * a.fixed_M;
    uint64_t e = offs ? (a.ends ? a.ends[i] : offs[i + 1]) : (i + 1) * a.fixed_M;
    int32_t ec = SPK_ERRC_OK;
    uint64_t pos = 0, dl = 0;
    uint32_t w = 1;
    const bool inr = e >= b && e <= a.wire_len && e - b >= a.prefix;
    b += a.prefix;
    if (!inr) {
      ec = SPK_ERRC_NO_BUFFER_SPACE;
    } else {
      ec = parse_hdr(a.fmt, wire + b, e - b, &pos, &w, &dl);
      if (!ec && e - b - pos < a.stride) ec = SPK_ERRC_NO_BUFFER_SPACE;
    }
    if (!ec && i >= a.rec_cap) {
      ec = SPK_ERRC_CAPACITY;
      atomicExch(&res->errc, SPK_ERRC_CAPACITY);
    }
    if (errc) errc[i] = ec;
    payload[i] = ec ? ~0ull : b + pos;
    if (!ec) {
      ++ok;
      const uint64_t used = pos + a.stride;
      consumed += used > dl ? used : dl;
    }
  }
  // wave reduce then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    ok += __shfl_down(ok, o);
    consumed += __shfl_down(consumed, o);
  }
  if ((threadIdx.x & 63) == 0 && (ok || consumed)) {
    atomicAdd((unsigned long long *)&res->count, ok);
    atomicAdd((unsigned long long *)&res->consumed, consumed);
  }
}

__global__ __launch_bounds__(256) void fixed_msg_gather(
    uint64_t n, uint32_t stride, const uint8_t *__restrict__ wire,
    const uint64_t *__restrict__ payload, uint8_t *__restrict__ out, const uint64_t *dn) {
  n = dev_count(n, dn);
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  if ((stride & 3) == 0) {
    const uint32_t Sw = stride >> 2;
    const uint64_t total = n * Sw;
    for (uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; d < total;
         d += gstride) {
      const uint64_t i = d / Sw;
      const uint32_t j = (uint32_t)(d - i * Sw);
      const uint64_t p = payload[i];
      if (p == ~0ull) continue;
      const uint8_t *src = wire + p + 4 * j;
      uint32_t v;
      if (((uintptr_t)src & 3) == 0) {
        v = *reinterpret_cast<const uint32_t *>(src);
      } else {
        v = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) |
            ((uint32_t)src[3] << 24);
      }
      reinterpret_cast<uint32_t *>(out)[d] = v;
    }
  } else {
    const uint64_t total = n * stride;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < total;
         b += gstride) {
      const uint64_t i = b / stride;
      const uint64_t p = payload[i];
      if (p == ~0ull) continue;
      out[b] = wire[p + (b - i * stride)];
    }
  }
}

hipError_t launch_fixed_decode_messages(const spk_layout *L, const void *d_wire,
                                           uint64_t wire_len, const uint64_t *d_offsets,
                                           uint64_t n, uint32_t prefix, void *d_recs,
                                           uint64_t rec_cap, spk_dresult_t *d_res,
                                           int32_t *d_errc, void *d_ws, hipStream_t s,
                                           const uint64_t *d_msg_ends, const uint64_t *d_n) {
  MsgDecArgs a;
  a.dn = d_n;
  a.prefix = prefix;
  a.ends = d_msg_ends;
  a.fmt = L->fmt_one;
  a.n = n;
  a.wire_len = wire_len;
  a.rec_cap = rec_cap;
  a.stride = L->rec_stride;
  uint8_t hb[4 + 1 + SPK_MAX_LITERAL + 1];
  a.fixed_M = prefix + write_hdr(hb, L->fmt_one, 1) + L->rec_stride;
  uint64_t *payload = reinterpret_cast<uint64_t *>((uint8_t *)d_ws + kWsScratch);
  hipError_t e;
  {
    MsgLdsArgs b = {};
    b.fmt = L->fmt_one;
    b.n = n;
    b.dn = d_n;
    b.wire_len = wire_len;
    b.rec_cap = rec_cap;
    b.stride = L->rec_stride;
    b.fixed_M = a.fixed_M;
    b.prefix = prefix;
    b.ends = d_msg_ends;
    b.R = msg_block_R(a.fixed_M);
    if (b.R && (uintptr_t)d_recs % 16 == 0 && n > 0 && b.stride % 4 == 0) {
      b.cap = b.R * a.fixed_M + 32;
      // groups are strided over the grid: one resident round of blocks
      const uint64_t blocks = resident_grid(fixed_msg_decode_lds, kMsgThreads, (size_t)b.cap + 16,
                                            (n + b.R - 1) / b.R, 4096);
      uint64_t *part = payload;  // workspace scratch: 2 words per block
      if (blocks == 1) {  // (the kernel resets d_res and writes it: one launch)
        SPK_LAUNCH(fixed_msg_decode_lds, dim3(1), dim3(kMsgThreads), (size_t)b.cap + 16, s, b,
                   (const uint8_t *)d_wire, d_offsets, d_errc, d_res, (uint8_t *)d_recs,
                   (uint64_t *)nullptr);
        return hipGetLastError();
      }
      if ((e = hipMemsetAsync(d_res, 0, sizeof(spk_dresult_t), s)) != hipSuccess) return e;
      SPK_LAUNCH(fixed_msg_decode_lds, dim3((unsigned)blocks), dim3(kMsgThreads),
                         (size_t)b.cap + 16, s, b, (const uint8_t *)d_wire, d_offsets, d_errc,
                         d_res, (uint8_t *)d_recs, part);
      SPK_LAUNCH(msg_sum_partials, dim3(1), dim3(1024), 0, s, (const uint64_t *)part,
                         (uint32_t)blocks, d_res);
      return hipGetLastError();
    }
  }
  if ((e = hipMemsetAsync(d_res, 0, sizeof(spk_dresult_t), s)) != hipSuccess) return e;
  SPK_LAUNCH(fixed_msg_parse, dim3(elem_grid(n)), dim3(256), 0, s, a,
                     (const uint8_t *)d_wire, d_offsets, payload, d_errc, d_res);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const uint64_t nrec = n < rec_cap ? n : rec_cap;
  const uint64_t items = (L->rec_stride % 4 == 0) ? nrec * (L->rec_stride / 4)
                                                  : nrec * L->rec_stride;
  SPK_LAUNCH(fixed_msg_gather, dim3(elem_grid(items)), dim3(256), 0, s, nrec,
                     (uint32_t)L->rec_stride, (const uint8_t *)d_wire,
                     (const uint64_t *)payload, (uint8_t *)d_recs, d_n);
  return hipGetLastError();
}

}  // namespace spk
