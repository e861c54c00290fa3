// spk_var.hip — gfx950 kernels for records with variable-length members
// (std::string / std::vector<trivially serializable>): the RecS (C3),
// Outer{vector<Inner>} (C4) and mixed coro_rpc payload (C5) configs.
//
// Reference behaviour restated (paths relative to
// /root/reference/include/ylt/struct_pack/):
//   size pass  calculate_one_size / get_serialize_runtime_info
//              (calculate_size.hpp:39-189, 407-474): the container-length
//              width is chosen from the max element count over EVERY
//              container of the message, including the outer vector's
//              count, so encode is reduce -> scan -> write.
//   write      packer::serialize_one (packer.hpp:237-527): members in
//              declaration order, no padding between members, length
//              prefixes as the low w bytes of the count (endian_wrapper.hpp).
//   read       unpacker::deserialize_one (unpacker.hpp:780-1349): every
//              payload failure is no_buffer_space.
//
// Encode (both modes): a plan pass reads only the span counts (block
// partials: sum of w-independent bytes, max count), a one-block finalize
// scans the partials and emits the header, and the write pass assembles each
// block's contiguous output range in LDS byte-by-byte and flushes it with
// 16-B aligned stores (byte stores only at the two range edges shared with
// the neighbouring blocks).
//
// Decode, SPK_MODE_MESSAGES: message boundaries come from the framing
// (offsets), so it is parse (per message) -> scan heap totals -> write.
// Decode, SPK_MODE_VECTOR: record k's start depends on every earlier length,
// so boundaries are recovered with a chunked transition function: the
// payload is cut into kChunk-byte chunks; for each chunk, 256 candidate entry
// offsets are walked in parallel in LDS (walks that land on a position
// another walk already visited stop and link to it), giving exit offset and
// record count per entry; the per-chunk maps are composed hierarchically
// (groups of 64) to get every chunk's true entry and first record index;
// then each chunk is re-walked to place its records. Records whose
// straddling part exceeds 255 bytes defeat the 256-entry table: that case
// falls back to one sequential walker (correct, slow) — see DESIGN.md.
#include "spk_internal.hpp"
#include "spk_nlayout.hpp"

#include <stdlib.h>

#ifndef SPK_TCHUNK
#define SPK_TCHUNK 256
#endif
#ifndef SPK_TWAVES
#define SPK_TWAVES 1
#endif
#ifndef SPK_ESPLIT
#define SPK_ESPLIT 2
#endif
#ifndef SPK_NT_REACH  // bytes K1's resolution walks of nested records may cover
#define SPK_NT_REACH 4096
#endif
#ifndef SPK_NT_PAST   // records a nested speculative walk checks past its chunk
// (0: none. Nested starts are screened well enough that the in-wave
// resolution catches the few wrong ones: cm K1 11.1 -> 9.8 ms; flat layouts
// keep 2 -- without the past walks C3 / C4 / cv tiles go wrong by the
// thousand and the sequential fixer takes 0.1-0.5 s)
#define SPK_NT_PAST 0
#endif
#ifndef SPK_SCAP      // K1's speculation caps from the message's first records (vec_hdr_sample)
// (round 4, after K1's lane state moved back into locals: bit 0 on by default
// -- C3 / c3r / cv K1 0.243 / 0.253 / 1.93 -> 0.194 / 0.209 / 1.72 ms, C4
// +1 %; the screen cap too: cv K1 1.71 -> 1.36 ms but C3 0.192 -> 0.216, so
// it is on for varint layouts only)
#define SPK_SCAP 5        // bit 0: on the speculative walks' records, bit 1: on the candidate screen,
                          // bit 2: on the candidate screen of varint layouts (NS = -1)
#endif
#ifndef SPK_SCAP_MINR     // ... applied only when the layout's first-count limit is this many times the cap
// (round 4: 32 -> 8, so C4's 1-byte counts (limit 511, cap ~32) take them: K1 0.362 -> 0.350 ms)
#define SPK_SCAP_MINR 8
#endif
#ifndef SPK_SCAP_MUL      // a span's cap: this multiple of its largest sampled count
#define SPK_SCAP_MUL 2
#endif
#ifndef SPK_NT_SCR2   // nested candidate starts screened on a second count
#define SPK_NT_SCR2 1
#endif

namespace spk {

// Heaps of the flat-record kernels in this file: a flat layout with more
// variable-length members runs the interpreter (spk_nested.hip).
constexpr uint32_t kVS = SPK_FLAT_SPANS;

// Span loops q < nsp with a compile-time trip count (the arrays they index
// stay in registers; a runtime bound would put them in scratch memory):
// QFOR in functions templated on NS, QFORV elsewhere, QFORS over SpecPath.
#define QFOR(q) _Pragma("unroll") for (uint32_t q = 0; q < (NS > 0 ? (uint32_t)NS : kVS); ++q) if (q < nsp)
#define QFORV(q) _Pragma("unroll") for (uint32_t q = 0; q < kVS; ++q) if (q < nsp)
#define QFORS(q) _Pragma("unroll") for (uint32_t q = 0; q < (uint32_t)SpecPath<NS>::kS; ++q) if (q < nsp)
constexpr int kThreads = 256;
constexpr int kIPT = 1;                     // records per thread (encode write; 2 measured
                                            // slower: C3 +19 %, C5 3x as big payloads
                                            // overflow the cooperative list)
constexpr uint64_t kRPB = kThreads * kIPT;  // records per block (encode write)
constexpr int kPlanSub = 4;                 // write blocks per plan block
constexpr uint64_t kPlanRPB = kRPB * kPlanSub;  // records per plan block

struct VarArgs {
  KLayout L;
  uint64_t n;
  const uint64_t *dn;  // MESSAGES: device count (min(*dn, n)) or null
  int mode;
  uint32_t fpre;      // MESSAGES: frame prefix bytes before every message
  const uint8_t *heaps[kVS];
  uint32_t fseq_off;  // frame u32 fields (SPK_FRAME_NONE: absent)
  uint32_t flen_off;
  uint32_t fseq_base;
  uint32_t pad_;
  SeqEcho echo;       // MESSAGES: seq_num echoed from request frames
  uint8_t ftmpl[SPK_MAX_FRAME];
};

static KLayout make_klayout(const spk_layout *L) {
  KLayout k = {};
  k.stride = L->rec_stride;
  k.n_ops = L->n_ops;
  k.trivial = (L->flags & SPK_LAYOUT_TRIVIAL) ? 1 : 0;
  for (uint32_t i = 0; i < L->n_ops && i < SPK_MAX_OPS; ++i) {
    k.ops[i] = L->ops[i];
    if (L->ops[i].kind == SPK_OP_COPY) {
      k.fixed_bytes += L->ops[i].size;
    } else if (L->ops[i].kind == SPK_OP_VARINT) {
      ++k.n_var;
    } else {
      ++k.n_spans;
      if (L->ops[i].kind == SPK_OP_SPAN)
        ++k.n_cont;
      else
        k.fixed_bytes += 1;  // OPTION: has_value byte
    }
  }
  return k;
}

__device__ __forceinline__ uint32_t rec_u32(const uint8_t *rec, uint32_t off) {
  return *reinterpret_cast<const uint32_t *>(rec + off);
}
__device__ __forceinline__ uint64_t rec_u64(const uint8_t *rec, uint32_t off) {
  return *reinterpret_cast<const uint64_t *>(rec + off);
}

typedef uint16_t u16_unaligned __attribute__((aligned(1)));
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
typedef uint64_t u64_unaligned __attribute__((aligned(1)));
typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
typedef v4u_t v4u_una __attribute__((aligned(1)));

// an encode window's 16-B chunk to the output (write-once streams):
// SPK_FLUSH_NT = 1 stores it non-temporally
#ifndef SPK_FLUSH_NT
#define SPK_FLUSH_NT 1  // (encode windows: C3 0.323 -> 0.318 ms, C4 0.375 -> 0.371, cm 2.865 -> 2.823, cvm 0.481 -> 0.473)
#endif
__device__ __forceinline__ void flush16(uint8_t *dst, const v4u_t &v) {
  if (SPK_FLUSH_NT)
    __builtin_nontemporal_store(v, reinterpret_cast<v4u_t *>(dst));
  else
    *reinterpret_cast<v4u_t *>(dst) = v;
}
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
// byte-aligned LDS words: gfx950 reads (and writes) them with one ds_read_b32 / b64 / b128
// (unaligned DS access), not with 2-5 aligned dword reads + alignbyte
typedef __attribute__((address_space(3))) uint16_t lds_u16_una __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint32_t lds_u32_una __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint64_t lds_u64_una __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) v4u_t lds_v4u_una __attribute__((aligned(1)));

// unaligned byte copy in 16/8/4/1-byte pieces (gfx950 runs in unaligned mode)
__device__ __forceinline__ void copy_bytes(uint8_t *d, const uint8_t *s, uint64_t n) {
  uint64_t i = 0;
  for (; i + 16 <= n; i += 16)
    *reinterpret_cast<v4u_una *>(d + i) = *reinterpret_cast<const v4u_una *>(s + i);
  if (n - i >= 8) {
    *reinterpret_cast<u64_unaligned *>(d + i) = *reinterpret_cast<const u64_unaligned *>(s + i);
    i += 8;
  }
  if (n - i >= 4) {
    *reinterpret_cast<u32_unaligned *>(d + i) = *reinterpret_cast<const u32_unaligned *>(s + i);
    i += 4;
  }
  for (; i < n; ++i) d[i] = s[i];
}

// little-endian w-byte store (unaligned)
__device__ __forceinline__ void store_le(uint8_t *d, uint64_t v, uint32_t w) {
  switch (w) {
    case 1: *d = (uint8_t)v; break;
    case 2: *reinterpret_cast<u16_unaligned *>(d) = (uint16_t)v; break;
    case 4: *reinterpret_cast<u32_unaligned *>(d) = (uint32_t)v; break;
    default: *reinterpret_cast<u64_unaligned *>(d) = v; break;
  }
}

// SPAN/OPTION helpers: an OPTION's count is 0/1 and its prefix one byte
__device__ __forceinline__ uint32_t op_pw(const spk_op &op, uint32_t w) {
  return op.kind == SPK_OP_OPTION ? 1u : w;
}
__device__ __forceinline__ uint64_t op_rec_count(const spk_op &op, const uint8_t *rec) {
  const uint32_t c = rec_u32(rec, op.rec_off);
  return op.kind == SPK_OP_OPTION ? (uint64_t)(c != 0) : (uint64_t)c;
}

// Payload bytes a SPAN/OPTION with count c consumes at pos (message end
// `end`). An OPTION's value read status is ignored by the reference
// (unpacker.hpp:1271-1273 drops deserialize_one's errc): a present value that
// does not fit leaves the reader where it was and the value value-initialised.
__device__ __forceinline__ uint64_t opt_nb(const spk_op &op, uint64_t c, uint64_t pos,
                                           uint64_t end) {
  const uint64_t nb = c * op.size;
  return (op.kind == SPK_OP_OPTION && nb > end - pos) ? 0 : nb;
}

// ---- varint members (struct_pack/varint.hpp) ---------------------------------
// The unsigned value serialize_varint writes (varint.hpp:245-268): sint<T>
// (var_int32_t / var_int64_t) is zigzag-mapped at its own width
// (encode_zigzag :194-210), varint<T> is the value itself.
__device__ __forceinline__ uint64_t vi_value(const spk_op &op, const uint8_t *rec) {
  if (op.size == 4) {
    uint32_t u = rec_u32(rec, op.rec_off);
    if (op.aux & SPK_VARINT_SEXT) return (uint64_t)(int64_t)(int32_t)u;  // plain int32_t: v = t
    if (op.aux & SPK_VARINT_ZIGZAG) u = (u << 1) ^ (uint32_t)(-(int32_t)(u >> 31));
    return u;
  }
  uint64_t u = rec_u64(rec, op.rec_off);
  if (op.aux & SPK_VARINT_ZIGZAG) u = (u << 1) ^ (uint64_t)(-(int64_t)(u >> 63));
  return u;
}
// LEB128 byte count, calculate_varint_size (varint.hpp:212-239)
__device__ __forceinline__ uint32_t vi_len(uint64_t v) {
  return (70u - (uint32_t)__builtin_clzll(v | 1)) / 7u;
}
constexpr uint32_t kViBad = 0xFFu;
// deserialize_varint_impl (varint.hpp:270-292) at pos (message end len):
// the byte count, 0 when truncated (no_buffer_space), kViBad after ten bytes
// that all carry the continuation bit (invalid_buffer)
template <typename ByteFn>
__device__ __forceinline__ uint32_t vi_read(ByteFn byte, uint64_t pos, uint64_t len,
                                            uint64_t *v) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < 10; ++i) {
    if (pos + i >= len) return 0;
    const uint32_t b = byte(pos + i);
    x |= (uint64_t)(b & 0x7fu) << (7 * i);
    if (!(b & 0x80u)) {
      *v = x;
      return i + 1;
    }
  }
  return kViBad;
}
// the decoded value truncated to the member (deserialize_varint :294-330:
// zigzag decoded at 64 bits for the signed types)
__device__ __forceinline__ void vi_store(const spk_op &op, uint8_t *rec, uint64_t v) {
  if (op.aux & SPK_VARINT_ZIGZAG) v = (v >> 1) ^ (uint64_t)(-(int64_t)(v & 1));
  if (op.size == 4)
    *reinterpret_cast<uint32_t *>(rec + op.rec_off) = (uint32_t)v;
  else
    *reinterpret_cast<uint64_t *>(rec + op.rec_off) = v;
}
// LEB128 from the 8 bytes b (little-endian) when it ends inside them: the
// terminator is the first byte without its high bit, the value gathers the
// 7-bit groups; 0 when all 8 bytes continue (the caller reads on)
__device__ __forceinline__ uint32_t vi_decode8(uint64_t b, uint64_t *v) {
  const uint64_t t = ~b & 0x8080808080808080ull;
  if (!t) return 0;
  const uint32_t l = ((uint32_t)__builtin_ctzll(t) >> 3) + 1;
  uint64_t m = b & 0x7F7F7F7F7F7F7F7Full;
  if (l < 8) m &= (1ull << (8 * l)) - 1;
  *v = (m & 0x7Full) | ((m >> 1) & (0x7Full << 7)) | ((m >> 2) & (0x7Full << 14)) |
       ((m >> 3) & (0x7Full << 21)) | ((m >> 4) & (0x7Full << 28)) |
       ((m >> 5) & (0x7Full << 35)) | ((m >> 6) & (0x7Full << 42)) | ((m >> 7) & (0x7Full << 49));
  return l;
}
struct WireBytes {
  const uint8_t *wire;
  __device__ __forceinline__ uint32_t operator()(uint64_t x) const { return wire[x]; }
};

// w-independent bytes of one record (fixed + span payloads) and its max count
__device__ __forceinline__ void rec_sizes(const KLayout &L, const uint8_t *rec,
                                          uint64_t &var, uint64_t &maxc) {
  var = L.fixed_bytes;
  maxc = 0;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_SPAN) {
      const uint64_t c = rec_u32(rec, op.rec_off);
      var += c * op.size;
      maxc = c > maxc ? c : maxc;
    } else if (op.kind == SPK_OP_OPTION) {
      var += op_rec_count(op, rec) * op.size;  // not a container: no width
    } else if (op.kind == SPK_OP_VARINT) {
      var += vi_len(vi_value(op, rec));
    }
  }
}

__device__ __forceinline__ uint32_t wlog(uint32_t w) {
  return w == 1 ? 0 : w == 2 ? 1 : w == 4 ? 2 : 3;
}

// ---- block-wide helpers ----------------------------------------------------
// v of the lane selected by DPP control CTRL in the rows of ROW_MASK, 0 where
// the source lane is outside the row / the row is masked (both halves moved
// by the same lane permutation)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK,
                                                             0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL,
                                                             ROW_MASK, 0xf, false);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
// Inclusive wave64 prefix sum on the DPP network (no LDS round trips, unlike
// __shfl_up's ds_bpermute): row_shr 1/2/4/8 within each row of 16 lanes, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3).
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  v += dpp_u64<0x111, 0xf>(v);
  v += dpp_u64<0x112, 0xf>(v);
  v += dpp_u64<0x114, 0xf>(v);
  v += dpp_u64<0x118, 0xf>(v);
  v += dpp_u64<0x142, 0xa>(v);
  v += dpp_u64<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ uint64_t wave_lane63(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// exclusive scan over the block; returns prefix, sets *total
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t *total, uint64_t *sh) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  uint64_t base = 0, tot = 0;
  for (uint32_t i = 0; i < blockDim.x / 64; ++i) {
    if (i < wv) base += sh[i];
    tot += sh[i];
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__device__ uint64_t block_max(uint64_t v, uint64_t *sh) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t u = __shfl_down(v, o);
    v = u > v ? u : v;
  }
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t m = 0;
  for (uint32_t i = 0; i < blockDim.x / 64; ++i) m = sh[i] > m ? sh[i] : m;
  __syncthreads();
  return m;
}

// ===========================================================================
// ENCODE
// ===========================================================================
// Plan scratch (ws + kWsScratch): per plan block b its byte sum psum[b] (after the scan: the block's base) and
// largest count pmax[b], and per write block its sum wsub[b * kPlanSub + j]
// (round 4: an array of {sum, maxc, sub[]} structs, which the single-block
// finalize read at a 48-B stride)
constexpr size_t kPlanHead = 256;
struct PlanScratch {
  uint64_t *psum, *pmax, *wsub;
};
__host__ __device__ inline PlanScratch plan_scratch(uint8_t *ws, uint64_t nb) {
  PlanScratch q;
  q.psum = reinterpret_cast<uint64_t *>(ws + kWsScratch + kPlanHead);
  q.pmax = q.psum + nb;
  q.wsub = q.pmax + nb;
  return q;
}
static size_t plan_scratch_bytes(uint64_t nb) { return kPlanHead + nb * (2 + kPlanSub) * 8; }

#ifndef SPK_PLAN_SMALL  // <= kPlanRPB records: one fused plan launch (var_plan_small)
#define SPK_PLAN_SMALL 1
#endif
struct FinArgs {
  spk_msgfmt fmt;
  uint64_t n;
  uint32_t n_cont;  // width-w count fields per record
  int mode;
};

// var_plan_finalize (one block): exclusive scan of psum[0, nb) in place (each
// block's base) and the largest count, then header bytes and the plan. Chunks
// of kFinThreads x kFinPer values (C3's 9,766 in one), loaded coalesced and
// all at once, with one wave scanning the chunk's wave totals (round 4: ten
// 1024-wide block scans over 48-B strided structs, 22 us).
constexpr uint32_t kFinPer = 16, kFinThreads = 1024;
constexpr uint32_t kFinTW = kFinPer * (kFinThreads / 64);  // wave totals per chunk
constexpr uint32_t kFinG = kFinTW / 64;                     // ... per lane of the scanning wave
__device__ __forceinline__ void plan_result(const FinArgs &a, uint64_t carry, uint64_t mx,
                                            uint8_t *__restrict__ ws,
                                            spk_plan_t *__restrict__ plan);
__global__ __launch_bounds__(kFinThreads) void var_plan_finalize(FinArgs a, uint64_t nb,
                                                                 uint8_t *__restrict__ ws,
                                                                 spk_plan_t *__restrict__ plan) {
  __shared__ uint64_t tw[kFinTW + 1];
  const PlanScratch q = plan_scratch(ws, nb);
  constexpr uint32_t NW = kFinThreads / 64;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint64_t carry = 0, mx = 0;
  for (uint64_t c0 = 0; c0 < nb; c0 += (uint64_t)kFinThreads * kFinPer) {
    uint64_t v[kFinPer], inc[kFinPer];
#pragma unroll
    for (uint32_t k = 0; k < kFinPer; ++k) {
      const uint64_t b = c0 + (uint64_t)k * kFinThreads + t;
      v[k] = b < nb ? q.psum[b] : 0;
      const uint64_t m = b < nb ? q.pmax[b] : 0;
      mx = m > mx ? m : mx;
    }
#pragma unroll
    for (uint32_t k = 0; k < kFinPer; ++k) {
      inc[k] = wave_incl_scan(v[k]);
      if (lane == 63) tw[k * NW + wv] = inc[k];
    }
    __syncthreads();
    if (wv == 0) {  // lane l: wave totals [l * kFinG, (l + 1) * kFinG)
      uint64_t x[kFinG], ls = 0;
#pragma unroll
      for (uint32_t g = 0; g < kFinG; ++g) {
        x[g] = tw[lane * kFinG + g];
        ls += x[g];
      }
      const uint64_t li = wave_incl_scan(ls);
      uint64_t run = li - ls;
#pragma unroll
      for (uint32_t g = 0; g < kFinG; ++g) {
        tw[lane * kFinG + g] = run;
        run += x[g];
      }
      if (lane == 63) tw[kFinTW] = li;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kFinPer; ++k) {
      const uint64_t b = c0 + (uint64_t)k * kFinThreads + t;
      if (b < nb) q.psum[b] = carry + tw[k * NW + wv] + inc[k] - v[k];
    }
    carry += tw[kFinTW];
    __syncthreads();  // tw is reused
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t u = __shfl_down(mx, o);
    mx = u > mx ? u : mx;
  }
  if (lane == 0) tw[wv] = mx;
  __syncthreads();
  if (t != 0) return;
  for (uint32_t w = 1; w < NW; ++w) mx = tw[w] > mx ? tw[w] : mx;
  plan_result(a, carry, mx, ws, plan);
}
// the plan from the payload byte sum and the largest count (one thread)
__device__ __forceinline__ void plan_result(const FinArgs &a, uint64_t carry, uint64_t mx,
                                            uint8_t *__restrict__ ws,
                                            spk_plan_t *__restrict__ plan) {
  spk_plan_t r;
  if (a.mode == SPK_MODE_VECTOR) {
    const uint64_t maxc = mx > a.n ? mx : a.n;  // outer vector counts too
    const uint32_t w = width_of(maxc);
    const HdrShape h = hdr_shape(a.fmt.flags, a.fmt.literal_len, w);
    uint8_t *hb = ws + kWsHdrVec;
    const uint32_t len = write_hdr(hb, a.fmt, w);
    for (uint32_t i = 0; i < w; ++i) hb[len + i] = (uint8_t)(a.n >> (8 * i));
    r.total_bytes = len + w + carry + a.n * (uint64_t)a.n_cont * w;
    r.max_count = maxc;
    r.var_bytes = carry;
    r.width = w;
    r.header_bytes = len + w;
    r.metainfo = h.meta;
    r.has_meta = h.has_meta;
  } else {
    r.total_bytes = carry;
    r.max_count = mx;
    r.var_bytes = 0;
    r.width = width_of(mx);
    r.header_bytes = 0;
    r.metainfo = 0;
    r.has_meta = 0;
  }
  *plan = r;
}

// Per plan block (kPlanSub write blocks of kRPB records): the byte sums and
// the largest count. (A last-block-out finalize inside this kernel measured
// 6x slower for C3: 9,766 agent-scope release fences and same-address adds.)
__device__ __forceinline__ void plan_reduce_body(const VarArgs &a, const uint8_t *__restrict__ recs,
                                                 uint8_t *__restrict__ ws,
                                                 const uint8_t *__restrict__ hdrlen_tbl,
                                                 uint64_t bx, uint64_t nb,
                                                 uint64_t (*red)[kThreads / 64]) {
  const uint64_t N = dev_count(a.n, a.dn);
  const uint64_t r0 = bx * kPlanRPB;
  // every record's sizes first (all loads in flight at once), then one block
  // reduction of the kPlanSub write-block sums and the max (round 4: a block
  // scan per write block, its loads waiting on the previous scan's barriers)
  uint64_t mx = 0, sub[kPlanSub];
#pragma unroll
  for (int j = 0; j < kPlanSub; ++j) {  // write block j: kIPT rounds of kThreads records
    sub[j] = 0;
#pragma unroll
    for (int q = 0; q < kIPT; ++q) {
      const uint64_t i = r0 + (uint64_t)j * kRPB + (uint64_t)q * kThreads + threadIdx.x;
      if (i < N) {
        uint64_t var, maxc;
        rec_sizes(a.L, recs + i * a.L.stride, var, maxc);
        if (a.mode == SPK_MODE_VECTOR) {
          sub[j] += var;
        } else {
          const uint32_t w = width_of(maxc);
          sub[j] += hdrlen_tbl[wlog(w)] + var + (uint64_t)a.L.n_cont * w;
        }
        mx = maxc > mx ? maxc : mx;
      }
    }
  }
#pragma unroll
  for (int j = 0; j <= kPlanSub; ++j) {
    uint64_t v = j < kPlanSub ? sub[j] : mx;
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t x = __shfl_down(v, o);
      v = j < kPlanSub ? v + x : (x > v ? x : v);
    }
    if ((threadIdx.x & 63) == 0) red[j][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  const PlanScratch q = plan_scratch(ws, nb);
  if (threadIdx.x == 0) {
    uint64_t sum = 0, m = 0;
    for (int j = 0; j < kPlanSub; ++j) {
      uint64_t t = 0;
      for (uint32_t w = 0; w < kThreads / 64; ++w) t += red[j][w];
      q.wsub[bx * kPlanSub + j] = t;
      sum += t;
    }
    for (uint32_t w = 0; w < kThreads / 64; ++w) m = red[kPlanSub][w] > m ? red[kPlanSub][w] : m;
    q.psum[bx] = sum;
    q.pmax[bx] = m;
  }
}
__global__ __launch_bounds__(kThreads) void var_plan_reduce(
    VarArgs a, const uint8_t *__restrict__ recs, uint8_t *__restrict__ ws,
    const uint8_t *__restrict__ hdrlen_tbl) {
  __shared__ uint64_t red[kPlanSub + 1][kThreads / 64];
  plan_reduce_body(a, recs, ws, hdrlen_tbl, blockIdx.x, gridDim.x, red);
}

// message headers per width for MESSAGES mode (host computes: no data needed)
struct MsgHdrTable {
  uint8_t len[4];
  uint8_t bytes[4][4 + 1 + SPK_MAX_LITERAL + 1];
};

__device__ __forceinline__ void msg_hdrs_body(const MsgHdrTable &t, uint8_t *ws) {
  for (int s = 0; s < 4; ++s)
    for (uint32_t i = threadIdx.x; i < t.len[s]; i += blockDim.x)
      ws[kWsHdrMsg + s * kWsHdrSlot + i] = t.bytes[s][i];
  if (threadIdx.x < 4) ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + threadIdx.x] = t.len[threadIdx.x];
}
__global__ void write_msg_hdrs(MsgHdrTable t, uint8_t *ws) { msg_hdrs_body(t, ws); }

// the plan of at most kPlanRPB records (a small call): header table, block
// sums and the plan in one launch of one block instead of three
__global__ __launch_bounds__(kThreads) void var_plan_small(VarArgs a, FinArgs f, MsgHdrTable t,
                                                           const uint8_t *__restrict__ recs,
                                                           uint8_t *__restrict__ ws,
                                                           spk_plan_t *__restrict__ plan) {
  __shared__ uint64_t red[kPlanSub + 1][kThreads / 64];
  if (a.mode == SPK_MODE_MESSAGES) msg_hdrs_body(t, ws);
  __syncthreads();
  plan_reduce_body(a, recs, ws, ws + kWsHdrMsg + 4 * kWsHdrSlot - 8, 0, 1, red);
  if (threadIdx.x != 0) return;
  const PlanScratch q = plan_scratch(ws, 1);
  const uint64_t carry = q.psum[0], mx = q.pmax[0];
  q.psum[0] = 0;  // (the exclusive scan of one block sum)
  plan_result(f, carry, mx, ws, plan);
}

// ---- LDS-staged output ------------------------------------------------------
// Partial, unaligned stores straight to HBM cost 2-4x their bytes in write
// traffic (measured with WRITE_SIZE), so a block assembles its contiguous
// output range in an LDS window with byte stores fed by wide unaligned
// global loads, then flushes it with aligned 16-B stores.
struct Win {
  uint8_t *lds;
  uint64_t lo, hi;  // output byte range currently held [lo, hi)
};

__device__ __forceinline__ void lds_put_u32(uint8_t *d, uint32_t v, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) d[i] = (uint8_t)(v >> (8 * i));
}

// bytes [pos, pos+n) of the output come from src[0, n): store the part that
// falls in the window. LDS: W.lds is the LDS window, written with byte-aligned
// 4 / 8 / 16-B DS stores (round 4: one ds_write_b8 per byte); otherwise it is
// global memory (the direct mode), written bytewise.
template <bool LDS = false>
__device__ __forceinline__ void win_put(const Win &W, uint64_t pos, const uint8_t *src,
                                        uint64_t n) {
  const uint64_t a = pos > W.lo ? pos : W.lo;
  const uint64_t b = pos + n < W.hi ? pos + n : W.hi;
  if (a >= b) return;
  uint64_t i = a - pos;
  const uint64_t e = b - pos;
  uint8_t *d = W.lds + (pos - W.lo);
  if constexpr (LDS) {
    for (; i + 16 <= e; i += 16)
      *(lds_v4u_una *)(d + i) = *reinterpret_cast<const v4u_una *>(src + i);
    if (e - i >= 8) {
      *(lds_u64_una *)(d + i) = *reinterpret_cast<const u64_unaligned *>(src + i);
      i += 8;
    }
    if (e - i >= 4) {
      *(lds_u32_una *)(d + i) = *reinterpret_cast<const u32_unaligned *>(src + i);
      i += 4;
    }
    for (; i < e; ++i) d[i] = src[i];
    return;
  }
  for (; i + 16 <= e; i += 16) {
    const v4u_t v = *reinterpret_cast<const v4u_una *>(src + i);
    lds_put_u32(d + i, v.x, 4);
    lds_put_u32(d + i + 4, v.y, 4);
    lds_put_u32(d + i + 8, v.z, 4);
    lds_put_u32(d + i + 12, v.w, 4);
  }
  if (e - i >= 8) {
    const uint64_t v = *reinterpret_cast<const u64_unaligned *>(src + i);
    lds_put_u32(d + i, (uint32_t)v, 4);
    lds_put_u32(d + i + 4, (uint32_t)(v >> 32), 4);
    i += 8;
  }
  if (e - i >= 4) {
    lds_put_u32(d + i, *reinterpret_cast<const u32_unaligned *>(src + i), 4);
    i += 4;
  }
  for (; i < e; ++i) d[i] = src[i];
}

// little-endian w-byte value at output position pos
__device__ __forceinline__ void win_put_le(const Win &W, uint64_t pos, uint64_t v, uint32_t w) {
  for (uint32_t i = 0; i < w; ++i) {
    const uint64_t x = pos + i;
    if (x >= W.lo && x < W.hi) W.lds[x - W.lo] = (uint8_t)(v >> (8 * i));
  }
}

// one record at output position pos (width w) into the window; span payloads
// whose bit is set in `skip` are copied cooperatively by the block instead
template <bool LDS = false>
__device__ __forceinline__ void win_record(const VarArgs &a, const uint8_t *rec, uint32_t w,
                                           uint64_t pos, const Win &W, uint32_t skip = 0) {
  uint32_t sk = 0;
  for (uint32_t o = 0; o < a.L.n_ops; ++o) {
    const spk_op op = a.L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      win_put<LDS>(W, pos, rec + op.rec_off, op.size);
      pos += op.size;
    } else if (op.kind == SPK_OP_VARINT) {  // serialize_varint (varint.hpp:245-268)
      uint64_t v = vi_value(op, rec);
      for (;;) {
        const uint8_t b = (uint8_t)(v >= 0x80 ? (v | 0x80u) : v);
        if (pos >= W.lo && pos < W.hi) W.lds[pos - W.lo] = b;
        ++pos;
        if (v < 0x80) break;
        v >>= 7;
      }
    } else {
      const uint64_t c = op_rec_count(op, rec);
      const uint32_t pw = op_pw(op, w);
      win_put_le(W, pos, c, pw);
      pos += pw;
      const uint64_t nb = c * op.size;
      if (nb && !(skip >> sk & 1)) win_put<LDS>(W, pos, a.heaps[sk] + rec_u64(rec, op.aux) * op.size, nb);
      pos += nb;
      ++sk;
    }
  }
}

// ---- block-cooperative copies of large span payloads --------------------------
// One lane copying a multi-KiB string / vector payload serialises the block
// (e.g. the std::vector<int>(1K) messages of C5). Payloads of at least
// kBigBytes are listed per block (in record order, via a block scan) and
// copied by all lanes together: aligned 16-B destination chunks fed by
// unaligned 16-B source loads.
constexpr uint32_t kBigBytes = 256;
constexpr uint32_t kBigMax = 256;  // list capacity per block (overflow: lane copies)

struct BigSeg {
  uint64_t dst;        // encode: output byte position; decode: unused
  uint8_t *dptr;       // decode: destination pointer
  const uint8_t *src;
  uint64_t n;
};

// bytes [pos, pos+n) of the output come from src: the part inside the window,
// written by the whole block (16-B aligned LDS chunks, bytes at the edges)
__device__ __forceinline__ void win_put_coop(const Win &W, uint64_t pos, const uint8_t *src,
                                             uint64_t n) {
  const uint64_t a = pos > W.lo ? pos : W.lo;
  const uint64_t b = pos + n < W.hi ? pos + n : W.hi;
  if (a >= b) return;
  const uint64_t ca = (a + 15) & ~15ull, cb = b & ~15ull;  // W.lo is 16-aligned
  if (ca >= cb) {
    for (uint64_t x = a + threadIdx.x; x < b; x += blockDim.x) W.lds[x - W.lo] = src[x - pos];
    return;
  }
  for (uint64_t x = a + threadIdx.x; x < ca; x += blockDim.x) W.lds[x - W.lo] = src[x - pos];
  for (uint64_t x = cb + threadIdx.x; x < b; x += blockDim.x) W.lds[x - W.lo] = src[x - pos];
  for (uint64_t c = ca + 16 * (uint64_t)threadIdx.x; c < cb; c += 16 * (uint64_t)blockDim.x)
    *reinterpret_cast<v4u_t *>(W.lds + (c - W.lo)) =
        *reinterpret_cast<const v4u_una *>(src + (c - pos));
}

#ifndef SPK_COOP_NT  // wave_copy_all: bit 0 non-temporal loads, bit 1 stores
#define SPK_COOP_NT 3  // (C5 1.667 -> 1.559 ms per step, c3l encode 1.707 -> 1.532 ms; same-box A/B)
#endif
#ifndef SPK_COOP_U
#define SPK_COOP_U 8
#endif
constexpr int kCoopU = SPK_COOP_U;  // loads in flight per lane in wave_copy_all
constexpr unsigned kYSplit = 8;  // blocks sharing one write block's output

// All m listed payloads (B[k].dptr <- B[k].src, B[k].n bytes), one wave per
// payload (payload k by wave k mod the waves of all nparts blocks): aligned
// 16-B destination chunks fed by unaligned 16-B source loads, kCoopU loads in
// flight per lane, head/tail bytes by single lanes. (A block-wide flattened
// chunk index over all payloads, searched per chunk, measured 13 % slower on
// C5's vector<int> messages.)
// one payload's head / tail bytes (single lanes) and its 16-B chunk count
__device__ __forceinline__ uint64_t seg_edges(const BigSeg &e, uint32_t lane, uint64_t *head) {
  uint64_t h = (16 - ((uintptr_t)e.dptr & 15)) & 15;
  if (h > e.n) h = e.n;
  const uint64_t nc = (e.n - h) >> 4, tail = h + 16 * nc;
  if (lane < h) e.dptr[lane] = e.src[lane];
  if (lane < e.n - tail) e.dptr[tail + lane] = e.src[tail + lane];
  *head = h;
  return nc;
}
__device__ __forceinline__ void wave_copy_all(const BigSeg *B, uint32_t m, uint32_t part,
                                              uint32_t nparts) {
  const uint32_t lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t gw = part * nw + (threadIdx.x >> 6), W = nparts * nw;
  for (uint32_t k = gw; k < m; k += W) {
    const BigSeg e = B[k];
    uint64_t head = (16 - ((uintptr_t)e.dptr & 15)) & 15;
    if (head > e.n) head = e.n;
    const uint64_t nc = (e.n - head) >> 4, tail = head + 16 * nc;
    if (lane < head) e.dptr[lane] = e.src[lane];
    if (lane < e.n - tail) e.dptr[tail + lane] = e.src[tail + lane];
    const uint8_t *src = e.src + head;
    uint8_t *dst = e.dptr + head;
    for (uint64_t c0 = lane; c0 < nc; c0 += 64 * kCoopU) {
      v4u_t v[kCoopU];
#pragma unroll
      for (int u = 0; u < kCoopU; ++u)
        if (c0 + 64 * u < nc) {
          const v4u_una *q = reinterpret_cast<const v4u_una *>(src + 16 * (c0 + 64 * u));
          v[u] = (SPK_COOP_NT & 1) ? __builtin_nontemporal_load(q) : *q;
        }
#pragma unroll
      for (int u = 0; u < kCoopU; ++u)
        if (c0 + 64 * u < nc) {
          v4u_t *q = reinterpret_cast<v4u_t *>(dst + 16 * (c0 + 64 * u));
          if (SPK_COOP_NT & 2) __builtin_nontemporal_store(v[u], q);
          else *q = v[u];
        }
    }
  }
}

// d[0, n) = s[0, n) by the whole block
__device__ __forceinline__ void coop_copy(uint8_t *d, const uint8_t *s, uint64_t n) {
  uint64_t head = (16 - ((uintptr_t)d & 15)) & 15;
  if (head > n) head = n;
  const uint64_t body = (n - head) & ~15ull;
  for (uint64_t x = threadIdx.x; x < head; x += blockDim.x) d[x] = s[x];
  for (uint64_t x = head + body + threadIdx.x; x < n; x += blockDim.x) d[x] = s[x];
  for (uint64_t c = threadIdx.x; c < body / 16; c += blockDim.x)
    *reinterpret_cast<v4u_t *>(d + head + 16 * c) =
        *reinterpret_cast<const v4u_una *>(s + head + 16 * c);
}

// frame prefix of message i (payload length plen) at output position pos:
// the template with the sequence number and length fields patched
__device__ __forceinline__ void win_frame(const VarArgs &a, const Win &W, uint64_t pos,
                                          uint64_t i, uint64_t plen) {
  for (uint32_t x = 0; x < a.fpre; ++x) {
    const uint64_t y = pos + x;
    if (y < W.lo || y >= W.hi) continue;
    uint8_t v = a.ftmpl[x];
    if (x >= a.fseq_off && x - a.fseq_off < 4)
      v = (uint8_t)(seq_value(a.echo, a.fseq_base, i) >> (8 * (x - a.fseq_off)));
    if (x >= a.flen_off && x - a.flen_off < 4) v = (uint8_t)(plen >> (8 * (x - a.flen_off)));
    W.lds[y - W.lo] = v;
  }
}

// LDS assembly window per block. (Round 6: the block's records staged in LDS
// beside a 16 KiB window: C3 0.321 -> 0.311 ms, but C4's 19 KiB blocks then
// took two window passes, 0.373 -> 0.477 ms; with the 20 KiB window the LDS
// leaves one block per SIMD less. Not kept.)
constexpr uint32_t kEncWin = 20 * 1024;

// Write pass: records r0 + j*kThreads + tid (consecutive lanes on consecutive
// records), byte offsets from a block scan per round on top of the block's
// planned base; the block's output range is assembled window by window.
__device__ __forceinline__ void encode_write_body(
    const VarArgs &a, const uint8_t *__restrict__ recs, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint8_t *__restrict__ ws, const spk_plan_t *__restrict__ plan,
    uint64_t *__restrict__ offs, uint64_t bx, uint64_t gx, uint32_t by, uint32_t gy,
    uint8_t *lds, uint64_t *sh, BigSeg *big) {
  const uint64_t N = dev_count(a.n, a.dn);
  const uint64_t total =
      plan->total_bytes + (a.mode == SPK_MODE_MESSAGES ? N * (uint64_t)a.fpre : 0);
  if (total > out_cap) return;  // caller reads plan->total_bytes
  const uint32_t w_vec = plan->width;
  const uint32_t hdr_vec = plan->header_bytes;
  const PlanScratch ps = plan_scratch(const_cast<uint8_t *>(ws), (gx + kPlanSub - 1) / kPlanSub);
  const uint64_t r0 = bx * kRPB;
  // output base of write block b (b == gridDim.x: the end of the output)
  auto base_of = [&](uint64_t b) -> uint64_t {
    if (b >= gx) return total;
    uint64_t gb = ps.psum[b / kPlanSub];
    for (uint32_t j = 0; j < b % kPlanSub; ++j) gb += ps.wsub[b / kPlanSub * kPlanSub + j];
    const uint64_t rb = b * kRPB;
    return a.mode == SPK_MODE_VECTOR ? hdr_vec + gb + rb * (uint64_t)a.L.n_cont * w_vec
                                     : gb + rb * (uint64_t)a.fpre;
  };
  const uint64_t g0 = base_of(bx);
  // Window split: gridDim.y blocks share one write block's output range, block
  // y assembling windows y, y + gridDim.y, ... (a few blocks of multi-KiB
  // messages would otherwise leave most CUs idle). The range end comes from
  // the next block's base, so a block without windows leaves before reading
  // any record.
  const uint32_t ysub = by, ny = gy;
  if (ysub > 0) {
    const uint64_t ge = base_of(bx + 1);
    if ((g0 & ~15ull) + (uint64_t)ysub * kEncWin >= ge) return;
  }
  if (a.mode == SPK_MODE_VECTOR && bx == 0 && ysub == 0)
    for (uint32_t i = threadIdx.x; i < hdr_vec; i += blockDim.x) out[i] = ws[kWsHdrVec + i];
  const uint8_t *rbase = recs + r0 * a.L.stride;
#define SPK_REC(i) (rbase + ((i) - r0) * a.L.stride)
  uint64_t pj[kIPT], szj[kIPT];
  uint32_t wj[kIPT];
  uint64_t g = g0;
  for (int j = 0; j < kIPT; ++j) {
    const uint64_t i = r0 + (uint64_t)j * kThreads + threadIdx.x;
    uint64_t sz = 0;
    uint32_t w = w_vec;
    if (i < N) {
      uint64_t var, maxc;
      rec_sizes(a.L, SPK_REC(i), var, maxc);
      if (a.mode == SPK_MODE_VECTOR) {
        sz = var + (uint64_t)a.L.n_cont * w_vec;
      } else {
        w = width_of(maxc);
        sz = a.fpre + ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + wlog(w)] + var +
             (uint64_t)a.L.n_cont * w;
      }
    }
    uint64_t btot;
    pj[j] = g + block_excl_scan(sz, &btot, sh);
    szj[j] = sz;
    wj[j] = w;
    g += btot;
    if (a.mode == SPK_MODE_MESSAGES && offs && i < N && ysub == 0) offs[i] = pj[j];
  }
  if (a.mode == SPK_MODE_MESSAGES && offs && bx == gx - 1 && threadIdx.x == 0 &&
      ysub == 0)
    offs[N] = total;
  const uint64_t g1 = g;
  if (g1 == g0) return;
  // large span payloads of this block's records -> cooperative list
  uint32_t skip[kIPT];
  uint64_t nbig_tot = 0, big_bytes = 0;
  for (int j = 0; j < kIPT; ++j) {  // list order = record order = output order
    skip[j] = 0;
    const uint64_t i = r0 + (uint64_t)j * kThreads + threadIdx.x;
    uint32_t nbig = 0;
    if (i < N) {
      const uint8_t *rec = SPK_REC(i);
      for (uint32_t o = 0; o < a.L.n_ops; ++o)
        if ((a.L.ops[o].kind == SPK_OP_SPAN || a.L.ops[o].kind == SPK_OP_OPTION) &&
            op_rec_count(a.L.ops[o], rec) * a.L.ops[o].size >= kBigBytes)
          ++nbig;
    }
    uint64_t round_tot;
    uint64_t slot = nbig_tot + block_excl_scan(nbig, &round_tot, sh);
    nbig_tot += round_tot;
    if (nbig && slot + nbig <= kBigMax) {
      const uint8_t *rec = SPK_REC(i);
      uint64_t q = pj[j];
      if (a.mode == SPK_MODE_MESSAGES)
        q += a.fpre + ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + wlog(wj[j])];
      uint32_t sk = 0;
      for (uint32_t o = 0; o < a.L.n_ops; ++o) {
        const spk_op op = a.L.ops[o];
        if (op.kind == SPK_OP_COPY) {
          q += op.size;
          continue;
        }
        if (op.kind == SPK_OP_VARINT) {
          q += vi_len(vi_value(op, rec));
          continue;
        }
        const uint64_t nb = op_rec_count(op, rec) * op.size;
        q += op_pw(op, wj[j]);
        if (nb >= kBigBytes) {
          big[slot++] = BigSeg{q, out + q, a.heaps[sk] + rec_u64(rec, op.aux) * op.size, nb};
          skip[j] |= 1u << sk;
          big_bytes += nb;
        }
        q += nb;
        ++sk;
      }
    }
  }
  // Direct mode: when the listed payloads are >= 7/8 of the block's output
  // (multi-KiB strings / vectors, e.g. C5's vector<int>), the LDS windows would
  // only relay payload bytes. The record bytes around them are then stored
  // straight to HBM by their lanes (a few partial stores per record) and the
  // payloads are copied HBM to HBM with aligned 16-B stores, the copy split
  // over the gridDim.y blocks of this write block.
  if (nbig_tot && nbig_tot <= kBigMax) {
    uint64_t bb_tot;
    block_excl_scan(big_bytes, &bb_tot, sh);
    if (bb_tot * 8 >= (g1 - g0) * 7) {
      if (ysub == 0) {
        const Win D{out, 0, ~0ull};
        for (int j = 0; j < kIPT; ++j) {
          const uint64_t i = r0 + (uint64_t)j * kThreads + threadIdx.x;
          if (i >= N) continue;
          uint64_t q = pj[j];
          if (a.mode == SPK_MODE_MESSAGES) {
            if (a.fpre) {
              win_frame(a, D, q, i, szj[j] - a.fpre);
              q += a.fpre;
            }
            const uint32_t sl = wlog(wj[j]);
            const uint32_t hl = ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + sl];
            win_put(D, q, ws + kWsHdrMsg + sl * kWsHdrSlot, hl);
            q += hl;
          }
          win_record(a, SPK_REC(i), wj[j], q, D, skip[j]);
        }
      }
      __syncthreads();  // the payload list
      // the blocks of this write block that did not leave at the top
      const uint64_t nwin = ((g1 - (g0 & ~15ull)) + kEncWin - 1) / kEncWin;
      wave_copy_all(big, (uint32_t)nbig_tot, ysub, nwin < ny ? (uint32_t)nwin : ny);
      return;
    }
  }
  if (nbig_tot > kBigMax) nbig_tot = kBigMax;
  __syncthreads();
  uint32_t k0 = 0;  // first list entry that may reach the current window
  for (uint64_t wlo = (g0 & ~15ull) + (uint64_t)ysub * kEncWin; wlo < g1; wlo += ny * kEncWin) {
    const Win W{lds, wlo, wlo + kEncWin < g1 ? wlo + kEncWin : g1};
    for (int j = 0; j < kIPT; ++j) {
      const uint64_t i = r0 + (uint64_t)j * kThreads + threadIdx.x;
      if (i >= N || pj[j] >= W.hi || pj[j] + szj[j] <= W.lo) continue;
      uint64_t q = pj[j];
      if (a.mode == SPK_MODE_MESSAGES) {
        if (a.fpre) {
          win_frame(a, W, q, i, szj[j] - a.fpre);
          q += a.fpre;
        }
        const uint32_t sl = wlog(wj[j]);
        const uint32_t hl = ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + sl];
        win_put<true>(W, q, ws + kWsHdrMsg + sl * kWsHdrSlot, hl);
        q += hl;
      }
      win_record<true>(a, SPK_REC(i), wj[j], q, W, skip[j]);
    }
    // listed payloads are in output order: fill the window slots they cover
    while (k0 < nbig_tot && big[k0].dst + big[k0].n <= W.lo) ++k0;
    for (uint32_t k = k0; k < nbig_tot && big[k].dst < W.hi; ++k)
      win_put_coop(W, big[k].dst, big[k].src, big[k].n);
    __syncthreads();
    // flush [max(W.lo, g0), W.hi): aligned 16-B chunks, bytes at the edges
    for (uint64_t c = W.lo + (uint64_t)threadIdx.x * 16; c < W.hi; c += kThreads * 16) {
      const uint64_t lo = c > g0 ? c : g0;
      const uint64_t hi = c + 16 < W.hi ? c + 16 : W.hi;
      if (lo == c && hi == c + 16) {
        flush16(out + c, *reinterpret_cast<const v4u_t *>(lds + (c - W.lo)));
      } else {
        for (uint64_t x = lo; x < hi; ++x) out[x] = lds[x - W.lo];
      }
    }
    __syncthreads();
  }
}
__global__ __launch_bounds__(kThreads, 5) void var_encode_write(
    VarArgs a, const uint8_t *__restrict__ recs, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint8_t *__restrict__ ws,
    const spk_plan_t *__restrict__ plan, uint64_t *__restrict__ offs) {
  __shared__ __align__(16) uint8_t lds[kEncWin];
  __shared__ uint64_t sh[kThreads / 64];
  __shared__ BigSeg big[kBigMax];
  encode_write_body(a, recs, out, out_cap, ws, plan, offs, blockIdx.x, gridDim.x, blockIdx.y,
                    gridDim.y, lds, sh, big);
}

// plan + write of at most kRPB records (a small call's message) in one launch
// of one block: var_plan_small's phases, then the one write block's
__global__ __launch_bounds__(kThreads) void var_plan_encode_small(
    VarArgs a, FinArgs f, MsgHdrTable t, const uint8_t *__restrict__ recs,
    uint8_t *__restrict__ out, uint64_t out_cap, uint8_t *__restrict__ ws,
    spk_plan_t *__restrict__ plan, uint64_t *__restrict__ offs) {
  __shared__ __align__(16) uint8_t lds[kEncWin];
  __shared__ uint64_t sh[kThreads / 64];
  __shared__ BigSeg big[kBigMax];
  __shared__ uint64_t red[kPlanSub + 1][kThreads / 64];
  if (a.mode == SPK_MODE_MESSAGES) msg_hdrs_body(t, ws);
  __syncthreads();
  plan_reduce_body(a, recs, ws, ws + kWsHdrMsg + 4 * kWsHdrSlot - 8, 0, 1, red);
  if (threadIdx.x == 0) {
    const PlanScratch q = plan_scratch(ws, 1);
    const uint64_t carry = q.psum[0], mx = q.pmax[0];
    q.psum[0] = 0;  // (the exclusive scan of one block sum)
    plan_result(f, carry, mx, ws, plan);
  }
  __syncthreads();
  encode_write_body(a, recs, out, out_cap, ws, plan, offs, 0, 1, 0, 1, lds, sh, big);
}
#undef SPK_REC

// ===========================================================================
// DECODE — shared record walker over the wire
// ===========================================================================

// Size of the record starting at `pos` (absolute), reading counts from
// `wire` (length len). Returns 0 if the record does not fit (incomplete).
// A bad varint sets *ec to invalid_buffer (otherwise a 0 is no_buffer_space).
__device__ __forceinline__ uint64_t rec_wire_len(const KLayout &L, const uint8_t *wire,
                                                 uint64_t len, uint64_t pos, uint32_t w,
                                                 int32_t *ec = nullptr) {
  const uint64_t p0 = pos;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      pos += op.size;
      if (pos > len) return 0;
    } else if (op.kind == SPK_OP_VARINT) {
      uint64_t v;
      const uint32_t l = vi_read(WireBytes{wire}, pos, len, &v);
      if (l == kViBad && ec) *ec = SPK_ERRC_INVALID_BUFFER;
      if (!l || l == kViBad) return 0;
      pos += l;
    } else {
      const uint32_t pw = op_pw(op, w);
      if (pos + pw > len) return 0;
      const uint64_t c = op.kind == SPK_OP_OPTION ? (uint64_t)(wire[pos] != 0) : ld_le(wire + pos, w);
      pos += pw;
      if (c) {
        uint64_t nb;
        if (!span_nb(c, op.size, &nb)) return 0;
        if (nb > len - pos) {
          if (op.kind != SPK_OP_OPTION) return 0;
        } else {
          pos += nb;
        }
      }
    }
  }
  return pos - p0;
}

// Decode the record at `pos` into `rec` (device record) and its heaps.
// heap_off[k] = element offset where this record's span k goes.
__device__ void decode_record(const KLayout &L, const uint8_t *wire, uint64_t pos,
                              uint32_t w, uint8_t *rec, uint8_t *const *heaps,
                              const uint64_t *heap_off, uint64_t end, uint32_t skip = 0) {
  uint32_t sk = 0;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      copy_bytes(rec + op.rec_off, wire + pos, op.size);
      pos += op.size;
    } else if (op.kind == SPK_OP_VARINT) {
      uint64_t v = 0;
      pos += vi_read(WireBytes{wire}, pos, end, &v);
      vi_store(op, rec, v);
    } else {
      const uint64_t c = op.kind == SPK_OP_OPTION ? (uint64_t)(wire[pos] != 0) : ld_le(wire + pos, w);
      pos += op_pw(op, w);
      *reinterpret_cast<uint32_t *>(rec + op.rec_off) = (uint32_t)c;
      *reinterpret_cast<uint64_t *>(rec + op.aux) = heap_off[sk];
      const uint64_t nb = opt_nb(op, c, pos, end);
      uint8_t *hp = heaps[sk] + heap_off[sk] * op.size;
      if (c && !nb && op.kind == SPK_OP_OPTION)
        for (uint32_t b = 0; b < op.size; ++b) hp[b] = 0;  // unreadable value
      else if (!(skip >> sk & 1))
        copy_bytes(hp, wire + pos, nb);
      pos += nb;
      ++sk;
    }
  }
}

// counts of the record at pos (assumes it is complete)
__device__ __forceinline__ void rec_counts(const KLayout &L, const uint8_t *wire,
                                           uint64_t pos, uint32_t w, uint64_t *cnt,
                                           uint64_t end) {
  uint32_t sk = 0;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      pos += op.size;
    } else if (op.kind == SPK_OP_VARINT) {
      uint64_t v;
      pos += vi_read(WireBytes{wire}, pos, end, &v);
    } else {
      const uint64_t c = op.kind == SPK_OP_OPTION ? (uint64_t)(wire[pos] != 0) : ld_le(wire + pos, w);
      cnt[sk++] = c;
      pos += op_pw(op, w);
      pos += opt_nb(op, c, pos, end);
    }
  }
}

struct DecArgs {
  KLayout L;
  spk_msgfmt fmt;
  uint64_t wire_len;
  uint64_t n_msgs;
  uint64_t rec_cap;
  uint64_t heap_cap[kVS];
  uint8_t *heaps[kVS];
  uint32_t prefix;  // MESSAGES: frame bytes before every message
  uint32_t body_w;  // VECTOR, spk_decode_body: no header, body_n records at this width
  uint64_t body_n;
  uint32_t range;   // spk_decode_shard_index: tiles [range_t0, ...) of the body
  uint32_t nested;  // VECTOR tile decode of a nested layout (NS = -2; the layout at nl)
  uint64_t range_t0, range_entry;
  const uint64_t *ends;  // MESSAGES: message i ends at ends[i] (null: offs[i + 1])
  const uint64_t *dn;    // MESSAGES: device count (min(*dn, n_msgs)) or null
  const void *nl;        // nested: the NTLayout in device memory (workspace)
  // VECTOR pass of a compatible-member layout (launch_compat_tiles): device
  // words {start, n, w, data_len} in place of the header, or null
  const uint64_t *chain;
};


// ===========================================================================
// DECODE, SPK_MODE_MESSAGES
// ===========================================================================
// per-message state in workspace: u64 payload_pos (~0 = failed) | width
// per-block slots of the MESSAGES decode scan buffer: span totals, then the
// block's ok-message count and consumed bytes (summed by var_scan_blocks:
// no same-address atomics across thousands of blocks)
constexpr uint32_t kBs = kVS + 2;

struct MsgState {
  uint64_t pos;    // absolute payload position, ~0 if the message failed
  uint32_t w;
  int32_t errc;
};

#ifndef SPK_MSG_SMALL  // <= kThreads MESSAGES: one fused decode launch (var_msg_decode_small)
#define SPK_MSG_SMALL 1
#endif
__device__ __forceinline__ void msg_parse_body(const DecArgs &a, const uint8_t *__restrict__ wire,
                                               const uint64_t *__restrict__ offs,
                                               uint8_t *__restrict__ ws,
                                               int32_t *__restrict__ errc_out, spk_dresult_t *res,
                                               uint64_t bx, uint64_t *sh) {
  MsgState *st = reinterpret_cast<MsgState *>(ws + kWsScratch);
  uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + kWsScratch +
                                                sizeof(MsgState) * a.n_msgs);
  const uint64_t i = bx * kThreads + threadIdx.x;
  uint64_t cnt[kVS] = {};
  uint64_t ok = 0, consumed = 0;
  // more frames than the caller's n_max: the excess is not decoded
  if (a.dn && i == 0 && *a.dn > a.n_msgs) atomicExch(&res->errc, SPK_ERRC_CAPACITY);
  if (i < dev_count(a.n_msgs, a.dn)) {
    const uint64_t f = offs[i], e = a.ends ? a.ends[i] : offs[i + 1];
    const uint64_t b = f + a.prefix;  // struct_pack message after the frame prefix
    MsgState s{~0ull, 1, SPK_ERRC_OK};
    if (e < f || e > a.wire_len || e - f < a.prefix) {
      s.errc = SPK_ERRC_NO_BUFFER_SPACE;
    } else {
      uint64_t pos, dl;
      uint32_t w;
      s.errc = parse_hdr(a.fmt, wire + b, e - b, &pos, &w, &dl);
      if (!s.errc) {
        int32_t ec = SPK_ERRC_NO_BUFFER_SPACE;
        const uint64_t rl = rec_wire_len(a.L, wire + b, e - b, pos, w, &ec);
        if (!rl) {
          s.errc = ec;
        } else {
          if (i >= a.rec_cap) s.errc = SPK_ERRC_CAPACITY;
          s.pos = b + pos;
          s.w = w;
          rec_counts(a.L, wire, b + pos, w, cnt, e);
          ok = 1;
          consumed = pos + rl > dl ? pos + rl : dl;
        }
      }
    }
    if (s.errc) {
      s.pos = ~0ull;
      ok = 0;
      consumed = 0;
      for (int k = 0; k < kVS; ++k) cnt[k] = 0;
    }
    st[i] = s;
    if (errc_out) errc_out[i] = s.errc;
    if (s.errc == SPK_ERRC_CAPACITY) atomicExch(&res->errc, SPK_ERRC_CAPACITY);
  }
  for (uint32_t k = 0; k < a.L.n_spans; ++k) {
    uint64_t tot;
    block_excl_scan(cnt[k], &tot, sh);
    if (threadIdx.x == 0) bsum[bx * kBs + k] = tot;
  }
  uint64_t tok, tcons;
  block_excl_scan(ok, &tok, sh);
  block_excl_scan(consumed, &tcons, sh);
  if (threadIdx.x == 0) {
    bsum[bx * kBs + kVS] = tok;
    bsum[bx * kBs + kVS + 1] = tcons;
  }
}
__global__ __launch_bounds__(kThreads) void var_msg_parse(
    DecArgs a, const uint8_t *__restrict__ wire, const uint64_t *__restrict__ offs,
    uint8_t *__restrict__ ws, int32_t *__restrict__ errc_out, spk_dresult_t *res) {
  __shared__ uint64_t sh[kThreads / 64];
  msg_parse_body(a, wire, offs, ws, errc_out, res, blockIdx.x, sh);
}

// one block: exclusive scan of per-block span totals (in place), heap_used,
// capacity check
__device__ __forceinline__ void scan_blocks_body(uint64_t nblocks, uint32_t n_spans,
                                                 uint64_t *__restrict__ bsum, const DecArgs &a,
                                                 spk_dresult_t *res, uint64_t *sh) {
  for (uint32_t k = 0; k < n_spans; ++k) {
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nblocks; b0 += blockDim.x) {
      const uint64_t b = b0 + threadIdx.x;
      const uint64_t v = b < nblocks ? bsum[b * kBs + k] : 0;
      uint64_t tot;
      const uint64_t ex = block_excl_scan(v, &tot, sh);
      if (b < nblocks) bsum[b * kBs + k] = carry + ex;
      carry += tot;
    }
    if (threadIdx.x == 0) {
      res->heap_used[k] = carry;
      if (carry > a.heap_cap[k] && res->errc == 0) res->errc = SPK_ERRC_CAPACITY;
    }
  }
  // count / consumed: sums of the per-block partials
  for (uint32_t k = kVS; k < kBs; ++k) {
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nblocks; b0 += blockDim.x) {
      const uint64_t b = b0 + threadIdx.x;
      uint64_t tot;
      block_excl_scan(b < nblocks ? bsum[b * kBs + k] : 0, &tot, sh);
      carry += tot;
    }
    if (threadIdx.x == 0) {
      if (k == kVS)
        res->count = carry;
      else
        res->consumed = carry;
    }
  }
}
__global__ __launch_bounds__(1024) void var_scan_blocks(uint64_t nblocks,
                                                        uint32_t n_spans,
                                                        uint64_t *__restrict__ bsum,
                                                        DecArgs a,
                                                        spk_dresult_t *res) {
  __shared__ uint64_t sh[1024 / 64];
  scan_blocks_body(nblocks, n_spans, bsum, a, res, sh);
}

__device__ __forceinline__ void msg_write_body(const DecArgs &a, const uint8_t *__restrict__ wire,
                                               const uint64_t *__restrict__ offs,
                                               const uint8_t *__restrict__ ws,
                                               uint8_t *__restrict__ recs,
                                               const spk_dresult_t *res, uint64_t bx, uint32_t by,
                                               uint32_t gy, uint64_t *sh, BigSeg *big) {
  const MsgState *st = reinterpret_cast<const MsgState *>(ws + kWsScratch);
  const uint64_t *bsum = reinterpret_cast<const uint64_t *>(ws + kWsScratch +
                                                            sizeof(MsgState) * a.n_msgs);
  // heaps too small: write nothing (messages past rec_cap carry their own
  // CAPACITY errc and are skipped below; the others are still written)
  for (uint32_t k = 0; k < a.L.n_spans; ++k)
    if (res->heap_used[k] > a.heap_cap[k]) return;
  const uint64_t i = bx * kThreads + threadIdx.x;
  MsgState s{~0ull, 1, 1};
  uint64_t cnt[kVS] = {};
  uint64_t end = 0;
  if (i < dev_count(a.n_msgs, a.dn)) {
    s = st[i];
    if (s.pos != ~0ull) {
      end = a.ends ? a.ends[i] : offs[i + 1];
      rec_counts(a.L, wire, s.pos, s.w, cnt, end);
    }
  }
  uint64_t hoff[kVS] = {};
  for (uint32_t k = 0; k < a.L.n_spans; ++k) {
    uint64_t tot;
    hoff[k] = bsum[bx * kBs + k] + block_excl_scan(cnt[k], &tot, sh);
  }
  const bool live = s.pos != ~0ull && !s.errc;
  // large payloads go to the block's cooperative list (record order)
  uint32_t nbig = 0, skip = 0;
  if (live) {
    uint32_t sk = 0;
    for (uint32_t o = 0; o < a.L.n_ops; ++o)
      if (a.L.ops[o].kind == SPK_OP_SPAN || a.L.ops[o].kind == SPK_OP_OPTION) {  // OPTION values: never listed
        if (a.L.ops[o].kind == SPK_OP_SPAN && cnt[sk] * a.L.ops[o].size >= kBigBytes) ++nbig;
        ++sk;
      }
  }
  uint64_t nbig_tot;
  uint64_t slot = block_excl_scan(nbig, &nbig_tot, sh);
  if (nbig && slot + nbig <= kBigMax) {
    uint64_t pos = s.pos;
    uint32_t sk = 0;
    for (uint32_t o = 0; o < a.L.n_ops; ++o) {
      const spk_op op = a.L.ops[o];
      if (op.kind == SPK_OP_COPY) {
        pos += op.size;
        continue;
      }
      if (op.kind == SPK_OP_VARINT) {
        uint64_t v;
        pos += vi_read(WireBytes{wire}, pos, end, &v);
        continue;
      }
      pos += op_pw(op, s.w);
      const uint64_t nb = opt_nb(op, cnt[sk], pos, end);
      if (op.kind == SPK_OP_SPAN && nb >= kBigBytes) {
        big[slot++] = BigSeg{0, a.heaps[sk] + hoff[sk] * op.size, wire + pos, nb};
        skip |= 1u << sk;
      }
      pos += nb;
      ++sk;
    }
  }
  // copy split: gridDim.y blocks share the block's listed payloads; block 0
  // also writes the records and the short payloads
  if (live && by == 0)
    decode_record(a.L, wire, s.pos, s.w, recs + i * a.L.stride, a.heaps, hoff, end, skip);
  __syncthreads();
  if (nbig_tot > kBigMax) nbig_tot = kBigMax;
  if (nbig_tot == 0) return;  // block-uniform
  wave_copy_all(big, (uint32_t)nbig_tot, by, gy);
}
__global__ __launch_bounds__(kThreads) void var_msg_write(
    DecArgs a, const uint8_t *__restrict__ wire, const uint64_t *__restrict__ offs,
    const uint8_t *__restrict__ ws, uint8_t *__restrict__ recs, const spk_dresult_t *res) {
  __shared__ uint64_t sh[kThreads / 64];
  __shared__ BigSeg big[kBigMax];
  msg_write_body(a, wire, offs, ws, recs, res, blockIdx.x, blockIdx.y, gridDim.y, sh, big);
}

// MESSAGES decode of at most kThreads messages (a coro_rpc call's one
// request or response): the result reset, parse, block scan and write in one
// launch of one block instead of a memset and three kernels (each dependent
// launch costs a small call ~4-5 us)
__global__ __launch_bounds__(kThreads) void var_msg_decode_small(
    DecArgs a, const uint8_t *__restrict__ wire, const uint64_t *__restrict__ offs,
    uint8_t *__restrict__ ws, int32_t *__restrict__ errc_out, uint8_t *__restrict__ recs,
    spk_dresult_t *res) {
  __shared__ uint64_t sh[kThreads / 64];
  __shared__ BigSeg big[kBigMax];
  if (threadIdx.x == 0) *res = spk_dresult_t{};
  __syncthreads();
  msg_parse_body(a, wire, offs, ws, errc_out, res, 0, sh);
  __syncthreads();
  scan_blocks_body(1, a.L.n_spans, reinterpret_cast<uint64_t *>(ws + kWsScratch +
                                                                 sizeof(MsgState) * a.n_msgs),
                   a, res, sh);
  __syncthreads();
  msg_write_body(a, wire, offs, ws, recs, res, 0, 0, 1, sh, big);
}

// ===========================================================================
// DECODE, SPK_MODE_VECTOR — speculative chunk walks
// ===========================================================================
// Record k's start depends on every earlier length field. The decoder below
// (the tile pipeline, vec_tile_*) cuts the payload into 16 KiB tiles of
// kSpec-byte chunks, walks every chunk speculatively in parallel and joins
// the walks; see the pipeline overview before kTChunk. (Round 1's multi-pass
// chunk walker with P/E lists and verification rounds was removed in round 2
// after the tile pipeline replaced it.)
#ifndef SPK_VSCREEN  // varint layouts: K1's candidate screen from a terminator mask
#define SPK_VSCREEN 1  // (cv K1 1.255 -> 0.988 ms, cv 3.077 -> 2.807 ms per step, same-box A/B)
#endif
constexpr uint32_t kSpec = 256;        // payload bytes per speculation chunk
constexpr uint32_t kWinExtra = 512;    // extension bytes staged past a wave's chunks
constexpr uint32_t kPlaus = 4096;      // longest record a speculative walk accepts
constexpr int kRounds = 6;             // parallel re-verification rounds (default)
constexpr int kRoundsMax = 16;         // ... for varint layouts (WalkProg::rounds)
constexpr uint32_t kNone32 = 0xFFFFFFFFu;

struct VCtl {
  uint64_t p0;       // payload start (after header + count)
  uint64_t n;        // record count from the header
  uint64_t nchunks;  // chunks covering [p0, wire_len)
  uint64_t data_len;
  unsigned long long end_pos;  // absolute end of record n-1
  unsigned long long total;    // complete records on the true path
  uint32_t w;
  int32_t errc;      // header errc
  uint32_t lp;       // P-list capacity per chunk
  uint32_t n_unver;  // chunks left for the sequential fixup (diagnostic)
  uint32_t term_chunk;  // first chunk where the true path terminates (kNone32)
  uint32_t overflow;    // a P list overflowed (records < 1 B impossible; guard)
  uint32_t wl_n[kRoundsMax + 1];  // re-verification worklist length per round
  uint32_t pad_;
  uint64_t cap;                // chunk capacity: stride of the per-span chunk arrays
  // K1's speculation caps (vec_hdr_sample): the largest count per span a
  // speculative walk accepts, from the counts of the message's first records;
  // spec_c0 is the first-count screen under them
  uint64_t scap[kVS];
  uint64_t spec_c0;
  uint64_t scap_on;  // the caps tighten something (else K1 walks as without them)
};

// control words of the tile vector decoder (vec_tile_*)
struct FCtl {
  unsigned long long broken[4];  // tiles re-walked by select pass k (K2)
  unsigned long long unresolved; // tiles no pass could select (never expected)
  unsigned long long seq;        // tiles the sequential fixer re-resolved or passed through
  unsigned long long njobs;      // deferred long-span copies (BigQ)
  unsigned long long term_tile;  // first tile whose path ends inside it (atomicMin), ~0
  unsigned long long term_pos;   // where the true path ends (atomicMin), ~0
  unsigned long long end_pos;    // end of record n-1
  unsigned long long total;      // records on the path (tile scan)
  unsigned long long htot[kVS];  // heap elements used by records 0..n-1
  unsigned long long entry0;     // tile 0's entry (range mode: injected, or kNoPos = its own guess)
  unsigned long long nglob;      // range mode: the message's record count
  uint32_t range;                // the tiles are a byte range of the body (spk_decode_shard_*)
  uint32_t last;                 // range mode: the range holds the message's end
  unsigned long long stot[kVS];  // span-count sums on the path
  unsigned long long nlist[4];   // tiles listed for re-resolution by select pass k
  unsigned long long diag[8];    // SPK_TILE_DBG & 4096: K1 statistics (scripts/diag_tiles.py)
  unsigned long long chain_ticket;  // tiles the chain's blocks have taken
  unsigned long long chain_arrive;  // chain blocks arrived (the first one finds the first tile)
  unsigned long long chain_ready;   // the chain's first tile + 1 (0: not yet found)
  unsigned long long chain_done;    // chain blocks out (the last one sums the tile scan)
  unsigned long long term_from;     // SPK_CHAIN_TERM1: entry words [term_from, nt) hold kEntTerm
  unsigned long long copy_done;     // vec_big_copy blocks done (the last one writes the result)
  // records of the tiles the chain has finalised, plus those before its first
  // tile (a running lower bound of the records before the chain's next tile)
  unsigned long long chain_cnt;
  // the first tile left unresolved: harmless when it starts at or past the
  // end of record n-1 (bytes after the message, which need not parse)
  unsigned long long unres_tile;
};
constexpr size_t kWsFCtl = kWsCtl + 1280;
static_assert(sizeof(VCtl) <= kWsFCtl - kWsCtl, "VCtl overlaps FCtl");
static_assert(kWsFCtl + sizeof(FCtl) <= kWsScratch, "FCtl overlaps the scratch area");

// Compact walk program of a record: fixed bytes, then per span
// [count:w][count*esz bytes][fixed bytes]. Built once on the host from the
// descriptor so the walker's loop constants sit in SGPRs.
struct WalkProg {
  uint32_t ns;
  uint32_t skip[kVS + 1];
  uint32_t esz[kVS];
  uint32_t c0max;                  // largest first count of a plausible record
  uint64_t cmax[kVS];    // largest count whose byte size fits 64 bits
  uint32_t optm;                   // bit k: span k is an OPTION ([has_value:1][U?])
  uint32_t pf_all;                 // no first-count screening of candidate starts
  // nested layouts whose first SPAN (esz0) is followed, after s2skip fixed
  // bytes, by another count: that count must be <= c1max too (scr2)
  uint32_t scr2, esz0, s2skip, c1max;
  uint32_t pf_var;                 // screening past segment 0's varints (NS = -1 walks)
  uint32_t rounds;                 // parallel re-verification rounds before the fixup
  uint32_t nv;                     // varint members
  uint32_t hscr;                   // pf_all, nested: a has_value byte at skip[0] (screened 0 / 1)
  uint8_t vfirst[kVS + 2];  // segment k's varints: [vfirst[k], vfirst[k+1])
  uint32_t vafter[SPK_MAX_VARINTS];   // fixed bytes after varint j (same segment)
};

static WalkProg make_walkprog(const spk_layout *L) {
  WalkProg p = {};
  uint32_t k = 0;
  // segment k (before span k; the last one after every span) = skip[k] fixed
  // bytes, then per varint j of the segment: [LEB128][vafter[j] fixed bytes]
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    if (L->ops[i].kind == SPK_OP_COPY) {
      if (p.nv > p.vfirst[k])
        p.vafter[p.nv - 1] += L->ops[i].size;
      else
        p.skip[k] += L->ops[i].size;
    } else if (L->ops[i].kind == SPK_OP_VARINT) {
      ++p.nv;
    } else {
      p.esz[k] = L->ops[i].size;
      if (L->ops[i].kind == SPK_OP_OPTION) p.optm |= 1u << k;
      ++k;
      p.vfirst[k] = (uint8_t)p.nv;
    }
  }
  p.ns = k;
  for (uint32_t j = k + 1; j < kVS + 2; ++j) p.vfirst[j] = (uint8_t)p.nv;
  for (uint32_t j = 0; j < k; ++j) p.cmax[j] = ~0ull / (p.esz[j] ? p.esz[j] : 1);
  p.c0max = k ? (kPlaus > p.skip[0] ? (kPlaus - p.skip[0]) / (p.esz[0] ? p.esz[0] : 1) : 0) : 0;
  // an OPTION's has_value byte is not a w-byte count: no screening on it
  if (p.optm & 1u) p.c0max = 0xFFFFFFFFu;
  // a varint before the first count (or no count at all): the first count's
  // position is data-dependent, so every byte may start a record
  p.pf_all = (p.optm & 1u) || k == 0;
  // (no has_value screen of candidate starts here: on Cmp's version passes,
  // [has][int64][has][int16] records, it left 3x the broken tiles)
  p.pf_var = !p.pf_all && p.vfirst[1] > 0;
  // varint walks leave longer chains of unverified chunks: more parallel
  // rounds keep the one-lane fixup short
  p.rounds = p.nv ? kRoundsMax : kRounds;
  return p;
}


// little-endian w-byte count at wire[x] (x + w <= len checked by the caller)
__device__ __forceinline__ uint64_t wire_le(const uint8_t *wire, uint64_t x, uint32_t w) {
  switch (w) {
    case 1: return wire[x];
    case 2: return (uint64_t)wire[x] | ((uint64_t)wire[x + 1] << 8);
    case 4: return *reinterpret_cast<const u32_unaligned *>(wire + x);
    default: return *reinterpret_cast<const u64_unaligned *>(wire + x);
  }
}

// the varints of segment k at p (advanced past them and their fixed bytes);
// false when one is truncated or overlong
template <typename ByteFn>
__device__ __forceinline__ bool vi_seg(const WalkProg &P, uint32_t k, ByteFn byte,
                                       uint64_t len, uint64_t &p) {
  for (uint32_t j = P.vfirst[k]; j < P.vfirst[k + 1]; ++j) {
    uint64_t v;
    const uint32_t l = vi_read(byte, p, len, &v);
    if (!l || l == kViBad) return false;
    p += l + P.vafter[j];
  }
  return true;
}

// vi_seg through a reader's vread (the LDS window reads 8 bytes at once)
template <typename Rd>
__device__ __forceinline__ bool vi_seg_rd(const WalkProg &P, uint32_t k, const Rd &rd,
                                          uint64_t len, uint64_t &p) {
  for (uint32_t j = P.vfirst[k]; j < P.vfirst[k + 1]; ++j) {
    uint64_t v;
    const uint32_t l = rd.vread(p, len, &v);
    if (!l || l == kViBad) return false;
    p += l + P.vafter[j];
  }
  return true;
}

// the nested walker (NS = -2, defined with the tile decoder below)
// walker level of a nested tile instantiation: NS = -2 the interpreter (0),
// -3 the walk program (1), -4 the walk program with optional / compatible
// groups of one SPAN (2, WP_OSPAN; an instantiation of its own so that the
// -3 kernels carry none of its code: Monster's K1 / K4 lost ~5 % to it)
constexpr int nt_level(int ns) { return ns == -3 ? 1 : ns == -4 ? 2 : 0; }
template <int SIMPLE, typename Rd>
__device__ uint64_t nt_len(const Rd &rd, uint64_t len, uint64_t pos, uint64_t *cnt,
                           uint64_t reach, uint32_t maxel);
// a bounded nested walk gave up (its reach or element limit): length unknown
constexpr uint64_t kLenLimit = ~0ull - 8;
// K1's walks of nested records stop this far past their start: a walk from
// a wrong entry could otherwise iterate far into the wire one element at a
// time; a tile whose true path needs more is resolved again by the repair
// passes, whose walks are unbounded
template <int NS>
constexpr uint64_t kK1Reach = NS <= -2 ? (uint64_t)SPK_NT_REACH : 0;

// Wire length of the record at `pos` (0 = incomplete: the reference fails it
// with no_buffer_space). NS > 0: compile-time span count; 0: runtime count;
// -1: runtime count and the record has varints; -2: a nested layout (the
// interpreter walk, nt_len).
template <int NS>
__device__ __forceinline__ uint64_t wlen(const WalkProg &P, const uint8_t *wire, uint64_t len,
                                         uint64_t pos, uint32_t w) {
  uint64_t p = pos + P.skip[0];
  const uint32_t ns = NS > 0 ? (uint32_t)NS : P.ns;
  if (NS < 0 && !vi_seg(P, 0, WireBytes{wire}, len, p)) return 0;
#pragma unroll
  for (uint32_t k = 0; k < (NS > 0 ? (uint32_t)NS : kVS); ++k) {
    if (NS <= 0 && k >= ns) break;
    const bool opt = (P.optm >> k) & 1u;
    const uint32_t pw = opt ? 1u : w;
    if (p + pw > len) return 0;
    const uint64_t c = opt ? (uint64_t)(wire[p] != 0) : wire_le(wire, p, w);
    p += pw;
    if (c) {
      if (c > P.cmax[k]) return 0;
      const uint64_t nb = c * P.esz[k];
      if (nb > len - p) {
        if (!opt) return 0;  // OPTION: value unreadable, reader stays (opt_nb)
      } else {
        p += nb;
      }
    }
    p += P.skip[k + 1];
    if (NS < 0 && !vi_seg(P, k + 1, WireBytes{wire}, len, p)) return 0;
  }
  if (p > len) return 0;
  return p - pos;
}

// wlen() with the count fields read through `rd`
// CAPS: while `tight`, the per-span count limits are K1's speculation caps
// scap[] (VCtl, wave-uniform scalar loads) instead of P.cmax
template <int NS, typename Rd, bool CAPS = false>
__device__ __forceinline__ uint64_t wlen_rd(const WalkProg &P, const Rd &rd, uint64_t len,
                                            uint64_t pos, uint32_t w, uint64_t *cnt = nullptr,
                                            uint64_t reach = 0, const uint64_t *scap = nullptr,
                                            bool tight = false) {
  if constexpr (NS <= -2) return nt_len<nt_level(NS)>(rd, len, pos, cnt, reach, ~0u);
  uint64_t p = pos + P.skip[0];
  const uint32_t ns = NS > 0 ? (uint32_t)NS : P.ns;
  if (NS < 0 && !vi_seg_rd(P, 0, rd, len, p)) return 0;
#pragma unroll
  for (uint32_t k = 0; k < (NS > 0 ? (uint32_t)NS : kVS); ++k) {
    if (NS <= 0 && k >= ns) break;
    const bool opt = (P.optm >> k) & 1u;
    const uint32_t pw = opt ? 1u : w;
    if (p + pw > len) return 0;
    const uint64_t c = opt ? (uint64_t)(rd.byte(p) != 0) : rd(p);
    p += pw;
    if (c) {
      if (c > (CAPS && tight ? scap[k] : P.cmax[k])) return 0;
      const uint64_t nb = c * P.esz[k];
      if (nb > len - p) {
        if (!opt) return 0;  // OPTION: value unreadable, reader stays (opt_nb)
      } else {
        p += nb;
      }
    }
    if (cnt) cnt[k] = c;
    p += P.skip[k + 1];
    if (NS < 0 && !vi_seg_rd(P, k + 1, rd, len, p)) return 0;
  }
  if (p > len) return 0;
  return p - pos;
}

// count-field reader straight from the wire (global memory)
struct GReader {
  const uint8_t *wire;
  uint32_t w;
  __device__ __forceinline__ uint64_t operator()(uint64_t x) const { return wire_le(wire, x, w); }
  __device__ __forceinline__ uint32_t byte(uint64_t x) const { return wire[x]; }
  __device__ __forceinline__ uint32_t vread(uint64_t x, uint64_t len, uint64_t *v) const {
    return vi_read(WireBytes{wire}, x, len, v);
  }
};

__device__ void vec_hdr_body(const DecArgs &a, const uint8_t *__restrict__ wire,
                             uint8_t *__restrict__ ws, spk_dresult_t *res, uint32_t lp,
                             uint64_t cap) {
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  uint64_t pos = 0, dl = 0;
  uint32_t w = a.body_w;
  int32_t e = a.body_w || a.chain ? SPK_ERRC_OK : parse_hdr(a.fmt, wire, a.wire_len, &pos, &w, &dl);
  uint64_t n = 0;
  if (a.chain) {  // a version pass: its records start where the previous pass ended
    pos = a.chain[0];
    n = a.chain[1];
    w = (uint32_t)a.chain[2];
    dl = a.chain[3];
    if (n && pos >= a.wire_len) e = SPK_ERRC_NO_BUFFER_SPACE;
  } else if (a.body_w) {
    n = a.body_n;
  } else if (!e) {
    if (a.wire_len < pos + w)
      e = SPK_ERRC_NO_BUFFER_SPACE;
    else
      n = ld_le(wire + pos, w);
    pos += w;
  }
  if (!e && n && !a.L.n_var) {
    // every record needs at least fixed + n_spans*w bytes: a payload that
    // cannot hold n of them fails in the reference's record loop with
    // no_buffer_space (unpacker.hpp:1208-1226). Not with varints: an
    // overlong one before the payload runs out is invalid_buffer.
    const uint64_t min_rec = a.L.fixed_bytes + (uint64_t)a.L.n_cont * w;
    const uint64_t payload = a.wire_len - pos;
    if (n > payload / (min_rec ? min_rec : 1)) e = SPK_ERRC_NO_BUFFER_SPACE;
  }
  c->p0 = pos;
  c->n = e ? 0 : n;
  {
    FCtl *f0 = reinterpret_cast<FCtl *>(ws + kWsFCtl);
    f0->range = a.range;
    f0->last = 0;
    f0->nglob = c->n;
    f0->entry0 = pos;
    if (a.range) {  // the tiles start range_t0 tiles into the body
      c->p0 = pos + a.range_t0 * (64ull * SPK_TCHUNK);  // kTileBytes
      f0->entry0 = a.range_t0 == 0 ? pos : a.range_entry;
    }
  }
  c->w = w;
  c->errc = e;
  c->data_len = dl;
  c->end_pos = 0;
  c->total = 0;
  c->lp = lp;
  c->cap = cap;
  c->n_unver = 0;
  for (int r = 0; r <= kRoundsMax; ++r) c->wl_n[r] = 0;
  c->term_chunk = kNone32;
  c->overflow = 0;
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);  // tile decoder state
  for (int k = 0; k < 4; ++k) fc->broken[k] = fc->nlist[k] = 0;
  fc->unresolved = 0;
  fc->unres_tile = ~0ull;
  for (int k = 0; k < 8; ++k) fc->diag[k] = 0;
  fc->seq = 0;
  fc->chain_ticket = 0;
  fc->chain_arrive = 0;
  fc->chain_ready = 0;
  fc->chain_done = 0;
  fc->term_from = ~0ull;
  fc->chain_cnt = 0;
  fc->copy_done = 0;
  fc->njobs = 0;
  fc->term_tile = ~0ull;
  fc->term_pos = ~0ull;
  fc->end_pos = 0;
  fc->total = 0;
  for (int k = 0; k < kVS; ++k) fc->htot[k] = fc->stot[k] = 0;
  const uint64_t payload = (!e && a.wire_len > pos) ? a.wire_len - pos : 0;
  c->nchunks = (c->n == 0) ? 0 : (payload + kSpec - 1) / kSpec;
  spk_dresult_t r = {};
  r.errc = e;
  r.width = w;
  r.count = c->n;
  *res = r;
}
__global__ void vec_hdr_kernel(DecArgs a, const uint8_t *__restrict__ wire,
                               uint8_t *__restrict__ ws, spk_dresult_t *res, uint32_t lp,
                               uint64_t cap) {
  if (threadIdx.x == 0) vec_hdr_body(a, wire, ws, res, lp, cap);
}

struct VecBufs {
  uint16_t *P;      // [nchunks][lp]   positions in the chunk (rel. chunk start)
  uint32_t *Pn;     // [nchunks]
  uint32_t *E;      // [nchunks][kExt] positions past the chunk (rel. chunk start)
  uint32_t *En;     // [nchunks]
  uint32_t *flags;  // [nchunks]
  uint64_t *T;      // [nchunks] first true record start >= chunk start (abs), ~0 none
  uint32_t *cnt;    // [nchunks] complete true records starting in the chunk
  uint64_t *base;   // [nchunks] index of the chunk's first true record
  uint32_t *wl;     // [2][nchunks] re-verification worklists (alternating)
  uint64_t *exitp;  // [nchunks] true exit of the chunk (first start past it)
  uint64_t *used;   // [nchunks] entry the chunk was last verified with
  uint32_t *dirty;  // [2][nchunks] round a chunk is listed for (alternating)
  uint32_t *mj;     // [nchunks] P index where the true path meets the spec walk
                    //           | records walked before it << 16
  uint64_t *psum;   // [n_spans][nchunks] span-count sums over the spec walk's records
  uint64_t *hs;     // [n_spans][nchunks] span-count sums over the chunk's true records
  uint64_t *hb;     // [n_spans][nchunks] heap element offset of the chunk's first record
  uint64_t *scan;   // block sums for the device-wide scans
};


// LDS window layout: window-relative byte o is dword o >> 2, byte o. (Rows
// padded to 69 dwords, so that the candidate screen's same-offset reads of a
// 32-lane half fall on 32 banks, were measured slower in round 4: the
// conflicts cost less than the address arithmetic.)
__device__ __forceinline__ uint32_t win_dw(uint32_t o) { return o >> 2; }
__device__ __forceinline__ uint32_t win_b(uint32_t o) { return o; }
// 16-B slots of LDS a window of nv staged 16-B slots takes (+ the read-past slack)
__host__ __device__ constexpr uint32_t win_slots(uint32_t nv) { return nv + 1; }

// Count-field reader over a chunk's LDS window: bytes [cs, wend) of the wire
// are staged in LDS; reads past the window go to global memory. LO (LDS
// only): the caller guarantees every read lies inside the window, so the
// reader never touches global memory -- and the compiler then has no load of
// it to wait for: a global fallback merged into a read makes every use wait
// vmcnt(0), i.e. for all of the wave's outstanding STORES too (gfx950 counts
// stores in vmcnt), which serialised K4's record stores.
// WinReader::copy_to with non-temporal 16-B stores: K4's payload pieces are
// small and unaligned, so nt stores leave partial lines (round-6 A/B: C4 K4
// 0.475 -> 1.475 ms, cm K4 2.65 -> 2.88); off
#ifndef SPK_COPYTO_NT
#define SPK_COPYTO_NT 0
#endif
template <bool LO>
struct WinReaderT {
  static constexpr bool kLO = LO;
  const lds_u32 *d;
  const uint8_t *wire;
  uint64_t cs, wend;
  uint32_t w;
  __device__ __forceinline__ const lds_u8 *at(uint64_t x) const {
    return reinterpret_cast<const lds_u8 *>(d) + (uint32_t)(x - cs);
  }
  __device__ __forceinline__ uint64_t operator()(uint64_t x) const {
    if (LO || x + w <= wend) {
      if (w == 1) return *at(x);  // ds_read_u8
      if (w == 2) return *reinterpret_cast<const lds_u16_una *>(at(x));
      if (w == 4) return *reinterpret_cast<const lds_u32_una *>(at(x));
      return *reinterpret_cast<const lds_u64_una *>(at(x));
    }
    return wire_le(wire, x, w);
  }
  __device__ __forceinline__ uint32_t byte(uint64_t x) const {
    if (LO || x < wend) return reinterpret_cast<const lds_u8 *>(d)[win_b((uint32_t)(x - cs))];
    return wire[x];
  }
  // LEB128 at x (message end len), as vi_read: eight bytes from the window at
  // once -- the terminator is the first byte without its high bit, the value
  // gathers the 7-bit groups -- and the byte loop for longer / edge varints
  __device__ __forceinline__ uint32_t vread(uint64_t x, uint64_t len, uint64_t *v) const {
    uint32_t l = 0;
    if (LO || x + 12 <= wend) {
      l = vi_decode8(*reinterpret_cast<const lds_u64_una *>(at(x)), v);
    } else if (!LO && x >= wend && x + 8 <= len) {
      // past the window: the 8 bytes in one load, not one dependent byte load
      // each (speculative walks of varint records leave the window)
      l = vi_decode8(*reinterpret_cast<const u64_unaligned *>(wire + x), v);
    }
    if (l) return l;
    auto bf = [this](uint64_t q) { return byte(q); };
    return vi_read(bf, x, len, v);
  }
  // count_at with a 32-bit wire offset (nested tile walks: wires below
  // kNT32Wire bytes, so x + 12 cannot wrap)
  __device__ __forceinline__ uint64_t count_at32(uint32_t x, uint64_t wmask, bool opt) const {
    if (LO || x + 12u <= (uint32_t)wend) {
      const uint64_t b = *reinterpret_cast<const lds_u64_una *>(
          reinterpret_cast<const lds_u8 *>(d) + (x - (uint32_t)cs));
      return opt ? (uint64_t)((b & 0xFFu) != 0) : (b & wmask);
    }
    return opt ? (uint64_t)(byte(x) != 0) : (*this)(x);
  }
  // the count field at x: its w low bytes (wmask) or, for an OPTION's
  // has_value byte, whether it is non-zero; inside the window one path (8
  // bytes from three dwords), past it the wire
  __device__ __forceinline__ uint64_t count_at(uint64_t x, uint64_t wmask, bool opt) const {
    if (LO || x + 12 <= wend) {
      const uint64_t b = *reinterpret_cast<const lds_u64_una *>(at(x));
      return opt ? (uint64_t)((b & 0xFFu) != 0) : (b & wmask);
    }
    return opt ? (uint64_t)(byte(x) != 0) : (*this)(x);
  }
  // 4 / 16 bytes at x (x + n <= wend: inside the staged window)
  __device__ __forceinline__ uint32_t ld4(uint64_t x) const {
    return *reinterpret_cast<const lds_u32_una *>(at(x));
  }
  __device__ __forceinline__ v4u_t ld16(uint64_t x) const {
    return *reinterpret_cast<const lds_v4u_una *>(at(x));
  }
  // dst[0, n) = wire[x, x + n): from LDS when inside the window
  __device__ __forceinline__ void copy_to(uint8_t *dst, uint64_t x, uint64_t n) const {
    if (!LO && x + n + 4 > wend) {
      copy_bytes(dst, wire + x, n);
      return;
    }
    uint64_t i = 0;
    for (; i + 16 <= n; i += 16) {
      if (SPK_COPYTO_NT)
        __builtin_nontemporal_store(ld16(x + i), reinterpret_cast<v4u_una *>(dst + i));
      else
        *reinterpret_cast<v4u_una *>(dst + i) = ld16(x + i);
    }
    if (n - i >= 8) {
      const uint64_t lo = ld4(x + i), hi = ld4(x + i + 4);
      *reinterpret_cast<u64_unaligned *>(dst + i) = lo | (hi << 32);
      i += 8;
    }
    if (n - i >= 4) {
      *reinterpret_cast<u32_unaligned *>(dst + i) = ld4(x + i);
      i += 4;
    }
    for (; i < n; ++i) dst[i] = (uint8_t)byte(x + i);
  }
  // the same window with reads that never leave it (see LO)
  __device__ __forceinline__ WinReaderT<true> lds() const { return {d, wire, cs, wend, w}; }
};
using WinReader = WinReaderT<false>;

// Long spans are not copied by the lane that emits their record: the lane
// queues them in <= kBigPiece pieces and vec_big_copy moves every piece with
// a whole block (a multi-MiB string would otherwise be one lane's serial copy).
constexpr uint64_t kBigCopy = 4096;
constexpr uint64_t kBigPiece = 64 * 1024;
struct BigJob {
  uint64_t src, n;
  uint8_t *dst;
};
struct BigQ {
  BigJob *jobs;
  unsigned long long *n;
  uint64_t cap;
};
__host__ __device__ constexpr uint64_t big_jobs_cap(uint64_t wire_len) {
  return wire_len / kBigCopy + wire_len / kBigPiece + 1;
}

// Spans of kWaveCopy bytes and more (below kBigCopy) in a group of records
// that leaves the window are copied by the whole wave after the group's
// records are written (copied by their own lanes, 64 strings of 100-3000 B
// went at the pace of the longest, every instruction touching 64 lines:
// c3l K4 5.3 ms). A group inside the window (the LDS-only reader) holds no
// such span, and its path has none of this code (registers: C3 K4).
#ifndef SPK_SPAN_NT  // wave_span_copy: non-temporal stores of the span bytes
#define SPK_SPAN_NT 1  // (c3l K4 2.202 -> 2.142 ms, same-box A/B)
#endif
constexpr uint64_t kWaveCopy = 256;
struct Deferred {
  uint64_t src, n;
  uint8_t *dst;
};
template <typename Rd>
__device__ __forceinline__ void wave_span_copy(const Rd &R, uint64_t x, uint8_t *dst, uint64_t n,
                                               uint32_t lane) {
  const uint64_t nc = n >> 4;
  for (uint64_t c = lane; c < nc; c += 64) {
    const uint64_t s = x + 16 * c;
    v4u_t v;
    if (s + 16 <= R.wend)
      v = R.ld16(s);
    else
      v = *reinterpret_cast<const v4u_una *>(R.wire + s);
    if (SPK_SPAN_NT)
      __builtin_nontemporal_store(v, reinterpret_cast<v4u_una *>(dst + 16 * c));
    else
      *reinterpret_cast<v4u_una *>(dst + 16 * c) = v;
  }
  const uint64_t t = nc << 4;
  if (lane < n - t) dst[t + lane] = (uint8_t)R.byte(x + t + lane);
}
// the spans the lanes of mask m listed (list[lane], LDS), each by the whole wave
template <typename Rd>
__device__ __forceinline__ void wave_copy_deferred(const Rd &R, const Deferred *list, uint64_t m,
                                                   uint32_t lane) {
  while (m) {
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    const Deferred d = list[l];
    wave_span_copy(R, d.src, d.dst, d.n, lane);
  }
}

// emit_record reading the wire through an LDS window reader; with df set,
// the first span of kWaveCopy bytes or more goes to *df (returns whether one
// did)
template <typename Rd>
__device__ __forceinline__ bool emit_record_rd(const KLayout &L, const Rd &rd,
                                               uint64_t pos, uint32_t w, uint8_t *rec,
                                               uint8_t *const *heaps, const uint64_t *off,
                                               uint64_t end, const BigQ &bq, uint32_t dbg = 0,
                                               Deferred *df = nullptr) {
  bool deferred = false;
  uint32_t sk = 0;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      if (!(dbg & 512)) rd.copy_to(rec + op.rec_off, pos, op.size);
      pos += op.size;
    } else if (op.kind == SPK_OP_VARINT) {
      uint64_t v = 0;
      pos += rd.vread(pos, end, &v);
      if (!(dbg & 512)) vi_store(op, rec, v);
    } else {
      const uint64_t cnt = op.kind == SPK_OP_OPTION ? (uint64_t)(rd.byte(pos) != 0) : rd(pos);
      pos += op_pw(op, w);
      if (!(dbg & 512)) {
        *reinterpret_cast<uint32_t *>(rec + op.rec_off) = (uint32_t)cnt;
        *reinterpret_cast<uint64_t *>(rec + op.aux) = off[sk];
      }
      const uint64_t nb = opt_nb(op, cnt, pos, end);
      uint8_t *hp = heaps[sk] + off[sk] * op.size;
      if (cnt && !nb && op.kind == SPK_OP_OPTION) {
        for (uint32_t b = 0; b < op.size; ++b) hp[b] = 0;  // unreadable value
      } else if (nb >= kBigCopy) {
        const uint64_t np = (nb + kBigPiece - 1) / kBigPiece;
        const uint64_t j0 = atomicAdd(bq.n, (unsigned long long)np);
        for (uint64_t p = 0; p < np; ++p) {
          const uint64_t o = p * kBigPiece, m = nb - o < kBigPiece ? nb - o : kBigPiece;
          if (j0 + p < bq.cap)
            bq.jobs[j0 + p] = BigJob{pos + o, m, hp + o};
          else
            copy_bytes(hp + o, rd.wire + pos + o, m);  // (the cap is never reached)
        }
      } else if (!Rd::kLO && df && nb >= kWaveCopy && !deferred) {
        *df = Deferred{pos, nb, hp};
        deferred = true;
      } else if (!(dbg & 256)) {
        rd.copy_to(hp, pos, nb);
      }
      pos += nb;
      ++sk;
    }
  }
  return deferred;
}

// ===========================================================================
// Nested layouts on the tile decoder (NS = -2)
// ===========================================================================
// VECTOR messages of layouts with ARRAY / VARIANT / OPTGROUP / FVAR ops (no
// compatible members, at most kVS heaps) run the tile pipeline below with the
// op-list interpreter as the record walker: nt_read restates n_read
// (spk_nested.hip; unpacker.hpp:1127-1292 for containers, optional, variant)
// over the tile's LDS window, with the element stack in registers (static
// indices over SPK_MAX_DEPTH frames) and the layout staged in LDS. A record's
// heap use per heap takes the place of the flat walker's span counts, so the
// speculation, selection, tile scan and the emission's wave scans are the flat
// pipeline's; emission writes the record, its element records and its heap
// payloads (long ones queued for vec_big_copy).
struct NTLayout {
  spk_op ops[SPK_MAX_OPS];
  uint8_t heap[SPK_MAX_OPS];  // heap of a SPAN / OPTION / ARRAY op
  uint8_t end[SPK_MAX_OPS];   // ARRAY: its END; VARIANT / OPTGROUP: the END of its last group
  uint32_t n_ops, n_heaps, fv_cnt, fv_has64, fv_bits;
  uint32_t groups;            // a VARIANT / OPTGROUP op: errors inside may be dropped
  uint32_t wp_n;              // walk program length (0: walks run nt_read)
  uint32_t wp_tail;           // fixed bytes after the last instruction
  uint8_t *heaps[kVS];
  // walk program of a layout of COPY / SPAN / OPTION / ARRAY ops only: per
  // instruction x = op | heap << 3 | arg << 8 (WP_*; arg: element size, or
  // an ARRAY's exit), y = the fixed bytes (COPYs) before it; record lengths
  // and heap use without the interpreter's bookkeeping
  uint2 wp[SPK_MAX_OPS];
};
constexpr uint32_t WP_SPAN = 1, WP_OPT = 2, WP_ARR = 3, WP_END = 4;
// an optional / compatible group holding one SPAN (optional<string>,
// compatible<vector<int>>): [has:1] then, if present, [count:w][payload]; an
// error inside the group is dropped with the reader where it stopped
// (unpacker.hpp:1251-1277) -- h / arg are the SPAN's heap and element size
constexpr uint32_t WP_OSPAN = 5;
// an optional / compatible group whose members are COPY / SPAN / OPTION ops
// and one-SPAN groups (compatible<ResponseCode{int32, optional<string>}>):
// [has] then, if present, the members (arg: the instruction after the group);
// an error inside it is dropped with the reader where it stopped. Its COPYs
// are instructions of their own (WP_CPY, fixed bytes = the COPY) so that a
// short COPY leaves the reader where the reference's does.
constexpr uint32_t WP_GRP = 6, WP_CPY = 7;
// (late round 5 measured it inside the NS = -3 kernels: cmpg 8.04 -> 6.0 ms
// per step, but Monster's K1 / K4 ~5 % slower for the extra code; round 6:
// layouts whose walk program holds a WP_OSPAN run NS = -4 kernels of their own)
static_assert(sizeof(NTLayout) % 16 == 0, "NTLayout staged as 16-B words");
static_assert(SPK_MAX_DEPTH == 4, "the walker's element stack has 4 register frames");

__device__ __forceinline__ uint32_t nt_lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ NTLayout &nt_lds() {
  __shared__ NTLayout s;
  return s;
}
// each lane's heap slots in use during a walk (LDS, [heap][lane]: the
// kernels of this path run one wave per block); u32: wires below 4 GiB
__device__ __forceinline__ uint32_t *nt_used() {
  __shared__ uint32_t u[kVS * 64];
  return u + nt_lane();
}
// the layout into LDS by one wave (every lane of the calling wave takes part)
__device__ __forceinline__ void nt_stage_wave(const void *src, uint32_t lane) {
  const v4u_t *s = reinterpret_cast<const v4u_t *>(src);
  v4u_t *d = reinterpret_cast<v4u_t *>(&nt_lds());
  for (uint32_t k = lane; k < sizeof(NTLayout) / 16; k += 64) d[k] = s[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
template <int NS>
__device__ __forceinline__ void nt_prologue(const DecArgs &a, uint32_t lane) {
  if constexpr (NS <= -2) nt_stage_wave(a.nl, lane);
}

// the walker's element stack: the top frame lives in registers, the frames
// below it in LDS ([frame][field][lane]); pointers only when emitting
__device__ __forceinline__ uint32_t *nt_frames() {
  __shared__ uint32_t f[(SPK_MAX_DEPTH - 1) * 3 * 64];
  return f + nt_lane();
}
__device__ __forceinline__ uint8_t **nt_fptrs() {
  __shared__ uint8_t *f[(SPK_MAX_DEPTH - 1) * 2 * 64];
  return f + nt_lane();
}
// first op of group a of the VARIANT / OPTGROUP at i; the END closing the group at j
__device__ __forceinline__ uint32_t nt_alt_start(const NTLayout &N, uint32_t i, uint32_t a) {
  uint32_t j = i + 1;
  while (a) {
    const uint32_t k = N.ops[j].kind;
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT || k == SPK_OP_OPTGROUP) {
      j = N.end[j] + 1u;
      continue;
    }
    if (k == SPK_OP_END) --a;
    ++j;
  }
  return j;
}
__device__ __forceinline__ uint32_t nt_alt_end(const NTLayout &N, uint32_t j) {
  for (;;) {
    const uint32_t k = N.ops[j].kind;
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT || k == SPK_OP_OPTGROUP) {
      j = N.end[j] + 1u;
      continue;
    }
    if (k == SPK_OP_END) return j;
    ++j;
  }
}

constexpr int32_t kNTLimit = 0x7FFF0001;
// the nested tile decoder's wire limit: positions fit 32 bits with room for
// a 12-byte count read past any of them
constexpr uint64_t kNT32Wire = (1ull << 32) - 4096;  // a bounded walk needed bytes past its limit
// a bounded (speculative) walk also gives up on a container of more elements:
// from a false start, element counts read from payload bytes would have the
// walk iterate up to its byte limit one element at a time
constexpr uint64_t kNTSpecElems = 64;

// deserialize_fast_varint of the top-level record (unpacker.hpp:642-747), as n_fv_read
template <bool EMIT, typename Rd>
__device__ __forceinline__ int32_t nt_fv_read(const NTLayout &N, const Rd &rd, uint64_t &pos,
                                              uint64_t lim, uint8_t *rec) {
  if (lim - pos < N.fv_bits) return SPK_ERRC_NO_BUFFER_SPACE;
  uint64_t bits = 0;
  for (uint32_t b = 0; b < N.fv_bits; ++b) bits |= (uint64_t)rd.byte(pos + b) << (8 * b);
  pos += N.fv_bits;
  const uint32_t code = (uint32_t)(bits >> N.fv_cnt) & 3u;
  if (code == 3 && !N.fv_has64) return SPK_ERRC_INVALID_BUFFER;
  const uint32_t wb = 1u << code;
  uint32_t j = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_FVAR) continue;
    uint64_t v = 0;
    if ((bits >> j) & 1u) {
      const uint32_t rw = wb < op.size ? wb : op.size;
      if (lim - pos < rw) return SPK_ERRC_NO_BUFFER_SPACE;
      for (uint32_t b = 0; b < rw; ++b) v |= (uint64_t)rd.byte(pos + b) << (8 * b);
      pos += rw;
      if ((op.aux & SPK_FVAR_SIGNED) && rw < 8 && ((v >> (8 * rw - 1)) & 1u)) v |= ~0ull << (8 * rw);
    }
    if constexpr (EMIT) {
      if (op.size == 4)
        *reinterpret_cast<uint32_t *>(rec + op.rec_off) = (uint32_t)v;
      else
        *reinterpret_cast<uint64_t *>(rec + op.rec_off) = v;
    }
    ++j;
  }
  return SPK_ERRC_OK;
}

// One record at pos (n_read over a reader; reads stop at lim, a bounded walk
// (lim short of the wire's end) gives up there with kNTLimit). used[k]: next
// slot of heap k. EMIT writes the record at rec, its element records and its
// heap payloads (the caller checked the capacities). `quick`: a container
// whose count exceeds the bytes left fails at once (exact for the walk's
// outcome when no variant / optional group can drop the error; the errc of
// a failing record is taken with quick = false).
template <bool EMIT, typename Rd>
__device__ int32_t nt_read(const NTLayout &N, const Rd &rd, uint64_t &pos, uint64_t lim,
                           bool bounded, uint8_t *rec, const BigQ *bq, bool quick,
                           uint32_t maxel = ~0u) {
  uint32_t *const U = nt_used();  // U[64 * k]: heap k
  const uint32_t w = rd.w;
  // top frame: aop | pend << 8 | first << 16 | ret << 24, element index and
  // count (a count past the bytes left is clamped to bytes left + 1: elements
  // take at least one byte, so the walk fails at the same element; the tile
  // decoder runs on wires below 4 GiB), element records and the record to
  // resume (EMIT); the frames below it in LDS
  uint32_t c_op = 0, c_j = 0, c_cnt = 0;
  uint8_t *c_el = nullptr, *c_pr = nullptr;
  uint32_t *const F = nt_frames();
  uint8_t **const FP = EMIT ? nt_fptrs() : nullptr;
  auto push = [&](uint32_t d0, uint32_t o, uint32_t cn, uint8_t *el, uint8_t *pr) {
    if (d0) {
      F[64 * (3 * (d0 - 1))] = c_op;
      F[64 * (3 * (d0 - 1) + 1)] = c_j;
      F[64 * (3 * (d0 - 1) + 2)] = c_cnt;
      if constexpr (EMIT) {
        FP[64 * (2 * (d0 - 1))] = c_el;
        FP[64 * (2 * (d0 - 1) + 1)] = c_pr;
      }
    }
    c_op = o;
    c_j = 0;
    c_cnt = cn;
    c_el = el;
    c_pr = pr;
  };
  auto pop = [&](uint32_t d1) {  // d1: the depth after the pop
    if (d1) {
      c_op = F[64 * (3 * (d1 - 1))];
      c_j = F[64 * (3 * (d1 - 1) + 1)];
      c_cnt = F[64 * (3 * (d1 - 1) + 2)];
      if constexpr (EMIT) {
        c_el = FP[64 * (2 * (d1 - 1))];
        c_pr = FP[64 * (2 * (d1 - 1) + 1)];
      }
    }
  };
  uint32_t d = 0, i = 0, iend = N.n_ops;
  uint8_t *r = rec;
  int32_t ec = SPK_ERRC_OK;
  if (N.fv_cnt && (ec = nt_fv_read<EMIT>(N, rd, pos, lim, r)))
    return bounded && ec == SPK_ERRC_NO_BUFFER_SPACE ? kNTLimit : ec;
  for (;;) {
    if (ec) {
      // unwind to the innermost variant / optional / expected group, whose
      // errc is dropped (unpacker.hpp:476-490, 1251-1277); an ARRAY keeps its
      // failing element and gives back the slots past it (:1208-1226)
      // (the members from the failing one on, at every level unwound, are
      // value-initialised: zero_rest, spk_internal.hpp)
      bool dropped = false;
      for (;;) {
        if constexpr (EMIT) zero_rest(N, r, i, iend);
        if (!d) break;
        const uint32_t fo = c_op;
        const spk_op &ao = N.ops[fo & 0xFFu];
        if (ao.kind == SPK_OP_VARIANT || ao.kind == SPK_OP_OPTGROUP) {
          i = fo >> 24;
          iend = (fo >> 8) & 0xFFu;
          if constexpr (EMIT) r = c_pr;
          pop(--d);
          dropped = true;
          break;
        }
        const uint32_t hk = N.heap[fo & 0xFFu];
        atomicSub(U + 64 * hk, c_cnt - (c_j + 1));
        if constexpr (EMIT) *reinterpret_cast<uint32_t *>(c_pr + ao.rec_off) = c_j + 1;
        i = fo >> 24;  // the rest of the enclosing level
        iend = (fo >> 8) & 0xFFu;
        if constexpr (EMIT) r = c_pr;
        pop(--d);
      }
      if (!dropped) return ec;
      ec = SPK_ERRC_OK;
      continue;
    }
    if (i >= iend) {
      if (!d) break;
      const uint32_t fo = c_op;
      if (++c_j < c_cnt) {
        if constexpr (EMIT) r = c_el + (uint64_t)c_j * N.ops[fo & 0xFFu].size;
        i = (fo >> 16) & 0xFFu;
        continue;
      }
      i = fo >> 24;
      iend = (fo >> 8) & 0xFFu;
      if constexpr (EMIT) r = c_pr;
      pop(--d);
      continue;
    }
    const spk_op op = N.ops[i];
    const uint32_t kind = op.kind;
    if (kind == SPK_OP_FVAR) {  // read with the group
      ++i;
      continue;
    }
    if (kind == SPK_OP_COPY) {
      if (lim - pos < op.size) {
        if (bounded) return kNTLimit;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      if constexpr (EMIT) rd.copy_to(r + op.rec_off, pos, op.size);
      pos += op.size;
      ++i;
      continue;
    }
    if (kind == SPK_OP_VARINT) {  // deserialize_varint (varint.hpp:270-330)
      uint64_t v = 0;
      const uint32_t l = rd.vread(pos, lim, &v);
      if (!l) {  // truncated: the bytes read stay consumed
        if (bounded) return kNTLimit;
        pos = lim;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      if (l == kViBad) {
        pos += 10;
        ec = SPK_ERRC_INVALID_BUFFER;
        continue;
      }
      pos += l;
      if constexpr (EMIT) vi_store(op, r, v);
      ++i;
      continue;
    }
    if (kind == SPK_OP_VARIANT || kind == SPK_OP_OPTGROUP) {
      // variant: unpacker.hpp:1278-1292; optional / expected: :1251-1277
      if (pos >= lim) {
        if (bounded) return kNTLimit;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      const uint32_t b = rd.byte(pos++);
      int a;
      if (kind == SPK_OP_VARIANT) {
        if (b >= op.size) {
          ec = SPK_ERRC_INVALID_BUFFER;
          continue;
        }
        a = (int)b;
        if constexpr (EMIT) *reinterpret_cast<uint32_t *>(r + op.rec_off) = b;
      } else {
        // (a bounded walk -- speculative, or the chain's map -- gives up on a
        // has_value byte other than the 0 / 1 every writer stores: a false
        // start inside string bytes dies at once; the exact walk that
        // replaces a given-up one reads any non-zero byte as present)
        if (bounded && b > 1) return kNTLimit;
        a = b ? 0 : (op.size == 2 ? 1 : -1);
        if constexpr (EMIT) *reinterpret_cast<uint32_t *>(r + op.rec_off) = b ? 1u : 0u;
      }
      if (a < 0) {
        i = N.end[i] + 1u;
        continue;
      }
      if (d == SPK_MAX_DEPTH) {  // (spk_layout_check bounds the nesting)
        ec = SPK_ERRC_INVALID_BUFFER;
        continue;
      }
      const uint32_t a0 = nt_alt_start(N, i, (uint32_t)a);
      push(d++, i | (iend << 8) | (a0 << 16) | ((N.end[i] + 1u) << 24), 1u, r, r);
      iend = nt_alt_end(N, a0);
      i = a0;
      continue;
    }
    // SPAN / OPTION / ARRAY
    const uint32_t hk = N.heap[i];
    const uint32_t pw = kind == SPK_OP_OPTION ? 1u : w;
    if (lim - pos < pw) {
      if (bounded) return kNTLimit;
      ec = SPK_ERRC_NO_BUFFER_SPACE;
      continue;
    }
    if (bounded && kind == SPK_OP_OPTION && rd.byte(pos) > 1) return kNTLimit;  // (as above)
    uint64_t cnt = kind == SPK_OP_OPTION ? (uint64_t)(rd.byte(pos) != 0) : rd(pos);
    pos += pw;
    uint64_t off = 0;
    if constexpr (EMIT) off = U[64 * hk];
    if (EMIT && kind != SPK_OP_SPAN) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = (uint32_t)cnt;
      *reinterpret_cast<uint64_t *>(r + op.aux) = off;
    }
    if (kind == SPK_OP_ARRAY) {
      // an element takes at least one wire byte
      if (bounded && cnt > maxel) return kNTLimit;
      if (cnt > lim - pos) {
        if (bounded) return kNTLimit;
        if (quick && !N.groups) {
          ec = SPK_ERRC_NO_BUFFER_SPACE;
          continue;
        }
      }
      if (cnt > lim - pos) cnt = lim - pos + 1;  // (the element past the bytes fails)
      atomicAdd(U + 64 * hk, (uint32_t)cnt);
      if (!cnt) {
        i = N.end[i] + 1u;
        continue;
      }
      if (d == SPK_MAX_DEPTH) {
        ec = SPK_ERRC_INVALID_BUFFER;
        continue;
      }
      uint8_t *el = EMIT ? N.heaps[hk] + off * op.size : nullptr;
      push(d++, i | (iend << 8) | ((i + 1u) << 16) | ((N.end[i] + 1u) << 24), (uint32_t)cnt, el, r);
      r = el;
      iend = N.end[i];
      ++i;
      continue;
    }
    if (kind == SPK_OP_OPTION) {
      if (cnt) {
        const bool fits = lim - pos >= op.size;
        if (!fits && bounded) return kNTLimit;
        if constexpr (EMIT) {
          uint8_t *hp = N.heaps[hk] + off * op.size;
          if (fits)
            rd.copy_to(hp, pos, op.size);
          else
            for (uint32_t b = 0; b < op.size; ++b) hp[b] = 0;  // unreadable value
        }
        if (fits) pos += op.size;
      }
      atomicAdd(U + 64 * hk, (uint32_t)cnt);
      ++i;
      continue;
    }
    // SPAN (unpacker.hpp:1127-1156): the whole payload must be present
    if (cnt) {
      uint64_t nb;
      if (!span_nb(cnt, op.size, &nb) || lim - pos < nb) {
        if (bounded) return kNTLimit;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      if constexpr (EMIT) {
        uint8_t *hp = N.heaps[hk] + off * op.size;
        if (nb >= kBigCopy) {
          const uint64_t np = (nb + kBigPiece - 1) / kBigPiece;
          const uint64_t j0 = atomicAdd(bq->n, (unsigned long long)np);
          for (uint64_t q = 0; q < np; ++q) {
            const uint64_t o = q * kBigPiece, m = nb - o < kBigPiece ? nb - o : kBigPiece;
            if (j0 + q < bq->cap)
              bq->jobs[j0 + q] = BigJob{pos + o, m, hp + o};
            else
              copy_bytes(hp + o, rd.wire + pos + o, m);  // (the cap is never reached)
          }
        } else {
          rd.copy_to(hp, pos, nb);
        }
      }
      pos += nb;
    }
    if constexpr (EMIT) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = (uint32_t)cnt;
      *reinterpret_cast<uint64_t *>(r + op.aux) = off;
    }
    atomicAdd(U + 64 * hk, (uint32_t)cnt);
    ++i;
  }
  return SPK_ERRC_OK;
}

// A record's wire length through the walk program (0: the record fails, or a
// bounded walk would need bytes past lim); heap use into the lane's LDS
// counters. Exact for the walk's outcome: these layouts have no group that
// could drop an error.
template <bool OSPAN, typename Rd>
__device__ uint64_t nt_walk(const NTLayout &N, const Rd &rd, uint64_t pos, uint64_t lim64,
                            bool bounded, uint32_t maxel) {
  // a check that fails on a bounded walk's limit: unknown (the full wire may
  // have held the record)
  const uint64_t bad = bounded ? kLenLimit : 0;
  uint32_t *const U = nt_used();
  uint32_t *const F = nt_frames();
  const uint32_t w = rd.w;
  const uint64_t wmask = w >= 8 ? ~0ull : (1ull << (8 * w)) - 1;
  // positions as 32-bit wire offsets (the nested tile path takes wires below
  // kNT32Wire bytes): half the VALU work of 64-bit position arithmetic
  const uint32_t lim = (uint32_t)lim64;
  uint32_t p = (uint32_t)pos;
  uint32_t pc = 0, d = 0, body = 0, rem = 0;  // top loop frame: body start, elements left
  // (OSPAN kernels) the instruction after the open optional / compatible
  // group (WP_GRP), 0: none. An exact walk drops an error inside it with the
  // reader where the failing read left it (unpacker.hpp:1251-1277): it goes
  // on after the group; a bounded walk gives up.
  uint32_t gend = 0;
  while (pc < N.wp_n) {
    if (OSPAN && pc == gend) gend = 0;
    const uint2 ins = N.wp[pc];
    const uint32_t op = ins.x & 7u, h = (ins.x >> 3) & 31u, arg = ins.x >> 8;
    if (lim - p < ins.y) {
      if (OSPAN && gend && !bounded) {  // a COPY inside the group (WP_CPY: not folded)
        pc = gend;
        gend = 0;
        continue;
      }
      return bad;
    }
    p += ins.y;
    if (OSPAN && op == WP_CPY) {  // (its bytes were the fixed bytes above)
      ++pc;
      continue;
    }
    if (OSPAN && op == WP_GRP) {  // [has] then the members up to instruction arg
      if (lim - p < 1) return bad;  // (not inside a group: the record fails)
      const uint32_t b = rd.byte(p);
      if (bounded && b > 1) return bad;  // (nt_read: a has_value byte above 1)
      ++p;
      if (b) {
        gend = arg;
        ++pc;
      } else {
        pc = arg;
      }
      continue;
    }
    if (op == WP_END) {
      if (--rem) {
        pc = body;
      } else {
        ++pc;
        if (--d) {  // the enclosing loop's frame back from LDS
          body = F[64 * (3 * (d - 1))];
          rem = F[64 * (3 * (d - 1) + 1)];
        }
      }
      continue;
    }
    if (OSPAN && op == WP_OSPAN) {
      if (lim - p < 1) {  // (the has byte itself: the record fails, or the outer group)
        if (gend && !bounded) {
          pc = gend;
          gend = 0;
          continue;
        }
        return bad;
      }
      const uint32_t b = rd.byte(p);
      if (bounded && b > 1) return bad;  // (nt_read: a has_value byte above 1)
      ++p;
      if (b) {
        // a count or payload that is not there: a bounded walk gives up, an
        // exact one drops the group's error (reader after what it read)
        if (lim - p < w) {
          if (bounded) return bad;
        } else {
          const uint64_t c = rd.count_at32(p, wmask, false);
          p += w;
          if (c > lim - p || c * arg > lim - p) {
            if (bounded) return bad;
          } else {
            atomicAdd(U + 64 * h, (uint32_t)c);
            p += (uint32_t)(c * arg);
          }
        }
      }
      ++pc;
      continue;
    }
    const bool opt = op == WP_OPT;
    const uint32_t cw = opt ? 1u : w;
    if (lim - p < cw) {
      if (OSPAN && gend && !bounded) {
        pc = gend;
        gend = 0;
        continue;
      }
      return bad;
    }
    if (bounded && opt && rd.byte(p) > 1) return bad;  // (nt_read: a has_value byte above 1)
    const uint64_t c = rd.count_at32(p, wmask, opt);
    p += cw;
    if (OSPAN && gend && op == WP_SPAN && (c > lim - p || c * arg > lim - p)) {
      if (bounded) return bad;
      pc = gend;  // (a failed SPAN adds no heap use: nt_read counts it on success)
      gend = 0;
      continue;
    }
    atomicAdd(U + 64 * h, (uint32_t)c);
    if (op == WP_ARR) {
      if (c > lim - p || c > maxel) return bad;  // elements take >= 1 byte
      if (!c) {
        pc = arg;
      } else {
        if (d) {
          F[64 * (3 * (d - 1))] = body;
          F[64 * (3 * (d - 1) + 1)] = rem;
        }
        ++d;
        body = ++pc;
        rem = (uint32_t)c;
      }
      continue;
    }
    // SPAN: the payload must be there; OPTION: an unreadable value leaves the reader
    // (c <= lim - p < 2^32 and arg < 2^24: the product cannot overflow)
    if (!opt && (c > lim - p || c * arg > lim - p)) return bad;
    if (!opt || (c && lim - p >= arg)) p += (uint32_t)(c * arg);
    ++pc;
  }
  if (lim - p < N.wp_tail) return bad;
  return (uint64_t)(p + N.wp_tail - (uint32_t)pos);
}


// wlen_rd for NS = -2: the record's wire length (0: the path fails here) and
// its heap use per heap; reach > 0 bounds a speculative walk (past it: longer
// than a plausible record, kPlaus + 1)
template <int SIMPLE, typename Rd>
__device__ uint64_t nt_len(const Rd &rd, uint64_t len, uint64_t pos, uint64_t *cnt,
                           uint64_t reach, uint32_t maxel) {
  const NTLayout &N = nt_lds();
  uint32_t *const U = nt_used();
  const uint32_t nh = N.n_heaps;
#pragma unroll
  for (uint32_t q = 0; q < kVS; ++q)
    if (q < nh) U[64 * q] = 0;
  const uint64_t lim = reach && reach < len - pos ? pos + reach : len;
  uint64_t p = pos;
  if constexpr (SIMPLE != 0) {
    const uint64_t l = nt_walk<SIMPLE == 2>(N, rd, pos, lim, lim < len, maxel);
    if (l == kLenLimit) return kLenLimit;
    p += l;
  } else {
    const int32_t ec = nt_read<false>(N, rd, p, lim, lim < len, nullptr, nullptr, true, maxel);
    if (ec == kNTLimit) return kLenLimit;
    if (ec) return 0;
  }
  if (p == pos) return 0;  // (a record takes at least one byte: spk_layout_check)
  if (cnt) {
#pragma unroll
    for (uint32_t q = 0; q < kVS; ++q)
      if (q < nh) cnt[q] = U[64 * q];
  }
  return p - pos;
}
// the speculative walk's record length (a nested walk is bounded)
template <int NS, typename Rd>
__device__ __forceinline__ uint64_t wlen_spec(const WalkProg &P, const Rd &rd, uint64_t len,
                                              uint64_t pos, uint32_t w, uint64_t *cnt,
                                              const uint64_t *scap, bool tight) {
  if constexpr (NS <= -2) {
    const uint64_t l = nt_len<nt_level(NS)>(rd, len, pos, cnt, (uint64_t)kPlaus + 1, kNTSpecElems);
    return l == kLenLimit ? (uint64_t)kPlaus + 1 : l;  // too long for a plausible start
  }
  return wlen_rd<NS, Rd, (SPK_SCAP & 1) != 0>(P, rd, len, pos, w, cnt, 0, scap, tight);
}
// payload of a SPAN into its heap slots (long ones queued for vec_big_copy)
template <typename Rd>
__device__ __forceinline__ void nt_put_payload(const Rd &rd, uint8_t *hp, uint64_t pos,
                                               uint64_t nb, const BigQ &bq) {
  if (nb >= kBigCopy) {
    const uint64_t np = (nb + kBigPiece - 1) / kBigPiece;
    const uint64_t j0 = atomicAdd(bq.n, (unsigned long long)np);
    for (uint64_t q = 0; q < np; ++q) {
      const uint64_t o = q * kBigPiece, m = nb - o < kBigPiece ? nb - o : kBigPiece;
      if (j0 + q < bq.cap)
        bq.jobs[j0 + q] = BigJob{pos + o, m, hp + o};
      else
        copy_bytes(hp + o, rd.wire + pos + o, m);  // (the cap is never reached)
    }
  } else {
    rd.copy_to(hp, pos, nb);
  }
}
// Emission of a record the walk program accepted (COPY / SPAN / OPTION /
// ARRAY layouts): the interpreter without error paths (the walk checked
// every read), frames below the top one in LDS
template <bool OSPAN, typename Rd>
__device__ uint64_t nt_emit_simple(const NTLayout &N, const Rd &rd, uint64_t pos,
                                   uint64_t len, uint8_t *rec, const BigQ &bq) {
  uint32_t *const U = nt_used();
  uint32_t *const F = nt_frames();
  uint8_t **const FP = nt_fptrs();
  const uint32_t w = rd.w;
  uint32_t d = 0, i = 0, iend = N.n_ops, aop = 0, j = 0, cnt = 0;
  uint8_t *r = rec, *el = nullptr, *pr = nullptr;
  for (;;) {
    if (i >= iend) {
      if (!d) break;
      if (++j < cnt) {
        r = el + (uint64_t)j * N.ops[aop].size;
        i = aop + 1;
        continue;
      }
      i = N.end[aop] + 1u;
      r = pr;
      if (--d) {
        aop = F[64 * (3 * (d - 1))];
        j = F[64 * (3 * (d - 1) + 1)];
        cnt = F[64 * (3 * (d - 1) + 2)];
        el = FP[64 * (2 * (d - 1))];
        pr = FP[64 * (2 * (d - 1) + 1)];
        iend = N.end[aop];
      } else {
        iend = N.n_ops;
      }
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_COPY) {
      rd.copy_to(r + op.rec_off, pos, op.size);
      pos += op.size;
      ++i;
      continue;
    }
    if (OSPAN && op.kind == SPK_OP_OPTGROUP) {
      // a one-SPAN group (WP_OSPAN: [has] [count][payload], its error dropped
      // with the SPAN empty) at op k; returns the op after it
      auto ospan = [&](uint32_t k) -> uint32_t {
        const spk_op go = N.ops[k];
        const uint32_t b = rd.byte(pos++);
        *reinterpret_cast<uint32_t *>(r + go.rec_off) = b ? 1u : 0u;
        if (b) {
          const spk_op sp = N.ops[k + 1];
          const uint32_t h = N.heap[k + 1];
          uint64_t c = 0, nb = 0;
          bool ok = len - pos >= w;
          if (ok) {
            c = rd(pos);
            pos += w;
            ok = span_nb(c, sp.size, &nb) && nb <= len - pos;
          }
          if (ok) {
            const uint32_t o = U[64 * h];
            U[64 * h] = o + (uint32_t)c;
            *reinterpret_cast<uint32_t *>(r + sp.rec_off) = (uint32_t)c;
            *reinterpret_cast<uint64_t *>(r + sp.aux) = o;
            if (c) nt_put_payload(rd, N.heaps[h] + (uint64_t)o * sp.size, pos, nb, bq);
            pos += nb;
          } else {  // the group's error dropped: its members value-initialised (zero_rest)
            *reinterpret_cast<uint32_t *>(r + sp.rec_off) = 0;
            *reinterpret_cast<uint64_t *>(r + sp.aux) = 0;
          }
        }
        return N.end[k] + 1u;
      };
      const uint32_t ge = N.end[i];
      if (ge == i + 2 && N.ops[i + 1].kind == SPK_OP_SPAN) {
        i = ospan(i);
        continue;
      }
      // WP_GRP: [has] then COPY / SPAN / OPTION / one-SPAN group members; an
      // error inside is dropped (nt_read: the members from the failing one on
      // value-initialised, the reader where the failing read left it)
      const uint32_t b = rd.byte(pos++);
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = b ? 1u : 0u;
      uint32_t k = i + 1;
      while (b && k < ge) {
        const spk_op m = N.ops[k];
        if (m.kind == SPK_OP_COPY) {
          if (len - pos < m.size) break;
          rd.copy_to(r + m.rec_off, pos, m.size);
          pos += m.size;
          ++k;
          continue;
        }
        if (m.kind == SPK_OP_OPTGROUP) {
          if (len - pos < 1) break;
          k = ospan(k);
          continue;
        }
        const bool mopt = m.kind == SPK_OP_OPTION;
        const uint32_t cw = mopt ? 1u : w;
        if (len - pos < cw) break;
        const uint64_t c = mopt ? (uint64_t)(rd.byte(pos) != 0) : rd(pos);
        pos += cw;
        const uint32_t hk = N.heap[k];
        uint8_t *hp = N.heaps[hk] + (uint64_t)U[64 * hk] * m.size;
        if (!mopt) {  // SPAN: the whole payload must be there
          uint64_t nb = 0;
          if (!span_nb(c, m.size, &nb) || nb > len - pos) break;
          const uint32_t o = U[64 * hk];
          U[64 * hk] = o + (uint32_t)c;
          *reinterpret_cast<uint32_t *>(r + m.rec_off) = (uint32_t)c;
          *reinterpret_cast<uint64_t *>(r + m.aux) = o;
          if (c) nt_put_payload(rd, hp, pos, nb, bq);
          pos += nb;
        } else {  // OPTION: an unreadable value leaves the reader and reads as zeros
          const uint32_t o = U[64 * hk];
          U[64 * hk] = o + (uint32_t)c;
          *reinterpret_cast<uint32_t *>(r + m.rec_off) = (uint32_t)c;
          *reinterpret_cast<uint64_t *>(r + m.aux) = o;
          if (c) {
            if (len - pos >= m.size) {
              rd.copy_to(hp, pos, m.size);
              pos += m.size;
            } else {
              for (uint32_t x = 0; x < m.size; ++x) hp[x] = 0;
            }
          }
        }
        ++k;
      }
      if (b && k < ge) zero_rest(N, r, k, ge);  // (the dropped error's members)
      i = ge + 1u;
      continue;
    }
    const uint32_t hk = N.heap[i];
    const bool opt = op.kind == SPK_OP_OPTION;
    const uint64_t c = opt ? (uint64_t)(rd.byte(pos) != 0) : rd(pos);
    pos += opt ? 1u : w;
    const uint32_t o = U[64 * hk];
    U[64 * hk] = o + (uint32_t)c;
    *reinterpret_cast<uint32_t *>(r + op.rec_off) = (uint32_t)c;
    *reinterpret_cast<uint64_t *>(r + op.aux) = o;
    uint8_t *hp = N.heaps[hk] + (uint64_t)o * op.size;
    if (op.kind == SPK_OP_SPAN) {
      if (c) nt_put_payload(rd, hp, pos, c * op.size, bq);
      pos += c * op.size;
      ++i;
    } else if (opt) {
      if (c) {
        if (len - pos >= op.size) {
          rd.copy_to(hp, pos, op.size);
          pos += op.size;
        } else {
          for (uint32_t b = 0; b < op.size; ++b) hp[b] = 0;  // unreadable value
        }
      }
      ++i;
    } else if (!c) {  // ARRAY
      i = N.end[i] + 1u;
    } else {
      if (d) {
        F[64 * (3 * (d - 1))] = aop;
        F[64 * (3 * (d - 1) + 1)] = j;
        F[64 * (3 * (d - 1) + 2)] = cnt;
        FP[64 * (2 * (d - 1))] = el;
        FP[64 * (2 * (d - 1) + 1)] = pr;
      }
      ++d;
      aop = i;
      j = 0;
      cnt = (uint32_t)c;
      el = hp;
      pr = r;
      r = hp;
      iend = N.end[i];
      ++i;
    }
  }
  return pos;
}

// emission with the lane's heap slots already in its LDS counters; the
// record's end
template <int SIMPLE, typename Rd>
__device__ __forceinline__ uint64_t nt_emit_here(const Rd &rd, uint64_t pos, uint64_t len,
                                                 uint8_t *rec, const BigQ &bq) {
  const NTLayout &N = nt_lds();
  if constexpr (SIMPLE != 0) {
    return nt_emit_simple<SIMPLE == 2>(N, rd, pos, len, rec, bq);
  } else {
    nt_read<true>(N, rd, pos, len, false, rec, &bq, false);
    return pos;
  }
}

// emission of the record at pos with heap bases off[]
template <int SIMPLE>
__device__ __forceinline__ void nt_emit(const WinReader &rd, uint64_t pos, uint64_t len,
                                        uint8_t *rec, const uint64_t *off, const BigQ &bq) {
  const NTLayout &N = nt_lds();
  uint32_t *const U = nt_used();
#pragma unroll
  for (uint32_t q = 0; q < kVS; ++q)
    if (q < N.n_heaps) U[64 * q] = (uint32_t)off[q];
  if constexpr (SIMPLE != 0)
    nt_emit_simple<SIMPLE == 2>(N, rd, pos, len, rec, bq);
  else
    nt_read<true>(N, rd, pos, len, false, rec, &bq, false);
}

constexpr uint64_t kTermPos = ~0ull;  // "the true path ended before this chunk"

__device__ __forceinline__ uint64_t wave_excl_scan_u64(uint64_t v, uint32_t lane, uint64_t *tot) {
  (void)lane;
  const uint64_t x = wave_incl_scan(v);
  *tot = wave_lane63(x);
  return x - v;
}

// One wave per group of G chunks: the group's true record starts go to an
// LDS table (P entries from the meeting index on, plus any records walked
// before it), then lanes take 64 consecutive records at a time, scan their
// span counts across the wave for heap offsets (group base from the chunk
// scan) and write the device records and heap bytes.
// ===========================================================================
// DECODE, SPK_MODE_VECTOR — tiles: speculate, select, scan, emit
// ===========================================================================
// A tile is 64 consecutive kSpec-byte chunks of the payload (16 KiB), owned
// by one wave (one lane per chunk) and staged in LDS.
//  K1 vec_tile_spec: every lane walks its chunk from its first plausible
//     record start (candidate screen above) -> spec start, exit (first record
//     start at or past the chunk end), record count, span-count sums. Chunk
//     0's start is cross-checked against chunk 1's independent speculation.
//     Resolution in registers: chunk c's entry is chunk c-1's exit, lanes
//     whose state came from another entry re-walk, in parallel rounds, until
//     the chain is consistent given the tile's assumed entry X. The tile then
//     publishes its FUNCTION: exit Y (the same for every entry below) and up
//     to kAlt entries (X and other start candidates of chunk 0 whose walk
//     reaches chunk 0's exit) with the tile's records / span sums for each.
//  K2 vec_tile_pick / vec_tile_repair: tile t's true entry is tile t-1's exit (tile 0: the
//     payload start). It selects the matching entry; a tile whose entry is
//     none of them re-walks from it (rare; twice, a cascade is rarer still,
//     then one wave fixes any rest in order).
//  K3 a prefix sum over the tiles' selected (records, span sums), zero past
//     the tile where the path ends -> every tile's first record index and heap
//     offsets.
//  K4 vec_tile_emit: each tile re-stages its bytes, takes its chunk states
//     for the selected entry, lists its record starts in LDS and writes 64
//     consecutive records at a time (span counts scanned across the wave for
//     heap offsets).
// No kernel waits on another workgroup.
constexpr uint32_t kTChunk = SPK_TCHUNK;                    // payload bytes per lane (chunk)
constexpr uint32_t kTileBytes = 64 * kTChunk;                // payload bytes per tile
static_assert(kTileBytes == SPK_DECODE_TILE_BYTES, "shard ranges are counted in these tiles");
constexpr uint32_t kTileVec = (kTileBytes + kWinExtra) / 16;  // staged 16-B slots
constexpr uint32_t kDecWaves = SPK_TWAVES;                   // tiles (waves) per block
constexpr uint32_t kTab = 2048;                              // record starts per emission pass
constexpr uint64_t kNoPos = ~0ull - 1;  // "no plausible start / unknown entry"
#ifndef SPK_SPEC_PAST
#define SPK_SPEC_PAST 2
#endif
constexpr uint32_t kSpecPast = SPK_SPEC_PAST;  // records a speculative walk checks past its chunk
// ... for a 2-byte count width: a random 16-bit count passes the first-count
// screen (c0max ~ 4K) one time in 16, so a false start inside binary string
// bytes survives kSpecPast more records one time in ~250 and half the tiles
// of a 100-3000 B binary-string message took a false entry; with 5 it is one
// in ~10^6 (a 4-byte count passes one time in ~10^6 already)
#ifndef SPK_SPEC_PAST_W2
#define SPK_SPEC_PAST_W2 5
#endif
constexpr uint32_t kAlt = 4;            // entries a tile function carries
constexpr uint32_t kAltWords = 2 + kVS;   // entry, cnt, sums
constexpr uint32_t kFnWords = 48;       // y, nalt, kAlt x kAltWords (+ pad)
constexpr int32_t kSelTerm = -2;        // the tile starts past the path's end
constexpr int32_t kSelBroken = -1;

struct TileBufs {
  uint64_t *fn;       // [ntiles][kFnWords]
  uint64_t *cused;    // [nchunks] entry each chunk state was computed from
  uint64_t *cex;      // [nchunks] its exit (first start past the chunk / kTermPos)
  uint32_t *ccnt;     // [nchunks] records starting in the chunk
  uint64_t *csum;     // [nsp][nchunks] span-count sums
  int32_t *sel;       // [ntiles] selected entry (kSelTerm / kSelBroken)
  uint64_t *contrib;  // [1 + nsp][ntiles] selected (records, sums) -> exclusive prefix
  uint64_t *scan;     // block sums of the tile scan
  uint32_t *blist;    // [ntiles] tiles a select pass found broken
  uint64_t *ent;      // [ntiles] the tile chain's tagged entry words
  uint64_t ntiles, nchunks;
};

// A true walk of chunk [.., ce) from `entry` (no plausibility limit): exit =
// first record start >= ce, or kTermPos when the path ends (incomplete record
// or wire end: *term_at = where); kTermPos / kNoPos entries propagate.
template <int NS, typename Rd>
__device__ __forceinline__ void walk_true(const WalkProg &P, const Rd &rd, uint64_t len,
                                          uint32_t w, uint64_t entry, uint64_t ce,
                                          uint64_t &ex, uint32_t &cnt, uint64_t *sums,
                                          uint64_t &term_at, uint64_t reach = 0) {
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  cnt = 0;
  QFOR(q) sums[q] = 0;
  term_at = kTermPos;
  if (entry == kTermPos || entry == kNoPos) {
    ex = entry;
    return;
  }
  uint64_t x = entry;
  while (x < ce) {
    uint64_t rc[NS > 0 ? NS : kVS];
    const uint64_t L = x < len ? wlen_rd<NS>(P, rd, len, x, w, rc, reach) : 0;
    if (L == kLenLimit) {  // (a bounded nested walk: the exit is unknown)
      ex = kNoPos;
      return;
    }
    if (!L) {
      term_at = x;
      ex = kTermPos;
      return;
    }
    ++cnt;
    QFOR(q) sums[q] += rc[q];
    x += L;
  }
  ex = x;
}

// The first records of a lane's speculative walk (chunk-relative starts and
// the span-count sums before each), so that a walk from another entry stops
// where it meets that path: paths through the same records coincide from
// there on, and the speculative walk's totals give the rest.
constexpr uint32_t kMergePts = 4;
template <int NS>
struct SpecPath {
  static constexpr int kS = NS > 0 ? NS : 2;
  uint32_t pos[kMergePts];
  uint32_t ps[kMergePts][kS];
  uint32_t np;     // valid entries (0: no merge information)
  uint32_t cnt;    // the speculative walk's records in the chunk
  uint64_t sums[kS];
  uint64_t ex, term_at;
};

template <int NS, typename Rd>
__device__ __forceinline__ void walk_merge(const WalkProg &P, const Rd &rd, uint64_t len,
                                           uint32_t w, uint64_t entry, uint64_t cs, uint64_t ce,
                                           const SpecPath<NS> &sp, uint64_t &ex, uint32_t &cnt,
                                           uint64_t *sums, uint64_t &term_at, uint64_t reach = 0) {
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  cnt = 0;
  QFOR(q) sums[q] = 0;
  term_at = kTermPos;
  if (entry == kTermPos || entry == kNoPos) {
    ex = entry;
    return;
  }
  uint64_t x = entry;
  while (x < ce) {
    uint32_t jm = kMergePts;  // joined the speculative path at its record jm
#pragma unroll
    for (uint32_t j = 0; j < kMergePts; ++j)
      if (jm == kMergePts && j < sp.np && x == cs + sp.pos[j]) jm = j;
    if (jm < kMergePts) {
      cnt += sp.cnt - jm;
      QFORS(q) {
        uint32_t pv = 0;
#pragma unroll
        for (uint32_t j = 0; j < kMergePts; ++j) pv = jm == j ? sp.ps[j][q] : pv;
        sums[q] += sp.sums[q] - pv;
      }
      ex = sp.ex;
      term_at = sp.term_at;
      return;
    }
    uint64_t rc[NS > 0 ? NS : kVS];
    const uint64_t L = x < len ? wlen_rd<NS>(P, rd, len, x, w, rc, reach) : 0;
    if (L == kLenLimit) {
      ex = kNoPos;
      return;
    }
    if (!L) {
      term_at = x;
      ex = kTermPos;
      return;
    }
    ++cnt;
    QFOR(q) sums[q] += rc[q];
    x += L;
  }
  ex = x;
}

// After a resolution round: the lanes following a lane that walked, up to the
// first whose chunk end lies past that walk's exit, hold no record start (a
// record spans their chunks): each takes that exit as its entry and its exit
// at once, as its own walk would, instead of one lane per round (c3l: the
// long strings of a tile cost ~60 rounds).
template <int NS>
__device__ __forceinline__ void pass_through_run(uint64_t walked, uint32_t lane, uint64_t ce,
                                                 uint32_t nsp, uint64_t &used, uint64_t &ex,
                                                 uint32_t &cnt, uint64_t *sums,
                                                 uint64_t &term_at) {
  const uint64_t below = walked & ((1ull << lane) - 1ull);
  const uint32_t k = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
  const uint64_t X = __shfl(ex, (int)k);  // the last walker below this lane
  if (below && !((walked >> lane) & 1ull) && X >= ce) {
    used = X;
    ex = X;
    cnt = 0;
    QFOR(q) sums[q] = 0;
    term_at = kTermPos;
  }
}

// In-wave resolution: until every lane's state was computed from its true
// entry (lane 0: entry0; lane c: lane c-1's exit), lanes that disagree re-walk.
template <int NS, typename Rd>
__device__ __forceinline__ void resolve_tile(const WalkProg &P, const Rd &rd, uint64_t len,
                                             uint32_t w, uint64_t ce, uint32_t lane,
                                             uint64_t entry0, uint64_t &used, uint64_t &ex,
                                             uint32_t &cnt, uint64_t *sums, uint64_t &term_at) {
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  for (int round = 0; round < 66; ++round) {
    const uint64_t prev = __shfl_up(ex, 1);
    const uint64_t entry = lane == 0 ? entry0 : prev;
    // (an unknown exit from a known entry: K1's bounded nested walk gave up)
    const bool need = entry != used || (ex == kNoPos && entry != kNoPos);
    const uint64_t m = __ballot(need);
    if (!m) return;
    // a lane with a start of its own waits while its predecessor re-walks
    // (that exit is about to change): walks from an exit that is itself wrong
    // would only pass the error on, one lane per round (the first mismatch
    // always proceeds). A lane without any start walks anyway: records
    // resynchronise, so its walk from a wrong entry is often already right.
    const bool go = need && (used == kNoPos || !(lane > 0 && ((m >> (lane - 1)) & 1)));
    if (go) {
      walk_true<NS>(P, rd, len, w, entry, ce, ex, cnt, sums, term_at);
      used = entry;
    }
    pass_through_run<NS>(__ballot(go), lane, ce, nsp, used, ex, cnt, sums, term_at);
  }
}
// ... with each lane's speculative path for early merges
template <int NS, typename Rd>
__device__ __forceinline__ void resolve_tile_sp(const WalkProg &P, const Rd &rd, uint64_t len,
                                                uint32_t w, uint64_t cs, uint64_t ce,
                                                uint32_t lane, uint64_t entry0,
                                                const SpecPath<NS> &sp, uint64_t &used,
                                                uint64_t &ex, uint32_t &cnt, uint64_t *sums,
                                                uint64_t &term_at, uint32_t *stat = nullptr,
                                                uint64_t reach = 0) {
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  for (int round = 0; round < 66; ++round) {
    const uint64_t prev = __shfl_up(ex, 1);
    const uint64_t entry = lane == 0 ? entry0 : prev;
    const bool need = entry != used;
    const uint64_t m = __ballot(need);
    if (!m) return;
    if (stat) ++stat[0];
    const bool go = need && (used == kNoPos || !(lane > 0 && ((m >> (lane - 1)) & 1)));
    if (go) {  // as resolve_tile
      if (stat) ++stat[1];
      walk_merge<NS>(P, rd, len, w, entry, cs, ce, sp, ex, cnt, sums, term_at, reach);
      used = entry;
    }
    pass_through_run<NS>(__ballot(go), lane, ce, nsp, used, ex, cnt, sums, term_at);
  }
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  return wave_lane63(wave_incl_scan(v));
}

// The candidate screen of the speculative walk for one start position.
template <int NS, typename Rd>
__device__ __forceinline__ bool screen_one(const WalkProg &P, const Rd &rd, uint64_t len,
                                           uint32_t w, uint64_t q) {
  if (P.pf_all) return true;
  uint64_t b = q + P.skip[0];
  if (NS < 0 && P.pf_var) {
    for (uint32_t j = 0; j < P.vfirst[1]; ++j) {
      uint64_t v;
      const uint32_t l = rd.vread(b, len, &v);
      if (!l || l == kViBad) return false;
      b += l + P.vafter[j];
    }
  }
  return (b + w <= len ? rd(b) : ~0ull) <= P.c0max;
}


// staged 16-B slot v of a window
__device__ __forceinline__ void win_put(v4u_t *win, uint32_t v, const v4u_t &x) { win[v] = x; }

// Stage tile t's bytes (+ extension) in this wave's LDS window; reader over it.
struct TileView {
  WinReader rd;
  uint64_t ts, wend;
};
// the reader over a window staged at ts (by this wave or, behind a barrier,
// another of the block)
template <uint32_t NV>
__device__ __forceinline__ TileView win_view(const v4u_t *win, const uint8_t *wire, uint64_t len,
                                             uint64_t ts, uint32_t w) {
  const uint64_t wend = ts + NV * 16 < len ? ts + NV * 16 : len;
  TileView tv;
  tv.rd.d = (const lds_u32 *)win;
  tv.rd.wire = wire;
  tv.rd.cs = ts;
  tv.rd.wend = wend;
  tv.rd.w = w;
  tv.ts = ts;
  tv.wend = wend;
  return tv;
}
template <uint32_t NV, bool NT = false>
__device__ __forceinline__ TileView stage_win(v4u_t *win, const uint8_t *wire, uint64_t len,
                                              uint64_t ts, uint32_t w, uint32_t lane) {
  if (ts + NV * 16 <= len) {
    // the whole window exists: every lane issues all its 16-B loads before
    // the first LDS write, so the wave waits for one load latency, not one
    // per 1 KiB (an un-unrolled loop serialises them)
    constexpr uint32_t kPer = (NV + 63) / 64;
    v4u_t val[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t v = lane + 64 * k;
      if (NV % 64 == 0 || v < NV) {
        const v4u_una *q = reinterpret_cast<const v4u_una *>(wire + ts + 16ull * v);
        val[k] = NT ? __builtin_nontemporal_load(q) : *q;
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t v = lane + 64 * k;
      if (NV % 64 == 0 || v < NV) win_put(win, v, val[k]);
    }
  } else
  for (uint32_t v = lane; v < NV; v += 64) {
    const uint64_t g = ts + 16ull * v;
    v4u_t val = {0u, 0u, 0u, 0u};
    if (g + 16 <= len) {
      val = *reinterpret_cast<const v4u_una *>(wire + g);
    } else if (g < len) {
      uint32_t tt[4] = {0u, 0u, 0u, 0u};
      for (uint64_t q = g; q < len; ++q) tt[(q - g) >> 2] |= (uint32_t)wire[q] << (8 * ((q - g) & 3));
      val = v4u_t{tt[0], tt[1], tt[2], tt[3]};
    }
    win_put(win, v, val);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return win_view<NV>(win, wire, len, ts, w);
}
__device__ __forceinline__ TileView stage_tile(v4u_t *win, const uint8_t *wire, uint64_t len,
                                               uint64_t ts, uint32_t w, uint32_t lane) {
  return stage_win<kTileVec>(win, wire, len, ts, w, lane);
}

__device__ __forceinline__ bool vec_live(const VCtl *c) { return !c->errc && c->n; }

// One lane's chunk state after the speculative walk and the in-wave
// resolution (K1 sections 1-2; also the fused decoder's first phase).
// records a speculative walk checks past its chunk (0: none, the walk stops at
// the first record start past it)
template <int NS>
constexpr uint32_t kNPast = NS <= -2 ? (uint32_t)SPK_NT_PAST : kSpecPast;

template <int NS>
struct TileLane {
  uint64_t used, ex, term_at;
  uint32_t cnt;
  uint64_t sums[NS > 0 ? NS : kVS];
  SpecPath<NS> sp;
};

// Speculative walk of this lane's chunk [cs, ce) of the tile staged at ts,
// the chunk-0 cross-check and the resolution under the tile's assumed entry;
// returns that entry X (kNoPos: none plausible). exact0: the tile starts at
// the payload start (its entry is p0, no search).
template <int NS>
__device__ __forceinline__ uint64_t tile_spec_resolve(const WalkProg &P, const WinReader &rd,
                                                      uint64_t len, uint32_t w, uint64_t ts,
                                                      uint64_t wend, uint64_t cs, uint64_t ce,
                                                      uint32_t lane, bool exact0, uint64_t p0,
                                                      uint32_t dbg, TileLane<NS> &st,
                                                      uint32_t *stat = nullptr,
                                                      const VCtl *sc = nullptr) {
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  // the lane state in locals, copied to st at the end: worked on through
  // references into st, the compiler kept it in scratch memory (round 3's C4
  // K1 0.43 -> 0.59 ms; locals: 0.36 ms, same-box A/B in DESIGN §6.1)
  uint64_t used, ex, term_at;
  uint32_t cnt;
  uint64_t sums[NS > 0 ? NS : kVS];
  SpecPath<NS> sp;
  used = kNoPos;
  ex = kNoPos;
  term_at = kTermPos;
  cnt = 0;
  QFOR(q) sums[q] = 0;
  const bool exact = exact0 && lane == 0;  // the payload start: no search
  const uint32_t npast = kNPast<NS> && w <= 2 ? (uint32_t)SPK_SPEC_PAST_W2 : kNPast<NS>;
  sp.np = 0;
  // speculation caps (flat layouts, sc: vec_hdr_sample's): a candidate start
  // and every record of its walk must keep each count within the caps, so
  // walks from false starts (a 1-byte count accepts any byte under P.cmax)
  // die within a record or two; a chunk with no start under them is searched
  // again with the layout's own limits
  const uint64_t *scap = nullptr;
  uint64_t c0t = P.c0max;
  bool tight = false;
  if constexpr (NS > -2) {
    if (sc && sc->scap_on && !(dbg & 65536)) {
      // (caps that tighten nothing would only add the search without them
      // for chunks holding no record start: long-string messages)
      tight = true;
      if ((SPK_SCAP & 2) || (NS == -1 && (SPK_SCAP & 4))) c0t = sc->spec_c0;
      if (SPK_SCAP & 1) scap = sc->scap;
    }
  }
  // ---- 1. speculative walk of this lane's chunk ----
  if (cs < len && !(dbg & 8)) {
    uint64_t tt = 0, x = cs, past = 0, sx = exact ? cs : kNoPos;
    bool searching = !exact, done = false;
    uint32_t k = 0;
    uint64_t ksum[NS > 0 ? NS : kVS];
    QFOR(q) ksum[q] = 0;
    const uint32_t s0 = P.skip[0];
    for (;;) {
    while (!done) {
      if (searching) {
        const uint64_t b0 = cs + tt + s0;  // first count field of candidate cs+tt
        uint32_t m = 0;
        if (NS < 0 && P.pf_var && SPK_VSCREEN && b0 + 48 <= wend) {
          // the terminator bytes (high bit clear) of the 32 bytes from b0 as
          // a mask: a varint's length is a ctz, not an 8-byte decode; a
          // candidate whose varints run past the mask takes vread
          const uint32_t o0 = (uint32_t)(b0 - ts), i = win_dw(o0), sh = o0 & 3;
          const lds_u32 *d = rd.d;
          uint32_t T = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t dk = __builtin_amdgcn_alignbyte(d[i + k + 1], d[i + k], sh);
            T |= ((((~dk) & 0x80808080u) * 0x00204081u) >> 28) << (4 * k);
          }
          for (int kk = 0; kk < 8; ++kk) {
            uint32_t off = (uint32_t)kk;
            bool ok = true;
            for (uint32_t j = 0; j < P.vfirst[1] && ok; ++j) {
              uint32_t l;
              if (off + 10 <= 32) {
                const uint32_t mm = T >> off;  // (off < 32)
                l = mm ? (uint32_t)__builtin_ctz(mm) + 1 : 11;
              } else {
                uint64_t v;
                l = rd.vread(b0 + off, len, &v);
                if (!l) l = 11;
              }
              if (l > 10) ok = false;
              off += l + P.vafter[j];
            }
            if (ok) ok = (b0 + off + w <= len ? rd(b0 + off) : ~0ull) <= c0t;
            m |= (ok ? 1u : 0u) << kk;
          }
        } else if (NS < 0 && P.pf_var) {
          for (int kk = 0; kk < 8; ++kk) {
            uint64_t q = b0 + kk;
            bool ok = true;
            for (uint32_t j = 0; j < P.vfirst[1]; ++j) {
              uint64_t v;
              const uint32_t l = rd.vread(q, len, &v);
              if (!l || l == kViBad) {
                ok = false;
                break;
              }
              q += l + P.vafter[j];
            }
            if (ok) ok = (q + w <= len ? rd(q) : ~0ull) <= c0t;
            m |= (ok ? 1u : 0u) << kk;
          }
        } else if (b0 + 20 <= wend) {
          const uint32_t o0 = (uint32_t)(b0 - ts), i = win_dw(o0), sh = o0 & 3;
          const lds_u32 *d = rd.d;
          const uint32_t d0 = d[i], d1 = d[i + 1], d2 = d[i + 2], d3 = d[i + 3], d4 = d[i + 4];
          const uint32_t wd[4] = {__builtin_amdgcn_alignbyte(d1, d0, sh),
                                  __builtin_amdgcn_alignbyte(d2, d1, sh),
                                  __builtin_amdgcn_alignbyte(d3, d2, sh),
                                  __builtin_amdgcn_alignbyte(d4, d3, sh)};
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const uint32_t lo = __builtin_amdgcn_alignbyte(wd[(kk >> 2) + 1], wd[kk >> 2], kk & 3);
            uint64_t cv = w == 1 ? (lo & 0xFFu) : w == 2 ? (lo & 0xFFFFu) : lo;
            if (w == 8)
              cv |= (uint64_t)__builtin_amdgcn_alignbyte(wd[(kk >> 2) + 2], wd[(kk >> 2) + 1], kk & 3)
                    << 32;
            m |= (cv <= c0t ? 1u : 0u) << kk;
          }
        } else {
          for (int kk = 0; kk < 8; ++kk) {
            const uint64_t q = b0 + kk;
            const uint64_t cv = q + w <= len ? rd(q) : ~0ull;
            m |= (cv <= c0t ? 1u : 0u) << kk;
          }
        }
        if (P.pf_all) {  // first span an OPTION / no span: any byte may start a record
          m = 0xFFu;
          if (NS <= -2 && P.hscr) {
            // ... but a nested record that opens with an optional / expected
            // group starts with a has_value byte, 0 or 1 from every writer
            // (a start behind a larger one is found by the exact repair walk)
            m = 0;
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
              m |= (b0 + kk < len && rd.byte(b0 + kk) <= 1u ? 1u : 0u) << kk;
          }
        }
        if (NS <= -2 && P.scr2 && m) {
          // the second count, past the first span's payload
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            if (!((m >> kk) & 1u)) continue;
            const uint64_t b = b0 + kk;
            const uint64_t c0 = rd(b);
            const uint64_t q2 = b + w + c0 * P.esz0 + P.s2skip;
            if (q2 + w > len || rd(q2) > P.c1max) m &= ~(1u << kk);
          }
        }
        const uint64_t rem = ce - (cs + tt);  // candidates must start in the chunk
        if (rem < 8) m &= (1u << rem) - 1u;
        if (!m) {
          tt += 8;
          if (cs + tt >= ce) done = true;
          continue;
        }
        tt += (uint32_t)__builtin_ctz(m);
        x = cs + tt;
        sx = x;
        k = 0;
        past = 0;
        ex = kNoPos;
        QFOR(q) ksum[q] = 0;
        searching = false;
      }
      if (kNPast<NS> == 0 && x >= ce) {  // no walks past the chunk: the exit is known
        ex = x;
        break;
      }
      uint64_t rc[NS > 0 ? NS : kVS];
      // (the exact start of tile 0 walks unbounded: its records may be long)
      const uint64_t L = x >= len ? 0
                         : exact  ? wlen_rd<NS>(P, rd, len, x, w, rc)
                                  : wlen_spec<NS>(P, rd, len, x, w, rc, scap, tight);
      if (stat) ++stat[2];
      if (!exact && ((L == 0 && x < len) || L > kPlaus)) {  // off the record grid
        if (stat) ++stat[3];
        tt += 1;
        searching = true;
        sx = kNoPos;
        if (cs + tt >= ce) done = true;
        continue;
      }
      if (x < ce) {
        if (!L) {  // the wire ends inside the chunk: the walk's path ends here
          ex = kTermPos;
          term_at = x;
          break;
        }
#pragma unroll
        for (uint32_t j = 0; j < kMergePts; ++j)  // (static indices: sp stays in registers)
          if (k == j) {
            sp.pos[j] = (uint32_t)(x - cs);
            QFORS(q) sp.ps[j][q] = (uint32_t)ksum[q];
          }
        ++k;
        QFOR(q) ksum[q] += rc[q];
      } else {
        if (!past) ex = x;
        ++past;
        if (!L || past >= npast) break;
      }
      x += L;
    }
    if (sx != kNoPos || !tight) break;
    // no start under the caps in this chunk: search it again without them
    tight = false;
    c0t = P.c0max;
    tt = 0;
    x = cs;
    searching = true;
    done = false;
    }
    if (sx != kNoPos) {
      used = sx;
      cnt = k;
      QFOR(q) sums[q] = ksum[q];
      // merge information: spans fit the path record, sums fit 32 bits
      bool mok = NS > 0 || P.ns <= (uint32_t)SpecPath<NS>::kS;
      QFORS(q) {
        mok = mok && ksum[q] < 0xFFFFFFFFull;
        sp.sums[q] = ksum[q];
      }
      sp.np = mok ? (k < kMergePts ? k : kMergePts) : 0;
      sp.cnt = k;
      sp.ex = ex;
      sp.term_at = term_at;
    } else {
      ex = kNoPos;
    }
  } else {
    // a lane past the wire end: no chunk; it passes its entry through
    used = kNoPos;
    ex = kNoPos;
  }
  // ---- 2. resolution given the tile's assumed entry ----
  const uint64_t used0 = used;
  uint64_t X = __shfl(used, 0);  // lane 0's spec start (kNoPos: no plausible start)
  if (exact0) X = p0;
  if (!exact0 && !(dbg & 16)) {
    // Two independent speculations that agree are far likelier true: when
    // chunk 0's walk does not exit where chunk 1's speculative walk starts,
    // take the first start candidate of chunk 0 whose walk does (in parallel,
    // one candidate per lane), so the tile rarely publishes a wrong assumption.
    const uint64_t x1 = __shfl(used, 1), e0 = __shfl(ex, 0), ce0 = __shfl(ce, 0);
    const uint64_t cs0 = ts;
    if (x1 != kNoPos && e0 != x1 && cs0 < len) {
      if (stat && lane == 0) ++stat[5];
      const uint64_t from = X != kNoPos ? X + 1 : cs0;
      for (uint64_t b = from; b < ce0; b += 64) {
        const uint64_t q = b + lane;
        bool ok = q < ce0 && screen_one<NS>(P, rd, len, w, q);
        uint64_t qe = kNoPos, qt;
        uint32_t qc = 0;
        uint64_t qs[NS > 0 ? NS : kVS];
        if (ok) {
          walk_true<NS>(P, rd, len, w, q, ce0, qe, qc, qs, qt, kK1Reach<NS>);
          ok = qe == x1;
        }
        const uint64_t m = __ballot(ok);
        if (m) {
          const uint32_t l = (uint32_t)__builtin_ctzll(m);
          const uint64_t nq = __shfl(q, l);
          const uint32_t nc = (uint32_t)__shfl((uint64_t)qc, l);
          QFOR(qq) {
            const uint64_t v = __shfl(ok ? qs[qq] : 0, l);
            if (lane == 0) sums[qq] = v;
          }
          if (lane == 0) {
            used = nq;
            ex = x1;
            cnt = nc;
            term_at = kTermPos;
            sp.np = 0;  // chunk 0 is not on its speculative path any more
          }
          X = nq;
          break;
        }
      }
    }
  }
  if (X == kNoPos && !exact0 && !(dbg & 8192)) {
    // chunk 0 holds no plausible start (it lies inside a long record: a
    // string of a few hundred bytes spans several chunks): the tile's first
    // record start is the first start some later chunk speculated. Without
    // this the tile published no entry at all, pick could not match it and
    // runs of such tiles fell through the repair passes to the sequential
    // fixer (binary strings of 100-3000 B: 35.8 ms for 62 MB)
    const uint64_t mv = __ballot(used != kNoPos);
    if (mv) X = __shfl(used, (int)__builtin_ctzll(mv));
  }
  if (X != kNoPos && !(dbg & 32))
    resolve_tile_sp<NS>(P, rd, len, w, cs, ce, lane, X, sp, used, ex, cnt, sums, term_at, stat,
                        kK1Reach<NS>);
  if (stat && used != used0) ++stat[4];
  st.used = used;
  st.ex = ex;
  st.term_at = term_at;
  st.cnt = cnt;
  QFOR(q) st.sums[q] = sums[q];
  st.sp = sp;
  return X;
}

// ---- K1 ----------------------------------------------------------------------
// SPK_K1_STATS=1: the K1 statistics of SPK_TILE_DBG=4096 (scripts/diag_tiles.py)
// compiled in (off by default: the run-time null checks in the walk loop
// cost C4's K1 2 %)
#ifndef SPK_K1_STATS
#define SPK_K1_STATS 0
#endif
// SPK_K1_PRINT=1 (with SPK_K1_STATS and SPK_TILE_DBG=4096, scripts/diag_k1.sh):
// the first pick of every decode prints them, the tile times in 10 ns ticks
#ifndef SPK_K1_PRINT
#define SPK_K1_PRINT 0
#endif
#if SPK_K1_PRINT
__device__ __forceinline__ uint64_t k1_clock() { return __builtin_amdgcn_s_memrealtime(); }
#else
__device__ __forceinline__ uint64_t k1_clock() { return __builtin_readcyclecounter(); }
#endif
// W: the count width as a compile-time constant (0: read from the header at
// run time). The walkers' count reads, screens and bounds checks then carry
// no width switch: nested walks are divergent loops, so every branch of the
// switch cost each step its scalar branch code
template <int NS, uint32_t W>
__device__ __forceinline__ void vec_tile_spec_body(const DecArgs &a, const WalkProg &P,
                                                   const uint8_t *__restrict__ wire,
                                                   const uint8_t *__restrict__ ws,
                                                   const TileBufs &TB, uint32_t dbg,
                                                   v4u_t *win, uint64_t t, uint32_t lane) {
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  const uint64_t tclk0 = (dbg & 4096) ? k1_clock() : 0;
  nt_prologue<NS>(a, lane);
  const uint32_t w = W ? W : c->w;
  const uint64_t len = a.wire_len, p0 = c->p0;
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  const uint64_t ts = p0 + t * kTileBytes;
  const TileView tv = stage_tile(win, wire, len, ts, w, lane);
  const WinReader &rd = tv.rd;
  const uint64_t wend = tv.wend;
  const uint64_t cs = ts + (uint64_t)lane * kTChunk;
  const uint64_t ce = cs + kTChunk < len ? cs + kTChunk : (cs < len ? len : cs);
  const bool rng = reinterpret_cast<const FCtl *>(ws + kWsFCtl)->range != 0;
  TileLane<NS> st;
  uint32_t stat[6] = {0, 0, 0, 0, 0, 0};
  const uint64_t X = tile_spec_resolve<NS>(P, rd, len, w, ts, wend, cs, ce, lane, t == 0 && !rng,
                                           p0, dbg, st, (SPK_K1_STATS && (dbg & 4096)) ? stat : nullptr,
                                           (NS > -2 && SPK_SCAP) ? c : nullptr);
  if (SPK_K1_STATS && (dbg & 4096)) {  // K1 statistics (scripts/diag_tiles.py)
    FCtl *fcd = reinterpret_cast<FCtl *>(const_cast<uint8_t *>(ws) + kWsFCtl);
    for (uint32_t k = 0; k < 6; ++k) {
      const uint64_t v = wave_sum_u64(stat[k]);
      if (lane == 0) atomicAdd(&fcd->diag[k], (unsigned long long)v);
    }
    const uint64_t dt = k1_clock() - tclk0;  // this tile's cycles (or ticks)
    if (lane == 0) {
      atomicMax(&fcd->diag[6], (unsigned long long)dt);
      atomicAdd(&fcd->diag[7], (unsigned long long)dt);
    }
  }
  const uint64_t used = st.used, ex = st.ex;
  const uint32_t cnt = st.cnt;
  const uint64_t *sums = st.sums;
  uint64_t tcnt = wave_sum_u64(cnt), tsum[NS > 0 ? NS : kVS];
  QFOR(q) tsum[q] = wave_sum_u64(sums[q]);
  // ---- 3. entry alternatives (tile 0's entry is exact) ----
  uint32_t nalt = X != kNoPos ? 1u : 0u;
  uint64_t alt_e = kNoPos, alt_c = 0, alt_s[NS > 0 ? NS : kVS];  // lane a holds alt a
  QFOR(q) alt_s[q] = 0;
  if (lane == 0 && nalt) {
    alt_e = X;
    alt_c = tcnt;
    QFOR(q) alt_s[q] = tsum[q];
  }
  if ((dbg & 4) && t > 0) {
    // ---- 3a. entry alternatives: other start candidates in chunk 0 after X
    // whose walk reaches chunk 0's exit; one per lane, in parallel ----
    const uint64_t e0 = __shfl(ex, 0), ce0 = __shfl(ce, 0);
    const uint32_t c0 = __shfl(cnt, 0);
    uint64_t s0[NS > 0 ? NS : kVS];
    QFOR(q) s0[q] = __shfl(sums[q], 0);
    const uint64_t lim = e0 < ce0 ? e0 : ce0;
    for (uint64_t b = X + 1; nalt && nalt < kAlt && b < lim && b < X + 1 + 128; b += 64) {
      const uint64_t q = b + lane;
      bool ok = q < lim && screen_one<NS>(P, rd, len, w, q);
      uint64_t qe = kNoPos, qt;
      uint32_t qc = 0;
      uint64_t qs[NS > 0 ? NS : kVS];
      if (ok) {
        walk_true<NS>(P, rd, len, w, q, ce0, qe, qc, qs, qt);
        ok = qe == e0;
      }
      uint64_t m = __ballot(ok);
      while (m && nalt < kAlt) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint64_t ae = __shfl(q, l);
        const uint64_t ac = tcnt - c0 + __shfl((uint64_t)qc, l);
        if (lane == nalt) {
          alt_e = ae;
          alt_c = ac;
        }
        QFOR(qq) {
          const uint64_t v = tsum[qq] - s0[qq] + __shfl(ok ? qs[qq] : 0, l);
          if (lane == nalt) alt_s[qq] = v;
        }
        ++nalt;
      }
    }
  }
  // ---- publish: chunk states and the tile function ----
  const uint64_t g = t * 64 + lane;
  TB.cused[g] = used;
  TB.cex[g] = ex;
  TB.ccnt[g] = cnt;
  QFOR(q) TB.csum[(uint64_t)q * TB.nchunks + g] = sums[q];
  uint64_t *fn = TB.fn + t * kFnWords;
  const uint64_t y63 = __shfl(ex, 63);
  if (lane == 0) {
    fn[0] = y63;
    fn[1] = nalt;
  }
  if (lane < kAlt) {
    uint64_t *al = fn + 2 + lane * kAltWords;
    al[0] = lane < nalt ? alt_e : kNoPos;
    al[1] = alt_c;
    QFOR(q) al[2 + q] = alt_s[q];
  }
}

#ifndef SPK_WSPEC  // 1: K1 of the nested walk program per count width; 2: every layout
#define SPK_WSPEC 2   // (2: C4 K1 -15 %, C3 -13 %, cv -5 % against 1, same-box A/B)
#endif
template <int NS>
__global__ __launch_bounds__(64 * kDecWaves) void vec_tile_spec(DecArgs a, WalkProg P,
                                                                const uint8_t *__restrict__ wire,
                                                                const uint8_t *__restrict__ ws,
                                                                TileBufs TB, uint32_t dbg) {
  __shared__ v4u_t win_s[kDecWaves][win_slots(kTileVec)];
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t t = (uint64_t)blockIdx.x * kDecWaves + wv;
  // varint layouts with the speculation caps: the walk program from LDS (the
  // compiler otherwise copied the by-value argument into scratch memory and
  // read it from there: 264 B per lane). (Every flat layout from LDS was
  // measured slower: C3 K1 0.193 -> 0.233 ms.) Staged before any wave of the
  // block may leave, so every wave reaches the barrier.
  constexpr bool kLdsProg = NS == -1 && SPK_SCAP != 0;
  __shared__ WalkProg Ps;
  if constexpr (kLdsProg) {
    if (threadIdx.x == 0) Ps = P;
    __syncthreads();
  }
  const WalkProg &Pk = kLdsProg ? Ps : P;
  if (t >= TB.ntiles || !vec_live(c)) return;  // wave-uniform
  if constexpr (SPK_WSPEC >= 2 || (SPK_WSPEC == 1 && NS == -3)) {
    switch (c->w) {  // (uniform: the header's width)
      case 1: vec_tile_spec_body<NS, 1>(a, Pk, wire, ws, TB, dbg, win_s[wv], t, lane); return;
      case 2: vec_tile_spec_body<NS, 2>(a, Pk, wire, ws, TB, dbg, win_s[wv], t, lane); return;
      case 4: vec_tile_spec_body<NS, 4>(a, Pk, wire, ws, TB, dbg, win_s[wv], t, lane); return;
      default: vec_tile_spec_body<NS, 8>(a, Pk, wire, ws, TB, dbg, win_s[wv], t, lane); return;
    }
  } else {
    vec_tile_spec_body<NS, 0>(a, Pk, wire, ws, TB, dbg, win_s[wv], t, lane);
  }
}

// tile t's entry: tile t-1's published exit (tile 0: the payload start)
__device__ __forceinline__ uint64_t tile_entry(const TileBufs &TB, const FCtl *fc, uint64_t t) {
  return t == 0 ? fc->entry0 : TB.fn[(t - 1) * kFnWords];
}

// K1's speculation caps (VCtl::scap), after the header: one wave stages the first 4 KiB of the
// records from tile 0's entry in LDS and lane 0 walks up to kSampRecs of them;
// a span's cap is twice its largest count there (at least 15), never above
// the layout's own limit. The caps only steer the speculation (a chunk with
// no start under them is searched without them; the true walks of the
// resolution, repair and emit passes never see them), so a message whose
// later records have longer containers decodes the same, a little slower.
constexpr uint32_t kSampVec = 4096 / 16;
#ifndef SPK_SAMP_RECS
#define SPK_SAMP_RECS 16
#endif
constexpr uint32_t kSampRecs = SPK_SAMP_RECS;
template <int NS>
__global__ __launch_bounds__(64) void vec_hdr_sample(DecArgs a, WalkProg P,
                                                     const uint8_t *__restrict__ wire,
                                                     uint8_t *__restrict__ ws,
                                                     spk_dresult_t *res) {
  __shared__ v4u_t win[win_slots(kSampVec)];
  if (threadIdx.x == 0) vec_hdr_body(a, wire, ws, res, 0u, (uint64_t)0);
  __syncthreads();
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  const FCtl *fc = reinterpret_cast<const FCtl *>(ws + kWsFCtl);
  const uint32_t lane = threadIdx.x, nsp = NS > 0 ? (uint32_t)NS : P.ns;
  const uint64_t len = a.wire_len, x0 = fc->entry0;
  const uint32_t w = c->w;
  uint64_t mx[NS > 0 ? NS : kVS];
  QFOR(q) mx[q] = 0;
  uint32_t got = 0;
  if (vec_live(c) && x0 < len && !P.pf_all) {  // (wave-uniform)
    const TileView tv = stage_win<kSampVec>(win, wire, len, x0, w, lane);
    if (lane == 0) {
      const uint64_t n = c->n < kSampRecs ? c->n : kSampRecs;
      uint64_t x = x0;
      for (uint64_t i = 0; i < n && x + 64 <= tv.wend; ++i) {
        uint64_t rc[NS > 0 ? NS : kVS];
        const uint64_t L = wlen_rd<NS>(P, tv.rd, len, x, w, rc);
        if (!L) break;
        QFOR(q) mx[q] = rc[q] > mx[q] ? rc[q] : mx[q];
        ++got;
        x += L;
      }
    }
  }
  if (lane == 0) {
    // caps only where they tighten the first-count screen by SPK_SCAP_MINR x
    // or more: a screen already that selective gains nothing from them (C4:
    // 511 vs 32 slower with them in round 3, faster since K1 keeps its state in
    // locals; C3 4092 vs ~96, cv 4096 vs 32 faster)
    {
      uint64_t t0 = mx[0] < (1ull << 60) ? SPK_SCAP_MUL * mx[0] : ~0ull;
      t0 = t0 < 15 ? 15 : t0;
      if ((P.optm & 1u) || (uint64_t)P.c0max < (uint64_t)SPK_SCAP_MINR * t0) got = 0;
    }
    uint64_t c0 = P.c0max;
    QFOR(q) {
      uint64_t cp = P.cmax[q];
      if (got && !((P.optm >> q) & 1u)) {
        const uint64_t t = mx[q] < (1ull << 60) ? SPK_SCAP_MUL * mx[q] : ~0ull;
        cp = t < 15 ? 15 : t;
        if (cp > P.cmax[q]) cp = P.cmax[q];
        if (q == 0 && cp < c0) c0 = cp;
      }
      c->scap[q] = cp;
    }
    c->spec_c0 = c0;
    c->scap_on = got ? 1u : 0u;
  }
}

// range mode, entry unknown: tile 0 assumes its own speculated entry
__global__ void vec_range_entry(uint8_t *__restrict__ ws, TileBufs TB) {
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  if (threadIdx.x == 0 && fc->range && fc->entry0 == kNoPos && TB.ntiles) fc->entry0 = TB.fn[2];
}

// Tile t whose entry lies at or past its end (inside a record that spans it):
// no records, exit = entry.
__device__ __forceinline__ void tile_pass_through(const TileBufs &TB, uint64_t t, uint64_t T,
                                                  uint32_t nsp) {
  uint64_t *fn = TB.fn + t * kFnWords;
  fn[0] = T;
  fn[1] = 1;
  fn[2] = T;
  fn[3] = 0;
  QFORV(q) fn[4 + q] = 0;
  TB.sel[t] = 0;
}

// Tile t's exit E lies past tile t+1: the tiles a record spans, t+1 ..
// tile(E)-1, pass E through (written here so that a long record costs one
// select pass, not one per tile; any race with those tiles' own waves is
// settled by the next pass and the sequential check).
__device__ __forceinline__ void tile_jump(const TileBufs &TB, uint64_t p0, uint64_t t, uint64_t E,
                                          uint32_t nsp, uint32_t lane,
                                          unsigned long long *changed, uint32_t step = 64) {
  if (E == kTermPos || E == kNoPos || E < p0) return;
  const uint64_t e0 = (E - p0) / kTileBytes;
  const uint64_t e = e0 < TB.ntiles ? e0 : TB.ntiles;
  if (t + 1 >= e) return;
  // the pass changed other tiles' functions: the next pass re-checks them
  if (lane == 0) atomicAdd(changed, 1ull);
  for (uint64_t v = t + 1 + lane; v < e; v += step) tile_pass_through(TB, v, E, nsp);
}

// tile t's selection given its current entry T (kSelBroken: none fits)
__device__ __forceinline__ int32_t tile_select_for(const TileBufs &TB, uint64_t t, uint64_t T) {
  if (T == kTermPos) return kSelTerm;
  const uint64_t *fn = TB.fn + t * kFnWords;
  const uint32_t nalt = (uint32_t)fn[1];
  for (uint32_t k = 0; k < nalt && k < kAlt; ++k)
    if (fn[2 + k * kAltWords] == T) return (int32_t)k;
  return kSelBroken;
}

#ifndef SPK_CHAIN_TERM1
#define SPK_CHAIN_TERM1 1  // (cmpg chain 0.506 -> 0.430 ms, 4.714 -> 4.649 ms per step, same box)
#endif
#ifndef SPK_PICK_WAVEJUMP
#define SPK_PICK_WAVEJUMP 1  // (cmpg 5.144 -> 4.772 ms per step, same-box A/B)
#endif
// ---- K2: select each tile's entry (one thread per tile); tiles whose entry
// is none of theirs are listed and re-walked by vec_tile_repair (one wave per
// listed tile, a fixed grid striding over the list) -------------------------
__global__ __launch_bounds__(256) void vec_tile_pick(uint8_t *__restrict__ ws, TileBufs TB,
                                                     uint32_t nsp, uint32_t pass) {
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!vec_live(c)) return;                               // (uniform)
#if SPK_K1_PRINT
  if (pass == 0 && t == 0)
    printf("[k1] ntiles %llu n %llu w %u p0 %llu rounds %llu walks %llu wlen %llu offgrid %llu "
           "changed %llu xchk %llu maxtile %llu sumtile %llu\n",
           (unsigned long long)TB.ntiles, (unsigned long long)c->n, c->w,
           (unsigned long long)c->p0, fc->diag[0], fc->diag[1], fc->diag[2], fc->diag[3],
           fc->diag[4], fc->diag[5], fc->diag[6], fc->diag[7]);
#endif
  if (pass > 0 && !fc->broken[pass - 1]) return;  // the previous pass fixed nothing
  // broken tiles are counted and listed with one atomic per wave (a broken
  // tile per thread adding to the same two words serialised thousands of
  // atomics: bytes after a message, e.g. a compatible member's version
  // passes, break most of their tiles)
  bool brk = false, list = false;
  uint64_t jE = kNoPos;  // SPK_PICK_WAVEJUMP: this tile's pass-through run, for the wave
  if (t < TB.ntiles) {
    const uint64_t T = tile_entry(TB, fc, t);
    int32_t sel = T == kNoPos ? kSelBroken : tile_select_for(TB, t, T);
    // (a nested tile whose K1 walk gave up has an unknown exit: walked again)
    if (sel >= 0 && TB.fn[t * kFnWords] == kNoPos) sel = kSelBroken;
    // a tile inside a record whose predecessor is inside it too: the run of
    // pass-through tiles was written from the record's first tiles, so it
    // does not write the rest again (every tile of an R-tile run rewriting
    // its remainder was R^2 / 2 tile writes: 0.2-0.5 ms a pick on cmpg)
    const uint64_t ts = c->p0 + t * kTileBytes;
    const bool inner = T != kNoPos && T >= ts + kTileBytes && t > 0 &&
                       tile_entry(TB, fc, t - 1) == T;
    if (sel != kSelBroken || T == kNoPos) {
      TB.sel[t] = sel;
      if (sel >= 0 && !inner) {
        if (SPK_PICK_WAVEJUMP)
          jE = TB.fn[t * kFnWords];
        else
          tile_jump(TB, c->p0, t, TB.fn[t * kFnWords], nsp, 0, &fc->broken[pass], 1);
      }
    } else {
      brk = true;
      if (T >= ts + kTileBytes) {  // inside a record that spans the tile
        tile_pass_through(TB, t, T, nsp);
        if (!inner) {
          if (SPK_PICK_WAVEJUMP)
            jE = T;
          else
            tile_jump(TB, c->p0, t, T, nsp, 0, &fc->broken[pass], 1);
        }
      } else {
        list = true;
      }
    }
  }
  const uint32_t lane = threadIdx.x & 63;
  if (SPK_PICK_WAVEJUMP) {
    // a run of pass-through tiles written by the whole wave, one run at a
    // time, not by its tile's one thread (a false exit far ahead in the bytes
    // after a message wrote thousands of tiles serially)
    const uint64_t E0 = c->p0;
    uint64_t mj = __ballot(jE != kNoPos && jE != kTermPos && jE >= E0 &&
                           (jE - E0) / kTileBytes > t + 1);
    while (mj) {
      const int l = (int)__builtin_ctzll(mj);
      mj &= mj - 1;
      tile_jump(TB, E0, __shfl(t, l), __shfl(jE, l), nsp, lane, &fc->broken[pass], 64);
    }
  }
  const uint64_t mb = __ballot(brk), ml = __ballot(list);
  if (lane == 0 && mb) atomicAdd(&fc->broken[pass], (unsigned long long)__popcll(mb));
  if (!ml) return;
  uint64_t base = 0;
  if (lane == 0) base = atomicAdd(&fc->nlist[pass], (unsigned long long)__popcll(ml));
  base = __shfl(base, 0);
  if (list) TB.blist[base + __popcll(ml & ((1ull << lane) - 1))] = (uint32_t)t;
}

// Tile t re-resolved from its true entry T, its window staged in tv: the
// chunk states and a one-entry tile function; returns the tile's exit.
template <int NS>
__device__ __forceinline__ uint64_t tile_resolve_from(const WalkProg &P, const TileView &tv,
                                                      const TileBufs &TB, uint64_t len, uint32_t w,
                                                      uint64_t t, uint64_t ts, uint64_t T,
                                                      uint32_t lane) {
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  const uint64_t cs = ts + (uint64_t)lane * kTChunk;
  const uint64_t ce = cs + kTChunk < len ? cs + kTChunk : (cs < len ? len : cs);
  const uint64_t g = t * 64 + lane;
  uint64_t used = TB.cused[g], ex = TB.cex[g], term_at = kTermPos;
  uint32_t cnt = TB.ccnt[g];
  uint64_t sums[NS > 0 ? NS : kVS];
  QFOR(q) sums[q] = TB.csum[(uint64_t)q * TB.nchunks + g];
  resolve_tile<NS>(P, tv.rd, len, w, ce, lane, T, used, ex, cnt, sums, term_at);
  const uint64_t tcnt = wave_sum_u64(cnt);
  uint64_t tsum[NS > 0 ? NS : kVS];
  QFOR(q) tsum[q] = wave_sum_u64(sums[q]);
  TB.cused[g] = used;
  TB.cex[g] = ex;
  TB.ccnt[g] = cnt;
  QFOR(q) TB.csum[(uint64_t)q * TB.nchunks + g] = sums[q];
  const uint64_t y63 = __shfl(ex, 63);
  if (lane == 0) {
    uint64_t *fn = TB.fn + t * kFnWords;
    fn[0] = y63;
    fn[1] = 1;
    fn[2] = T;
    fn[3] = tcnt;
    QFOR(q) fn[4 + q] = tsum[q];
    TB.sel[t] = 0;
  }
  return y63;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

constexpr unsigned kRepairGrid = 2048;
template <int NS>
__global__ __launch_bounds__(64) void vec_tile_repair(DecArgs a, WalkProg P,
                                                      const uint8_t *__restrict__ wire,
                                                      uint8_t *__restrict__ ws, TileBufs TB,
                                                      uint32_t pass) {
  __shared__ v4u_t win_s[1][win_slots(kTileVec)];
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  const uint32_t lane = threadIdx.x;
  if (!vec_live(c)) return;
  const uint64_t nl = fc->nlist[pass];
  if (!nl) return;
  nt_prologue<NS>(a, lane);
  const uint32_t w = c->w;
  const uint64_t len = a.wire_len, p0 = c->p0;
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  for (uint64_t j = blockIdx.x; j < nl; j += gridDim.x) {
    const uint64_t t = TB.blist[j];
    const uint64_t T = tile_entry(TB, fc, t);  // (re-read: a predecessor may have moved)
    const uint64_t ts = p0 + t * kTileBytes;
    if (T == kNoPos) {
      if (lane == 0) TB.sel[t] = kSelBroken;
      continue;
    }
    if (T >= ts + kTileBytes) {
      if (lane == 0) tile_pass_through(TB, t, T, nsp);
      tile_jump(TB, p0, t, T, nsp, lane, &fc->broken[pass]);
      continue;
    }
    const TileView tv = stage_tile(win_s[0], wire, len, ts, w, lane);
    const uint64_t y63 = tile_resolve_from<NS>(P, tv, TB, len, w, t, ts, T, lane);
    tile_jump(TB, p0, t, y63, nsp, lane, &fc->broken[pass]);
    wave_lds_sync();  // the window is restaged for the next listed tile
  }
}

// ---- K3: the selected contribution of tile t (vec_tile_chain, once the
// tile's selection is final); the first tile whose path ends inside it (its
// exit is kTermPos) ----------------------------------------------------------
__device__ __forceinline__ uint64_t tile_contrib(const TileBufs &TB, FCtl *fc, uint64_t t,
                                                 uint32_t nsp, uint64_t *col = nullptr) {
  const uint64_t *fn = TB.fn + t * kFnWords;
  const int32_t sel = TB.sel[t];
  uint64_t cnt = 0, s[kVS] = {};
  if (sel >= 0) {
    cnt = fn[2 + sel * kAltWords + 1];
    QFORV(q) s[q] = fn[2 + sel * kAltWords + 2 + q];
    if (fn[0] == kTermPos) atomicMin(&fc->term_tile, (unsigned long long)t);
  } else if (sel == kSelTerm) {
    atomicMin(&fc->term_tile, (unsigned long long)t);
  } else {
    atomicAdd(&fc->unresolved, 1ull);  // (only past the message's end: bytes after it)
    atomicMin(&fc->unres_tile, (unsigned long long)t);
  }
  TB.contrib[t] = cnt;
  QFORV(q) TB.contrib[(uint64_t)(1 + q) * TB.ntiles + t] = s[q];
  if (col) {
    col[0] += cnt;
    QFORV(q) col[1 + q] += s[q];
  }
  return cnt;
}

// K3: tscan_apply blocks cover kTScanBlock consecutive tiles; their carries
// are sums of the segment sums (kTSeg tiles each) that vec_tile_chain writes
// (segments of a whole apply block kept 12 of its blocks busy for C3, each
// thread 8 tiles deep: 9.7 us)
constexpr uint32_t kTScanIPT = 8;
constexpr uint64_t kTScanBlock = 256ull * kTScanIPT;
constexpr uint64_t kTSeg = 256;
// segment seg's column sums into TB.scan[col * nb + seg] (a block of NT
// threads); CONTRIB: each tile's contribution is written on the way
template <uint32_t NT, bool CONTRIB>
__device__ void tscan_segment(const TileBufs &TB, FCtl *fc, uint64_t seg, uint64_t nb,
                              uint32_t nsp, uint64_t *sh) {
  uint64_t v[1 + kVS] = {};
  const uint64_t b0 = seg * kTSeg;
  for (uint64_t k = threadIdx.x; k < kTSeg; k += NT) {
    const uint64_t i = b0 + k;
    if (i >= TB.ntiles) break;
    if (CONTRIB) {
      tile_contrib(TB, fc, i, nsp, v);
    } else {
      v[0] += TB.contrib[i];
      QFORV(q) v[1 + q] += TB.contrib[(uint64_t)(1 + q) * TB.ntiles + i];
    }
  }
  for (uint32_t c = 0; c < 1 + nsp && c < 1 + kVS; ++c) {
    uint64_t x = v[0];
#pragma unroll
    for (uint32_t k = 1; k < 1 + kVS; ++k) x = c == k ? v[k] : x;
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t t = 0;
      for (uint32_t w = 0; w < NT / 64; ++w) t += sh[w];
      TB.scan[(uint64_t)c * nb + seg] = t;
    }
    __syncthreads();
  }
}

// ---- K2, what the passes leave: the tile chain ------------------------------
// A tile whose entry none of its alternatives takes after the three passes
// starts a chain: each later tile's true entry is known only once its
// predecessor's is (strings whose bytes are themselves a record stream: every
// tile inside one speculates a plausible false grid, and where such a string
// ends the true entry is none of the speculated ones). vec_chain_first finds
// the chain's first tile f0; in vec_tile_chain a persistent grid of one-wave
// blocks takes the tiles from f0 on in order and, before it needs the entry,
// computes each tile's exit for EVERY entry byte in LDS: the next record start
// of each byte (one record walk per byte), then pointer jumping to the last
// record start of each path inside the tile. The chain itself is then one
// hand-off per entered tile: its block looks the exit up (one more record
// walk) and stores it, tagged, into the entry word of the tile it lands in
// (the tiles between pass it through), then re-resolves its own chunk states
// from the entry off the chain's critical path. Hand-offs are 8-B agent-scope
// atomic stores polled with agent-scope loads (no payload rides on them: the
// word is the value); every other output is read by later launches.
constexpr uint64_t kEntEnter = 1ull << 62, kEntThru = 2ull << 62, kEntTerm = 3ull << 62;
constexpr uint64_t kEntPos = (1ull << 62) - 1;
// map entries (u16): below kTileBytes the next record start in the tile (the
// byte itself: its record ends too far past the tile to code); from kMapExit
// the path's exit, coded as its distance past the tile's end
constexpr uint16_t kMapBad = 0xFFFFu;  // the path from this byte fails inside the tile
constexpr uint16_t kMapUnk = 0xFFFEu;  // a bounded nested walk gave up: walked at the hand-off
constexpr uint32_t kMapExit = kTileBytes, kMapNear = 0xFFF0u - kMapExit;
static_assert(kTileBytes <= 0x8000u, "chain map entries are u16 tile offsets");
constexpr unsigned kChainGrid = 512;
#ifndef SPK_PICK_PASSES  // pick / repair passes before the chain takes what they leave (1..3)
#define SPK_PICK_PASSES 2
#endif
constexpr uint32_t kPickPasses = SPK_PICK_PASSES;
constexpr uint32_t kChainSpin = 1u << 20;  // poll rounds (~1 us each) before a lost hand-off is an error

template <uint32_t NW>
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t *sh) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_down(v, o);
    v = x < v ? x : v;
  }
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t m = sh[0];
#pragma unroll
  for (uint32_t k = 1; k < NW; ++k) m = sh[k] < m ? sh[k] : m;
  __syncthreads();
  return m;
}

// tile t's selection under its current entry (kSelBroken also when the
// selected exit is unknown); *bad: broken although its entry is known
__device__ __forceinline__ int32_t tile_sel_now(const TileBufs &TB, const FCtl *fc, uint64_t t,
                                                bool *bad) {
  const uint64_t T = tile_entry(TB, fc, t);
  int32_t sel = tile_select_for(TB, t, T);
  if (sel >= 0 && TB.fn[t * kFnWords] == kNoPos) sel = kSelBroken;  // exit unknown
  *bad = sel == kSelBroken && T != kNoPos;
  return sel;
}

// waves per chain block: the map of a flat or varint layout is built by four
// (one-wave blocks were bound by it: 31 MB screen-defeating 3.96 ms at 256
// blocks, 2.59 at 768); the nested walker keeps its stack per lane in LDS, so
// one wave per block
template <int NS>
constexpr uint32_t kChainWaves = NS <= -2 ? 1u : 4u;

// the path ends before tile u + 1: every later tile's entry word is kEntTerm
// (one wave). SPK_CHAIN_TERM1: each word is written once -- the range past
// what an earlier end already covered (term_from) -- not once per tile past
// the end (the bytes after a message: thousands of tiles, each rewriting all
// the words after it)
__device__ __forceinline__ void chain_term_after(uint64_t *ent, FCtl *fc, uint64_t u, uint64_t nt,
                                                 uint32_t lane) {
  uint64_t hi = nt;
  if (SPK_CHAIN_TERM1) {
    uint64_t old = 0;
    if (lane == 0) old = atomicMin(&fc->term_from, (unsigned long long)(u + 1));
    old = __shfl(old, 0);
    hi = old < nt ? old : nt;
  }
  for (uint64_t v = u + 1 + lane; v < hi; v += 64)
    __hip_atomic_store(&ent[v], kEntTerm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NS>
__global__ __launch_bounds__(64 * kChainWaves<NS>) void vec_tile_chain(
    DecArgs a, WalkProg P, const uint8_t *__restrict__ wire, uint8_t *__restrict__ ws,
    TileBufs TB, uint32_t last_pass) {
  constexpr uint32_t kNT = 64 * kChainWaves<NS>;
  __shared__ v4u_t win_s[win_slots(kTileVec)];
  __shared__ uint16_t nxt[kTileBytes];
  __shared__ uint64_t tile_s, red_s[kChainWaves<NS>];
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const bool w0 = tid < 64;
  if (!vec_live(c)) return;  // (block-uniform)
  const uint64_t nt = TB.ntiles, gstride = (uint64_t)gridDim.x * kNT;
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  const uint64_t nb = (nt + kTSeg - 1) / kTSeg;
  if (!fc->broken[last_pass]) {
    // the passes left nothing: every tile's contribution and the tile scan's
    // segment sums (no tscan_reduce launch)
    for (uint64_t seg = blockIdx.x; seg < nb; seg += gridDim.x)
      tscan_segment<kNT, true>(TB, fc, seg, nb, nsp, red_s);
    return;
  }
  uint64_t *ent = TB.ent;
  // ---- the chain's first tile f0: found by the first block to arrive (it
  // runs, so the others may wait for it), which also clears the entry words ----
  if (tid == 0) tile_s = atomicAdd(&fc->chain_arrive, 1ull);
  __syncthreads();
  if (tile_s == 0) {
    uint64_t m = ~0ull;
    for (uint64_t t = tid; t < nt; t += kNT) {
      bool bad;
      tile_sel_now(TB, fc, t, &bad);
      if (bad && t < m) m = t;
    }
    m = block_min_u64<kChainWaves<NS>>(m, red_s);
    for (uint64_t t = m + tid; t < nt; t += kNT)
      __hip_atomic_store(&ent[t], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the records of the tiles before the chain (as the passes selected
    // them): the chain's running count starts there
    uint64_t pre = 0;
    for (uint64_t t = tid; t < m && t < nt; t += kNT) {
      bool bad;
      const int32_t sel = tile_sel_now(TB, fc, t, &bad);
      if (sel >= 0) pre += TB.fn[t * kFnWords + 2 + sel * kAltWords + 1];
    }
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_down(pre, o);
    if (lane == 0 && pre) atomicAdd(&fc->chain_cnt, (unsigned long long)pre);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(&fc->chain_ready, (m < nt ? m : nt) + 1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    tile_s = m < nt ? m : nt;
  } else if (tid == 0) {
    uint64_t r;
    for (uint32_t i = 0;; ++i) {
      r = __hip_atomic_load(&fc->chain_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (r) break;
      if (i >= kChainSpin) {  // (never expected: a decode error, not a hang)
        r = nt + 1;
        atomicAdd(&fc->unresolved, 1ull);
        atomicMin(&fc->unres_tile, 0ull);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    tile_s = r - 1;
  }
  __syncthreads();
  const uint64_t f0 = tile_s;
  // tiles before f0: selected as the passes left them
  for (uint64_t t = (uint64_t)blockIdx.x * kNT + tid; t < f0; t += gstride) {
    bool bad;
    TB.sel[t] = tile_sel_now(TB, fc, t, &bad);
    tile_contrib(TB, fc, t, nsp);
  }
  __syncthreads();
  if (w0) nt_prologue<NS>(a, lane);
  const uint32_t w = c->w;
  const uint64_t len = a.wire_len, p0 = c->p0;
  for (;;) {
    if (f0 >= nt) break;
    // tiles in order: a block waits only for tiles claimed before its own,
    // and those belong to blocks already running
    if (tid == 0) tile_s = f0 + atomicAdd(&fc->chain_ticket, 1ull);
    __syncthreads();
    const uint64_t u = tile_s;
    if (u >= nt) break;
    // the tiles before this one already hold the message's n records: this
    // and every later tile lie past its end (bytes after a message, e.g. a
    // compatible-member message's version passes, need not be chained
    // through; the count only lags, so a tile is never cut early)
    if (!fc->range && c->n &&
        __hip_atomic_load(&fc->chain_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= c->n) {
      if (w0) {
        if (lane == 0) {
          TB.sel[u] = kSelTerm;
          tile_contrib(TB, fc, u, nsp);
        }
        chain_term_after(ent, fc, u, nt, lane);
      }
      __syncthreads();
      continue;
    }
    const uint64_t ts = p0 + u * kTileBytes;
    if (w0) stage_tile(win_s, wire, len, ts, w, lane);
    __syncthreads();
    const TileView tv = win_view<kTileVec>(win_s, wire, len, ts, w);
    // ---- the next in-tile record start of every byte (the byte itself: its
    // record ends too far past the tile to code; bytes at or past the wire
    // end: the path's end) ----
    for (uint32_t o = tid; o < kTileBytes; o += kNT) {
      const uint64_t x = ts + o;
      uint16_t v = (uint16_t)o;
      if (x < len) {
        const uint64_t L = wlen_rd<NS>(P, tv.rd, len, x, w, nullptr, kK1Reach<NS>);
        v = L == kLenLimit ? kMapUnk
            : !L           ? kMapBad
            : L < kTileBytes - o ? (uint16_t)(o + L)
            : L - (kTileBytes - o) < kMapNear ? (uint16_t)(kMapExit + (o + L - kTileBytes))
                                              : (uint16_t)o;
      }
      nxt[o] = v;
    }
    __syncthreads();
    // ---- pointer jumping: every byte to its path's exit code (or to the
    // start of its last record, when that record's end is too far to code) ----
    for (uint32_t r = 0; r < 32; ++r) {
      int ch = 0;
#pragma unroll 4
      for (uint32_t o = tid; o < kTileBytes; o += kNT) {
        const uint32_t v = nxt[o];
        if (v < kTileBytes && v != o) {
          const uint32_t v2 = nxt[v];
          if (v2 != v) {
            nxt[o] = (uint16_t)v2;
            ch = 1;
          }
        }
      }
      if (!__syncthreads_or(ch)) break;
    }
    if (w0) {
      // this tile's function words (entry alternatives), loaded before the wait
      const uint64_t fnw = lane < 2 + kAlt * kAltWords ? TB.fn[u * kFnWords + lane] : 0;
      // ---- the entry ----
      uint64_t ev = 0;
      if (u == f0) {
        ev = kEntEnter | tile_entry(TB, fc, u);
      } else {
        if (lane == 0) {
          // kPoll polls in flight, a few hundred cycles apart
          constexpr int kPoll = 8;
          uint64_t pv[kPoll];
#pragma unroll
          for (int k = 0; k < kPoll; ++k) {
            pv[k] = __hip_atomic_load(&ent[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_s_sleep(3);
          }
          for (uint32_t i = 0; !ev; ++i) {
#pragma unroll
            for (int k = 0; k < kPoll; ++k) {
              if (pv[k]) {
                ev = pv[k];
                break;
              }
              pv[k] = __hip_atomic_load(&ent[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __builtin_amdgcn_s_sleep(3);
            }
            if (!ev && i >= kChainSpin) {  // (never expected: a decode error, not a hang)
              ev = kEntTerm;
              atomicAdd(&fc->unresolved, 1ull);
              atomicMin(&fc->unres_tile, (unsigned long long)u);
            }
          }
        }
        ev = __shfl(ev, 0);
      }
      const uint64_t kind = ev & ~kEntPos, e = ev & kEntPos;
      if (kind == kEntThru) {  // inside a record spanning the tile
        if (lane == 0) {
          tile_pass_through(TB, u, e, nsp);
          const uint64_t k = tile_contrib(TB, fc, u, nsp);
          if (k) atomicAdd(&fc->chain_cnt, (unsigned long long)k);
          atomicAdd(&fc->seq, 1ull);
        }
      } else if (kind == kEntTerm) {  // past the path's end
        if (lane == 0) {
          TB.sel[u] = kSelTerm;
          tile_contrib(TB, fc, u, nsp);
        }
      } else {
        // ---- entered at e: the exit X ----
        uint64_t X;
        bool redo = false;
        if (e >= ts + kTileBytes) {  // (f0 only: its entry lies past it)
          if (lane == 0) tile_pass_through(TB, u, e, nsp);
          X = e;
        } else {
          const uint32_t nalt = (uint32_t)__shfl(fnw, 1);
          const uint32_t ai = (lane - 2) / kAltWords;
          const bool hit = lane >= 2 && lane < 2 + kAlt * kAltWords &&
                           (lane - 2) % kAltWords == 0 && ai < nalt && fnw == e;
          const uint64_t hm = __ballot(hit);
          const uint64_t fn0 = __shfl(fnw, 0);
          if (hm && fn0 != kNoPos) {  // one of its own alternatives
            if (lane == 0) TB.sel[u] = (int32_t)(((uint32_t)__builtin_ctzll(hm) - 2) / kAltWords);
            X = fn0;
          } else {
            // X from the map; kNoPos: from the re-resolution below (a nested
            // walk the map gave up on, the wire's end inside this tile, or an
            // entry before it: a tile past the wire's end)
            redo = true;
            X = kNoPos;
            if (e >= ts) {
              uint32_t r = nxt[e - ts];
              while (r < kTileBytes && nxt[r] != r) r = nxt[r];  // (jumping converged: no steps)
              if (r == kMapBad) {
                X = kTermPos;
              } else if (r >= kMapExit && r < kMapExit + kMapNear) {
                X = ts + kTileBytes + (r - kMapExit);
              } else if (r < kTileBytes && ts + r < len) {
                uint64_t L = 0;
                if (lane == 0) L = wlen_rd<NS>(P, tv.rd, len, ts + r, w);
                L = __shfl(L, 0);
                X = L ? ts + r + L : kTermPos;
              }
            }
          }
        }
        // ---- hand-off: the landing tile's entry first, then the tiles between ----
        auto publish = [&](uint64_t Y) {
          // (kNoPos: no exit from this entry -- only in bytes past the
          // message, which need not parse: the path ends here, so that no
          // later tile waits for an entry)
          if (Y == kTermPos || Y == kNoPos) {
            chain_term_after(ent, fc, u, nt, lane);
            return;
          }
          uint64_t l0 = Y >= p0 ? (Y - p0) / kTileBytes : 0;
          if (l0 <= u) {
            if (Y < len) return;  // (no exit: never)
            l0 = u + 1;  // the wire's end: the tile after, if any (past the end), enters there
          }
          const uint64_t l = l0 < nt ? l0 : nt;
          if (lane == 0 && l < nt)
            __hip_atomic_store(&ent[l], kEntEnter | Y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (uint64_t v = u + 1 + lane; v < l; v += 64)
            __hip_atomic_store(&ent[v], kEntThru | Y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        if (X != kNoPos) publish(X);
        if (redo) {
          const uint64_t y = tile_resolve_from<NS>(P, tv, TB, len, w, u, ts, e, lane);
          if (X == kNoPos) publish(y);
          if (lane == 0) {
            atomicAdd(&fc->broken[3], 1ull);
#if SPK_DIAG
            if (X != kNoPos && X < len && y != X) atomicAdd(&fc->diag[0], 1ull);  // map vs walk
#endif
          }
        }
        if (lane == 0) {
          // (its selection and function as this lane wrote them)
          const uint64_t k = tile_contrib(TB, fc, u, nsp);
          if (k) atomicAdd(&fc->chain_cnt, (unsigned long long)k);
          atomicAdd(&fc->seq, 1ull);
        }
      }
    }
    __syncthreads();  // the window, the map and tile_s are reused
  }
  // every tile is final once all blocks are out: the last block out adds up
  // the tile scan's segment sums (the producer / consumer fences of the
  // counter hand-off: every wave's stores drained, then an agent release
  // before the add; the last one acquires before it reads)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tile_s = atomicAdd(&fc->chain_done, 1ull) == gridDim.x - 1 ? 1ull : 0ull;
    if (tile_s) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (tile_s)
    for (uint64_t seg = 0; seg < nb; ++seg) tscan_segment<kNT, false>(TB, fc, seg, nb, nsp, red_s);
}

// exclusive prefix sums of the 1 + nsp contribution columns over the tiles up
// to fc->term_tile; totals -> fc->total / fc->stot (the carry of each block:
// the segment sums before its tiles, added up here from the sums
// vec_tile_chain wrote; the block holding the path's last tile writes the
// totals)
__global__ __launch_bounds__(256) void tscan_apply(uint8_t *__restrict__ ws, TileBufs TB,
                                                   uint32_t ncol) {
  __shared__ uint64_t sh[4], carry_s[1 + kVS];
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  if (!vec_live(c)) return;
  // segments past the one holding the path's last tile: K4 reads no prefix there
  const uint64_t lim = fc->term_tile < TB.ntiles ? fc->term_tile + 1 : TB.ntiles;
  const uint64_t lb = lim ? (lim - 1) / kTScanBlock : 0;
  if (blockIdx.x > lb) return;
  const uint64_t nseg = (TB.ntiles + kTSeg - 1) / kTSeg;
  const uint64_t s0 = (uint64_t)blockIdx.x * (kTScanBlock / kTSeg);  // segments before it
  for (uint32_t col = 0; col < ncol; ++col) {
    const uint64_t *bs = TB.scan + (uint64_t)col * nseg;
    uint64_t before = 0;
    for (uint64_t b = threadIdx.x; b < s0; b += blockDim.x) before += bs[b];
    for (int o = 32; o > 0; o >>= 1) before += __shfl_down(before, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = before;
    __syncthreads();
    if (threadIdx.x == 0) carry_s[col] = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
  }
  const uint64_t b0 = (uint64_t)blockIdx.x * kTScanBlock;
  const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kTScanIPT;
  for (uint32_t col = 0; col < ncol; ++col) {
    uint64_t *io = TB.contrib + (uint64_t)col * TB.ntiles;
    uint64_t v[kTScanIPT], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < kTScanIPT; ++j) {
      v[j] = i0 + j < lim ? io[i0 + j] : 0;
      s += v[j];
    }
    uint64_t tot;
    uint64_t run = carry_s[col] + block_excl_scan(s, &tot, sh);
#pragma unroll
    for (uint32_t j = 0; j < kTScanIPT; ++j) {
      if (i0 + j < TB.ntiles) io[i0 + j] = run;
      run += v[j];
    }
    // the totals: records and heap elements on the path
    if (blockIdx.x == lb && threadIdx.x == 0) {
      if (col == 0)
        fc->total = carry_s[0] + tot;
      else
        fc->stot[col - 1] = carry_s[col] + tot;
    }
  }
}

// ---- K4 ----------------------------------------------------------------------
// kEmitSplit waves per tile, each on kEmitChunks consecutive chunks: half the
// LDS per wave of a whole tile, so twice the waves per CU hide the walks'
// LDS latencies. A later part's first record and heap offsets are the
// tile's selected totals minus what its own and later parts hold.
// Nested layouts (NS <= -2) emit one lane per chunk: with two waves per tile
// half of each wave's lanes had no chunk, so they take one wave per tile
// (SPK_ESPLIT_NT; cm K4 4.68 ms with 2)
#ifndef SPK_ESPLIT_NT
#define SPK_ESPLIT_NT 1
#endif
template <int NS>
constexpr uint32_t kEmitSplit = NS <= -2 ? SPK_ESPLIT_NT : SPK_ESPLIT;
template <int NS>
constexpr uint32_t kEmitChunks = 64 / kEmitSplit<NS>;
template <int NS>
constexpr uint32_t kEmitBytes = kEmitChunks<NS> * kTChunk;
template <int NS>
constexpr uint32_t kEmitVec = (kEmitBytes<NS> + kWinExtra) / 16;
template <int NS>  // record starts per emission pass (the nested path keeps none)
constexpr uint32_t kEmitTab = NS <= -2 ? 1u : kTab / kEmitSplit<NS>;
constexpr uint16_t kTabFar = 0xFFFFu;  // a table end past the window

// DEFER: spans of kWaveCopy bytes or more in groups that leave the window
// are copied by the whole wave (wave_copy_deferred). The launch takes it when
// the caller's records average kWaveCopy wire bytes or more (wire_len /
// rec_cap): its registers cost K4 a wave per SIMD (C3 K4 0.304 -> 0.326 ms),
// which messages of short records need not pay (c3l K4 5.3 -> 2.2 ms).
#ifndef SPK_K4_NT  // K4: bit 0 non-temporal window loads (the wire's last read; round-6
                   // A/B on C3 / C4 / cv: within noise, off)
#define SPK_K4_NT 0
#endif
#ifndef SPK_K4_REV  // K4 takes the tiles last to first
#define SPK_K4_REV 1  // (reversed: K4 first reads the tiles K1 read last; c3 K4 0.306 -> 0.298 ms, c4 0.483 -> 0.476, cv 1.136 -> 1.113, same-box A/B)
#endif
template <int NS, bool DEFER = false>
__global__ __launch_bounds__(64 * kDecWaves) void vec_tile_emit(DecArgs a, WalkProg P,
                                                                const uint8_t *__restrict__ wire,
                                                                uint8_t *__restrict__ ws,
                                                                TileBufs TB,
                                                                uint8_t *__restrict__ recs,
                                                                BigQ bq, uint32_t dbg) {
  constexpr uint32_t kEmitSplit = spk::kEmitSplit<NS>, kEmitChunks = spk::kEmitChunks<NS>;
  constexpr uint32_t kEmitBytes = spk::kEmitBytes<NS>, kEmitVec = spk::kEmitVec<NS>;
  constexpr uint32_t kEmitTab = spk::kEmitTab<NS>;
  __shared__ v4u_t win_s[kDecWaves][win_slots(kEmitVec)];
  __shared__ uint16_t tab_s[kDecWaves][kEmitTab + 2];  // (+ the pass's end)
  __shared__ Deferred dfl_s[kDecWaves][DEFER ? 64 : 1];  // spans for the wave
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)(SPK_K4_REV ? gridDim.x - 1 - blockIdx.x : blockIdx.x) * kDecWaves + wv;
  const uint64_t t = gw / kEmitSplit;
  const uint32_t part = (uint32_t)(gw % kEmitSplit);
  if (t >= TB.ntiles || !vec_live(c)) return;
  const uint64_t term_tile = fc->term_tile;
  if (t > term_tile) return;
  const uint64_t n = c->n;
  const uint32_t w = c->w;
  const uint64_t len = a.wire_len, p0 = c->p0;
  const uint32_t nsp = NS > 0 ? (uint32_t)NS : P.ns;
  const uint64_t ts = p0 + t * kTileBytes;
  const uint64_t wb = ts + (uint64_t)part * kEmitBytes;  // this part's window
  const bool own = lane < kEmitChunks;
  const uint32_t ch = part * kEmitChunks + lane;  // tile-relative chunk
  const uint64_t cs = ts + (uint64_t)ch * kTChunk;
  const uint64_t ce = cs + kTChunk < len ? cs + kTChunk : (cs < len ? len : cs);
  const uint64_t g = t * 64 + ch;
  // Everything the part reads from the tile's state is loaded in one round
  // trip, before the window is staged: the selection, the tile's exclusive
  // contributions, every entry alternative of its function (lane k: word k of
  // the alternatives, selected below), its chunks' states and, for a later
  // part, the counts and sums of the chunks after it. (Loaded one after the
  // other, the selection -> alternative -> chunk states -> sums chain cost
  // the wave four memory latencies before any work.)
  const uint64_t tbase = TB.contrib[t];
  const int32_t sel = TB.sel[t];
  uint64_t psum[kVS];
  QFOR(q) psum[q] = TB.contrib[(uint64_t)(1 + q) * TB.ntiles + t];
  const uint64_t fnw = lane < kAlt * kAltWords ? TB.fn[t * kFnWords + 2 + lane] : 0;
  uint64_t used = own ? TB.cused[g] : kNoPos, ex = own ? TB.cex[g] : kNoPos;
  uint32_t cnt = own ? TB.ccnt[g] : 0;
  uint64_t rest = 0, rs[kVS];
  QFOR(q) rs[q] = 0;
  if (part > 0) {  // everything from this part to the tile's end (chunk 0 is not among it)
    for (uint32_t cc = ch; cc < 64; cc += kEmitChunks) {
      rest += TB.ccnt[t * 64 + cc];
      QFOR(q) rs[q] += TB.csum[(uint64_t)q * TB.nchunks + t * 64 + cc];
    }
  }
  nt_prologue<NS>(a, lane);
  const TileView tv = stage_win<kEmitVec, (SPK_K4_NT & 1) != 0>(win_s[wv], wire, len, wb, w, lane);
  const WinReader &rd = tv.rd;
  if (tbase >= n || sel < 0) return;
  // the selected alternative: entry, records, sums (words of lane sel * kAltWords + k)
  const uint32_t sb = (uint32_t)sel * kAltWords;
  const uint64_t alt_e = __shfl(fnw, (int)sb), alt_c = __shfl(fnw, (int)sb + 1);
  // a tile without records (inside a record that spans it) emits nothing,
  // unless the path ends in it (term_pos below)
  if (!alt_c && t != term_tile) return;
  if (dbg & 128) {
    if (lane == 0 && rd.byte(wb) == 0x1234) fc->end_pos = 1;  // keep the staging alive
    return;
  }
  uint64_t qs[NS > 0 ? NS : kVS];  // (nested: chunk 0's heap sums from that entry)
  const bool alt0 = sel > 0 && part == 0 && lane == 0;
  if (alt0) {  // another entry of chunk 0 (same exit)
    const uint64_t T = alt_e;
    uint64_t qe, qt;
    walk_true<NS>(P, rd, len, w, T, ce, qe, cnt, qs, qt);
    used = T;
  }
  const uint64_t pcnt = wave_sum_u64(cnt);  // records starting in this part
  uint64_t base = tbase;
  if (part > 0) {
    base += alt_c - wave_sum_u64(own ? rest : 0);
    QFOR(q) psum[q] += __shfl(fnw, (int)sb + 2 + (int)q) - wave_sum_u64(own ? rs[q] : 0);
  }
  if (own && ex == kTermPos && used != kNoPos && used != kTermPos && t == term_tile) {
    // where the true path ends: past this chunk's records
    uint64_t x = used;
    for (uint32_t r = 0; r < cnt; ++r) {
      uint64_t rc[NS > 0 ? NS : kVS];
      x += wlen_rd<NS>(P, rd, len, x, w, rc);
    }
    atomicMin(&fc->term_pos, (unsigned long long)x);
  }
  if (base >= n) return;
  if constexpr (NS <= -2) {
    // nested records: each lane emits its own chunk's records in order, from
    // the chunk state K1 published (first record index and heap bases by a
    // wave scan of the chunks' counts and heap sums): one walk per record
    // (the interpreter's walks dominate here, not the stores)
    uint64_t tot;
    const uint64_t rofs = wave_excl_scan_u64(cnt, lane, &tot);
    uint64_t hb[kVS], hs[kVS];
    bool fits_all = true;
    QFOR(q) {
      hs[q] = !own ? 0ull : alt0 ? qs[q] : TB.csum[(uint64_t)q * TB.nchunks + g];
      hb[q] = psum[q] + wave_excl_scan_u64(hs[q], lane, &tot);
      if (hb[q] + hs[q] > a.heap_cap[q]) fits_all = false;
    }
    uint64_t idx = base + rofs;
    // every read of the lane's records lies below its chunk's exit (+ the
    // readers' 12-byte word fetches): when that holds for every lane the
    // records are emitted through the LDS-only reader (no store waits on a load)
    const bool live = own && cnt && idx < n && used != kNoPos && used != kTermPos;
    const bool inside = !live || (ex != kTermPos && ex != kNoPos && ex + 16 <= tv.wend);
    if (!live) return;
    uint32_t *const U = nt_used();
    QFOR(q) U[64 * q] = (uint32_t)hb[q];
    auto emit_lane = [&](const auto &R) {
      uint64_t x = used;
      for (uint32_t r = 0; r < cnt && idx < n; ++r, ++idx) {
        const uint64_t x0 = x;
        if (idx < a.rec_cap && fits_all) {
          x = nt_emit_here<nt_level(NS)>(R, x, len, recs + idx * a.L.stride, bq);
        } else {
          // near a capacity: this record's heap use first, written only if it fits
          uint64_t b[kVS], rc[kVS];
          QFOR(q) b[q] = U[64 * q];
          x += wlen_rd<NS>(P, R, len, x, w, rc);
          bool fit = idx < a.rec_cap;
          QFOR(q) fit = fit && b[q] + rc[q] <= a.heap_cap[q];
          QFOR(q) U[64 * q] = (uint32_t)b[q];
          if (fit)
            nt_emit_here<nt_level(NS)>(R, x0, len, recs + idx * a.L.stride, bq);
          else
            QFOR(q) U[64 * q] = (uint32_t)(b[q] + rc[q]);
        }
        if (idx == n - 1) {
          fc->end_pos = x;
          QFOR(q) fc->htot[q] = U[64 * q];
        }
      }
    };
    if (__all(inside))
      emit_lane(rd.lds());
    else
      emit_lane(rd);
    return;
  }
  uint64_t rofs;  // this chunk's first record, part-relative
  {
    uint64_t tot;
    rofs = wave_excl_scan_u64(cnt, lane, &tot);
  }
  uint16_t *tab = tab_s[wv];
  uint64_t carry[NS > 0 ? NS : kVS];
  QFOR(q) carry[q] = psum[q];
  const uint64_t nemit = (n - base < pcnt) ? n - base : pcnt;
  for (uint64_t pass0 = 0; pass0 < nemit; pass0 += kEmitTab) {
    const uint64_t pend = pass0 + kEmitTab < nemit ? pass0 + kEmitTab : nemit;
    // record starts of this pass into the table, and after the last one its
    // end (kTabFar when it lies too far past the window for the fast path)
    if (cnt && rofs < pend && rofs + cnt > pass0) {
      uint64_t x = used;
      for (uint32_t r = 0; r < cnt; ++r) {
        const uint64_t i = rofs + r;
        if (i >= pend) break;
        if (i >= pass0) tab[i - pass0] = (uint16_t)(x - wb);
        uint64_t rc[NS > 0 ? NS : kVS];
        x += wlen_rd<NS>(P, rd, len, x, w, rc);
        if (i + 1 == pend)
          tab[pend - pass0] = x + 16 <= tv.wend ? (uint16_t)(x - wb) : kTabFar;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t nrec = pend - pass0;
    // 64 records at a time: positions from the table, heap offsets by wave
    // scans of their counts, then the record and its payloads written. R: the
    // window reader; the LDS-only one when all 64 records lie inside the
    // window (their stores then never wait on a load)
    auto emit64 = [&](const auto &R, uint64_t i0) -> uint64_t {
      const uint64_t i = i0 + lane;
      const bool act = i < nrec;
      const uint64_t pos = wb + (act ? tab[i] : 0);
      uint64_t rc[kVS] = {};
      uint64_t L = 0;
      if (act) L = wlen_rd<NS>(P, R, len, pos, w, rc);
      uint64_t off[kVS];
      bool fits = true;
      QFOR(q) {
        uint64_t tot;
        off[q] = carry[q] + wave_excl_scan_u64(act ? rc[q] : 0, lane, &tot);
        carry[q] += tot;
        if (off[q] + rc[q] > a.heap_cap[q]) fits = false;
      }
      const uint64_t gr = base + pass0 + i;
      bool dfd = false;
      if (act && gr < a.rec_cap && fits && !(dbg & 64)) {
        if constexpr (NS <= -2)
          nt_emit<nt_level(NS)>(rd, pos, len, recs + gr * a.L.stride, off, bq);
        else if constexpr (!DEFER || std::decay_t<decltype(R)>::kLO)
          emit_record_rd(a.L, R, pos, w, recs + gr * a.L.stride, a.heaps, off, len, bq, dbg);
        else
          dfd = emit_record_rd(a.L, R, pos, w, recs + gr * a.L.stride, a.heaps, off, len, bq,
                               dbg, &dfl_s[wv][lane]);
      }
      if (act && gr == n - 1) {
        fc->end_pos = pos + L;
        QFOR(q) fc->htot[q] = off[q] + rc[q];
      }
      return __ballot(dfd);
    };
    for (uint64_t i0 = 0; i0 < nrec; i0 += 64) {
      if constexpr (NS > -2) {
        // every read of a record lies below its end (+ 12 bytes of the
        // readers' word fetches): the next record's start in the table
        const uint64_t i = i0 + lane;
        const uint32_t e = i < nrec ? tab[i + 1] : 0u;
        const bool inside = i >= nrec || (e != kTabFar && wb + e + 16 <= tv.wend);
        if (__all(inside)) {
          emit64(rd.lds(), i0);
          continue;
        }
      }
      const uint64_t dm = emit64(rd, i0);
      if (DEFER && dm) wave_copy_deferred(rd, dfl_s[wv], dm, lane);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

__device__ void tile_finish(const DecArgs &a, const uint8_t *__restrict__ wire,
                            const uint8_t *__restrict__ ws, spk_dresult_t *res);
// The queued long-span pieces: one block per piece, 16-B aligned stores; the
// last block to finish writes the result (tile_finish: one launch less).
__global__ __launch_bounds__(256) void vec_big_copy(DecArgs a, const uint8_t *__restrict__ wire,
                                                    uint8_t *__restrict__ ws, BigQ bq,
                                                    spk_dresult_t *res) {
  __shared__ uint32_t last_s;
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  const uint64_t nj = fc->njobs < bq.cap ? fc->njobs : bq.cap;
  for (uint64_t j = blockIdx.x; j < nj; j += gridDim.x) {
    const BigJob jb = bq.jobs[j];
    const uint8_t *src = wire + jb.src;
    uint8_t *dst = jb.dst;
    const uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    const uint64_t h = head < jb.n ? head : jb.n;
    if (threadIdx.x < h) dst[threadIdx.x] = src[threadIdx.x];
    const uint64_t nv = (jb.n - h) / 16;
    // 4 loads in flight per thread (a piece is <= 64 KiB: one round), the
    // wire's last read and a write-once destination: non-temporal both ways
    for (uint64_t v0 = threadIdx.x; v0 < nv; v0 += 4 * (uint64_t)blockDim.x) {
      v4u_t x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (v0 + u * blockDim.x < nv)
          x[u] = __builtin_nontemporal_load(
              reinterpret_cast<const v4u_una *>(src + h + 16 * (v0 + u * blockDim.x)));
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (v0 + u * blockDim.x < nv)
          __builtin_nontemporal_store(
              x[u], reinterpret_cast<v4u_t *>(dst + h + 16 * (v0 + u * blockDim.x)));
    }
    for (uint64_t b = h + 16 * nv + threadIdx.x; b < jb.n; b += blockDim.x) dst[b] = src[b];
  }
  // (blocks without a piece take no part: one counter add per busy block)
  const uint64_t busy = nj < gridDim.x ? nj : gridDim.x;
  if (blockIdx.x >= (busy ? busy : 1)) return;
  if (threadIdx.x == 0) last_s = !busy || atomicAdd(&fc->copy_done, 1ull) == busy - 1;
  __syncthreads();
  if (last_s && threadIdx.x < 64) tile_finish(a, wire, ws, res);
}

// spk_decode_shard_index's summary of the range
__global__ void vec_shard_summary(const uint8_t *__restrict__ ws, TileBufs TB, uint32_t nsp,
                                  spk_shard_t *out) {
  if (threadIdx.x != 0) return;
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  const FCtl *fc = reinterpret_cast<const FCtl *>(ws + kWsFCtl);
  spk_shard_t r = {};
  r.errc = c->errc;
  r.width = c->w;
  r.n = fc->nglob;
  r.entry = fc->entry0;
  if (!c->errc && c->n) {
    const bool term = fc->term_tile < TB.ntiles;
    r.exit = term ? ~0ull : (TB.ntiles ? TB.fn[(TB.ntiles - 1) * kFnWords] : fc->entry0);
    r.count = fc->total;
    for (uint32_t q = 0; q < nsp && q < kVS; ++q) r.heap[q] = fc->stot[q];
    r.tiles_repaired = fc->broken[0] + fc->broken[1] + fc->broken[2] + fc->broken[3];
  }
  *out = r;
}

// spk_decode_shard_emit: the range's share of the message's count
__global__ void vec_shard_setn(uint8_t *__restrict__ ws, uint64_t first, uint32_t last,
                               spk_dresult_t *res) {
  if (threadIdx.x != 0) return;
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  FCtl *fc = reinterpret_cast<FCtl *>(ws + kWsFCtl);
  spk_dresult_t r0 = {};
  r0.errc = c->errc;
  r0.width = c->w;
  *res = r0;
  if (c->errc) return;
  c->n = fc->nglob > first ? fc->nglob - first : 0;
  fc->last = last;
  fc->end_pos = 0;
  fc->njobs = 0;
  fc->copy_done = 0;
  for (int k = 0; k < kVS; ++k) fc->htot[k] = 0;
}

// Result: count / consume_len / heap use, or the errc of a short payload
// (no_buffer_space; invalid_buffer for an overlong varint where the path ends).
// One wave (lane 0 writes).
__device__ void tile_finish(const DecArgs &a, const uint8_t *__restrict__ wire,
                            const uint8_t *__restrict__ ws, spk_dresult_t *res) {
  if (a.nested) nt_stage_wave(a.nl, threadIdx.x & 63);
  if (threadIdx.x != 0) return;
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  const FCtl *fc = reinterpret_cast<const FCtl *>(ws + kWsFCtl);
  if (c->errc) return;  // the header errc is already in *res
  spk_dresult_t r = *res;
  uint64_t rep = 0;
  for (int k = 0; k < 4; ++k) rep += fc->broken[k];
  r.tiles_repaired = (uint32_t)(rep < 0xFFFFFFFFull ? rep : 0xFFFFFFFFull);
  r.tiles_sequential = (uint32_t)(fc->seq < 0xFFFFFFFFull ? fc->seq : 0xFFFFFFFFull);
  const uint64_t total = c->n ? (uint64_t)fc->total : 0;
  // an unresolved tile is an internal error unless it starts at or past the
  // end of record n-1: the bytes after a message need not parse as records
  // (the reference stops at its count, struct_pack.hpp:343-357). A shard
  // knows that end only in its emit of the range that holds it (fc->last,
  // c->n = the records from the range's first on, end_pos from K4); any
  // other range's unresolved tile is an error.
  if (fc->unresolved &&
      ((fc->range && !fc->last) || !c->n || total < c->n ||
       c->p0 + fc->unres_tile * (uint64_t)kTileBytes < (uint64_t)fc->end_pos)) {
    r.errc = SPK_ERRC_INTERNAL;
    *res = r;
    return;
  }
  if (fc->range && !fc->last) {  // a middle shard: its records, up to the message's count
    const uint64_t k = total < c->n ? total : c->n;
    r.count = k;
    r.consumed = k == c->n && k ? (uint64_t)fc->end_pos : 0;
    for (uint32_t q = 0; q < a.L.n_spans; ++q) {
      r.heap_used[q] = k == c->n && k ? fc->htot[q] : fc->stot[q];
      if (r.heap_used[q] > a.heap_cap[q] && r.errc == 0) r.errc = SPK_ERRC_CAPACITY;
    }
    if (k > a.rec_cap && r.errc == 0) r.errc = SPK_ERRC_CAPACITY;
    *res = r;
    return;
  }
  if (c->n && total < c->n) {
    r.errc = SPK_ERRC_NO_BUFFER_SPACE;
    if (a.nested && fc->term_pos < a.wire_len) {
      // the errc of the record the path fails at (the exact walk, no quick exits)
      uint64_t p = fc->term_pos;
      const GReader g{wire, c->w};
      const int32_t ec = nt_read<false>(nt_lds(), g, p, a.wire_len, false, nullptr, nullptr, false);
      if (ec) r.errc = ec;
    } else if (a.L.n_var && fc->term_pos < a.wire_len) {
      int32_t ec = SPK_ERRC_NO_BUFFER_SPACE;
      rec_wire_len(a.L, wire, a.wire_len, fc->term_pos, c->w, &ec);
      if (ec == SPK_ERRC_INVALID_BUFFER) r.errc = ec;
    }
    r.count = 0;
    r.consumed = 0;
    for (int k = 0; k < kVS; ++k) r.heap_used[k] = 0;
  } else {
    r.count = c->n;
    const uint64_t end = c->n ? (uint64_t)fc->end_pos : c->p0;
    r.consumed = end > c->data_len ? end : c->data_len;
    if (c->n > a.rec_cap && r.errc == 0) r.errc = SPK_ERRC_CAPACITY;
    for (uint32_t k = 0; k < a.L.n_spans; ++k) {
      r.heap_used[k] = c->n ? fc->htot[k] : 0;
      if (r.heap_used[k] > a.heap_cap[k] && r.errc == 0) r.errc = SPK_ERRC_CAPACITY;
    }
  }
  *res = r;
}
__global__ void vec_tile_finish(DecArgs a, const uint8_t *__restrict__ wire,
                                const uint8_t *__restrict__ ws, spk_dresult_t *res) {
  tile_finish(a, wire, ws, res);  // (launched with one wave)
}

// ===========================================================================
// host launchers
// ===========================================================================
static unsigned grid_for(uint64_t items, uint64_t per_block) {
  uint64_t b = (items + per_block - 1) / per_block;
  return (unsigned)(b ? b : 1);
}

// ---- tile decoder: workspace and launch ---------------------------------------
struct TileWs {
  size_t fn, cused, cex, ccnt, csum, sel, contrib, scan, blist, ent, jobs, nl, end;
  uint64_t ntiles, nchunks, nsb;
};
// ns: span counts per record (flat: SPAN + OPTION members; nested: heaps)
static TileWs tile_ws_layout(uint32_t ns, uint64_t wire_len) {
  TileWs f = {};
  if (!ns) ns = 1;
  f.ntiles = wire_len / kTileBytes + 1;  // the payload starts past the header
  f.nchunks = f.ntiles * 64;
  f.nsb = (f.ntiles + kTSeg - 1) / kTSeg + 1;  // (tile scan segment sums)
  size_t off = kWsScratch;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  f.fn = take(f.ntiles * kFnWords * 8);
  f.cused = take(f.nchunks * 8);
  f.cex = take(f.nchunks * 8);
  f.ccnt = take(f.nchunks * 4);
  f.csum = take(f.nchunks * 8 * ns);
  f.sel = take(f.ntiles * 4);
  f.contrib = take(f.ntiles * 8 * (1 + ns));
  f.scan = take(f.nsb * 8 * (1 + ns));
  f.blist = take(f.ntiles * 4);
  f.ent = take(f.ntiles * 8);
  f.jobs = take(big_jobs_cap(wire_len) * sizeof(BigJob));
  f.nl = take(sizeof(NTLayout));                  // nested layouts: the walker's layout
  f.end = off;
  return f;
}

// Diagnostic bits of the tile kernels (K1 statistics, stages switched off for
// timing, alternative entries): read from SPK_TILE_DBG only in a build with
// -DSPK_DIAG=1 (scripts/ab_dbg.sh); a release build always runs 0.
static uint32_t tile_dbg() {
#if SPK_DIAG
  static const uint32_t v = [] {
    const char *e = getenv("SPK_TILE_DBG");
    return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
  }();
  return v;
#else
  return 0u;
#endif
}

// phase: kTilesAll (one decode), kTilesIndex (spk_decode_shard_index: K1-K3
// over tiles [a.range_t0, +ntiles) and the summary), kTilesEmit
// (spk_decode_shard_emit: K4 + finish over the same tiles)
constexpr int kTilesAll = 0, kTilesIndex = 1, kTilesEmit = 2;
struct ShardCall {
  uint64_t ntiles;     // range tiles (0: the whole message)
  spk_shard_t *summary;
  uint64_t first;      // emit: global index of the range's first record
  uint32_t last;
};

template <int NS>
static hipError_t launch_vec_tiles_ns(const DecArgs &a, const WalkProg &P, const spk_layout *L,
                                      const uint8_t *wire, uint8_t *ws, spk_dresult_t *d_res,
                                      uint8_t *d_recs, hipStream_t s, int phase = kTilesAll,
                                      const ShardCall &sc = ShardCall{}) {
  TileWs f = tile_ws_layout(P.ns, a.wire_len);
  if (phase != kTilesAll) f.ntiles = sc.ntiles < f.ntiles ? sc.ntiles : f.ntiles;
  TileBufs TB;
  TB.fn = reinterpret_cast<uint64_t *>(ws + f.fn);
  TB.cused = reinterpret_cast<uint64_t *>(ws + f.cused);
  TB.cex = reinterpret_cast<uint64_t *>(ws + f.cex);
  TB.ccnt = reinterpret_cast<uint32_t *>(ws + f.ccnt);
  TB.csum = reinterpret_cast<uint64_t *>(ws + f.csum);
  TB.sel = reinterpret_cast<int32_t *>(ws + f.sel);
  TB.contrib = reinterpret_cast<uint64_t *>(ws + f.contrib);
  TB.scan = reinterpret_cast<uint64_t *>(ws + f.scan);
  TB.blist = reinterpret_cast<uint32_t *>(ws + f.blist);
  TB.ent = reinterpret_cast<uint64_t *>(ws + f.ent);
  TB.ntiles = f.ntiles;
  TB.nchunks = f.nchunks;
  const uint32_t nsp = P.ns ? P.ns : 1;
  const unsigned nb = (unsigned)((f.ntiles + kTScanBlock - 1) / kTScanBlock);
  if (phase != kTilesAll && f.ntiles == 0) {  // an empty range: header + summary only
    if (phase == kTilesIndex) {
      SPK_LAUNCH(vec_hdr_kernel, dim3(1), dim3(64), 0, s, a, wire, ws, d_res, 0u, (uint64_t)0);
      SPK_LAUNCH(vec_shard_summary, dim3(1), dim3(64), 0, s, (const uint8_t *)ws, TB, nsp,
                 sc.summary);
    } else {
      SPK_LAUNCH(vec_shard_setn, dim3(1), dim3(64), 0, s, ws, sc.first, sc.last, d_res);
      SPK_LAUNCH(vec_tile_finish, dim3(1), dim3(64), 0, s, a, wire, (const uint8_t *)ws, d_res);
    }
    return hipGetLastError();
  }
  if (phase != kTilesEmit) {
  if (NS > -2 && SPK_SCAP)  // (the header, then K1's speculation caps)
    SPK_LAUNCH(vec_hdr_sample<NS <= -2 ? 0 : NS>, dim3(1), dim3(64), 0, s, a, P, wire, ws, d_res);
  else
    SPK_LAUNCH(vec_hdr_kernel, dim3(1), dim3(64), 0, s, a, wire, ws, d_res, 0u, (uint64_t)0);
  SPK_LAUNCH(vec_tile_spec<NS>, dim3(grid_for(f.ntiles, kDecWaves)), dim3(64 * kDecWaves), 0, s,
             a, P, wire, (const uint8_t *)ws, TB, tile_dbg());
  if (tile_dbg() & 8192) return hipGetLastError();  // (A/B timing of K1 alone)
  if (phase == kTilesIndex) SPK_LAUNCH(vec_range_entry, dim3(1), dim3(64), 0, s, ws, TB);
  for (uint32_t pass = 0; pass < kPickPasses; ++pass) {
    SPK_LAUNCH(vec_tile_pick, dim3(grid_for(f.ntiles, 256)), dim3(256), 0, s, ws, TB, nsp, pass);
    SPK_LAUNCH(vec_tile_repair<NS>, dim3(kRepairGrid), dim3(64), 0, s, a, P, wire, ws, TB, pass);
  }
  SPK_LAUNCH(vec_tile_chain<NS>, dim3(kChainGrid), dim3(64 * kChainWaves<NS>), 0, s, a, P, wire,
             ws, TB, kPickPasses - 1);
  SPK_LAUNCH(tscan_apply, dim3(nb), dim3(256), 0, s, ws, TB, 1 + nsp);
  }
  if (phase == kTilesIndex) {
    SPK_LAUNCH(vec_shard_summary, dim3(1), dim3(64), 0, s, (const uint8_t *)ws, TB, nsp,
               sc.summary);
    return hipGetLastError();
  }
  if (phase == kTilesEmit)
    SPK_LAUNCH(vec_shard_setn, dim3(1), dim3(64), 0, s, ws, sc.first, sc.last, d_res);
  BigQ bq;
  bq.jobs = reinterpret_cast<BigJob *>(ws + f.jobs);
  bq.n = &reinterpret_cast<FCtl *>(ws + kWsFCtl)->njobs;
  bq.cap = big_jobs_cap(a.wire_len);
  if (NS > -2 && a.rec_cap && a.wire_len / a.rec_cap >= kWaveCopy)
    SPK_LAUNCH((vec_tile_emit<NS, (NS > -2)>), dim3(grid_for(f.ntiles * kEmitSplit<NS>, kDecWaves)),
               dim3(64 * kDecWaves), 0, s, a, P, wire, ws, TB, d_recs, bq, tile_dbg());
  else
    SPK_LAUNCH(vec_tile_emit<NS>, dim3(grid_for(f.ntiles * kEmitSplit<NS>, kDecWaves)),
               dim3(64 * kDecWaves), 0, s, a, P, wire, ws, TB, d_recs, bq, tile_dbg());
  if (P.ns) {
    const uint64_t gb = bq.cap < 2048 ? bq.cap : 2048;
    SPK_LAUNCH(vec_big_copy, dim3((unsigned)gb), dim3(256), 0, s, a, wire, ws, bq, d_res);
  } else {
    SPK_LAUNCH(vec_tile_finish, dim3(1), dim3(64), 0, s, a, wire, (const uint8_t *)ws, d_res);
  }
  return hipGetLastError();
}

static int nested_args(const spk_layout *L, uint64_t wire_len, uint64_t rec_cap,
                       void *const *d_heaps, const uint64_t *heap_caps, uint8_t *ws,
                       hipStream_t s, DecArgs &a, WalkProg &P);
hipError_t launch_var_shard(const spk_layout *L, int phase, const void *d_wire, uint64_t wire_len,
                            uint64_t tile_lo, uint64_t tile_hi, uint64_t entry,
                            spk_shard_t *d_summary, uint64_t first, uint32_t last, void *d_recs,
                            uint64_t rec_cap, void *const *d_heaps, const uint64_t *heap_caps,
                            spk_dresult_t *d_res, void *d_ws, hipStream_t s) {
  DecArgs a = {};
  WalkProg P;
  bool nested = false;
  int lvl = 0;
  if (layout_nested(L)) {  // nested layouts: the interpreter walker (var_nested_tile_ok)
    nested = true;
    lvl = nested_args(L, wire_len, rec_cap, d_heaps, heap_caps, (uint8_t *)d_ws, s, a, P);
  } else {
    a.L = make_klayout(L);
    a.fmt = L->fmt_vector;
    a.wire_len = wire_len;
    a.rec_cap = rec_cap;
    for (uint32_t k = 0; k < a.L.n_spans; ++k) {
      a.heaps[k] = d_heaps ? (uint8_t *)d_heaps[k] : nullptr;
      a.heap_cap[k] = heap_caps ? heap_caps[k] : 0;
    }
    P = make_walkprog(L);
  }
  a.range = 1;
  a.range_t0 = tile_lo;
  a.range_entry = entry == ~0ull ? kNoPos : entry;
  ShardCall sc;
  sc.ntiles = tile_hi > tile_lo ? tile_hi - tile_lo : 0;
  sc.summary = d_summary;
  sc.first = first;
  sc.last = last;
  const int ph = phase == 0 ? kTilesIndex : kTilesEmit;
  const uint8_t *wire = (const uint8_t *)d_wire;
  uint8_t *ws = (uint8_t *)d_ws, *r = (uint8_t *)d_recs;
  if (nested && lvl == 2) return launch_vec_tiles_ns<-4>(a, P, L, wire, ws, d_res, r, s, ph, sc);
  if (nested && lvl == 1) return launch_vec_tiles_ns<-3>(a, P, L, wire, ws, d_res, r, s, ph, sc);
  if (nested) return launch_vec_tiles_ns<-2>(a, P, L, wire, ws, d_res, r, s, ph, sc);
  if (P.nv) return launch_vec_tiles_ns<-1>(a, P, L, wire, ws, d_res, r, s, ph, sc);
  if (P.ns == 1) return launch_vec_tiles_ns<1>(a, P, L, wire, ws, d_res, r, s, ph, sc);
  if (P.ns == 2) return launch_vec_tiles_ns<2>(a, P, L, wire, ws, d_res, r, s, ph, sc);
  return launch_vec_tiles_ns<0>(a, P, L, wire, ws, d_res, r, s, ph, sc);
}


// ---- nested layouts on the tile decoder -------------------------------------------
static NTLayout make_ntlayout(const NLayout &N, void *const *heaps) {
  NTLayout t = {};
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    t.ops[i] = N.ops[i];
    t.heap[i] = N.heap[i];
    t.end[i] = N.end[i];
    if (N.ops[i].kind == SPK_OP_VARIANT || N.ops[i].kind == SPK_OP_OPTGROUP) t.groups = 1;
  }
  t.n_ops = N.n_ops;
  t.n_heaps = N.n_heaps;
  t.fv_cnt = N.fv_cnt;
  t.fv_has64 = N.fv_has64;
  t.fv_bits = N.fv_bits;
  for (uint32_t k = 0; k < N.n_heaps && k < kVS; ++k) t.heaps[k] = heaps ? (uint8_t *)heaps[k] : nullptr;
  // the walk program, when every op is COPY / SPAN / OPTION / ARRAY (+ END):
  // COPYs fold into the next instruction's fixed bytes (or the tail)
  uint32_t n = 0, open[SPK_MAX_DEPTH + 1], d = 0;
  uint64_t fix = 0;
  bool ok = !N.fv_cnt;
  // an open WP_GRP: its instruction and its END op (~0u: none)
  uint32_t grp_ins = 0, grp_end = ~0u;
  auto ospan_at = [&](uint32_t i) {  // a one-SPAN optional / compatible group at op i
    return N.ops[i].kind == SPK_OP_OPTGROUP && N.ops[i].size == 1 && i + 2 < N.n_ops &&
           N.ops[i + 1].kind == SPK_OP_SPAN && N.ops[i + 2].kind == SPK_OP_END &&
           N.end[i] == i + 2 && N.ops[i + 1].size < (1u << 24);
  };
  for (uint32_t i = 0; i < N.n_ops && ok; ++i) {
    const spk_op &op = N.ops[i];
    if (grp_end != ~0u && i == grp_end) {  // the group's END: its members end here
      t.wp[grp_ins].x |= n << 8;
      grp_end = ~0u;
      continue;
    }
    if (op.kind == SPK_OP_COPY) {
      if (grp_end != ~0u) {  // inside a group: an instruction of its own (exact drop point)
        t.wp[n] = make_uint2(WP_CPY, op.size);
        ++n;
        continue;
      }
      fix += op.size;
      continue;
    }
    if (op.kind == SPK_OP_OPTGROUP && op.size == 1 && !ospan_at(i) && grp_end == ~0u && !d) {
      // WP_GRP: members COPY / SPAN / OPTION / one-SPAN groups only
      bool simple_members = true;
      for (uint32_t k = i + 1; k < N.end[i] && simple_members;) {
        const uint32_t mk = N.ops[k].kind;
        if (mk == SPK_OP_COPY || mk == SPK_OP_OPTION ||
            (mk == SPK_OP_SPAN && N.ops[k].size < (1u << 24))) {
          ++k;
        } else if (ospan_at(k)) {
          k += 3;
        } else {
          simple_members = false;
        }
      }
      if (simple_members) {
        if (fix >= (1ull << 32)) ok = false;
        t.wp[n] = make_uint2(WP_GRP, (uint32_t)fix);  // (the exit patched at its END)
        fix = 0;
        grp_ins = n++;
        grp_end = N.end[i];
        continue;
      }
    }
    uint32_t x;
    if ((op.kind == SPK_OP_SPAN || op.kind == SPK_OP_OPTION) && op.size < (1u << 24)) {
      x = (op.kind == SPK_OP_SPAN ? WP_SPAN : WP_OPT) | ((uint32_t)N.heap[i] << 3) |
          ((op.size ? op.size : 1u) << 8);
    } else if (op.kind == SPK_OP_ARRAY && d < SPK_MAX_DEPTH) {
      open[d++] = n;
      x = WP_ARR | ((uint32_t)N.heap[i] << 3);
    } else if (ospan_at(i)) {
      x = WP_OSPAN | ((uint32_t)N.heap[i + 1] << 3) |
          ((N.ops[i + 1].size ? N.ops[i + 1].size : 1u) << 8);
      i += 2;  // (the group's SPAN and END are this instruction)
    } else if (op.kind == SPK_OP_END && d) {
      x = WP_END;
      --d;
    } else {
      ok = false;
      break;
    }
    if (fix >= (1ull << 32)) ok = false;
    t.wp[n] = make_uint2(x, (uint32_t)fix);
    fix = 0;
    ++n;
    if ((x & 7u) == WP_END) t.wp[open[d]].x |= n << 8;  // the loop's exit
  }
  t.wp_n = ok && !d && grp_end == ~0u && fix < (1ull << 32) ? n : 0;
  t.wp_tail = (uint32_t)fix;
  return t;
}
// the tile pipeline's walk program for a nested layout: heap use as the span
// sums; candidate starts screened on the first count (NLayout::scr_off)
static WalkProg make_walkprog_nested(const NLayout &N) {
  WalkProg p = {};
  p.ns = N.n_heaps;
  if (N.scr_off != ~0u) {
    p.skip[0] = N.scr_off;
    p.c0max = kPlaus > N.scr_off ? (kPlaus - N.scr_off) / (N.scr_esz ? N.scr_esz : 1) : 0;
    // the op after the first count: a SPAN whose payload is followed (after
    // COPYs) by another SPAN / ARRAY count
    uint32_t i = 0, fix = 0;
    while (i < N.n_ops && N.ops[i].kind == SPK_OP_COPY) ++i;
    if (SPK_NT_SCR2 && i < N.n_ops && N.ops[i].kind == SPK_OP_SPAN) {
      uint32_t j = i + 1;
      while (j < N.n_ops && N.ops[j].kind == SPK_OP_COPY) fix += N.ops[j++].size;
      if (j < N.n_ops && (N.ops[j].kind == SPK_OP_SPAN || N.ops[j].kind == SPK_OP_ARRAY)) {
        p.scr2 = 1;
        p.esz0 = N.ops[i].size;
        p.s2skip = fix;
        p.c1max = kPlaus / (N.ops[j].kind == SPK_OP_SPAN && N.ops[j].size ? N.ops[j].size : 1);
      }
    }
  } else {
    p.pf_all = 1;
    // a record opening (after fixed bytes) with an optional / expected group
    // or an OPTION: K1 screens candidate starts on that has_value byte
    uint32_t i = 0, pre = 0;
    while (i < N.n_ops && N.ops[i].kind == SPK_OP_COPY) pre += N.ops[i++].size;
    if (i < N.n_ops && !N.fv_cnt &&
        (N.ops[i].kind == SPK_OP_OPTGROUP || N.ops[i].kind == SPK_OP_OPTION)) {
      p.hscr = 1;
      p.skip[0] = pre;
    }
  }
  p.rounds = kRounds;
  return p;
}
__global__ void nt_put(NTLayout t, uint8_t *dst) {
  const uint32_t *src = reinterpret_cast<const uint32_t *>(&t);
  for (uint32_t k = threadIdx.x; k < sizeof(NTLayout) / 4; k += blockDim.x)
    reinterpret_cast<uint32_t *>(dst)[k] = src[k];
}

bool var_nested_tile_ok(const spk_layout *L) {
  const NLayout N = make_nlayout(L);
  return !N.n_ranks && N.n_heaps <= kVS;
}
size_t var_nested_tile_ws_bytes(const spk_layout *L, uint64_t wire_len) {
  return tile_ws_layout(make_nlayout(L).n_heaps, wire_len).end + 256;
}

// decode arguments of a nested layout on the tile decoder; its walker layout
// goes into the workspace. Returns whether the walk program applies (NS = -3).
static int nested_args(const spk_layout *L, uint64_t wire_len, uint64_t rec_cap,
                       void *const *d_heaps, const uint64_t *heap_caps, uint8_t *ws,
                       hipStream_t s, DecArgs &a, WalkProg &P) {
  const NLayout N = make_nlayout(L);
  a = DecArgs{};
  a.L.stride = N.stride;
  a.L.n_spans = N.n_heaps;
  a.L.n_var = 1;  // (no minimum-record-size screen in the header kernel)
  a.fmt = L->fmt_vector;
  a.wire_len = wire_len;
  a.rec_cap = rec_cap;
  for (uint32_t k = 0; k < N.n_heaps && k < kVS; ++k) {
    a.heaps[k] = d_heaps ? (uint8_t *)d_heaps[k] : nullptr;
    a.heap_cap[k] = heap_caps ? heap_caps[k] : 0;
  }
  a.nested = 1;
  P = make_walkprog_nested(N);
  const TileWs f = tile_ws_layout(P.ns, wire_len);
  a.nl = ws + f.nl;
  const NTLayout t = make_ntlayout(N, d_heaps);
  SPK_LAUNCH(nt_put, dim3(1), dim3(256), 0, s, t, ws + f.nl);
  if (!t.wp_n) return 0;  // the interpreter (NS = -2)
  for (uint32_t k = 0; k < t.wp_n; ++k) {
    const uint32_t o = t.wp[k].x & 7u;
    if (o == WP_OSPAN || o == WP_GRP || o == WP_CPY) return 2;  // NS = -4
  }
  return 1;                                      // NS = -3
}

hipError_t launch_var_nested_decode(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                                    void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                                    const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                                    hipStream_t s, uint32_t body_w, uint64_t body_n) {
  DecArgs a;
  WalkProg P;
  uint8_t *ws = (uint8_t *)d_ws;
  const int lvl = nested_args(L, wire_len, rec_cap, d_heaps, heap_caps, ws, s, a, P);
  a.body_w = body_w;
  a.body_n = body_n;
  // NS = -3 / -4: every walk runs the walk program; -2: the interpreter
  const uint8_t *wire = (const uint8_t *)d_wire;
  if (lvl == 2) return launch_vec_tiles_ns<-4>(a, P, L, wire, ws, d_res, (uint8_t *)d_recs, s);
  if (lvl == 1) return launch_vec_tiles_ns<-3>(a, P, L, wire, ws, d_res, (uint8_t *)d_recs, s);
  return launch_vec_tiles_ns<-2>(a, P, L, wire, ws, d_res, (uint8_t *)d_recs, s);
}

// ---- compatible members, VECTOR mode, on the tile decoder --------------------------
// unpacker.hpp:292-366,1354-1376: the main pass reads every record without its
// compatible members; then, per version rank in ascending order, a pass reads
// [has:1][U if has] of that rank's members of every record (packer.hpp:66-78,
// 453-461 writes them so). Each pass is a record stream of its own: a derived
// layout (the main one without the members; a rank's of its members, COMPAT
// as OPTION and CGROUP as OPTGROUP, which read alike: a value that does not
// fit reads as present and zero, a group's errc is dropped with the rest of
// the group zeroed) runs the whole tile pipeline, its start and record count
// chained on the device from the previous pass (DecArgs::chain). The
// reference's data-length rule (a has byte at or past the header's length
// ends every pass, no error) is taken exactly in the clean cases: a pass that
// starts at or past the length is skipped and its members read as absent (an
// older writer), and a pass that ends at or before it never met it. Anything
// else -- an error, a capacity overflow, a pass running past the length --
// sets CompatCtl::serial, and the one-lane walk that spk_nested.hip enqueues
// behind it on that flag decodes the whole message instead.
struct CompatSplit {
  spk_layout L;
  uint32_t nh;
  uint8_t hmap[SPK_MAX_SPANS];  // the derived layout's heap j -> the layout's heap
};
// rank < 0: the main pass's layout; else the version pass of that rank
static CompatSplit compat_split(const spk_layout *L, const NLayout &N, int rank) {
  CompatSplit c = {};
  c.L = *L;
  c.L.n_ops = 0;
  auto push = [&](spk_op op, uint32_t i) {
    c.L.ops[c.L.n_ops++] = op;
    if (op_has_heap(op.kind)) c.hmap[c.nh++] = N.heap[i];
  };
  for (uint32_t i = 0; i < L->n_ops;) {
    const spk_op op = L->ops[i];
    const uint32_t k = SPK_OP_KIND(op.kind);
    if (k != SPK_OP_COMPAT && k != SPK_OP_CGROUP) {
      if (rank < 0) push(op, i);
      ++i;
      continue;
    }
    const uint32_t last = k == SPK_OP_CGROUP ? N.end[i] : i;  // a CGROUP: through its END
    if (rank >= 0 && N.crank[i] == (uint32_t)rank) {
      spk_op o = op;
      if (k == SPK_OP_COMPAT) {
        o.kind = SPK_OP_OPTION;
      } else {
        o.kind = SPK_OP_OPTGROUP;
        o.size = 1;
        o.aux = 0;
      }
      push(o, i);
      for (uint32_t j = i + 1; j <= last; ++j) push(L->ops[j], j);
    }
    i = last + 1;
  }
  return c;
}

// a derived layout the tile pipeline takes
static bool tiles_layout_ok(const spk_layout *L) {
  uint32_t h = 0, v = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const uint32_t k = SPK_OP_KIND(L->ops[i].kind);
    h += op_has_heap(k);
    v += k == SPK_OP_VARINT || k == SPK_OP_FVAR || k == SPK_OP_VARIANT || k == SPK_OP_OPTGROUP;
  }
  if (!h && !v) return false;  // (fixed-size records: never a non-trivial layout's pass)
  return layout_nested(L) ? var_nested_tile_ok(L) : true;
}
static size_t tiles_ws_bytes(const spk_layout *L, uint64_t wire_len) {
  if (layout_nested(L)) return var_nested_tile_ws_bytes(L, wire_len);
  uint32_t ns = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i)
    ns += L->ops[i].kind == SPK_OP_SPAN || L->ops[i].kind == SPK_OP_OPTION;
  return tile_ws_layout(ns, wire_len).end + 256;
}
// one VECTOR pass of a derived layout on the tile pipeline
static hipError_t tiles_decode(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                               void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                               const uint64_t *heap_caps, spk_dresult_t *d_res, uint8_t *ws,
                               hipStream_t s, const uint64_t *chain) {
  DecArgs a = {};
  WalkProg P;
  const uint8_t *wire = (const uint8_t *)d_wire;
  uint8_t *r = (uint8_t *)d_recs;
  if (layout_nested(L)) {
    const int lvl = nested_args(L, wire_len, rec_cap, d_heaps, heap_caps, ws, s, a, P);
    a.chain = chain;
    if (lvl == 2) return launch_vec_tiles_ns<-4>(a, P, L, wire, ws, d_res, r, s);
    if (lvl == 1) return launch_vec_tiles_ns<-3>(a, P, L, wire, ws, d_res, r, s);
    return launch_vec_tiles_ns<-2>(a, P, L, wire, ws, d_res, r, s);
  }
  a.L = make_klayout(L);
  a.fmt = L->fmt_vector;
  a.wire_len = wire_len;
  a.rec_cap = rec_cap;
  for (uint32_t k = 0; k < a.L.n_spans; ++k) {
    a.heaps[k] = (uint8_t *)d_heaps[k];
    a.heap_cap[k] = heap_caps[k];
  }
  a.chain = chain;
  P = make_walkprog(L);
  if (P.nv) return launch_vec_tiles_ns<-1>(a, P, L, wire, ws, d_res, r, s);
  if (P.ns == 1) return launch_vec_tiles_ns<1>(a, P, L, wire, ws, d_res, r, s);
  if (P.ns == 2) return launch_vec_tiles_ns<2>(a, P, L, wire, ws, d_res, r, s);
  return launch_vec_tiles_ns<0>(a, P, L, wire, ws, d_res, r, s);
}

bool compat_tiles_ok(const spk_layout *L, uint64_t wire_len) {
  const NLayout N = make_nlayout(L);
  if (!N.n_ranks || wire_len >= (1ull << 32) - 4096) return false;
  for (int rk = -1; rk < (int)N.n_ranks; ++rk) {
    const CompatSplit c = compat_split(L, N, rk);
    if (!tiles_layout_ok(&c.L)) return false;
  }
  return true;
}
size_t compat_tiles_ws_bytes(const spk_layout *L, uint64_t wire_len) {
  const NLayout N = make_nlayout(L);
  size_t b = 0;
  for (int rk = -1; rk < (int)N.n_ranks; ++rk) {
    const CompatSplit c = compat_split(L, N, rk);
    const size_t t = tiles_ws_bytes(&c.L, wire_len);
    b = t > b ? t : b;
  }
  return b;
}

struct HeapMap {
  uint32_t nh;
  uint8_t h[SPK_MAX_SPANS];
};
// after a pass (rank -1: the main one): is it clean, where does the next start
__global__ void compat_link(const uint8_t *ws, CompatCtl *cc, spk_dresult_t *res, HeapMap hm,
                            int rank, uint32_t n_ranks) {
  if (threadIdx.x) return;
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  const FCtl *fc = reinterpret_cast<const FCtl *>(ws + kWsFCtl);
  const uint64_t end = c->n ? (uint64_t)fc->end_pos : c->p0;
  if (rank < 0) {
    cc->serial = 0;
    cc->stop = n_ranks;
    spk_dresult_t r = *res;
    // a record or heap capacity below the message's needs (CAPACITY: the
    // pass walked every record, K4 wrote the ones that fit) is no reason for
    // the one-lane walk: the version passes run on, the errc stays, and a
    // read error of a later pass still takes precedence (the serial walk
    // reports it). A capacity probe (rec_cap 0) of a compatible message took
    // the one-lane walk: ~1.8 s for 200K records.
    if ((r.errc && r.errc != SPK_ERRC_CAPACITY) || c->errc) {
      cc->serial = 1;
      cc->chain[1] = 0;
      return;
    }
    uint64_t hu[SPK_MAX_SPANS] = {};
    for (uint32_t j = 0; j < hm.nh; ++j) hu[hm.h[j]] = r.heap_used[j];
    for (uint32_t k = 0; k < SPK_MAX_SPANS; ++k) r.heap_used[k] = hu[k];
    *res = r;
    cc->end = end;
    cc->chain[0] = end;
    cc->chain[1] = c->n;
    cc->chain[2] = c->w;
    cc->chain[3] = c->data_len;
    if (end >= c->data_len) {  // no version pass was written (or none fits): all absent
      cc->stop = 0;
      cc->chain[1] = 0;
    }
    return;
  }
  if (cc->serial || cc->stop <= (uint32_t)rank) return;  // (the pass read no record)
  const spk_dresult_t p = cc->pres;
  if ((p.errc && p.errc != SPK_ERRC_CAPACITY) || c->errc || end > cc->chain[3]) {
    cc->serial = 1;
    cc->chain[1] = 0;
    return;
  }
  if (p.errc && !res->errc) res->errc = p.errc;  // (a version member's heap overflowed)
  for (uint32_t j = 0; j < hm.nh; ++j) res->heap_used[hm.h[j]] = p.heap_used[j];
  cc->end = end;
  cc->chain[0] = end;
  if (end >= cc->chain[3]) {  // the next pass's first has byte is at or past the length
    cc->stop = (uint32_t)rank + 1;
    cc->chain[1] = 0;
  }
}

// the compatible members of the ranks from CompatCtl::stop on read as absent
// (no pass wrote them): count 0 at element offset 0 (the heap holds none of
// them), a CGROUP's has_value 0 -- what the one-lane walk leaves
struct CompatOps {
  uint32_t n, n_ranks, stride, pad_;
  uint32_t rec_off[SPK_MAX_OPS], aux[SPK_MAX_OPS];
  uint8_t group[SPK_MAX_OPS], rank[SPK_MAX_OPS];
};
__global__ void compat_absent(CompatOps co, const CompatCtl *cc, const spk_dresult_t *res,
                              uint8_t *recs, uint64_t rec_cap) {
  if (cc->serial || cc->stop >= co.n_ranks) return;
  const uint32_t stop = cc->stop;
  const uint64_t n = res->count < rec_cap ? res->count : rec_cap;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t *r = recs + i * co.stride;
    for (uint32_t q = 0; q < co.n; ++q) {
      if (co.rank[q] < stop) continue;
      *reinterpret_cast<uint32_t *>(r + co.rec_off[q]) = 0;
      if (!co.group[q]) *reinterpret_cast<uint64_t *>(r + co.aux[q]) = 0;
    }
  }
}

// the message's result when every pass was clean
__global__ void compat_done(const CompatCtl *cc, spk_dresult_t *res) {
  if (threadIdx.x || cc->serial) return;
  const uint64_t dl = cc->chain[3];
  res->consumed = cc->end > dl ? cc->end : dl;
}

hipError_t launch_compat_tiles(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                               void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                               const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                               size_t ctl_off, hipStream_t s) {
  const NLayout N = make_nlayout(L);
  uint8_t *ws = (uint8_t *)d_ws;
  CompatCtl *cc = reinterpret_cast<CompatCtl *>(ws + ctl_off);
  hipError_t er;
  for (int rk = -1; rk < (int)N.n_ranks; ++rk) {
    const CompatSplit c = compat_split(L, N, rk);
    void *hp[SPK_MAX_SPANS];
    uint64_t hc[SPK_MAX_SPANS];
    HeapMap hm = {};
    hm.nh = c.nh;
    for (uint32_t j = 0; j < c.nh; ++j) {
      hp[j] = d_heaps[c.hmap[j]];
      hc[j] = heap_caps[c.hmap[j]];
      hm.h[j] = c.hmap[j];
    }
    // the main pass writes the message's result; a version pass its own
    if ((er = tiles_decode(&c.L, d_wire, wire_len, d_recs, rec_cap, hp, hc,
                           rk < 0 ? d_res : &cc->pres, ws, s,
                           rk < 0 ? nullptr : reinterpret_cast<const uint64_t *>(cc->chain))) !=
        hipSuccess)
      return er;
    SPK_LAUNCH(compat_link, dim3(1), dim3(64), 0, s, (const uint8_t *)ws, cc, d_res, hm, rk,
               N.n_ranks);
  }
  CompatOps co = {};
  co.n_ranks = N.n_ranks;
  co.stride = L->rec_stride;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const uint32_t k = N.ops[i].kind;
    if (k != SPK_OP_COMPAT && k != SPK_OP_CGROUP) continue;
    co.rec_off[co.n] = N.ops[i].rec_off;
    co.aux[co.n] = N.ops[i].aux;
    co.group[co.n] = k == SPK_OP_CGROUP;
    co.rank[co.n++] = N.crank[i];
  }
  if (rec_cap)
    SPK_LAUNCH(compat_absent, dim3(grid_for(rec_cap, 256) < 4096 ? grid_for(rec_cap, 256) : 4096),
               dim3(256), 0, s, co, (const CompatCtl *)cc, (const spk_dresult_t *)d_res,
               (uint8_t *)d_recs, rec_cap);
  SPK_LAUNCH(compat_done, dim3(1), dim3(64), 0, s, (const CompatCtl *)cc, d_res);
  return hipGetLastError();
}

size_t var_workspace_bytes(const spk_layout *L, int mode, uint64_t n, uint64_t wire_len) {
  size_t enc = kWsScratch + plan_scratch_bytes(grid_for(n, kPlanRPB) + 1) + 256;
  size_t dec_msg = kWsScratch + n * sizeof(MsgState) +
                   (grid_for(n, kThreads) + 1) * kBs * 8 + 256;
  uint32_t ns = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i)
    ns += L->ops[i].kind == SPK_OP_SPAN || L->ops[i].kind == SPK_OP_OPTION;
  const size_t dec_vec = tile_ws_layout(ns, wire_len).end + 256;
  size_t m = enc;
  if (mode == SPK_MODE_MESSAGES) m = m > dec_msg ? m : dec_msg;
  if (mode == SPK_MODE_VECTOR) m = m > dec_vec ? m : dec_vec;
  return m;
}

static VarArgs make_varargs(const spk_layout *L, int mode, uint64_t n,
                            const void *const *heaps) {
  VarArgs a = {};
  a.L = make_klayout(L);
  a.n = n;
  a.mode = mode;
  a.fseq_off = a.flen_off = SPK_FRAME_NONE;
  for (uint32_t k = 0; k < a.L.n_spans && k < kVS; ++k)
    a.heaps[k] = heaps ? (const uint8_t *)heaps[k] : nullptr;
  return a;
}

static MsgHdrTable msg_hdr_table(const spk_layout *L) {
  MsgHdrTable t = {};
  const uint32_t ws_[4] = {1, 2, 4, 8};
  for (int s = 0; s < 4; ++s) t.len[s] = (uint8_t)write_hdr(t.bytes[s], L->fmt_one, ws_[s]);
  return t;
}

hipError_t launch_var_plan(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                           spk_plan_t *d_plan, void *d_ws, size_t ws_bytes,
                           hipStream_t s, const uint64_t *d_n) {
  VarArgs a = make_varargs(L, mode, n, nullptr);
  a.dn = d_n;
  uint8_t *ws = (uint8_t *)d_ws;
  const uint64_t nb = n ? grid_for(n, kPlanRPB) : 1;  // (n = 0: one block of no records)
  FinArgs f;
  f.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  f.n = n;
  f.n_cont = a.L.n_cont;
  f.mode = mode;
  if (SPK_PLAN_SMALL && nb == 1) {
    const MsgHdrTable t = mode == SPK_MODE_MESSAGES ? msg_hdr_table(L) : MsgHdrTable{};
    SPK_LAUNCH(var_plan_small, dim3(1), dim3(kThreads), 0, s, a, f, t, (const uint8_t *)d_recs,
               ws, d_plan);
    (void)ws_bytes;
    return hipGetLastError();
  }
  if (mode == SPK_MODE_MESSAGES) {  // (the per-width header table: messages only)
    const MsgHdrTable t = msg_hdr_table(L);
    SPK_LAUNCH(write_msg_hdrs, dim3(1), dim3(256), 0, s, t, ws);
  }
  const uint8_t *tbl = ws + kWsHdrMsg + 4 * kWsHdrSlot - 8;
  SPK_LAUNCH(var_plan_reduce, dim3(nb), dim3(kThreads), 0, s, a, (const uint8_t *)d_recs, ws,
             tbl);
  SPK_LAUNCH(var_plan_finalize, dim3(1), dim3(kFinThreads), 0, s, f, nb, ws, d_plan);
  (void)ws_bytes;
  return hipGetLastError();
}

hipError_t launch_var_encode(const spk_layout *L, int mode, uint64_t n,
                             const void *d_recs, const void *const *d_heaps,
                             const spk_plan_t *d_plan, void *d_out, uint64_t out_cap,
                             uint64_t *d_offsets, const spk_frame *F, void *d_ws,
                             size_t ws_bytes, hipStream_t s, const SeqEcho *echo,
                             const uint64_t *d_n) {
  VarArgs a = make_varargs(L, mode, n, d_heaps);
  a.dn = d_n;
  if (echo) a.echo = *echo;
  if (F && mode == SPK_MODE_MESSAGES) {
    a.fpre = F->prefix_len;
    a.fseq_off = F->seq_off;
    a.flen_off = F->len_off;
    a.fseq_base = F->seq_base;
    for (uint32_t k = 0; k < F->prefix_len; ++k) a.ftmpl[k] = F->tmpl[k];
  }
  uint8_t *ws = (uint8_t *)d_ws;
  if (n == 0) {
    // header (+ zero count) only; reuse the write kernel with one block
  }
  // window split (var_encode_write): up to 8 blocks per write block while the
  // grid stays under ~8K blocks, i.e. for batches of a few thousand blocks
  const unsigned nb = grid_for(n ? n : 1, kRPB);
  const unsigned ny = nb >= 8192 ? 1u : (8192u / nb < kYSplit ? 8192u / nb : kYSplit);
  SPK_LAUNCH(var_encode_write, dim3(nb, ny), dim3(kThreads), 0,
                     s, a, (const uint8_t *)d_recs, (uint8_t *)d_out, out_cap,
                     (const uint8_t *)ws, d_plan, d_offsets);
  (void)ws_bytes;
  return hipGetLastError();
}

bool var_plan_encode_small_ok(const spk_layout *L, uint64_t n) {
  return SPK_PLAN_SMALL && n >= 1 && n <= kRPB && !layout_nested(L);
}
hipError_t launch_var_plan_encode_small(const spk_layout *L, int mode, uint64_t n,
                                        const void *d_recs, const void *const *d_heaps,
                                        spk_plan_t *d_plan, void *d_out, uint64_t out_cap,
                                        uint64_t *d_offsets, void *d_ws, hipStream_t s) {
  VarArgs a = make_varargs(L, mode, n, d_heaps);
  FinArgs f;
  f.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  f.n = n;
  f.n_cont = a.L.n_cont;
  f.mode = mode;
  const MsgHdrTable t = mode == SPK_MODE_MESSAGES ? msg_hdr_table(L) : MsgHdrTable{};
  SPK_LAUNCH(var_plan_encode_small, dim3(1), dim3(kThreads), 0, s, a, f, t,
             (const uint8_t *)d_recs, (uint8_t *)d_out, out_cap, (uint8_t *)d_ws, d_plan,
             d_offsets);
  return hipGetLastError();
}

// plan override for a sharded body: imposed width, no header
__global__ void body_plan_kernel(spk_plan_t *plan, uint64_t n, uint32_t n_spans,
                                 uint32_t width) {
  if (threadIdx.x != 0) return;
  spk_plan_t p = *plan;
  p.width = width;
  p.header_bytes = 0;
  p.total_bytes = p.var_bytes + n * (uint64_t)n_spans * width;
  *plan = p;
}

hipError_t launch_var_encode_body(const spk_layout *L, uint64_t n, const void *d_recs,
                                  const void *const *d_heaps, uint32_t width, void *d_out,
                                  uint64_t out_cap, void *d_ws, size_t ws_bytes,
                                  hipStream_t s) {
  // the plan lives in the workspace control area for this call
  spk_plan_t *plan = reinterpret_cast<spk_plan_t *>((uint8_t *)d_ws + kWsCtl + 1024);
  hipError_t e = launch_var_plan(L, SPK_MODE_VECTOR, n, d_recs, plan, d_ws, ws_bytes, s);
  if (e != hipSuccess) return e;
  uint32_t ns = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) ns += L->ops[i].kind == SPK_OP_SPAN;  // width-w counts
  SPK_LAUNCH(body_plan_kernel, dim3(1), dim3(64), 0, s, plan, n, ns, width);
  return launch_var_encode(L, SPK_MODE_VECTOR, n, d_recs, d_heaps, plan, d_out, out_cap,
                           nullptr, nullptr, d_ws, ws_bytes, s);
}

hipError_t launch_var_decode(const spk_layout *L, int mode, const void *d_wire,
                             uint64_t wire_len, const uint64_t *d_offsets,
                             uint64_t n_msgs, uint32_t prefix, void *d_recs,
                             uint64_t rec_cap, void *const *d_heaps,
                             const uint64_t *heap_caps, spk_dresult_t *d_res,
                             int32_t *d_errc, void *d_ws, size_t ws_bytes, hipStream_t s,
                             uint32_t body_w, uint64_t body_n, const uint64_t *d_msg_ends,
                             const uint64_t *d_n) {
  DecArgs a = {};
  a.ends = d_msg_ends;
  a.dn = d_n;
  a.prefix = prefix;
  a.body_w = body_w;
  a.body_n = body_n;
  a.L = make_klayout(L);
  a.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  a.wire_len = wire_len;
  a.n_msgs = n_msgs;
  a.rec_cap = rec_cap;
  for (uint32_t k = 0; k < a.L.n_spans; ++k) {
    a.heaps[k] = (uint8_t *)d_heaps[k];
    a.heap_cap[k] = heap_caps[k];
  }
  uint8_t *ws = (uint8_t *)d_ws;
  const uint8_t *wire = (const uint8_t *)d_wire;
  hipError_t e;
  if (mode == SPK_MODE_MESSAGES) {
    if (SPK_MSG_SMALL && n_msgs && n_msgs <= kThreads) {
      SPK_LAUNCH(var_msg_decode_small, dim3(1), dim3(kThreads), 0, s, a, wire, d_offsets, ws,
                 d_errc, (uint8_t *)d_recs, d_res);
      return hipGetLastError();
    }
    if ((e = hipMemsetAsync(d_res, 0, sizeof(spk_dresult_t), s)) != hipSuccess) return e;
    if (n_msgs == 0) return hipSuccess;
    const unsigned nb = grid_for(n_msgs, kThreads);
    SPK_LAUNCH(var_msg_parse, dim3(nb), dim3(kThreads), 0, s, a, wire, d_offsets,
                       ws, d_errc, d_res);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + kWsScratch + sizeof(MsgState) * n_msgs);
    SPK_LAUNCH(var_scan_blocks, dim3(1), dim3(1024), 0, s, (uint64_t)nb,
                       a.L.n_spans, bsum, a, d_res);
    // (a copy split over gridDim.y blocks, as the encode's, measured no faster
    // here with one wave per payload: C5 vector<int> decode 0.682 / 0.686 ms)
    SPK_LAUNCH(var_msg_write, dim3(nb, 1), dim3(kThreads), 0, s, a, wire, d_offsets,
                       (const uint8_t *)ws, (uint8_t *)d_recs, (const spk_dresult_t *)d_res);
    (void)ws_bytes;
    return hipGetLastError();
  }
  // ---- VECTOR ----
  const WalkProg P = make_walkprog(L);
  (void)e;
  (void)ws_bytes;
  // NS = -1: the walkers read varints (kept out of the other instantiations:
  // the inlined LEB128 loops cost registers in the hot walks)
  uint8_t *r = (uint8_t *)d_recs;
  if (P.nv) return launch_vec_tiles_ns<-1>(a, P, L, wire, ws, d_res, r, s);
  if (P.ns == 1) return launch_vec_tiles_ns<1>(a, P, L, wire, ws, d_res, r, s);
  if (P.ns == 2) return launch_vec_tiles_ns<2>(a, P, L, wire, ws, d_res, r, s);
  return launch_vec_tiles_ns<0>(a, P, L, wire, ws, d_res, r, s);
}

}  // namespace spk
