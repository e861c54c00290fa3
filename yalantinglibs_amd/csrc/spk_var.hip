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

namespace spk {

constexpr int kThreads = 256;
constexpr int kIPT = 4;                     // records per thread (encode)
constexpr uint64_t kRPB = kThreads * kIPT;  // records per block (encode)
constexpr uint32_t kWin = 40 * 1024;        // LDS assembly window (bytes)

struct VarArgs {
  KLayout L;
  uint64_t n;
  int mode;
  uint32_t pad_;
  const uint8_t *heaps[SPK_MAX_SPANS];
};

static KLayout make_klayout(const spk_layout *L) {
  KLayout k = {};
  k.stride = L->rec_stride;
  k.n_ops = L->n_ops;
  k.trivial = (L->flags & SPK_LAYOUT_TRIVIAL) ? 1 : 0;
  for (uint32_t i = 0; i < L->n_ops && i < SPK_MAX_OPS; ++i) {
    k.ops[i] = L->ops[i];
    if (L->ops[i].kind == SPK_OP_COPY)
      k.fixed_bytes += L->ops[i].size;
    else
      ++k.n_spans;
  }
  return k;
}

__device__ __forceinline__ uint32_t rec_u32(const uint8_t *rec, uint32_t off) {
  return *reinterpret_cast<const uint32_t *>(rec + off);
}
__device__ __forceinline__ uint64_t rec_u64(const uint8_t *rec, uint32_t off) {
  return *reinterpret_cast<const uint64_t *>(rec + off);
}

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
    }
  }
}

__device__ __forceinline__ uint32_t wlog(uint32_t w) {
  return w == 1 ? 0 : w == 2 ? 1 : w == 4 ? 2 : 3;
}

// ---- block-wide helpers ----------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(v, o);
    if (lane >= (uint32_t)o) v += u;
  }
  return v;
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
struct Partial {
  uint64_t sum;   // VECTOR: sum of w-independent bytes; MESSAGES: message bytes
  uint64_t maxc;  // max element count
};

__global__ __launch_bounds__(kThreads) void var_plan_reduce(
    VarArgs a, const uint8_t *__restrict__ recs, uint8_t *__restrict__ ws,
    const uint8_t *__restrict__ hdrlen_tbl) {
  __shared__ uint64_t sh[kThreads / 64];
  const uint64_t r0 = (uint64_t)blockIdx.x * kRPB;
  uint64_t sum = 0, mx = 0;
  for (int j = 0; j < kIPT; ++j) {
    const uint64_t i = r0 + (uint64_t)j * kThreads + threadIdx.x;  // coalesced
    if (i >= a.n) break;
    uint64_t var, maxc;
    rec_sizes(a.L, recs + i * a.L.stride, var, maxc);
    if (a.mode == SPK_MODE_VECTOR) {
      sum += var;
    } else {
      const uint32_t w = width_of(maxc);
      sum += hdrlen_tbl[wlog(w)] + var + (uint64_t)a.L.n_spans * w;
    }
    mx = maxc > mx ? maxc : mx;
  }
  uint64_t tot;
  block_excl_scan(sum, &tot, sh);
  const uint64_t m = block_max(mx, sh);
  if (threadIdx.x == 0) {
    Partial *p = reinterpret_cast<Partial *>(ws + kWsScratch);
    p[blockIdx.x] = Partial{tot, m};
  }
}

struct FinArgs {
  spk_msgfmt fmt;
  uint64_t n;
  uint64_t nblocks;
  uint32_t n_spans;
  int mode;
};

// one block: exclusive scan of the block partials (in place: .sum becomes the
// block's base), header bytes, plan.
__global__ __launch_bounds__(1024) void var_plan_finalize(FinArgs a,
                                                          uint8_t *__restrict__ ws,
                                                          spk_plan_t *__restrict__ plan) {
  __shared__ uint64_t sh[1024 / 64];
  Partial *p = reinterpret_cast<Partial *>(ws + kWsScratch);
  uint64_t carry = 0, mx = 0;
  for (uint64_t b0 = 0; b0 < a.nblocks; b0 += blockDim.x) {
    const uint64_t b = b0 + threadIdx.x;
    const Partial v = b < a.nblocks ? p[b] : Partial{0, 0};
    uint64_t tot;
    const uint64_t ex = block_excl_scan(v.sum, &tot, sh);
    if (b < a.nblocks) p[b].sum = carry + ex;
    carry += tot;
    mx = v.maxc > mx ? v.maxc : mx;
  }
  mx = block_max(mx, sh);
  if (threadIdx.x != 0) return;
  spk_plan_t r;
  if (a.mode == SPK_MODE_VECTOR) {
    const uint64_t maxc = mx > a.n ? mx : a.n;  // outer vector counts too
    const uint32_t w = width_of(maxc);
    const HdrShape h = hdr_shape(a.fmt.flags, a.fmt.literal_len, w);
    uint8_t *hb = ws + kWsHdrVec;
    const uint32_t len = write_hdr(hb, a.fmt, w);
    for (uint32_t i = 0; i < w; ++i) hb[len + i] = (uint8_t)(a.n >> (8 * i));
    r.total_bytes = len + w + carry + a.n * (uint64_t)a.n_spans * w;
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

// message headers per width for MESSAGES mode (host computes: no data needed)
struct MsgHdrTable {
  uint8_t len[4];
  uint8_t bytes[4][4 + 1 + SPK_MAX_LITERAL + 1];
};

__global__ void write_msg_hdrs(MsgHdrTable t, uint8_t *ws) {
  for (int s = 0; s < 4; ++s)
    for (uint32_t i = threadIdx.x; i < t.len[s]; i += blockDim.x)
      ws[kWsHdrMsg + s * kWsHdrSlot + i] = t.bytes[s][i];
  if (threadIdx.x < 4) ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + threadIdx.x] = t.len[threadIdx.x];
}

// LDS window writer ----------------------------------------------------------
struct Win {
  uint8_t *lds;
  uint64_t lo, hi;  // global byte range currently held [lo, hi)
};

__device__ __forceinline__ void win_put_bytes_global(const Win &W, uint64_t pos,
                                                     const uint8_t *src, uint64_t len) {
  uint64_t a = pos > W.lo ? pos : W.lo;
  uint64_t b = pos + len < W.hi ? pos + len : W.hi;
  for (uint64_t x = a; x < b; ++x) W.lds[x - W.lo] = src[x - pos];
}
__device__ __forceinline__ void win_put_le(const Win &W, uint64_t pos, uint64_t v,
                                           uint32_t w) {
  for (uint32_t i = 0; i < w; ++i) {
    const uint64_t x = pos + i;
    if (x >= W.lo && x < W.hi) W.lds[x - W.lo] = (uint8_t)(v >> (8 * i));
  }
}

// emit one record at global position pos (width w) into the window
__device__ void emit_record(const VarArgs &a, const uint8_t *rec, uint32_t w,
                            uint64_t pos, const Win &W) {
  uint32_t sk = 0;
  for (uint32_t o = 0; o < a.L.n_ops; ++o) {
    const spk_op op = a.L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      win_put_bytes_global(W, pos, rec + op.rec_off, op.size);
      pos += op.size;
    } else {
      const uint64_t c = rec_u32(rec, op.rec_off);
      win_put_le(W, pos, c, w);
      pos += w;
      const uint64_t nb = c * op.size;
      if (nb) {
        const uint8_t *src = a.heaps[sk] + rec_u64(rec, op.aux) * op.size;
        win_put_bytes_global(W, pos, src, nb);
      }
      pos += nb;
      ++sk;
    }
  }
}

__global__ __launch_bounds__(kThreads) void var_encode_write(
    VarArgs a, const uint8_t *__restrict__ recs, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint8_t *__restrict__ ws,
    const spk_plan_t *__restrict__ plan, uint64_t *__restrict__ offs) {
  extern __shared__ __align__(16) uint8_t lds[];
  __shared__ uint64_t sh[kThreads / 64];
  __shared__ uint64_t s_g0, s_tot;
  const uint64_t total = plan->total_bytes;
  if (total > out_cap) return;  // caller reads plan->total_bytes
  const uint32_t w_vec = plan->width;
  const uint32_t hdr_vec = plan->header_bytes;
  const Partial *part = reinterpret_cast<const Partial *>(ws + kWsScratch);
  const uint64_t r0 = (uint64_t)blockIdx.x * kRPB;
  // this thread's records are contiguous: r0 + t*kIPT + j (output contiguity)
  const uint64_t t0 = r0 + (uint64_t)threadIdx.x * kIPT;
  uint64_t sz[kIPT];
  uint32_t wr[kIPT];
  uint64_t tsum = 0;
  for (int j = 0; j < kIPT; ++j) {
    const uint64_t i = t0 + j;
    sz[j] = 0;
    wr[j] = 1;
    if (i < a.n) {
      uint64_t var, maxc;
      rec_sizes(a.L, recs + i * a.L.stride, var, maxc);
      if (a.mode == SPK_MODE_VECTOR) {
        wr[j] = w_vec;
        sz[j] = var + (uint64_t)a.L.n_spans * w_vec;
      } else {
        wr[j] = width_of(maxc);
        sz[j] = ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + wlog(wr[j])] + var +
                (uint64_t)a.L.n_spans * wr[j];
      }
    }
    tsum += sz[j];
  }
  uint64_t btot;
  const uint64_t toff = block_excl_scan(tsum, &btot, sh);
  if (threadIdx.x == 0) {
    s_g0 = a.mode == SPK_MODE_VECTOR
               ? hdr_vec + part[blockIdx.x].sum + r0 * (uint64_t)a.L.n_spans * w_vec
               : part[blockIdx.x].sum;
    s_tot = btot;
  }
  __syncthreads();
  const uint64_t g0 = s_g0, g1 = s_g0 + s_tot;
  if (a.mode == SPK_MODE_VECTOR && blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < hdr_vec; i += blockDim.x) out[i] = ws[kWsHdrVec + i];
  if (a.mode == SPK_MODE_MESSAGES && offs) {
    uint64_t p = g0 + toff;
    for (int j = 0; j < kIPT; ++j) {
      if (t0 + j < a.n) offs[t0 + j] = p;
      p += sz[j];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) offs[a.n] = total;
  }
  if (g1 == g0) return;
  const uint64_t abase = g0 & ~15ull;
  for (uint64_t wlo = abase; wlo < g1; wlo += kWin) {
    Win W{lds, wlo, wlo + kWin < g1 ? wlo + kWin : g1};
    uint64_t p = g0 + toff;
    if (p < W.hi && p + tsum > W.lo) {
      for (int j = 0; j < kIPT; ++j) {
        const uint64_t i = t0 + j;
        if (i >= a.n) break;
        if (p < W.hi && p + sz[j] > W.lo) {
          uint64_t q = p;
          if (a.mode == SPK_MODE_MESSAGES) {
            const uint32_t s = wlog(wr[j]);
            const uint32_t hl = ws[kWsHdrMsg + 4 * kWsHdrSlot - 8 + s];
            win_put_bytes_global(W, q, ws + kWsHdrMsg + s * kWsHdrSlot, hl);
            q += hl;
          }
          emit_record(a, recs + i * a.L.stride, wr[j], q, W);
        }
        p += sz[j];
      }
    }
    __syncthreads();
    // flush [max(W.lo,g0), W.hi): aligned 16-B chunks, bytes at the edges
    for (uint64_t c = W.lo + (uint64_t)threadIdx.x * 16; c < W.hi; c += kThreads * 16) {
      const uint64_t lo = c > g0 ? c : g0;
      const uint64_t hi = c + 16 < W.hi ? c + 16 : W.hi;
      if (lo == c && hi == c + 16) {
        *reinterpret_cast<uint4 *>(out + c) =
            *reinterpret_cast<const uint4 *>(lds + (c - W.lo));
      } else {
        for (uint64_t x = lo; x < hi; ++x) out[x] = lds[x - W.lo];
      }
    }
    __syncthreads();
  }
}

// ===========================================================================
// DECODE — shared record walker over the wire
// ===========================================================================

// Size of the record starting at `pos` (absolute), reading counts from
// `wire` (length len). Returns 0 if the record does not fit (incomplete).
__device__ __forceinline__ uint64_t rec_wire_len(const KLayout &L, const uint8_t *wire,
                                                 uint64_t len, uint64_t pos, uint32_t w) {
  const uint64_t p0 = pos;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      pos += op.size;
      if (pos > len) return 0;
    } else {
      if (pos + w > len) return 0;
      const uint64_t c = ld_le(wire + pos, w);
      pos += w;
      if (c) {
        if (op.size > 1 && c > ~0ull / op.size) return 0;
        const uint64_t nb = c * op.size;
        if (nb > len - pos) return 0;
        pos += nb;
      }
    }
  }
  return pos - p0;
}

// Decode the record at `pos` into `rec` (device record) and its heaps.
// heap_off[k] = element offset where this record's span k goes.
__device__ void decode_record(const KLayout &L, const uint8_t *wire, uint64_t pos,
                              uint32_t w, uint8_t *rec, uint8_t *const *heaps,
                              const uint64_t *heap_off) {
  uint32_t sk = 0;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      for (uint32_t b = 0; b < op.size; ++b) rec[op.rec_off + b] = wire[pos + b];
      pos += op.size;
    } else {
      const uint64_t c = ld_le(wire + pos, w);
      pos += w;
      *reinterpret_cast<uint32_t *>(rec + op.rec_off) = (uint32_t)c;
      *reinterpret_cast<uint64_t *>(rec + op.aux) = heap_off[sk];
      const uint64_t nb = c * op.size;
      uint8_t *dst = heaps[sk] + heap_off[sk] * op.size;
      for (uint64_t b = 0; b < nb; ++b) dst[b] = wire[pos + b];
      pos += nb;
      ++sk;
    }
  }
}

// counts of the record at pos (assumes it is complete)
__device__ __forceinline__ void rec_counts(const KLayout &L, const uint8_t *wire,
                                           uint64_t pos, uint32_t w, uint64_t *cnt) {
  uint32_t sk = 0;
  for (uint32_t o = 0; o < L.n_ops; ++o) {
    const spk_op op = L.ops[o];
    if (op.kind == SPK_OP_COPY) {
      pos += op.size;
    } else {
      const uint64_t c = ld_le(wire + pos, w);
      cnt[sk++] = c;
      pos += w + c * op.size;
    }
  }
}

struct DecArgs {
  KLayout L;
  spk_msgfmt fmt;
  uint64_t wire_len;
  uint64_t n_msgs;
  uint64_t rec_cap;
  uint64_t heap_cap[SPK_MAX_SPANS];
  uint8_t *heaps[SPK_MAX_SPANS];
};


// ===========================================================================
// DECODE, SPK_MODE_MESSAGES
// ===========================================================================
// per-message state in workspace: u64 payload_pos (~0 = failed) | width
struct MsgState {
  uint64_t pos;    // absolute payload position, ~0 if the message failed
  uint32_t w;
  int32_t errc;
};

__global__ __launch_bounds__(kThreads) void var_msg_parse(
    DecArgs a, const uint8_t *__restrict__ wire, const uint64_t *__restrict__ offs,
    uint8_t *__restrict__ ws, int32_t *__restrict__ errc_out, spk_dresult_t *res) {
  __shared__ uint64_t sh[kThreads / 64];
  MsgState *st = reinterpret_cast<MsgState *>(ws + kWsScratch);
  uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + kWsScratch +
                                                sizeof(MsgState) * a.n_msgs);
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  uint64_t cnt[SPK_MAX_SPANS] = {};
  uint64_t ok = 0, consumed = 0;
  if (i < a.n_msgs) {
    const uint64_t b = offs[i], e = offs[i + 1];
    MsgState s{~0ull, 1, SPK_ERRC_OK};
    if (e < b || e > a.wire_len) {
      s.errc = SPK_ERRC_NO_BUFFER_SPACE;
    } else {
      uint64_t pos, dl;
      uint32_t w;
      s.errc = parse_hdr(a.fmt, wire + b, e - b, &pos, &w, &dl);
      if (!s.errc) {
        const uint64_t rl = rec_wire_len(a.L, wire + b, e - b, pos, w);
        if (!rl) {
          s.errc = SPK_ERRC_NO_BUFFER_SPACE;
        } else {
          if (i >= a.rec_cap) s.errc = SPK_ERRC_CAPACITY;
          s.pos = b + pos;
          s.w = w;
          rec_counts(a.L, wire, b + pos, w, cnt);
          ok = 1;
          consumed = pos + rl > dl ? pos + rl : dl;
        }
      }
    }
    if (s.errc) {
      s.pos = ~0ull;
      ok = 0;
      consumed = 0;
      for (int k = 0; k < SPK_MAX_SPANS; ++k) cnt[k] = 0;
    }
    st[i] = s;
    if (errc_out) errc_out[i] = s.errc;
    if (s.errc == SPK_ERRC_CAPACITY) atomicExch(&res->errc, SPK_ERRC_CAPACITY);
  }
  for (uint32_t k = 0; k < a.L.n_spans; ++k) {
    uint64_t tot;
    block_excl_scan(cnt[k], &tot, sh);
    if (threadIdx.x == 0) bsum[(uint64_t)blockIdx.x * SPK_MAX_SPANS + k] = tot;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ok += __shfl_down(ok, o);
    consumed += __shfl_down(consumed, o);
  }
  if ((threadIdx.x & 63) == 0 && (ok | consumed)) {
    atomicAdd((unsigned long long *)&res->count, (unsigned long long)ok);
    atomicAdd((unsigned long long *)&res->consumed, (unsigned long long)consumed);
  }
}

// one block: exclusive scan of per-block span totals (in place), heap_used,
// capacity check
__global__ __launch_bounds__(1024) void var_scan_blocks(uint64_t nblocks,
                                                        uint32_t n_spans,
                                                        uint64_t *__restrict__ bsum,
                                                        DecArgs a,
                                                        spk_dresult_t *res) {
  __shared__ uint64_t sh[1024 / 64];
  for (uint32_t k = 0; k < n_spans; ++k) {
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nblocks; b0 += blockDim.x) {
      const uint64_t b = b0 + threadIdx.x;
      const uint64_t v = b < nblocks ? bsum[b * SPK_MAX_SPANS + k] : 0;
      uint64_t tot;
      const uint64_t ex = block_excl_scan(v, &tot, sh);
      if (b < nblocks) bsum[b * SPK_MAX_SPANS + k] = carry + ex;
      carry += tot;
    }
    if (threadIdx.x == 0) {
      res->heap_used[k] = carry;
      if (carry > a.heap_cap[k] && res->errc == 0) res->errc = SPK_ERRC_CAPACITY;
    }
  }
}

__global__ __launch_bounds__(kThreads) void var_msg_write(
    DecArgs a, const uint8_t *__restrict__ wire, const uint8_t *__restrict__ ws,
    uint8_t *__restrict__ recs, const spk_dresult_t *res) {
  __shared__ uint64_t sh[kThreads / 64];
  const MsgState *st = reinterpret_cast<const MsgState *>(ws + kWsScratch);
  const uint64_t *bsum = reinterpret_cast<const uint64_t *>(ws + kWsScratch +
                                                            sizeof(MsgState) * a.n_msgs);
  if (res->errc == SPK_ERRC_CAPACITY) return;  // heaps too small: write nothing
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  MsgState s{~0ull, 1, 1};
  uint64_t cnt[SPK_MAX_SPANS] = {};
  if (i < a.n_msgs) {
    s = st[i];
    if (s.pos != ~0ull) rec_counts(a.L, wire, s.pos, s.w, cnt);
  }
  uint64_t hoff[SPK_MAX_SPANS] = {};
  for (uint32_t k = 0; k < a.L.n_spans; ++k) {
    uint64_t tot;
    hoff[k] = bsum[(uint64_t)blockIdx.x * SPK_MAX_SPANS + k] + block_excl_scan(cnt[k], &tot, sh);
  }
  if (s.pos == ~0ull || s.errc) return;
  decode_record(a.L, wire, s.pos, s.w, recs + i * a.L.stride, a.heaps, hoff);
}

// ===========================================================================
// DECODE, SPK_MODE_VECTOR — chunked transition functions
// ===========================================================================
// The payload is cut into kChunk-byte chunks. For every byte position p of a
// chunk a block computes, fully in parallel, "if a record started at p, where
// would the next one start" (one parse per position, in LDS), then pointer-
// jumps those links in place (one packed 32-bit (next, count) word per
// position, so asynchronous updates keep the invariant) until every position
// knows the first record start at/after the chunk end and how many complete
// records lie on the way. The first kK entries form the chunk's transition
// table; tables are composed hierarchically (fan-in kGroup) to give each
// chunk its true entry and first record index. A second pass re-derives the
// links with 256-byte sub-chunk boundaries so 32 lanes can place the records
// of a chunk in parallel.
constexpr uint32_t kChunk = 8192;           // payload bytes per chunk
constexpr uint32_t kChunkShift = 13;
constexpr uint32_t kK = 1024;               // table entries (entry offsets) per chunk
constexpr uint32_t kSubShift = 8;           // 256-byte sub-chunks in the start pass
constexpr uint32_t kNSub = kChunk >> kSubShift;
constexpr uint32_t kGroup = 64;             // composition fan-in
constexpr uint32_t kStage = kChunk + 1024;  // bytes staged in LDS per chunk
constexpr uint32_t kVThreads = 256;

constexpr uint32_t kFlagIncomplete = 1u;  // a record runs past the wire end
constexpr uint32_t kFlagTooBig = 2u;      // exit offset >= kK
constexpr uint32_t kNoStart = 4u;         // (entries only) no record starts here

// level >= 1 tables (u64): exit (16) | flags (3) << 16 | count << 32
__host__ __device__ __forceinline__ uint64_t tpack(uint32_t exit, uint32_t flags,
                                                   uint64_t count) {
  return (uint64_t)(exit & 0xFFFF) | ((uint64_t)(flags & 7) << 16) | (count << 32);
}
// level 0 tables (u32): exit (11) | flags (2) << 11 | count << 16
__host__ __device__ __forceinline__ uint32_t t0pack(uint32_t exit, uint32_t flags,
                                                    uint32_t count) {
  return (exit & 0x7FF) | ((flags & 3) << 11) | (count << 16);
}
__host__ __device__ __forceinline__ uint32_t t_exit(uint64_t t) { return (uint32_t)t & 0xFFFF; }
__host__ __device__ __forceinline__ uint32_t t_flags(uint64_t t) { return (uint32_t)(t >> 16) & 7; }
__host__ __device__ __forceinline__ uint64_t t_count(uint64_t t) { return t >> 32; }
__host__ __device__ __forceinline__ uint32_t t_exit(uint32_t t) { return t & 0x7FF; }
__host__ __device__ __forceinline__ uint32_t t_flags(uint32_t t) { return (t >> 11) & 3; }
__host__ __device__ __forceinline__ uint64_t t_count(uint32_t t) { return t >> 16; }

struct VCtl {
  uint64_t p0;       // payload start (after header + count)
  uint64_t n;        // record count from the header
  uint64_t nchunks;  // chunks covering [p0, wire_len) (0 if n == 0)
  uint64_t data_len;
  unsigned long long end_pos;  // absolute end of record n-1
  uint32_t w;
  int32_t errc;  // header errc
  uint32_t need_fallback;
  uint32_t pad;
};

// Compact walk program of a record: fixed bytes, then per span
// [count:w][count*esz bytes][fixed bytes]. Built once on the host from the
// descriptor so the walker's loop constants sit in SGPRs.
struct WalkProg {
  uint32_t ns;
  uint32_t skip[SPK_MAX_SPANS + 1];
  uint32_t esz[SPK_MAX_SPANS];
};

static WalkProg make_walkprog(const spk_layout *L) {
  WalkProg p = {};
  uint32_t k = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    if (L->ops[i].kind == SPK_OP_COPY) {
      p.skip[k] += L->ops[i].size;
    } else {
      p.esz[k] = L->ops[i].size;
      ++k;
    }
  }
  p.ns = k;
  return p;
}

// LDS pointers carry address space 3 so reads lower to ds_read_u8, not
// flat_load_ubyte (a generic pointer would go through the flat path).
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

struct StagedReader {  // bytes [base, base+kStage) from LDS, others from HBM
  lds_cu8 *lds;
  const uint8_t *wire;
  uint64_t base;
  __device__ __forceinline__ uint8_t operator()(uint64_t x) const {
    const uint64_t r = x - base;
    if (r < kStage) return lds[r];
    return wire[x];
  }
};
__device__ __forceinline__ lds_cu8 *as_lds(const uint8_t *p) {
  return (lds_cu8 *)(p);
}
struct GlobalReader {
  const uint8_t *wire;
  __device__ __forceinline__ uint8_t operator()(uint64_t x) const { return wire[x]; }
};

template <class Rd>
__device__ __forceinline__ uint64_t rd_le(const Rd &rd, uint64_t x, uint32_t w) {
  uint64_t v = rd(x);
  if (w > 1) v |= (uint64_t)rd(x + 1) << 8;
  if (w > 2) {
    v |= (uint64_t)rd(x + 2) << 16;
    v |= (uint64_t)rd(x + 3) << 24;
  }
  if (w > 4)
    for (uint32_t i = 4; i < 8; ++i) v |= (uint64_t)rd(x + i) << (8 * i);
  return v;
}

// Wire length of the record at `pos` (0 = incomplete: the reference fails it
// with no_buffer_space). NS > 0: compile-time span count.
template <int NS, class Rd>
__device__ __forceinline__ uint64_t wlen(const WalkProg &P, const Rd &rd, uint64_t len,
                                         uint64_t pos, uint32_t w, uint64_t *acc) {
  uint64_t p = pos + P.skip[0];
  const uint32_t ns = NS > 0 ? (uint32_t)NS : P.ns;
#pragma unroll
  for (uint32_t k = 0; k < (NS > 0 ? (uint32_t)NS : SPK_MAX_SPANS); ++k) {
    if (NS == 0 && k >= ns) break;
    if (p + w > len) return 0;
    const uint64_t c = rd_le(rd, p, w);
    p += w;
    if (c) {
      if (P.esz[k] > 1 && c > ~0ull / P.esz[k]) return 0;
      const uint64_t nb = c * P.esz[k];
      if (nb > len - p) return 0;
      p += nb;
    }
    if (acc) acc[k] += c;
    p += P.skip[k + 1];
  }
  if (p > len) return 0;
  return p - pos;
}

__device__ __forceinline__ void stage_chunk(uint8_t *stage, const uint8_t *wire, uint64_t cs,
                                            uint64_t wire_len) {
  typedef uint32_t u32_unaligned __attribute__((aligned(1)));
  uint32_t *st32 = reinterpret_cast<uint32_t *>(stage);
  for (uint32_t x = threadIdx.x; x < kStage / 4; x += blockDim.x) {
    const uint64_t a = cs + 4ull * x;
    uint32_t v;
    if (a + 4 <= wire_len) {
      v = *reinterpret_cast<const u32_unaligned *>(wire + a);
    } else {
      v = 0;
      for (uint32_t i = 0; i < 4; ++i)
        if (a + i < wire_len) v |= (uint32_t)wire[a + i] << (8 * i);
    }
    st32[x] = v;
  }
}

// Packed per-position state (u32): count << 16 | link, link = next position
// (< kChunk) or terminal (bit 15) with q = first start at/after the boundary
// (bits 0-13, clamped to 16383) and bit 14 = incomplete record.
constexpr uint32_t kTerm = 0x8000u, kInc = 0x4000u, kQMask = 0x3FFFu;

constexpr uint32_t kPPT = kChunk / kVThreads;  // positions per thread (32)

// Each thread owns positions p = tid + 256*j (j < 32) and keeps their
// states in registers, so every jump round issues 32 independent LDS loads
// back to back instead of a dependent load chain per position.
template <int NS>
__device__ void build_links(uint32_t *S, const WalkProg &P, const uint8_t *stage,
                            const uint8_t *wire, uint64_t cs, uint64_t wire_len, uint32_t w,
                            uint32_t sh) {
  const StagedReader rd{as_lds(stage), wire, cs};
#pragma unroll 4
  for (uint32_t j = 0; j < kPPT; ++j) {
    const uint32_t p = threadIdx.x + j * kVThreads;
    uint32_t v;
    if (cs + p >= wire_len) {
      v = kTerm | p;  // wire end: no record here
    } else {
      const uint64_t L = wlen<NS>(P, rd, wire_len, cs + p, w, (uint64_t *)nullptr);
      if (!L) {
        v = kTerm | kInc | p;
      } else {
        const uint64_t q = p + L;
        const uint64_t bnd = (uint64_t)((p >> sh) + 1) << sh;
        v = (1u << 16) | (q >= bnd ? (kTerm | (uint32_t)(q < kQMask ? q : kQMask))
                                   : (uint32_t)q);
      }
    }
    S[p] = v;
  }
  __syncthreads();
  uint32_t st[kPPT];
#pragma unroll
  for (uint32_t j = 0; j < kPPT; ++j) st[j] = S[threadIdx.x + j * kVThreads];
  for (;;) {
    uint32_t u[kPPT];
#pragma unroll
    for (uint32_t j = 0; j < kPPT; ++j) u[j] = (st[j] & kTerm) ? 0u : S[st[j] & 0x7FFF];
    bool more = false;
#pragma unroll
    for (uint32_t j = 0; j < kPPT; ++j) {
      if (!(st[j] & kTerm)) {
        st[j] = (u[j] & 0xFFFF) | (((st[j] >> 16) + (u[j] >> 16)) << 16);
        S[threadIdx.x + j * kVThreads] = st[j];
        more |= !(u[j] & kTerm);
      }
    }
    if (!__syncthreads_or(more)) break;
  }
}

__global__ void vec_hdr_kernel(DecArgs a, const uint8_t *__restrict__ wire,
                               uint8_t *__restrict__ ws, spk_dresult_t *res) {
  if (threadIdx.x != 0) return;
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  uint64_t pos, dl;
  uint32_t w;
  int32_t e = parse_hdr(a.fmt, wire, a.wire_len, &pos, &w, &dl);
  uint64_t n = 0;
  if (!e) {
    if (a.wire_len < pos + w)
      e = SPK_ERRC_NO_BUFFER_SPACE;
    else
      n = ld_le(wire + pos, w);
    pos += w;
  }
  if (!e && n) {
    // every record needs at least fixed + n_spans*w bytes: a payload that
    // cannot hold n of them fails in the reference's record loop with
    // no_buffer_space (unpacker.hpp:1208-1226)
    const uint64_t min_rec = a.L.fixed_bytes + (uint64_t)a.L.n_spans * w;
    const uint64_t payload = a.wire_len - pos;
    if (n > payload / (min_rec ? min_rec : 1)) e = SPK_ERRC_NO_BUFFER_SPACE;
  }
  c->p0 = pos;
  c->n = e ? 0 : n;
  c->w = w;
  c->errc = e;
  c->data_len = dl;
  c->end_pos = 0;  // set by the lane that places record n-1
  c->need_fallback = 0;
  const uint64_t payload = (!e && a.wire_len > pos) ? a.wire_len - pos : 0;
  c->nchunks = (c->n == 0) ? 0 : (payload + kChunk - 1) / kChunk;
  spk_dresult_t r = {};
  r.errc = e;
  r.width = w;
  r.count = c->n;
  *res = r;
}

// per chunk: transition table for entry offsets [0, kK)
template <int NS>
__global__ __launch_bounds__(kVThreads) void vec_tables(DecArgs a, WalkProg P,
                                                        const uint8_t *__restrict__ wire,
                                                        const uint8_t *__restrict__ ws,
                                                        uint32_t *__restrict__ table) {
  __shared__ uint32_t S[kChunk];
  __shared__ __align__(16) uint8_t stage[kStage];
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  const uint64_t nchunks = c->nchunks;
  const uint32_t w = c->w;
  for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const uint64_t cs = c->p0 + ch * kChunk;
    stage_chunk(stage, wire, cs, a.wire_len);
    __syncthreads();
    build_links<NS>(S, P, stage, wire, cs, a.wire_len, w, kChunkShift);
    for (uint32_t e = threadIdx.x; e < kK; e += blockDim.x) {
      const uint32_t v = S[e];
      const uint32_t q = v & kQMask, cnt = v >> 16;
      uint32_t t;
      if (v & kInc)
        t = t0pack(0, kFlagIncomplete, cnt);
      else if (q < kChunk)  // clean wire end inside the (last) chunk
        t = t0pack(0, 0, cnt);
      else if (q - kChunk >= kK || q == kQMask)
        t = t0pack(0, kFlagTooBig, cnt);
      else
        t = t0pack(q - kChunk, 0, cnt);
      table[ch * kK + e] = t;
    }
    __syncthreads();
  }
}

// up-sweep: out[g][e] = T[g*G+G-1] o ... o T[g*G] (e)
template <typename TIn>
__global__ __launch_bounds__(256) void vec_compose_up(const TIn *__restrict__ in,
                                                      uint64_t n_in,
                                                      uint64_t *__restrict__ out) {
  const uint64_t g = blockIdx.x;
  for (uint32_t e0 = threadIdx.x; e0 < kK; e0 += blockDim.x) {
    uint32_t e = e0, fl = 0;
    uint64_t cnt = 0;
    for (uint64_t j = g * kGroup; j < n_in && j < (g + 1) * kGroup; ++j) {
      const TIn t = in[j * kK + e];
      cnt += t_count(t);
      if (t_flags(t)) {
        fl = t_flags(t);
        break;
      }
      e = t_exit(t);
    }
    out[g * kK + e0] = tpack(e, fl, cnt);
  }
}

// down-sweep: entry/base of each group -> entry/base of each member.
// Entries are (offset | flags << 16); a flagged entry propagates unchanged.
template <typename TIn>
__global__ void vec_compose_down(const TIn *__restrict__ tab, uint64_t n_in,
                                 uint64_t n_groups, const uint32_t *__restrict__ g_entry,
                                 const uint64_t *__restrict__ g_base,
                                 uint32_t *__restrict__ m_entry,
                                 uint64_t *__restrict__ m_base) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  uint32_t ent = g_entry[g];
  uint64_t base = g_base[g];
  for (uint64_t j = g * kGroup; j < n_in && j < (g + 1) * kGroup; ++j) {
    m_entry[j] = ent;
    m_base[j] = base;
    if (ent >> 16) continue;
    const TIn t = tab[j * kK + ent];
    base += t_count(t);
    ent = t_flags(t) ? (t_flags(t) << 16) : t_exit(t);
  }
}

// TooBig before record n: records straddle chunk boundaries by >= kK bytes;
// request the sequential fallback.
__global__ void vec_check_entries(uint8_t *__restrict__ ws,
                                  const uint32_t *__restrict__ m_entry,
                                  const uint64_t *__restrict__ m_base) {
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  const uint64_t ch = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c->nchunks || c->errc) return;
  if (m_base[ch] < c->n && ((m_entry[ch] >> 16) & kFlagTooBig)) c->need_fallback = 1;
}

// Sequential fallback: one lane walks every record (global reads) and writes
// each chunk's entry/base directly. Correct for any record size; slow.
__global__ void vec_seq_walk(DecArgs a, WalkProg P, const uint8_t *__restrict__ wire,
                             uint8_t *__restrict__ ws, uint32_t *__restrict__ m_entry,
                             uint64_t *__restrict__ m_base) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  if (!c->need_fallback) return;
  const GlobalReader rd{wire};
  uint64_t pos = c->p0, rec = 0, ch = 0;
  uint32_t flag = 0;
  while (rec < c->n) {
    while (ch < c->nchunks && c->p0 + (ch + 1) * kChunk <= pos) {  // chunks passed over
      m_entry[ch] = kNoStart << 16;
      m_base[ch] = rec;
      ++ch;
    }
    if (ch < c->nchunks && c->p0 + ch * kChunk <= pos) {  // first start in chunk ch
      m_entry[ch] = (uint32_t)(pos - (c->p0 + ch * kChunk));
      m_base[ch] = rec;
      ++ch;
    }
    const uint64_t rl = wlen<0>(P, rd, a.wire_len, pos, c->w, (uint64_t *)nullptr);
    if (!rl) {
      flag = kFlagIncomplete;
      break;
    }
    pos += rl;
    ++rec;
  }
  for (; ch < c->nchunks; ++ch) {
    m_entry[ch] = (flag ? kFlagIncomplete : kNoStart) << 16;
    m_base[ch] = rec;
  }
}

// Start pass, block per chunk with a known entry: sub-chunk links, thread 0
// chains the 32 sub-chunk entries, then one lane per sub-chunk places its
// records (starts[]), sums span counts, and detects a short payload / the
// end of record n-1.
template <int NS>
__global__ __launch_bounds__(kVThreads) void vec_starts(
    DecArgs a, WalkProg P, const uint8_t *__restrict__ wire, uint8_t *__restrict__ ws,
    const uint32_t *__restrict__ m_entry, const uint64_t *__restrict__ m_base,
    uint64_t *__restrict__ starts, uint64_t *__restrict__ csum, spk_dresult_t *res) {
  __shared__ uint32_t S[kChunk];
  __shared__ __align__(16) uint8_t stage[kStage];
  __shared__ uint32_t sub_ent[kNSub], sub_base[kNSub];
  __shared__ uint64_t red[kVThreads / 64];
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  if (c->errc) return;
  const uint64_t nchunks = c->nchunks, n = c->n;
  const uint32_t w = c->w;
  for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const uint32_t ent = m_entry[ch];
    const uint64_t base = m_base[ch];
    if ((ent >> 16) || base >= n) continue;  // block-uniform
    const uint64_t cs = c->p0 + ch * kChunk;
    stage_chunk(stage, wire, cs, a.wire_len);
    __syncthreads();
    build_links<NS>(S, P, stage, wire, cs, a.wire_len, w, kSubShift);
    if (threadIdx.x < kNSub) sub_ent[threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t e = ent, k = 0;
      while (e < kChunk) {
        const uint32_t j = e >> kSubShift;
        sub_ent[j] = e;
        sub_base[j] = k;
        const uint32_t v = S[e];
        k += v >> 16;
        const uint32_t q = v & kQMask;
        if ((v & kInc) || q < ((j + 1) << kSubShift)) break;  // incomplete / wire end
        e = q;
      }
    }
    __syncthreads();
    uint64_t acc[SPK_MAX_SPANS] = {};
    if (threadIdx.x < kNSub && sub_ent[threadIdx.x] != 0xFFFFFFFFu) {
      const StagedReader rd{as_lds(stage), wire, cs};
      const uint32_t j = threadIdx.x;
      uint64_t pos = cs + sub_ent[j], k = base + sub_base[j];
      const uint64_t bnd = cs + ((uint64_t)(j + 1) << kSubShift);
      while (pos < bnd && k < n) {
        const uint64_t L = wlen<NS>(P, rd, a.wire_len, pos, w, acc);
        if (!L) break;
        if (k < a.rec_cap) starts[k] = pos;
        pos += L;
        ++k;
      }
      if (k == n) atomicMax(&c->end_pos, (unsigned long long)pos);
      // stopped before record n without crossing the sub-chunk boundary:
      // an incomplete record or the wire end (reference: no_buffer_space)
      if (k < n && pos < bnd) atomicCAS(&res->errc, 0, SPK_ERRC_NO_BUFFER_SPACE);
    }
    for (uint32_t s2 = 0; s2 < P.ns; ++s2) {
      uint64_t v = acc[s2];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (uint32_t i = 0; i < kVThreads / 64; ++i) t += red[i];
        csum[ch * SPK_MAX_SPANS + s2] = t;
      }
      __syncthreads();
    }
    __syncthreads();
  }
}

__global__ void vec_finish(DecArgs a, uint8_t *__restrict__ ws, spk_dresult_t *res) {
  if (threadIdx.x != 0) return;
  VCtl *c = reinterpret_cast<VCtl *>(ws + kWsCtl);
  if (c->errc) return;
  spk_dresult_t r = *res;
  // record n-1 was never placed: the payload holds fewer than n records
  if (c->n && c->end_pos == 0 && r.errc == 0) r.errc = SPK_ERRC_NO_BUFFER_SPACE;
  if (r.errc == SPK_ERRC_NO_BUFFER_SPACE) {
    r.count = 0;
    r.consumed = 0;
    for (int k = 0; k < SPK_MAX_SPANS; ++k) r.heap_used[k] = 0;
  } else {
    r.count = c->n;
    const uint64_t end = c->n ? (uint64_t)c->end_pos : c->p0;
    r.consumed = end > c->data_len ? end : c->data_len;
    if (c->n > a.rec_cap && r.errc == 0) r.errc = SPK_ERRC_CAPACITY;
  }
  *res = r;
}

// decode pass, block per chunk: records [base, next_base) from starts[]
__global__ __launch_bounds__(kThreads) void vec_chunk_decode(
    DecArgs a, const uint8_t *__restrict__ wire, const uint8_t *__restrict__ ws,
    const uint32_t *__restrict__ m_entry, const uint64_t *__restrict__ m_base,
    const uint64_t *__restrict__ starts, const uint64_t *__restrict__ csum,
    uint8_t *__restrict__ recs, const spk_dresult_t *res) {
  __shared__ uint64_t sh[kThreads / 64];
  __shared__ uint64_t run[SPK_MAX_SPANS];
  const VCtl *c = reinterpret_cast<const VCtl *>(ws + kWsCtl);
  if (c->errc || res->errc) return;
  const uint64_t nchunks = c->nchunks, n = c->n;
  const uint32_t w = c->w;
  for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const uint32_t ent = m_entry[ch];
    const uint64_t base = m_base[ch];
    if ((ent >> 16) || base >= n) continue;
    // records of this chunk end where the next chunk with a start begins
    uint64_t hi = n;
    for (uint64_t c2 = ch + 1; c2 < nchunks; ++c2) {
      if (!(m_entry[c2] >> 16)) {
        hi = m_base[c2] < n ? m_base[c2] : n;
        break;
      }
      if ((m_entry[c2] >> 16) & (kFlagIncomplete | kFlagTooBig)) break;
    }
    if (threadIdx.x < SPK_MAX_SPANS) run[threadIdx.x] = csum[ch * SPK_MAX_SPANS + threadIdx.x];
    __syncthreads();
    for (uint64_t r0 = base; r0 < hi; r0 += kThreads) {
      const uint64_t i = r0 + threadIdx.x;
      uint64_t cnt[SPK_MAX_SPANS] = {};
      if (i < hi) rec_counts(a.L, wire, starts[i], w, cnt);
      uint64_t hoff[SPK_MAX_SPANS] = {};
      for (uint32_t k = 0; k < a.L.n_spans; ++k) {
        uint64_t tot;
        hoff[k] = run[k] + block_excl_scan(cnt[k], &tot, sh);
        __syncthreads();
        if (threadIdx.x == 0) run[k] += tot;
      }
      if (i < hi) decode_record(a.L, wire, starts[i], w, recs + i * a.L.stride, a.heaps, hoff);
      __syncthreads();
    }
  }
}

// ===========================================================================
// host launchers
// ===========================================================================
static unsigned grid_for(uint64_t items, uint64_t per_block) {
  uint64_t b = (items + per_block - 1) / per_block;
  return (unsigned)(b ? b : 1);
}

struct VecWs {  // byte offsets inside the workspace for vector decode
  size_t table, lv[8], ent[8], base[8], csum, starts, end;
  uint64_t nlev[8];
  int levels;
};

static VecWs vec_ws_layout(uint64_t wire_len, uint64_t max_records) {
  VecWs v = {};
  const uint64_t nch = wire_len / kChunk + 2;
  size_t off = kWsScratch;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  v.table = take(nch * kK * 4);
  uint64_t cnt = nch;
  v.nlev[0] = nch;
  v.levels = 0;
  while (cnt > 1 && v.levels < 7) {
    cnt = (cnt + kGroup - 1) / kGroup;
    ++v.levels;
    v.nlev[v.levels] = cnt;
    v.lv[v.levels] = take(cnt * kK * 8);
  }
  for (int l = 0; l <= v.levels; ++l) {
    v.ent[l] = take(v.nlev[l] * 4 + 8);
    v.base[l] = take(v.nlev[l] * 8 + 8);
  }
  v.csum = take(nch * SPK_MAX_SPANS * 8);
  v.starts = take(max_records * 8 + 8);
  v.end = off;
  return v;
}

template <int NS>
static void launch_vec_tables(unsigned grid, hipStream_t s, const DecArgs &a, const WalkProg &P,
                              const uint8_t *wire, const uint8_t *ws, uint32_t *table) {
  hipLaunchKernelGGL(vec_tables<NS>, dim3(grid), dim3(kVThreads), 0, s, a, P, wire, ws, table);
}
template <int NS>
static void launch_vec_starts(unsigned grid, hipStream_t s, const DecArgs &a, const WalkProg &P,
                              const uint8_t *wire, uint8_t *ws, const uint32_t *m_entry,
                              const uint64_t *m_base, uint64_t *starts, uint64_t *csum,
                              spk_dresult_t *res) {
  hipLaunchKernelGGL(vec_starts<NS>, dim3(grid), dim3(kVThreads), 0, s, a, P, wire, ws, m_entry,
                     m_base, starts, csum, res);
}

size_t var_workspace_bytes(const spk_layout *L, int mode, uint64_t n, uint64_t wire_len) {
  size_t enc = kWsScratch + (grid_for(n, kRPB) + 1) * sizeof(Partial) + 256;
  size_t dec_msg = kWsScratch + n * sizeof(MsgState) +
                   (grid_for(n, kThreads) + 1) * SPK_MAX_SPANS * 8 + 256;
  size_t dec_vec = vec_ws_layout(wire_len, n).end + 256;
  size_t m = enc;
  if (mode == SPK_MODE_MESSAGES) m = m > dec_msg ? m : dec_msg;
  if (mode == SPK_MODE_VECTOR) m = m > dec_vec ? m : dec_vec;
  (void)L;
  return m;
}

static VarArgs make_varargs(const spk_layout *L, int mode, uint64_t n,
                            const void *const *heaps) {
  VarArgs a = {};
  a.L = make_klayout(L);
  a.n = n;
  a.mode = mode;
  for (uint32_t k = 0; k < a.L.n_spans && k < SPK_MAX_SPANS; ++k)
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
                           hipStream_t s) {
  VarArgs a = make_varargs(L, mode, n, nullptr);
  uint8_t *ws = (uint8_t *)d_ws;
  const MsgHdrTable t = msg_hdr_table(L);
  hipLaunchKernelGGL(write_msg_hdrs, dim3(1), dim3(256), 0, s, t, ws);
  const uint64_t nb = grid_for(n, kRPB);
  const uint8_t *tbl = ws + kWsHdrMsg + 4 * kWsHdrSlot - 8;
  if (n)
    hipLaunchKernelGGL(var_plan_reduce, dim3(nb), dim3(kThreads), 0, s, a,
                       (const uint8_t *)d_recs, ws, tbl);
  FinArgs f;
  f.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  f.n = n;
  f.nblocks = n ? nb : 0;
  f.n_spans = a.L.n_spans;
  f.mode = mode;
  hipLaunchKernelGGL(var_plan_finalize, dim3(1), dim3(1024), 0, s, f, ws, d_plan);
  (void)ws_bytes;
  return hipGetLastError();
}

hipError_t launch_var_encode(const spk_layout *L, int mode, uint64_t n,
                             const void *d_recs, const void *const *d_heaps,
                             const spk_plan_t *d_plan, void *d_out, uint64_t out_cap,
                             uint64_t *d_offsets, void *d_ws, size_t ws_bytes,
                             hipStream_t s) {
  VarArgs a = make_varargs(L, mode, n, d_heaps);
  uint8_t *ws = (uint8_t *)d_ws;
  if (n == 0) {
    // header (+ zero count) only; reuse the write kernel with one block
  }
  hipLaunchKernelGGL(var_encode_write, dim3(grid_for(n ? n : 1, kRPB)), dim3(kThreads), kWin,
                     s, a, (const uint8_t *)d_recs, (uint8_t *)d_out, out_cap,
                     (const uint8_t *)ws, d_plan, d_offsets);
  (void)ws_bytes;
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
  for (uint32_t i = 0; i < L->n_ops; ++i) ns += L->ops[i].kind == SPK_OP_SPAN;
  hipLaunchKernelGGL(body_plan_kernel, dim3(1), dim3(64), 0, s, plan, n, ns, width);
  return launch_var_encode(L, SPK_MODE_VECTOR, n, d_recs, d_heaps, plan, d_out, out_cap,
                           nullptr, d_ws, ws_bytes, s);
}

hipError_t launch_var_decode(const spk_layout *L, int mode, const void *d_wire,
                             uint64_t wire_len, const uint64_t *d_offsets,
                             uint64_t n_msgs, void *d_recs, uint64_t rec_cap,
                             void *const *d_heaps, const uint64_t *heap_caps,
                             spk_dresult_t *d_res, int32_t *d_errc, void *d_ws,
                             size_t ws_bytes, hipStream_t s) {
  DecArgs a = {};
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
    if ((e = hipMemsetAsync(d_res, 0, sizeof(spk_dresult_t), s)) != hipSuccess) return e;
    if (n_msgs == 0) return hipSuccess;
    const unsigned nb = grid_for(n_msgs, kThreads);
    hipLaunchKernelGGL(var_msg_parse, dim3(nb), dim3(kThreads), 0, s, a, wire, d_offsets,
                       ws, d_errc, d_res);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + kWsScratch + sizeof(MsgState) * n_msgs);
    hipLaunchKernelGGL(var_scan_blocks, dim3(1), dim3(1024), 0, s, (uint64_t)nb,
                       a.L.n_spans, bsum, a, d_res);
    hipLaunchKernelGGL(var_msg_write, dim3(nb), dim3(kThreads), 0, s, a, wire,
                       (const uint8_t *)ws, (uint8_t *)d_recs, (const spk_dresult_t *)d_res);
    (void)ws_bytes;
    return hipGetLastError();
  }
  // ---- VECTOR ----
  const VecWs v = vec_ws_layout(wire_len, rec_cap);
  const WalkProg P = make_walkprog(L);
  const int NS = P.ns == 1 ? 1 : P.ns == 2 ? 2 : 0;
  uint32_t *table = reinterpret_cast<uint32_t *>(ws + v.table);
  hipLaunchKernelGGL(vec_hdr_kernel, dim3(1), dim3(64), 0, s, a, wire, ws, d_res);
  const uint64_t max_chunks = v.nlev[0];
  const unsigned tb = (unsigned)(max_chunks < 16384 ? max_chunks : 16384);
  if (NS == 1)
    launch_vec_tables<1>(tb, s, a, P, wire, ws, table);
  else if (NS == 2)
    launch_vec_tables<2>(tb, s, a, P, wire, ws, table);
  else
    launch_vec_tables<0>(tb, s, a, P, wire, ws, table);
  const uint64_t *lvl_tab[8] = {};
  for (int l = 1; l <= v.levels; ++l) {
    uint64_t *out = reinterpret_cast<uint64_t *>(ws + v.lv[l]);
    if (l == 1)
      hipLaunchKernelGGL(vec_compose_up<uint32_t>, dim3((unsigned)v.nlev[l]), dim3(256), 0, s,
                         (const uint32_t *)table, v.nlev[0], out);
    else
      hipLaunchKernelGGL(vec_compose_up<uint64_t>, dim3((unsigned)v.nlev[l]), dim3(256), 0, s,
                         lvl_tab[l - 1], v.nlev[l - 1], out);
    lvl_tab[l] = out;
  }
  if ((e = hipMemsetAsync(ws + v.ent[v.levels], 0, 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(ws + v.base[v.levels], 0, 16, s)) != hipSuccess) return e;
  for (int l = v.levels; l >= 1; --l) {
    const uint64_t ng = v.nlev[l];
    const uint32_t *ge = (const uint32_t *)(ws + v.ent[l]);
    const uint64_t *gb = (const uint64_t *)(ws + v.base[l]);
    uint32_t *me = reinterpret_cast<uint32_t *>(ws + v.ent[l - 1]);
    uint64_t *mb = reinterpret_cast<uint64_t *>(ws + v.base[l - 1]);
    if (l == 1)
      hipLaunchKernelGGL(vec_compose_down<uint32_t>, dim3(grid_for(ng, 64)), dim3(64), 0, s,
                         (const uint32_t *)table, v.nlev[0], ng, ge, gb, me, mb);
    else
      hipLaunchKernelGGL(vec_compose_down<uint64_t>, dim3(grid_for(ng, 64)), dim3(64), 0, s,
                         lvl_tab[l - 1], v.nlev[l - 1], ng, ge, gb, me, mb);
  }
  uint32_t *m_entry = reinterpret_cast<uint32_t *>(ws + v.ent[0]);
  uint64_t *m_base = reinterpret_cast<uint64_t *>(ws + v.base[0]);
  hipLaunchKernelGGL(vec_check_entries, dim3(grid_for(max_chunks, 256)), dim3(256), 0, s, ws,
                     (const uint32_t *)m_entry, (const uint64_t *)m_base);
  hipLaunchKernelGGL(vec_seq_walk, dim3(1), dim3(64), 0, s, a, P, wire, ws, m_entry, m_base);
  uint64_t *csum = reinterpret_cast<uint64_t *>(ws + v.csum);
  uint64_t *starts = reinterpret_cast<uint64_t *>(ws + v.starts);
  if ((e = hipMemsetAsync(csum, 0, max_chunks * SPK_MAX_SPANS * 8, s)) != hipSuccess) return e;
  if (NS == 1)
    launch_vec_starts<1>(tb, s, a, P, wire, ws, m_entry, m_base, starts, csum, d_res);
  else if (NS == 2)
    launch_vec_starts<2>(tb, s, a, P, wire, ws, m_entry, m_base, starts, csum, d_res);
  else
    launch_vec_starts<0>(tb, s, a, P, wire, ws, m_entry, m_base, starts, csum, d_res);
  hipLaunchKernelGGL(var_scan_blocks, dim3(1), dim3(1024), 0, s, max_chunks, a.L.n_spans,
                     csum, a, d_res);
  hipLaunchKernelGGL(vec_finish, dim3(1), dim3(64), 0, s, a, ws, d_res);
  const unsigned db = (unsigned)(max_chunks < 16384 ? max_chunks : 16384);
  hipLaunchKernelGGL(vec_chunk_decode, dim3(db), dim3(kThreads), 0, s, a, wire,
                     (const uint8_t *)ws, (const uint32_t *)m_entry,
                     (const uint64_t *)m_base, (const uint64_t *)starts,
                     (const uint64_t *)csum, (uint8_t *)d_recs, (const spk_dresult_t *)d_res);
  (void)ws_bytes;
  return hipGetLastError();
}

}  // namespace spk
