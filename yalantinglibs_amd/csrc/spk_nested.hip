// spk_nested.hip — layouts with SPK_OP_ARRAY: containers whose elements are
// not trivially serializable (vector<string>, vector<struct with a string>,
// vector<vector<string>> ...).
//
// Reference behaviour restated (paths relative to
// /root/reference/include/ylt/struct_pack/):
//   size      calculate_size.hpp:76-87 (a container of non-trivial elements
//             sums its elements; every container adds a count and bounds the
//             width by its length)
//   encode    packer.hpp:365-367 (length, then serialize_one per element)
//   decode    unpacker.hpp:1208-1226 (length, then emplace_back + decode per
//             element, stopping at the first failing one)
//
// The record's wire length depends on every element it holds, so these
// layouts run an op-list interpreter: one lane per record (encode, MESSAGES
// decode) with an explicit element stack (SPK_MAX_DEPTH levels). A VECTOR
// message's record boundaries come from one wave that walks the counts
// through an LDS window (payload bytes are skipped, not read), then every
// record is decoded by its own lane into heap offsets from a per-heap scan.
//
// compatible<U, ver> members (SPK_OP_COMPAT, top-level record only) run here
// too: the main pass skips them, then one version pass per rank writes
// [has][U] of every record (packer.hpp:66-78,453-461; unpacker.hpp:292-366,
// 1354-1376). A VECTOR decode's walker records where each record's group of
// each version starts; the record's lane decodes its groups from there.
#include "spk_internal.hpp"
#include "spk_nlayout.hpp"

#include <stdlib.h>

namespace spk {

typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
typedef v4u_t v4u_una __attribute__((aligned(1)));


// layouts the interpreter runs: an ARRAY (element layouts), a VARIANT, an
// OPTGROUP, a compatible member, a fast-varint group, or more heaps than the
// flat-record kernels carry
bool layout_nested(const spk_layout *L) {
  uint32_t heaps = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const uint32_t k = SPK_OP_KIND(L->ops[i].kind);
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT || k == SPK_OP_COMPAT || k == SPK_OP_FVAR ||
        k == SPK_OP_OPTGROUP || k == SPK_OP_CGROUP)
      return true;
    heaps += op_has_heap(k);
  }
  return heaps > SPK_FLAT_SPANS;  // more heaps than the flat kernels carry
}

// ---- shared helpers ---------------------------------------------------------
__device__ __forceinline__ uint64_t n_vi_value(const spk_op &op, const uint8_t *rec) {
  // serialize_varint (varint.hpp:245-268): sint<T> zigzag at its own width
  if (op.size == 4) {
    uint32_t u = *reinterpret_cast<const uint32_t *>(rec + op.rec_off);
    if (op.aux & SPK_VARINT_SEXT) return (uint64_t)(int64_t)(int32_t)u;  // plain int32_t: v = t
    if (op.aux & SPK_VARINT_ZIGZAG) u = (u << 1) ^ (uint32_t)(-(int32_t)(u >> 31));
    return u;
  }
  uint64_t u = *reinterpret_cast<const uint64_t *>(rec + op.rec_off);
  if (op.aux & SPK_VARINT_ZIGZAG) u = (u << 1) ^ (uint64_t)(-(int64_t)(u >> 63));
  return u;
}
__device__ __forceinline__ uint32_t n_vi_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
// (unaligned 16-, 8- and 4-B accesses: one load and one store each on gfx950;
// a string copied byte by byte was one partial-line store per byte)
typedef uint64_t n_u64_una __attribute__((aligned(1)));
typedef uint32_t n_u32_una __attribute__((aligned(1)));
typedef v4u_t n_v4u_una __attribute__((aligned(1)));

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
__device__ __forceinline__ void n_copy(uint8_t *d, const uint8_t *s, uint64_t n) {
  uint64_t i = 0;
  for (; i + 16 <= n; i += 16)
    *reinterpret_cast<n_v4u_una *>(d + i) = *reinterpret_cast<const n_v4u_una *>(s + i);
  if (i + 8 <= n) {
    *reinterpret_cast<n_u64_una *>(d + i) = *reinterpret_cast<const n_u64_una *>(s + i);
    i += 8;
  }
  if (i + 4 <= n) {
    *reinterpret_cast<n_u32_una *>(d + i) = *reinterpret_cast<const n_u32_una *>(s + i);
    i += 4;
  }
  for (; i < n; ++i) d[i] = s[i];
}

// The interpreter's byte reader: the wire in global memory, or a wave's
// staged LDS copy of [lo, hi) with the bytes outside it from global memory
// (MESSAGES decode: the wave's 64 consecutive messages, loaded with aligned
// 16-B loads instead of each lane's scattered byte loads). A raw pointer is
// the global-only reader.
typedef __attribute__((address_space(3))) uint8_t nlds_u8;
typedef __attribute__((address_space(3))) uint32_t nlds_u32_una __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint64_t nlds_u64_una __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) v4u_t nlds_v4u_una __attribute__((aligned(1)));
struct NRd {
  const uint8_t *w;
  const nlds_u8 *lds;
  uint64_t lo, hi;
  __device__ __forceinline__ uint8_t operator[](uint64_t p) const {
    return p - lo < hi - lo ? lds[(uint32_t)(p - lo)] : w[p];
  }
};
__device__ __forceinline__ void n_copy_rd(uint8_t *d, const uint8_t *w, uint64_t p, uint64_t n) {
  n_copy(d, w + p, n);
}
__device__ __forceinline__ void n_copy_rd(uint8_t *d, const NRd &rd, uint64_t p, uint64_t n) {
  if (p - rd.lo < rd.hi - rd.lo && rd.hi - p >= n) {
    const nlds_u8 *l = rd.lds + (uint32_t)(p - rd.lo);
    uint32_t i = 0;
    for (; i + 16 <= n; i += 16)
      *reinterpret_cast<n_v4u_una *>(d + i) = *reinterpret_cast<const nlds_v4u_una *>(l + i);
    if (i + 8 <= n) {
      *reinterpret_cast<n_u64_una *>(d + i) = *reinterpret_cast<const nlds_u64_una *>(l + i);
      i += 8;
    }
    if (i + 4 <= n) {
      *reinterpret_cast<n_u32_una *>(d + i) = *reinterpret_cast<const nlds_u32_una *>(l + i);
      i += 4;
    }
    for (; i < n; ++i) d[i] = l[i];
  } else {
    n_copy(d, rd.w + p, n);
  }
}

// the layout in LDS: the interpreter reads an op per step, and a kernel
// argument indexed per lane would be fetched from memory every time
__device__ __forceinline__ void n_stage(NLayout &dst, const NLayout &src) {
  static_assert(sizeof(NLayout) % 4 == 0, "NLayout staged as words");
  const uint32_t *s = reinterpret_cast<const uint32_t *>(&src);
  uint32_t *d = reinterpret_cast<uint32_t *>(&dst);
  for (uint32_t k = threadIdx.x; k < sizeof(NLayout) / 4; k += blockDim.x) d[k] = s[k];
  __syncthreads();
}

// one open ARRAY or group on the interpreter's stack
struct NFrame {
  uint32_t aop, pend;      // the ARRAY / group op; the op range end to resume
  uint64_t j, cnt;         // element index, element count (a group: 0 of 1)
  const uint8_t *el;       // element records (encode) / output slots (decode)
  const uint8_t *prec;     // record to resume
  uint32_t first, ret;     // first op of an element / group; op to resume at
};

// first op of group `a` of the VARIANT / OPTGROUP at i (groups closed by END)
__device__ __forceinline__ uint32_t n_alt_start(const NLayout &N, uint32_t i, uint32_t a) {
  uint32_t j = i + 1;
  while (a) {
    const uint32_t k = N.ops[j].kind;
    if (k == SPK_OP_ARRAY || n_group(k)) {
      j = N.end[j] + 1;  // skip a nested one whole
      continue;
    }
    if (k == SPK_OP_END) --a;
    ++j;
  }
  return j;
}
// the END that closes the group starting at j
__device__ __forceinline__ uint32_t n_alt_end(const NLayout &N, uint32_t j) {
  for (;;) {
    const uint32_t k = N.ops[j].kind;
    if (k == SPK_OP_ARRAY || n_group(k)) {
      j = N.end[j] + 1;
      continue;
    }
    if (k == SPK_OP_END) return j;
    ++j;
  }
}
// the group a VARIANT / OPTGROUP / CGROUP at i writes for record r: the
// variant's index; group 0 (the value) when has_value, else group 1 of an
// expected (its error) or none (-1) (packer.hpp:382-410)
__device__ __forceinline__ int n_active(const NLayout &N, uint32_t i, const uint8_t *r) {
  const uint32_t v = *reinterpret_cast<const uint32_t *>(r + N.ops[i].rec_off);
  if (N.ops[i].kind == SPK_OP_VARIANT) return (int)v;
  return v ? 0 : (N.ops[i].size == 2 ? 1 : -1);
}

// ---- USE_FAST_VARINT group of the top-level record (packer.hpp:152-235,
// calculate_size.hpp:191-390, unpacker.hpp:642-747): a bitset of non-zero
// flags + 2 width bits, then the non-zero values at min(2^code, size) bytes --
__device__ __forceinline__ uint64_t n_fv_raw(const spk_op &op, const uint8_t *rec) {
  return op.size == 4 ? *reinterpret_cast<const uint32_t *>(rec + op.rec_off)
                      : *reinterpret_cast<const uint64_t *>(rec + op.rec_off);
}
__device__ uint32_t n_fv_code(const NLayout &N, const uint8_t *rec) {
  uint64_t um = 0, sm = 0;
  bool hu = false, hs = false;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_FVAR) continue;
    const uint64_t r = n_fv_raw(op, rec);
    if (op.aux & SPK_FVAR_SIGNED) {
      hs = true;
      const int64_t v = op.size == 4 ? (int64_t)(int32_t)(uint32_t)r : (int64_t)r;
      const uint64_t m = v > 0 ? (uint64_t)v : (uint64_t)(-(v + 1));
      if (v && m > sm) sm = m;
    } else {
      hu = true;
      if (r > um) um = r;
    }
  }
  const uint32_t cu = !hu ? 0u : um <= 0xFFull ? 0u : um <= 0xFFFFull ? 1u : um <= 0xFFFFFFFFull ? 2u : 3u;
  const uint32_t cs = !hs ? 0u : sm <= 0x7Full ? 0u : sm <= 0x7FFFull ? 1u : sm <= 0x7FFFFFFFull ? 2u : 3u;
  return cu > cs ? cu : cs;
}
__device__ uint64_t n_fv_size(const NLayout &N, const uint8_t *rec) {
  if (!N.fv_cnt) return 0;
  const uint32_t wb = 1u << n_fv_code(N, rec);
  uint64_t b = N.fv_bits;
  for (uint32_t i = 0; i < N.n_ops; ++i)
    if (N.ops[i].kind == SPK_OP_FVAR && n_fv_raw(N.ops[i], rec))
      b += wb < N.ops[i].size ? wb : N.ops[i].size;
  return b;
}
// the group's wire length from its bitset at wire[pos] (the caller checked
// the bitset is there); 0 for the invalid width code
__device__ __forceinline__ uint64_t n_fv_len(const NLayout &N, const uint8_t *bs) {
  const uint32_t code = ((bs[N.fv_cnt / 8] >> (N.fv_cnt % 8)) & 1u) |
                        (((bs[(N.fv_cnt + 1) / 8] >> ((N.fv_cnt + 1) % 8)) & 1u) << 1);
  if (code == 3 && !N.fv_has64) return 0;
  const uint32_t wb = 1u << code;
  uint64_t b = N.fv_bits;
  uint32_t j = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    if (N.ops[i].kind != SPK_OP_FVAR) continue;
    if ((bs[j / 8] >> (j % 8)) & 1u) b += wb < N.ops[i].size ? wb : N.ops[i].size;
    ++j;
  }
  return b;
}
// deserialize_fast_varint: errc; values into rec (zero when the bit is clear)
template <typename Rd>
__device__ int32_t n_fv_read(const NLayout &N, const Rd &wire, uint64_t &pos, uint64_t end,
                             uint8_t *rec) {
  if (end - pos < N.fv_bits) return SPK_ERRC_NO_BUFFER_SPACE;
  uint8_t bs[(SPK_MAX_VARINTS + 2 + 7) / 8];
  for (uint32_t b = 0; b < N.fv_bits; ++b) bs[b] = wire[pos + b];
  pos += N.fv_bits;
  const uint32_t code = ((bs[N.fv_cnt / 8] >> (N.fv_cnt % 8)) & 1u) |
                        (((bs[(N.fv_cnt + 1) / 8] >> ((N.fv_cnt + 1) % 8)) & 1u) << 1);
  if (code == 3 && !N.fv_has64) return SPK_ERRC_INVALID_BUFFER;
  const uint32_t wb = 1u << code;
  uint32_t j = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_FVAR) continue;
    uint64_t v = 0;
    if ((bs[j / 8] >> (j % 8)) & 1u) {
      const uint32_t rw = wb < op.size ? wb : op.size;
      if (end - pos < rw) return SPK_ERRC_NO_BUFFER_SPACE;
      for (uint32_t b = 0; b < rw; ++b) v |= (uint64_t)wire[pos + b] << (8 * b);
      pos += rw;
      if ((op.aux & SPK_FVAR_SIGNED) && rw < 8 && ((v >> (8 * rw - 1)) & 1u)) v |= ~0ull << (8 * rw);
    }
    if (rec) {
      if (op.size == 4)
        *reinterpret_cast<uint32_t *>(rec + op.rec_off) = (uint32_t)v;
      else
        *reinterpret_cast<uint64_t *>(rec + op.rec_off) = v;
    }
    ++j;
  }
  return SPK_ERRC_OK;
}

// ---- encode: the interpreter's element stack and output sinks ---------------------
// The top frame lives in registers and D - 1 frames below it (D = the layout's
// depth: 1, 2 or SPK_MAX_DEPTH); only D = SPK_MAX_DEPTH indexes them at run
// time (a runtime index puts the stack in scratch memory).
template <int D>
struct NStk {
  NFrame top;
  NFrame sv[D > 1 ? D - 1 : 1];
  __device__ __forceinline__ void push(uint32_t d, const NFrame &f) {  // d: depth before
    if constexpr (D > 1) {
      if (d) {
        if constexpr (D == 2)
          sv[0] = top;
        else
          sv[d - 1] = top;
      }
    }
    top = f;
  }
  __device__ __forceinline__ void pop(uint32_t d) {  // d: depth after
    if constexpr (D > 1) {
      if (d) {
        if constexpr (D == 2)
          top = sv[0];
        else
          top = sv[d - 1];
      }
    }
  }
};
// the kernels' D for a layout
static inline int n_dclass(const NLayout &N) { return N.depth <= 1 ? 1 : N.depth <= 2 ? 2 : 4; }
#define NEST_D(depth_class, ...)            \
  do {                                      \
    if ((depth_class) == 1) {               \
      constexpr int D = 1;                  \
      __VA_ARGS__;                          \
    } else if ((depth_class) == 2) {        \
      constexpr int D = 2;                  \
      __VA_ARGS__;                          \
    } else {                                \
      constexpr int D = SPK_MAX_DEPTH;      \
      __VA_ARGS__;                          \
    }                                       \
  } while (0)

// output sinks of the write interpreter: output byte q
struct NDirect {  // straight to memory at base + q
  uint8_t *base;
  __device__ __forceinline__ void put(uint64_t q, const uint8_t *src, uint64_t n) const {
    n_copy(base + q, src, n);
  }
  __device__ __forceinline__ void byte(uint64_t q, uint32_t b) const { base[q] = (uint8_t)b; }
};
struct NWin {  // the part inside an LDS window holding output bytes [lo, hi)
  uint8_t *lds;
  uint64_t lo, hi;
  __device__ __forceinline__ void put(uint64_t q, const uint8_t *src, uint64_t n) const {
    const uint64_t a = q > lo ? q : lo;
    const uint64_t b = q + n < hi ? q + n : hi;
    if (a >= b) return;
    uint64_t i = a - q;
    const uint64_t e = b - q;
    uint8_t *d = lds + (q - lo);
    for (; i + 16 <= e; i += 16) {  // wide unaligned loads, byte stores into LDS
      const v4u_t v = *reinterpret_cast<const v4u_una *>(src + i);
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) d[i + k] = (uint8_t)(x[k >> 2] >> (8 * (k & 3)));
    }
    for (; i < e; ++i) d[i] = src[i];
  }
  __device__ __forceinline__ void byte(uint64_t q, uint32_t b) const {
    if (q >= lo && q < hi) lds[q - lo] = (uint8_t)b;
  }
};
template <typename Sk>
__device__ __forceinline__ void n_put_le(const Sk &sk, uint64_t q, uint64_t v, uint32_t w) {
  for (uint32_t b = 0; b < w; ++b) sk.byte(q + b, (uint32_t)(v >> (8 * b)) & 0xFFu);
}
// the fast-varint group (packer.hpp:152-235) at q; returns the position past it
template <typename Sk>
__device__ uint64_t n_fv_write(const NLayout &N, const uint8_t *rec, const Sk &sk, uint64_t q0) {
  if (!N.fv_cnt) return q0;
  const uint32_t code = n_fv_code(N, rec), wb = 1u << code;
  uint64_t bits = 0, q = q0 + N.fv_bits;
  uint32_t j = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_FVAR) continue;
    const uint64_t v = n_fv_raw(op, rec);
    if (v) {
      bits |= 1ull << j;
      const uint32_t rw = wb < op.size ? wb : op.size;
      n_put_le(sk, q, v, rw);
      q += rw;
    }
    ++j;
  }
  bits |= (uint64_t)code << N.fv_cnt;
  n_put_le(sk, q0, bits, N.fv_bits);
  return q;
}

// ---- encode: size of one record (or of an op range of it) ----------------------
struct NSize {
  uint64_t bytes, cnts, maxc;  // payload bytes w/o counts, count fields, longest container
  uint64_t cbytes, ccnts;      // of which in the version passes (compatible members)
};
// calculate_one_size (calculate_size.hpp:39-183) of ops [i0, i1) of `rec`;
// `top`: the whole top-level record (its fast-varint group counts too)
template <int D>
__device__ NSize n_size(const NLayout &N, const uint8_t *rec, const uint8_t *const *heaps,
                        uint32_t i0, uint32_t i1, bool top) {
  NSize s = {0, 0, 0, 0, 0};
  if (top) s.bytes = n_fv_size(N, rec);
  NStk<D> st;
  uint32_t d = 0, i = i0, iend = i1;
  uint32_t cd = 0;  // depth of an open compatible group (its bytes are version-pass bytes)
  const uint8_t *r = rec;
  for (;;) {
    if (i >= iend) {
      if (!d) break;
      NFrame &f = st.top;
      if (++f.j < f.cnt) {
        r = f.el + f.j * N.ops[f.aop].size;
        i = f.first;
        continue;
      }
      i = f.ret;
      iend = f.pend;
      r = f.prec;
      if (cd == d) cd = 0;
      st.pop(--d);
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_FVAR) {  // in the group
      ++i;
    } else if (op.kind == SPK_OP_COPY) {
      s.bytes += op.size;
      if (cd) s.cbytes += op.size;
      ++i;
    } else if (op.kind == SPK_OP_VARINT) {
      const uint32_t b = n_vi_len(n_vi_value(op, r));
      s.bytes += b;
      if (cd) s.cbytes += b;
      ++i;
    } else if (n_group(op.kind)) {  // [index / has_value:1] + the active group
      s.bytes += 1;
      if (cd || op.kind == SPK_OP_CGROUP) s.cbytes += 1;
      const int a = n_active(N, i, r);
      if (a < 0) {
        i = N.end[i] + 1u;
        continue;
      }
      const uint32_t a0 = n_alt_start(N, i, (uint32_t)a);
      st.push(d++, NFrame{i, iend, 0, 1, r, r, a0, (uint32_t)N.end[i] + 1u});
      if (op.kind == SPK_OP_CGROUP) cd = d;
      iend = n_alt_end(N, a0);
      i = a0;
    } else {
      const uint64_t c = *reinterpret_cast<const uint32_t *>(r + op.rec_off);
      if (op.kind == SPK_OP_OPTION || op.kind == SPK_OP_COMPAT) {  // calculate_size.hpp:100-105
        const uint64_t b = 1 + (c ? op.size : 0);
        s.bytes += b;
        if (cd || op.kind == SPK_OP_COMPAT) s.cbytes += b;
        ++i;
        continue;
      }
      s.cnts += 1;
      if (cd) s.ccnts += 1;
      if (c > s.maxc) s.maxc = c;
      if (op.kind == SPK_OP_SPAN) {
        s.bytes += c * op.size;
        if (cd) s.cbytes += c * op.size;
        ++i;
      } else if (!c) {
        i = N.end[i] + 1;
      } else {
        const uint64_t off = *reinterpret_cast<const uint64_t *>(r + op.aux);
        const uint8_t *el = heaps[N.heap[i]] + off * op.size;
        st.push(d++, NFrame{i, iend, 0, c, el, r, i + 1, (uint32_t)N.end[i] + 1u});
        r = el;
        iend = N.end[i];
        ++i;
      }
    }
  }
  return s;
}

// ---- encode: bytes of one record (or of an op range of it) at output byte q ------
template <int D, typename Sk>
__device__ uint64_t n_write(const NLayout &N, const uint8_t *rec, const uint8_t *const *heaps,
                            uint32_t w, const Sk &sk, uint64_t q, uint32_t i0, uint32_t i1,
                            bool top) {
  NStk<D> st;
  uint32_t d = 0, i = i0, iend = i1;
  const uint8_t *r = rec;
  if (top) q = n_fv_write(N, rec, sk, q);  // before the members (packer.hpp:432-440)
  for (;;) {
    if (i >= iend) {
      if (!d) break;
      NFrame &f = st.top;
      if (++f.j < f.cnt) {
        r = f.el + f.j * N.ops[f.aop].size;
        i = f.first;
        continue;
      }
      i = f.ret;
      iend = f.pend;
      r = f.prec;
      st.pop(--d);
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_FVAR) {
      ++i;
    } else if (op.kind == SPK_OP_COPY) {
      sk.put(q, r + op.rec_off, op.size);
      q += op.size;
      ++i;
    } else if (op.kind == SPK_OP_VARINT) {
      uint64_t v = n_vi_value(op, r);
      while (v >= 0x80) {
        sk.byte(q++, (uint32_t)(v | 0x80u) & 0xFFu);
        v >>= 7;
      }
      sk.byte(q++, (uint32_t)v);
      ++i;
    } else if (op.kind == SPK_OP_COMPAT || op.kind == SPK_OP_CGROUP) {
      // version UINT64_MAX: nothing (packer.hpp:246-249); written by the
      // version pass of its version
      i = op.kind == SPK_OP_CGROUP ? N.end[i] + 1u : i + 1u;
    } else if (n_group(op.kind)) {
      // variant: [index:1] (packer.hpp:389-398); optional / expected:
      // [has_value:1] (:382-388, :400-410); then the active group
      const uint32_t v = *reinterpret_cast<const uint32_t *>(r + op.rec_off);
      sk.byte(q++, op.kind == SPK_OP_VARIANT ? (v & 0xFFu) : (v ? 1u : 0u));
      const int a = n_active(N, i, r);
      if (a < 0) {
        i = N.end[i] + 1u;
        continue;
      }
      const uint32_t a0 = n_alt_start(N, i, (uint32_t)a);
      st.push(d++, NFrame{i, iend, 0, 1, r, r, a0, (uint32_t)N.end[i] + 1u});
      iend = n_alt_end(N, a0);
      i = a0;
    } else {
      const uint64_t c = *reinterpret_cast<const uint32_t *>(r + op.rec_off);
      const uint64_t off = *reinterpret_cast<const uint64_t *>(r + op.aux);
      if (op.kind == SPK_OP_OPTION) {
        sk.byte(q++, c ? 1u : 0u);
        if (c) {
          sk.put(q, heaps[N.heap[i]] + off * op.size, op.size);
          q += op.size;
        }
        ++i;
        continue;
      }
      n_put_le(sk, q, c, w);
      q += w;
      if (op.kind == SPK_OP_SPAN) {
        sk.put(q, heaps[N.heap[i]] + off * op.size, c * op.size);
        q += c * op.size;
        ++i;
      } else if (!c) {
        i = N.end[i] + 1;
      } else {
        const uint8_t *el = heaps[N.heap[i]] + off * op.size;
        st.push(d++, NFrame{i, iend, 0, c, el, r, i + 1, (uint32_t)N.end[i] + 1u});
        r = el;
        iend = N.end[i];
        ++i;
      }
    }
  }
  return q;
}

// ---- compatible members: the version pass of rank rk over one top-level record ----
// (COMPAT / CGROUP ops sit at the top level only: spk_layout_check)
template <int D>
__device__ uint64_t n_compat_size(const NLayout &N, const uint8_t *rec,
                                  const uint8_t *const *heaps, uint32_t rk, uint32_t w) {
  uint64_t b = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    if (N.crank[i] != rk) continue;
    const uint32_t has = *reinterpret_cast<const uint32_t *>(rec + N.ops[i].rec_off);
    if (N.ops[i].kind == SPK_OP_COMPAT) {
      b += 1 + (has ? N.ops[i].size : 0);
    } else if (N.ops[i].kind == SPK_OP_CGROUP) {
      b += 1;
      if (has) {
        const NSize g = n_size<D>(N, rec, heaps, i + 1, N.end[i], false);
        b += g.bytes + g.cnts * w;
      }
    }
  }
  return b;
}
// packer.hpp:453-461: [has_value:1][U if present] per member of that version
template <int D, typename Sk>
__device__ uint64_t n_write_compat(const NLayout &N, const uint8_t *rec,
                                   const uint8_t *const *heaps, uint32_t rk, uint32_t w,
                                   const Sk &sk, uint64_t q) {
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if ((op.kind != SPK_OP_COMPAT && op.kind != SPK_OP_CGROUP) || N.crank[i] != rk) continue;
    const uint32_t c = *reinterpret_cast<const uint32_t *>(rec + op.rec_off);
    sk.byte(q++, c ? 1u : 0u);
    if (!c) continue;
    if (op.kind == SPK_OP_CGROUP) {
      q = n_write<D>(N, rec, heaps, w, sk, q, i + 1, N.end[i], false);
    } else {
      const uint64_t off = *reinterpret_cast<const uint64_t *>(rec + op.aux);
      sk.put(q, heaps[N.heap[i]] + off * op.size, op.size);
      q += op.size;
    }
  }
  return q;
}

// ---- decode: one record (or an op range of it) from the wire ---------------------
// A bounded walk (speculation from a guessed start, `end` short of the wire's
// end) gives up with kNLimit wherever a read would need bytes past `end`: its
// result is then unknown, never a different decode.
constexpr int32_t kNLimit = 0x7FFF0001;
// Parses wire[pos, end) and advances pos. used[k]: next element slot of heap
// k (counted even when nothing is written). With `rec` set, writes the record,
// its element records and heap payloads, skipping (and flagging in *ovf) what
// does not fit heap_cap. Any non-zero OPTION / OPTGROUP byte is "has value";
// a value that does not fit leaves the reader in place (a trivially
// serializable one zero-filled) (unpacker.hpp:1251-1277). `top`: the whole
// top-level record, its fast-varint group first.
// D: the layout's depth class (n_dclass); the stack's top frame in registers
// and, for D <= 2, the one below it too (a runtime-indexed frame array lives in
// scratch memory)
template <int D = (int)SPK_MAX_DEPTH, typename Rd>
__device__ int32_t n_read(const NLayout &N, const Rd &wire, uint64_t &pos, uint64_t end,
                          uint32_t w, uint8_t *rec, uint8_t *const *heaps, uint64_t *used,
                          const uint64_t *heap_cap, uint32_t *ovf, uint32_t i0, uint32_t i1,
                          bool top, bool bounded = false) {
  NStk<D> st;
  uint32_t d = 0, i = i0, iend = i1;
  uint8_t *r = rec;
  int32_t ec = SPK_ERRC_OK;
  if (top && N.fv_cnt && (ec = n_fv_read(N, wire, pos, end, rec)))
    return bounded && ec == SPK_ERRC_NO_BUFFER_SPACE ? kNLimit : ec;
  for (;;) {
    if (ec) {
      // unwind to the innermost variant / optional / expected group: their
      // decode's errc is dropped (variant_construct_helper::run,
      // unpacker.hpp:476-490; optional / expected, :1251-1277); an ARRAY
      // keeps its failing element (emplace_back, unpacker.hpp:1208-1226)
      // The members from the failing one on, at every level unwound, are
      // value-initialised (zero_rest): the reference default-constructs the
      // value before its decode, and the output may hold anything.
      bool dropped = false;
      for (;;) {
        if (r) zero_rest(N, r, i, iend);
        if (!d) break;
        const NFrame &f = st.top;
        const spk_op &fo = N.ops[f.aop];
        if (fo.kind == SPK_OP_VARIANT || fo.kind == SPK_OP_OPTGROUP) {
          i = f.ret;
          iend = f.pend;
          r = const_cast<uint8_t *>(f.prec);
          st.pop(--d);
          dropped = true;
          break;
        }
        used[N.heap[f.aop]] -= f.cnt - (f.j + 1);
        if (f.el) *reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(f.prec) + fo.rec_off) =
            (uint32_t)(f.j + 1);
        i = f.ret;  // the rest of the enclosing level
        iend = f.pend;
        r = const_cast<uint8_t *>(f.prec);
        st.pop(--d);
      }
      if (!dropped) return ec;
      ec = SPK_ERRC_OK;
      continue;
    }
    if (i >= iend) {
      if (!d) break;
      NFrame &f = st.top;
      if (++f.j < f.cnt) {
        r = f.el ? const_cast<uint8_t *>(f.el) + f.j * N.ops[f.aop].size : nullptr;
        i = f.first;
        continue;
      }
      i = f.ret;
      iend = f.pend;
      r = const_cast<uint8_t *>(f.prec);
      st.pop(--d);
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_FVAR) {  // read with the group
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_COPY) {
      if (end - pos < op.size) {
        if (bounded) return kNLimit;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      if (r) n_copy_rd(r + op.rec_off, wire, pos, op.size);
      pos += op.size;
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_VARINT) {  // deserialize_varint (varint.hpp:270-330)
      uint64_t v = 0;
      int32_t vec = SPK_ERRC_INVALID_BUFFER;  // 10 bytes, all continued
      for (uint32_t k = 0; k < 10; ++k) {
        if (pos >= end) {
          if (bounded) return kNLimit;
          vec = SPK_ERRC_NO_BUFFER_SPACE;  // (the bytes read stay consumed)
          break;
        }
        const uint8_t b = wire[pos++];
        v |= (uint64_t)(b & 0x7fu) << (7 * k);
        if (!(b & 0x80u)) {
          vec = SPK_ERRC_OK;
          break;
        }
      }
      if (vec) {
        ec = vec;
        continue;
      }
      if (r) {
        if (op.aux & SPK_VARINT_ZIGZAG) v = (v >> 1) ^ (uint64_t)(-(int64_t)(v & 1));
        if (op.size == 4)
          *reinterpret_cast<uint32_t *>(r + op.rec_off) = (uint32_t)v;
        else
          *reinterpret_cast<uint64_t *>(r + op.rec_off) = v;
      }
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_VARIANT || op.kind == SPK_OP_OPTGROUP) {
      // variant: unpacker.hpp:1278-1292; optional / expected: :1251-1277
      if (pos >= end) {
        if (bounded) return kNLimit;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      const uint32_t b = wire[pos++];
      int a;
      if (op.kind == SPK_OP_VARIANT) {
        if (b >= op.size) { ec = SPK_ERRC_INVALID_BUFFER; continue; }
        a = (int)b;
        if (r) *reinterpret_cast<uint32_t *>(r + op.rec_off) = b;
      } else {
        a = b ? 0 : (op.size == 2 ? 1 : -1);
        if (r) *reinterpret_cast<uint32_t *>(r + op.rec_off) = b ? 1u : 0u;
      }
      if (a < 0) {
        i = N.end[i] + 1u;
        continue;
      }
      const uint32_t a0 = n_alt_start(N, i, (uint32_t)a);
      if (d == (uint32_t)D) { ec = SPK_ERRC_INVALID_BUFFER; continue; }  // (n_dclass bounds it)
      st.push(d++, NFrame{i, iend, 0, 1, r, r, a0, (uint32_t)N.end[i] + 1});
      iend = n_alt_end(N, a0);
      i = a0;
      continue;
    }
    if (op.kind == SPK_OP_CGROUP) {  // absent until its version pass
      if (r) *reinterpret_cast<uint32_t *>(r + op.rec_off) = 0;
      i = N.end[i] + 1u;
      continue;
    }
    const uint32_t hk = N.heap[i];
    if (op.kind == SPK_OP_COMPAT) {  // absent until its version pass
      if (r) {
        *reinterpret_cast<uint32_t *>(r + op.rec_off) = 0;
        *reinterpret_cast<uint64_t *>(r + op.aux) = used[hk];
      }
      ++i;
      continue;
    }
    const uint32_t pw = op.kind == SPK_OP_OPTION ? 1u : w;
    if (end - pos < pw) {
      if (bounded) return kNLimit;
      ec = SPK_ERRC_NO_BUFFER_SPACE;
      continue;
    }
    uint64_t cnt;
    if (op.kind == SPK_OP_OPTION) {
      cnt = wire[pos] != 0;
    } else {
      cnt = 0;
      for (uint32_t b = 0; b < w; ++b) cnt |= (uint64_t)wire[pos + b] << (8 * b);
    }
    pos += pw;
    const uint64_t off = used[hk];
    bool put = r != nullptr;
    // slots an ARRAY can fill: an element takes at least one byte, so at most
    // (bytes left + 1) get decoded (the last one may fail and stay)
    // (a SPAN whose payload is not there fails below without using its heap)
    uint64_t snb = 0;
    const bool sfit = op.kind == SPK_OP_SPAN && span_nb(cnt, op.size, &snb) && snb <= end - pos;
    const uint64_t need = op.kind == SPK_OP_ARRAY ? (cnt > end - pos ? end - pos + 1 : cnt)
                          : op.kind == SPK_OP_SPAN && !sfit ? 0
                                                            : cnt;
    if (put && (need > 0xFFFFFFFFull || need > heap_cap[hk] - (off < heap_cap[hk] ? off : heap_cap[hk]))) {
      *ovf = 1;
      put = false;
    }
    // a SPAN's fields are set only once its payload is there (the reference
    // checks before it resizes: a failing string stays empty)
    if (put && op.kind != SPK_OP_SPAN) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = (uint32_t)cnt;
      *reinterpret_cast<uint64_t *>(r + op.aux) = off;
    }
    if (op.kind == SPK_OP_ARRAY) {
      // (an element takes at least one wire byte: a bounded walk gives up on
      // a count the bytes left cannot hold)
      if (bounded && cnt > end - pos) return kNLimit;
      used[hk] = off + cnt;
      if (!cnt) {
        i = N.end[i] + 1;
        continue;
      }
      if (d == (uint32_t)D) { ec = SPK_ERRC_INVALID_BUFFER; continue; }  // (layout_check bounds it)
      st.push(d++, NFrame{i, iend, 0, cnt, put ? heaps[hk] + off * op.size : nullptr, r, i + 1,
                          (uint32_t)N.end[i] + 1});
      r = put ? heaps[hk] + off * op.size : nullptr;
      iend = N.end[i];
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_OPTION) {
      if (cnt) {
        const bool fits = end - pos >= op.size;
        if (!fits && bounded) return kNLimit;
        if (put) {
          if (fits)
            n_copy_rd(heaps[hk] + off * op.size, wire, pos, op.size);
          else
            for (uint32_t b = 0; b < op.size; ++b) heaps[hk][off * op.size + b] = 0;
        }
        if (fits) pos += op.size;
      }
      used[hk] = off + cnt;
      ++i;
      continue;
    }
    // SPAN (unpacker.hpp:1127-1156): the whole payload must be present
    if (cnt) {
      if (!sfit) {
        if (bounded) return kNLimit;
        ec = SPK_ERRC_NO_BUFFER_SPACE;
        continue;
      }
      const uint64_t nb = cnt * op.size;
      if (put) n_copy_rd(heaps[hk] + off * op.size, wire, pos, nb);
      pos += nb;
    }
    if (put) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = (uint32_t)cnt;
      *reinterpret_cast<uint64_t *>(r + op.aux) = off;
    }
    used[hk] = off + cnt;
    ++i;
  }
  return SPK_ERRC_OK;
}

// unpacker.hpp:1354-1376 over one record: a member whose has byte would start
// at or past data_end ends every version pass without an error (returns 1,
// size_type_ = UCHAR_MAX, :360-365); a missing has byte before it is
// no_buffer_space (*ec, returns 1); the value's errc is dropped (a trivially
// serializable one that does not fit reads as present and zero; a group stops
// where its decode stopped). The main pass left every member absent.
template <int D = (int)SPK_MAX_DEPTH, typename Rd>
__device__ int n_read_compat(const NLayout &N, const Rd &wire, uint64_t &pos, uint64_t end,
                             uint64_t data_end, uint32_t rk, uint32_t w, uint8_t *rec,
                             uint8_t *const *heaps, uint64_t *used, const uint64_t *heap_cap,
                             uint32_t *ovf, int32_t *ec) {
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if ((op.kind != SPK_OP_COMPAT && op.kind != SPK_OP_CGROUP) || N.crank[i] != rk) continue;
    if (pos >= data_end) return 1;
    if (pos >= end) {
      *ec = SPK_ERRC_NO_BUFFER_SPACE;
      return 1;
    }
    if (!wire[pos++]) continue;
    if (op.kind == SPK_OP_CGROUP) {
      if (rec) *reinterpret_cast<uint32_t *>(rec + op.rec_off) = 1;
      (void)n_read<D>(N, wire, pos, end, w, rec, heaps, used, heap_cap, ovf, i + 1, N.end[i], false);
      continue;
    }
    const bool fits = end - pos >= op.size;
    const uint32_t hk = N.heap[i];
    const uint64_t off = used[hk];
    if (rec) {
      if (off >= heap_cap[hk]) {
        *ovf = 1;
      } else {
        *reinterpret_cast<uint32_t *>(rec + op.rec_off) = 1;
        *reinterpret_cast<uint64_t *>(rec + op.aux) = off;
        if (fits)
          n_copy_rd(heaps[hk] + off * op.size, wire, pos, op.size);
        else
          for (uint32_t b = 0; b < op.size; ++b) heaps[hk][off * op.size + b] = 0;
      }
    }
    used[hk] = off + 1;
    if (fits) pos += op.size;
  }
  return 0;
}

// ---- device-wide exclusive scan of C u64 columns [C][n] (in place) ---------------
constexpr uint32_t kNScanT = 256, kNScanIPT = 8;
constexpr uint64_t kNScanBlk = (uint64_t)kNScanT * kNScanIPT;
constexpr uint64_t kNScanFold = 2048;

__device__ __forceinline__ uint64_t n_block_excl(uint64_t v, uint64_t *sh, uint64_t *tot) {
  const uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < kNScanT; o <<= 1) {
    const uint64_t x = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  const uint64_t incl = sh[t];
  *tot = sh[kNScanT - 1];
  __syncthreads();
  return incl - v;
}

// plan token of the VECTOR encode (see nest_tok_hash below)
constexpr size_t kWsPlanTok = 1536;  // [1536, 2048) is free (spk_internal.hpp)
constexpr unsigned long long kTokMagic = 0x4e53504b544f4b31ull;
struct NTok {
  unsigned long long magic, n, recs, heaps, layout, tot0, maxc, hash;
  unsigned long long chk;  // the encode's hash of the same column
  uint32_t stale, pad_;
};
static_assert(kWsPlanTok + sizeof(NTok) <= kWsCtl, "NTok overlaps the control block");

// cond (device, non-null): the kernel runs only while *cond is non-zero (the
// encode: NTok::stale; a compatible-member VECTOR decode: CompatCtl::serial)
__device__ __forceinline__ bool tok_skip(const uint8_t *ws, const uint32_t *cond) {
  (void)ws;
  return cond && !*cond;
}

__global__ __launch_bounds__(kNScanT) void nscan_reduce(const uint64_t *__restrict__ col,
                                                        uint64_t n, uint64_t *__restrict__ part,
                                                        uint64_t nb, const uint8_t *ws,
                                                        const uint32_t *cond) {
  __shared__ uint64_t sh[kNScanT];
  if (tok_skip(ws, cond)) return;
  const uint64_t c = blockIdx.y;
  const uint64_t base = (uint64_t)blockIdx.x * kNScanBlk;
  uint64_t s = 0;
  for (uint32_t k = 0; k < kNScanIPT; ++k) {
    const uint64_t i = base + (uint64_t)k * kNScanT + threadIdx.x;
    if (i < n) s += col[c * n + i];
  }
  uint64_t tot;
  n_block_excl(s, sh, &tot);
  if (threadIdx.x == 0) part[c * nb + blockIdx.x] = tot;
}

// one block per column: exclusive scan of the block partials, total at [nb]
__global__ __launch_bounds__(1024) void nscan_top(uint64_t *__restrict__ part, uint64_t nb,
                                                      const uint8_t *ws, const uint32_t *cond) {
  __shared__ uint64_t sh[1024];
  __shared__ uint64_t carry;
  if (tok_skip(ws, cond)) return;
  const uint64_t c = blockIdx.x;
  uint64_t *p = part + c * (nb + 1);
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint64_t b = b0 + threadIdx.x;
    const uint64_t v = b < nb ? p[b] : 0;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
      const uint64_t x = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
      __syncthreads();
      sh[threadIdx.x] += x;
      __syncthreads();
    }
    const uint64_t incl = sh[threadIdx.x];
    const uint64_t cy = carry;
    if (b < nb) p[b] = cy + incl - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = cy + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) p[nb] = carry;
}

__device__ __forceinline__ uint64_t n_wave_incl(uint64_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint64_t x = __shfl_up(v, o);
    if (lane >= o) v += x;
  }
  return v;
}
// sum over the block (every thread gets it)
__device__ __forceinline__ uint64_t n_block_sum(uint64_t v, uint64_t *sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (uint32_t w = 0; w < kNScanT / 64; ++w) t += sh[w];
  __syncthreads();
  return t;
}
// Each wave scans 512 consecutive elements loaded 64 at a time (coalesced;
// round 4 loaded 8 consecutive per thread: every load instruction touched 64
// lines). fold: the block adds up the partial sums of the blocks before it
// (nscan_top not launched; block 0 writes the column total at [nb]).
__global__ __launch_bounds__(kNScanT) void nscan_apply(uint64_t *__restrict__ col, uint64_t n,
                                                       uint64_t *__restrict__ part,
                                                       uint64_t nb, const uint8_t *ws,
                                                       const uint32_t *cond, uint32_t fold) {
  __shared__ uint64_t sh[kNScanT / 64], wsum[kNScanT / 64];
  if (tok_skip(ws, cond)) return;
  const uint64_t c = blockIdx.y;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * kNScanBlk + (uint64_t)wv * 64 * kNScanIPT;
  uint64_t *cc = col + c * n;
  uint64_t v[kNScanIPT], ex[kNScanIPT], run = 0;
#pragma unroll
  for (uint32_t k = 0; k < kNScanIPT; ++k) {
    const uint64_t i = base + (uint64_t)k * 64 + lane;
    v[k] = i < n ? cc[i] : 0;
  }
#pragma unroll
  for (uint32_t k = 0; k < kNScanIPT; ++k) {
    const uint64_t incl = n_wave_incl(v[k], lane);
    ex[k] = run + incl - v[k];
    run += __shfl(incl, 63);
  }
  if (lane == 0) wsum[wv] = run;
  uint64_t *p = part + c * (nb + 1);
  uint64_t carry;
  if (fold) {
    uint64_t before = 0, all = 0;
    for (uint64_t b = threadIdx.x; b < nb; b += kNScanT) {
      const uint64_t x = p[b];
      before += b < blockIdx.x ? x : 0;
      all += x;
    }
    carry = n_block_sum(before, sh);
    if (blockIdx.x == 0) {
      all = n_block_sum(all, sh);
      if (threadIdx.x == 0) p[nb] = all;
    }
  } else {
    carry = p[blockIdx.x];
    __syncthreads();
  }
  uint64_t woff = 0;
  for (uint32_t w = 0; w < wv; ++w) woff += wsum[w];
#pragma unroll
  for (uint32_t k = 0; k < kNScanIPT; ++k) {
    const uint64_t i = base + (uint64_t)k * 64 + lane;
    if (i < n) cc[i] = carry + woff + ex[k];
  }
}

// note: nscan_reduce writes partials with row stride nb; nscan_top/apply read
// them with stride nb + 1 — the host lays the partial table out with nb + 1
// slots per column and passes nb + 1 to the reduce as its stride.
// ws + cond: the encode's conditional size pass (skipped while the plan
// token holds, see NTok); null cond: always run
static hipError_t nscan(uint64_t *col, uint64_t n, uint32_t ncols, uint64_t *part,
                        hipStream_t s, const uint8_t *ws = nullptr,
                        const uint32_t *cond = nullptr) {
  if (!n || !ncols) return hipSuccess;
  const uint64_t nb = (n + kNScanBlk - 1) / kNScanBlk;
  SPK_LAUNCH(nscan_reduce, dim3((unsigned)nb, ncols), dim3(kNScanT), 0, s, (const uint64_t *)col,
             n, part, nb + 1, ws, cond);
  // (up to kNScanFold blocks a column, each apply block adds up the partials
  // before it: one launch less)
  const uint32_t fold = nb <= kNScanFold ? 1u : 0u;
  if (!fold) SPK_LAUNCH(nscan_top, dim3(ncols), dim3(1024), 0, s, part, nb, ws, cond);
  SPK_LAUNCH(nscan_apply, dim3((unsigned)nb, ncols), dim3(kNScanT), 0, s, col, n, part, nb, ws,
             cond, fold);
  return hipGetLastError();
}
static size_t nscan_part_bytes(uint64_t n, uint32_t ncols) {
  return ((n + kNScanBlk - 1) / kNScanBlk + 1) * ncols * 8 + 64;
}

// ---- workspace ------------------------------------------------------------------
struct NWs {
  size_t a, b, part, starts, cpos, end;  // a/b: [C][n] u64 columns; starts: [n] u64
};                                       // cpos: [ranks][n] u64 version-group starts
static NWs nws_layout(uint64_t n, uint32_t n_heaps, uint32_t n_ranks) {
  NWs f = {};
  size_t off = kWsScratch;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  // encode: 2 + n_ranks columns; decode: n_heaps
  const uint32_t cols = (n_heaps > n_ranks ? n_heaps : n_ranks) + 2;
  f.a = take((n + 1) * 8 * cols);
  f.b = take((n + 1) * 8);
  f.part = take(nscan_part_bytes(n + 1, cols));
  f.starts = take((n + 1) * 8);
  f.cpos = take((n + 1) * 8 * (n_ranks ? n_ranks : 1));
  f.end = off;
  return f;
}

// ---- chunked VECTOR decode (layouts without compatible members) -----------------
// The body is cut into kNCh-byte chunks, one lane each. A record starts where
// the previous one ends, so a chunk's first record start (its entry) is known
// only from its predecessor; every lane therefore GUESSES its entry (the
// first byte from which whole records parse up to the chunk's end, a bounded
// walk) and walks its records from there. Records resynchronise, so a lane
// that guessed wrong usually exits where the true path does. Rounds then
// check every entry against the predecessor's exit and re-walk the chunks
// that disagree from that exit (chunk 0's entry is exact), a one-wave fixer
// settles what the rounds left, a scan over the chunks' record counts and heap
// use gives every chunk its first record index and heap bases, and each lane
// decodes its records into place.
constexpr uint32_t kNCh = 1024;        // wire bytes per chunk
constexpr uint32_t kNBound = 4096;     // a speculative walk's reach past its chunk
constexpr int kNRounds = 4;            // parallel re-check rounds
constexpr uint32_t kNT = 128;          // lanes per block of the chunk kernels
constexpr uint64_t kNUnk = ~0ull - 1;  // entry / exit unknown (no plausible start; walk gave up)
constexpr uint64_t kNFail = ~0ull;     // the path failed before this point

struct CWs {
  size_t ent, ext, err, dirty, cols, part, end;  // cols: [1 + heaps][nch] u64 (count, heap use)
};
static uint64_t cws_chunks(uint64_t wire_len) { return wire_len / kNCh + 2; }
static CWs cws_layout(uint64_t wire_len, uint32_t n_heaps) {
  CWs f = {};
  size_t off = kWsScratch;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const uint64_t nch = cws_chunks(wire_len);
  f.ent = take(nch * 8);
  f.ext = take(nch * 8);
  f.err = take(nch * 4);
  f.dirty = take((nch + 63) / 64 * 8);
  f.cols = take(nch * 8 * (1 + n_heaps));
  f.part = take(nscan_part_bytes(nch, 1 + n_heaps));
  f.end = off;
  return f;
}


// a compatible-member VECTOR decode on the tile passes: its CompatCtl, past
// the workspace of every pass and of the one-lane walk behind them
static size_t compat_ctl_off(const spk_layout *L, uint64_t rows, uint64_t wire_len) {
  const NLayout N = make_nlayout(L);
  const size_t b = nws_layout(rows, N.n_heaps, N.n_ranks).end;
  const size_t t = compat_tiles_ws_bytes(L, wire_len);
  return ((b > t ? b : t) + 255) & ~size_t(255);
}

size_t nested_workspace_bytes(const spk_layout *L, int mode, uint64_t n, uint64_t wire_len) {
  const NLayout N = make_nlayout(L);
  size_t b = nws_layout(n, N.n_heaps, N.n_ranks).end;
  if (mode == SPK_MODE_VECTOR && N.n_ranks && compat_tiles_ok(L, wire_len))
    b = compat_ctl_off(L, n, wire_len) + sizeof(CompatCtl);
  if (mode == SPK_MODE_VECTOR && !N.n_ranks) {
    const size_t c = cws_layout(wire_len, N.n_heaps).end;
    if (c > b) b = c;
    if (var_nested_tile_ok(L)) {
      const size_t t = var_nested_tile_ws_bytes(L, wire_len);
      if (t > b) b = t;
    }
  }
  return b + 256;
}

// control block of the nested path (at kWsCtl)
struct NCtl {
  unsigned long long maxc;   // encode: longest container (atomicMax)
  unsigned long long nrec;   // vector decode: records in the message
  unsigned long long end;    // vector decode: position after the last record
  unsigned long long data_len;
  unsigned long long ovf;
  uint32_t w, errc;          // errc: the header's
  // chunked vector decode
  unsigned long long p0;                      // first record start
  unsigned long long nch;                     // chunks
  unsigned long long changed[kNRounds];       // round r moved an exit or left a chunk open
  unsigned long long cmin, cmax, ndirty;      // chunks the rounds left open
  unsigned long long rewalks, fixed;          // chunks re-walked by the rounds / the fixer
  unsigned long long htot[SPK_MAX_SPANS];     // heap elements of records 0..n-1
  int32_t werr;                               // the errc of the record the path fails at
  uint32_t pad_;
  unsigned long long m_ok, m_cap;             // MESSAGES decode: messages ok / over capacity
};
static_assert(kWsCtl + sizeof(NCtl) <= kWsScratch, "NCtl overlaps the scratch area");

// ---- encode kernels ------------------------------------------------------------------
struct NEnc {
  NLayout N;
  uint64_t n;
  int mode;
  uint32_t fixed_w;        // spk_encode_body: imposed width (0: from the plan)
  uint32_t fpre, fseq_off, flen_off, fseq_base;
  SeqEcho echo;
  uint8_t ftmpl[SPK_MAX_FRAME];
  spk_msgfmt fmt;          // the message format of `mode`
  const uint8_t *heaps[SPK_MAX_SPANS];
};

// ---- plan token -----------------------------------------------------------------------
// A VECTOR encode of a layout without compatible members reuses the offsets
// its plan left in the workspace (column 0, the scan totals, maxc). The plan
// leaves a token beside them: the batch (n, records, heaps, layout) and an
// order-free hash of the offsets column, the total and maxc. The encode
// checks it on the device and re-runs the size pass only when it does not
// match (another call used the workspace in between, or no plan preceded),
// so a stale workspace never steers the window writes.
__device__ __forceinline__ uint64_t tok_mix(uint64_t i, uint64_t v) {
  uint64_t z = v + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t tok_heaps(const NEnc &e) {
  uint64_t h = 0;
  for (uint32_t k = 0; k < e.N.n_heaps && k < SPK_MAX_SPANS; ++k)
    h = h * 0x100000001B3ull ^ (uint64_t)(uintptr_t)e.heaps[k];
  return h;
}
static uint64_t tok_layout(const spk_layout *L, int mode = SPK_MODE_VECTOR, uint32_t fpre = 0) {
  // (MESSAGES sizes hold each message's header and frame prefix)
  return ((uint64_t)L->fmt_vector.code << 32) ^ ((uint64_t)L->n_ops << 16) ^ L->rec_stride ^
         ((uint64_t)L->fmt_vector.flags << 48) ^
         (mode == SPK_MODE_VECTOR ? 0ull : 0x9E3779B97F4A7C15ull * (1ull + fpre));
}

// XOR over the records of tok_mix(i, a[i]) into *dst (order-free, one
// atomic per wave)
__global__ __launch_bounds__(256) void nest_tok_hash(const uint64_t *__restrict__ a, uint64_t n,
                                                     unsigned long long *dst) {
  uint64_t h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    h ^= tok_mix(i, a[i]);
  for (int o = 32; o > 0; o >>= 1) h ^= __shfl_xor(h, o);
  // one atomic per block (thousands on one address serialise at its L2 channel)
  __shared__ uint64_t wh[4];
  if ((threadIdx.x & 63) == 0) wh[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t b = wh[0] ^ wh[1] ^ wh[2] ^ wh[3];
    if (b) atomicXor(dst, (unsigned long long)b);
  }
}

// encode: start the check (static fields) and clear the recomputed hash
__global__ void nest_tok_begin(uint8_t *ws, uint64_t n, uint64_t recs, uint64_t heaps,
                               uint64_t layout) {
  NTok *t = reinterpret_cast<NTok *>(ws + kWsPlanTok);
  t->chk = 0;
  t->stale = t->magic != kTokMagic || t->n != n || t->recs != recs || t->heaps != heaps ||
             t->layout != layout;
}

// encode: the verdict (hash, total, maxc); a stale token is dropped
__global__ void nest_tok_verdict(uint8_t *ws, const uint64_t *__restrict__ part, uint64_t nb,
                                 uint64_t n) {
  NTok *t = reinterpret_cast<NTok *>(ws + kWsPlanTok);
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t tot0 = n ? part[nb] : 0;
  const uint32_t stale = t->stale || t->chk != t->hash || t->tot0 != tot0 || t->maxc != ctl->maxc;
  t->stale = stale;
  if (stale) t->magic = 0;
}


// a[0][i] = payload bytes, a[1][i] = count fields (VECTOR) or the whole
// message size (MESSAGES); the longest container into ctl->maxc
// the block's records staged in LDS with coalesced 16-B loads when they fit:
// the interpreter's reads of one record's count fields are dependent (one
// load per op), so from LDS they cost LDS latencies, not HBM ones
constexpr uint32_t kNSizeStage = 28 * 1024;
template <int D>
__global__ __launch_bounds__(256) void nest_size(NEnc e, const uint8_t *__restrict__ recs,
                                                 uint64_t *__restrict__ a, uint8_t *ws,
                                                 const uint32_t *cond) {
  __shared__ NLayout N;
  __shared__ __align__(16) uint8_t rs[kNSizeStage];
  if (tok_skip(ws, cond)) return;
  n_stage(N, e.N);
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x;
  const uint64_t nb = r0 < e.n ? (e.n - r0 < blockDim.x ? e.n - r0 : blockDim.x) : 0;
  const uint64_t bytes = nb * N.stride;
  // (device records are 8-aligned, their stride a multiple of 8)
  const bool staged = (uint64_t)blockDim.x * N.stride <= kNSizeStage && !(N.stride & 7) &&
                      !((uintptr_t)recs & 7);
  if (staged) {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(recs + r0 * N.stride);
    uint64_t *dst = reinterpret_cast<uint64_t *>(rs);
    for (uint64_t k = threadIdx.x; k < bytes / 8; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
  }
  uint64_t m = 0;
  if (i < e.n) {
    const uint8_t *rec = staged ? rs + (i - r0) * N.stride : recs + i * N.stride;
    const NSize s = n_size<D>(N, rec, e.heaps, 0, N.n_ops, true);
    m = s.maxc;
    if (e.mode == SPK_MODE_MESSAGES) {
      const uint32_t w = width_of(s.maxc);
      const uint64_t body = s.bytes + s.cnts * w;
      const uint32_t hl = N.n_ranks ? compat_hdr(nullptr, e.fmt, w, body)
                                      : hdr_shape(e.fmt.flags, e.fmt.literal_len, w).len;
      a[i] = e.fpre + hl + body;
      a[e.n + i] = s.bytes;
    } else {
      // main pass bytes and count fields (the version passes' columns
      // need the width: nest_vec_sizes)
      a[i] = s.bytes - s.cbytes;
      a[e.n + i] = s.cnts - s.ccnts;
    }
  }
  // wave max -> an atomic only when it raises the running maximum (one
  // atomic per wave on one address serialises 10M-record batches)
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(m, o);
    m = x > m ? x : m;
  }
  if ((threadIdx.x & 63) == 0 && m &&
      m > __hip_atomic_load(&ctl->maxc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(&ctl->maxc, (unsigned long long)m);
}

__global__ void nest_ctl_init(uint8_t *ws, const uint32_t *cond) {
  if (tok_skip(ws, cond)) return;
  if (!cond) {  // an unconditional size pass (a plan) drops any earlier token
    NTok *t = reinterpret_cast<NTok *>(ws + kWsPlanTok);
    t->magic = 0;
    t->hash = 0;
  }
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  ctl->maxc = 0;
  ctl->nrec = 0;
  ctl->end = 0;
  ctl->data_len = 0;
  ctl->ovf = 0;
  ctl->w = 1;
  ctl->errc = 0;
  ctl->m_ok = 0;
  ctl->m_cap = 0;
}

// VECTOR: sizes[i] = bytes + cnts * w (in place over a[0]), w from maxc;
// column 2 + rk: the bytes of record i in the version pass of rank rk
template <int D>
__global__ void nest_vec_sizes(NEnc e, const uint8_t *__restrict__ recs,
                               uint64_t *__restrict__ a, uint8_t *ws,
                               const uint32_t *cond) {
  __shared__ NLayout N;
  if (tok_skip(ws, cond)) return;
  n_stage(N, e.N);
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t mx = ctl->maxc > e.n ? ctl->maxc : e.n;
  const uint32_t w = e.fixed_w ? e.fixed_w : width_of(mx);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < e.n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    a[i] = a[i] + a[e.n + i] * w;
    for (uint32_t rk = 0; rk < N.n_ranks; ++rk)
      a[(2 + rk) * e.n + i] = n_compat_size<D>(N, recs + i * N.stride, e.heaps, rk, w);
  }
}

// plan result from the column sums (part tables after the scan)
// (VECTOR without compatible members: also the plan token, tok_* set, whose
// hash nest_tok_hash accumulated)
__global__ void nest_plan_fin(NEnc e, const uint64_t *__restrict__ a,
                              const uint64_t *__restrict__ part, uint64_t nb, uint8_t *ws,
                              spk_plan_t *plan, uint32_t tok, uint64_t recs, uint64_t heaps,
                              uint64_t layout) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  if (tok) {
    NTok *t = reinterpret_cast<NTok *>(ws + kWsPlanTok);
    t->n = e.n;
    t->recs = recs;
    t->heaps = heaps;
    t->layout = layout;
    t->tot0 = e.n ? part[nb] : 0;
    t->maxc = ctl->maxc;
    t->magic = kTokMagic;
  }
  spk_plan_t p = {};
  const uint64_t tot0 = e.n ? part[nb] : 0;                 // column 0 total
  const uint64_t tot1 = e.n ? part[(nb + 1) + nb] : 0;      // column 1 total
  if (e.mode == SPK_MODE_VECTOR) {
    const uint64_t mx = ctl->maxc > e.n ? ctl->maxc : e.n;
    const uint32_t w = width_of(mx);
    const HdrShape h = hdr_shape(e.fmt.flags, e.fmt.literal_len, w);
    uint64_t totc = 0;  // the version passes
    for (uint32_t rk = 0; rk < e.N.n_ranks; ++rk)
      totc += e.n ? part[(2 + rk) * (nb + 1) + nb] : 0;
    uint32_t hl = h.len, meta = h.meta, has_meta = h.has_meta;
    if (e.N.n_ranks) {
      uint8_t hb[4 + 1 + 8 + SPK_MAX_LITERAL + 1];
      hl = compat_hdr(hb, e.fmt, w, w + tot0 + totc);
      meta = hb[4];
      has_meta = 1;
    }
    p.max_count = mx;
    p.width = w;
    p.header_bytes = hl + w;
    p.metainfo = meta;
    p.has_meta = has_meta;
    p.var_bytes = tot0 - tot1 * w + totc;  // column 0 holds bytes + counts * w
    p.total_bytes = hl + w + tot0 + totc;
  } else {
    p.max_count = ctl->maxc;
    p.width = width_of(ctl->maxc);
    p.var_bytes = tot1;
    p.total_bytes = tot0;
  }
  *plan = p;
}

// record i's bytes at its scanned offset (after the VECTOR header, or its
// message with header and frame in MESSAGES mode)
template <int D>
__global__ __launch_bounds__(256) void nest_write(NEnc e, const uint8_t *__restrict__ recs,
                                                  const uint64_t *__restrict__ off,
                                                  const uint64_t *__restrict__ part, uint64_t nb,
                                                  uint8_t *ws, uint8_t *__restrict__ out,
                                                  uint64_t *__restrict__ msg_offsets,
                                                  uint32_t with_header, uint64_t out_cap) {
  __shared__ NLayout N;
  n_stage(N, e.N);
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e.mode == SPK_MODE_VECTOR) {
    const uint64_t mx = ctl->maxc > e.n ? ctl->maxc : e.n;
    const uint32_t w = e.fixed_w ? e.fixed_w : width_of(mx);
    uint32_t hl = 0;
    const uint64_t tot0 = e.n ? part[nb] : 0;
    uint64_t totc = 0;
    for (uint32_t rk = 0; rk < N.n_ranks; ++rk) totc += e.n ? part[(2 + rk) * (nb + 1) + nb] : 0;
    // (the header straight into the output by thread 0: a local byte array
    // indexed at run time would live in scratch memory for every lane)
    if (with_header)
      hl = N.n_ranks ? compat_hdr(nullptr, e.fmt, w, w + tot0 + totc)
                     : hdr_shape(e.fmt.flags, e.fmt.literal_len, w).len;
    // the whole message must fit, or nothing is written (spk_encode's
    // contract; the caller reads the plan's total_bytes)
    if ((with_header ? hl + w : 0) + tot0 + totc > out_cap) return;
    if (with_header) {
      if (i == 0) {
        if (N.n_ranks)
          compat_hdr(out, e.fmt, w, w + tot0 + totc);
        else
          write_hdr(out, e.fmt, w);
        for (uint32_t b = 0; b < w; ++b) out[hl + b] = (uint8_t)(e.n >> (8 * b));
      }
      hl += w;
    }
    if (i < e.n) {
      const uint8_t *rec = recs + i * N.stride;
      const NDirect sk{out};
      n_write<D>(N, rec, e.heaps, w, sk, hl + off[i], 0, N.n_ops, true);
      // version passes after every record's main pass (packer.hpp:66-78)
      uint64_t sec = hl + tot0;
      for (uint32_t rk = 0; rk < N.n_ranks; ++rk) {
        n_write_compat<D>(N, rec, e.heaps, rk, w, sk, sec + off[(2 + rk) * e.n + i]);
        sec += part[(2 + rk) * (nb + 1) + nb];
      }
    }
    return;
  }
  if ((e.n ? part[nb] : 0) > out_cap) return;  // every message with its frame
  if (i == 0 && msg_offsets) msg_offsets[e.n] = e.n ? part[nb] : 0;
  if (i >= e.n) return;
  const uint8_t *rec = recs + i * N.stride;
  const NSize s = n_size<D>(N, rec, e.heaps, 0, N.n_ops, true);
  const uint32_t w = width_of(s.maxc);
  uint8_t *p = out + off[i];
  if (msg_offsets) msg_offsets[i] = off[i];
  uint8_t *m = p + e.fpre;
  const uint32_t hl = N.n_ranks ? compat_hdr(m, e.fmt, w, s.bytes + s.cnts * w)
                                  : write_hdr(m, e.fmt, w);
  const NDirect sk{m};
  uint64_t qo = n_write<D>(N, rec, e.heaps, w, sk, hl, 0, N.n_ops, true);
  for (uint32_t rk = 0; rk < N.n_ranks; ++rk) qo = n_write_compat<D>(N, rec, e.heaps, rk, w, sk, qo);
  uint8_t *q = m + qo;
  if (e.fpre) {
    for (uint32_t b = 0; b < e.fpre; ++b) p[b] = e.ftmpl[b];
    const uint32_t mlen = (uint32_t)(q - m);
    if (e.fseq_off != SPK_FRAME_NONE) {
      const uint32_t sq = seq_value(e.echo, e.fseq_base, i);
      for (uint32_t b = 0; b < 4; ++b) p[e.fseq_off + b] = (uint8_t)(sq >> (8 * b));
    }
    if (e.flen_off != SPK_FRAME_NONE)
      for (uint32_t b = 0; b < 4; ++b) p[e.flen_off + b] = (uint8_t)(mlen >> (8 * b));
  }
}


// VECTOR without compatible members: each block's contiguous output range
// (its 256 records at their scanned offsets) is assembled in an LDS window,
// kNEncWin bytes at a time (a lane writes the part of its record inside the
// window), and flushed with aligned 16-B stores; unaligned byte stores
// straight to HBM cost several times their bytes in write traffic. (Staging
// the block's records in LDS as well was measured slower: cm 2.86 -> 4.04 ms,
// the LDS halves the occupancy.)
constexpr uint32_t kNEncWin = 24 * 1024;
template <int D>
__global__ __launch_bounds__(256) void nest_write_win(NEnc e, const uint8_t *__restrict__ recs,
                                                      const uint64_t *__restrict__ off,
                                                      const uint64_t *__restrict__ part,
                                                      uint64_t nb, uint8_t *ws,
                                                      uint8_t *__restrict__ out, uint64_t out_cap) {
  __shared__ NLayout N;
  __shared__ __align__(16) uint8_t lds[kNEncWin];
  n_stage(N, e.N);
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t mx = ctl->maxc > e.n ? ctl->maxc : e.n;
  const uint32_t w = width_of(mx);
  const uint64_t tot0 = e.n ? part[nb] : 0;
  const uint32_t hl = hdr_shape(e.fmt.flags, e.fmt.literal_len, w).len + w;
  if (hl + tot0 > out_cap) return;  // nothing is written (the caller reads the plan)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    write_hdr(out, e.fmt, w);
    for (uint32_t b = 0; b < w; ++b) out[hl - w + b] = (uint8_t)(e.n >> (8 * b));
  }
  const uint64_t r0 = (uint64_t)blockIdx.x * 256, i = r0 + threadIdx.x;
  if (r0 >= e.n) return;
  const uint64_t rend = r0 + 256 < e.n ? r0 + 256 : e.n;
  const uint64_t g0 = hl + off[r0], g1 = hl + (rend < e.n ? off[rend] : tot0);
  const uint64_t q0 = i < e.n ? hl + off[i] : 0;
  const uint64_t q1 = i < e.n ? (i + 1 < e.n ? hl + off[i + 1] : hl + tot0) : 0;
  const uint8_t *rec = recs + i * N.stride;
  for (uint64_t wlo = g0 & ~15ull; wlo < g1; wlo += kNEncWin) {
    const NWin W{lds, wlo, wlo + kNEncWin < g1 ? wlo + kNEncWin : g1};
    if (i < e.n && q0 < W.hi && q1 > W.lo) n_write<D>(N, rec, e.heaps, w, W, q0, 0, N.n_ops, true);
    __syncthreads();
    // flush [max(W.lo, g0), min(W.hi, out_cap)): aligned 16-B chunks, bytes
    // at the edges (the clamp: no offset, however it was planned, writes
    // past the caller's buffer)
    const uint64_t whi = W.hi < out_cap ? W.hi : out_cap;
    for (uint64_t c = W.lo + (uint64_t)threadIdx.x * 16; c < whi; c += 256 * 16) {
      const uint64_t lo = c > g0 ? c : g0;
      const uint64_t hi = c + 16 < whi ? c + 16 : whi;
      if (lo == c && hi == c + 16)
        flush16(out + c, *reinterpret_cast<const v4u_t *>(lds + (c - W.lo)));
      else
        for (uint64_t x = lo; x < hi; ++x) out[x] = lds[x - W.lo];
    }
    __syncthreads();
  }
}

// MESSAGES encode (every message with its header and frame, at the scanned
// offsets): as nest_write_win, the block's 256 consecutive messages are one
// contiguous output range assembled in the LDS window and flushed with
// aligned 16-B stores (nest_write stored each lane's bytes straight to HBM).
// A message's width comes from its own size walk (calculate_one_size), its
// frame length from the offsets.
template <int D>
__global__ __launch_bounds__(256) void nest_write_mwin(NEnc e, const uint8_t *__restrict__ recs,
                                                       const uint64_t *__restrict__ off,
                                                       const uint64_t *__restrict__ part,
                                                       uint64_t nb, uint8_t *__restrict__ out,
                                                       uint64_t *__restrict__ msg_offsets,
                                                       uint64_t out_cap) {
  __shared__ NLayout N;
  __shared__ __align__(16) uint8_t lds[kNEncWin];
  n_stage(N, e.N);
  const uint64_t tot = e.n ? part[nb] : 0;
  if (tot > out_cap) return;  // every message with its frame, or nothing
  if (blockIdx.x == 0 && threadIdx.x == 0 && msg_offsets) msg_offsets[e.n] = tot;
  const uint64_t r0 = (uint64_t)blockIdx.x * 256, i = r0 + threadIdx.x;
  if (r0 >= e.n) return;
  const uint64_t rend = r0 + 256 < e.n ? r0 + 256 : e.n;
  const uint64_t g0 = off[r0], g1 = rend < e.n ? off[rend] : tot;
  const bool live = i < e.n;
  const uint8_t *rec = recs + i * N.stride;
  uint64_t q0 = 0, q1 = 0, body = 0;
  uint32_t w = 1;
  if (live) {
    q0 = off[i];
    q1 = i + 1 < e.n ? off[i + 1] : tot;
    if (msg_offsets) msg_offsets[i] = q0;
    const NSize sz = n_size<D>(N, rec, e.heaps, 0, N.n_ops, true);
    w = width_of(sz.maxc);
    body = sz.bytes + sz.cnts * w;
  }
  const uint32_t mlen = (uint32_t)(q1 - q0 - e.fpre);
  const uint32_t sq = live && e.fseq_off != SPK_FRAME_NONE ? seq_value(e.echo, e.fseq_base, i) : 0u;
  for (uint64_t wlo = g0 & ~15ull; wlo < g1; wlo += kNEncWin) {
    const NWin W{lds, wlo, wlo + kNEncWin < g1 ? wlo + kNEncWin : g1};
    if (live && q0 < W.hi && q1 > W.lo) {
      for (uint32_t b = 0; b < e.fpre; ++b) {  // the frame: template, seq_num, length
        uint32_t v = e.ftmpl[b];
        if (e.fseq_off != SPK_FRAME_NONE && b >= e.fseq_off && b < e.fseq_off + 4)
          v = (sq >> (8 * (b - e.fseq_off))) & 0xFFu;
        if (e.flen_off != SPK_FRAME_NONE && b >= e.flen_off && b < e.flen_off + 4)
          v = (mlen >> (8 * (b - e.flen_off))) & 0xFFu;
        W.byte(q0 + b, v);
      }
      const uint64_t m = q0 + e.fpre;
      auto put = [&W, m](uint32_t p, uint8_t b) { W.byte(m + p, b); };
      const uint32_t hl = N.n_ranks ? compat_hdr_with(put, e.fmt, w, body, true)
                                    : write_hdr_with(put, e.fmt, w);
      uint64_t qo = n_write<D>(N, rec, e.heaps, w, W, m + hl, 0, N.n_ops, true);
      for (uint32_t rk = 0; rk < N.n_ranks; ++rk) qo = n_write_compat<D>(N, rec, e.heaps, rk, w, W, qo);
    }
    __syncthreads();
    const uint64_t whi = W.hi < out_cap ? W.hi : out_cap;
    for (uint64_t c = W.lo + (uint64_t)threadIdx.x * 16; c < whi; c += 256 * 16) {
      const uint64_t lo = c > g0 ? c : g0;
      const uint64_t hi = c + 16 < whi ? c + 16 : whi;
      if (lo == c && hi == c + 16)
        flush16(out + c, *reinterpret_cast<const v4u_t *>(lds + (c - W.lo)));
      else
        for (uint64_t x = lo; x < hi; ++x) out[x] = lds[x - W.lo];
    }
    __syncthreads();
  }
}

static unsigned nblocks(uint64_t n, uint32_t t) {
  const uint64_t b = (n + t - 1) / t;
  return (unsigned)(b ? b : 1);
}

static NEnc make_nenc(const spk_layout *L, int mode, uint64_t n, const void *const *heaps) {
  NEnc e = {};
  e.N = make_nlayout(L);
  e.n = n;
  e.mode = mode;
  e.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  e.fseq_off = e.flen_off = SPK_FRAME_NONE;
  for (uint32_t k = 0; k < e.N.n_heaps && k < SPK_MAX_SPANS; ++k)
    e.heaps[k] = heaps ? (const uint8_t *)heaps[k] : nullptr;
  return e;
}

// size pass + scan; leaves per-record offsets in column a[0]
// cond (device, non-null): every kernel returns at once while the plan token
// holds (the encode's check, NTok)
static hipError_t nest_size_scan(const NEnc &e, const void *d_recs, uint8_t *ws, hipStream_t s,
                                 uint64_t **a_out, uint64_t **part_out, uint64_t *nb_out,
                                 const uint32_t *cond = nullptr) {
  const NWs f = nws_layout(e.n, e.N.n_heaps, e.N.n_ranks);
  uint64_t *a = reinterpret_cast<uint64_t *>(ws + f.a);
  uint64_t *part = reinterpret_cast<uint64_t *>(ws + f.part);
  SPK_LAUNCH(nest_ctl_init, dim3(1), dim3(1), 0, s, ws, cond);
  if (e.n) {
    NEST_D(n_dclass(e.N),
           SPK_LAUNCH(nest_size<D>, dim3(nblocks(e.n, 256)), dim3(256), 0, s, e,
                      (const uint8_t *)d_recs, a, ws, cond));
    if (e.mode == SPK_MODE_VECTOR)
      NEST_D(n_dclass(e.N),
             SPK_LAUNCH(nest_vec_sizes<D>, dim3(nblocks(e.n, 256) < 4096 ? nblocks(e.n, 256) : 4096),
                        dim3(256), 0, s, e, (const uint8_t *)d_recs, a, ws, cond));
  }
  hipError_t er = hipGetLastError();
  if (er != hipSuccess) return er;
  // VECTOR: column 0 = sizes at w, column 1 = count fields, 2.. = version
  // passes; MESSAGES: column 0 = message sizes, column 1 = payload bytes. All
  // scanned (totals in part).
  const uint32_t cols = e.mode == SPK_MODE_VECTOR ? 2 + e.N.n_ranks : 2;
  if ((er = nscan(a, e.n, cols, part, s, ws, cond)) != hipSuccess) return er;
  *a_out = a;
  *part_out = part;
  *nb_out = (e.n + kNScanBlk - 1) / kNScanBlk;
  return hipSuccess;
}

hipError_t launch_nested_plan(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                              const void *const *d_heaps, spk_plan_t *d_plan, void *d_ws,
                              hipStream_t s) {
  NEnc e = make_nenc(L, mode, n, d_heaps);
  uint8_t *ws = (uint8_t *)d_ws;
  uint64_t *a, *part, nb;
  hipError_t er = nest_size_scan(e, d_recs, ws, s, &a, &part, &nb);
  if (er != hipSuccess) return er;
  const uint32_t tok = !e.N.n_ranks;
  if (tok && n)
    SPK_LAUNCH(nest_tok_hash, dim3(nblocks(n, 256) < 512 ? nblocks(n, 256) : 512), dim3(256), 0,
               s, (const uint64_t *)a, n,
               &reinterpret_cast<NTok *>(ws + kWsPlanTok)->hash);
  SPK_LAUNCH(nest_plan_fin, dim3(1), dim3(1), 0, s, e, (const uint64_t *)a,
             (const uint64_t *)part, nb, ws, d_plan, tok, (uint64_t)(uintptr_t)d_recs,
             tok_heaps(e), tok_layout(L, mode));
  return hipGetLastError();
}

hipError_t launch_nested_encode(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                                const void *const *d_heaps, void *d_out, uint64_t out_cap,
                                uint64_t *d_msg_offsets, const spk_frame *F, uint32_t fixed_w,
                                void *d_ws, hipStream_t s, const SeqEcho *echo) {
  NEnc e = make_nenc(L, mode, n, d_heaps);
  if (echo) e.echo = *echo;
  e.fixed_w = fixed_w;
  if (F) {
    e.fpre = F->prefix_len;
    e.fseq_off = F->seq_off;
    e.flen_off = F->len_off;
    e.fseq_base = F->seq_base;
    for (uint32_t k = 0; k < F->prefix_len; ++k) e.ftmpl[k] = F->tmpl[k];
  }
  uint8_t *ws = (uint8_t *)d_ws;
  uint64_t *a, *part, nb;
  const bool vec_win = mode == SPK_MODE_VECTOR && !e.N.n_ranks && !fixed_w;
  const bool msg_win = mode == SPK_MODE_MESSAGES;
  if (vec_win || msg_win) {
    hipError_t er;
    if (!e.N.n_ranks) {
      // the plan that precedes this call on the workspace (spk_encode's
      // contract, as for the flat layouts) left every record's offset (or
      // message size) in column 0, the totals in the partials and the longest
      // container in the control block, with its token: the token is checked
      // on the device and the size pass re-runs (each kernel returns at once
      // otherwise) when it fails
      NTok *t = reinterpret_cast<NTok *>(ws + kWsPlanTok);
      const NWs f = nws_layout(e.n, e.N.n_heaps, e.N.n_ranks);
      a = reinterpret_cast<uint64_t *>(ws + f.a);
      part = reinterpret_cast<uint64_t *>(ws + f.part);
      nb = (e.n + kNScanBlk - 1) / kNScanBlk;
      SPK_LAUNCH(nest_tok_begin, dim3(1), dim3(1), 0, s, ws, n, (uint64_t)(uintptr_t)d_recs,
                 tok_heaps(e), tok_layout(L, mode, e.fpre));
      if (n)
        SPK_LAUNCH(nest_tok_hash, dim3(nblocks(n, 256) < 512 ? nblocks(n, 256) : 512),
                   dim3(256), 0, s, (const uint64_t *)a, n, &t->chk);
      SPK_LAUNCH(nest_tok_verdict, dim3(1), dim3(1), 0, s, ws, (const uint64_t *)part, nb, n);
      uint64_t *a2, *part2, nb2;
      er = nest_size_scan(e, d_recs, ws, s, &a2, &part2, &nb2, &t->stale);
    } else {
      er = nest_size_scan(e, d_recs, ws, s, &a, &part, &nb);
    }
    if (er != hipSuccess) return er;
    if (vec_win)
      NEST_D(n_dclass(e.N),
             SPK_LAUNCH(nest_write_win<D>, dim3(nblocks(n, 256)), dim3(256), 0, s, e,
                        (const uint8_t *)d_recs, (const uint64_t *)a, (const uint64_t *)part, nb,
                        ws, (uint8_t *)d_out, out_cap));
    else
      NEST_D(n_dclass(e.N),
             SPK_LAUNCH(nest_write_mwin<D>, dim3(nblocks(n, 256)), dim3(256), 0, s, e,
                        (const uint8_t *)d_recs, (const uint64_t *)a, (const uint64_t *)part, nb,
                        (uint8_t *)d_out, d_msg_offsets, out_cap));
    return hipGetLastError();
  }
  hipError_t er = nest_size_scan(e, d_recs, ws, s, &a, &part, &nb);
  if (er != hipSuccess) return er;
  NEST_D(n_dclass(e.N),
         SPK_LAUNCH(nest_write<D>, dim3(nblocks(n, 256)), dim3(256), 0, s, e,
                    (const uint8_t *)d_recs, (const uint64_t *)a, (const uint64_t *)part, nb, ws,
                    (uint8_t *)d_out, d_msg_offsets, fixed_w ? 0u : 1u, out_cap));
  return hipGetLastError();
}

// ---- decode kernels -----------------------------------------------------------------
struct NDec {
  NLayout N;
  spk_msgfmt fmt;
  uint64_t wire_len, n_msgs, rec_cap;
  uint32_t prefix, body_w;  // body_w: spk_decode_body (no header, body_n records)
  uint64_t body_n;
  uint8_t *heaps[SPK_MAX_SPANS];
  uint64_t heap_cap[SPK_MAX_SPANS];
  const uint64_t *ends;  // MESSAGES: message i ends at ends[i] (null: offs[i + 1])
  // compatible-member VECTOR decode behind the tile passes: the one-lane walk's
  // kernels run only while *serial is non-zero (CompatCtl); null: always
  const uint32_t *serial;
};
__device__ __forceinline__ bool n_skip(const NDec &a) { return a.serial && !*a.serial; }

// VECTOR header (deserialize_metainfo, unpacker.hpp:548-619, + the count) or
// the body of spk_decode_body; initialises the control block and *res
__global__ void nest_vhdr(NDec a, const uint8_t *__restrict__ wire, uint8_t *ws,
                          spk_dresult_t *res) {
  if (n_skip(a)) return;
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint64_t len = a.wire_len;
  uint64_t pos = 0, n = 0, dl = 0;
  uint32_t w = 1;
  int32_t errc = 0;
  if (a.body_w) {
    w = a.body_w;
    n = a.body_n;
  } else {
    errc = parse_hdr(a.fmt, wire, len, &pos, &w, &dl);
    if (!errc) {
      if (len - pos < w) {
        errc = SPK_ERRC_NO_BUFFER_SPACE;
      } else {
        n = ld_le(wire + pos, w);
        pos += w;
      }
    }
  }
  ctl->maxc = 0;
  ctl->nrec = errc ? 0 : n;
  ctl->end = pos;
  ctl->data_len = dl;
  ctl->ovf = 0;
  ctl->w = w;
  ctl->errc = (uint32_t)errc;
  ctl->p0 = pos;
  ctl->nch = (errc || !n || len <= pos) ? 0 : (len - pos + kNCh - 1) / kNCh;
  for (int r = 0; r < kNRounds; ++r) ctl->changed[r] = 0;
  ctl->cmin = ~0ull;
  ctl->cmax = 0;
  ctl->ndirty = 0;
  ctl->rewalks = 0;
  ctl->fixed = 0;
  for (uint32_t k = 0; k < SPK_MAX_SPANS; ++k) ctl->htot[k] = 0;
  ctl->werr = 0;
  spk_dresult_t r = {};
  r.errc = errc;
  r.width = w;
  *res = r;
}

struct CPtrs {
  uint64_t *ent, *ext, *cols;  // cols[0][c]: records; cols[1 + k][c]: heap k use
  unsigned long long *dirty;   // bitmap of the chunks the rounds left open
  int32_t *err;
  uint64_t nch_cap;            // column stride = chunks the wire allows (the scan's length)
};

struct CWalk {
  uint64_t ext, cnt;
  int32_t err;
};

// the records of the path from s that start before c1; lim < wire_len makes
// the walk speculative (kNUnk when a read would pass lim); hs += heap use
__device__ CWalk nc_walk(const NLayout &N, const NDec &a, const uint8_t *__restrict__ wire,
                         uint64_t s, uint64_t c1, uint64_t lim, uint32_t w, uint64_t *hs) {
  CWalk r = {s, 0, 0};
  if (s == kNFail || s == kNUnk) return r;
  const bool bounded = lim < a.wire_len;
  uint64_t pos = s;
  uint32_t ovf = 0;
  while (pos < c1) {
    const uint64_t before = pos;
    const int32_t ec = n_read(N, wire, pos, lim, w, nullptr, nullptr, hs, a.heap_cap, &ovf, 0,
                              N.n_ops, true, bounded);
    if (ec == kNLimit) {
      r.ext = kNUnk;
      return r;
    }
    if (ec) {
      r.ext = kNFail;
      r.err = ec;
      return r;
    }
    if (pos == before) {  // (a record takes at least one byte: layout_check)
      r.ext = kNFail;
      r.err = SPK_ERRC_INTERNAL;
      return r;
    }
    ++r.cnt;
  }
  r.ext = pos;
  return r;
}

__device__ __forceinline__ void nc_store(const CPtrs &P, uint32_t H, uint64_t c, uint64_t ent,
                                         const CWalk &r, const uint64_t *hs) {
  P.ent[c] = ent;
  P.ext[c] = r.ext;
  P.err[c] = r.err;
  P.cols[c] = r.cnt;
  for (uint32_t k = 0; k < H; ++k) P.cols[(uint64_t)(1 + k) * P.nch_cap + c] = hs[k];
}

// speculation: chunk c's entry guessed (chunk 0's is exact) and its records walked
__global__ __launch_bounds__(kNT) void nest_cspec(NDec a, const uint8_t *__restrict__ wire,
                                                  const uint8_t *ws, CPtrs P) {
  __shared__ NLayout N;
  n_stage(N, a.N);
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = ctl->w, H = N.n_heaps;
  uint64_t hs[SPK_MAX_SPANS];
  for (uint32_t k = 0; k < H; ++k) hs[k] = 0;
  if (c >= ctl->nch) {  // past the header's chunks: nothing in the scanned columns
    if (c < P.nch_cap) nc_store(P, H, c, kNFail, CWalk{kNFail, 0, 0}, hs);
    return;
  }
  const uint64_t len = a.wire_len, c0 = ctl->p0 + c * kNCh;
  const uint64_t c1 = c0 + kNCh < len ? c0 + kNCh : len;
  uint64_t ent = kNUnk;
  CWalk r = {kNUnk, 0, 0};
  if (c == 0) {
    ent = c0;
    r = nc_walk(N, a, wire, c0, c1, len, w, hs);
  } else {
    // the first byte from which two whole records parse (a bounded walk)
    const uint64_t lim = c1 + kNBound < len ? c1 + kNBound : len;
    for (uint64_t q = c0; q < c1 && ent == kNUnk; ++q) {
      if (N.scr_off != ~0u) {  // the first count must fit the bytes the walk may use
        const uint64_t x = q + N.scr_off;
        if (x + w > lim) continue;
        const uint64_t cnt = ld_le(wire + x, w);
        if (cnt > (lim - x - w) / N.scr_esz) continue;
      }
      uint64_t p = q;
      uint32_t ovf = 0;
      int32_t ec = 0;
      for (int k2 = 0; k2 < 2 && !ec && p < lim; ++k2)
        ec = n_read(N, wire, p, lim, w, nullptr, nullptr, hs, a.heap_cap, &ovf, 0, N.n_ops,
                    true, lim < len);
      if (!ec) ent = q;
    }
    for (uint32_t k = 0; k < H; ++k) hs[k] = 0;
    // its records up to the chunk's end (kNUnk / kNFail when that walk fails:
    // the rounds walk the chunk again from its predecessor's exit)
    if (ent != kNUnk) r = nc_walk(N, a, wire, ent, c1, lim, w, hs);
  }
  nc_store(P, H, c, ent, r, hs);
}

// round `round`: a chunk whose entry is not its predecessor's exit (or whose
// walk gave up) is walked again from that exit
__global__ __launch_bounds__(kNT) void nest_cround(NDec a, const uint8_t *__restrict__ wire,
                                                   uint8_t *ws, CPtrs P, int round) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  if (round > 0 && !ctl->changed[round - 1]) return;  // settled (the same for every lane)
  __shared__ NLayout N;
  n_stage(N, a.N);
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 || c >= ctl->nch) return;
  const uint64_t E = __atomic_load_n(&P.ext[c - 1], __ATOMIC_RELAXED);
  const uint64_t ent = P.ent[c], ext = P.ext[c];
  if (E == ent && ext != kNUnk) return;
  // walk again only from the exit of a predecessor that agrees with its own
  // predecessor: a predecessor that is about to change would hand a wrong
  // entry on, and the wrong exit one chunk further each round
  const bool pred_open =
      E == kNUnk || (c >= 2 && (__atomic_load_n(&P.ext[c - 2], __ATOMIC_RELAXED) != P.ent[c - 1]));
  if (pred_open) {
    atomicAdd(&ctl->changed[round], 1ull);
    return;
  }
  const uint64_t len = a.wire_len, c0 = ctl->p0 + c * kNCh;
  const uint64_t c1 = c0 + kNCh < len ? c0 + kNCh : len;
  const uint32_t H = N.n_heaps;
  uint64_t hs[SPK_MAX_SPANS];
  for (uint32_t k = 0; k < H; ++k) hs[k] = 0;
  const CWalk r = nc_walk(N, a, wire, E, c1, len, ctl->w, hs);
  nc_store(P, H, c, E, r, hs);
  atomicAdd(&ctl->rewalks, 1ull);
  if (r.ext != ext) atomicAdd(&ctl->changed[round], 1ull);
}

// after the rounds: the chunks still open (only when the last round moved something)
__global__ __launch_bounds__(kNT) void nest_cverify(uint8_t *ws, CPtrs P) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  if (!ctl->changed[kNRounds - 1]) return;
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 || c >= ctl->nch) return;
  if (P.ext[c - 1] != P.ent[c] || P.ext[c] == kNUnk) {
    atomicMin(&ctl->cmin, (unsigned long long)c);
    atomicMax(&ctl->cmax, (unsigned long long)c);
    atomicAdd(&ctl->ndirty, 1ull);
    atomicOr(&P.dirty[c >> 6], 1ull << (c & 63));
  }
}

// one wave settles the open chunks in order: the next open chunk from the
// bitmap (64 words = 4096 chunks per look), walked again from its
// predecessor's exit; a walk that moves a chunk's exit makes the next chunk
// open too. (A chunk is walked by lane 0 and its exit carried in a register,
// so the wave never re-reads what it wrote.)
__global__ __launch_bounds__(64) void nest_cfix(NDec a, const uint8_t *__restrict__ wire,
                                                uint8_t *ws, CPtrs P) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  if (!ctl->ndirty) return;
  __shared__ NLayout N;
  n_stage(N, a.N);
  const uint32_t lane = threadIdx.x;
  const uint64_t nch = ctl->nch, len = a.wire_len;
  const uint64_t nwords = (nch + 63) >> 6;
  const uint32_t H = N.n_heaps;
  uint64_t c = ctl->cmin;  // >= 1: chunk 0 is never open
  bool carry = false;      // chunk c follows a chunk whose exit moved
  uint64_t cext = 0;       // that exit
  uint64_t nfix = 0;
  while (c < nch) {
    if (!carry) {  // the next open chunk at or after c
      uint64_t found = ~0ull;
      for (uint64_t w0 = c >> 6; w0 < nwords && found == ~0ull; w0 += 64) {
        const uint64_t wi = w0 + lane;
        uint64_t bits = wi < nwords ? P.dirty[wi] : 0;
        if (wi == (c >> 6)) bits &= ~0ull << (c & 63);
        const uint64_t m = __ballot(bits != 0);
        if (m) {
          const uint32_t l = (uint32_t)__ffsll((unsigned long long)m) - 1;
          const uint64_t b = __shfl(bits, (int)l);
          found = ((w0 + l) << 6) + (uint64_t)(__ffsll((unsigned long long)b) - 1);
        }
      }
      if (found == ~0ull || found >= nch) break;
      c = found;
    }
    uint64_t nx = 0, moved = 0;
    if (lane == 0) {
      const uint64_t E = carry ? cext : P.ext[c - 1];
      const uint64_t ent = P.ent[c], old = P.ext[c];
      if (E != ent || old == kNUnk) {
        const uint64_t c0 = ctl->p0 + c * kNCh;
        const uint64_t c1 = c0 + kNCh < len ? c0 + kNCh : len;
        uint64_t hs[SPK_MAX_SPANS];
        for (uint32_t k = 0; k < H; ++k) hs[k] = 0;
        // (E is settled: never kNUnk; guarded anyway)
        const CWalk r = E == kNUnk ? CWalk{kNFail, 0, SPK_ERRC_INTERNAL}
                                   : nc_walk(N, a, wire, E, c1, len, ctl->w, hs);
        nc_store(P, H, c, E == kNUnk ? kNFail : E, r, hs);
        nx = r.ext;
        moved = r.ext != old;
        ++nfix;
      }
    }
    moved = __shfl(moved, 0);
    nx = __shfl(nx, 0);
    carry = moved != 0;
    cext = nx;
    ++c;
  }
  if (lane == 0) ctl->fixed = nfix;
}

// each chunk's records into place: record index and heap bases from the
// scanned columns; the record the path fails at sets the errc
__global__ __launch_bounds__(kNT) void nest_cemit(NDec a, const uint8_t *__restrict__ wire,
                                                  uint8_t *ws, CPtrs P, uint8_t *__restrict__ recs) {
  __shared__ NLayout N;
  n_stage(N, a.N);
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ctl->nch) return;
  const uint64_t n = ctl->nrec, first = P.cols[c];
  const uint64_t s = P.ent[c];
  if (first >= n || s == kNFail || s == kNUnk) return;
  const uint64_t len = a.wire_len, c0 = ctl->p0 + c * kNCh;
  const uint64_t c1 = c0 + kNCh < len ? c0 + kNCh : len;
  const uint32_t H = N.n_heaps, w = ctl->w;
  uint64_t used[SPK_MAX_SPANS];
  for (uint32_t k = 0; k < H; ++k) used[k] = P.cols[(uint64_t)(1 + k) * P.nch_cap + c];
  uint32_t ovf = 0;
  uint64_t pos = s;
  for (uint64_t idx = first; pos < c1 && idx < n; ++idx) {
    uint8_t *rec = idx < a.rec_cap ? recs + idx * N.stride : nullptr;
    const int32_t ec = n_read(N, wire, pos, len, w, rec, a.heaps, used, a.heap_cap, &ovf, 0,
                              N.n_ops, true);
    if (ec) {
      ctl->werr = ec;  // the one record of the path that fails before n
      break;
    }
    if (idx == n - 1) {
      ctl->end = pos;
      for (uint32_t k = 0; k < H; ++k) ctl->htot[k] = used[k];
    }
  }
  if (ovf) atomicAdd(&ctl->ovf, 1ull);
}

// result of the chunked decode: count, consume_len, heap use, capacity
__global__ void nest_cfinish(NDec a, const uint64_t *__restrict__ part, uint64_t nb,
                             const uint8_t *ws, spk_dresult_t *res) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  if (ctl->errc) return;  // the header errc is already in *res
  spk_dresult_t r = *res;
  const uint64_t n = ctl->nrec;
  const uint64_t total = ctl->nch ? part[nb] : 0;  // records on the path (column 0)
  r.tiles_repaired = (uint32_t)(ctl->rewalks < 0xFFFFFFFFull ? ctl->rewalks : 0xFFFFFFFFull);
  r.tiles_sequential = (uint32_t)(ctl->fixed < 0xFFFFFFFFull ? ctl->fixed : 0xFFFFFFFFull);
  if (ctl->werr || total < n) {
    r.errc = ctl->werr ? ctl->werr : SPK_ERRC_NO_BUFFER_SPACE;
  } else {
    r.count = n;
    r.consumed = ctl->end;
    for (uint32_t k = 0; k < a.N.n_heaps; ++k) {
      r.heap_used[k] = ctl->htot[k];
      if (r.heap_used[k] > a.heap_cap[k]) r.errc = SPK_ERRC_CAPACITY;
    }
    if (n > a.rec_cap || ctl->ovf) r.errc = SPK_ERRC_CAPACITY;
  }
  *res = r;
}

// p[0, n) = v while *cond (null: always)
__global__ void nest_fill_u64(uint64_t *p, uint64_t n, uint64_t v, const uint32_t *cond) {
  if (cond && !*cond) return;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// VECTOR layouts with compatible members: the version passes trail every
// record's main pass, so one lane walks the message (main pass, then the
// version passes, unpacker.hpp:292-366,1354-1376) and records each record's
// start, its heap use U[k][i] and where its group of each version starts
__global__ void nest_vec_serial(NDec a, const uint8_t *__restrict__ wire, uint8_t *ws,
                                uint64_t *__restrict__ U, uint64_t *__restrict__ starts,
                                uint64_t *__restrict__ cpos) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  if (threadIdx.x || n_skip(a) || ctl->errc) return;
  const NLayout &N = a.N;
  const uint64_t n = ctl->nrec, len = a.wire_len, data_end = ctl->data_len;
  const uint32_t w = ctl->w;
  uint64_t pos = ctl->p0, used[SPK_MAX_SPANS] = {}, base[SPK_MAX_SPANS];
  uint32_t ovf = 0;
  int32_t errc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (i < a.rec_cap) starts[i] = pos;
    for (uint32_t k = 0; k < N.n_heaps; ++k) base[k] = used[k];
    errc = n_read(N, wire, pos, len, w, nullptr, nullptr, used, a.heap_cap, &ovf, 0, N.n_ops, true);
    if (errc) break;
    if (i < a.rec_cap)
      for (uint32_t k = 0; k < N.n_heaps; ++k) U[(uint64_t)k * a.rec_cap + i] = used[k] - base[k];
  }
  bool stop = errc != 0;
  for (uint32_t rk = 0; rk < N.n_ranks && !stop; ++rk) {
    for (uint64_t i = 0; i < n && !stop; ++i) {
      if (i < a.rec_cap) cpos[(uint64_t)rk * a.rec_cap + i] = pos;
      for (uint32_t k = 0; k < N.n_heaps; ++k) base[k] = used[k];
      stop = n_read_compat(N, wire, pos, len, data_end, rk, w, nullptr, nullptr, used, a.heap_cap,
                           &ovf, &errc) != 0;
      if (i < a.rec_cap)
        for (uint32_t k = 0; k < N.n_heaps; ++k) U[(uint64_t)k * a.rec_cap + i] += used[k] - base[k];
    }
  }
  ctl->werr = errc;
  ctl->end = pos;
}

// MESSAGES count pass: errc and heap use of every message (no writes)
// MESSAGES decode: each wave stages its 64 consecutive messages (the first
// kMsgWin bytes from a 16-B aligned base) in LDS with 16-B loads; the lanes'
// interpreter walks read them there (NRd). Frames routed out of order
// (a.ends) and irregular offsets read the wire in place.
constexpr uint32_t kMsgWin = 4096;
__device__ __forceinline__ NRd n_stage_msgs(v4u_t *win, const NDec &a, const uint8_t *wire,
                                            const uint64_t *offs, uint64_t i0, uint32_t lane) {
  NRd rd{wire, (const nlds_u8 *)win, 0, 0};
  const uint64_t n = a.n_msgs;
  if (a.ends || i0 >= n) return rd;
  const uint64_t b = offs[i0], e = offs[i0 + 64 < n ? i0 + 64 : n];
  if (e <= b || e > a.wire_len) return rd;
  const uint64_t base = b & ~15ull;
  const uint64_t span = e - base < kMsgWin ? e - base : kMsgWin;
  const uint64_t whole = (a.wire_len - base) / 16;  // 16-B words inside the wire
  const uint64_t nv = (span + 15) / 16 < whole ? (span + 15) / 16 : whole;
  constexpr uint32_t kPer = kMsgWin / 16 / 64;
  v4u_t val[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t v = lane + 64 * k;
    if (v < nv) val[k] = *reinterpret_cast<const v4u_una *>(wire + base + 16ull * v);
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t v = lane + 64 * k;
    if (v < nv) win[v] = val[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  rd.lo = base;
  rd.hi = base + 16 * nv;
  return rd;
}

// the lane's heap-use counters: LDS ([lane][heap], dynamic shared memory of
// 256 x nh words) when the layout has at most kNUseLds heaps, else a local
// array (runtime-indexed: scratch memory)
constexpr uint32_t kNUseLds = 16;
template <bool LU>
struct NUse {
  uint64_t loc[LU ? 1 : SPK_MAX_SPANS];
  __device__ __forceinline__ uint64_t *ptr(uint32_t nh) {
    if constexpr (LU) {
      extern __shared__ uint64_t nuse_s[];
      return nuse_s + threadIdx.x * (nh ? nh : 1u);
    } else {
      return loc;
    }
  }
};
static inline size_t n_use_lds(const NLayout &N) {
  return N.n_heaps <= kNUseLds ? (size_t)256 * 8 * (N.n_heaps ? N.n_heaps : 1) : 0;
}

template <int D, bool LU>
__global__ __launch_bounds__(256) void nest_msg_count(NDec a, const uint8_t *__restrict__ wire_g,
                                                      const uint64_t *__restrict__ offs,
                                                      uint64_t *__restrict__ U,
                                                      int32_t *__restrict__ ec,
                                                      uint64_t *__restrict__ cons) {
  __shared__ v4u_t win_s[4][kMsgWin / 16];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const NRd wire = n_stage_msgs(win_s[threadIdx.x >> 6], a, wire_g, offs, i & ~63ull,
                                threadIdx.x & 63);
  if (i >= a.n_msgs) return;
  const NLayout &N = a.N;
  NUse<LU> us;
  uint64_t *const used = us.ptr(N.n_heaps);
  for (uint32_t k = 0; k < N.n_heaps; ++k) used[k] = 0;
  const uint64_t b = offs[i], e = a.ends ? a.ends[i] : offs[i + 1];
  int32_t errc = SPK_ERRC_OK;
  uint64_t consumed = 0;
  if (e < b || e > a.wire_len || e - b < a.prefix) {
    errc = SPK_ERRC_NO_BUFFER_SPACE;
  } else {
    const uint64_t m0 = b + a.prefix;
    uint64_t p0, dl;
    uint32_t w;
    errc = parse_hdr(a.fmt, wire_g + m0, e - m0, &p0, &w, &dl);
    if (!errc) {
      uint64_t pos = m0 + p0;
      uint32_t ovf = 0;
      errc = n_read<D>(N, wire, pos, e, w, nullptr, nullptr, used, a.heap_cap, &ovf, 0, N.n_ops,
                       true);
      for (uint32_t rk = 0; !errc && rk < N.n_ranks; ++rk)
        if (n_read_compat<D>(N, wire, pos, e, m0 + dl, rk, w, nullptr, nullptr, used, a.heap_cap,
                          &ovf, &errc))
          break;
      consumed = pos - m0 > dl ? pos - m0 : dl;  // consume_len (struct_pack.hpp:343-357)
    }
    if (!errc && i >= a.rec_cap) errc = SPK_ERRC_CAPACITY;
  }
  ec[i] = errc;
  cons[i] = errc ? 0 : consumed;
  for (uint32_t k = 0; k < N.n_heaps; ++k) U[(uint64_t)k * a.n_msgs + i] = errc ? 0 : used[k];
}

// write pass (MESSAGES, and VECTOR with compatible members): record i from
// its start with heap bases B[k][i]
template <int D, bool LU>
__global__ __launch_bounds__(256) void nest_emit(NDec a, const uint8_t *__restrict__ wire,
                                                 const uint64_t *__restrict__ offs,
                                                 const uint64_t *__restrict__ starts,
                                                 const uint64_t *__restrict__ B, uint64_t nrows,
                                                 const int32_t *__restrict__ ec, uint8_t *ws,
                                                 const uint64_t *__restrict__ cpos,
                                                 uint8_t *__restrict__ recs, int mode,
                                                 int32_t *__restrict__ errc_out) {
  __shared__ v4u_t win_s[4][kMsgWin / 16];
  if (n_skip(a)) return;  // (uniform)
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const NLayout &N = a.N;
  const NRd rdm = mode == SPK_MODE_MESSAGES
                      ? n_stage_msgs(win_s[threadIdx.x >> 6], a, wire, offs, i & ~63ull,
                                     threadIdx.x & 63)
                      : NRd{wire, nullptr, 0, 0};
  if (mode == SPK_MODE_MESSAGES) {
    // the per-message verdicts: copied out and tallied here, one wave reduce
    // and one atomic per wave (a one-block loop over 1M messages in
    // nest_finish took 1.6 ms)
    const bool in = i < a.n_msgs;
    const int32_t e = in ? ec[i] : 0;
    if (in && errc_out) errc_out[i] = e;
    uint64_t okc = in && e == 0;
    for (int o = 32; o > 0; o >>= 1) okc += __shfl_xor(okc, o);
    const uint64_t capm = __ballot(in && e == SPK_ERRC_CAPACITY);
    if ((threadIdx.x & 63) == 0) {
      if (okc) atomicAdd(&ctl->m_ok, (unsigned long long)okc);
      if (capm) atomicOr(&ctl->m_cap, 1ull);
    }
  }
  uint64_t pos, end, data_end;
  uint32_t w;
  if (mode == SPK_MODE_VECTOR) {
    if (ctl->errc || ctl->werr || i >= ctl->nrec || i >= a.rec_cap) return;
    pos = starts[i];
    end = a.wire_len;
    w = ctl->w;
    data_end = ctl->data_len;
  } else {
    if (i >= a.n_msgs || i >= a.rec_cap || ec[i]) return;
    const uint64_t m0 = offs[i] + a.prefix;
    end = a.ends ? a.ends[i] : offs[i + 1];
    uint64_t p0, dl;
    parse_hdr(a.fmt, wire + m0, end - m0, &p0, &w, &dl);
    pos = m0 + p0;
    data_end = m0 + dl;
  }
  NUse<LU> us;
  uint64_t *const used = us.ptr(N.n_heaps);
  for (uint32_t k = 0; k < N.n_heaps; ++k) used[k] = B[(uint64_t)k * nrows + i];
  uint32_t ovf = 0;
  uint8_t *rec = recs + i * N.stride;
  n_read<D>(N, rdm, pos, end, w, rec, a.heaps, used, a.heap_cap, &ovf, 0, N.n_ops, true);
  int32_t cec = 0;
  for (uint32_t rk = 0; rk < N.n_ranks; ++rk) {
    if (mode == SPK_MODE_VECTOR) {  // this record's group of version rk (walker)
      pos = cpos[(uint64_t)rk * a.rec_cap + i];
      if (pos == ~0ull) break;
    }
    if (n_read_compat<D>(N, rdm, pos, end, data_end, rk, w, rec, a.heaps, used, a.heap_cap, &ovf,
                      &cec))
      break;
  }
  if (ovf) atomicAdd(&ctl->ovf, 1ull);
}

// result: count, consume_len, heap use (column totals), capacity errors
__global__ void nest_finish(NDec a, const uint64_t *__restrict__ part, uint64_t nb,
                            const int32_t *__restrict__ ec, uint8_t *ws, int mode,
                            spk_dresult_t *res, int32_t *__restrict__ errc_out) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  // (MESSAGES: nest_emit copied the per-message errc out and tallied them)
  (void)ec;
  (void)errc_out;
  if (threadIdx.x || n_skip(a)) return;
  const unsigned long long s_ok = ctl->m_ok, s_cap = ctl->m_cap;
  spk_dresult_t r = *res;
  const uint32_t nh = a.N.n_heaps;
  if (mode == SPK_MODE_VECTOR) {
    if (ctl->errc) return;  // errc already in *res
    if (ctl->werr) {
      r.errc = ctl->werr;
      *res = r;
      return;
    }
    const uint64_t n = ctl->nrec;
    r.count = n;
    r.consumed = ctl->end > ctl->data_len ? ctl->end : ctl->data_len;
    const uint64_t rows = n < a.rec_cap ? n : a.rec_cap;
    for (uint32_t k = 0; k < nh; ++k) r.heap_used[k] = rows ? part[(uint64_t)k * (nb + 1) + nb] : 0;
    if (n > a.rec_cap || ctl->ovf) r.errc = SPK_ERRC_CAPACITY;
    for (uint32_t k = 0; k < nh; ++k)
      if (r.heap_used[k] > a.heap_cap[k]) r.errc = SPK_ERRC_CAPACITY;
  } else {
    r.count = s_ok;
    for (uint32_t k = 0; k < nh; ++k)
      r.heap_used[k] = a.n_msgs ? part[(uint64_t)k * (nb + 1) + nb] : 0;
    r.errc = s_cap || ctl->ovf ? SPK_ERRC_CAPACITY : SPK_ERRC_OK;
    for (uint32_t k = 0; k < nh; ++k)
      if (r.heap_used[k] > a.heap_cap[k]) r.errc = SPK_ERRC_CAPACITY;
  }
  *res = r;
}

__global__ void nest_put_consumed(const uint64_t *__restrict__ part, uint64_t nb, uint64_t n,
                                  spk_dresult_t *res) {
  spk_dresult_t r = *res;
  r.consumed = n ? part[nb] : 0;
  *res = r;
}

hipError_t launch_nested_decode(const spk_layout *L, int mode, const void *d_wire,
                                uint64_t wire_len, const uint64_t *d_msg_offsets,
                                uint64_t n_msgs, uint32_t prefix, void *d_recs, uint64_t rec_cap,
                                void *const *d_heaps, const uint64_t *heap_caps,
                                spk_dresult_t *d_res, int32_t *d_errc, void *d_ws,
                                hipStream_t s, uint32_t body_w, uint64_t body_n,
                                const uint64_t *d_msg_ends) {
  // (the tile decoder counts heap slots in 32 bits: wires below 4 GiB)
  if (mode == SPK_MODE_VECTOR && var_nested_tile_ok(L) && wire_len < (1ull << 32) - 4096)
    return launch_var_nested_decode(L, d_wire, wire_len, d_recs, rec_cap, d_heaps, heap_caps,
                                    d_res, d_ws, s, body_w, body_n);
  NDec a = {};
  a.ends = d_msg_ends;
  a.body_w = body_w;
  a.body_n = body_n;
  a.N = make_nlayout(L);
  a.fmt = mode == SPK_MODE_VECTOR ? L->fmt_vector : L->fmt_one;
  a.wire_len = wire_len;
  a.n_msgs = n_msgs;
  a.rec_cap = rec_cap;
  a.prefix = prefix;
  for (uint32_t k = 0; k < a.N.n_heaps; ++k) {
    a.heaps[k] = (uint8_t *)d_heaps[k];
    a.heap_cap[k] = heap_caps[k];
  }
  uint8_t *ws = (uint8_t *)d_ws;
  hipError_t er;
  if (mode == SPK_MODE_VECTOR && !a.N.n_ranks) {  // the chunked decode
    const CWs f = cws_layout(wire_len, a.N.n_heaps);
    const uint64_t cap = cws_chunks(wire_len);
    CPtrs P;
    P.ent = reinterpret_cast<uint64_t *>(ws + f.ent);
    P.ext = reinterpret_cast<uint64_t *>(ws + f.ext);
    P.err = reinterpret_cast<int32_t *>(ws + f.err);
    P.dirty = reinterpret_cast<unsigned long long *>(ws + f.dirty);
    if ((er = hipMemsetAsync(P.dirty, 0, (cap + 63) / 64 * 8, s)) != hipSuccess) return er;
    P.cols = reinterpret_cast<uint64_t *>(ws + f.cols);
    const uint64_t nch_max = (wire_len + kNCh - 1) / kNCh;
    P.nch_cap = nch_max;
    (void)cap;
    uint64_t *part = reinterpret_cast<uint64_t *>(ws + f.part);
    // the header decides the chunk count on the device: launch for the
    // largest one the wire allows, lanes past it leave at once
    const unsigned g = nblocks(nch_max, kNT);
    SPK_LAUNCH(nest_vhdr, dim3(1), dim3(1), 0, s, a, (const uint8_t *)d_wire, ws, d_res);
    SPK_LAUNCH(nest_cspec, dim3(g), dim3(kNT), 0, s, a, (const uint8_t *)d_wire,
               (const uint8_t *)ws, P);
    for (int r = 0; r < kNRounds; ++r)
      SPK_LAUNCH(nest_cround, dim3(g), dim3(kNT), 0, s, a, (const uint8_t *)d_wire, ws, P, r);
    SPK_LAUNCH(nest_cverify, dim3(g), dim3(kNT), 0, s, ws, P);
    SPK_LAUNCH(nest_cfix, dim3(1), dim3(64), 0, s, a, (const uint8_t *)d_wire, ws, P);
    // columns scanned over the chunks the wire allows (the speculation
    // pass zeroed the ones past the header's count)
    if ((er = nscan(P.cols, nch_max, 1 + a.N.n_heaps, part, s)) != hipSuccess) return er;
    SPK_LAUNCH(nest_cemit, dim3(g), dim3(kNT), 0, s, a, (const uint8_t *)d_wire, ws, P,
               (uint8_t *)d_recs);
    const uint64_t nb = (nch_max + kNScanBlk - 1) / kNScanBlk;
    SPK_LAUNCH(nest_cfinish, dim3(1), dim3(1), 0, s, a, (const uint64_t *)part, nb,
               (const uint8_t *)ws, d_res);
    return hipGetLastError();
  }
  const uint64_t rows = mode == SPK_MODE_VECTOR ? rec_cap : n_msgs;
  const NWs f = nws_layout(rows, a.N.n_heaps, a.N.n_ranks);
  uint64_t *cpos = reinterpret_cast<uint64_t *>(ws + f.cpos);
  uint64_t *U = reinterpret_cast<uint64_t *>(ws + f.a);
  uint64_t *cons = reinterpret_cast<uint64_t *>(ws + f.b);
  uint64_t *part = reinterpret_cast<uint64_t *>(ws + f.part);
  uint64_t *starts = reinterpret_cast<uint64_t *>(ws + f.starts);
  int32_t *ec = reinterpret_cast<int32_t *>(ws + f.starts);  // MESSAGES: errc per message
  const uint64_t nb = (rows + kNScanBlk - 1) / kNScanBlk;
  if (mode == SPK_MODE_VECTOR && !body_w && compat_tiles_ok(L, wire_len)) {
    // compatible members on the tile decoder, pass by pass; the one-lane walk
    // below runs only when a pass was not clean (CompatCtl::serial)
    const size_t co = compat_ctl_off(L, rows, wire_len);
    if ((er = launch_compat_tiles(L, d_wire, wire_len, d_recs, rec_cap, d_heaps, heap_caps, d_res,
                                  d_ws, co, s)) != hipSuccess)
      return er;
    a.serial = &reinterpret_cast<CompatCtl *>(ws + co)->serial;
  } else if ((er = hipMemsetAsync(d_res, 0, sizeof(spk_dresult_t), s)) != hipSuccess) {
    return er;
  }
  if (mode == SPK_MODE_VECTOR) {  // compatible members: one lane walks the message
    if (rows) {
      const unsigned g = nblocks(rows, 256) < 4096 ? nblocks(rows, 256) : 4096;
      SPK_LAUNCH(nest_fill_u64, dim3(g), dim3(256), 0, s, U, rows * a.N.n_heaps, 0ull, a.serial);
      SPK_LAUNCH(nest_fill_u64, dim3(g), dim3(256), 0, s, cpos, rows * a.N.n_ranks, ~0ull,
                 a.serial);
    }
    SPK_LAUNCH(nest_vhdr, dim3(1), dim3(1), 0, s, a, (const uint8_t *)d_wire, ws, d_res);
    SPK_LAUNCH(nest_vec_serial, dim3(1), dim3(64), 0, s, a, (const uint8_t *)d_wire, ws, U,
               starts, cpos);
    if ((er = nscan(U, rows, a.N.n_heaps, part, s, ws, a.serial)) != hipSuccess) return er;
    if (rows)
      SPK_LAUNCH((nest_emit<SPK_MAX_DEPTH, false>), dim3(nblocks(rows, 256)), dim3(256), 0, s, a,
                 (const uint8_t *)d_wire, d_msg_offsets, (const uint64_t *)starts,
                 (const uint64_t *)U, rows, (const int32_t *)ec, ws, (const uint64_t *)cpos,
                 (uint8_t *)d_recs, mode, (int32_t *)nullptr);
    SPK_LAUNCH(nest_finish, dim3(1), dim3(64), 0, s, a, (const uint64_t *)part, nb,
               (const int32_t *)ec, ws, mode, d_res, (int32_t *)nullptr);
    return hipGetLastError();
  }
  SPK_LAUNCH(nest_ctl_init, dim3(1), dim3(1), 0, s, ws, (const uint32_t *)nullptr);
  if (!n_msgs) return hipGetLastError();
  // (the layout's depth class and heap-use placement select the kernels)
  const size_t ul = n_use_lds(a.N);
  const unsigned gm = nblocks(n_msgs, 256), ge = nblocks(rows, 256);
#define SPK_NMSG_LAUNCH(LU)                                                                    \
  NEST_D(n_dclass(a.N),                                                                        \
         SPK_LAUNCH((nest_msg_count<D, LU>), dim3(gm), dim3(256), ul, s, a,                     \
                    (const uint8_t *)d_wire, d_msg_offsets, U, ec, cons))
#define SPK_NEMIT_LAUNCH(LU)                                                                   \
  NEST_D(n_dclass(a.N),                                                                        \
         SPK_LAUNCH((nest_emit<D, LU>), dim3(ge), dim3(256), ul, s, a, (const uint8_t *)d_wire, \
                    d_msg_offsets, (const uint64_t *)starts, (const uint64_t *)U, rows,         \
                    (const int32_t *)ec, ws, (const uint64_t *)cpos, (uint8_t *)d_recs, mode,   \
                    d_errc))
  if (ul)
    SPK_NMSG_LAUNCH(true);
  else
    SPK_NMSG_LAUNCH(false);
  if ((er = nscan(U, rows, a.N.n_heaps, part, s)) != hipSuccess) return er;
  if (ul)
    SPK_NEMIT_LAUNCH(true);
  else
    SPK_NEMIT_LAUNCH(false);
#undef SPK_NMSG_LAUNCH
#undef SPK_NEMIT_LAUNCH
  SPK_LAUNCH(nest_finish, dim3(1), dim3(64), 0, s, a, (const uint64_t *)part, nb,
             (const int32_t *)ec, ws, mode, d_res, d_errc);
  uint64_t *cpart = reinterpret_cast<uint64_t *>(ws + f.part) + (nb + 1) * a.N.n_heaps;
  if ((er = nscan(cons, rows, 1, cpart, s)) != hipSuccess) return er;
  SPK_LAUNCH(nest_put_consumed, dim3(1), dim3(1), 0, s, (const uint64_t *)cpart, nb, rows,
             d_res);
  return hipGetLastError();
}

}  // namespace spk
