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

namespace spk {

struct NLayout {
  spk_op ops[SPK_MAX_OPS];
  uint8_t heap[SPK_MAX_OPS];  // heap index of a SPAN / OPTION / ARRAY op
  uint8_t end[SPK_MAX_OPS];   // ARRAY: its END; VARIANT: the END of its last alternative
  uint8_t crank[SPK_MAX_OPS]; // COMPAT: its version rank (ops[i].kind is SPK_OP_COMPAT)
  uint32_t n_ops, stride, n_heaps, n_ranks;
  uint32_t fv_cnt, fv_has64, fv_bits;  // USE_FAST_VARINT group: FVAR ops, a 64-bit one, bitset bytes
};

// layouts the interpreter runs: an ARRAY (element layouts), a VARIANT or a
// compatible member
bool layout_nested(const spk_layout *L) {
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const uint32_t k = SPK_OP_KIND(L->ops[i].kind);
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT || k == SPK_OP_COMPAT || k == SPK_OP_FVAR)
      return true;
  }
  return false;
}

static NLayout make_nlayout(const spk_layout *L) {
  NLayout N = {};
  N.n_ops = L->n_ops;
  N.stride = L->rec_stride;
  // open ARRAYs / VARIANTs and the alternatives a VARIANT still has to close
  uint32_t stack[SPK_MAX_DEPTH + 1], left[SPK_MAX_DEPTH + 1], d = 0, h = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    N.ops[i] = L->ops[i];
    const uint32_t k = SPK_OP_KIND(L->ops[i].kind);
    if (k == SPK_OP_COMPAT) {
      N.ops[i].kind = k;
      N.crank[i] = (uint8_t)SPK_OP_RANK(L->ops[i].kind);
      if (N.crank[i] + 1u > N.n_ranks) N.n_ranks = N.crank[i] + 1u;
    }
    if (op_has_heap(k)) N.heap[i] = (uint8_t)h++;
    if (k == SPK_OP_FVAR) {
      ++N.fv_cnt;
      N.fv_has64 |= L->ops[i].size == 8;
    }
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT) {
      stack[d] = i;
      left[d++] = k == SPK_OP_VARIANT ? L->ops[i].size : 1;
    }
    if (k == SPK_OP_END && d && --left[d - 1] == 0) N.end[stack[--d]] = (uint8_t)i;
  }
  N.n_heaps = h;
  N.fv_bits = N.fv_cnt ? (N.fv_cnt + 2 + 7) / 8 : 0;
  return N;
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
__device__ __forceinline__ void n_copy(uint8_t *d, const uint8_t *s, uint64_t n) {
  uint64_t i = 0;
  if ((((uintptr_t)d | (uintptr_t)s) & 7) == 0)
    for (; i + 8 <= n; i += 8)
      *reinterpret_cast<uint64_t *>(d + i) = *reinterpret_cast<const uint64_t *>(s + i);
  for (; i < n; ++i) d[i] = s[i];
}

// one open ARRAY on the interpreter's stack
struct NFrame {
  uint32_t aop, pend;      // the ARRAY / VARIANT op; the op range end to resume
  uint64_t j, cnt;         // element index, element count (a VARIANT: 0 of 1)
  const uint8_t *el;       // element records (encode) / output slots (decode)
  const uint8_t *prec;     // record to resume
  uint32_t first, ret;     // first op of an element / alternative; op to resume at
};

// first op of alternative `a` of the VARIANT at i (groups closed by END)
__device__ __forceinline__ uint32_t n_alt_start(const NLayout &N, uint32_t i, uint32_t a) {
  uint32_t j = i + 1;
  while (a) {
    const uint32_t k = N.ops[j].kind;
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT) {
      j = N.end[j] + 1;  // skip a nested one whole
      continue;
    }
    if (k == SPK_OP_END) --a;
    ++j;
  }
  return j;
}
// the END that closes the alternative starting at j
__device__ __forceinline__ uint32_t n_alt_end(const NLayout &N, uint32_t j) {
  for (;;) {
    const uint32_t k = N.ops[j].kind;
    if (k == SPK_OP_ARRAY || k == SPK_OP_VARIANT) {
      j = N.end[j] + 1;
      continue;
    }
    if (k == SPK_OP_END) return j;
    ++j;
  }
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
__device__ uint8_t *n_fv_write(const NLayout &N, const uint8_t *rec, uint8_t *p) {
  if (!N.fv_cnt) return p;
  const uint32_t code = n_fv_code(N, rec), wb = 1u << code;
  uint8_t bs[(SPK_MAX_VARINTS + 2 + 7) / 8] = {};
  uint8_t *q = p + N.fv_bits;
  uint32_t j = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_FVAR) continue;
    const uint64_t v = n_fv_raw(op, rec);
    if (v) {
      bs[j / 8] |= (uint8_t)(1u << (j % 8));
      const uint32_t rw = wb < op.size ? wb : op.size;
      for (uint32_t b = 0; b < rw; ++b) q[b] = (uint8_t)(v >> (8 * b));
      q += rw;
    }
    ++j;
  }
  bs[N.fv_cnt / 8] |= (uint8_t)((code & 1u) << (N.fv_cnt % 8));
  bs[(N.fv_cnt + 1) / 8] |= (uint8_t)(((code >> 1) & 1u) << ((N.fv_cnt + 1) % 8));
  for (uint32_t b = 0; b < N.fv_bits; ++b) p[b] = bs[b];
  return q;
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
__device__ int32_t n_fv_read(const NLayout &N, const uint8_t *wire, uint64_t &pos, uint64_t end,
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

// ---- encode: size of one record -----------------------------------------------
struct NSize {
  uint64_t bytes, cnts, maxc;  // payload bytes w/o counts, count fields, longest container
  uint64_t cbytes;             // of which in the version passes (compatible members)
};
__device__ NSize n_size(const NLayout &N, const uint8_t *rec, const uint8_t *const *heaps) {
  NSize s = {0, 0, 0, 0};
  s.bytes = n_fv_size(N, rec);
  NFrame st[SPK_MAX_DEPTH];
  uint32_t d = 0, i = 0, iend = N.n_ops;
  const uint8_t *r = rec;
  for (;;) {
    if (i >= iend) {
      if (!d) break;
      NFrame &f = st[d - 1];
      if (++f.j < f.cnt) {
        r = f.el + f.j * N.ops[f.aop].size;
        i = f.first;
        continue;
      }
      i = f.ret;
      iend = f.pend;
      r = f.prec;
      --d;
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_FVAR) {  // in the group
      ++i;
    } else if (op.kind == SPK_OP_COPY) {
      s.bytes += op.size;
      ++i;
    } else if (op.kind == SPK_OP_VARINT) {
      s.bytes += n_vi_len(n_vi_value(op, r));
      ++i;
    } else {
      const uint64_t c = *reinterpret_cast<const uint32_t *>(r + op.rec_off);
      if (op.kind == SPK_OP_VARIANT) {  // [index:1] + the active alternative
        s.bytes += 1;
        const uint32_t a0 = n_alt_start(N, i, (uint32_t)c);
        st[d] = NFrame{i, iend, 0, 1, r, r, a0, (uint32_t)N.end[i] + 1u};
        ++d;
        iend = n_alt_end(N, a0);
        i = a0;
        continue;
      }
      if (op.kind == SPK_OP_OPTION || op.kind == SPK_OP_COMPAT) {  // calculate_size.hpp:100-105
        const uint64_t b = 1 + (c ? op.size : 0);
        s.bytes += b;
        if (op.kind == SPK_OP_COMPAT) s.cbytes += b;
        ++i;
        continue;
      }
      s.cnts += 1;
      if (c > s.maxc) s.maxc = c;
      if (op.kind == SPK_OP_SPAN) {
        s.bytes += c * op.size;
        ++i;
      } else if (!c) {
        i = N.end[i] + 1;
      } else {
        const uint64_t off = *reinterpret_cast<const uint64_t *>(r + op.aux);
        st[d] = NFrame{i, iend, 0, c, heaps[N.heap[i]] + off * op.size, r, i + 1, (uint32_t)N.end[i] + 1u};
        r = st[d].el;
        ++d;
        iend = N.end[i];
        ++i;
      }
    }
  }
  return s;
}

// ---- encode: bytes of one record ----------------------------------------------
__device__ uint8_t *n_write(const NLayout &N, const uint8_t *rec, const uint8_t *const *heaps,
                            uint32_t w, uint8_t *p) {
  NFrame st[SPK_MAX_DEPTH];
  uint32_t d = 0, i = 0, iend = N.n_ops;
  const uint8_t *r = rec;
  p = n_fv_write(N, rec, p);  // before the members (packer.hpp:432-440)
  for (;;) {
    if (i >= iend) {
      if (!d) break;
      NFrame &f = st[d - 1];
      if (++f.j < f.cnt) {
        r = f.el + f.j * N.ops[f.aop].size;
        i = f.first;
        continue;
      }
      i = f.ret;
      iend = f.pend;
      r = f.prec;
      --d;
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_FVAR) {
      ++i;
    } else if (op.kind == SPK_OP_COPY) {
      n_copy(p, r + op.rec_off, op.size);
      p += op.size;
      ++i;
    } else if (op.kind == SPK_OP_VARINT) {
      uint64_t v = n_vi_value(op, r);
      while (v >= 0x80) {
        *p++ = (uint8_t)(v | 0x80u);
        v >>= 7;
      }
      *p++ = (uint8_t)v;
      ++i;
    } else {
      const uint64_t c = *reinterpret_cast<const uint32_t *>(r + op.rec_off);
      if (op.kind == SPK_OP_VARIANT) {
        *p++ = (uint8_t)c;
        const uint32_t a0 = n_alt_start(N, i, (uint32_t)c);
        st[d] = NFrame{i, iend, 0, 1, r, r, a0, (uint32_t)N.end[i] + 1u};
        ++d;
        iend = n_alt_end(N, a0);
        i = a0;
        continue;
      }
      if (op.kind == SPK_OP_COMPAT) {  // version UINT64_MAX: nothing (packer.hpp:246-249)
        ++i;
        continue;
      }
      const uint64_t off = *reinterpret_cast<const uint64_t *>(r + op.aux);
      if (op.kind == SPK_OP_OPTION) {
        *p++ = c ? 1 : 0;
        if (c) {
          n_copy(p, heaps[N.heap[i]] + off * op.size, op.size);
          p += op.size;
        }
        ++i;
        continue;
      }
      for (uint32_t b = 0; b < w; ++b) p[b] = (uint8_t)(c >> (8 * b));
      p += w;
      if (op.kind == SPK_OP_SPAN) {
        n_copy(p, heaps[N.heap[i]] + off * op.size, c * op.size);
        p += c * op.size;
        ++i;
      } else if (!c) {
        i = N.end[i] + 1;
      } else {
        st[d] = NFrame{i, iend, 0, c, heaps[N.heap[i]] + off * op.size, r, i + 1, (uint32_t)N.end[i] + 1u};
        r = st[d].el;
        ++d;
        iend = N.end[i];
        ++i;
      }
    }
  }
  return p;
}

// ---- compatible members: the version pass of rank rk over one top-level record ----
__device__ uint64_t n_compat_size(const NLayout &N, const uint8_t *rec, uint32_t rk) {
  uint64_t b = 0;
  for (uint32_t i = 0; i < N.n_ops; ++i)
    if (N.ops[i].kind == SPK_OP_COMPAT && N.crank[i] == rk)
      b += 1 + (*reinterpret_cast<const uint32_t *>(rec + N.ops[i].rec_off) ? N.ops[i].size : 0);
  return b;
}
// packer.hpp:453-461: [has_value:1][U if present] per member of that version
__device__ uint8_t *n_write_compat(const NLayout &N, const uint8_t *rec,
                                   const uint8_t *const *heaps, uint32_t rk, uint8_t *p) {
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_COMPAT || N.crank[i] != rk) continue;
    const uint32_t c = *reinterpret_cast<const uint32_t *>(rec + op.rec_off);
    *p++ = c ? 1 : 0;
    if (c) {
      const uint64_t off = *reinterpret_cast<const uint64_t *>(rec + op.aux);
      n_copy(p, heaps[N.heap[i]] + off * op.size, op.size);
      p += op.size;
    }
  }
  return p;
}
// unpacker.hpp:1354-1376 over one record: a member whose has byte would start
// at or past data_end ends every version pass without an error (returns 1,
// size_type_ = UCHAR_MAX, :360-365); a missing has byte before it is
// no_buffer_space (*ec, returns 1); a value that does not fit reads as present
// and zero (its errc is dropped). The main pass left every member absent.
__device__ int n_read_compat(const NLayout &N, const uint8_t *wire, uint64_t &pos, uint64_t end,
                             uint64_t data_end, uint32_t rk, uint8_t *rec, uint8_t *const *heaps,
                             uint64_t *used, const uint64_t *heap_cap, uint32_t *ovf,
                             int32_t *ec) {
  for (uint32_t i = 0; i < N.n_ops; ++i) {
    const spk_op op = N.ops[i];
    if (op.kind != SPK_OP_COMPAT || N.crank[i] != rk) continue;
    if (pos >= data_end) return 1;
    if (pos >= end) {
      *ec = SPK_ERRC_NO_BUFFER_SPACE;
      return 1;
    }
    if (!wire[pos++]) continue;
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
          n_copy(heaps[hk] + off * op.size, wire + pos, op.size);
        else
          for (uint32_t b = 0; b < op.size; ++b) heaps[hk][off * op.size + b] = 0;
      }
    }
    used[hk] = off + 1;
    if (fits) pos += op.size;
  }
  return 0;
}

// ---- decode: one record from the wire -------------------------------------------
// Parses wire[pos, end) and advances pos. used[k]: next element slot of heap
// k (counted even when nothing is written). With `rec` set, writes the record,
// its element records and heap payloads, skipping (and flagging in *ovf) what
// does not fit heap_cap. Any non-zero OPTION byte is "has value"; a value that
// does not fit leaves the reader in place and is zero-filled
// (unpacker.hpp:1251-1275).
__device__ int32_t n_read(const NLayout &N, const uint8_t *wire, uint64_t &pos, uint64_t end,
                          uint32_t w, uint8_t *rec, uint8_t *const *heaps, uint64_t *used,
                          const uint64_t *heap_cap, uint32_t *ovf) {
  NFrame st[SPK_MAX_DEPTH];
  uint32_t d = 0, i = 0, iend = N.n_ops;
  uint8_t *r = rec;
  int32_t ec = SPK_ERRC_OK;
  if (N.fv_cnt && (ec = n_fv_read(N, wire, pos, end, rec))) return ec;
  for (;;) {
    if (ec) {
      // unwind to the innermost VARIANT: variant_construct_helper::run
      // (unpacker.hpp:476-490) drops its alternative's errc; an ARRAY keeps
      // its failing element (emplace_back, unpacker.hpp:1208-1226)
      bool dropped = false;
      while (d) {
        NFrame &f = st[d - 1];
        const spk_op &fo = N.ops[f.aop];
        if (fo.kind == SPK_OP_VARIANT) {
          i = f.ret;
          iend = f.pend;
          r = const_cast<uint8_t *>(f.prec);
          --d;
          dropped = true;
          break;
        }
        used[N.heap[f.aop]] -= f.cnt - (f.j + 1);
        if (f.el) *reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(f.prec) + fo.rec_off) =
            (uint32_t)(f.j + 1);
        --d;
      }
      if (!dropped) return ec;
      ec = SPK_ERRC_OK;
      continue;
    }
    if (i >= iend) {
      if (!d) break;
      NFrame &f = st[d - 1];
      if (++f.j < f.cnt) {
        r = f.el ? const_cast<uint8_t *>(f.el) + f.j * N.ops[f.aop].size : nullptr;
        i = f.first;
        continue;
      }
      i = f.ret;
      iend = f.pend;
      r = const_cast<uint8_t *>(f.prec);
      --d;
      continue;
    }
    const spk_op op = N.ops[i];
    if (op.kind == SPK_OP_FVAR) {  // read with the group
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_COPY) {
      if (end - pos < op.size) { ec = SPK_ERRC_NO_BUFFER_SPACE; continue; }
      if (r) n_copy(r + op.rec_off, wire + pos, op.size);
      pos += op.size;
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_VARINT) {  // deserialize_varint (varint.hpp:270-330)
      uint64_t v = 0;
      int32_t vec = SPK_ERRC_INVALID_BUFFER;  // 10 bytes, all continued
      for (uint32_t k = 0; k < 10; ++k) {
        if (pos >= end) {
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
    if (op.kind == SPK_OP_VARIANT) {  // unpacker.hpp:1278-1292
      if (pos >= end) { ec = SPK_ERRC_NO_BUFFER_SPACE; continue; }
      const uint32_t idx = wire[pos++];
      if (idx >= op.size) { ec = SPK_ERRC_INVALID_BUFFER; continue; }
      if (r) *reinterpret_cast<uint32_t *>(r + op.rec_off) = idx;
      const uint32_t a0 = n_alt_start(N, i, idx);
      st[d] = NFrame{i, iend, 0, 1, r, r, a0, (uint32_t)N.end[i] + 1};
      ++d;
      iend = n_alt_end(N, a0);
      i = a0;
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
    if (end - pos < pw) { ec = SPK_ERRC_NO_BUFFER_SPACE; continue; }
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
    if (put && (cnt > 0xFFFFFFFFull || cnt > heap_cap[hk] - (off < heap_cap[hk] ? off : heap_cap[hk]))) {
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
      used[hk] = off + cnt;
      if (!cnt) {
        i = N.end[i] + 1;
        continue;
      }
      st[d] = NFrame{i, iend, 0, cnt, put ? heaps[hk] + off * op.size : nullptr, r, i + 1,
                     (uint32_t)N.end[i] + 1};
      r = put ? heaps[hk] + off * op.size : nullptr;
      ++d;
      iend = N.end[i];
      ++i;
      continue;
    }
    if (op.kind == SPK_OP_OPTION) {
      if (cnt) {
        const bool fits = end - pos >= op.size;
        if (put) {
          if (fits)
            n_copy(heaps[hk] + off * op.size, wire + pos, op.size);
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
      if (op.size > 1 && cnt > ~0ull / op.size) { ec = SPK_ERRC_NO_BUFFER_SPACE; continue; }
      const uint64_t nb = cnt * op.size;
      if (end - pos < nb) { ec = SPK_ERRC_NO_BUFFER_SPACE; continue; }
      if (put) n_copy(heaps[hk] + off * op.size, wire + pos, nb);
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

// ---- device-wide exclusive scan of C u64 columns [C][n] (in place) ---------------
constexpr uint32_t kNScanT = 256, kNScanIPT = 8;
constexpr uint64_t kNScanBlk = (uint64_t)kNScanT * kNScanIPT;

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

__global__ __launch_bounds__(kNScanT) void nscan_reduce(const uint64_t *__restrict__ col,
                                                        uint64_t n, uint64_t *__restrict__ part,
                                                        uint64_t nb) {
  __shared__ uint64_t sh[kNScanT];
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
__global__ __launch_bounds__(1024) void nscan_top(uint64_t *__restrict__ part, uint64_t nb) {
  __shared__ uint64_t sh[1024];
  __shared__ uint64_t carry;
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

__global__ __launch_bounds__(kNScanT) void nscan_apply(uint64_t *__restrict__ col, uint64_t n,
                                                       const uint64_t *__restrict__ part,
                                                       uint64_t nb) {
  __shared__ uint64_t sh[kNScanT];
  const uint64_t c = blockIdx.y;
  const uint64_t base = (uint64_t)blockIdx.x * kNScanBlk + (uint64_t)threadIdx.x * kNScanIPT;
  uint64_t v[kNScanIPT], s = 0;
  for (uint32_t k = 0; k < kNScanIPT; ++k) {
    const uint64_t i = base + k;
    v[k] = i < n ? col[c * n + i] : 0;
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = part[c * (nb + 1) + blockIdx.x] + n_block_excl(s, sh, &tot);
  for (uint32_t k = 0; k < kNScanIPT; ++k) {
    const uint64_t i = base + k;
    if (i < n) col[c * n + i] = run;
    run += v[k];
  }
}

// note: nscan_reduce writes partials with row stride nb; nscan_top/apply read
// them with stride nb + 1 — the host lays the partial table out with nb + 1
// slots per column and passes nb + 1 to the reduce as its stride.
static hipError_t nscan(uint64_t *col, uint64_t n, uint32_t ncols, uint64_t *part,
                        hipStream_t s) {
  if (!n || !ncols) return hipSuccess;
  const uint64_t nb = (n + kNScanBlk - 1) / kNScanBlk;
  SPK_LAUNCH(nscan_reduce, dim3((unsigned)nb, ncols), dim3(kNScanT), 0, s, (const uint64_t *)col,
             n, part, nb + 1);
  SPK_LAUNCH(nscan_top, dim3(ncols), dim3(1024), 0, s, part, nb);
  SPK_LAUNCH(nscan_apply, dim3((unsigned)nb, ncols), dim3(kNScanT), 0, s, col, n,
             (const uint64_t *)part, nb);
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
  const uint32_t cols = n_heaps + 2;
  f.a = take((n + 1) * 8 * cols);
  f.b = take((n + 1) * 8);
  f.part = take(nscan_part_bytes(n + 1, cols));
  f.starts = take((n + 1) * 8);
  f.cpos = take((n + 1) * 8 * (n_ranks ? n_ranks : 1));
  f.end = off;
  return f;
}

size_t nested_workspace_bytes(const spk_layout *L, int, uint64_t n, uint64_t) {
  const NLayout N = make_nlayout(L);
  return nws_layout(n, N.n_heaps, N.n_ranks).end + 256;
}

// control block of the nested path (at kWsCtl)
struct NCtl {
  unsigned long long maxc;   // encode: longest container (atomicMax)
  unsigned long long nrec;   // vector decode: records in the message
  unsigned long long end;    // vector decode: position after the last record
  unsigned long long data_len;
  unsigned long long ovf;
  uint32_t w, errc;
};

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

// a[0][i] = payload bytes, a[1][i] = count fields (VECTOR) or the whole
// message size (MESSAGES); the longest container into ctl->maxc
__global__ __launch_bounds__(256) void nest_size(NEnc e, const uint8_t *__restrict__ recs,
                                                 uint64_t *__restrict__ a, uint8_t *ws) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t m = 0;
  if (i < e.n) {
    const NSize s = n_size(e.N, recs + i * e.N.stride, e.heaps);
    m = s.maxc;
    if (e.mode == SPK_MODE_MESSAGES) {
      const uint32_t w = width_of(s.maxc);
      const uint64_t body = s.bytes + s.cnts * w;
      const uint32_t hl = e.N.n_ranks ? compat_hdr(nullptr, e.fmt, w, body)
                                      : hdr_shape(e.fmt.flags, e.fmt.literal_len, w).len;
      a[i] = e.fpre + hl + body;
      a[e.n + i] = s.bytes;
    } else {
      // main pass bytes; count fields; then one column per version pass
      a[i] = s.bytes - s.cbytes;
      a[e.n + i] = s.cnts;
      for (uint32_t rk = 0; rk < e.N.n_ranks; ++rk)
        a[(2 + rk) * e.n + i] = n_compat_size(e.N, recs + i * e.N.stride, rk);
    }
  }
  // block max -> one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(m, o);
    m = x > m ? x : m;
  }
  if ((threadIdx.x & 63) == 0 && m) atomicMax(&ctl->maxc, (unsigned long long)m);
}

__global__ void nest_ctl_init(uint8_t *ws) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  ctl->maxc = 0;
  ctl->nrec = 0;
  ctl->end = 0;
  ctl->data_len = 0;
  ctl->ovf = 0;
  ctl->w = 1;
  ctl->errc = 0;
}

// VECTOR: sizes[i] = bytes + cnts * w (in place over a[0]), w from maxc
__global__ void nest_vec_sizes(NEnc e, uint64_t *__restrict__ a, uint8_t *ws) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t mx = ctl->maxc > e.n ? ctl->maxc : e.n;
  const uint32_t w = e.fixed_w ? e.fixed_w : width_of(mx);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < e.n;
       i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = a[i] + a[e.n + i] * w;
}

// plan result from the column sums (part tables after the scan)
__global__ void nest_plan_fin(NEnc e, const uint64_t *__restrict__ a,
                              const uint64_t *__restrict__ part, uint64_t nb, uint8_t *ws,
                              spk_plan_t *plan) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
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
__global__ __launch_bounds__(256) void nest_write(NEnc e, const uint8_t *__restrict__ recs,
                                                  const uint64_t *__restrict__ off,
                                                  const uint64_t *__restrict__ part, uint64_t nb,
                                                  uint8_t *ws, uint8_t *__restrict__ out,
                                                  uint64_t *__restrict__ msg_offsets,
                                                  uint32_t with_header, uint64_t out_cap) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e.mode == SPK_MODE_VECTOR) {
    const uint64_t mx = ctl->maxc > e.n ? ctl->maxc : e.n;
    const uint32_t w = e.fixed_w ? e.fixed_w : width_of(mx);
    uint32_t hl = 0;
    const uint64_t tot0 = e.n ? part[nb] : 0;
    uint64_t totc = 0;
    for (uint32_t rk = 0; rk < e.N.n_ranks; ++rk) totc += e.n ? part[(2 + rk) * (nb + 1) + nb] : 0;
    uint8_t hb[4 + 1 + 8 + SPK_MAX_LITERAL + 1];
    if (with_header)
      hl = e.N.n_ranks ? compat_hdr(hb, e.fmt, w, w + tot0 + totc) : write_hdr(hb, e.fmt, w);
    // the whole message must fit, or nothing is written (spk_encode's
    // contract; the caller reads the plan's total_bytes)
    if ((with_header ? hl + w : 0) + tot0 + totc > out_cap) return;
    if (with_header) {
      if (i == 0) {
        for (uint32_t b = 0; b < hl; ++b) out[b] = hb[b];
        for (uint32_t b = 0; b < w; ++b) out[hl + b] = (uint8_t)(e.n >> (8 * b));
      }
      hl += w;
    }
    if (i < e.n) {
      const uint8_t *rec = recs + i * e.N.stride;
      n_write(e.N, rec, e.heaps, w, out + hl + off[i]);
      // version passes after every record's main pass (packer.hpp:66-78)
      uint64_t sec = hl + tot0;
      for (uint32_t rk = 0; rk < e.N.n_ranks; ++rk) {
        n_write_compat(e.N, rec, e.heaps, rk, out + sec + off[(2 + rk) * e.n + i]);
        sec += part[(2 + rk) * (nb + 1) + nb];
      }
    }
    return;
  }
  if ((e.n ? part[nb] : 0) > out_cap) return;  // every message with its frame
  if (i == 0 && msg_offsets) msg_offsets[e.n] = e.n ? part[nb] : 0;
  if (i >= e.n) return;
  const uint8_t *rec = recs + i * e.N.stride;
  const NSize s = n_size(e.N, rec, e.heaps);
  const uint32_t w = width_of(s.maxc);
  uint8_t *p = out + off[i];
  if (msg_offsets) msg_offsets[i] = off[i];
  uint8_t *m = p + e.fpre;
  uint8_t hb[4 + 1 + 8 + SPK_MAX_LITERAL + 1];
  const uint32_t hl = e.N.n_ranks ? compat_hdr(hb, e.fmt, w, s.bytes + s.cnts * w)
                                  : write_hdr(hb, e.fmt, w);
  for (uint32_t b = 0; b < hl; ++b) m[b] = hb[b];
  uint8_t *q = n_write(e.N, rec, e.heaps, w, m + hl);
  for (uint32_t rk = 0; rk < e.N.n_ranks; ++rk) q = n_write_compat(e.N, rec, e.heaps, rk, q);
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
static hipError_t nest_size_scan(const NEnc &e, const void *d_recs, uint8_t *ws, hipStream_t s,
                                 uint64_t **a_out, uint64_t **part_out, uint64_t *nb_out) {
  const NWs f = nws_layout(e.n, e.N.n_heaps, e.N.n_ranks);
  uint64_t *a = reinterpret_cast<uint64_t *>(ws + f.a);
  uint64_t *part = reinterpret_cast<uint64_t *>(ws + f.part);
  SPK_LAUNCH(nest_ctl_init, dim3(1), dim3(1), 0, s, ws);
  if (e.n) {
    SPK_LAUNCH(nest_size, dim3(nblocks(e.n, 256)), dim3(256), 0, s, e, (const uint8_t *)d_recs,
               a, ws);
    if (e.mode == SPK_MODE_VECTOR)
      SPK_LAUNCH(nest_vec_sizes, dim3(nblocks(e.n, 256) < 4096 ? nblocks(e.n, 256) : 4096),
                 dim3(256), 0, s, e, a, ws);
  }
  hipError_t er = hipGetLastError();
  if (er != hipSuccess) return er;
  // VECTOR: column 0 = sizes at w, column 1 = count fields, 2.. = version
  // passes; MESSAGES: column 0 = message sizes, column 1 = payload bytes. All
  // scanned (totals in part).
  const uint32_t cols = e.mode == SPK_MODE_VECTOR ? 2 + e.N.n_ranks : 2;
  if ((er = nscan(a, e.n, cols, part, s)) != hipSuccess) return er;
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
  SPK_LAUNCH(nest_plan_fin, dim3(1), dim3(1), 0, s, e, (const uint64_t *)a,
             (const uint64_t *)part, nb, ws, d_plan);
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
  hipError_t er = nest_size_scan(e, d_recs, ws, s, &a, &part, &nb);
  if (er != hipSuccess) return er;
  SPK_LAUNCH(nest_write, dim3(nblocks(n, 256)), dim3(256), 0, s, e, (const uint8_t *)d_recs,
             (const uint64_t *)a, (const uint64_t *)part, nb, ws, (uint8_t *)d_out,
             d_msg_offsets, fixed_w ? 0u : 1u, out_cap);
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
};

// VECTOR boundary walk: one wave; lane 0 interprets the record counts while
// the wave keeps a window of the wire in LDS (payload bytes are skipped).
// Writes starts[i] (i < rec_cap) and the heap use U[k][i] of every record,
// ctl->nrec / end / errc / w.
constexpr uint32_t kNWin = 4096;
__global__ __launch_bounds__(64) void nest_vec_walk(NDec a, const uint8_t *__restrict__ wire,
                                                    uint8_t *ws, uint64_t *__restrict__ U,
                                                    uint64_t *__restrict__ starts,
                                                    uint64_t *__restrict__ cpos,
                                                    spk_dresult_t *res) {
  __shared__ uint8_t win[kNWin + 16];
  __shared__ unsigned long long s_pos;
  __shared__ int s_done;
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint32_t lane = threadIdx.x;
  const uint64_t len = a.wire_len;
  const NLayout &N = a.N;
  // lane 0's interpreter state
  uint64_t pos = 0, n = 0, rec = 0, used[SPK_MAX_SPANS] = {}, base[SPK_MAX_SPANS] = {};
  uint32_t w = 1, i = 0, iend = N.n_ops, d = 0;
  int32_t errc = 0;
  uint64_t data_len = 0;
  // the version passes of compatible members (ph 1): rank rk, record crec, op ci
  uint32_t ph = 0, rk = 0, ci = 0;
  uint64_t crec = 0;
  bool fvg = false;  // this record's fast-varint group is behind the walk
  struct Fr {
    uint32_t aop, pend;
    uint64_t j, cnt;
    uint32_t first, ret;
  } st[SPK_MAX_DEPTH];
  if (lane == 0 && a.body_w) {
    w = a.body_w;
    n = a.body_n;
    s_pos = 0;
    s_done = n == 0;
    if (n && a.rec_cap) starts[0] = 0;
  } else if (lane == 0) {
    uint64_t p0;
    errc = parse_hdr(a.fmt, wire, len, &p0, &w, &data_len);
    pos = p0;
    if (!errc) {
      if (len - pos < w) {
        errc = SPK_ERRC_NO_BUFFER_SPACE;
      } else {
        n = ld_le(wire + pos, w);
        pos += w;
      }
    }
    s_pos = pos;
    s_done = errc != 0 || n == 0;
    if (!errc && n && a.rec_cap) starts[0] = pos;
  }
  __syncthreads();
  uint64_t wbase = ~0ull;
  while (!s_done) {
    // refill the window at the walk position
    const uint64_t wp = s_pos;
    if (wp != wbase) {
      for (uint32_t b = lane * 16; b < kNWin; b += 64 * 16)
        for (uint32_t q = 0; q < 16; ++q)
          win[b + q] = wp + b + q < len ? wire[wp + b + q] : 0;
      wbase = wp;
    }
    __syncthreads();
    if (lane == 0) {
      const uint64_t wend = wbase + kNWin < len ? wbase + kNWin : len;
      auto byte = [&](uint64_t x) -> uint32_t { return win[x - wbase]; };
      // an error inside a VARIANT alternative is dropped (the walk goes on
      // after the variant, unpacker.hpp:476-490); an ARRAY keeps its failing
      // element. Returns false when the error ends the message.
      auto fail = [&](int32_t e) -> bool {
        while (d) {
          Fr &f = st[d - 1];
          if (N.ops[f.aop].kind == SPK_OP_VARIANT) {
            i = f.ret;
            iend = f.pend;
            --d;
            return true;
          }
          used[N.heap[f.aop]] -= f.cnt - (f.j + 1);
          --d;
        }
        errc = e;
        return false;
      };
      bool stall = false, done = false;
      while (!stall && !done) {
        if (ph) {  // unpacker.hpp:292-366,1354-1376
          if (rk >= N.n_ranks) {
            done = true;
            break;
          }
          if (crec >= n) {
            ++rk;
            crec = 0;
            ci = 0;
            continue;
          }
          if (ci == 0 && crec < a.rec_cap) cpos[(uint64_t)rk * a.rec_cap + crec] = pos;
          while (ci < N.n_ops && !(N.ops[ci].kind == SPK_OP_COMPAT && N.crank[ci] == rk)) ++ci;
          if (ci >= N.n_ops) {
            ++crec;
            ci = 0;
            continue;
          }
          if (pos >= data_len) {  // an older writer: the legal end
            done = true;
            break;
          }
          if (wend < len && pos + 1 > wend) {
            stall = true;
            break;
          }
          if (pos >= len) {
            errc = SPK_ERRC_NO_BUFFER_SPACE;
            done = true;
            break;
          }
          if (byte(pos++)) {
            if (crec < a.rec_cap) U[(uint64_t)N.heap[ci] * a.rec_cap + crec] = 1;
            if (len - pos >= N.ops[ci].size) pos += N.ops[ci].size;
          }
          ++ci;
          continue;
        }
        if (i >= iend) {
          if (d) {
            Fr &f = st[d - 1];
            if (++f.j < f.cnt) {
              i = f.first;
              continue;
            }
            i = f.ret;
            iend = f.pend;
            --d;
            continue;
          }
          // record `rec` complete
          if (rec < a.rec_cap)
            for (uint32_t k = 0; k < N.n_heaps; ++k) U[(uint64_t)k * a.rec_cap + rec] = used[k] - base[k];
          for (uint32_t k = 0; k < N.n_heaps; ++k) base[k] = used[k];
          ++rec;
          if (rec == n) {
            if (N.n_ranks) {
              ph = 1;
              continue;
            }
            done = true;
            break;
          }
          if (rec < a.rec_cap) starts[rec] = pos;
          i = 0;
          iend = N.n_ops;
          fvg = false;
          continue;
        }
        if (N.fv_cnt && !fvg) {  // the record's USE_FAST_VARINT group comes first
          if (wend < len && pos + N.fv_bits > wend) {
            stall = true;
            break;
          }
          int32_t ge = SPK_ERRC_OK;
          uint64_t g = 0;
          if (len - pos < N.fv_bits) {
            ge = SPK_ERRC_NO_BUFFER_SPACE;
          } else {
            uint8_t bs[(SPK_MAX_VARINTS + 2 + 7) / 8];
            for (uint32_t b = 0; b < N.fv_bits; ++b) bs[b] = (uint8_t)byte(pos + b);
            g = n_fv_len(N, bs);
            ge = !g ? SPK_ERRC_INVALID_BUFFER : len - pos < g ? SPK_ERRC_NO_BUFFER_SPACE : 0;
          }
          if (ge) {
            if (!fail(ge)) {
              done = true;
              break;
            }
            continue;
          }
          pos += g;
          fvg = true;
          continue;
        }
        const spk_op op = N.ops[i];
        if (op.kind == SPK_OP_FVAR) {  // in the group
          ++i;
          continue;
        }
        if (op.kind == SPK_OP_COMPAT) {  // main pass: nothing on the wire
          ++i;
          continue;
        }
        if (op.kind == SPK_OP_COPY) {
          if (len - pos < op.size) {
            if (!fail(SPK_ERRC_NO_BUFFER_SPACE)) {
              done = true;
              break;
            }
            continue;
          }
          pos += op.size;  // skipped, not read
          ++i;
          continue;
        }
        // every other op reads at most 10 bytes: refill when the window (not
        // the wire) ends before them
        const uint64_t need = op.kind == SPK_OP_VARINT ? 10
                              : (op.kind == SPK_OP_OPTION || op.kind == SPK_OP_VARIANT) ? 1
                                                                                          : w;
        if (wend < len && pos + need > wend) {
          stall = true;
          break;
        }
        if (op.kind == SPK_OP_VARINT) {
          int32_t vec = SPK_ERRC_INVALID_BUFFER;
          for (uint32_t k = 0; k < 10; ++k) {
            if (pos >= len) {
              vec = SPK_ERRC_NO_BUFFER_SPACE;
              break;
            }
            if (!(byte(pos++) & 0x80u)) {
              vec = SPK_ERRC_OK;
              break;
            }
          }
          if (vec) {
            if (!fail(vec)) {
              done = true;
              break;
            }
            continue;
          }
          ++i;
          continue;
        }
        if (op.kind == SPK_OP_VARIANT) {
          if (pos >= len) {
            if (!fail(SPK_ERRC_NO_BUFFER_SPACE)) {
              done = true;
              break;
            }
            continue;
          }
          const uint32_t idx = byte(pos++);
          if (idx >= op.size || d == SPK_MAX_DEPTH) {
            if (!fail(SPK_ERRC_INVALID_BUFFER)) {
              done = true;
              break;
            }
            continue;
          }
          const uint32_t a0 = n_alt_start(N, i, idx);
          st[d++] = Fr{i, iend, 0, 1, a0, (uint32_t)N.end[i] + 1};
          iend = n_alt_end(N, a0);
          i = a0;
          continue;
        }
        const uint32_t hk = N.heap[i];
        const uint32_t pw = op.kind == SPK_OP_OPTION ? 1u : w;
        if (len - pos < pw) {
          if (!fail(SPK_ERRC_NO_BUFFER_SPACE)) {
            done = true;
            break;
          }
          continue;
        }
        uint64_t cnt = 0;
        if (op.kind == SPK_OP_OPTION)
          cnt = byte(pos) != 0;
        else
          for (uint32_t b = 0; b < w; ++b) cnt |= (uint64_t)byte(pos + b) << (8 * b);
        pos += pw;
        if (op.kind != SPK_OP_SPAN) used[hk] += cnt;
        if (op.kind == SPK_OP_ARRAY) {
          if (!cnt) {
            i = N.end[i] + 1;
            continue;
          }
          if (d == SPK_MAX_DEPTH) {  // (layout_check bounds the depth)
            if (!fail(SPK_ERRC_INVALID_BUFFER)) {
              done = true;
              break;
            }
            continue;
          }
          st[d++] = Fr{i, iend, 0, cnt, i + 1, (uint32_t)N.end[i] + 1};
          iend = N.end[i];
          ++i;
          continue;
        }
        if (op.kind == SPK_OP_OPTION) {
          if (cnt && len - pos >= op.size) pos += op.size;  // else: unreadable, reader stays
          ++i;
          continue;
        }
        if (cnt) {
          if ((op.size > 1 && cnt > ~0ull / op.size) || len - pos < cnt * op.size) {
            if (!fail(SPK_ERRC_NO_BUFFER_SPACE)) {
              done = true;
              break;
            }
            continue;
          }
          pos += cnt * op.size;
        }
        used[hk] += cnt;
        ++i;
      }
      s_pos = pos;
      s_done = done;
    }
    __syncthreads();
  }
  if (lane == 0) {
    ctl->errc = (uint32_t)errc;
    ctl->w = w;
    ctl->nrec = errc ? 0 : n;
    ctl->end = pos;
    ctl->data_len = data_len;
    spk_dresult_t r = {};
    r.errc = errc;
    r.width = w;
    *res = r;
  }
}

// MESSAGES count pass: errc and heap use of every message (no writes)
__global__ __launch_bounds__(256) void nest_msg_count(NDec a, const uint8_t *__restrict__ wire,
                                                      const uint64_t *__restrict__ offs,
                                                      uint64_t *__restrict__ U,
                                                      int32_t *__restrict__ ec,
                                                      uint64_t *__restrict__ cons) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_msgs) return;
  const NLayout &N = a.N;
  uint64_t used[SPK_MAX_SPANS] = {};
  const uint64_t b = offs[i], e = a.ends ? a.ends[i] : offs[i + 1];
  int32_t errc = SPK_ERRC_OK;
  uint64_t consumed = 0;
  if (e < b || e > a.wire_len || e - b < a.prefix) {
    errc = SPK_ERRC_NO_BUFFER_SPACE;
  } else {
    const uint64_t m0 = b + a.prefix;
    uint64_t p0, dl;
    uint32_t w;
    errc = parse_hdr(a.fmt, wire + m0, e - m0, &p0, &w, &dl);
    if (!errc) {
      uint64_t pos = m0 + p0;
      uint32_t ovf = 0;
      errc = n_read(N, wire, pos, e, w, nullptr, nullptr, used, a.heap_cap, &ovf);
      for (uint32_t rk = 0; !errc && rk < N.n_ranks; ++rk)
        if (n_read_compat(N, wire, pos, e, m0 + dl, rk, nullptr, nullptr, used, a.heap_cap, &ovf,
                          &errc))
          break;
      consumed = pos - m0 > dl ? pos - m0 : dl;  // consume_len (struct_pack.hpp:343-357)
    }
    if (!errc && i >= a.rec_cap) errc = SPK_ERRC_CAPACITY;
  }
  ec[i] = errc;
  cons[i] = errc ? 0 : consumed;
  for (uint32_t k = 0; k < N.n_heaps; ++k) U[(uint64_t)k * a.n_msgs + i] = errc ? 0 : used[k];
}

// write pass (both modes): record i from its start with heap bases B[k][i]
__global__ __launch_bounds__(256) void nest_emit(NDec a, const uint8_t *__restrict__ wire,
                                                 const uint64_t *__restrict__ offs,
                                                 const uint64_t *__restrict__ starts,
                                                 const uint64_t *__restrict__ B, uint64_t nrows,
                                                 const int32_t *__restrict__ ec, uint8_t *ws,
                                                 const uint64_t *__restrict__ cpos,
                                                 uint8_t *__restrict__ recs, int mode) {
  NCtl *ctl = reinterpret_cast<NCtl *>(ws + kWsCtl);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const NLayout &N = a.N;
  uint64_t pos, end, data_end;
  uint32_t w;
  if (mode == SPK_MODE_VECTOR) {
    if (ctl->errc || i >= ctl->nrec || i >= a.rec_cap) return;
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
  uint64_t used[SPK_MAX_SPANS];
  for (uint32_t k = 0; k < N.n_heaps; ++k) used[k] = B[(uint64_t)k * nrows + i];
  uint32_t ovf = 0;
  uint8_t *rec = recs + i * N.stride;
  n_read(N, wire, pos, end, w, rec, a.heaps, used, a.heap_cap, &ovf);
  int32_t cec = 0;
  for (uint32_t rk = 0; rk < N.n_ranks; ++rk) {
    if (mode == SPK_MODE_VECTOR) {  // this record's group of version rk (walker)
      pos = cpos[(uint64_t)rk * a.rec_cap + i];
      if (pos == ~0ull) break;
    }
    if (n_read_compat(N, wire, pos, end, data_end, rk, rec, a.heaps, used, a.heap_cap, &ovf, &cec))
      break;
  }
  if (ovf) atomicAdd(&ctl->ovf, 1ull);
}

// result: count, consume_len, heap use (column totals), capacity errors
__global__ void nest_finish(NDec a, const uint64_t *__restrict__ part, uint64_t nb,
                            const int32_t *__restrict__ ec, uint8_t *ws, int mode,
                            spk_dresult_t *res, int32_t *__restrict__ errc_out) {
  const NCtl *ctl = reinterpret_cast<const NCtl *>(ws + kWsCtl);
  __shared__ unsigned long long s_ok, s_cap;
  if (threadIdx.x == 0) {
    s_ok = 0;
    s_cap = 0;
  }
  __syncthreads();
  if (mode == SPK_MODE_MESSAGES) {
    unsigned long long ok = 0, cap = 0;
    for (uint64_t i = threadIdx.x; i < a.n_msgs; i += blockDim.x) {
      if (errc_out) errc_out[i] = ec[i];
      cap |= ec[i] == SPK_ERRC_CAPACITY;
      ok += ec[i] == 0;
    }
    atomicAdd(&s_ok, ok);
    if (cap) atomicOr(&s_cap, 1ull);
  }
  __syncthreads();
  if (threadIdx.x) return;
  spk_dresult_t r = *res;
  const uint32_t nh = a.N.n_heaps;
  if (mode == SPK_MODE_VECTOR) {
    if (ctl->errc) return;  // errc already in *res
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
  const uint64_t rows = mode == SPK_MODE_VECTOR ? rec_cap : n_msgs;
  const NWs f = nws_layout(rows, a.N.n_heaps, a.N.n_ranks);
  uint64_t *cpos = reinterpret_cast<uint64_t *>(ws + f.cpos);
  uint64_t *U = reinterpret_cast<uint64_t *>(ws + f.a);
  uint64_t *cons = reinterpret_cast<uint64_t *>(ws + f.b);
  uint64_t *part = reinterpret_cast<uint64_t *>(ws + f.part);
  uint64_t *starts = reinterpret_cast<uint64_t *>(ws + f.starts);
  int32_t *ec = reinterpret_cast<int32_t *>(ws + f.starts);  // MESSAGES: errc per message
  const uint64_t nb = (rows + kNScanBlk - 1) / kNScanBlk;
  hipError_t er = hipMemsetAsync(d_res, 0, sizeof(spk_dresult_t), s);
  if (er != hipSuccess) return er;
  SPK_LAUNCH(nest_ctl_init, dim3(1), dim3(1), 0, s, ws);
  if (mode == SPK_MODE_VECTOR) {
    if (rows && (er = hipMemsetAsync(U, 0, rows * 8 * a.N.n_heaps, s)) != hipSuccess) return er;
    if (rows && a.N.n_ranks &&
        (er = hipMemsetAsync(cpos, 0xFF, rows * 8 * a.N.n_ranks, s)) != hipSuccess)
      return er;
    SPK_LAUNCH(nest_vec_walk, dim3(1), dim3(64), 0, s, a, (const uint8_t *)d_wire, ws, U, starts,
               cpos, d_res);
    if ((er = nscan(U, rows, a.N.n_heaps, part, s)) != hipSuccess) return er;
    if (rows)
      SPK_LAUNCH(nest_emit, dim3(nblocks(rows, 256)), dim3(256), 0, s, a, (const uint8_t *)d_wire,
                 d_msg_offsets, (const uint64_t *)starts, (const uint64_t *)U, rows,
                 (const int32_t *)ec, ws, (const uint64_t *)cpos, (uint8_t *)d_recs, mode);
    SPK_LAUNCH(nest_finish, dim3(1), dim3(256), 0, s, a, (const uint64_t *)part, nb,
               (const int32_t *)ec, ws, mode, d_res, (int32_t *)nullptr);
    return hipGetLastError();
  }
  if (!n_msgs) return hipGetLastError();
  SPK_LAUNCH(nest_msg_count, dim3(nblocks(n_msgs, 256)), dim3(256), 0, s, a,
             (const uint8_t *)d_wire, d_msg_offsets, U, ec, cons);
  if ((er = nscan(U, rows, a.N.n_heaps, part, s)) != hipSuccess) return er;
  SPK_LAUNCH(nest_emit, dim3(nblocks(rows, 256)), dim3(256), 0, s, a, (const uint8_t *)d_wire,
             d_msg_offsets, (const uint64_t *)starts, (const uint64_t *)U, rows,
             (const int32_t *)ec, ws, (const uint64_t *)cpos, (uint8_t *)d_recs, mode);
  SPK_LAUNCH(nest_finish, dim3(1), dim3(256), 0, s, a, (const uint64_t *)part, nb,
             (const int32_t *)ec, ws, mode, d_res, d_errc);
  uint64_t *cpart = reinterpret_cast<uint64_t *>(ws + f.part) + (nb + 1) * a.N.n_heaps;
  if ((er = nscan(cons, rows, 1, cpart, s)) != hipSuccess) return er;
  SPK_LAUNCH(nest_put_consumed, dim3(1), dim3(1), 0, s, (const uint64_t *)cpart, nb, rows,
             d_res);
  return hipGetLastError();
}

}  // namespace spk
