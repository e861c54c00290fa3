/*
 * spk_oracle.c — plain-C restatement of struct_pack's encode/decode for the
 * record model of include/spk_codec.h. TEST INFRASTRUCTURE ONLY (see
 * spk_oracle.h); pinned against the reference's own bytes in tests/golden/.
 *
 * Every function cites the reference code (paths relative to
 * /root/reference/include/ylt/) whose behaviour it restates.
 */
#include "spk_oracle.h"

#include <string.h>

/* ---- little-endian primitives: struct_pack/endian_wrapper.hpp:136-271 -- */
static void put_le(uint8_t *p, uint64_t v, unsigned w) {
  for (unsigned i = 0; i < w; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
static uint64_t get_le(const uint8_t *p, unsigned w) {
  uint64_t v = 0;
  for (unsigned i = 0; i < w; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

/* ---- varints: struct_pack/varint.hpp ------------------------------------ */
/* the unsigned value serialize_varint puts on the wire (varint.hpp:245-268):
 * sint<T> is zigzag-mapped at its own width (encode_zigzag, :194-210),
 * varint<T> is the value itself */
static uint64_t vi_value(const uint8_t *rec, const spk_op *op) {
  if (op->size == 4) {
    uint32_t u;
    memcpy(&u, rec + op->rec_off, 4);
    if (op->aux & SPK_VARINT_SEXT) return (uint64_t)(int64_t)(int32_t)u; /* v = t */
    if (op->aux & SPK_VARINT_ZIGZAG) u = (u << 1) ^ (uint32_t)(-(int32_t)(u >> 31));
    return u;
  }
  uint64_t u;
  memcpy(&u, rec + op->rec_off, 8);
  if (op->aux & SPK_VARINT_ZIGZAG) u = (u << 1) ^ (uint64_t)(-(int64_t)(u >> 63));
  return u;
}
/* calculate_varint_size (varint.hpp:212-239) */
static unsigned vi_len(uint64_t v) {
  unsigned n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
/* deserialize_varint (varint.hpp:270-330): LEB128 of at most 10 bytes; the
 * value is truncated to the member width, zigzag-decoded at 64 bits first
 * for the signed types */
static void vi_store(uint8_t *rec, const spk_op *op, uint64_t v) {
  if (op->aux & SPK_VARINT_ZIGZAG) v = (v >> 1) ^ (uint64_t)(-(int64_t)(v & 1));
  put_le(rec + op->rec_off, v, op->size);
}

/* ---- layout helpers ---------------------------------------------------- */
/* Heaps are numbered in op order over SPAN, OPTION and ARRAY ops at every
 * nesting level; an ARRAY's element ops run to its matching END. */
static int is_heap_op(uint32_t k) {
  k = SPK_OP_KIND(k);
  return k == SPK_OP_SPAN || k == SPK_OP_OPTION || k == SPK_OP_ARRAY || k == SPK_OP_COMPAT;
}
/* compatible<U, ver> members: top-level ops only (include/spk_codec.h);
 * COMPAT holds a trivially serializable U in a heap, CGROUP its ops inline */
static int is_compat(uint32_t k) { return SPK_OP_KIND(k) == SPK_OP_COMPAT; }
static int is_cgroup(uint32_t k) { return SPK_OP_KIND(k) == SPK_OP_CGROUP; }
/* VARIANT / OPTGROUP / CGROUP: op groups closed by END in the same record */
static int is_group(uint32_t k) {
  k = SPK_OP_KIND(k);
  return k == SPK_OP_VARIANT || k == SPK_OP_OPTGROUP || k == SPK_OP_CGROUP;
}
/* number of distinct version ranks (max rank + 1), 0 without compat members */
static unsigned compat_ranks(const spk_layout *L) {
  unsigned r = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i)
    if ((is_compat(L->ops[i].kind) || is_cgroup(L->ops[i].kind)) &&
        SPK_OP_RANK(L->ops[i].kind) + 1 > r)
      r = SPK_OP_RANK(L->ops[i].kind) + 1;
  return r;
}
static unsigned heap_of(const spk_layout *L, uint32_t i) {
  unsigned k = 0;
  for (uint32_t j = 0; j < i; ++j) k += is_heap_op(L->ops[j].kind);
  return k;
}
static uint32_t end_of(const spk_layout *L, uint32_t i);
/* the END closing the op group (element layout / alternative) starting at j */
static uint32_t group_end(const spk_layout *L, uint32_t j) {
  while (j < L->n_ops) {
    const uint32_t k = L->ops[j].kind;
    if (k == SPK_OP_ARRAY || is_group(k)) {
      j = end_of(L, j) + 1;
      continue;
    }
    if (k == SPK_OP_END) return j;
    ++j;
  }
  return L->n_ops;
}
/* ARRAY at i -> its END; a group op at i -> the END of its last group */
static uint32_t end_of(const spk_layout *L, uint32_t i) {
  if (L->ops[i].kind == SPK_OP_ARRAY) return group_end(L, i + 1);
  uint32_t j = i + 1;
  for (uint32_t a = 0; a < L->ops[i].size; ++a) j = group_end(L, j) + 1;
  return j - 1;
}
/* first op of alternative a of the VARIANT (group a of the OPTGROUP) at i */
static uint32_t alt_start(const spk_layout *L, uint32_t i, uint32_t a) {
  uint32_t j = i + 1;
  while (a--) j = group_end(L, j) + 1;
  return j;
}
/* the group a VARIANT / OPTGROUP writes: the variant's index; for an optional
 * / expected (packer.hpp:382-388,400-410) group 0 (the value) when has_value,
 * else group 1 of an expected (its error) or none (-1) */
static int active_group(const spk_layout *L, uint32_t i, const uint8_t *rec) {
  uint32_t v;
  memcpy(&v, rec + L->ops[i].rec_off, 4);
  if (L->ops[i].kind == SPK_OP_VARIANT) return (int)v;
  return v ? 0 : (L->ops[i].size == 2 ? 1 : -1);
}
/* ---- USE_FAST_VARINT group of the top-level record (packer.hpp:152-235,
 * calculate_size.hpp:191-390, unpacker.hpp:642-747) ---------------------- */
typedef struct fv_t {
  unsigned cnt, has64, bits; /* FVAR ops, any 64-bit one, bitset bytes */
} fv_t;
static fv_t fv_shape(const spk_layout *L) {
  fv_t f = {0, 0, 0};
  for (uint32_t i = 0; i < L->n_ops; ++i)
    if (L->ops[i].kind == SPK_OP_FVAR) {
      ++f.cnt;
      f.has64 |= L->ops[i].size == 8;
    }
  f.bits = f.cnt ? (f.cnt + 2 + 7) / 8 : 0;
  return f;
}
static int64_t fv_signed(const uint8_t *rec, const spk_op *op) {
  if (op->size == 4) {
    int32_t v;
    memcpy(&v, rec + op->rec_off, 4);
    return v;
  }
  int64_t v;
  memcpy(&v, rec + op->rec_off, 8);
  return v;
}
static uint64_t fv_raw(const uint8_t *rec, const spk_op *op) {
  uint64_t v = 0;
  memcpy(&v, rec + op->rec_off, op->size);
  return v;
}
/* get_fast_varint_width_from_max: 0..3 from the largest unsigned value and
   the largest signed magnitude (v > 0 ? v : -(v + 1)) of the non-zero ones */
static unsigned fv_code(const spk_layout *L, const uint8_t *rec) {
  uint64_t um = 0, sm = 0;
  int hu = 0, hs = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const spk_op *op = &L->ops[i];
    if (op->kind != SPK_OP_FVAR) continue;
    if (op->aux & SPK_FVAR_SIGNED) {
      hs = 1;
      const int64_t v = fv_signed(rec, op);
      const uint64_t m = v > 0 ? (uint64_t)v : (uint64_t)(-(v + 1));
      if (v && m > sm) sm = m;
    } else {
      hu = 1;
      const uint64_t v = fv_raw(rec, op);
      if (v > um) um = v;
    }
  }
  unsigned cu = um <= 0xFFull ? 0 : um <= 0xFFFFull ? 1 : um <= 0xFFFFFFFFull ? 2 : 3;
  unsigned cs = sm <= 0x7Full ? 0 : sm <= 0x7FFFull ? 1 : sm <= 0x7FFFFFFFull ? 2 : 3;
  if (!hu) cu = 0;
  if (!hs) cs = 0;
  return cu > cs ? cu : cs;
}
static uint64_t fv_size(const spk_layout *L, const uint8_t *rec) {
  const fv_t f = fv_shape(L);
  if (!f.cnt) return 0;
  const unsigned wb = 1u << fv_code(L, rec);
  uint64_t b = f.bits;
  for (uint32_t i = 0; i < L->n_ops; ++i)
    if (L->ops[i].kind == SPK_OP_FVAR && fv_raw(rec, &L->ops[i]))
      b += wb < L->ops[i].size ? wb : L->ops[i].size;
  return b;
}
static uint8_t *fv_write(const spk_layout *L, const uint8_t *rec, uint8_t *p) {
  const fv_t f = fv_shape(L);
  if (!f.cnt) return p;
  const unsigned code = fv_code(L, rec), wb = 1u << code;
  uint8_t *bs = p;
  memset(bs, 0, f.bits);
  p += f.bits;
  unsigned j = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const spk_op *op = &L->ops[i];
    if (op->kind != SPK_OP_FVAR) continue;
    const uint64_t v = fv_raw(rec, op);
    if (v) {
      bs[j / 8] |= (uint8_t)(1u << (j % 8));
      const unsigned rw = wb < op->size ? wb : op->size;
      put_le(p, v, rw); /* low_bytes_write_wrapper */
      p += rw;
    }
    ++j;
  }
  bs[f.cnt / 8] |= (uint8_t)((code & 1u) << (f.cnt % 8));
  bs[(f.cnt + 1) / 8] |= (uint8_t)(((code >> 1) & 1u) << ((f.cnt + 1) % 8));
  return p;
}

static uint64_t rec_count(const uint8_t *rec, const spk_op *op) {
  uint32_t c;
  memcpy(&c, rec + op->rec_off, 4);
  if (op->kind == SPK_OP_OPTION || is_compat(op->kind)) return c != 0; /* has_value() */
  return c;
}
/* prefix bytes of a SPAN / ARRAY (container length, width w) or an OPTION
 * (the bool has_value: write_wrapper<sizeof(bool)>, packer.hpp:382-388) */
static unsigned op_pw(const spk_op *op, unsigned w) {
  return (op->kind == SPK_OP_OPTION || is_compat(op->kind)) ? 1u : w;
}
static uint64_t rec_heapoff(const uint8_t *rec, const spk_op *op) {
  uint64_t o;
  memcpy(&o, rec + op->aux, 8);
  return o;
}

/* width selection: calculate_size.hpp:426-447 */
static unsigned width_of(uint64_t max_count) {
  if (max_count < (1ull << 8)) return 1;
  if (max_count < (1ull << 16)) return 2;
  if (max_count < (1ull << 32)) return 4;
  return 8;
}
static unsigned width_bits(unsigned w) {
  return w == 1 ? 0u : w == 2 ? 0x08u : w == 4 ? 0x10u : 0x18u;
}

/* Header shape: check_has_metainfo (type_calculate.hpp:884-891),
 * get_serialize_runtime_info (calculate_size.hpp:407-474) and
 * serialize_metainfo (packer.hpp:100-139). With compatible members the
 * metainfo byte is always present and is followed by the total message
 * length in 2/4/8 bytes; `body` = every byte after the header. */
typedef struct hdr_t {
  unsigned head, lit, has_meta, len, lenw;
  uint8_t meta;
  uint64_t total;
} hdr_t;

static hdr_t header_shape(const spk_msgfmt *f, unsigned w, int compat, uint64_t body) {
  hdr_t h;
  unsigned has_container = (f->flags & SPK_MF_HAS_CONTAINER) != 0;
  h.head = (f->flags & SPK_MF_HASH_HEAD) != 0;
  h.lit = h.head && (f->flags & SPK_MF_TYPE_LITERAL);
  unsigned meta_fixed = compat || h.lit || (!h.head && has_container);
  if (!has_container) w = 1;
  h.has_meta = meta_fixed || w > 1;
  h.meta = (uint8_t)(width_bits(w) | (h.lit ? 0x04u : 0u));
  h.len = (h.head ? 4u : 0u) + (h.has_meta ? 1u : 0u) +
          (h.lit ? f->literal_len + 1u : 0u);
  h.lenw = 0;
  if (compat && h.head) { /* calculate_size.hpp:457-470 */
    const uint64_t l = h.len + body;
    if (l + 2 < (1ull << 16)) h.lenw = 2, h.meta |= 1;
    else if (l + 4 < (1ull << 32)) h.lenw = 4, h.meta |= 2;
    else h.lenw = 8, h.meta |= 3;
  }
  h.len += h.lenw;
  h.total = h.len + body;
  return h;
}

static uint8_t *write_header(uint8_t *p, const spk_msgfmt *f, const hdr_t *h) {
  if (h->head) { /* packer.hpp:103-107: LSB = more metainfo follows */
    put_le(p, (f->code & ~1u) | (h->has_meta ? 1u : 0u), 4);
    p += 4;
  }
  if (h->has_meta) *p++ = h->meta; /* packer.hpp:108-110 */
  if (h->lenw) {                   /* packer.hpp:111-130: info_.size() */
    put_le(p, h->total, h->lenw);
    p += h->lenw;
  }
  if (h->lit) {                    /* packer.hpp:132-137: literal + NUL */
    memcpy(p, f->literal, f->literal_len);
    p += f->literal_len;
    *p++ = 0;
  }
  return p;
}

/* calculate_one_size (calculate_size.hpp:39-183) of ops [i0, i1) over one
 * (element) record: payload bytes without count fields in *bytes, count
 * fields (size_cnt) in *cnts, the largest container length (max_size) in
 * *maxc; a container of non-trivially-serializable elements sums its
 * elements (calculate_size.hpp:76-87) */
static void ops_size(const spk_layout *L, uint32_t i0, uint32_t i1, const uint8_t *rec,
                     const void *const *heaps, uint64_t *bytes, uint64_t *cnts,
                     uint64_t *maxc) {
  for (uint32_t i = i0; i < i1; ++i) {
    const spk_op *op = &L->ops[i];
    if (op->kind == SPK_OP_COPY) {
      *bytes += op->size;
    } else if (is_compat(op->kind)) { /* calculate_size.hpp:100-105 (optional) */
      *bytes += 1 + rec_count(rec, op) * op->size;
    } else if (op->kind == SPK_OP_VARINT) {
      *bytes += vi_len(vi_value(rec, op));
    } else if (op->kind == SPK_OP_OPTION) {
      *bytes += 1 + rec_count(rec, op) * op->size;
    } else if (op->kind == SPK_OP_SPAN) {
      uint64_t c = rec_count(rec, op);
      *cnts += 1;
      *bytes += c * op->size;
      if (c > *maxc) *maxc = c;
    } else if (op->kind == SPK_OP_VARIANT || op->kind == SPK_OP_OPTGROUP) {
      /* index / has_value byte + the active group (calculate_size.hpp:100-105) */
      const int a = active_group(L, i, rec);
      *bytes += 1;
      if (a >= 0) {
        const uint32_t a0 = alt_start(L, i, (uint32_t)a);
        ops_size(L, a0, group_end(L, a0), rec, heaps, bytes, cnts, maxc);
      }
      i = end_of(L, i);
    } else if (is_cgroup(op->kind)) { /* [has_value] + U, in its version pass */
      uint32_t has;
      memcpy(&has, rec + op->rec_off, 4);
      *bytes += 1;
      if (has) ops_size(L, i + 1, end_of(L, i), rec, heaps, bytes, cnts, maxc);
      i = end_of(L, i);
    } else if (op->kind == SPK_OP_ARRAY) {
      const uint32_t e = end_of(L, i);
      const uint64_t c = rec_count(rec, op);
      const uint8_t *el = (const uint8_t *)heaps[heap_of(L, i)] + rec_heapoff(rec, op) * op->size;
      *cnts += 1;
      if (c > *maxc) *maxc = c;
      for (uint64_t j = 0; j < c; ++j) ops_size(L, i + 1, e, el + j * op->size, heaps, bytes, cnts, maxc);
      i = e;
    }
  }
}

static void rec_size(const spk_layout *L, const uint8_t *rec, const void *const *heaps,
                     uint64_t *bytes, uint64_t *cnts, uint64_t *maxc) {
  *bytes = *cnts = *maxc = 0;
  if (L->flags & SPK_LAYOUT_TRIVIAL) {
    *bytes = L->rec_stride;
    return;
  }
  ops_size(L, 0, L->n_ops, rec, heaps, bytes, cnts, maxc);
  *bytes += fv_size(L, rec);
}

/* serialize_one (packer.hpp:237-527) of ops [i0, i1) over one (element)
 * record; a container of non-trivially-serializable elements writes its
 * length then each element (packer.hpp:365-367) */
static uint8_t *ops_write(const spk_layout *L, uint32_t i0, uint32_t i1, const uint8_t *rec,
                          const void *const *heaps, unsigned w, uint8_t *p) {
  for (uint32_t i = i0; i < i1; ++i) {
    const spk_op *op = &L->ops[i];
    if (op->kind == SPK_OP_COPY) { /* write_wrapper<sizeof(T)> :264-267 */
      memcpy(p, rec + op->rec_off, op->size);
      p += op->size;
    }
    else if (is_compat(op->kind) || op->kind == SPK_OP_FVAR) {
      /* version UINT64_MAX: nothing (:246-249); fast varints: in the group */
    }
    else if (is_cgroup(op->kind)) {
      i = end_of(L, i); /* written by its version pass */
    }
    else if (op->kind == SPK_OP_OPTGROUP) { /* packer.hpp:382-388,400-410 */
      uint32_t has;
      memcpy(&has, rec + op->rec_off, 4);
      *p++ = has ? 1 : 0;
      const int a = active_group(L, i, rec);
      if (a >= 0) {
        const uint32_t a0 = alt_start(L, i, (uint32_t)a);
        p = ops_write(L, a0, group_end(L, a0), rec, heaps, w, p);
      }
      i = end_of(L, i);
    }
    else if (op->kind == SPK_OP_VARINT) { /* serialize_varint :245-268 */
      uint64_t v = vi_value(rec, op);
      while (v >= 0x80) {
        *p++ = (uint8_t)(v | 0x80u);
        v >>= 7;
      }
      *p++ = (uint8_t)v;
    }
    else if (op->kind == SPK_OP_VARIANT) { /* packer.hpp:389-398 */
      uint32_t idx;
      memcpy(&idx, rec + op->rec_off, 4);
      const uint32_t a0 = alt_start(L, i, idx);
      *p++ = (uint8_t)idx;
      p = ops_write(L, a0, group_end(L, a0), rec, heaps, w, p);
      i = end_of(L, i);
    }
    else if (op->kind == SPK_OP_ARRAY) {
      const uint32_t e = end_of(L, i);
      const uint64_t c = rec_count(rec, op);
      const uint8_t *el = (const uint8_t *)heaps[heap_of(L, i)] + rec_heapoff(rec, op) * op->size;
      put_le(p, c, w);
      p += w;
      for (uint64_t j = 0; j < c; ++j) p = ops_write(L, i + 1, e, el + j * op->size, heaps, w, p);
      i = e;
    }
    else { /* container: low_bytes_write_wrapper<w> + memcpy (:304-363);
              optional: bool has_value + the value (:382-388) */
      uint64_t c = rec_count(rec, op);
      put_le(p, c, op_pw(op, w));
      p += op_pw(op, w);
      uint64_t nb = c * op->size;
      if (nb) {
        const uint8_t *src =
            (const uint8_t *)heaps[heap_of(L, i)] + rec_heapoff(rec, op) * op->size;
        memcpy(p, src, nb);
        p += nb;
      }
    }
  }
  return p;
}

static uint8_t *write_record(const spk_layout *L, const uint8_t *rec,
                             const void *const *heaps, unsigned w, uint8_t *p) {
  if (L->flags & SPK_LAYOUT_TRIVIAL) { /* packer.hpp:418-421 (incl. padding) */
    memcpy(p, rec, L->rec_stride);
    return p + L->rec_stride;
  }
  p = fv_write(L, rec, p); /* before the members (packer.hpp:432-440) */
  return ops_write(L, 0, L->n_ops, rec, heaps, w, p);
}

/* the version pass of rank `rk` over one record (packer.hpp:453-461):
 * [has_value][U] for each compatible member of that version */
static uint8_t *write_compat(const spk_layout *L, unsigned rk, const uint8_t *rec,
                             const void *const *heaps, unsigned w, uint8_t *p) {
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const spk_op *op = &L->ops[i];
    if (is_cgroup(op->kind) && SPK_OP_RANK(op->kind) == rk) {
      uint32_t has;
      memcpy(&has, rec + op->rec_off, 4);
      *p++ = has ? 1 : 0;
      if (has) p = ops_write(L, i + 1, end_of(L, i), rec, heaps, w, p);
      i = end_of(L, i);
      continue;
    }
    if (!is_compat(op->kind) || SPK_OP_RANK(op->kind) != rk) continue;
    const uint64_t c = rec_count(rec, op);
    *p++ = (uint8_t)c;
    if (c) {
      memcpy(p, (const uint8_t *)heaps[heap_of(L, i)] + rec_heapoff(rec, op) * op->size,
             op->size);
      p += op->size;
    }
  }
  return p;
}

int spko_plan(const spk_layout *L, int mode, uint64_t n, const void *recs,
              const void *const *heaps, spk_plan_t *plan) {
  if (!L || !plan || (n && !recs)) return SPK_E_ARG;
  const uint8_t *r = (const uint8_t *)recs;
  memset(plan, 0, sizeof(*plan));
  if (mode == SPK_MODE_VECTOR) {
    /* calculate_one_size container branch: size_cnt += 1, max_size = n */
    uint64_t maxc = n, var = 0, cnts = 0;
    for (uint64_t i = 0; i < n; ++i) {
      uint64_t b, c, m;
      rec_size(L, r + i * L->rec_stride, heaps, &b, &c, &m);
      if (m > maxc) maxc = m;
      var += b;
      cnts += c;
    }
    unsigned w = width_of(maxc);
    hdr_t h = header_shape(&L->fmt_vector, w, compat_ranks(L) > 0, w + var + cnts * w);
    plan->max_count = maxc;
    plan->var_bytes = var;
    plan->width = w;
    plan->header_bytes = h.len + w;
    plan->metainfo = h.meta;
    plan->has_meta = h.has_meta;
    plan->total_bytes = h.total;
  }
  else if (mode == SPK_MODE_MESSAGES) {
    uint64_t tot = 0, maxc = 0, var = 0;
    for (uint64_t i = 0; i < n; ++i) {
      uint64_t b, c, m;
      rec_size(L, r + i * L->rec_stride, heaps, &b, &c, &m);
      unsigned w = width_of(m);
      hdr_t h = header_shape(&L->fmt_one, w, compat_ranks(L) > 0, b + c * w);
      if (m > maxc) maxc = m;
      var += b;
      tot += h.total;
    }
    plan->max_count = maxc;
    plan->var_bytes = var;
    plan->width = width_of(maxc);
    plan->total_bytes = tot;
  }
  else
    return SPK_E_ARG;
  return SPK_OK;
}

int spko_encode(const spk_layout *L, int mode, uint64_t n, const void *recs,
                const void *const *heaps, void *out, uint64_t out_cap,
                uint64_t *msg_offsets, uint64_t *written) {
  spk_plan_t plan;
  int rc = spko_plan(L, mode, n, recs, heaps, &plan);
  if (rc) return rc;
  if (written) *written = plan.total_bytes;
  if (plan.total_bytes > out_cap) return SPK_E_CAPACITY;
  const uint8_t *r = (const uint8_t *)recs;
  uint8_t *p = (uint8_t *)out;
  if (mode == SPK_MODE_VECTOR) {
    unsigned w = plan.width;
    hdr_t h = header_shape(&L->fmt_vector, w, compat_ranks(L) > 0,
                           plan.total_bytes - plan.header_bytes + w);
    p = write_header(p, &L->fmt_vector, &h);
    put_le(p, n, w); /* outer vector length prefix */
    p += w;
    for (uint64_t i = 0; i < n; ++i)
      p = write_record(L, r + i * L->rec_stride, heaps, w, p);
    for (unsigned rk = 0; rk < compat_ranks(L); ++rk) /* packer.hpp:66-78 */
      for (uint64_t i = 0; i < n; ++i)
        p = write_compat(L, rk, r + i * L->rec_stride, heaps, w, p);
  }
  else {
    uint8_t *base = p;
    for (uint64_t i = 0; i < n; ++i) {
      const uint8_t *rec = r + i * L->rec_stride;
      uint64_t b, c, m;
      rec_size(L, rec, heaps, &b, &c, &m);
      unsigned w = width_of(m);
      hdr_t h = header_shape(&L->fmt_one, w, compat_ranks(L) > 0, b + c * w);
      if (msg_offsets) msg_offsets[i] = (uint64_t)(p - base);
      p = write_header(p, &L->fmt_one, &h);
      p = write_record(L, rec, heaps, w, p);
      for (unsigned rk = 0; rk < compat_ranks(L); ++rk) p = write_compat(L, rk, rec, heaps, w, p);
    }
    if (msg_offsets) msg_offsets[n] = (uint64_t)(p - base);
  }
  return SPK_OK;
}

int spko_encode_body(const spk_layout *L, uint64_t n, const void *recs,
                     const void *const *heaps, unsigned width, void *out,
                     uint64_t out_cap, uint64_t *written) {
  if (!L || (n && !recs) || (width != 1 && width != 2 && width != 4 && width != 8) ||
      compat_ranks(L)) /* the version passes trail the whole body */
    return SPK_E_ARG;
  const uint8_t *r = (const uint8_t *)recs;
  uint64_t tot = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t b, c, m;
    rec_size(L, r + i * L->rec_stride, heaps, &b, &c, &m);
    tot += b + c * width;
  }
  if (written) *written = tot;
  if (tot > out_cap) return SPK_E_CAPACITY;
  uint8_t *p = (uint8_t *)out;
  for (uint64_t i = 0; i < n; ++i)
    p = write_record(L, r + i * L->rec_stride, heaps, width, p);
  return SPK_OK;
}

/* ---- decode ------------------------------------------------------------ */
typedef struct rd_t {
  const uint8_t *now, *end;
} rd_t; /* memory_reader (unpacker.hpp:46-76) */

static int rd_take(rd_t *r, uint64_t n, const uint8_t **p) {
  if ((uint64_t)(r->end - r->now) < n) return 0;
  *p = r->now;
  r->now += n;
  return 1;
}

/* deserialize_metainfo (unpacker.hpp:548-619) */
static int32_t parse_header(const spk_msgfmt *f, rd_t *r, unsigned *w,
                            uint64_t *data_len) {
  const uint8_t *p;
  unsigned has_container = (f->flags & SPK_MF_HAS_CONTAINER) != 0;
  *data_len = 0;
  *w = 1;
  if (!(f->flags & SPK_MF_HASH_HEAD)) { /* :551-569 */
    if (has_container) {
      if (!rd_take(r, 1, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
      *w = 1u << ((p[0] >> 3) & 3);
    }
    return SPK_ERRC_OK;
  }
  if (!rd_take(r, 4, &p)) return SPK_ERRC_NO_BUFFER_SPACE; /* :579-581 */
  uint32_t cur = (uint32_t)get_le(p, 4);
  if ((cur >> 1) != (f->code >> 1)) return SPK_ERRC_INVALID_BUFFER; /* :583 */
  if (!(cur & 1)) return SPK_ERRC_OK; /* :586-590 no metainfo: width 1 */
  if (!rd_take(r, 1, &p)) return SPK_ERRC_NO_BUFFER_SPACE; /* :596-600 */
  uint8_t meta = p[0];
  unsigned csz = meta & 3; /* compatible length field, :601-608, :494-512 */
  if (csz) {
    unsigned nb = csz == 1 ? 2 : csz == 2 ? 4 : 8;
    if (!rd_take(r, nb, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
    *data_len = get_le(p, nb);
  }
  if (meta & 4) { /* deserialize_type_literal :523-546 */
    if (!rd_take(r, (uint64_t)f->literal_len + 1, &p))
      return SPK_ERRC_NO_BUFFER_SPACE;
    if (memcmp(p, f->literal, f->literal_len) || p[f->literal_len] != 0)
      return SPK_ERRC_HASH_CONFLICT;
  }
  *w = 1u << ((meta >> 3) & 3);
  return SPK_ERRC_OK;
}

typedef struct dctx_t {
  const spk_layout *L;
  void *const *heaps;
  const uint64_t *heap_caps;
  uint64_t used[SPK_MAX_SPANS];
  int overflow;
} dctx_t;

/* deserialize_one of ops [i0, i1) over one (element) record
 * (unpacker.hpp:780-1349): every payload failure is no_buffer_space
 * (memory_reader::read/check). A container of non-trivially-serializable
 * elements reads its length, then emplaces and decodes element after element,
 * stopping at the first failure (unpacker.hpp:1208-1226). `rec` NULL: parse
 * only (no output slot). */
static int32_t ops_read(dctx_t *c, rd_t *r, unsigned w, uint32_t i0, uint32_t i1,
                        uint8_t *rec) {
  const spk_layout *L = c->L;
  const uint8_t *p;
  for (uint32_t i = i0; i < i1; ++i) {
    const spk_op *op = &L->ops[i];
    if (op->kind == SPK_OP_COPY) {
      if (!rd_take(r, op->size, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
      if (rec) memcpy(rec + op->rec_off, p, op->size);
      continue;
    }
    if (op->kind == SPK_OP_FVAR) continue; /* read with the record's group */
    if (is_compat(op->kind)) { /* main pass: absent until its version pass */
      if (rec) {
        const uint32_t z = 0;
        const uint64_t off = c->used[heap_of(L, i)];
        memcpy(rec + op->rec_off, &z, 4);
        memcpy(rec + op->aux, &off, 8);
      }
      continue;
    }
    if (op->kind == SPK_OP_VARINT) { /* deserialize_varint_impl :270-292 */
      uint64_t v = 0;
      int k = 0;
      for (; k < 10; ++k) {
        if (!rd_take(r, 1, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
        v |= (uint64_t)(p[0] & 0x7fu) << (k * 7);
        if (!(p[0] & 0x80u)) break;
      }
      if (k == 10) return SPK_ERRC_INVALID_BUFFER;
      if (rec) vi_store(rec, op, v);
      continue;
    }
    if (is_cgroup(op->kind)) { /* main pass: absent until its version pass */
      if (rec) {
        const uint32_t z = 0;
        memcpy(rec + op->rec_off, &z, 4);
      }
      i = end_of(L, i);
      continue;
    }
    if (op->kind == SPK_OP_OPTGROUP) { /* unpacker.hpp:1251-1277 */
      if (!rd_take(r, 1, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
      const uint32_t has = p[0] != 0;
      if (rec) memcpy(rec + op->rec_off, &has, 4);
      const int a = has ? 0 : (op->size == 2 ? 1 : -1);
      if (a >= 0) {
        /* deserialize_one(*item) / (item.error()): the errc is dropped, the
           reader stays where the decode stopped */
        const uint32_t a0 = alt_start(L, i, (uint32_t)a);
        (void)ops_read(c, r, w, a0, group_end(L, a0), rec);
      }
      i = end_of(L, i);
      continue;
    }
    if (op->kind == SPK_OP_VARIANT) { /* unpacker.hpp:1278-1292 */
      if (!rd_take(r, 1, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
      const uint32_t idx = p[0];
      if (idx >= op->size) return SPK_ERRC_INVALID_BUFFER;
      if (rec) memcpy(rec + op->rec_off, &idx, 4);
      const uint32_t a0 = alt_start(L, i, idx);
      /* variant_construct_helper::run (unpacker.hpp:476-490) drops the
         alternative's errc: the reader stays wherever its decode stopped and
         the alternative keeps what was decoded */
      (void)ops_read(c, r, w, a0, group_end(L, a0), rec);
      i = end_of(L, i);
      continue;
    }
    const unsigned hk = heap_of(L, i);
    if (op->kind == SPK_OP_ARRAY) {
      const uint32_t e = end_of(L, i);
      if (!rd_take(r, w, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
      const uint64_t cnt = get_le(p, w);
      uint8_t *el = NULL;
      if (rec) {
        const uint64_t off = c->used[hk];
        /* an element takes at least one byte: at most (bytes left + 1)
           elements get decoded (the last one may fail and stay) */
        const uint64_t left = (uint64_t)(r->end - r->now);
        const uint64_t need = cnt < left + 1 ? cnt : left + 1;
        if (need > 0xFFFFFFFFull || need > c->heap_caps[hk] - off) {
          c->overflow = 1;
          rec = NULL;
        } else {
          uint32_t c32 = (uint32_t)cnt;
          memcpy(rec + op->rec_off, &c32, 4);
          memcpy(rec + op->aux, &off, 8);
          c->used[hk] = off + cnt;
          el = (uint8_t *)c->heaps[hk] + off * op->size;
        }
      }
      for (uint64_t j = 0; j < cnt; ++j) {
        int32_t ec = ops_read(c, r, w, i + 1, e, el ? el + j * op->size : NULL);
        if (ec) { /* emplace_back + decode (unpacker.hpp:1208-1226): the failing
                     element stays in the container */
          if (el) {
            uint32_t c32 = (uint32_t)(j + 1);
            memcpy(rec + op->rec_off, &c32, 4);
            c->used[hk] -= cnt - (j + 1);
          }
          return ec;
        }
      }
      i = e;
      continue;
    }
    /* container length :905-979; optional: read_wrapper<sizeof(bool)>, any
       non-zero byte is "has value" (unpacker.hpp:1251-1275) */
    if (!rd_take(r, op_pw(op, w), &p)) return SPK_ERRC_NO_BUFFER_SPACE;
    uint64_t cnt = op->kind == SPK_OP_OPTION ? (uint64_t)(p[0] != 0) : get_le(p, w);
    int unreadable = 0;
    if (cnt && op->kind == SPK_OP_OPTION) {
      /* deserialize_one(*item)'s errc is dropped (unpacker.hpp:1271-1273):
         a value that does not fit leaves the reader in place and the value
         value-initialised */
      if (!rd_take(r, op->size, &p)) unreadable = 1;
    }
    else if (cnt) { /* size==0 returns early (:980-982) */
      if (op->size > 1 && cnt > UINT64_MAX / op->size) /* :1128-1132 */
        return SPK_ERRC_NO_BUFFER_SPACE;
      if (!rd_take(r, cnt * op->size, &p)) /* check(mem_sz) :1147-1149 */
        return SPK_ERRC_NO_BUFFER_SPACE;
    }
    if (rec) {
      uint64_t off = c->used[hk];
      if (cnt > 0xFFFFFFFFull || off + cnt > c->heap_caps[hk]) {
        c->overflow = 1;
      }
      else {
        uint32_t c32 = (uint32_t)cnt;
        memcpy(rec + op->rec_off, &c32, 4);
        memcpy(rec + op->aux, &off, 8);
        if (unreadable)
          memset((uint8_t *)c->heaps[hk] + off * op->size, 0, op->size);
        else if (cnt)
          memcpy((uint8_t *)c->heaps[hk] + off * op->size, p, cnt * op->size);
        c->used[hk] = off + cnt;
      }
    }
  }
  return SPK_ERRC_OK;
}

static int32_t read_record(dctx_t *c, rd_t *r, unsigned w, uint8_t *rec) {
  const spk_layout *L = c->L;
  const uint8_t *p;
  if (L->flags & SPK_LAYOUT_TRIVIAL) {
    if (!rd_take(r, L->rec_stride, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
    if (rec) memcpy(rec, p, L->rec_stride);
    return SPK_ERRC_OK;
  }
  const fv_t f = fv_shape(L);
  if (f.cnt) { /* deserialize_fast_varint (unpacker.hpp:702-747) */
    if (!rd_take(r, f.bits, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
    const uint8_t *bs = p;
    const unsigned code = ((bs[f.cnt / 8] >> (f.cnt % 8)) & 1u) |
                          (((bs[(f.cnt + 1) / 8] >> ((f.cnt + 1) % 8)) & 1u) << 1);
    if (code == 3 && !f.has64) return SPK_ERRC_INVALID_BUFFER;
    const unsigned wb = 1u << code;
    unsigned j = 0;
    for (uint32_t i = 0; i < L->n_ops; ++i) {
      const spk_op *op = &L->ops[i];
      if (op->kind != SPK_OP_FVAR) continue;
      uint64_t v = 0;
      if ((bs[j / 8] >> (j % 8)) & 1u) { /* deserialize_one_fast_varint :642-682 */
        const unsigned rw = wb < op->size ? wb : op->size;
        if (!rd_take(r, rw, &p)) return SPK_ERRC_NO_BUFFER_SPACE;
        v = get_le(p, rw);
        if ((op->aux & SPK_FVAR_SIGNED) && rw < 8 && (v >> (8 * rw - 1)) & 1u)
          v |= ~0ull << (8 * rw); /* int_t<real_width> -> the member */
      }
      if (rec) put_le(rec + op->rec_off, v, op->size);
      ++j;
    }
  }
  return ops_read(c, r, w, 0, L->n_ops, rec);
}

/* the version pass of rank `rk` over one record (unpacker.hpp:1354-1376).
 * Returns 1 when the reader reached data_len before a member: the legal end
 * of an older writer's message (size_type_ = UCHAR_MAX, :360-365). */
static int read_compat(dctx_t *c, rd_t *r, const uint8_t *msg, uint64_t data_len,
                       unsigned rk, unsigned w, uint8_t *rec, int32_t *err) {
  const spk_layout *L = c->L;
  const uint8_t *p;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const spk_op *op = &L->ops[i];
    if (is_cgroup(op->kind) && SPK_OP_RANK(op->kind) == rk) {
      const uint32_t e = end_of(L, i);
      if ((uint64_t)(r->now - msg) >= data_len) return 1;
      if (!rd_take(r, 1, &p)) {
        *err = SPK_ERRC_NO_BUFFER_SPACE;
        return 1;
      }
      if (p[0]) { /* item = U{}; deserialize_one(*item) with its errc dropped */
        if (rec) {
          const uint32_t one = 1;
          memcpy(rec + op->rec_off, &one, 4);
        }
        (void)ops_read(c, r, w, i + 1, e, rec);
      }
      i = e;
      continue;
    }
    if (!is_compat(op->kind) || SPK_OP_RANK(op->kind) != rk) continue;
    if ((uint64_t)(r->now - msg) >= data_len) return 1;
    if (!rd_take(r, 1, &p)) {
      *err = SPK_ERRC_NO_BUFFER_SPACE;
      return 1;
    }
    if (!p[0]) continue;
    /* item = U{}; deserialize_one(*item) with its errc dropped */
    const uint8_t *v = NULL;
    if (!rd_take(r, op->size, &v)) v = NULL;
    if (!rec) continue;
    const unsigned hk = heap_of(L, i);
    const uint64_t off = c->used[hk];
    if (off + 1 > c->heap_caps[hk]) {
      c->overflow = 1;
      continue;
    }
    const uint32_t one = 1;
    memcpy(rec + op->rec_off, &one, 4);
    memcpy(rec + op->aux, &off, 8);
    uint8_t *dst = (uint8_t *)c->heaps[hk] + off * op->size;
    if (v) memcpy(dst, v, op->size);
    else memset(dst, 0, op->size);
    c->used[hk] = off + 1;
  }
  return 0;
}

int spko_decode(const spk_layout *L, int mode, const void *wire,
                uint64_t wire_len, const uint64_t *msg_offsets, uint64_t n_msgs,
                void *recs, uint64_t rec_cap, void *const *heaps,
                const uint64_t *heap_caps, spk_dresult_t *res, int32_t *errc) {
  if (!L || !res || (wire_len && !wire)) return SPK_E_ARG;
  dctx_t c;
  memset(&c, 0, sizeof(c));
  c.L = L;
  c.heaps = heaps;
  c.heap_caps = heap_caps;
  memset(res, 0, sizeof(*res));
  const uint8_t *base = (const uint8_t *)wire;
  uint8_t *out = (uint8_t *)recs;
  if (mode == SPK_MODE_VECTOR) {
    rd_t r = {base, base + wire_len};
    unsigned w;
    uint64_t data_len;
    int32_t e = parse_header(&L->fmt_vector, &r, &w, &data_len);
    res->width = w;
    if (e) {
      res->errc = e;
      return SPK_OK;
    }
    const uint8_t *p;
    if (!rd_take(&r, w, &p)) {
      res->errc = SPK_ERRC_NO_BUFFER_SPACE;
      return SPK_OK;
    }
    uint64_t n = get_le(p, w);
    if (L->flags & SPK_LAYOUT_TRIVIAL) { /* unpacker.hpp:1127-1156 */
      if (n > UINT64_MAX / L->rec_stride ||
          (uint64_t)(r.end - r.now) < n * L->rec_stride) {
        res->errc = SPK_ERRC_NO_BUFFER_SPACE;
        return SPK_OK;
      }
    }
    for (uint64_t i = 0; i < n; ++i) { /* emplace_back loop :1208-1226 */
      uint8_t *rec = (i < rec_cap && out) ? out + i * L->rec_stride : NULL;
      if (i >= rec_cap) c.overflow = 1;
      e = read_record(&c, &r, w, rec);
      if (e) {
        res->errc = e;
        return SPK_OK;
      }
    }
    /* deserialize_compatibles (unpacker.hpp:292-366): version by version,
       record by record */
    int stop = 0;
    for (unsigned rk = 0; rk < compat_ranks(L) && !stop; ++rk)
      for (uint64_t i = 0; i < n && !stop; ++i)
        stop = read_compat(&c, &r, base, data_len, rk, w,
                           (i < rec_cap && out) ? out + i * L->rec_stride : NULL, &e);
    if (e) {
      res->errc = e;
      return SPK_OK;
    }
    /* an absent member's heap offset: the values before its record (as for
       an absent optional, and what the device decoder's per-record bases give) */
    for (uint32_t k = 0; k < L->n_ops && compat_ranks(L); ++k) {
      if (!is_compat(L->ops[k].kind)) continue;
      uint64_t run = 0;
      for (uint64_t i = 0; i < n && i < rec_cap && out; ++i) {
        uint8_t *rec = out + i * L->rec_stride;
        if (rec_count(rec, &L->ops[k])) {
          ++run;
          continue;
        }
        memcpy(rec + L->ops[k].aux, &run, 8);
      }
    }
    res->count = n;
    uint64_t pos = (uint64_t)(r.now - base);
    res->consumed = pos > data_len ? pos : data_len;
    for (unsigned k = 0; k < SPK_MAX_SPANS; ++k) res->heap_used[k] = c.used[k];
    if (c.overflow) res->errc = SPK_ERRC_CAPACITY;
    return SPK_OK;
  }
  if (mode != SPK_MODE_MESSAGES || (n_msgs && !msg_offsets)) return SPK_E_ARG;
  /* Batch contract (ours, not the reference's: it has no batches): message i
   * is wire[offsets[i], offsets[i+1]); a range that is reversed or ends past
   * the wire reads as truncated (no_buffer_space); a well-formed message with
   * no output slot (i >= rec_cap) gets SPK_ERRC_CAPACITY, is not counted and
   * uses no heap. */
  uint64_t ok = 0, consumed = 0;
  for (uint64_t i = 0; i < n_msgs; ++i) {
    uint64_t a = msg_offsets[i], b = msg_offsets[i + 1];
    int32_t e = SPK_ERRC_OK;
    rd_t r = {base, base};
    unsigned w = 1;
    uint64_t data_len = 0;
    if (b < a || b > wire_len) {
      e = SPK_ERRC_NO_BUFFER_SPACE;
    } else {
      r.now = base + a;
      r.end = base + b;
      e = parse_header(&L->fmt_one, &r, &w, &data_len);
    }
    if (!e) {
      uint64_t save[SPK_MAX_SPANS];
      memcpy(save, c.used, sizeof(save));
      uint8_t *rec = (i < rec_cap && out) ? out + i * L->rec_stride : NULL;
      e = read_record(&c, &r, w, rec);
      for (unsigned rk = 0; !e && rk < compat_ranks(L); ++rk)
        if (read_compat(&c, &r, base + a, data_len, rk, w, rec, &e)) break;
      if (!e && i >= rec_cap) {
        e = SPK_ERRC_CAPACITY;
        c.overflow = 1;
      }
      if (e) memcpy(c.used, save, sizeof(save)); /* failed: no heap use */
    }
    if (errc) errc[i] = e;
    if (!e) {
      ++ok;
      uint64_t pos = (uint64_t)(r.now - (base + a));
      consumed += pos > data_len ? pos : data_len;
    }
  }
  res->count = ok;
  res->consumed = consumed;
  for (unsigned k = 0; k < SPK_MAX_SPANS; ++k) res->heap_used[k] = c.used[k];
  res->errc = c.overflow ? SPK_ERRC_CAPACITY : SPK_ERRC_OK;
  return SPK_OK;
}
