// spk_api.hip — the extern "C" boundary of include/spk_codec.h.
//
// Host-side argument validation and dispatch only: trivially-serializable
// layouts go to spk_fixed.hip, layouts with variable-length members to
// spk_var.hip. No allocation, no synchronisation: everything is enqueued on
// the caller's stream. There is no CPU path behind these symbols.
#include "spk_internal.hpp"

#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

using namespace spk;

// ---- kernel tracing state (SPK_LAUNCH, spk_trace_*) -------------------------
namespace spk {
volatile int g_trace_on = 0;
namespace {
struct TraceRec {
  const char *name;
  hipEvent_t e0, e1;
};
struct TraceAcc {
  uint64_t launches = 0;
  double ms = 0;
};
std::mutex g_trace_mu;
std::vector<TraceRec> g_trace_pending;
std::map<std::string, TraceAcc> g_trace_acc;
thread_local long g_trace_open = -1;  // index of this thread's open launch

void trace_settle_locked() {
  for (TraceRec &r : g_trace_pending) {
    if (r.e1) {
      float ms = 0;
      if (hipEventSynchronize(r.e1) == hipSuccess && hipEventElapsedTime(&ms, r.e0, r.e1) == hipSuccess) {
        TraceAcc &a = g_trace_acc[r.name];
        ++a.launches;
        a.ms += ms;
      }
      (void)hipEventDestroy(r.e1);
    }
    (void)hipEventDestroy(r.e0);
  }
  g_trace_pending.clear();
}
}  // namespace

void trace_mark(const char *name, hipStream_t s, int end) {
  std::lock_guard<std::mutex> lk(g_trace_mu);
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return;
  if (hipEventRecord(e, s) != hipSuccess) {
    (void)hipEventDestroy(e);
    return;
  }
  if (!end) {
    g_trace_open = (long)g_trace_pending.size();
    g_trace_pending.push_back(TraceRec{name, e, nullptr});
  } else if (g_trace_open >= 0 && g_trace_open < (long)g_trace_pending.size()) {
    g_trace_pending[g_trace_open].e1 = e;
    g_trace_open = -1;
  } else {
    (void)hipEventDestroy(e);
  }
}
}  // namespace spk

static int hip_rc(hipError_t e) { return e == hipSuccess ? SPK_OK : SPK_E_HIP; }

static bool is_trivial(const spk_layout *L) { return (L->flags & SPK_LAYOUT_TRIVIAL) != 0; }
static bool has_compat(const spk_layout *L) {
  for (uint32_t i = 0; i < L->n_ops; ++i)
    if (SPK_OP_KIND(L->ops[i].kind) == SPK_OP_COMPAT ||
        SPK_OP_KIND(L->ops[i].kind) == SPK_OP_CGROUP)
      return true;
  return false;
}
static uint32_t heap_count(const spk_layout *L) {
  uint32_t k = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) k += op_has_heap(L->ops[i].kind);
  return k;
}

extern "C" {

uint32_t spk_abi_version(void) { return SPK_ABI_VERSION; }

// error_code.hpp:28-43 (make_error_message)
const char *spk_errc_message(int32_t e) {
  switch (e) {
    case SPK_ERRC_OK: return "ok";
    case SPK_ERRC_NO_BUFFER_SPACE: return "no buffer space";
    case SPK_ERRC_INVALID_BUFFER: return "invalid argument";
    case SPK_ERRC_HASH_CONFLICT: return "hash conflict";
    case SPK_ERRC_INVALID_WIDTH: return "invalid width of container length";
    case SPK_ERRC_CAPACITY: return "device output capacity exceeded";
    default: return "(unrecognized error)";
  }
}

int spk_layout_check(const spk_layout *L) {
  if (!L || L->abi != SPK_ABI_VERSION) return SPK_E_LAYOUT;
  if (L->n_ops == 0 || L->n_ops > SPK_MAX_OPS || L->rec_stride == 0) return SPK_E_LAYOUT;
  if (L->fmt_vector.literal_len > SPK_MAX_LITERAL || L->fmt_one.literal_len > SPK_MAX_LITERAL)
    return SPK_E_LAYOUT;
  if (!(L->fmt_vector.flags & SPK_MF_HAS_CONTAINER)) return SPK_E_LAYOUT;  // vector<T>
  if (is_trivial(L)) {
    const spk_op &o = L->ops[0];
    if (L->n_ops != 1 || o.kind != SPK_OP_COPY || o.rec_off != 0 || o.size != L->rec_stride)
      return SPK_E_LAYOUT;
    if (L->fmt_one.flags & SPK_MF_HAS_CONTAINER) return SPK_E_LAYOUT;
    return SPK_OK;
  }
  uint32_t spans = 0, conts = 0, vars = 0, fvars = 0;
  // open ARRAY element layouts / VARIANT alternatives (level 0: the top
  // record): the record stride, ops seen, alternatives still to close
  uint32_t stride[SPK_MAX_DEPTH + 1] = {L->rec_stride}, depth = 0, nops[SPK_MAX_DEPTH + 1] = {0};
  uint32_t alts[SPK_MAX_DEPTH + 1] = {0};
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const spk_op &o = L->ops[i];
    const uint32_t rs = stride[depth];
    ++nops[depth];
    const uint32_t kk = SPK_OP_KIND(o.kind);
    if (kk == SPK_OP_VARIANT || kk == SPK_OP_OPTGROUP || kk == SPK_OP_CGROUP) {
      // u32 index / has_value in this record; the groups follow in it:
      // variant 1..255 alternatives, optional 1 group / expected 2, compatible
      // 1 (top-level record only, with the hash head: type_calculate.hpp:
      // 868-876)
      const uint32_t maxg = kk == SPK_OP_VARIANT ? 255u : kk == SPK_OP_OPTGROUP ? 2u : 1u;
      if (o.size == 0 || o.size > maxg || o.aux || o.rec_off % 4 || o.rec_off + 4 > rs ||
          depth == SPK_MAX_DEPTH || (kk != SPK_OP_CGROUP && (o.kind >> 8)))
        return SPK_E_LAYOUT;
      if (kk == SPK_OP_CGROUP &&
          (depth || (o.kind & ~0xFFFFu) || !(L->fmt_one.flags & SPK_MF_HASH_HEAD) ||
           !(L->fmt_vector.flags & SPK_MF_HASH_HEAD)))
        return SPK_E_LAYOUT;
      ++vars;  // a variable-length member
      stride[++depth] = rs;
      nops[depth] = 0;
      alts[depth] = o.size;
      continue;
    }
    if (o.kind == SPK_OP_END && depth && alts[depth]) {  // closes one alternative
      nops[depth] = 0;
      if (--alts[depth] == 0) --depth;
      continue;
    }
    if (o.kind == SPK_OP_COPY) {
      if (o.size == 0 || (uint64_t)o.rec_off + o.size > rs) return SPK_E_LAYOUT;
    } else if (o.kind == SPK_OP_SPAN || o.kind == SPK_OP_OPTION || o.kind == SPK_OP_ARRAY) {
      if (o.size == 0 || o.rec_off % 4 || o.aux % 8 || o.rec_off + 4 > rs || o.aux + 8 > rs)
        return SPK_E_LAYOUT;
      ++spans;
      conts += o.kind != SPK_OP_OPTION;
      if (o.kind == SPK_OP_ARRAY) {  // element records: 8-byte aligned, one more level
        if (o.size % 8 || depth == SPK_MAX_DEPTH) return SPK_E_LAYOUT;
        stride[++depth] = o.size;
        nops[depth] = 0;
        alts[depth] = 0;
      }
    } else if (SPK_OP_KIND(o.kind) == SPK_OP_COMPAT) {
      // compatible<U, ver> of the top-level record only; OPTION's fields;
      // DISABLE_ALL_META_INFO is a compile error in the reference
      // (type_calculate.hpp:868-876)
      if (depth || (o.kind & ~0xFFFFu) || o.size == 0 || o.rec_off % 4 || o.aux % 8 ||
          o.rec_off + 4 > rs || o.aux + 8 > rs || !(L->fmt_one.flags & SPK_MF_HASH_HEAD) ||
          !(L->fmt_vector.flags & SPK_MF_HASH_HEAD))
        return SPK_E_LAYOUT;
      ++spans;
    } else if (o.kind == SPK_OP_END) {
      --nops[depth];
      if (depth == 0 || nops[depth] == 0) return SPK_E_LAYOUT;  // unmatched / empty element
      --depth;
    } else if (o.kind == SPK_OP_VARINT) {  // var_(u)int32_t / var_(u)int64_t member
      if ((o.size != 4 && o.size != 8) || o.rec_off % o.size || o.rec_off + o.size > rs ||
          (o.aux & ~(SPK_VARINT_ZIGZAG | SPK_VARINT_SEXT)) ||
          ((o.aux & SPK_VARINT_SEXT) && (o.size != 4 || (o.aux & SPK_VARINT_ZIGZAG))))
        return SPK_E_LAYOUT;
      ++vars;
    } else if (o.kind == SPK_OP_FVAR) {  // the top-level record's fast-varint group
      if (depth || (o.size != 4 && o.size != 8) || o.rec_off % o.size ||
          o.rec_off + o.size > rs || (o.aux & ~SPK_FVAR_SIGNED) || ++fvars > SPK_MAX_VARINTS)
        return SPK_E_LAYOUT;
      ++vars;
    } else {
      return SPK_E_LAYOUT;
    }
  }
  if (depth) return SPK_E_LAYOUT;  // an ARRAY / VARIANT without its END(s)
  // a non-trivial record has a variable-length member: a span/option or a varint
  if ((spans == 0 && vars == 0) || spans > SPK_MAX_SPANS || vars > SPK_MAX_VARINTS ||
      L->rec_stride % 8)
    return SPK_E_LAYOUT;
  // check_if_has_container<T>: a container member (an optional alone is none)
  if (!(L->fmt_one.flags & SPK_MF_HAS_CONTAINER) != !conts) return SPK_E_LAYOUT;
  return SPK_OK;
}

size_t spk_workspace_bytes(const spk_layout *L, int mode, uint64_t n, uint64_t wire_len) {
  if (spk_layout_check(L) != SPK_OK) return 0;
  // trivial: per-message payload positions (fallback gather) or 2 words per
  // decode block (<= 4096 blocks), whichever is larger
  if (is_trivial(L)) return kWsScratch + ((n + 1) * 8 > 65536 ? (n + 1) * 8 : 65536) + 256;
  if (layout_nested(L)) return nested_workspace_bytes(L, mode, n, wire_len);
  return var_workspace_bytes(L, mode, n, wire_len);
}

// SPAN / OPTION / ARRAY members read their payloads from d_heaps[k]: a
// non-empty batch needs every one of them (a layout of varints only may pass
// NULL); ARRAY heaps hold element records, read and written as u32/u64 fields
static int heaps_check(const spk_layout *L, uint64_t n, const void *const *d_heaps) {
  uint32_t spans = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    const uint32_t k = L->ops[i].kind;
    if (!op_has_heap(k)) continue;
    if (n && d_heaps && k == SPK_OP_ARRAY && d_heaps[spans] && (uintptr_t)d_heaps[spans] % 8)
      return SPK_E_ARG;
    ++spans;
  }
  if (!spans || !n) return SPK_OK;
  if (!d_heaps) return SPK_E_ARG;
  for (uint32_t k = 0; k < spans; ++k)
    if (!d_heaps[k]) return SPK_E_ARG;
  return SPK_OK;
}

int spk_plan_ex(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                const void *const *d_heaps, spk_plan_t *d_plan, void *d_ws, size_t ws_bytes,
                void *stream) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if ((mode != SPK_MODE_VECTOR && mode != SPK_MODE_MESSAGES) || !d_plan || !d_ws)
    return SPK_E_ARG;
  if (n && !d_recs) return SPK_E_ARG;
  if (ws_bytes < spk_workspace_bytes(L, mode, n, 0)) return SPK_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (is_trivial(L)) return hip_rc(launch_fixed_plan(L, mode, n, d_plan, d_ws, s));
  if ((uintptr_t)d_recs % 8) return SPK_E_ARG;
  if (layout_nested(L)) {  // the sizes live in the element records
    if ((rc = heaps_check(L, n, d_heaps))) return rc;
    return hip_rc(launch_nested_plan(L, mode, n, d_recs, d_heaps, d_plan, d_ws, s));
  }
  return hip_rc(launch_var_plan(L, mode, n, d_recs, d_plan, d_ws, ws_bytes, s));
}

int spk_plan_dn(const spk_layout *L, const uint64_t *d_n, uint64_t n_max, const void *d_recs,
                const void *const *d_heaps, spk_plan_t *d_plan, void *d_ws, size_t ws_bytes,
                void *stream) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (!d_n || !d_plan || !d_ws || (n_max && !d_recs)) return SPK_E_ARG;
  if (layout_nested(L)) return SPK_E_LAYOUT;
  if (ws_bytes < spk_workspace_bytes(L, SPK_MODE_MESSAGES, n_max, 0)) return SPK_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (is_trivial(L))
    return hip_rc(launch_fixed_plan(L, SPK_MODE_MESSAGES, n_max, d_plan, d_ws, s, d_n));
  if ((uintptr_t)d_recs % 8) return SPK_E_ARG;
  (void)d_heaps;
  return hip_rc(launch_var_plan(L, SPK_MODE_MESSAGES, n_max, d_recs, d_plan, d_ws, ws_bytes, s,
                                d_n));
}

int spk_plan(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
             spk_plan_t *d_plan, void *d_ws, size_t ws_bytes, void *stream) {
  if (L && spk_layout_check(L) == SPK_OK && layout_nested(L) && n) return SPK_E_ARG;
  return spk_plan_ex(L, mode, n, d_recs, nullptr, d_plan, d_ws, ws_bytes, stream);
}

static int frame_check(const spk_frame *F) {
  if (!F) return SPK_OK;
  if (F->prefix_len > SPK_MAX_FRAME) return SPK_E_ARG;
  if (F->seq_off != SPK_FRAME_NONE && (uint64_t)F->seq_off + 4 > F->prefix_len) return SPK_E_ARG;
  if (F->len_off != SPK_FRAME_NONE && (uint64_t)F->len_off + 4 > F->prefix_len) return SPK_E_ARG;
  return SPK_OK;
}

static int encode_impl(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                       const void *const *d_heaps, const spk_plan_t *d_plan, void *d_out,
                       uint64_t out_cap, uint64_t *d_msg_offsets, const spk_frame *F,
                       void *d_ws, size_t ws_bytes, void *stream,
                       const SeqEcho *echo = nullptr, const uint64_t *d_n = nullptr) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (d_n && layout_nested(L)) return SPK_E_LAYOUT;
  if ((mode != SPK_MODE_VECTOR && mode != SPK_MODE_MESSAGES) || !d_plan || !d_ws || !d_out)
    return SPK_E_ARG;
  if (n && !d_recs) return SPK_E_ARG;
  if (ws_bytes < spk_workspace_bytes(L, mode, n, 0)) return SPK_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (is_trivial(L)) {
    uint8_t hb[4 + 1 + SPK_MAX_LITERAL + 1];
    if (mode == SPK_MODE_VECTOR) {
      const uint32_t w = width_of(n);
      const uint64_t total = write_hdr(hb, L->fmt_vector, w) + w + n * (uint64_t)L->rec_stride;
      if (total > out_cap) return SPK_E_CAPACITY;
      return hip_rc(launch_fixed_encode_vector(L, n, d_recs, d_out, d_ws, s));
    }
    const uint32_t P = F ? F->prefix_len : 0;
    const uint64_t total = n * (uint64_t)(P + write_hdr(hb, L->fmt_one, 1) + L->rec_stride);
    if (total > out_cap) return SPK_E_CAPACITY;
    return hip_rc(launch_fixed_encode_messages(L, n, d_recs, d_out, d_msg_offsets, F, s, echo,
                                               d_n));
  }
  if ((uintptr_t)d_recs % 8) return SPK_E_ARG;
  if ((rc = heaps_check(L, n, d_heaps))) return rc;
  if (layout_nested(L))
    return hip_rc(launch_nested_encode(L, mode, n, d_recs, d_heaps, d_out, out_cap, d_msg_offsets, F, 0,
                                       d_ws, s, echo));
  return hip_rc(launch_var_encode(L, mode, n, d_recs, d_heaps, d_plan, d_out, out_cap,
                                  d_msg_offsets, F, d_ws, ws_bytes, s, echo, d_n));
}

int spk_encode(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
               const void *const *d_heaps, const spk_plan_t *d_plan, void *d_out,
               uint64_t out_cap, uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes,
               void *stream) {
  return encode_impl(L, mode, n, d_recs, d_heaps, d_plan, d_out, out_cap, d_msg_offsets,
                     nullptr, d_ws, ws_bytes, stream);
}

int spk_plan_encode(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                    const void *const *d_heaps, spk_plan_t *d_plan, void *d_out,
                    uint64_t out_cap, uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes,
                    void *stream) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if ((mode != SPK_MODE_VECTOR && mode != SPK_MODE_MESSAGES) || !d_plan || !d_ws || !d_out)
    return SPK_E_ARG;
  if (n && !d_recs) return SPK_E_ARG;
  if (ws_bytes < spk_workspace_bytes(L, mode, n, 0)) return SPK_E_WORKSPACE;
  if (is_trivial(L) && mode == SPK_MODE_MESSAGES) {
    // the plan is the host's: the encode kernel stores it (one launch)
    uint8_t hb[4 + 1 + SPK_MAX_LITERAL + 1];
    const uint64_t total = n * (uint64_t)(write_hdr(hb, L->fmt_one, 1) + L->rec_stride);
    if (total > out_cap) {
      if ((rc = spk_plan_ex(L, mode, n, d_recs, d_heaps, d_plan, d_ws, ws_bytes, stream)))
        return rc;
      return SPK_E_CAPACITY;
    }
    return hip_rc(launch_fixed_plan_encode_messages(L, n, d_recs, d_out, d_msg_offsets, d_plan,
                                                    d_ws, (hipStream_t)stream));
  }
  if (!is_trivial(L) && var_plan_encode_small_ok(L, n)) {
    // a small batch of a flat variable-size layout: plan and write in one launch
    if ((uintptr_t)d_recs % 8) return SPK_E_ARG;
    if ((rc = heaps_check(L, n, d_heaps))) return rc;
    return hip_rc(launch_var_plan_encode_small(L, mode, n, d_recs, d_heaps, d_plan, d_out,
                                               out_cap, d_msg_offsets, d_ws,
                                               (hipStream_t)stream));
  }
  if ((rc = spk_plan_ex(L, mode, n, d_recs, d_heaps, d_plan, d_ws, ws_bytes, stream))) return rc;
  return spk_encode(L, mode, n, d_recs, d_heaps, d_plan, d_out, out_cap, d_msg_offsets, d_ws,
                    ws_bytes, stream);
}

int spk_encode_framed(const spk_layout *L, uint64_t n, const void *d_recs,
                      const void *const *d_heaps, const spk_plan_t *d_plan,
                      const spk_frame *F, void *d_out, uint64_t out_cap,
                      uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes, void *stream) {
  if (!F) return SPK_E_ARG;
  int rc = frame_check(F);
  if (rc) return rc;
  return encode_impl(L, SPK_MODE_MESSAGES, n, d_recs, d_heaps, d_plan, d_out, out_cap,
                     d_msg_offsets, F, d_ws, ws_bytes, stream);
}

int spk_encode_framed_echo(const spk_layout *L, uint64_t n, const void *d_recs,
                           const void *const *d_heaps, const spk_plan_t *d_plan,
                           const spk_frame *F, const void *d_seq_src,
                           const uint64_t *d_seq_offsets, uint32_t seq_src_off, void *d_out,
                           uint64_t out_cap, uint64_t *d_msg_offsets, void *d_ws,
                           size_t ws_bytes, void *stream) {
  if (!F || F->seq_off == SPK_FRAME_NONE) return SPK_E_ARG;
  if (n && (!d_seq_src || !d_seq_offsets)) return SPK_E_ARG;
  int rc = frame_check(F);
  if (rc) return rc;
  const SeqEcho echo{(const uint8_t *)d_seq_src, d_seq_offsets, seq_src_off, 0};
  return encode_impl(L, SPK_MODE_MESSAGES, n, d_recs, d_heaps, d_plan, d_out, out_cap,
                     d_msg_offsets, F, d_ws, ws_bytes, stream, n ? &echo : nullptr);
}

static int decode_impl(const spk_layout *L, int mode, const void *d_wire, uint64_t wire_len,
                       const uint64_t *d_msg_offsets, uint64_t n_msgs, uint32_t prefix,
                       void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                       const uint64_t *heap_caps, spk_dresult_t *d_res, int32_t *d_errc,
                       void *d_ws, size_t ws_bytes, void *stream,
                       const uint64_t *d_msg_ends = nullptr, const uint64_t *d_n = nullptr) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (d_n && layout_nested(L)) return SPK_E_LAYOUT;
  if ((mode != SPK_MODE_VECTOR && mode != SPK_MODE_MESSAGES) || !d_res || !d_ws)
    return SPK_E_ARG;
  if (wire_len && !d_wire) return SPK_E_ARG;
  if (rec_cap && !d_recs) return SPK_E_ARG;
  const uint64_t nrec = mode == SPK_MODE_VECTOR ? rec_cap : n_msgs;
  if (ws_bytes < spk_workspace_bytes(L, mode, nrec, wire_len)) return SPK_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (is_trivial(L)) {
    if (mode == SPK_MODE_VECTOR)
      return hip_rc(launch_fixed_decode_vector(L, d_wire, wire_len, d_recs, rec_cap, d_res,
                                               d_ws, s));
    return hip_rc(launch_fixed_decode_messages(L, d_wire, wire_len, d_msg_offsets, n_msgs,
                                               prefix, d_recs, rec_cap, d_res, d_errc, d_ws,
                                               s, d_msg_ends, d_n));
  }
  if (d_recs && (uintptr_t)d_recs % 8) return SPK_E_ARG;
  const uint32_t spans = heap_count(L);
  if (spans && (!d_heaps || !heap_caps)) return SPK_E_ARG;
  if (mode == SPK_MODE_MESSAGES && n_msgs && !d_msg_offsets) return SPK_E_ARG;
  if (layout_nested(L)) {
    for (uint32_t k = 0; k < spans; ++k)
      if (!d_heaps[k] || (uintptr_t)d_heaps[k] % 8) return SPK_E_ARG;
    return hip_rc(launch_nested_decode(L, mode, d_wire, wire_len, d_msg_offsets, n_msgs, prefix,
                                       d_recs, rec_cap, d_heaps, heap_caps, d_res, d_errc, d_ws,
                                       s, 0, 0, d_msg_ends));
  }
  return hip_rc(launch_var_decode(L, mode, d_wire, wire_len, d_msg_offsets, n_msgs, prefix,
                                  d_recs, rec_cap, d_heaps, heap_caps, d_res, d_errc, d_ws,
                                  ws_bytes, s, 0, 0, d_msg_ends, d_n));
}

int spk_decode(const spk_layout *L, int mode, const void *d_wire, uint64_t wire_len,
               const uint64_t *d_msg_offsets, uint64_t n_msgs, void *d_recs,
               uint64_t rec_cap, void *const *d_heaps, const uint64_t *heap_caps,
               spk_dresult_t *d_res, int32_t *d_errc, void *d_ws, size_t ws_bytes,
               void *stream) {
  return decode_impl(L, mode, d_wire, wire_len, d_msg_offsets, n_msgs, 0, d_recs, rec_cap,
                     d_heaps, heap_caps, d_res, d_errc, d_ws, ws_bytes, stream);
}

int spk_decode_framed(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                      const uint64_t *d_msg_offsets, uint64_t n_msgs, uint32_t prefix_len,
                      void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                      const uint64_t *heap_caps, spk_dresult_t *d_res, int32_t *d_errc,
                      void *d_ws, size_t ws_bytes, void *stream) {
  if (prefix_len > SPK_MAX_FRAME || (n_msgs && !d_msg_offsets)) return SPK_E_ARG;
  return decode_impl(L, SPK_MODE_MESSAGES, d_wire, wire_len, d_msg_offsets, n_msgs,
                     prefix_len, d_recs, rec_cap, d_heaps, heap_caps, d_res, d_errc, d_ws,
                     ws_bytes, stream);
}

int spk_decode_frames(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                      const uint64_t *d_begins, const uint64_t *d_ends, uint64_t n_msgs,
                      uint32_t prefix_len, void *d_recs, uint64_t rec_cap,
                      void *const *d_heaps, const uint64_t *heap_caps, spk_dresult_t *d_res,
                      int32_t *d_errc, void *d_ws, size_t ws_bytes, void *stream) {
  if (prefix_len > SPK_MAX_FRAME || (n_msgs && (!d_begins || !d_ends))) return SPK_E_ARG;
  return decode_impl(L, SPK_MODE_MESSAGES, d_wire, wire_len, d_begins, n_msgs, prefix_len,
                     d_recs, rec_cap, d_heaps, heap_caps, d_res, d_errc, d_ws, ws_bytes, stream,
                     d_ends);
}

int spk_decode_frames_dn(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                         const uint64_t *d_begins, const uint64_t *d_ends, const uint64_t *d_n,
                         uint64_t n_max, uint32_t prefix_len, void *d_recs, uint64_t rec_cap,
                         void *const *d_heaps, const uint64_t *heap_caps, spk_dresult_t *d_res,
                         int32_t *d_errc, void *d_ws, size_t ws_bytes, void *stream) {
  if (!d_n || prefix_len > SPK_MAX_FRAME || (n_max && (!d_begins || !d_ends))) return SPK_E_ARG;
  return decode_impl(L, SPK_MODE_MESSAGES, d_wire, wire_len, d_begins, n_max, prefix_len,
                     d_recs, rec_cap, d_heaps, heap_caps, d_res, d_errc, d_ws, ws_bytes, stream,
                     d_ends, d_n);
}

int spk_encode_framed_echo_dn(const spk_layout *L, const uint64_t *d_n, uint64_t n_max,
                              const void *d_recs, const void *const *d_heaps,
                              const spk_plan_t *d_plan, const spk_frame *F,
                              const void *d_seq_src, const uint64_t *d_seq_offsets,
                              uint32_t seq_src_off, void *d_out, uint64_t out_cap,
                              uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes,
                              void *stream) {
  if (!d_n || !F || F->seq_off == SPK_FRAME_NONE) return SPK_E_ARG;
  if (n_max && (!d_seq_src || !d_seq_offsets)) return SPK_E_ARG;
  int rc = frame_check(F);
  if (rc) return rc;
  const SeqEcho echo{(const uint8_t *)d_seq_src, d_seq_offsets, seq_src_off, 0};
  return encode_impl(L, SPK_MODE_MESSAGES, n_max, d_recs, d_heaps, d_plan, d_out, out_cap,
                     d_msg_offsets, F, d_ws, ws_bytes, stream, n_max ? &echo : nullptr, d_n);
}

int spk_encode_body(const spk_layout *L, uint64_t n, const void *d_recs,
                    const void *const *d_heaps, uint32_t width, void *d_out,
                    uint64_t out_cap, void *d_ws, size_t ws_bytes, void *stream) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (has_compat(L)) return SPK_E_LAYOUT;  // the version passes trail the whole message
  if (width != 1 && width != 2 && width != 4 && width != 8) return SPK_E_ARG;
  if ((n && !d_recs) || !d_out || !d_ws) return SPK_E_ARG;
  if (ws_bytes < spk_workspace_bytes(L, SPK_MODE_VECTOR, n, 0)) return SPK_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (is_trivial(L)) {  // body == the records verbatim (packer.hpp:418-421)
    const uint64_t nb = n * (uint64_t)L->rec_stride;
    if (nb > out_cap) return SPK_E_CAPACITY;
    return hip_rc(hipMemcpyAsync(d_out, d_recs, nb, hipMemcpyDeviceToDevice, s));
  }
  if ((uintptr_t)d_recs % 8) return SPK_E_ARG;
  if ((rc = heaps_check(L, n, d_heaps))) return rc;
  if (layout_nested(L))
    return hip_rc(launch_nested_encode(L, SPK_MODE_VECTOR, n, d_recs, d_heaps, d_out, out_cap, nullptr,
                                       nullptr, width, d_ws, s));
  return hip_rc(launch_var_encode_body(L, n, d_recs, d_heaps, width, d_out, out_cap, d_ws,
                                       ws_bytes, s));
}

int spk_decode_body(const spk_layout *L, const void *d_body, uint64_t body_len, uint32_t width,
                    uint64_t n, void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                    const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                    size_t ws_bytes, void *stream) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (has_compat(L)) return SPK_E_LAYOUT;
  if (width != 1 && width != 2 && width != 4 && width != 8) return SPK_E_ARG;
  if (!d_res || !d_ws || (body_len && !d_body) || (rec_cap && !d_recs)) return SPK_E_ARG;
  if (ws_bytes < spk_workspace_bytes(L, SPK_MODE_VECTOR, rec_cap, body_len))
    return SPK_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (is_trivial(L))
    return hip_rc(launch_fixed_decode_vector(L, d_body, body_len, d_recs, rec_cap, d_res, d_ws,
                                             s, width, n));
  if (d_recs && (uintptr_t)d_recs % 8) return SPK_E_ARG;
  const uint32_t spans = heap_count(L);
  if (spans && (!d_heaps || !heap_caps)) return SPK_E_ARG;
  if (layout_nested(L)) {
    for (uint32_t k = 0; k < spans; ++k)
      if (!d_heaps[k] || (uintptr_t)d_heaps[k] % 8) return SPK_E_ARG;
    return hip_rc(launch_nested_decode(L, SPK_MODE_VECTOR, d_body, body_len, nullptr, 0, 0,
                                       d_recs, rec_cap, d_heaps, heap_caps, d_res, nullptr, d_ws,
                                       s, width, n));
  }
  return hip_rc(launch_var_decode(L, SPK_MODE_VECTOR, d_body, body_len, nullptr, 0, 0, d_recs,
                                  rec_cap, d_heaps, heap_caps, d_res, nullptr, d_ws, ws_bytes, s,
                                  width, n));
}

static int shard_check(const spk_layout *L, const void *d_wire, uint64_t wire_len, void *d_ws,
                       size_t ws_bytes, uint64_t rec_cap) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (is_trivial(L)) return SPK_E_LAYOUT;
  // nested layouts: on the tile decoder (no compatible members, at most
  // SPK_FLAT_SPANS heaps, wires below 4 GiB)
  if (layout_nested(L) && (!var_nested_tile_ok(L) || wire_len >= (1ull << 32) - 4096))
    return SPK_E_LAYOUT;
  if (!d_ws || (wire_len && !d_wire)) return SPK_E_ARG;
  if (ws_bytes < spk_workspace_bytes(L, SPK_MODE_VECTOR, rec_cap, wire_len)) return SPK_E_WORKSPACE;
  return SPK_OK;
}

int spk_decode_shard_index(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                           uint64_t tile_lo, uint64_t tile_hi, uint64_t entry,
                           spk_shard_t *d_summary, void *d_ws, size_t ws_bytes, void *stream) {
  int rc = shard_check(L, d_wire, wire_len, d_ws, ws_bytes, 0);
  if (rc) return rc;
  if (!d_summary || tile_hi < tile_lo) return SPK_E_ARG;
  spk_dresult_t *scratch = (spk_dresult_t *)((uint8_t *)d_ws + kWsCtl - sizeof(spk_dresult_t));
  return hip_rc(launch_var_shard(L, 0, d_wire, wire_len, tile_lo, tile_hi, entry, d_summary, 0, 0,
                                 nullptr, 0, nullptr, nullptr, scratch, d_ws,
                                 (hipStream_t)stream));
}

int spk_decode_shard_emit(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                          uint64_t tile_lo, uint64_t tile_hi, uint64_t first, int last,
                          void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                          const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                          size_t ws_bytes, void *stream) {
  // the tile decoder's workspace does not depend on rec_cap
  int rc = shard_check(L, d_wire, wire_len, d_ws, ws_bytes, 0);
  if (rc) return rc;
  if (!d_res || tile_hi < tile_lo || (rec_cap && !d_recs) || (d_recs && (uintptr_t)d_recs % 8))
    return SPK_E_ARG;
  if ((rc = heaps_check(L, rec_cap, d_heaps))) return rc;
  if (!heap_caps) return SPK_E_ARG;
  return hip_rc(launch_var_shard(L, 1, d_wire, wire_len, tile_lo, tile_hi, 0, nullptr, first,
                                 last ? 1u : 0u, d_recs, rec_cap, d_heaps, heap_caps, d_res, d_ws,
                                 (hipStream_t)stream));
}

int32_t spk_parse_vector_header(const spk_layout *L, const void *h_wire, uint64_t len,
                                uint64_t *n, uint32_t *width, uint32_t *header_len) {
  if (spk_layout_check(L) != SPK_OK) return SPK_E_LAYOUT;
  if ((len && !h_wire) || !n || !width || !header_len) return SPK_E_ARG;
  const uint8_t *p = (const uint8_t *)h_wire;
  uint64_t pos, dl;
  uint32_t w;
  int32_t e = parse_hdr(L->fmt_vector, p, len, &pos, &w, &dl);
  if (e) return e;
  if (len < pos + w) return SPK_ERRC_NO_BUFFER_SPACE;
  *n = ld_le(p + pos, w);
  *width = w;
  *header_len = (uint32_t)(pos + w);
  return SPK_ERRC_OK;
}

int spk_vector_header(const spk_layout *L, uint64_t total_n, uint32_t width, uint8_t *h_out,
                      uint32_t cap) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (has_compat(L)) return SPK_E_LAYOUT;
  if ((width != 1 && width != 2 && width != 4 && width != 8) || !h_out) return SPK_E_ARG;
  if (width < width_of(total_n)) return SPK_E_ARG;  // the count itself must fit
  uint8_t hb[4 + 1 + SPK_MAX_LITERAL + 1 + 8];
  uint32_t len = write_hdr(hb, L->fmt_vector, width);
  for (uint32_t i = 0; i < width; ++i) hb[len + i] = (uint8_t)(total_n >> (8 * i));
  len += width;
  if (len > cap) return SPK_E_CAPACITY;
  for (uint32_t i = 0; i < len; ++i) h_out[i] = hb[i];
  return (int)len;
}

int spk_message_header(const spk_layout *L, uint32_t width, uint8_t *h_out, uint32_t cap) {
  int rc = spk_layout_check(L);
  if (rc) return rc;
  if (has_compat(L)) return SPK_E_LAYOUT;
  if ((width != 1 && width != 2 && width != 4 && width != 8) || !h_out) return SPK_E_ARG;
  uint8_t hb[4 + 1 + SPK_MAX_LITERAL + 1];
  const uint32_t len = write_hdr(hb, L->fmt_one, width);
  if (len > cap) return SPK_E_CAPACITY;
  for (uint32_t i = 0; i < len; ++i) h_out[i] = hb[i];
  return (int)len;
}

int32_t spk_parse_message_header(const spk_layout *L, const void *h_wire, uint64_t len,
                                 uint32_t *width, uint32_t *header_len) {
  if (spk_layout_check(L) != SPK_OK) return SPK_E_LAYOUT;
  if ((len && !h_wire) || !width || !header_len) return SPK_E_ARG;
  uint64_t pos, dl;
  uint32_t w;
  const int32_t e = parse_hdr(L->fmt_one, (const uint8_t *)h_wire, len, &pos, &w, &dl);
  if (e) return e;
  *width = w;
  *header_len = (uint32_t)pos;
  return SPK_ERRC_OK;
}

// ---- kernel tracing ---------------------------------------------------------
int spk_trace_enable(int on) {
  std::lock_guard<std::mutex> lk(g_trace_mu);
  g_trace_on = on ? 1 : 0;
  return SPK_OK;
}
int spk_trace_reset(void) {
  std::lock_guard<std::mutex> lk(g_trace_mu);
  trace_settle_locked();
  g_trace_acc.clear();
  return SPK_OK;
}
// {"kernel": [launches, total_ms], ...} into buf (NUL-terminated when it
// fits); returns the full length, or a negative SPK_E_*
int spk_trace_read(char *buf, size_t cap) {
  std::lock_guard<std::mutex> lk(g_trace_mu);
  trace_settle_locked();
  std::string js = "{";
  for (const auto &kv : g_trace_acc) {
    char tmp[96];
    std::snprintf(tmp, sizeof tmp, "[%llu, %.6f]", (unsigned long long)kv.second.launches,
                  kv.second.ms);
    if (js.size() > 1) js += ", ";
    js += "\"" + kv.first + "\": " + tmp;
  }
  js += "}";
  if (buf && cap) {
    const size_t n = js.size() < cap - 1 ? js.size() : cap - 1;
    for (size_t i = 0; i < n; ++i) buf[i] = js[i];
    buf[n] = 0;
  }
  return (int)js.size();
}

// ---- runtime helpers: front ends in any language stage batches through
// these, so none of them needs the HIP headers --------------------------------
int spk_device_alloc(void **d_ptr, size_t bytes) {
  if (!d_ptr) return SPK_E_ARG;
  *d_ptr = nullptr;
  return hip_rc(hipMalloc(d_ptr, bytes ? bytes : 1));
}
int spk_device_free(void *d_ptr) { return d_ptr ? hip_rc(hipFree(d_ptr)) : SPK_OK; }
int spk_host_alloc_pinned(void **h_ptr, size_t bytes) {
  if (!h_ptr) return SPK_E_ARG;
  *h_ptr = nullptr;
  return hip_rc(hipHostMalloc(h_ptr, bytes ? bytes : 1, hipHostMallocDefault));
}
int spk_host_free_pinned(void *h_ptr) { return h_ptr ? hip_rc(hipHostFree(h_ptr)) : SPK_OK; }
int spk_copy_async(void *dst, const void *src, size_t bytes, int kind, void *stream) {
  if (!bytes) return SPK_OK;
  if (!dst || !src) return SPK_E_ARG;
  hipMemcpyKind k;
  switch (kind) {
    case SPK_COPY_H2D: k = hipMemcpyHostToDevice; break;
    case SPK_COPY_D2H: k = hipMemcpyDeviceToHost; break;
    case SPK_COPY_D2D: k = hipMemcpyDeviceToDevice; break;
    default: return SPK_E_ARG;
  }
  return hip_rc(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream));
}
int spk_stream_create(void **stream) {
  if (!stream) return SPK_E_ARG;
  hipStream_t s = nullptr;
  const int rc = hip_rc(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return rc;
}
int spk_stream_destroy(void *stream) {
  return stream ? hip_rc(hipStreamDestroy((hipStream_t)stream)) : SPK_OK;
}
int spk_stream_sync(void *stream) { return hip_rc(hipStreamSynchronize((hipStream_t)stream)); }

}  // extern "C"
