// spk_internal.hpp — shared device/host definitions of the gfx950 struct_pack
// batch codec (not part of the public ABI; see include/spk_codec.h).
//
// Wire-format rules restated here follow the reference (paths relative to
// /root/reference/include/ylt/struct_pack/):
//   width selection     calculate_size.hpp:426-447
//   header / metainfo   packer.hpp:90-139, type_calculate.hpp:884-891
//   header validation   unpacker.hpp:548-619
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/spk_codec.h"

namespace spk {

constexpr int kWave = 64;

// Heaps the flat-record kernels (spk_var.hip) carry per record; layouts with
// more run the op-list interpreter (spk_nested.hip).
#define SPK_FLAT_SPANS 8u
// diagnostics build (-DSPK_DIAG=1): SPK_TILE_DBG switches the tile kernels'
// diagnostic bits at run time; a release build never reads the environment
#ifndef SPK_DIAG
#define SPK_DIAG 0
#endif

// Kernel-argument copy of the descriptor, without the literal tables (the
// type literal lives in the device header buffer produced by the plan).
struct KLayout {
  uint32_t stride;
  uint32_t n_ops;
  uint32_t trivial;
  uint32_t n_spans;      // SPAN + OPTION members (one heap each)
  uint32_t fixed_bytes;  // sum of COPY sizes + one has_value byte per OPTION
  uint32_t n_cont;       // SPAN members: the ones with a width-w count
  uint32_t n_var;        // VARINT members (LEB128, 1-10 wire bytes each)
  uint32_t pad_;
  spk_op ops[SPK_MAX_OPS];
};

// Everything the write pass needs about one message format, resolved for a
// given width. Computed on the host when the width is known there (trivial
// records) and on the device otherwise (plan kernel).
struct MsgHdr {
  uint32_t len;   // header bytes (head + meta + literal + NUL)
  uint32_t code;  // type code (LSB clear)
  uint32_t flags; // SPK_MF_*
  uint32_t lit_len;
};

__host__ __device__ inline uint32_t width_of(uint64_t max_count) {
  return max_count < (1ull << 8)    ? 1u
         : max_count < (1ull << 16) ? 2u
         : max_count < (1ull << 32) ? 4u
                                    : 8u;
}
__host__ __device__ inline uint32_t width_bits(uint32_t w) {
  return w == 1 ? 0u : w == 2 ? 0x08u : w == 4 ? 0x10u : 0x18u;
}

// Header shape for message format (flags, literal_len) at width w.
struct HdrShape {
  uint32_t head, lit, has_meta, len, meta;
};
__host__ __device__ inline HdrShape hdr_shape(uint32_t flags, uint32_t lit_len,
                                              uint32_t w) {
  HdrShape h;
  const uint32_t has_container = (flags & SPK_MF_HAS_CONTAINER) != 0;
  h.head = (flags & SPK_MF_HASH_HEAD) != 0;
  h.lit = h.head && (flags & SPK_MF_TYPE_LITERAL);
  const uint32_t meta_fixed = h.lit || (!h.head && has_container);
  if (!has_container) w = 1;
  h.has_meta = meta_fixed || w > 1;
  h.meta = width_bits(w) | (h.lit ? 0x04u : 0u);
  h.len = (h.head ? 4u : 0u) + (h.has_meta ? 1u : 0u) + (h.lit ? lit_len + 1u : 0u);
  return h;
}

// compatible<T> members (SPK_OP_COMPAT): the metainfo byte is always there
// and is followed by the message's total length in 2/4/8 bytes
// (calculate_size.hpp:457-470; packer.hpp:111-130). `body` = the bytes after
// the header. Returns the header length; writes it into dst when set.
// (put(p, byte): header byte p; compat_hdr / write_hdr below write to memory)
template <typename Put>
__host__ __device__ inline uint32_t compat_hdr_with(Put &&put, const spk_msgfmt &f, uint32_t w,
                                                    uint64_t body, bool emit) {
  const HdrShape h = hdr_shape(f.flags, f.literal_len, w);
  const uint32_t base = h.len + (h.has_meta ? 0u : 1u);
  const uint64_t l = base + body;
  const uint32_t lw = l + 2 < (1ull << 16) ? 2u : l + 4 < (1ull << 32) ? 4u : 8u;
  if (emit) {
    uint32_t p = 0;
    const uint32_t head = f.code | 1u;
    for (uint32_t b = 0; b < 4; ++b) put(p++, (uint8_t)(head >> (8 * b)));
    put(p++, (uint8_t)(h.meta | (lw == 2 ? 1u : lw == 4 ? 2u : 3u)));
    const uint64_t total = l + lw;
    for (uint32_t b = 0; b < lw; ++b) put(p++, (uint8_t)(total >> (8 * b)));
    if (h.lit) {
      for (uint32_t i = 0; i < f.literal_len; ++i) put(p++, f.literal[i]);
      put(p++, (uint8_t)0);
    }
  }
  return base + lw;
}
__host__ __device__ inline uint32_t compat_hdr(uint8_t *dst, const spk_msgfmt &f, uint32_t w,
                                               uint64_t body) {
  return compat_hdr_with([dst](uint32_t p, uint8_t b) { dst[p] = b; }, f, w, body, dst != nullptr);
}

__host__ __device__ inline bool op_has_heap(uint32_t kind) {
  kind = SPK_OP_KIND(kind);
  return kind == SPK_OP_SPAN || kind == SPK_OP_OPTION || kind == SPK_OP_ARRAY ||
         kind == SPK_OP_COMPAT;
}

// The header bytes (at most 4+1+SPK_MAX_LITERAL+1) through put(p, byte).
template <typename Put>
__host__ __device__ inline uint32_t write_hdr_with(Put &&put, const spk_msgfmt &f, uint32_t w) {
  HdrShape h = hdr_shape(f.flags, f.literal_len, w);
  uint32_t p = 0;
  if (h.head) {
    uint32_t head = (f.code & ~1u) | (h.has_meta ? 1u : 0u);
    put(p++, (uint8_t)head);
    put(p++, (uint8_t)(head >> 8));
    put(p++, (uint8_t)(head >> 16));
    put(p++, (uint8_t)(head >> 24));
  }
  if (h.has_meta) put(p++, (uint8_t)h.meta);
  if (h.lit) {
    for (uint32_t i = 0; i < f.literal_len; ++i) put(p++, f.literal[i]);
    put(p++, (uint8_t)0);
  }
  return p;
}
// Writes the header bytes into dst.
__host__ __device__ inline uint32_t write_hdr(uint8_t *dst, const spk_msgfmt &f, uint32_t w) {
  return write_hdr_with([dst](uint32_t p, uint8_t b) { dst[p] = b; }, f, w);
}

// Workspace layout (device): fixed region first, then per-launch scratch.
//   [0, 512)        : header bytes of the VECTOR message (+ count prefix)
//   [512, 1536)     : header bytes of the MESSAGES format, one 256-B slot
//                     per width 1/2/4/8 (slot = log2(w))
//   [2048, 2304)    : control words (CopyJob / decode state)
//   [4096, ...)     : per-block partials, scan buffers, boundary tables
constexpr size_t kWsHdrVec = 0;
constexpr size_t kWsHdrMsg = 512;
constexpr size_t kWsHdrSlot = 256;
constexpr size_t kWsCtl = 2048;
constexpr size_t kWsScratch = 4096;

// control words (uint64) at kWsCtl
struct Ctl {
  unsigned long long max_count;   // atomicMax target
  unsigned long long err_pos;     // first failing position (decode)
  unsigned long long flags;       // misc
  unsigned long long n_records;   // decode: records found
  int32_t errc;                   // decode errc (atomicMin of nonzero)
  uint32_t pad;
};

// c elements of `size` bytes: their byte count without a 64-bit division
// (a runtime divisor is a long software sequence on the GPU); false when the
// product overflows
__host__ __device__ __forceinline__ bool span_nb(uint64_t c, uint64_t size, uint64_t *nb) {
  return !__builtin_mul_overflow(c, size, nb);
}

// A decode error inside a variant / optional group is dropped by the
// reference (unpacker.hpp:476-490,1251-1277) with the value value-initialised
// before its decode: the members from the failing one to the end of each
// level being unwound read as zero / empty / absent. Writes those fields of
// ops [i, iend) of record r (any output content before the decode): COPY /
// varint bytes zero, a container / option count 0 at element
// offset 0 (the oracle's untouched zero), an optional / compatible group
// absent, a variant alternative 0 with its fields zeroed (the walk goes
// through every alternative, no stack).
template <typename Lay>
__device__ __forceinline__ void zero_rest(const Lay &N, uint8_t *r, uint32_t i, uint32_t iend) {
  while (i < iend) {
    const spk_op op = N.ops[i];
    const uint32_t k = op.kind & 0xFFu;
    if (k == SPK_OP_COPY || k == SPK_OP_VARINT || k == SPK_OP_FVAR) {
      for (uint32_t b = 0; b < op.size; ++b) r[op.rec_off + b] = 0;
      ++i;
    } else if (k == SPK_OP_SPAN || k == SPK_OP_OPTION || k == SPK_OP_COMPAT ||
               k == SPK_OP_ARRAY) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = 0;
      *reinterpret_cast<uint64_t *>(r + op.aux) = 0;
      i = k == SPK_OP_ARRAY ? N.end[i] + 1u : i + 1;
    } else if (k == SPK_OP_OPTGROUP || k == SPK_OP_CGROUP) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = 0;
      i = N.end[i] + 1u;
    } else if (k == SPK_OP_VARIANT) {
      *reinterpret_cast<uint32_t *>(r + op.rec_off) = 0;
      ++i;  // into the alternatives (all of them zeroed; 0 is the one read)
    } else {
      ++i;  // END
    }
  }
}

__host__ __device__ __forceinline__ uint64_t ld_le(const uint8_t *p, uint32_t w) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < w; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// Parse a message header at p[0..len). Returns errc; sets *pos to the first
// payload byte, *w to the width, *data_len to the compatible length field.
__host__ __device__ inline int32_t parse_hdr(const spk_msgfmt &f, const uint8_t *p, uint64_t len,
                             uint64_t *pos, uint32_t *w, uint64_t *data_len) {
  *w = 1;
  *data_len = 0;
  *pos = 0;
  const bool has_container = (f.flags & SPK_MF_HAS_CONTAINER) != 0;
  if (!(f.flags & SPK_MF_HASH_HEAD)) {
    if (has_container) {
      if (len < 1) return SPK_ERRC_NO_BUFFER_SPACE;
      *w = 1u << ((p[0] >> 3) & 3);
      *pos = 1;
    }
    return SPK_ERRC_OK;
  }
  if (len < 4) return SPK_ERRC_NO_BUFFER_SPACE;
  const uint32_t cur = (uint32_t)ld_le(p, 4);
  if ((cur >> 1) != (f.code >> 1)) return SPK_ERRC_INVALID_BUFFER;
  uint64_t at = 4;
  if (!(cur & 1)) {
    *pos = at;
    return SPK_ERRC_OK;
  }
  if (len < at + 1) return SPK_ERRC_NO_BUFFER_SPACE;
  const uint8_t meta = p[at++];
  const uint32_t csz = meta & 3;
  if (csz) {
    const uint32_t nb = csz == 1 ? 2 : csz == 2 ? 4 : 8;
    if (len < at + nb) return SPK_ERRC_NO_BUFFER_SPACE;
    *data_len = ld_le(p + at, nb);
    at += nb;
  }
  if (meta & 4) {
    if (len < at + f.literal_len + 1) return SPK_ERRC_NO_BUFFER_SPACE;
    for (uint32_t i = 0; i < f.literal_len; ++i)
      if (p[at + i] != f.literal[i]) return SPK_ERRC_HASH_CONFLICT;
    if (p[at + f.literal_len] != 0) return SPK_ERRC_HASH_CONFLICT;
    at += f.literal_len + 1;
  }
  *w = 1u << ((meta >> 3) & 3);
  *pos = at;
  return SPK_ERRC_OK;
}

}  // namespace spk

// ---- kernel tracing (spk_trace_*, SURVEY.md §5 "tracing / profiling") -----
// Every kernel launch of the codec goes through SPK_LAUNCH. With tracing
// switched on (spk_trace_enable) it is bracketed by two hipEvents recorded on
// the launch stream; spk_trace_read sums their elapsed times per kernel. Off
// (the default) it costs one load and branch per launch.
namespace spk {
extern volatile int g_trace_on;
void trace_mark(const char *name, hipStream_t s, int end);
}  // namespace spk
#define SPK_LAUNCH(kern, grid, block, shm, stream, ...)                 \
  do {                                                                  \
    const bool spk_tr_ = ::spk::g_trace_on != 0;                        \
    if (spk_tr_) ::spk::trace_mark(#kern, (stream), 0);                 \
    hipLaunchKernelGGL(kern, grid, block, shm, stream, __VA_ARGS__);    \
    if (spk_tr_) ::spk::trace_mark(#kern, (stream), 1);                 \
  } while (0)

// ---- frame sequence numbers ------------------------------------------------
namespace spk {
// A framed encode writes message i's seq_num as seq_base + i, or, echoing
// requests (spk_encode_framed_echo), as the u32 LE at src[offs[i] + off].
struct SeqEcho {
  const uint8_t *src;
  const uint64_t *offs;
  uint32_t off;
  uint32_t pad_;
};
__device__ __forceinline__ uint32_t seq_value(const SeqEcho &e, uint32_t base, uint64_t i) {
  if (!e.src) return base + (uint32_t)i;
  const uint8_t *p = e.src + e.offs[i] + e.off;
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
}  // namespace spk

// ---- launch wrappers implemented in the kernel TUs -----------------------
namespace spk {
// spk_var.hip: sharded VECTOR decode (phase 0 = index, 1 = emit)
hipError_t launch_var_shard(const spk_layout *L, int phase, const void *d_wire, uint64_t wire_len,
                            uint64_t tile_lo, uint64_t tile_hi, uint64_t entry,
                            spk_shard_t *d_summary, uint64_t first, uint32_t last, void *d_recs,
                            uint64_t rec_cap, void *const *d_heaps, const uint64_t *heap_caps,
                            spk_dresult_t *d_res, void *d_ws, hipStream_t s);
// spk_var.hip: VECTOR decode of a nested layout (no compatible members, at
// most SPK_FLAT_SPANS heaps) on the tile decoder
bool var_nested_tile_ok(const spk_layout *L);
size_t var_nested_tile_ws_bytes(const spk_layout *L, uint64_t wire_len);
hipError_t launch_var_nested_decode(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                                    void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                                    const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                                    hipStream_t s, uint32_t body_w, uint64_t body_n);
// spk_var.hip: VECTOR decode of a layout with compatible members on the tile
// decoder: the main pass (the layout without them), then one pass per version
// rank (its members as OPTIONs / OPTGROUPs) from where the previous pass
// ended. Control words at ws + ctl_off (past every pass's workspace); when a
// pass is not clean (an error, or the data length ending it part-way),
// CompatCtl::serial is set and spk_nested.hip's one-lane walk, launched
// behind it on that flag, decodes the message instead.
struct CompatCtl {
  unsigned long long chain[4];  // the next pass: start, records, width, data length
  unsigned long long end;       // where the last pass that ran ended
  uint32_t serial;              // 1: the one-lane walk decodes the message
  uint32_t stop;                // first rank whose pass starts at or past the data length
  spk_dresult_t pres;           // a version pass's result
};
bool compat_tiles_ok(const spk_layout *L, uint64_t wire_len);
size_t compat_tiles_ws_bytes(const spk_layout *L, uint64_t wire_len);
hipError_t launch_compat_tiles(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                               void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                               const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                               size_t ctl_off, hipStream_t s);
// spk_nested.hip: layouts with SPK_OP_ARRAY
bool layout_nested(const spk_layout *L);
size_t nested_workspace_bytes(const spk_layout *L, int mode, uint64_t n, uint64_t wire_len);
hipError_t launch_nested_plan(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                              const void *const *d_heaps, spk_plan_t *d_plan, void *d_ws,
                              hipStream_t s);
hipError_t launch_nested_encode(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                                const void *const *d_heaps, void *d_out, uint64_t out_cap,
                                uint64_t *d_msg_offsets, const spk_frame *F, uint32_t fixed_w,
                                void *d_ws, hipStream_t s, const SeqEcho *echo = nullptr);
hipError_t launch_nested_decode(const spk_layout *L, int mode, const void *d_wire,
                                uint64_t wire_len, const uint64_t *d_msg_offsets,
                                uint64_t n_msgs, uint32_t prefix, void *d_recs, uint64_t rec_cap,
                                void *const *d_heaps, const uint64_t *heap_caps,
                                spk_dresult_t *d_res, int32_t *d_errc, void *d_ws,
                                hipStream_t s, uint32_t body_w = 0, uint64_t body_n = 0,
                                const uint64_t *d_msg_ends = nullptr);
// spk_fixed.hip
// d_n (MESSAGES mode, nullable): the message count is min(*d_n, n), read on
// the device (spk_*_dn); grids and workspace stay sized for n
__device__ __forceinline__ uint64_t dev_count(uint64_t n, const uint64_t *d_n) {
  if (!d_n) return n;
  const uint64_t m = *d_n;
  return m < n ? m : n;
}
hipError_t launch_fixed_plan(const spk_layout *L, int mode, uint64_t n,
                             spk_plan_t *d_plan, void *d_ws, hipStream_t s,
                             const uint64_t *d_n = nullptr);
hipError_t launch_fixed_encode_vector(const spk_layout *L, uint64_t n,
                                      const void *d_recs, void *d_out,
                                      const void *d_ws, hipStream_t s);
hipError_t launch_fixed_encode_messages(const spk_layout *L, uint64_t n,
                                        const void *d_recs, void *d_out,
                                        uint64_t *d_offsets, const spk_frame *F,
                                        hipStream_t s, const SeqEcho *echo = nullptr,
                                        const uint64_t *d_n = nullptr,
                                        spk_plan_t *d_plan_out = nullptr,
                                        const spk_plan_t *plan_val = nullptr);
hipError_t launch_fixed_plan_encode_messages(const spk_layout *L, uint64_t n,
                                             const void *d_recs, void *d_out,
                                             uint64_t *d_offsets, spk_plan_t *d_plan,
                                             void *d_ws, hipStream_t s);
// body_w != 0: d_wire is a message BODY of body_n records at width body_w
// (no header / count: spk_decode_body)
hipError_t launch_fixed_decode_vector(const spk_layout *L, const void *d_wire,
                                      uint64_t wire_len, void *d_recs,
                                      uint64_t rec_cap, spk_dresult_t *d_res,
                                      void *d_ws, hipStream_t s, uint32_t body_w = 0,
                                      uint64_t body_n = 0);
hipError_t launch_fixed_decode_messages(const spk_layout *L, const void *d_wire,
                                        uint64_t wire_len,
                                        const uint64_t *d_offsets, uint64_t n,
                                        uint32_t prefix, void *d_recs, uint64_t rec_cap,
                                        spk_dresult_t *d_res, int32_t *d_errc,
                                        void *d_ws, hipStream_t s,
                                        const uint64_t *d_msg_ends = nullptr,
                                        const uint64_t *d_n = nullptr);
// spk_var.hip
size_t var_workspace_bytes(const spk_layout *L, int mode, uint64_t n,
                           uint64_t wire_len);
hipError_t launch_var_plan(const spk_layout *L, int mode, uint64_t n,
                           const void *d_recs, spk_plan_t *d_plan, void *d_ws,
                           size_t ws_bytes, hipStream_t s, const uint64_t *d_n = nullptr);
bool var_plan_encode_small_ok(const spk_layout *L, uint64_t n);
hipError_t launch_var_plan_encode_small(const spk_layout *L, int mode, uint64_t n,
                                        const void *d_recs, const void *const *d_heaps,
                                        spk_plan_t *d_plan, void *d_out, uint64_t out_cap,
                                        uint64_t *d_offsets, void *d_ws, hipStream_t s);
hipError_t launch_var_encode(const spk_layout *L, int mode, uint64_t n,
                             const void *d_recs, const void *const *d_heaps,
                             const spk_plan_t *d_plan, void *d_out,
                             uint64_t out_cap, uint64_t *d_offsets, const spk_frame *F,
                             void *d_ws, size_t ws_bytes, hipStream_t s,
                             const SeqEcho *echo = nullptr, const uint64_t *d_n = nullptr);
hipError_t launch_var_encode_body(const spk_layout *L, uint64_t n, const void *d_recs,
                                  const void *const *d_heaps, uint32_t width, void *d_out,
                                  uint64_t out_cap, void *d_ws, size_t ws_bytes,
                                  hipStream_t s);
hipError_t launch_var_decode(const spk_layout *L, int mode, const void *d_wire,
                             uint64_t wire_len, const uint64_t *d_offsets,
                             uint64_t n_msgs, uint32_t prefix, void *d_recs, uint64_t rec_cap,
                             void *const *d_heaps, const uint64_t *heap_caps,
                             spk_dresult_t *d_res, int32_t *d_errc, void *d_ws,
                             size_t ws_bytes, hipStream_t s, uint32_t body_w = 0, uint64_t body_n = 0,
                             const uint64_t *d_msg_ends = nullptr,
                             const uint64_t *d_n = nullptr);
}  // namespace spk
