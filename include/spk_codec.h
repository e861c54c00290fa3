/*
 * spk_codec.h — C ABI of the MI355X struct_pack batch codec.
 *
 * This is the drop-in boundary between a host-side struct_pack front end
 * (our C++20 header include/ylt/struct_pack_gpu.hpp, or the Python mirror
 * yalantinglibs_amd/struct_pack.py) and the hand-written gfx950 HIP kernels
 * in yalantinglibs_amd/csrc/ (spk_api.hip, spk_fixed.hip, spk_var.hip). Plain C: no HIP/torch types, all
 * buffers are raw pointers + sizes, streams are opaque `void*` (hipStream_t).
 *
 * The reference has no C ABI: struct_pack is a header-only template library.
 * Each entry point below replaces one template entry point of
 * /root/reference/include/ylt/struct_pack.hpp for a *batch* of records that
 * lives in device memory (cited per function). The wire bytes are the
 * reference's, byte for byte.
 *
 * Record model ("device record" = what a layout descriptor describes)
 * -------------------------------------------------------------------
 * A record type T is flattened by host reflection into `rec_stride`-byte
 * device records plus one heap per variable-length member:
 *   SPK_OP_COPY  {rec_off, size}            `size` raw bytes of the record
 *                                           (fundamentals, enums, std::array,
 *                                           trivially-serializable sub-structs
 *                                           incl. their padding) — written
 *                                           verbatim, in declaration order.
 *   SPK_OP_SPAN  {rec_off, size, aux}       a std::string / std::vector<U> with
 *                                           U trivially serializable: the record
 *                                           holds a u32 element count at
 *                                           rec_off and a u64 element offset into
 *                                           this span's heap at aux; `size` =
 *                                           sizeof(U). Wire: [count:w][bytes].
 *   SPK_OP_OPTION {rec_off, size, aux}     a std::optional<U> with U trivially
 *                                           serializable: same record fields as
 *                                           SPAN with a count of 0 or 1 (the
 *                                           value sits in this member's heap).
 *                                           Wire: [has_value:1][U if present]
 *                                           (packer.hpp:382-388; any non-zero
 *                                           byte decodes as present like
 *                                           unpacker.hpp:1251-1275). It is not
 *                                           a container: it never sets the
 *                                           width (calculate_size.hpp:100-105).
 *   SPK_OP_VARINT {rec_off, size, aux}     a struct_pack::var_uint32_t /
 *                                           var_uint64_t (aux 0) or var_int32_t /
 *                                           var_int64_t (aux SPK_VARINT_ZIGZAG)
 *                                           held as a plain `size`-byte (4/8)
 *                                           integer at rec_off. Wire: LEB128 of
 *                                           the value (zigzag-mapped first for
 *                                           the signed types), 1-10 bytes
 *                                           (varint.hpp:245-330); aux
 *                                           SPK_VARINT_SEXT: a plain int32_t of an
 *                                           ENCODING_WITH_VARINT record, sign-
 *                                           extended to 64 bits, no zigzag
 *                                           (reflection.hpp:843, varint.hpp:
 *                                           249-259). Decode: a
 *                                           10th byte with its high bit set is
 *                                           invalid_buffer; a truncated varint
 *                                           is no_buffer_space. Not a container.
 *   SPK_OP_ARRAY {rec_off, size, aux}      a std::vector<U> / std::string-like
 *                                           container whose element U is NOT
 *                                           trivially serializable (e.g.
 *                                           vector<string>, vector<struct with
 *                                           a string>): the record holds a u32
 *                                           element count at rec_off and a u64
 *                                           element offset at aux into this
 *                                           op's heap of `size`-byte element
 *                                           records; the ops that follow, up
 *                                           to the matching SPK_OP_END, are
 *                                           U's flattened layout (offsets
 *                                           relative to an element record; they
 *                                           may nest further ARRAYs). Wire:
 *                                           [count:w] then each element as
 *                                           serialize_one(U) (packer.hpp:
 *                                           365-367; decode: unpacker.hpp:
 *                                           1208-1226, stops at the first
 *                                           failing element).
 *   SPK_OP_VARIANT {rec_off, size, 0}      a std::variant of `size` (1..255)
 *                                           alternatives: the record holds the
 *                                           u32 active index at rec_off; the
 *                                           ops that follow are `size` groups,
 *                                           each closed by SPK_OP_END: the
 *                                           flattened alternatives, placed in
 *                                           the same record (an empty group is
 *                                           std::monostate). Wire: [index:1]
 *                                           then the active alternative
 *                                           (packer.hpp:389-398); decode: an
 *                                           index >= size is invalid_buffer
 *                                           (unpacker.hpp:1278-1292).
 *   SPK_OP_END {0, 0, 0, 0}                closes the innermost open ARRAY, VARIANT
 *                                           alternative, OPTGROUP group or CGROUP.
 *   SPK_OP_FVAR {rec_off, size, aux}       a varint member of a top-level record
 *                                           whose sp_config has USE_FAST_VARINT
 *                                           (var_* types; with ENCODING_WITH_VARINT
 *                                           also plain (u)int32/64): a `size`-byte
 *                                           integer at rec_off, aux
 *                                           SPK_FVAR_SIGNED for the signed types.
 *                                           Wire: before the record's other
 *                                           members, a bitset of ceil((k+2)/8)
 *                                           bytes (bit j: FVAR j is non-zero; bits
 *                                           k, k+1: width code c) then every
 *                                           non-zero FVAR in op order as its low
 *                                           min(2^c, size) bytes; c from the
 *                                           largest unsigned value / signed
 *                                           magnitude (v<0: -(v+1)) (packer.hpp:
 *                                           152-235). Decode sign-extends the
 *                                           signed ones; c = 3 without a 64-bit
 *                                           FVAR is invalid_buffer (unpacker.hpp:
 *                                           642-747).
 *   SPK_OP_COMPAT {rec_off, size, aux}     a struct_pack::compatible<U, ver>
 *                                           member (U trivially serializable) of
 *                                           the top-level record: record fields
 *                                           as OPTION. kind = SPK_OP_COMPAT |
 *                                           rank << 8, rank = index of `ver` in
 *                                           the record's sorted distinct versions
 *                                           (only the order reaches the wire). It
 *                                           is skipped by the main pass; after
 *                                           it, one pass per rank writes
 *                                           [has_value:1][U if present] for that
 *                                           rank's members of every record, in
 *                                           record then op order (packer.hpp:
 *                                           66-78,453-461). Excluded from the
 *                                           type literal / hash (type_calculate
 *                                           .hpp:298-303); the message gets a
 *                                           metainfo byte and a total-length
 *                                           field of 2/4/8 bytes after it
 *                                           (calculate_size.hpp:457-470, packer
 *                                           .hpp:108-130). Decode stops the
 *                                           version passes, with no error, at the
 *                                           first member whose has byte would
 *                                           start at or past that length (an
 *                                           older writer); members never reached
 *                                           read as absent; the value read's errc
 *                                           is dropped as for OPTION; consumed =
 *                                           max(position, length), skipping
 *                                           newer versions (unpacker.hpp:
 *                                           292-366,1354-1376). Requires
 *                                           SPK_MF_HASH_HEAD and a non-trivial
 *                                           layout (type_calculate.hpp:868-876).
 *   SPK_OP_OPTGROUP {rec_off, size, 0}     a std::optional<U> (size 1) or
 *                                           std::expected<U, E> (size 2) whose
 *                                           value is NOT trivially serializable
 *                                           (optional<string>, optional<struct
 *                                           with a string> ...): the record holds
 *                                           a u32 has_value at rec_off (0 / 1);
 *                                           the ops that follow are `size`
 *                                           groups closed by SPK_OP_END, placed
 *                                           in the same record like VARIANT
 *                                           alternatives: group 0 = U (present),
 *                                           group 1 = E (expected without a
 *                                           value). Wire: [has_value:1] then
 *                                           U if present (packer.hpp:382-388),
 *                                           else E for an expected (:400-410).
 *                                           Decode: any non-zero byte is
 *                                           present; the errc of the group's
 *                                           decode is dropped and the reader
 *                                           stays where it stopped
 *                                           (unpacker.hpp:1251-1277). Not a
 *                                           container; its value may hold some.
 *   SPK_OP_CGROUP {rec_off, 1, 0}          a struct_pack::compatible<U, ver>
 *                                           member of the top-level record with a
 *                                           U that is NOT trivially serializable:
 *                                           kind = SPK_OP_CGROUP | rank << 8 (as
 *                                           COMPAT); a u32 has_value at rec_off,
 *                                           then U's ops closed by SPK_OP_END,
 *                                           in the same record. Written, read
 *                                           and skipped like COMPAT ([has:1][U]
 *                                           in its version pass), U's containers
 *                                           at the message width.
 * Heaps are numbered in op order over SPAN, OPTION, ARRAY and COMPAT ops at every
 * nesting level; heap k of an ARRAY holds element records, counted in
 * elements like the others. Decode writes every heap packed in wire order.
 * A trivially-serializable T (SPK_LAYOUT_TRIVIAL) is a single COPY of the
 * whole record (reference packer.hpp:418-421, unpacker.hpp:1300-1312).
 *
 * Batch modes
 *   SPK_MODE_VECTOR   one message  == serialize(std::vector<T>{recs...})
 *   SPK_MODE_MESSAGES n messages   == serialize(rec_i) back to back
 *                                     (coro_rpc payload batch), with a u64
 *                                     offsets array of n+1 entries.
 *
 * Error model: functions return SPK_OK or a negative SPK_E_* (bad argument,
 * unsupported layout, HIP failure). Data-dependent wire errors are reported
 * stream-ordered in device memory with the reference's errc values
 * (error_code.hpp:21-27): 0 ok, 1 no_buffer_space, 2 invalid_buffer,
 * 3 hash_conflict, 4 invalid_width_of_container_length.
 *
 * Threading: every call is reentrant; the library keeps no mutable global
 * state; descriptors are immutable and may be cached per type. All device
 * work is enqueued on `stream` with no host synchronisation and no
 * allocation (caller-owned workspace), so calls are hipGraph-capturable.
 */
#ifndef SPK_CODEC_H
#define SPK_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPK_ABI_VERSION 2u
#define SPK_MAX_OPS 64u
#define SPK_MAX_SPANS 32u  /* heaps (variable-length members) per layout */
#define SPK_MAX_LITERAL 240u

/* return codes (host-side; negative) */
#define SPK_OK 0
#define SPK_E_ARG -1         /* null pointer / bad size / bad mode          */
#define SPK_E_LAYOUT -2      /* descriptor malformed or unsupported         */
#define SPK_E_WORKSPACE -3   /* workspace too small                         */
#define SPK_E_CAPACITY -4    /* output buffer provably too small            */
#define SPK_E_HIP -5         /* a HIP runtime call failed                   */

/* reference errc (include/ylt/struct_pack/error_code.hpp:21-27) */
#define SPK_ERRC_OK 0
#define SPK_ERRC_NO_BUFFER_SPACE 1
#define SPK_ERRC_INVALID_BUFFER 2
#define SPK_ERRC_HASH_CONFLICT 3
#define SPK_ERRC_INVALID_WIDTH 4
/* device-side capacity overflow during decode (not a reference errc) */
#define SPK_ERRC_CAPACITY 100
/* internal failure of the decoder (an in-kernel wait timed out; never
 * expected; not a reference errc) */
#define SPK_ERRC_INTERNAL 101

#define SPK_OP_COPY 1u
#define SPK_OP_SPAN 2u
#define SPK_OP_OPTION 3u
#define SPK_OP_VARINT 4u
#define SPK_OP_ARRAY 5u
#define SPK_OP_END 6u
#define SPK_OP_VARIANT 7u
#define SPK_OP_COMPAT 8u       /* | rank << 8 (see above)                    */
#define SPK_OP_FVAR 9u
#define SPK_OP_OPTGROUP 10u
#define SPK_OP_CGROUP 11u      /* | rank << 8                                */
#define SPK_OP_KIND(k) ((k) & 0xFFu)
#define SPK_OP_RANK(k) ((k) >> 8)
#define SPK_MAX_DEPTH 4u       /* ARRAY / VARIANT nesting levels             */

/* spk_op.aux of an SPK_OP_VARINT */
#define SPK_VARINT_ZIGZAG 0x1u /* var_int32_t / var_int64_t (sint<T>): zigzag */
#define SPK_VARINT_SEXT 0x2u   /* plain int32_t under ENCODING_WITH_VARINT     */
/* spk_op.aux of an SPK_OP_FVAR */
#define SPK_FVAR_SIGNED 0x1u
#define SPK_MAX_VARINTS 16u    /* varint members per record                  */

#define SPK_MODE_VECTOR 0
#define SPK_MODE_MESSAGES 1

/* spk_msgfmt.flags — resolved per message type by the host front end from
 * the type and its sp_config exactly like type_calculate.hpp:744-891 */
#define SPK_MF_HASH_HEAD 0x1u     /* !check_if_disable_hash_head            */
#define SPK_MF_TYPE_LITERAL 0x2u  /* check_if_add_type_literal (debug/ENABLE_TYPE_INFO) */
#define SPK_MF_HAS_CONTAINER 0x4u /* check_if_has_container<T>              */

/* spk_layout.flags */
#define SPK_LAYOUT_TRIVIAL 0x1u   /* is_trivial_serializable<T>: 1 COPY op  */

typedef struct spk_op {
  uint32_t kind;    /* SPK_OP_COPY | SPAN | OPTION | VARINT | ARRAY | END | VARIANT | COMPAT | FVAR */
  uint32_t rec_off; /* COPY: source byte offset; SPAN: u32 count offset      */
  uint32_t size;    /* COPY: byte length;       SPAN: element size (bytes)   */
  uint32_t aux;     /* SPAN: u64 heap element-offset field offset; COPY: 0   */
} spk_op;

/* Wire format of one message type (get_type_code / get_type_literal). */
typedef struct spk_msgfmt {
  uint32_t code;           /* get_type_code<M>() : MD5_32(literal) & ~1      */
  uint32_t flags;          /* SPK_MF_*                                       */
  uint32_t literal_len;    /* strlen of get_type_literal<M>() (no NUL)       */
  uint32_t reserved;
  uint8_t literal[SPK_MAX_LITERAL]; /* always filled: decode checks it when
                                       a buffer carries type info            */
} spk_msgfmt;

typedef struct spk_layout {
  uint32_t abi;        /* SPK_ABI_VERSION                                   */
  uint32_t flags;      /* SPK_LAYOUT_*                                      */
  uint32_t rec_stride; /* bytes per device record (multiple of 4)           */
  uint32_t n_ops;
  spk_op ops[SPK_MAX_OPS];
  spk_msgfmt fmt_vector; /* message type std::vector<T> (SPK_MODE_VECTOR)   */
  spk_msgfmt fmt_one;    /* message type T             (SPK_MODE_MESSAGES)  */
} spk_layout;

/* Size pass result (device memory, written by spk_plan).
 * Mirrors serialize_buffer_size {len_, metainfo_} (calculate_size.hpp:391-405). */
typedef struct spk_plan_t {
  uint64_t total_bytes; /* SPK_MODE_VECTOR: message length; MESSAGES: sum  */
  uint64_t max_count;   /* max element count over every container          */
  uint64_t var_bytes;   /* sum of span payload bytes                       */
  uint32_t width;       /* container-length width in bytes (1/2/4/8)       */
  uint32_t header_bytes;/* bytes before the first record (VECTOR mode)     */
  uint32_t metainfo;    /* metainfo byte value (valid if has_meta)         */
  uint32_t has_meta;
} spk_plan_t;

/* spk_plan with the span heaps: required for layouts with SPK_OP_ARRAY
 * (their sizes depend on the element records; spk_plan rejects such a
 * non-empty batch with SPK_E_ARG), accepted for every layout. */
int spk_plan_ex(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                const void *const *d_heaps, spk_plan_t *d_plan, void *d_ws,
                size_t ws_bytes, void *stream);

/* Decode result (device memory, written by spk_decode). */
typedef struct spk_dresult_t {
  int32_t errc;         /* reference errc, or SPK_ERRC_CAPACITY            */
  uint32_t width;
  uint64_t count;       /* records decoded (VECTOR) / messages ok (MESSAGES)*/
  uint64_t consumed;    /* consume_len (struct_pack.hpp:343-357)           */
  uint64_t heap_used[SPK_MAX_SPANS]; /* elements written per span heap     */
  /* diagnostics of the SPK_MODE_VECTOR decoder for variable-size records
   * (zero otherwise; not part of the reference's result): 16 KiB tiles whose
   * speculated record grid missed and were re-resolved in parallel, and tiles
   * the one-wave sequential fixer then had to visit (a record spanning k
   * tiles counts k). */
  uint32_t tiles_repaired;
  uint32_t tiles_sequential;
} spk_dresult_t;

/* ------------------------------------------------------------------------ */
uint32_t spk_abi_version(void);
const char *spk_errc_message(int32_t errc); /* error_code.hpp:28-43 */

/* Validate a descriptor (host only, no device work). SPK_OK or SPK_E_LAYOUT. */
int spk_layout_check(const spk_layout *L);

/* Device workspace needed for `n` records (encode) or a `wire_len`-byte
 * input (decode) in `mode`. */
size_t spk_workspace_bytes(const spk_layout *L, int mode, uint64_t n,
                           uint64_t wire_len);

/* Size pass: get_needed_size / get_serialize_runtime_info
 * (ref struct_pack.hpp:131-135, calculate_size.hpp:407-474).
 * Reads only the span counts of variable records; O(1) for trivial T.
 * Writes *d_plan (device). */
int spk_plan(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
             spk_plan_t *d_plan, void *d_ws, size_t ws_bytes, void *stream);

/* Write pass: serialize_to(char*, serialize_buffer_size, vector<T>) for
 * SPK_MODE_VECTOR (ref struct_pack.hpp:161-167, packer.hpp:535-585), or n
 * independent serialize_to calls for SPK_MODE_MESSAGES (then
 * d_msg_offsets[0..n] receives the message boundaries; nullable).
 * `d_heaps` is a HOST array of n_span DEVICE pointers. `d_plan` must come
 * from spk_plan on the same records (stream-ordered), run on the same
 * workspace: the write pass reads the size pass's partials (or, for layouts
 * with element records, its per-record offsets) from it. Writes at most
 * out_cap bytes; if the plan exceeds out_cap nothing is written and
 * d_plan->total_bytes tells the caller the size needed. */
int spk_encode(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
               const void *const *d_heaps, const spk_plan_t *d_plan,
               void *d_out, uint64_t out_cap, uint64_t *d_msg_offsets,
               void *d_ws, size_t ws_bytes, void *stream);

/* Plan + encode in one call: serialize(t) as get_needed_size then
 * serialize_to (ref struct_pack.hpp:75-190), spk_plan_ex followed by
 * spk_encode with the same arguments -- d_plan receives the plan, d_out the
 * bytes when plan->total_bytes <= out_cap (a variable-size layout's write
 * otherwise writes nothing: read the plan, encode again with spk_encode).
 * A batch of at most 256 records of a flat variable-size layout (a small
 * call's message) takes one kernel launch instead of three to five. */
int spk_plan_encode(const spk_layout *L, int mode, uint64_t n, const void *d_recs,
                    const void *const *d_heaps, spk_plan_t *d_plan, void *d_out,
                    uint64_t out_cap, uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes,
                    void *stream);

/* Decode: deserialize_to(vector<T>&, const char*, size_t, size_t&)
 * (ref struct_pack.hpp:343-357, unpacker.hpp:101-162,548-619,780-1349) for
 * SPK_MODE_VECTOR; for SPK_MODE_MESSAGES, message i is
 * d_wire[d_msg_offsets[i] .. d_msg_offsets[i+1]) and is decoded into record
 * i with its errc in d_errc[i] (nullable) and d_res->count = #ok.
 * Records go to d_recs (capacity rec_cap records); span elements go to
 * d_heaps[k] (capacity heap_caps[k] elements; HOST arrays of device
 * pointers / sizes) at canonical offsets (record order, packed).
 * SPK_MODE_VECTOR with rec_cap below the message's count (or a heap too
 * small): the records that fit are written, d_res->count = the message's
 * count, consumed = its length, errc SPK_ERRC_CAPACITY -- unless the wire has
 * a read error, whose errc wins as in the reference -- so rec_cap 0 is a
 * count probe (compatible-member layouts included). */
int spk_decode(const spk_layout *L, int mode, const void *d_wire,
               uint64_t wire_len, const uint64_t *d_msg_offsets, uint64_t n_msgs,
               void *d_recs, uint64_t rec_cap, void *const *d_heaps,
               const uint64_t *heap_caps, spk_dresult_t *d_res,
               int32_t *d_errc, void *d_ws, size_t ws_bytes, void *stream);

/* ---- framed message batches (coro_rpc payloads, SPK_MODE_MESSAGES) -----
 * coro_rpc sends every request as [req_header (20 B)][serialize(args)] and
 * every response as [resp_header (16 B)][serialize(ret)]: the client reserves
 * the header with serialize_to_with_offset (ref struct_pack.hpp:176-189,
 * coro_rpc_client.hpp:1285-1335) and fills it with the DISABLE_ALL_META_INFO
 * encoding of the header struct, i.e. its raw bytes; the server does the same
 * with resp_header (coro_rpc_protocol.hpp:191-240). A spk_frame describes
 * that prefix: a template plus two u32 LE fields patched per message — the
 * sequence number (seq_base + message index) and the payload length. */
#define SPK_MAX_FRAME 64u
#define SPK_FRAME_NONE 0xFFFFFFFFu
typedef struct spk_frame {
  uint32_t prefix_len;  /* bytes before every message (0..SPK_MAX_FRAME)     */
  uint32_t seq_off;     /* u32 LE = seq_base + i at this offset, or NONE     */
  uint32_t len_off;     /* u32 LE = struct_pack message length, or NONE      */
  uint32_t seq_base;
  uint8_t tmpl[SPK_MAX_FRAME]; /* the other prefix bytes (magic, version,
                                  function_id, attach_length ...)           */
} spk_frame;

/* spk_encode for SPK_MODE_MESSAGES with a frame prefix before every message:
 * message i = [prefix][serialize(rec_i)], d_msg_offsets[i] = its frame start;
 * total = d_plan->total_bytes + n * prefix_len. */
int spk_encode_framed(const spk_layout *L, uint64_t n, const void *d_recs,
                      const void *const *d_heaps, const spk_plan_t *d_plan,
                      const spk_frame *F, void *d_out, uint64_t out_cap,
                      uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes,
                      void *stream);
/* spk_decode for SPK_MODE_MESSAGES where frame i is
 * d_wire[d_msg_offsets[i] .. d_msg_offsets[i+1]) and its struct_pack message
 * starts prefix_len bytes in (the header fields were already checked by the
 * transport, coro_rpc_protocol.hpp:98-117). A frame shorter than the prefix
 * reads as no_buffer_space; `consumed` counts message bytes only. */
int spk_decode_framed(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                      const uint64_t *d_msg_offsets, uint64_t n_msgs,
                      uint32_t prefix_len, void *d_recs, uint64_t rec_cap,
                      void *const *d_heaps, const uint64_t *heap_caps,
                      spk_dresult_t *d_res, int32_t *d_errc, void *d_ws,
                      size_t ws_bytes, void *stream);

/* ---- mixed-type request batches in arrival order (coro_rpc server) -------
 * A connection's request frames interleave function ids; the reference
 * server looks each one up in its handler map and decodes it with that
 * handler's argument types (router.hpp:226-240, coro_rpc_protocol.hpp:60-95).
 * spk_route_frames does the lookup for a whole batch in one pass: frame i is
 * d_wire[d_frame_offsets[i] .. d_frame_offsets[i+1]); its u32 LE key at byte
 * key_off (req_header.function_id: key_off 8) is looked up in h_keys[0..n_keys)
 * (n_keys <= SPK_MAX_ROUTES, distinct). For every key k the frames carrying it
 * are listed IN ARRIVAL ORDER: d_begins[k][j] / d_ends[k][j] = the j-th such
 * frame's bounds, d_index[k][j] (nullable) = its arrival index i;
 * d_counts[k] = how many. Frames with another key, or shorter than
 * key_off + 4 bytes, are counted in d_counts[n_keys] and listed in list
 * n_keys when d_begins[n_keys] is non-null (host arrays of n_keys + 1 device
 * pointers, each list with room for n_frames entries). d_counts (device,
 * n_keys + 1 words) is written in stream order: read it before launching the
 * per-type decodes (spk_decode_frames). */
#define SPK_MAX_ROUTES 16u
size_t spk_route_workspace_bytes(uint64_t n_frames, uint32_t n_keys);
int spk_route_frames(const void *d_wire, uint64_t wire_len, const uint64_t *d_frame_offsets,
                     uint64_t n_frames, uint32_t key_off, const uint32_t *h_keys,
                     uint32_t n_keys, uint64_t *const *d_begins, uint64_t *const *d_ends,
                     uint64_t *const *d_index, uint64_t *d_counts, void *d_ws,
                     size_t ws_bytes, void *stream);
/* The frame header check the reference server makes before dispatching
 * (coro_rpc_protocol.hpp:98-117 read_head: magic == 21, version <= 0;
 * get_serialize_protocol: serialize_type == 0; read_payload: `length` body
 * bytes then `attach_length` attachment bytes). With it, frame i is routed
 * only if it holds head_len bytes, passes every check that is not -1 and
 * head_len + length + attach_length == its size; the others go to the
 * unrouted list n_keys. d_ends[k][j] is then the END OF THE MESSAGE,
 * begin + head_len + length (the attachment, which follows it, is not
 * struct_pack bytes), so spk_decode_frames sees only the message.
 * attach_off = SPK_FRAME_NONE: the header has no attachment length. */
typedef struct spk_route_hdr {
  uint32_t head_len;       /* 20 (req_header)                        */
  uint32_t len_off;        /* 12: u32 LE body length                 */
  uint32_t attach_off;     /* 16: u32 LE attachment length, or NONE  */
  int32_t magic;           /* byte 0 (21), or -1                     */
  int32_t max_version;     /* byte 1 <= this (0), or -1              */
  int32_t serialize_type;  /* byte 2 (0), or -1                      */
} spk_route_hdr;
/* spk_route_frames with the header check (hdr NULL = spk_route_frames). */
int spk_route_frames_checked(const void *d_wire, uint64_t wire_len,
                             const uint64_t *d_frame_offsets, uint64_t n_frames,
                             uint32_t key_off, const uint32_t *h_keys, uint32_t n_keys,
                             const spk_route_hdr *hdr, uint64_t *const *d_begins,
                             uint64_t *const *d_ends, uint64_t *const *d_index,
                             uint64_t *d_counts, void *d_ws, size_t ws_bytes, void *stream);
/* spk_decode_framed over frames that need not be adjacent: frame i is
 * d_wire[d_begins[i] .. d_ends[i]) (one type's lists from spk_route_frames). */
int spk_decode_frames(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                      const uint64_t *d_begins, const uint64_t *d_ends, uint64_t n_msgs,
                      uint32_t prefix_len, void *d_recs, uint64_t rec_cap,
                      void *const *d_heaps, const uint64_t *heap_caps,
                      spk_dresult_t *d_res, int32_t *d_errc, void *d_ws,
                      size_t ws_bytes, void *stream);
/* spk_encode_framed whose message i carries, instead of seq_base + i, the
 * u32 LE at d_seq_src[d_seq_offsets[i] + seq_src_off] in its frame's seq
 * field: responses encoded per type echo their requests' seq_num
 * (coro_rpc_protocol.hpp:191-201) with d_seq_src = the request frames and
 * d_seq_offsets = that type's d_begins from spk_route_frames, seq_src_off = 4.
 * F->seq_off must name the field. */
int spk_encode_framed_echo(const spk_layout *L, uint64_t n, const void *d_recs,
                           const void *const *d_heaps, const spk_plan_t *d_plan,
                           const spk_frame *F, const void *d_seq_src,
                           const uint64_t *d_seq_offsets, uint32_t seq_src_off, void *d_out,
                           uint64_t out_cap, uint64_t *d_msg_offsets, void *d_ws,
                           size_t ws_bytes, void *stream);
/* ---- device-resident message counts (graph-capturable server steps) ------
 * The _dn forms of the plan, the echo encode and the frames decode take the
 * MESSAGES-mode message count from device memory: the count is
 * min(*d_n, n_max), read by the kernels when they run. After
 * spk_route_frames, d_n = &d_counts[k] sizes function id k's decode and
 * response encode without the host reading the counts back, so route ->
 * decode -> encode is one stream-ordered (and capturable) sequence. Grids,
 * workspace and the trivial-record capacity check are sized for n_max (the
 * caller's buffers: rec_cap / out_cap / offsets for n_max messages). A decode
 * whose *d_n exceeds n_max decodes the first n_max frames and reports
 * SPK_ERRC_CAPACITY. Flat layouts only (SPK_E_LAYOUT for ARRAY / VARIANT /
 * group / FVAR layouts, whose kernels size on the host). */
int spk_plan_dn(const spk_layout *L, const uint64_t *d_n, uint64_t n_max, const void *d_recs,
                const void *const *d_heaps, spk_plan_t *d_plan, void *d_ws, size_t ws_bytes,
                void *stream);
int spk_decode_frames_dn(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                         const uint64_t *d_begins, const uint64_t *d_ends, const uint64_t *d_n,
                         uint64_t n_max, uint32_t prefix_len, void *d_recs, uint64_t rec_cap,
                         void *const *d_heaps, const uint64_t *heap_caps, spk_dresult_t *d_res,
                         int32_t *d_errc, void *d_ws, size_t ws_bytes, void *stream);
int spk_encode_framed_echo_dn(const spk_layout *L, const uint64_t *d_n, uint64_t n_max,
                              const void *d_recs, const void *const *d_heaps,
                              const spk_plan_t *d_plan, const spk_frame *F,
                              const void *d_seq_src, const uint64_t *d_seq_offsets,
                              uint32_t seq_src_off, void *d_out, uint64_t out_cap,
                              uint64_t *d_msg_offsets, void *d_ws, size_t ws_bytes,
                              void *stream);
/* For i < n: copy `bytes` (1..8) from d_src[d_src_offsets[i] + src_off] to
 * d_dst[d_dst_offsets[i] + dst_off]: the response header echoes its request's
 * seq_num (coro_rpc_protocol.hpp:191-201) when responses were encoded per
 * type (spk_encode_framed numbers them seq_base + j): src = the request
 * frames at d_begins[k] (seq_num at 4), dst = the response frames (at 4). */
int spk_copy_frame_field(void *d_dst, const uint64_t *d_dst_offsets, uint32_t dst_off,
                         const void *d_src, const uint64_t *d_src_offsets, uint32_t src_off,
                         uint32_t bytes, uint64_t n, void *stream);

/* ---- sharded single-message encode (multi-GPU, SPK_MODE_VECTOR) --------
 * One std::vector<T> message whose records are spread over several GPUs:
 * every shard encodes only its records' bytes ("body") with the GLOBAL
 * container-length width (max over all shards' counts and the global record
 * count: calculate_size.hpp:426-447), and the shard holding record 0 also
 * writes the header + global count (spk_vector_header). Concatenating the
 * shard bodies after the header in shard order gives exactly the bytes of
 * serialize(vector<T>) over all records.
 * spk_plan(SPK_MODE_VECTOR) on the shard gives max_count (local) and
 * var_bytes; body size = var_bytes + n * n_spans * width. */
int spk_encode_body(const spk_layout *L, uint64_t n, const void *d_recs,
                    const void *const *d_heaps, uint32_t width, void *d_out,
                    uint64_t out_cap, void *d_ws, size_t ws_bytes, void *stream);
/* Decode exactly n records from a message BODY — the bytes after the header
 * and the container count of a SPK_MODE_VECTOR message of width `width` —
 * into d_recs / d_heaps: the counterpart of spk_encode_body, for pipelined
 * (chunked H2D) and sharded decodes where the front end has parsed the
 * header already (spk_parse_vector_header). Errors and d_res as spk_decode;
 * d_res->consumed counts body bytes. Heaps are written from element 0. */
int spk_decode_body(const spk_layout *L, const void *d_body, uint64_t body_len,
                    uint32_t width, uint64_t n, void *d_recs, uint64_t rec_cap,
                    void *const *d_heaps, const uint64_t *heap_caps,
                    spk_dresult_t *d_res, void *d_ws, size_t ws_bytes, void *stream);

/* ---- sharded decode of one SPK_MODE_VECTOR message ----------------------
 * Every rank holds the message; rank r decodes the records that START in
 * its tiles [tile_lo, tile_hi) of the body (SPK_DECODE_TILE_BYTES each,
 * counted from the first byte after the header and count). Records are
 * self-delimiting only from a known start, so:
 *   1. spk_decode_shard_index: speculative index of the range from `entry`
 *      (the wire offset of the range's first record start; SPK_ENTRY_UNKNOWN
 *      lets the range guess it) -> *d_summary: the entry used, the exit
 *      (first record start at or past the range end), the records and heap
 *      elements on that path;
 *   2. the ranks exchange summaries: the range is right when its entry is
 *      the previous range's exit (range 0's entry is exact); a wrong one is
 *      indexed again from that exit (normally never);
 *   3. spk_decode_shard_emit (same workspace, same tiles): the range's
 *      records into rank-local buffers (record 0 = global record `first`,
 *      heaps from element 0), clipped at the message's count; `last` marks
 *      the range holding the message's end (its shortfall is the errc).
 * Layouts with SPK_OP_ARRAY / SPK_OP_VARIANT, and trivially-serializable
 * records (plain offset arithmetic, spk_decode_body), are rejected
 * (SPK_E_LAYOUT). */
#define SPK_DECODE_TILE_BYTES 16384u
#define SPK_ENTRY_UNKNOWN (~0ull)
typedef struct spk_shard_t {
  int32_t errc;         /* header errc                                       */
  uint32_t width;
  uint64_t n;           /* the message's record count                        */
  uint64_t entry;       /* first record start the range was indexed from     */
  uint64_t exit;        /* first record start at/past the range end; ~0 when
                           the path ends inside the range                    */
  uint64_t count;       /* records starting in the range on that path        */
  uint64_t heap[SPK_MAX_SPANS]; /* their heap elements per span            */
  uint64_t tiles_repaired;
} spk_shard_t;
int spk_decode_shard_index(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                           uint64_t tile_lo, uint64_t tile_hi, uint64_t entry,
                           spk_shard_t *d_summary, void *d_ws, size_t ws_bytes,
                           void *stream);
int spk_decode_shard_emit(const spk_layout *L, const void *d_wire, uint64_t wire_len,
                          uint64_t tile_lo, uint64_t tile_hi, uint64_t first, int last,
                          void *d_recs, uint64_t rec_cap, void *const *d_heaps,
                          const uint64_t *heap_caps, spk_dresult_t *d_res, void *d_ws,
                          size_t ws_bytes, void *stream);

/* HOST function: deserialize_metainfo of a SPK_MODE_VECTOR message in host
 * memory (unpacker.hpp:548-619) plus its container count. Returns the
 * reference errc (0 ok) or a negative SPK_E_*; on success *n = records,
 * *width, *header_len = bytes before the first record. */
int32_t spk_parse_vector_header(const spk_layout *L, const void *h_wire, uint64_t len,
                                uint64_t *n, uint32_t *width, uint32_t *header_len);

/* Host-side: the header of ONE message of the layout's message type
 * (fmt_one) at container width `width` into h_out (HOST memory): the whole
 * message when the type has no payload bytes, e.g. std::monostate, the reply
 * of a void coro_rpc handler (struct_pack_protocol.hpp:34-36; packer.hpp:
 * 90-139,250-252). Returns its length, or a negative SPK_E_*. */
int spk_message_header(const spk_layout *L, uint32_t width, uint8_t *h_out, uint32_t cap);
/* Host-side: deserialize_metainfo of one message (fmt_one) in host memory
 * (unpacker.hpp:548-619): reference errc (0 ok) or a negative SPK_E_*; on
 * success *width and *header_len = bytes before the payload. */
int32_t spk_parse_message_header(const spk_layout *L, const void *h_wire, uint64_t len,
                                 uint32_t *width, uint32_t *header_len);

/* Host-side: header + count prefix of a VECTOR message of total_n records at
 * `width` into h_out (HOST memory, capacity cap). Returns its length, or a
 * negative SPK_E_*. (packer.hpp:100-139) */
int spk_vector_header(const spk_layout *L, uint64_t total_n, uint32_t width,
                      uint8_t *h_out, uint32_t cap);

/* ---- synthetic inputs (bench / tests): the seeded generator of
 * oracle/ref/types.hpp, restated on the device so the GPU box regenerates
 * exactly the inputs the golden digests were taken from. ---------------- */
#define SPK_SYNTH_REC64 1
#define SPK_SYNTH_RECS 2
#define SPK_SYNTH_OUTER 3
#define SPK_SYNTH_RPCRECT 4 /* C5 coro_rpc payload shapes */
#define SPK_SYNTH_PERSON 5
#define SPK_SYNTH_INTS 6
#define SPK_SYNTH_MONSTER 7 /* the reference benchmark's Monster: six heaps */
int spk_synth(int kind, uint64_t seed, uint64_t first, uint64_t n,
              uint32_t param, void *d_recs, void *d_heap,
              const uint64_t *d_heap_offsets, void *stream);
/* per-record span counts for variable kinds (to size/prefix the heap) */
int spk_synth_counts(int kind, uint64_t seed, uint64_t first, uint64_t n,
                     uint32_t param, uint64_t *d_counts, void *stream);
/* kinds with several heaps (SPK_SYNTH_MONSTER): d_counts and d_heap_offsets
 * are [heaps][n] columns (elements of each heap per record; their exclusive
 * prefix sums); d_heaps a HOST array of the heaps' device pointers */
int spk_synth_counts_ex(int kind, uint64_t seed, uint64_t first, uint64_t n,
                        uint32_t param, uint64_t *d_counts, void *stream);
int spk_synth_ex(int kind, uint64_t seed, uint64_t first, uint64_t n, uint32_t param,
                 void *d_recs, void *const *d_heaps, const uint64_t *d_heap_offsets,
                 void *stream);

/* ---- runtime helpers ----------------------------------------------------
 * Device / pinned-host memory, async copies and streams, so that a front end
 * (our C++ header, a cgo / JNI / ctypes binding) needs no HIP headers of its
 * own. Return SPK_OK or SPK_E_ARG / SPK_E_HIP. */
#define SPK_COPY_H2D 1
#define SPK_COPY_D2H 2
#define SPK_COPY_D2D 3
int spk_device_alloc(void **d_ptr, size_t bytes);
int spk_device_free(void *d_ptr);
int spk_host_alloc_pinned(void **h_ptr, size_t bytes);
int spk_host_free_pinned(void *h_ptr);
int spk_copy_async(void *dst, const void *src, size_t bytes, int kind, void *stream);
int spk_stream_create(void **stream); /* non-blocking stream */
int spk_stream_destroy(void *stream);
int spk_stream_sync(void *stream);

/* ---- kernel tracing ------------------------------------------------------
 * Off by default. When enabled, every kernel the codec launches is bracketed
 * by hipEvents on its stream; spk_trace_read (after the work completes)
 * writes {"<kernel>": [launches, total_ms], ...} accumulated since the last
 * reset into buf and returns the JSON length. For profiling runs: the events
 * cost a few microseconds per launch. */
int spk_trace_enable(int on);
int spk_trace_reset(void);
int spk_trace_read(char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SPK_CODEC_H */
