"""ctypes mirror of include/spk_codec.h and loaders for the two native
libraries:

  * yalantinglibs_amd/libspk_codec.so — the product: HIP kernels + C ABI.
    `load_codec()` raises if it is missing; there is no CPU fallback.
  * oracle/libspk_oracle.so — the CPU restatement used ONLY as a checker by
    tests/, smoke() and bench.py's cpu_baseline (`load_oracle()`).
"""
from __future__ import annotations

import ctypes as ct
import os

SPK_ABI_VERSION = 2
SPK_MAX_OPS = 64
SPK_MAX_SPANS = 32
SPK_MAX_LITERAL = 240
SPK_MAX_FRAME = 64
SPK_MAX_ROUTES = 16
SPK_FRAME_NONE = 0xFFFFFFFF

SPK_OK = 0
SPK_E_ARG = -1
SPK_E_LAYOUT = -2
SPK_E_WORKSPACE = -3
SPK_E_CAPACITY = -4
SPK_E_HIP = -5

ERRC_OK = 0
ERRC_NO_BUFFER_SPACE = 1
ERRC_INVALID_BUFFER = 2
ERRC_HASH_CONFLICT = 3
ERRC_INVALID_WIDTH = 4
ERRC_CAPACITY = 100

SPK_OP_COPY = 1
SPK_OP_SPAN = 2
SPK_OP_OPTION = 3
SPK_OP_VARINT = 4
SPK_OP_ARRAY = 5
SPK_OP_END = 6
SPK_OP_VARIANT = 7
SPK_OP_COMPAT = 8  # | version rank << 8
SPK_OP_FVAR = 9
SPK_OP_OPTGROUP = 10
SPK_OP_CGROUP = 11  # | version rank << 8
SPK_FVAR_SIGNED = 1
SPK_VARINT_SEXT = 2
SPK_MAX_DEPTH = 4
SPK_VARINT_ZIGZAG = 1
SPK_MAX_VARINTS = 16
SPK_MODE_VECTOR = 0
SPK_MODE_MESSAGES = 1

SPK_MF_HASH_HEAD = 0x1
SPK_MF_TYPE_LITERAL = 0x2
SPK_MF_HAS_CONTAINER = 0x4
SPK_LAYOUT_TRIVIAL = 0x1

SPK_SYNTH_REC64 = 1
SPK_SYNTH_RECS = 2
SPK_SYNTH_OUTER = 3
SPK_SYNTH_RPCRECT = 4
SPK_SYNTH_PERSON = 5
SPK_SYNTH_INTS = 6
SPK_SYNTH_MONSTER = 7


class spk_op(ct.Structure):
    _fields_ = [("kind", ct.c_uint32), ("rec_off", ct.c_uint32),
                ("size", ct.c_uint32), ("aux", ct.c_uint32)]


class spk_msgfmt(ct.Structure):
    _fields_ = [("code", ct.c_uint32), ("flags", ct.c_uint32),
                ("literal_len", ct.c_uint32), ("reserved", ct.c_uint32),
                ("literal", ct.c_uint8 * SPK_MAX_LITERAL)]


class spk_layout(ct.Structure):
    _fields_ = [("abi", ct.c_uint32), ("flags", ct.c_uint32),
                ("rec_stride", ct.c_uint32), ("n_ops", ct.c_uint32),
                ("ops", spk_op * SPK_MAX_OPS),
                ("fmt_vector", spk_msgfmt), ("fmt_one", spk_msgfmt)]


class spk_plan_t(ct.Structure):
    _fields_ = [("total_bytes", ct.c_uint64), ("max_count", ct.c_uint64),
                ("var_bytes", ct.c_uint64), ("width", ct.c_uint32),
                ("header_bytes", ct.c_uint32), ("metainfo", ct.c_uint32),
                ("has_meta", ct.c_uint32)]


class spk_dresult_t(ct.Structure):
    _fields_ = [("errc", ct.c_int32), ("width", ct.c_uint32),
                ("count", ct.c_uint64), ("consumed", ct.c_uint64),
                ("heap_used", ct.c_uint64 * SPK_MAX_SPANS),
                ("tiles_repaired", ct.c_uint32), ("tiles_sequential", ct.c_uint32)]


class spk_shard_t(ct.Structure):
    _fields_ = [("errc", ct.c_int32), ("width", ct.c_uint32), ("n", ct.c_uint64),
                ("entry", ct.c_uint64), ("exit", ct.c_uint64), ("count", ct.c_uint64),
                ("heap", ct.c_uint64 * SPK_MAX_SPANS), ("tiles_repaired", ct.c_uint64)]


SPK_DECODE_TILE_BYTES = 16384


class spk_frame(ct.Structure):
    _fields_ = [("prefix_len", ct.c_uint32), ("seq_off", ct.c_uint32),
                ("len_off", ct.c_uint32), ("seq_base", ct.c_uint32),
                ("tmpl", ct.c_uint8 * SPK_MAX_FRAME)]


class spk_route_hdr(ct.Structure):
    _fields_ = [("head_len", ct.c_uint32), ("len_off", ct.c_uint32),
                ("attach_off", ct.c_uint32), ("magic", ct.c_int32),
                ("max_version", ct.c_int32), ("serialize_type", ct.c_int32)]


PLAN_BYTES = ct.sizeof(spk_plan_t)
DRES_BYTES = ct.sizeof(spk_dresult_t)

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
# SPK_CODEC_LIB: dev-only override to A/B alternative builds of the same ABI
CODEC_PATH = os.environ.get("SPK_CODEC_LIB") or os.path.join(_HERE, "libspk_codec.so")
ORACLE_PATH = os.path.join(_ROOT, "oracle", "libspk_oracle.so")

# exported symbols of include/spk_codec.h (checked by tests/test_capi.py)
CODEC_SYMBOLS = ["spk_abi_version", "spk_errc_message", "spk_layout_check",
                 "spk_workspace_bytes", "spk_plan", "spk_plan_ex", "spk_encode", "spk_plan_encode",
                 "spk_decode",
                 "spk_synth", "spk_synth_counts", "spk_synth_ex", "spk_synth_counts_ex",
                 "spk_encode_body",
                 "spk_vector_header", "spk_encode_framed", "spk_decode_framed",
                 "spk_decode_body", "spk_parse_vector_header",
                 "spk_message_header", "spk_parse_message_header",
                 "spk_decode_shard_index", "spk_decode_shard_emit",
                 # mixed-type frame batches in arrival order
                 "spk_route_workspace_bytes", "spk_route_frames", "spk_route_frames_checked", "spk_decode_frames",
                 "spk_plan_dn", "spk_decode_frames_dn", "spk_encode_framed_echo_dn",
                 "spk_copy_frame_field", "spk_encode_framed_echo",
                 # runtime helpers (front ends without HIP headers)
                 "spk_device_alloc", "spk_device_free", "spk_host_alloc_pinned",
                 "spk_host_free_pinned", "spk_copy_async", "spk_stream_create",
                 "spk_stream_destroy", "spk_stream_sync",
                 # kernel tracing
                 "spk_trace_enable", "spk_trace_reset", "spk_trace_read"]

_codec = None
_oracle = None

P = ct.c_void_p
U64 = ct.c_uint64
PL = ct.POINTER(spk_layout)


def _bind_codec(lib):
    lib.spk_abi_version.restype = ct.c_uint32
    lib.spk_errc_message.restype = ct.c_char_p
    lib.spk_errc_message.argtypes = [ct.c_int32]
    lib.spk_layout_check.argtypes = [PL]
    lib.spk_workspace_bytes.restype = ct.c_size_t
    lib.spk_workspace_bytes.argtypes = [PL, ct.c_int, U64, U64]
    lib.spk_plan.argtypes = [PL, ct.c_int, U64, P, P, P, ct.c_size_t, P]
    lib.spk_plan_ex.argtypes = [PL, ct.c_int, U64, P, ct.POINTER(P), P, P, ct.c_size_t, P]
    lib.spk_encode.argtypes = [PL, ct.c_int, U64, P, ct.POINTER(P), P, P, U64,
                               P, P, ct.c_size_t, P]
    lib.spk_plan_encode.argtypes = [PL, ct.c_int, U64, P, ct.POINTER(P), P, P, U64,
                                    P, P, ct.c_size_t, P]
    lib.spk_decode.argtypes = [PL, ct.c_int, P, U64, P, U64, P, U64,
                               ct.POINTER(P), ct.POINTER(U64), P, P, P,
                               ct.c_size_t, P]
    lib.spk_synth.argtypes = [ct.c_int, U64, U64, U64, ct.c_uint32, P, P, P, P]
    lib.spk_encode_body.argtypes = [PL, U64, P, ct.POINTER(P), ct.c_uint32, P, U64, P,
                                    ct.c_size_t, P]
    lib.spk_vector_header.argtypes = [PL, U64, ct.c_uint32, ct.POINTER(ct.c_uint8),
                                      ct.c_uint32]
    lib.spk_decode_body.argtypes = [PL, P, U64, ct.c_uint32, U64, P, U64, ct.POINTER(P),
                                    ct.POINTER(U64), P, P, ct.c_size_t, P]
    lib.spk_parse_vector_header.argtypes = [PL, P, U64, ct.POINTER(U64),
                                            ct.POINTER(ct.c_uint32), ct.POINTER(ct.c_uint32)]
    lib.spk_parse_vector_header.restype = ct.c_int32
    lib.spk_message_header.argtypes = [PL, ct.c_uint32, ct.POINTER(ct.c_uint8), ct.c_uint32]
    lib.spk_parse_message_header.argtypes = [PL, P, U64, ct.POINTER(ct.c_uint32),
                                             ct.POINTER(ct.c_uint32)]
    lib.spk_parse_message_header.restype = ct.c_int32
    lib.spk_decode_shard_index.argtypes = [PL, P, U64, U64, U64, U64, P, P, ct.c_size_t, P]
    lib.spk_decode_shard_emit.argtypes = [PL, P, U64, U64, U64, U64, ct.c_int, P, U64,
                                          ct.POINTER(P), ct.POINTER(U64), P, P, ct.c_size_t, P]
    lib.spk_encode_framed.argtypes = [PL, U64, P, ct.POINTER(P), P, ct.POINTER(spk_frame),
                                      P, U64, P, P, ct.c_size_t, P]
    lib.spk_decode_framed.argtypes = [PL, P, U64, P, U64, ct.c_uint32, P, U64,
                                      ct.POINTER(P), ct.POINTER(U64), P, P, P,
                                      ct.c_size_t, P]
    lib.spk_synth_counts.argtypes = [ct.c_int, U64, U64, U64, ct.c_uint32, P, P]
    lib.spk_synth_counts_ex.argtypes = [ct.c_int, U64, U64, U64, ct.c_uint32, P, P]
    lib.spk_synth_ex.argtypes = [ct.c_int, U64, U64, U64, ct.c_uint32, P, ct.POINTER(P), P, P]
    lib.spk_route_workspace_bytes.restype = ct.c_size_t
    lib.spk_route_workspace_bytes.argtypes = [U64, ct.c_uint32]
    lib.spk_route_frames.argtypes = [P, U64, P, U64, ct.c_uint32, ct.POINTER(ct.c_uint32),
                                     ct.c_uint32, ct.POINTER(P), ct.POINTER(P), ct.POINTER(P),
                                     P, P, ct.c_size_t, P]
    lib.spk_route_frames_checked.argtypes = [P, U64, P, U64, ct.c_uint32,
                                             ct.POINTER(ct.c_uint32), ct.c_uint32,
                                             ct.POINTER(spk_route_hdr), ct.POINTER(P),
                                             ct.POINTER(P), ct.POINTER(P), P, P, ct.c_size_t, P]
    lib.spk_decode_frames.argtypes = [PL, P, U64, P, P, U64, ct.c_uint32, P, U64,
                                      ct.POINTER(P), ct.POINTER(U64), P, P, P,
                                      ct.c_size_t, P]
    lib.spk_encode_framed_echo.argtypes = [PL, U64, P, ct.POINTER(P), P, ct.POINTER(spk_frame),
                                           P, P, ct.c_uint32, P, U64, P, P, ct.c_size_t, P]
    lib.spk_plan_dn.argtypes = [PL, P, U64, P, ct.POINTER(P), P, P, ct.c_size_t, P]
    lib.spk_decode_frames_dn.argtypes = [PL, P, U64, P, P, P, U64, ct.c_uint32, P, U64,
                                         ct.POINTER(P), ct.POINTER(U64), P, P, P, ct.c_size_t, P]
    lib.spk_encode_framed_echo_dn.argtypes = [PL, P, U64, P, ct.POINTER(P), P,
                                              ct.POINTER(spk_frame), P, P, ct.c_uint32, P, U64,
                                              P, P, ct.c_size_t, P]
    lib.spk_copy_frame_field.argtypes = [P, P, ct.c_uint32, P, P, ct.c_uint32, ct.c_uint32,
                                         U64, P]
    lib.spk_trace_enable.argtypes = [ct.c_int]
    lib.spk_trace_read.argtypes = [ct.c_char_p, ct.c_size_t]
    return lib


def trace_enable(on: bool = True):
    """Bracket every codec kernel launch with hipEvents (spk_trace_enable)."""
    load_codec().spk_trace_enable(1 if on else 0)


def trace_reset():
    load_codec().spk_trace_reset()


def trace_read() -> dict:
    """{kernel: (launches, total_ms)} since the last reset (syncs the events)."""
    import json
    lib = load_codec()
    n = lib.spk_trace_read(None, 0)
    buf = ct.create_string_buffer(n + 1)
    lib.spk_trace_read(buf, n + 1)
    return {k: (int(v[0]), float(v[1])) for k, v in json.loads(buf.value.decode()).items()}


def load_codec():
    """The HIP codec. Fails loudly when the extension is missing."""
    global _codec
    if _codec is None:
        if not os.path.exists(CODEC_PATH):
            raise RuntimeError(
                f"libspk_codec.so not built ({CODEC_PATH}); run "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        _codec = _bind_codec(ct.CDLL(CODEC_PATH))
        if _codec.spk_abi_version() != SPK_ABI_VERSION:
            raise RuntimeError("libspk_codec.so ABI mismatch")
    return _codec


def load_oracle():
    """CPU restatement — a checker for tests/bench only."""
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_PATH):
            raise RuntimeError(f"oracle not built ({ORACLE_PATH}); make -C oracle oracle")
        lib = ct.CDLL(ORACLE_PATH)
        lib.spko_plan.argtypes = [PL, ct.c_int, U64, P, ct.POINTER(P), ct.POINTER(spk_plan_t)]
        lib.spko_encode.argtypes = [PL, ct.c_int, U64, P, ct.POINTER(P), P, U64,
                                    P, ct.POINTER(U64)]
        lib.spko_encode_body.argtypes = [PL, U64, P, ct.POINTER(P), ct.c_uint, P, U64,
                                         ct.POINTER(U64)]
        lib.spko_decode.argtypes = [PL, ct.c_int, P, U64, P, U64, P, U64,
                                    ct.POINTER(P), ct.POINTER(U64),
                                    ct.POINTER(spk_dresult_t), P]
        _oracle = lib
    return _oracle


def fill_msgfmt(dst: spk_msgfmt, code: int, flags: int, literal: bytes):
    if len(literal) > SPK_MAX_LITERAL:
        raise NotImplementedError("type literal longer than SPK_MAX_LITERAL")
    dst.code = code
    dst.flags = flags
    dst.literal_len = len(literal)
    for i, b in enumerate(literal):
        dst.literal[i] = b
