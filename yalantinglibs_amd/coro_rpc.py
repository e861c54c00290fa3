"""coro_rpc payload framing for batched struct_pack messages (host side).

coro_rpc (ref include/ylt/coro_rpc/) frames every call on the wire as

  request : [req_header  20 B][struct_pack::serialize(args...)]
  response: [resp_header 16 B][struct_pack::serialize(ret)]

The client reserves the header with struct_pack::serialize_to_with_offset and
then writes the header struct with sp_config::DISABLE_ALL_META_INFO, which for
these trivially serializable structs is their raw little-endian bytes
(coro_rpc_client.hpp:1285-1335); the server builds resp_header the same way
(coro_rpc_protocol.hpp:191-240) and checks magic / version on read
(coro_rpc_protocol.hpp:98-117). Function ids are MD5Hash32 of the function
name (router.hpp:121-127).

On MI355X a batch of such calls is one spk_encode_framed / spk_decode_framed
launch per record type (include/spk_codec.h): the kernels write the header
template with the per-message sequence number and payload length patched in,
and skip it on decode. This module builds those frame descriptors and
restates the header layout for host-side checks.
"""
from __future__ import annotations

import struct

from . import _capi as C
from . import schema as S

# coro_rpc_protocol.hpp:45, 250 and the header structs at :60-79
MAGIC_NUMBER = 21
VERSION_NUMBER = 0
REQ_HEAD_LEN = 20
RESP_HEAD_LEN = 16
_REQ = struct.Struct("<BBBBIIII")   # magic version serialize_type msg_type seq fid len attach
_RESP = struct.Struct("<BBBBIII")   # magic version err_code msg_type seq len attach
assert _REQ.size == REQ_HEAD_LEN and _RESP.size == RESP_HEAD_LEN


def func_id(name: str) -> int:
    """router::auto_gen_register_key: MD5Hash32Constexpr of the function name."""
    return S.md5_hash32(name.encode())


def pack_req_header(seq_num: int, function_id: int, length: int, attach_length: int = 0,
                    serialize_type: int = 0, msg_type: int = 0) -> bytes:
    return _REQ.pack(MAGIC_NUMBER, VERSION_NUMBER, serialize_type, msg_type,
                     seq_num & 0xFFFFFFFF, function_id, length, attach_length)


def pack_resp_header(seq_num: int, length: int, attach_length: int = 0, err_code: int = 0,
                     msg_type: int = 0) -> bytes:
    return _RESP.pack(MAGIC_NUMBER, VERSION_NUMBER, err_code, msg_type,
                      seq_num & 0xFFFFFFFF, length, attach_length)


def unpack_req_header(b: bytes) -> dict:
    m, v, st, mt, seq, fid, ln, at = _REQ.unpack(b[:REQ_HEAD_LEN])
    return {"magic": m, "version": v, "serialize_type": st, "msg_type": mt,
            "seq_num": seq, "function_id": fid, "length": ln, "attach_length": at}


def _frame(tmpl: bytes, seq_off: int, len_off: int, seq_base: int) -> C.spk_frame:
    f = C.spk_frame()
    f.prefix_len = len(tmpl)
    f.seq_off = seq_off
    f.len_off = len_off
    f.seq_base = seq_base & 0xFFFFFFFF
    for i, b in enumerate(tmpl):
        f.tmpl[i] = b
    return f


def req_frame(function_id: int, seq_base: int = 0, attach_length: int = 0) -> C.spk_frame:
    """Frame of a request batch: message i carries seq_num = seq_base + i
    (client request_id_++, coro_rpc_client.hpp:1304-1308)."""
    return _frame(pack_req_header(0, function_id, 0, attach_length), 4, 12, seq_base)


def resp_frame(seq_base: int = 0, err_code: int = 0) -> C.spk_frame:
    """Frame of a response batch (prepare_response, coro_rpc_protocol.hpp:191-240):
    seq_num echoes the request's."""
    return _frame(pack_resp_header(0, 0, 0, err_code), 4, 8, seq_base)


def frame_offsets_from_stream(buf: bytes, head_len: int = REQ_HEAD_LEN, len_off: int = 12):
    """Host walk of a received byte stream of frames (what coro_connection's
    read_head / read_payload loop sees): returns the n+1 frame offsets."""
    offs = [0]
    p = 0
    while p + head_len <= len(buf):
        (ln,) = struct.unpack_from("<I", buf, p + len_off)
        p += head_len + ln
        offs.append(p)
    return offs
