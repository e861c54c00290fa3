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
and skip it on decode. A connection's frames arrive with their function ids
interleaved: FrameRouter splits such a batch per function id in one pass
(spk_route_frames, arrival order kept per id) for spk_decode_frames, and
echoes each request's seq_num into its response (spk_copy_frame_field).
This module builds those frame descriptors and restates the header layout
for host-side checks.
"""
from __future__ import annotations

import ctypes as ct
import struct

from . import _capi as C
from . import schema as S

# coro_rpc_protocol.hpp:45, 250 and the header structs at :60-79
MAGIC_NUMBER = 21
REQ_SEQ_OFF, REQ_FID_OFF, RESP_SEQ_OFF = 4, 8, 4
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


def frame_offsets_from_stream(buf: bytes, head_len: int = REQ_HEAD_LEN, len_off: int = 12,
                              attach_off: int | None = None):
    """Host walk of a received byte stream of frames (what coro_connection's
    read_head / read_payload loop sees: `length` body bytes, then
    `attach_length` attachment bytes, coro_rpc_protocol.hpp:138-159; the
    attachment length follows the length in both headers): returns the n+1
    frame offsets (attach_off -1: no attachment field)."""
    if attach_off is None:
        attach_off = len_off + 4
    offs = [0]
    p = 0
    while p + head_len <= len(buf):
        (ln,) = struct.unpack_from("<I", buf, p + len_off)
        (at,) = struct.unpack_from("<I", buf, p + attach_off) if attach_off >= 0 else (0,)
        p += head_len + ln + at
        offs.append(p)
    return offs


def req_route_hdr() -> C.spk_route_hdr:
    """The server's check of a request header before dispatch (read_head,
    coro_rpc_protocol.hpp:98-117; get_serialize_protocol :84-91)."""
    return C.spk_route_hdr(REQ_HEAD_LEN, 12, 16, MAGIC_NUMBER, VERSION_NUMBER, 0)


def _stream(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ct.c_void_p(s.cuda_stream)


class FrameRouter:
    """Dispatch of a batch of request frames by function id, as the server's
    handler lookup does frame by frame (router.hpp:226-240): for function id
    k the frames are listed in arrival order (begins[k] / ends[k] / index[k]),
    frames with unknown ids in the extra list n_keys. counts (device) holds
    n_keys + 1 sizes after route(); counts_host() reads them."""

    def __init__(self, function_ids, capacity: int, device="cuda", check=True):
        import torch
        if len(function_ids) > C.SPK_MAX_ROUTES:
            raise ValueError(f"at most {C.SPK_MAX_ROUTES} function ids per router")
        self.lib = C.load_codec()
        self.keys = [int(f) & 0xFFFFFFFF for f in function_ids]
        self.capacity = capacity
        self.device = device
        nk = len(self.keys)
        mk = lambda: [torch.empty(max(capacity, 1), dtype=torch.int64, device=device)
                      for _ in range(nk + 1)]
        self.begins, self.ends, self.index = mk(), mk(), mk()
        self.counts = torch.zeros(nk + 1, dtype=torch.int64, device=device)
        need = int(self.lib.spk_route_workspace_bytes(capacity, nk))
        self._ws = torch.empty(need, dtype=torch.uint8, device=device)
        ptrs = lambda ts: (ct.c_void_p * (nk + 1))(*[t.data_ptr() for t in ts])
        self._pb, self._pe, self._pi = ptrs(self.begins), ptrs(self.ends), ptrs(self.index)
        self._keys = (ct.c_uint32 * max(nk, 1))(*(self.keys or [0]))
        # check: frames the server would reject (bad magic / version /
        # serialize_type, sizes that disagree with length + attach_length) are
        # unrouted, and ends[k] is where the message ends (attachment excluded)
        self._hdr = ct.pointer(req_route_hdr()) if check else None

    def route(self, wire, offsets, n: int, stream=None):
        """Stream-ordered: frame i = wire[offsets[i] .. offsets[i+1])."""
        if n > self.capacity:
            raise ValueError("more frames than the router's capacity")
        rc = self.lib.spk_route_frames_checked(
            ct.c_void_p(wire.data_ptr()), wire.numel(), ct.c_void_p(offsets.data_ptr()), n,
            REQ_FID_OFF, self._keys, len(self.keys), self._hdr, self._pb, self._pe, self._pi,
            ct.c_void_p(self.counts.data_ptr()), ct.c_void_p(self._ws.data_ptr()),
            self._ws.numel(), _stream(stream))
        if rc != 0:
            raise RuntimeError(f"spk_route_frames failed with {rc}")
        return self.counts

    def counts_host(self):
        return [int(x) for x in self.counts.cpu().tolist()]


def copy_frame_field(dst, dst_offsets, dst_off: int, src, src_offsets, src_off: int,
                     nbytes: int, n: int, stream=None):
    """spk_copy_frame_field: dst[dst_offsets[i] + dst_off ..] = src[src_offsets[i] +
    src_off ..] (nbytes) for i < n — e.g. response seq_num = request seq_num."""
    lib = C.load_codec()
    rc = lib.spk_copy_frame_field(ct.c_void_p(dst.data_ptr()), ct.c_void_p(dst_offsets.data_ptr()),
                                  dst_off, ct.c_void_p(src.data_ptr()),
                                  ct.c_void_p(src_offsets.data_ptr()), src_off, nbytes, n,
                                  _stream(stream))
    if rc != 0:
        raise RuntimeError(f"spk_copy_frame_field failed with {rc}")
