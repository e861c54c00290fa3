"""struct_pack entry points over the MI355X codec (Python host mirror).

Mirrors the reference's API (include/ylt/struct_pack.hpp) for batches of
records resident in device memory:

  get_type_code(T)                      struct_pack.hpp:75-92
  get_needed_size(batch, mode)          struct_pack.hpp:131-135
  serialize_to(out, batch, mode)        struct_pack.hpp:161-167
  serialize(batch, mode)                struct_pack.hpp:198-207
  deserialize_to(batch_out, wire, ...)  struct_pack.hpp:343-357
  deserialize(T, wire, ...)             struct_pack.hpp:393-413

A batch is `RecordBatch(layout, recs, heaps)`: `recs` is a (n, stride)
uint8 CUDA tensor of device records (schema.flatten), `heaps` one uint8
CUDA tensor per variable-length member. Errors follow the reference's errc
values (error_code.hpp:21-27) via `errc` below; there is no CPU fallback —
every call goes through libspk_codec.so and fails loudly without it.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import _capi as C
from . import schema as S
from .layout import Layout, make_layout

MODE_VECTOR = C.SPK_MODE_VECTOR
MODE_MESSAGES = C.SPK_MODE_MESSAGES


class errc:  # struct_pack::errc
    ok = C.ERRC_OK
    no_buffer_space = C.ERRC_NO_BUFFER_SPACE
    invalid_buffer = C.ERRC_INVALID_BUFFER
    hash_conflict = C.ERRC_HASH_CONFLICT
    invalid_width_of_container_length = C.ERRC_INVALID_WIDTH
    capacity = C.ERRC_CAPACITY  # device-side output capacity (not in the reference)


def get_type_code(*types: S.SpType) -> int:
    return S.get_type_code(*types)


def _stream(stream=None) -> ct.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return ct.c_void_p(s.cuda_stream)


def _p(t: Optional[torch.Tensor]) -> ct.c_void_p:
    return ct.c_void_p(t.data_ptr() if t is not None and t.numel() else 0)


@dataclass
class RecordBatch:
    layout: Layout
    recs: torch.Tensor                      # (n, stride) uint8, device
    heaps: List[torch.Tensor] = field(default_factory=list)

    @property
    def n(self) -> int:
        return int(self.recs.shape[0])


class Codec:
    """Per-type codec: descriptor + cached workspace / plan buffers."""

    def __init__(self, layout: Layout, device="cuda"):
        self.L = layout
        self.lib = C.load_codec()
        self.device = torch.device(device)
        rc = self.lib.spk_layout_check(self.L.ptr)
        if rc != 0:
            raise ValueError(f"layout rejected by spk_layout_check ({rc})")
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.plan_buf = torch.zeros(C.PLAN_BYTES, dtype=torch.uint8, device=self.device)
        self.res_buf = torch.zeros(C.DRES_BYTES, dtype=torch.uint8, device=self.device)

    @classmethod
    def for_type(cls, t: S.SpType, conf: int = S.DEFAULT, debug: bool = False,
                 vector_config=None, device="cuda"):
        return cls(make_layout(t, conf, debug, vector_config), device)

    # ---- workspace -------------------------------------------------------
    def workspace(self, mode: int, n: int, wire_len: int = 0) -> torch.Tensor:
        need = int(self.lib.spk_workspace_bytes(self.L.ptr, mode, n, wire_len))
        if need == 0:
            raise ValueError("spk_workspace_bytes rejected the layout")
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def _heap_ptrs(self, heaps):
        # empty heaps (all counts zero) still need a valid device pointer
        if not hasattr(self, "_dummy"):
            self._dummy = torch.zeros(16, dtype=torch.uint8, device=self.device)
        k = max(self.L.n_spans, 1)
        ptrs = [h.data_ptr() if h.numel() else self._dummy.data_ptr() for h in heaps]
        return (ct.c_void_p * k)(*(ptrs or [0]))

    @staticmethod
    def _check(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed with {rc}")

    # ---- encode ----------------------------------------------------------
    def plan(self, batch: RecordBatch, mode: int, stream=None) -> torch.Tensor:
        """Size pass (stream-ordered): writes spk_plan_t into self.plan_buf."""
        ws = self.workspace(mode, batch.n)
        self._check(self.lib.spk_plan_ex(self.L.ptr, mode, batch.n, _p(batch.recs),
                                         self._heap_ptrs(batch.heaps), _p(self.plan_buf),
                                         _p(ws), ws.numel(), _stream(stream)), "spk_plan_ex")
        return self.plan_buf

    def get_needed_size(self, batch: RecordBatch, mode: int = MODE_VECTOR) -> C.spk_plan_t:
        """Host copy of the size pass (synchronises)."""
        self.plan(batch, mode)
        return C.spk_plan_t.from_buffer_copy(bytes(self.plan_buf.cpu().numpy()))

    def serialize_to(self, out: torch.Tensor, batch: RecordBatch, mode: int = MODE_VECTOR,
                     offsets: Optional[torch.Tensor] = None, stream=None,
                     planned: bool = False, frame: Optional[C.spk_frame] = None):
        """Plan + write into a caller-owned device buffer (no host sync).
        `frame` (MODE_MESSAGES only) reserves and fills a per-message prefix
        such as coro_rpc's req_header (see yalantinglibs_amd.coro_rpc)."""
        ws = self.workspace(mode, batch.n)
        if not planned and frame is None:  # (one launch for a small batch)
            self._check(self.lib.spk_plan_encode(
                self.L.ptr, mode, batch.n, _p(batch.recs), self._heap_ptrs(batch.heaps),
                _p(self.plan_buf), _p(out), out.numel(), _p(offsets), _p(ws), ws.numel(),
                _stream(stream)), "spk_plan_encode")
            return
        if not planned:
            self.plan(batch, mode, stream)
        if frame is not None:
            if mode != MODE_MESSAGES:
                raise ValueError("frames apply to MODE_MESSAGES batches")
            self._check(self.lib.spk_encode_framed(
                self.L.ptr, batch.n, _p(batch.recs), self._heap_ptrs(batch.heaps),
                _p(self.plan_buf), ct.byref(frame), _p(out), out.numel(), _p(offsets),
                _p(ws), ws.numel(), _stream(stream)), "spk_encode_framed")
            return
        self._check(self.lib.spk_encode(self.L.ptr, mode, batch.n, _p(batch.recs),
                                        self._heap_ptrs(batch.heaps), _p(self.plan_buf),
                                        _p(out), out.numel(), _p(offsets), _p(ws),
                                        ws.numel(), _stream(stream)), "spk_encode")

    def serialize_echo(self, out: torch.Tensor, batch: RecordBatch, offsets: torch.Tensor,
                       frame: C.spk_frame, seq_src: torch.Tensor, seq_offsets: torch.Tensor,
                       seq_src_off: int = 4, stream=None, d_count: Optional[torch.Tensor] = None):
        """spk_encode_framed_echo (plan + write, no host sync): message i's
        frame carries seq_src[seq_offsets[i] + seq_src_off ..+4] as its
        seq_num — responses echoing their routed requests. d_count (a device
        int64 tensor, e.g. a FrameRouter count): encode its first
        min(*d_count, batch.n) records (spk_plan_dn / spk_encode_framed_echo_dn)
        without reading the count on the host."""
        ws = self.workspace(MODE_MESSAGES, batch.n)
        if d_count is not None:
            self._check(self.lib.spk_plan_dn(
                self.L.ptr, _p(d_count), batch.n, _p(batch.recs), self._heap_ptrs(batch.heaps),
                _p(self.plan_buf), _p(ws), ws.numel(), _stream(stream)), "spk_plan_dn")
            self._check(self.lib.spk_encode_framed_echo_dn(
                self.L.ptr, _p(d_count), batch.n, _p(batch.recs), self._heap_ptrs(batch.heaps),
                _p(self.plan_buf), ct.byref(frame), _p(seq_src), _p(seq_offsets), seq_src_off,
                _p(out), out.numel(), _p(offsets), _p(ws), ws.numel(), _stream(stream)),
                "spk_encode_framed_echo_dn")
            return
        self.plan(batch, MODE_MESSAGES, stream)
        self._check(self.lib.spk_encode_framed_echo(
            self.L.ptr, batch.n, _p(batch.recs), self._heap_ptrs(batch.heaps),
            _p(self.plan_buf), ct.byref(frame), _p(seq_src), _p(seq_offsets), seq_src_off,
            _p(out), out.numel(), _p(offsets), _p(ws), ws.numel(), _stream(stream)),
            "spk_encode_framed_echo")

    def serialize(self, batch: RecordBatch, mode: int = MODE_VECTOR):
        """Returns (wire uint8 tensor, message offsets or None)."""
        plan = self.get_needed_size(batch, mode)
        out = torch.empty(max(plan.total_bytes, 1), dtype=torch.uint8, device=self.device)
        offs = (torch.empty(batch.n + 1, dtype=torch.int64, device=self.device)
                if mode == MODE_MESSAGES else None)
        self.serialize_to(out, batch, mode, offs, planned=True)
        return out[:plan.total_bytes], offs

    # ---- decode ----------------------------------------------------------
    def deserialize_to(self, out: RecordBatch, wire: torch.Tensor, mode: int = MODE_VECTOR,
                       offsets: Optional[torch.Tensor] = None, n_msgs: int = 0,
                       errc_out: Optional[torch.Tensor] = None, heap_caps=None,
                       stream=None, prefix: int = 0) -> torch.Tensor:
        """Decode into caller-owned buffers; returns the device result
        (spk_dresult_t bytes). Stream-ordered, no host sync. `prefix`
        (MODE_MESSAGES only) skips a frame header before every message."""
        cap = out.n
        ws = self.workspace(mode, cap if mode == MODE_VECTOR else n_msgs, wire.numel())
        caps = heap_caps or [h.numel() // sp.elem.size
                             for h, sp in zip(out.heaps, self.L.dev.spans)]
        hc = (ct.c_uint64 * max(len(caps), 1))(*(caps or [0]))
        if prefix:
            if mode != MODE_MESSAGES:
                raise ValueError("frames apply to MODE_MESSAGES batches")
            self._check(self.lib.spk_decode_framed(
                self.L.ptr, _p(wire), wire.numel(), _p(offsets), n_msgs, prefix, _p(out.recs),
                cap, self._heap_ptrs(out.heaps), hc, _p(self.res_buf), _p(errc_out), _p(ws),
                ws.numel(), _stream(stream)), "spk_decode_framed")
            return self.res_buf
        self._check(self.lib.spk_decode(self.L.ptr, mode, _p(wire), wire.numel(), _p(offsets),
                                        n_msgs, _p(out.recs), cap, self._heap_ptrs(out.heaps),
                                        hc, _p(self.res_buf), _p(errc_out), _p(ws),
                                        ws.numel(), _stream(stream)), "spk_decode")
        return self.res_buf

    def deserialize_frames(self, out: RecordBatch, wire: torch.Tensor, begins: torch.Tensor,
                           ends: torch.Tensor, n_msgs: int, prefix: int,
                           errc_out: Optional[torch.Tensor] = None, heap_caps=None,
                           stream=None, d_count: Optional[torch.Tensor] = None) -> torch.Tensor:
        """spk_decode_frames: message i = wire[begins[i] + prefix .. ends[i]) —
        one record type's frames routed out of a mixed batch
        (coro_rpc.FrameRouter). Stream-ordered, no host sync. d_count (device
        int64): the frame count read on the device, n_msgs its upper bound
        (spk_decode_frames_dn)."""
        ws = self.workspace(MODE_MESSAGES, n_msgs, wire.numel())
        caps = heap_caps or [h.numel() // sp.elem.size
                             for h, sp in zip(out.heaps, self.L.dev.spans)]
        hc = (ct.c_uint64 * max(len(caps), 1))(*(caps or [0]))
        if d_count is not None:
            self._check(self.lib.spk_decode_frames_dn(
                self.L.ptr, _p(wire), wire.numel(), _p(begins), _p(ends), _p(d_count), n_msgs,
                prefix, _p(out.recs), out.n, self._heap_ptrs(out.heaps), hc, _p(self.res_buf),
                _p(errc_out), _p(ws), ws.numel(), _stream(stream)), "spk_decode_frames_dn")
            return self.res_buf
        self._check(self.lib.spk_decode_frames(
            self.L.ptr, _p(wire), wire.numel(), _p(begins), _p(ends), n_msgs, prefix,
            _p(out.recs), out.n, self._heap_ptrs(out.heaps), hc, _p(self.res_buf),
            _p(errc_out), _p(ws), ws.numel(), _stream(stream)), "spk_decode_frames")
        return self.res_buf

    def deserialize_body(self, out: RecordBatch, body: torch.Tensor, width: int, n: int,
                         heap_caps=None, stream=None) -> torch.Tensor:
        """spk_decode_body: n records from a VECTOR message body (after the
        header and count) at `width` — chunked / sharded decodes."""
        ws = self.workspace(MODE_VECTOR, out.n, body.numel())
        caps = heap_caps or [h.numel() // sp.elem.size
                             for h, sp in zip(out.heaps, self.L.dev.spans)]
        hc = (ct.c_uint64 * max(len(caps), 1))(*(caps or [0]))
        self._check(self.lib.spk_decode_body(self.L.ptr, _p(body), body.numel(), width, n,
                                             _p(out.recs), out.n, self._heap_ptrs(out.heaps),
                                             hc, _p(self.res_buf), _p(ws), ws.numel(),
                                             _stream(stream)), "spk_decode_body")
        return self.res_buf

    def shard_index(self, wire: torch.Tensor, tile_lo: int, tile_hi: int, entry: int,
                    stream=None):
        """spk_decode_shard_index -> host ShardSummary (synchronises)."""
        from .parallel import ShardSummary
        ws = self.workspace(MODE_VECTOR, 0, wire.numel())
        if not hasattr(self, "_shard_buf"):
            self._shard_buf = torch.zeros(ct.sizeof(C.spk_shard_t), dtype=torch.uint8,
                                          device=self.device)
        self._check(self.lib.spk_decode_shard_index(
            self.L.ptr, _p(wire), wire.numel(), tile_lo, tile_hi, entry, _p(self._shard_buf),
            _p(ws), ws.numel(), _stream(stream)), "spk_decode_shard_index")
        r = C.spk_shard_t.from_buffer_copy(bytes(self._shard_buf.cpu().numpy()))
        return ShardSummary(r.errc, r.width, r.n, r.entry, r.exit, r.count, list(r.heap))

    def shard_emit(self, out: RecordBatch, wire: torch.Tensor, tile_lo: int, tile_hi: int,
                   first: int, last: bool, stream=None) -> C.spk_dresult_t:
        """spk_decode_shard_emit into `out` (same workspace as shard_index)."""
        ws = self.workspace(MODE_VECTOR, 0, wire.numel())  # the index pass's buffer
        caps = [h.numel() // sp.elem.size for h, sp in zip(out.heaps, self.L.dev.spans)]
        hc = (ct.c_uint64 * max(len(caps), 1))(*(caps or [0]))
        self._check(self.lib.spk_decode_shard_emit(
            self.L.ptr, _p(wire), wire.numel(), tile_lo, tile_hi, first, 1 if last else 0,
            _p(out.recs), out.n, self._heap_ptrs(out.heaps), hc, _p(self.res_buf), _p(ws),
            ws.numel(), _stream(stream)), "spk_decode_shard_emit")
        return self.result()

    def parse_vector_header(self, host_bytes: bytes):
        """Host parse of a VECTOR message head: (errc, n, width, header_len)."""
        n, w, hl = ct.c_uint64(), ct.c_uint32(), ct.c_uint32()
        buf = (ct.c_uint8 * max(len(host_bytes), 1)).from_buffer_copy(host_bytes or b"\0")
        e = self.lib.spk_parse_vector_header(self.L.ptr, buf, len(host_bytes), ct.byref(n),
                                             ct.byref(w), ct.byref(hl))
        return int(e), n.value, w.value, hl.value

    def result(self) -> C.spk_dresult_t:
        return C.spk_dresult_t.from_buffer_copy(bytes(self.res_buf.cpu().numpy()))

    def alloc_batch(self, n: int, heap_elems: Optional[List[int]] = None) -> RecordBatch:
        recs = torch.zeros((max(n, 0), self.L.stride), dtype=torch.uint8, device=self.device)
        heaps = []
        for k, sp in enumerate(self.L.dev.spans):
            cnt = heap_elems[k] if heap_elems else 0
            heaps.append(torch.zeros(max(cnt, 1) * sp.elem.size, dtype=torch.uint8,
                                     device=self.device))
        return RecordBatch(self.L, recs, heaps)

    def deserialize(self, wire: torch.Tensor, mode: int = MODE_VECTOR,
                    offsets: Optional[torch.Tensor] = None, n_msgs: int = 0):
        """Allocating decode: capacities bounded by the wire length.
        Returns (result, RecordBatch, errc tensor or None)."""
        wl = wire.numel()
        min_rec = S.min_record_wire_bytes(self.L.dev)
        cap = (wl // min_rec + 1) if mode == MODE_VECTOR else n_msgs
        elems = S.heap_caps_for_wire(self.L.dev, wl, cap)
        out = self.alloc_batch(cap, elems)
        ec = (torch.zeros(max(n_msgs, 1), dtype=torch.int32, device=self.device)
              if mode == MODE_MESSAGES else None)
        self.deserialize_to(out, wire, mode, offsets, n_msgs, ec)
        res = self.result()
        n = res.count if mode == MODE_VECTOR else n_msgs
        out = RecordBatch(self.L, out.recs[:n], out.heaps)
        return res, out, ec


def synth_batch(codec: Codec, kind: str, n: int, seed: int, param: int = 48,
                first: int = 0, stream=None) -> RecordBatch:
    """Device-generated synthetic batch (spk_synth) for rec64 / recs / outer
    and the C5 coro_rpc shapes rpcrect / person / ints."""
    lib = codec.lib
    dev = codec.device
    kinds = {"rec64": C.SPK_SYNTH_REC64, "recs": C.SPK_SYNTH_RECS, "outer": C.SPK_SYNTH_OUTER,
             "rpcrect": C.SPK_SYNTH_RPCRECT, "person": C.SPK_SYNTH_PERSON,
             "ints": C.SPK_SYNTH_INTS}
    if kind == "monster":
        return _synth_multi(codec, C.SPK_SYNTH_MONSTER, n, seed, param, first, stream)
    k = kinds[kind]
    recs = torch.empty((n, codec.L.stride), dtype=torch.uint8, device=dev)
    st = _stream(stream)
    if k in (C.SPK_SYNTH_REC64, C.SPK_SYNTH_RPCRECT):
        Codec._check(lib.spk_synth(k, seed, first, n, param, _p(recs), None, None, st),
                     "spk_synth")
        return RecordBatch(codec.L, recs, [])
    cnt = torch.empty(n, dtype=torch.int64, device=dev)
    Codec._check(lib.spk_synth_counts(k, seed, first, n, param, _p(cnt), st), "spk_synth_counts")
    offs = torch.cumsum(cnt, 0) - cnt
    total = int(cnt.sum().item()) if n else 0
    esz = codec.L.dev.spans[0].elem.size
    heap = torch.zeros(max(total, 1) * esz, dtype=torch.uint8, device=dev)
    Codec._check(lib.spk_synth(k, seed, first, n, param, _p(recs), _p(heap), _p(offs), st),
                 "spk_synth")
    return RecordBatch(codec.L, recs, [heap])


def _synth_multi(codec: Codec, k: int, n: int, seed: int, param: int, first: int,
                 stream=None) -> RecordBatch:
    """spk_synth_ex: a kind with one heap per variable-length member
    (counts pass, exclusive scans per heap, fill pass)."""
    lib, dev, st = codec.lib, codec.device, _stream(stream)
    nh = len(codec.L.dev.spans)
    # the device generator writes the Monster's 96-B records and its 6 heaps
    # (csrc/spk_synth.hip kMonHeaps): any other layout would be written past
    if k == C.SPK_SYNTH_MONSTER and (nh != 6 or codec.L.stride != 96):
        raise ValueError(f"monster synth needs the Monster layout (6 heaps, 96-B records), "
                         f"got {nh} heaps and stride {codec.L.stride}")
    cnt = torch.empty((nh, max(n, 1)), dtype=torch.int64, device=dev)
    Codec._check(lib.spk_synth_counts_ex(k, seed, first, n, param, _p(cnt), st),
                 "spk_synth_counts_ex")
    cnt = cnt[:, :n]
    offs = (torch.cumsum(cnt, 1) - cnt).contiguous()
    totals = cnt.sum(1).tolist() if n else [0] * nh
    heaps = [torch.zeros(max(int(t), 1) * sp.elem.size, dtype=torch.uint8, device=dev)
             for t, sp in zip(totals, codec.L.dev.spans)]
    recs = torch.empty((n, codec.L.stride), dtype=torch.uint8, device=dev)
    hp = (ct.c_void_p * nh)(*[h.data_ptr() for h in heaps])
    Codec._check(lib.spk_synth_ex(k, seed, first, n, param, _p(recs), hp, _p(offs), st),
                 "spk_synth_ex")
    heaps = [h[:int(t) * sp.elem.size] for h, t, sp in zip(heaps, totals, codec.L.dev.spans)]
    return RecordBatch(codec.L, recs, heaps)
