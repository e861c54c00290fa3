"""Multi-GPU struct_pack: record-range shards, one process per GPU.

Two shapes:

* Independent shards (the bench's weak-scaling path): every rank encodes /
  decodes its own records as its own messages. No data-path collective.

* One message over all shards (`ShardedVectorEncoder`): the bytes of
  serialize(std::vector<T>) over the concatenation of every rank's records.
  The container-length width is a whole-message property (max element count
  over every container, incl. the global record count:
  calculate_size.hpp:426-447), so the ranks agree on it with one 8-byte
  all-reduce(MAX); an all-gather of each rank's body size gives its byte
  offset; every rank encodes its body with the global width (spk_encode_body)
  and rank 0 prepends the header (spk_vector_header). Concatenation is a
  grouped RCCL send/recv of the bodies into rank 0's output buffer (over
  xGMI), or — for the coro_rpc destination — each rank's D2H into its offset
  of one pinned host buffer.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _capi as C
from .struct_pack import Codec, RecordBatch, _p, _stream


@dataclass
class ShardPlan:
    global_n: int
    width: int
    header: bytes            # rank 0's header + count prefix
    body_bytes: List[int]    # per rank
    offsets: List[int]       # byte offset of each rank's body in the message
    total_bytes: int


def width_of(max_count: int) -> int:
    """calculate_size.hpp:426-447."""
    return 1 if max_count < 1 << 8 else 2 if max_count < 1 << 16 else 4 if max_count < 1 << 32 else 8


def count_fields(plan) -> int:
    """Width-w count fields in the body of a local VECTOR plan (every SPAN and
    ARRAY length, at every nesting level): total = header + var + fields * w."""
    if plan.width == 0:
        return 0
    return (plan.total_bytes - plan.header_bytes - plan.var_bytes) // plan.width


def agree_shard_plan(local_n: int, local_max_count: int, local_var_bytes: int,
                     n_cont: int, header_fn, group=None, device=None,
                     local_fields: Optional[int] = None) -> ShardPlan:
    """Collective part of the sharded encode (works on gloo or nccl):
    all-reduce(SUM) of record counts, all-reduce(MAX) of the largest element
    count, all-gather of body sizes. The body holds local_fields count fields
    (n_cont per record for flat layouts; count_fields(plan) in general)."""
    world = dist.get_world_size(group)
    dev = device if device is not None else torch.device("cpu")
    t = torch.tensor([local_n, local_max_count], dtype=torch.int64, device=dev)
    s = t.clone()
    dist.all_reduce(s[:1], op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(s[1:], op=dist.ReduceOp.MAX, group=group)
    global_n, gmax = int(s[0].item()), int(s[1].item())
    w = width_of(max(global_n, gmax))
    fields = local_n * n_cont if local_fields is None else local_fields
    body = local_var_bytes + fields * w
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([body], dtype=torch.int64, device=dev), group=group)
    body_bytes = [int(x.item()) for x in sizes]
    header = header_fn(global_n, w)
    offsets, off = [], len(header)
    for b in body_bytes:
        offsets.append(off)
        off += b
    return ShardPlan(global_n, w, header, body_bytes, offsets, off)


class ShardedVectorEncoder:
    """serialize(std::vector<T>) of records spread over the ranks of a
    process group (one GPU per rank)."""

    def __init__(self, codec: Codec, group=None):
        self.cd = codec
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def header(self, global_n: int, width: int) -> bytes:
        buf = (ct.c_uint8 * 512)()
        n = self.cd.lib.spk_vector_header(self.cd.L.ptr, global_n, width, buf, 512)
        if n < 0:
            raise RuntimeError(f"spk_vector_header failed ({n})")
        return bytes(buf[:n])

    def plan(self, batch: RecordBatch) -> ShardPlan:
        p = self.cd.get_needed_size(batch, C.SPK_MODE_VECTOR)
        return agree_shard_plan(batch.n, p.max_count, p.var_bytes, 0,
                                self.header, self.group,
                                None if self._host_staged() else self.cd.device,
                                local_fields=count_fields(p))

    def encode_body(self, batch: RecordBatch, width: int, out: torch.Tensor, stream=None):
        ws = self.cd.workspace(C.SPK_MODE_VECTOR, batch.n)
        rc = self.cd.lib.spk_encode_body(self.cd.L.ptr, batch.n, _p(batch.recs),
                                         self.cd._heap_ptrs(batch.heaps), width, _p(out),
                                         out.numel(), _p(ws), ws.numel(), _stream(stream))
        if rc != 0:
            raise RuntimeError(f"spk_encode_body failed ({rc})")

    def _host_staged(self) -> bool:
        # gloo moves host tensors only (CPU rehearsals); RCCL moves HBM directly
        return dist.get_backend(self.group) == "gloo"

    def gather(self, sp: ShardPlan, body: torch.Tensor, out: Optional[torch.Tensor],
               root: int = 0) -> None:
        """P2P concatenation: every rank's body goes into its slice of root's
        message buffer `out` (grouped RCCL send/recv over xGMI; root also
        writes the header and its own body). `out` is ignored off root."""
        mine = sp.body_bytes[self.rank]
        staged = self._host_staged()
        if self.rank == root:
            o = sp.offsets[self.rank]
            out[:len(sp.header)].copy_(torch.frombuffer(bytearray(sp.header), dtype=torch.uint8))
            out[o:o + mine].copy_(body[:mine])
            ops, bufs = [], []
            for r in range(self.world):
                if r != root and sp.body_bytes[r]:
                    o = sp.offsets[r]
                    dst = out[o:o + sp.body_bytes[r]]
                    if staged:
                        dst = torch.empty(sp.body_bytes[r], dtype=torch.uint8)
                        bufs.append((o, dst))
                    ops.append(dist.P2POp(dist.irecv, dst, r, self.group))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            for o, b in bufs:
                out[o:o + b.numel()].copy_(b)
        elif mine:
            src = body[:mine].cpu() if staged else body[:mine]
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, src, root, self.group)]):
                req.wait()

    def all_gather(self, sp: ShardPlan, body: torch.Tensor, out: torch.Tensor,
                   slab: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Every rank receives the whole message: one RCCL all-gather of the
        bodies padded to the largest, then an on-device compaction behind the
        header. `slab` (world x max body bytes) may be passed to reuse it."""
        mb = max(max(sp.body_bytes), 1)
        mine = sp.body_bytes[self.rank]
        staged = self._host_staged()
        dev = torch.device("cpu") if staged else body.device
        if slab is None or slab.device != dev:
            slab = torch.empty(self.world * mb, dtype=torch.uint8, device=dev)
        send = torch.zeros(mb, dtype=torch.uint8, device=dev)
        send[:mine].copy_(body[:mine])
        if staged:
            dist.all_gather(list(slab.view(self.world, mb).unbind(0)), send, group=self.group)
        else:
            dist.all_gather_into_tensor(slab, send, group=self.group)
        out[:len(sp.header)].copy_(torch.frombuffer(bytearray(sp.header), dtype=torch.uint8))
        for r in range(self.world):
            o, b = sp.offsets[r], sp.body_bytes[r]
            out[o:o + b].copy_(slab[r * mb:r * mb + b])
        return slab

    def encode(self, batch: RecordBatch, root: int = 0) -> Optional[torch.Tensor]:
        """Returns the whole message on `root` (None elsewhere). The bodies
        move to root with grouped RCCL point-to-point transfers straight into
        their slices of the output buffer."""
        sp = self.plan(batch)
        mine = sp.body_bytes[self.rank]
        body = torch.empty(max(mine, 1), dtype=torch.uint8, device=self.cd.device)
        self.encode_body(batch, sp.width, body)
        out = (torch.empty(sp.total_bytes, dtype=torch.uint8, device=self.cd.device)
               if self.rank == root else None)
        self.gather(sp, body, out, root)
        return out

    def encode_to_host(self, batch: RecordBatch, host_out: torch.Tensor) -> ShardPlan:
        """coro_rpc destination: every rank copies its body D2H straight into
        its offset of one (shared, pinned) host buffer; rank 0 also writes
        the header. `host_out` must be visible to all ranks (e.g. a shared
        memory tensor) and at least plan.total_bytes long."""
        sp = self.plan(batch)
        mine = sp.body_bytes[self.rank]
        body = torch.empty(max(mine, 1), dtype=torch.uint8, device=self.cd.device)
        self.encode_body(batch, sp.width, body)
        o = sp.offsets[self.rank]
        host_out[o:o + mine].copy_(body[:mine])
        if self.rank == 0:
            host_out[:len(sp.header)].copy_(torch.frombuffer(bytearray(sp.header),
                                                             dtype=torch.uint8))
        torch.cuda.synchronize(self.cd.device)
        dist.barrier(self.group)
        return sp


# ---------------------------------------------------------------------------
# Sharded decode of ONE vector message (spk_decode_shard_index / _emit)
# ---------------------------------------------------------------------------
TILE_BYTES = C.SPK_DECODE_TILE_BYTES
ENTRY_UNKNOWN = (1 << 64) - 1


@dataclass
class ShardSummary:
    errc: int
    width: int
    n: int
    entry: int
    exit: int
    count: int
    heap: List[int]

    def as_list(self) -> List[int]:
        return [self.errc, self.width, self.n, self.entry, self.exit, self.count] + list(self.heap)

    @staticmethod
    def from_list(v) -> "ShardSummary":
        v = [int(x) for x in v]
        return ShardSummary(v[0], v[1], v[2], v[3], v[4], v[5], v[6:])


def tile_ranges(n_tiles: int, world: int) -> List[tuple]:
    """Even split of the body's tiles over the ranks."""
    return [(n_tiles * r // world, n_tiles * (r + 1) // world) for r in range(world)]


def settle_entries(sums: List[ShardSummary]) -> List[Optional[int]]:
    """The exchange step: range r stands when its entry is range r-1's exit
    (range 0 starts at the payload: exact). Returns, per rank, None when its
    summary stands, else the entry to index it again from: the previous
    range's current exit. A chain of k wrong ranges settles in at most k
    rounds; a range after the one where the path ends is left alone (it
    holds no records)."""
    redo: List[Optional[int]] = [None] * len(sums)
    for r in range(1, len(sums)):
        want = sums[r - 1].exit
        if want != ENTRY_UNKNOWN and sums[r].entry != want:
            redo[r] = want
    return redo


def shard_plan(sums: List[ShardSummary]):
    """(first record index, records, last flag) per rank from settled
    summaries: a range after the one where the path ends holds nothing; the
    message's count clips the ranges."""
    n = sums[0].n
    out, first, ended = [], 0, False
    for s in sums:
        if ended or first >= n:
            out.append((min(first, n), 0, False))
            continue
        k = min(s.count, n - first)
        out.append((first, k, False))
        first += k
        if s.exit == ENTRY_UNKNOWN:
            ended = True
    # the range holding the message's end (or the last one that has records)
    last = max((i for i, (_, k, _) in enumerate(out) if k), default=0)
    f, k, _ = out[last]
    out[last] = (f, k, True)
    return out


class DeviceShardBackend:
    """The HIP kernels behind ShardedVectorDecoder (one Codec = one
    workspace: an index and its emit must use the same one)."""

    def __init__(self, codec: Codec):
        self.cd = codec

    def header(self, wire):
        return self.cd.parse_vector_header(bytes(wire[:1024].cpu().numpy()))

    def wire_len(self, wire) -> int:
        return int(wire.numel())

    def index(self, wire, lo, hi, entry) -> ShardSummary:
        return self.cd.shard_index(wire, lo, hi, entry)

    def empty(self, first):
        """The batch and result of a rank that holds no records."""
        cd = self.cd
        out = cd.alloc_batch(1, [1] * len(cd.L.dev.spans))
        return RecordBatch(cd.L, out.recs[:0], out.heaps), C.spk_dresult_t()

    def emit(self, wire, lo, hi, first, last, count, summary):
        cd = self.cd
        out = cd.alloc_batch(count + 1, [max(h, 1) for h in summary.heap[:len(cd.L.dev.spans)]])
        res = cd.shard_emit(out, wire, lo, hi, first, last)
        return RecordBatch(cd.L, out.recs[:count], out.heaps), res


def has_compat(ops) -> bool:
    """A layout with compatible members (SPK_OP_COMPAT / CGROUP ops)."""
    return any((op[0] & 0xFF) in (C.SPK_OP_COMPAT, C.SPK_OP_CGROUP) for op in ops)


def replica_decode(backends, wire, world: int, gather, mine_ranks):
    """Layouts with compatible members: the message is a main pass followed by
    one pass per version (ref:include/ylt/struct_pack/unpacker.hpp:1354-1376),
    record i's members spread over every pass, so a byte range holds no whole
    records; sharding the passes would need an all-to-all of members. Every
    rank decodes the whole message on its GPU (the tile passes) and keeps the
    even share [first, first + k) of the records: its records index the full
    heaps with their global offsets (a valid RecordBatch, no rebasing). The
    verdict is the same on every rank (one gather of the results)."""
    out = []
    for i, r in enumerate(mine_ranks):
        res, full, _ = backends[i].cd.deserialize(wire, C.SPK_MODE_VECTOR)
        n = int(res.count) if res.errc == 0 else 0
        first, last = n * r // world, n * (r + 1) // world
        b = RecordBatch(full.layout, full.recs[first:last], full.heaps)
        res.count = last - first
        out.append((b, first, res))
    verdicts = gather([ShardSummary(int(res.errc), int(res.width), 0, 0, 0, int(res.count),
                                    [0] * C.SPK_MAX_SPANS) for _, _, res in out])
    errc = next((v.errc for v in verdicts if v.errc), 0)
    for _, _, res in out:
        res.errc = errc
    return out


def shard_decode(backends, wire, world: int, gather, rank: Optional[int] = None):
    """The protocol of ShardedVectorDecoder. `backends[r]` runs rank r's
    kernels (one entry when `rank` is given: this process is that rank);
    `gather(list_of_my_summaries) -> all ranks' summaries`. Returns
    [(batch, first, result)] for the ranks this process runs.

    Every rank returns the same verdict: after the emits the ranks exchange
    their results, and the errc of the lowest rank that failed (the range
    holding the message's shortfall reports no_buffer_space / invalid_buffer
    like the reference, unpacker.hpp:1208-1226; a rank out of output capacity
    SPK_ERRC_CAPACITY) is written into every rank's result."""
    mine_ranks = [rank] if rank is not None else list(range(world))
    be0 = backends[0]
    cd0 = getattr(be0, "cd", None)  # (device backends; test backends may have none)
    if cd0 is not None and has_compat(cd0.L.dev.ops):
        return replica_decode(backends, wire, world, gather, mine_ranks), 0
    e, n, w, hl = be0.header(wire)
    if e:
        raise ValueError(f"header errc {e}")
    n_tiles = max(1, (be0.wire_len(wire) - hl + TILE_BYTES - 1) // TILE_BYTES)
    rng = tile_ranges(n_tiles, world)
    local = {r: backends[i].index(wire, rng[r][0], rng[r][1], ENTRY_UNKNOWN)
             for i, r in enumerate(mine_ranks)}
    rounds = 0
    settled = False
    for _ in range(world + 1):
        sums = gather([local[r] for r in mine_ranks])
        redo = settle_entries(sums)
        if not any(x is not None for x in redo):
            settled = True
            break
        rounds += 1
        for i, r in enumerate(mine_ranks):
            if redo[r] is not None:
                local[r] = backends[i].index(wire, rng[r][0], rng[r][1], redo[r])
    if not settled:  # k wrong ranges settle in <= k rounds (range 0 is exact)
        raise RuntimeError(f"sharded decode: range entries did not settle in {world} rounds")
    plan = shard_plan(sums)
    out = []
    for i, r in enumerate(mine_ranks):
        first, k, last = plan[r]
        if k == 0 and not last:
            # a range past the message's end (or past the point where the path
            # ends) holds none of its records: nothing to emit
            b, res = backends[i].empty(first)
        else:
            b, res = backends[i].emit(wire, rng[r][0], rng[r][1], first, last, k, local[r])
        out.append((b, first, res))
    # one verdict on every rank
    verdicts = gather([ShardSummary(int(res.errc), int(res.width), n, 0, 0, int(res.count),
                                    [0] * C.SPK_MAX_SPANS) for _, _, res in out])
    errc = next((v.errc for v in verdicts if v.errc), 0)
    for _, _, res in out:
        res.errc = errc
    return out, rounds


class ShardedVectorDecoder:
    """Decode of one serialize(std::vector<T>) message that every rank holds
    (one GPU per rank): rank r decodes the records that start in its share of
    the body's 16 KiB tiles into rank-local buffers (record 0 = global record
    `first`; heaps from element 0). One all-gather of a ~100-byte summary per
    rank per round (normally one round) is the only collective."""

    def __init__(self, codec: Codec, group=None, backend=None):
        self.be = backend or DeviceShardBackend(codec)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.rounds = 0

    def _gather(self, mine: List[ShardSummary]) -> List[ShardSummary]:
        v = mine[0].as_list()
        t = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in v], dtype=torch.int64)
        if dist.get_backend(self.group) != "gloo":
            t = t.to(self.be.cd.device)
        outs = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(outs, t, group=self.group)
        return [ShardSummary.from_list([x & ((1 << 64) - 1) for x in o.tolist()]) for o in outs]

    def decode(self, wire):
        """Returns (RecordBatch of this rank's records, first, result)."""
        out, self.rounds = shard_decode([self.be], wire, self.world, self._gather, self.rank)
        return out[0]
