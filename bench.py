#!/usr/bin/env python3
"""bench.py — struct_pack encode+decode throughput on MI355X (device-resident).

A "step" = one serialize + one deserialize of this rank's whole record batch
through the C ABI (spk_plan + spk_encode + spk_decode), inputs already in HBM.
Default workload (BASELINE.json configs[1], "C2"): 100M 64-byte Rec64 records
per GPU as one struct_pack message, serialize(std::vector<Rec64>) and
deserialize_to back. Multi-GPU: each rank owns an independent 100M-record
shard (record-range partition, no data-path collective) => weak scaling; the
RCCL concatenation of one message sharded over the ranks is timed after the
headline as `concat` (not part of `value`).

value = algorithmic bytes of all ranks / max-over-ranks wall time, in GiB/s:
  per record: encode reads the record and writes its wire bytes, decode reads
  the wire bytes and writes the record: 4 x 64 B for C2.

At N=1 the same line carries `extra.configs`: the other BASELINE configs
(C2 mode B, C3, C4, C5) and the varint config, each timed the same way, with
per-kernel times (HIP events around every codec launch, spk_trace_*), the
dominant kernel's roofline and the reference CPU baseline on the same N.

At N>1 the line carries the sharded BASELINE configs as `extra.configs`
too: C4 (10M Outer per rank) and C5 (1M request frames per rank), each
rank its own batch (weak scaling, value = all ranks' bytes / max time).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2b|c3|c4|c5|cv|cm]
`--gpus N` alone launches the N ranks (torch.distributed.run, 127.0.0.1);
under a launcher, WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (case, records per GPU, param, mode, description)
    "c2": ("rec64", 100_000_000, 0, "A",
           "C2: 100M x 64-byte Rec64{int32 x4, float x4, double x4} per GPU, "
           "serialize(vector<Rec64>) + deserialize_to"),
    "c2b": ("rec64", 100_000_000, 0, "B",
            "C2 mode B: 100M independent 68-byte Rec64 messages per GPU (coro_rpc payload shape)"),
    "c3": ("recs", 10_000_000, 48, "A",
           "C3: 10M RecS{int32, std::string len U[0,48], double} per GPU, one vector message"),
    "c3r": ("recs", 10_000_000, 48 | 1 << 31, "A",
            "C3 with binary strings: 10M RecS{int32, std::string of random bytes len U[0,48], "
            "double} per GPU, one vector message"),
    "c3l": ("recs", 2_000_000, 3000 | 100 << 16 | 1 << 31, "A",
            "C3 with long binary strings: 2M RecS{int32, std::string of random bytes len "
            "U[100,3000], double} per GPU, one vector message"),
    "c4": ("outer", 10_000_000, 16, "A",
           "C4: 10M Outer{int64, vector<Inner{int32,float}> n U[0,16]} per GPU, one vector message"),
    "cv": ("var", 10_000_000, 16, "A",
           "varint records: 10M Var{var_int32_t, std::string len U[0,16], var_uint64_t, double, "
           "var_int64_t, var_uint32_t} per GPU (LEB128 lengths 1-10 B), one vector message"),
    "cvm": ("valreq", 1_000_000, 16, "B",
            "coro_rpc benchmark's ValidateRequest (src/coro_rpc/benchmark/api/ValidateRequest.h): "
            "1M independent messages per GPU (nested: optional, vector<string>)"),
    "cm": ("monster", 10_000_000, 20, "A",
           "the reference benchmark's Monster (src/struct_pack/benchmark/data_def.hpp: Vec3, "
           "2 x int16, 2 strings, enum, vector<Weapon{string,int16}>, Weapon, vector<Vec3>): "
           "10M per GPU, one vector message"),
    "cmpg": ("cmpg", 2_000_000, 16, "A",
             "compatible members: 2M CmpG{int32, compatible<string, v1>, string, "
             "compatible<vector<int32>, v1>, compatible<Inner, v2>, compatible<ResponseCode, v2>} "
             "per GPU, one vector message (a main pass and two version passes)"),
}
EXTRA = ["c2b", "c3", "c3r", "c3l", "c4", "c5", "cv", "cm", "cvm", "cmpg"]  # timed beside the C2 headline at N=1
SEEDS = {"rec64": 0x5EED0002, "recs": 0x5EED0003, "outer": 0x5EED0004, "var": 0x5EED000C,
         "monster": 0x5EED001E, "valreq": 0x5EED001B, "cmpg": 0x5EED0021}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROFILE_ROUND = "r06"

C5_TYPES = [  # (case, share of messages, param, rpc function name) — coro_rpc bench shapes
    ("rpcrect", 1, 0, "echo_rect"),          # rect{point p1, p2}   (api/Rect.h)
    ("person", 1, 48, "echo_person"),        # person{id, name, age, salary}
    ("ints", 1, 2000, "array_1K_int"),       # std::vector<int>, ~1K elements (data_gen.cpp:61)
]
C5_SEEDS = {"rpcrect": 0x5EED0007, "person": 0x5EED0008, "ints": 0x5EED0009}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + ["c5"])
    ap.add_argument("--records", type=int, default=0, help="override records per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="headline config only (no extra.configs at N=1)")
    ap.add_argument("--extra-steps", type=int, default=10)
    ap.add_argument("--settle", type=float, default=1.0,
                    help="seconds of untimed steps before the warmup (GPU clock ramp)")
    ap.add_argument("--host-path", action="store_true",
                    help="time H2D + encode + decode + D2H from pinned host buffers for every "
                         "config (the default run times it for C2 and C5 only)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-inclusive (PCIe) timings of the default run")
    ap.add_argument("--full-line", action="store_true",
                    help="print the full detail object as the stdout line (A/B scripts); the "
                         "default line is compact and the detail goes to --detail-out")
    ap.add_argument("--detail-out", default="",
                    help="file for the full detail JSON (default gpurun_out/bench_detail_<cfg>"
                         "_n<N>.json)")
    ap.add_argument("--pmc-dir", default="", help="directory of pmc_<config>.json summaries")
    ap.add_argument("--no-concat", action="store_true",
                    help="N>1: skip the one-message concatenation timing (concat_*)")
    ap.add_argument("--concat-records", type=int, default=8_000_000,
                    help="N>1: Rec64 records per rank of the one-message concatenation")
    ap.add_argument("--no-shard-extra", action="store_true",
                    help="N>1: skip the per-rank C4 / C5 weak-scaling entries")
    ap.add_argument("--spawn-probe", action="store_true",
                    help="(test of the launcher) each rank prints RANK/WORLD_SIZE and exits "
                         "before touching torch")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# N ranks from one command: `python bench.py --gpus N` without a launcher
# starts N fresh rank processes through torch.distributed.run and exits with
# their status. The parent never touches a GPU (no torch import), so nothing
# that initialised the GPU is ever replaced or forked.
# ---------------------------------------------------------------------------
def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(gpus, argv, port):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1", "--master-port",
            str(port), os.path.abspath(__file__)] + list(argv)


def spawn_ranks(gpus, argv):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL
    print(f"[bench] launching {gpus} ranks (torch.distributed.run)", file=sys.stderr, flush=True)
    return subprocess.call(launcher_cmd(gpus, argv, free_port()), env=env)


def check_world(gpus, world):
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} "
                         f"ranks; run `python bench.py --gpus {gpus}` (it launches the ranks) "
                         f"or pass --gpus equal to --nproc-per-node")


# ---------------------------------------------------------------------------
# CPU baseline: the reference struct_pack (oracle/_ref/ref_bench, built from
# the unmodified reference headers) on this box's host cores
# ---------------------------------------------------------------------------
def cpu_share():
    """Threads = the lease's CPU share: OMP_NUM_THREADS when the pool sets it
    (16 per GPU), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        share = 0
    return max(1, min(aff, share) if share > 0 else aff), aff


def cpu_quota():
    """The cgroup CPU quota (cgroup v2 cpu.max, in CPUs), or None: the box
    reports nproc / affinity of the whole machine, but its lease is a share."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(case, n, param, algo_bytes, per="record"):
    """Reference CPU serialize+deserialize of the SAME n as the GPU leg on the
    host cores this process may use (the lease's share: the pool sizes worker
    pools to it, and its cgroup quota bounds them), median of 5 timed runs
    after a warmup, plus one thread on n/10."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    if not os.path.exists(exe):
        return None
    threads, aff = cpu_share()
    seed = {"c5": 0, "rec64msg": SEEDS["rec64"], "valreqmsg": SEEDS["valreq"]}.get(
        case, SEEDS.get(case, 0))

    def run(nn, t, reps):
        r = subprocess.run([exe, case, str(nn), str(seed), str(param), str(t), str(reps)],
                           capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            return None
        return json.loads(r.stdout.strip().splitlines()[-1])

    full = run(n, threads, 5)
    one = run(max(n // 10, 1), 1, 3)
    if not full:
        return None
    per_unit = algo_bytes / n
    med = full["median_encode_s"] + full["median_decode_s"]
    best = full["encode_s"] + full["decode_s"]
    mean = full["mean_encode_s"] + full["mean_decode_s"]
    out = {"value": round(per_unit * n / med / 2**30, 3), "unit": "GiB/s", "cores": threads,
           "kind": "reference",
           "sample": (f"{n} {case} {per}s (same N as the GPU leg), reference struct_pack "
                      f"serialize_to + deserialize_to (-O3 -DNDEBUG -DSTRUCT_PACK_OPTIMIZE), "
                      f"{threads} threads x contiguous slices, median of 5 after a warmup"),
           "best_gib_s": round(per_unit * n / best / 2**30, 3),
           "mean_gib_s": round(per_unit * n / mean / 2**30, 3),
           f"m{per[:3]}_per_s": round(n / med / 1e6, 3),
           "encode_s": full["median_encode_s"], "decode_s": full["median_decode_s"],
           "host": {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity": aff,
                    "cgroup_cpu_quota": cpu_quota(), "threads_used": threads}}
    # (no run at the whole affinity mask: the box reports 256 CPUs under a
    # 16-CPU cgroup quota, so such a run only measures oversubscription)
    if one:
        out["single_thread_gib_s"] = round(
            per_unit * one["n"] / (one["median_encode_s"] + one["median_decode_s"]) / 2**30, 3)
        out["single_thread_sample"] = f"{one['n']} {per}s, 1 thread, median of 3"
    return out


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
class VecWorkload:
    """One config of CONFIGS: plan + encode + decode of this rank's batch."""

    def __init__(self, torch, cfg, n, rank, dev):
        from yalantinglibs_amd import layout as LY
        from yalantinglibs_amd import struct_pack as SP
        self.torch, self.SP, self.dev = torch, SP, dev
        self.cfg = cfg
        case, n0, param, modech, desc = CONFIGS[cfg]
        self.case, self.param, self.desc = case, param, desc
        self.n = n or n0
        self.mode = SP.MODE_VECTOR if modech == "A" else SP.MODE_MESSAGES
        self.cd = cd = SP.Codec(LY.case_layout(case), device=dev)
        n = self.n
        # this rank's shard: global records [rank*n, (rank+1)*n)
        if case in ("rec64", "recs", "outer", "monster"):
            self.batch = SP.synth_batch(cd, case, n, SEEDS[case], param, first=rank * n)
            self.data = f"spk_synth seeded {case}, seed {SEEDS[case]:#x}"
        else:  # host generator (yalantinglibs_amd/synth.py), uploaded before timing
            import numpy as np
            from yalantinglibs_amd import synth as SY
            _, recs_np, heaps_np = SY.make_batch(case, n, SEEDS[case], param)
            self.batch = SP.RecordBatch(
                cd.L, torch.from_numpy(recs_np.view(np.uint8).reshape(n, cd.L.stride)).to(dev),
                [torch.from_numpy(np.ascontiguousarray(h).view(np.uint8).reshape(-1)).to(dev)
                 for h in heaps_np])
            self.data = f"host synth.py seeded {case}, seed {SEEDS[case]:#x}"
        self.plan = cd.get_needed_size(self.batch, self.mode)
        self.wire = torch.empty(self.plan.total_bytes + 64, dtype=torch.uint8, device=dev)
        self.offs = (torch.empty(n + 1, dtype=torch.int64, device=dev)
                     if self.mode == SP.MODE_MESSAGES else None)
        elems = [int(h.numel()) // sp.elem.size for h, sp in zip(self.batch.heaps, cd.L.dev.spans)]
        self.dec = cd.alloc_batch(n, elems)
        self.rec_bytes = self.batch.recs.numel() + sum(int(h.numel()) for h in self.batch.heaps)
        self.wire_bytes = self.plan.total_bytes
        self.algo_bytes = 2 * self.rec_bytes + 2 * self.wire_bytes  # enc in/out + dec in/out
        self.units = n

    def phases(self):
        return ("plan", "encode", "decode")

    def step(self, stream, marks=None):
        SP = self.SP
        if marks is not None:
            marks[0].record(stream)
        self.cd.plan(self.batch, self.mode, stream)
        if marks is not None:
            marks[1].record(stream)
        self.cd.serialize_to(self.wire, self.batch, self.mode, self.offs, stream=stream,
                             planned=True)
        if marks is not None:
            marks[2].record(stream)
        self.cd.deserialize_to(self.dec, self.wire[:self.plan.total_bytes], self.mode, self.offs,
                               self.n if self.mode == SP.MODE_MESSAGES else 0, stream=stream)
        if marks is not None:
            marks[3].record(stream)

    def check(self):
        """Round trip must be exact: records AND every heap byte in use."""
        torch = self.torch
        res = self.cd.result()
        if res.errc != 0 or res.count != self.n or not torch.equal(self.dec.recs, self.batch.recs):
            return f"records (errc {res.errc}, count {res.count})"
        for k, (h_in, h_out) in enumerate(zip(self.batch.heaps, self.dec.heaps)):
            used = int(res.heap_used[k]) * self.cd.L.dev.spans[k].elem.size
            if used != h_in.numel() or not torch.equal(h_out[:used], h_in[:used]):
                return f"heap {k}"
        return None

    def kernel_bytes(self):
        """Algorithmic bytes per step of the byte-moving kernels (SURVEY.md
        §8d per-unit figures x units per launch); scratch-only kernels
        (plan reductions, scans, tile selection) carry none."""
        rb, wb = self.rec_bytes, self.wire_bytes
        if self.mode == self.SP.MODE_VECTOR:
            if self.cd.L.dev.trivial:  # one shift_copy per phase: records <-> body
                return {"shift_copy_kernel": 4 * rb}
            if any(op[0] & 0xFF in (5, 7, 8, 9, 10, 11) for op in self.cd.L.dev.ops):
                # nested layouts: the encode's window pass writes each record's
                # bytes; the decode is the tile pipeline with the nested walker
                # (K1 reads the wire, K4 reads it again and writes records +
                # element records + heaps); the chunked interpreter's kernels
                # for layouts the tile decoder does not take
                return {"nest_write_win": rb + wb, "nest_write": rb + wb,
                        "vec_tile_emit": wb + rb, "vec_tile_spec": wb,
                        "nest_cemit": wb + rb, "nest_cspec": wb}
            # wait-free tile decoder: K1 reads the wire once, K4 reads it again
            # and writes the records + heaps
            return {"var_encode_write": rb + wb, "vec_tile_emit": wb + rb,
                    "vec_tile_spec": wb}
        ob = 8 * (self.n + 1)
        if self.cd.L.dev.trivial:
            return {"fixed_msg_encode_lds": rb + wb + ob, "fixed_msg_decode_lds": wb + ob + rb}
        if any(op[0] & 0xFF in (5, 7, 8, 9, 10, 11) for op in self.cd.L.dev.ops):
            # nested layouts: one lane per message in both directions
            return {"nest_write": rb + wb + ob, "nest_emit": wb + ob + rb}
        return {"var_encode_write": rb + wb + ob, "var_msg_write": wb + ob + rb}

    def config(self):
        SP = self.SP
        return {"workload": self.desc, "records_per_gpu": self.n,
                "mode": "vector" if self.mode == SP.MODE_VECTOR else "messages",
                "wire_bytes_per_gpu": self.wire_bytes, "record_bytes_per_gpu": self.rec_bytes,
                "algorithmic_bytes_per_step_per_gpu": self.algo_bytes}

    def cpu_case(self):
        if self.mode == self.SP.MODE_MESSAGES:
            return {"rec64": "rec64msg", "valreq": "valreqmsg"}.get(self.case)
        return self.case


class C5Workload:
    """C5: a coro_rpc server step over one batch of request frames of three
    record types whose function ids arrive interleaved (seeded order, each
    type's own order kept): route the frames by function id (spk_route_frames,
    the handler lookup of router.hpp:226-240 for the whole batch), read the
    per-type counts, decode each type's [req_header][args] frames where they
    lie (spk_decode_frames), echo, encode each type's [resp_header][ret]
    frames carrying every request's seq_num (spk_encode_framed_echo)."""

    def __init__(self, torch, n_total, rank, dev):
        import numpy as np
        from yalantinglibs_amd import coro_rpc as RPC
        from yalantinglibs_amd import layout as LY
        from yalantinglibs_amd import struct_pack as SP
        self.torch, self.SP, self.RPC, self.dev = torch, SP, RPC, dev
        self.cfg = "c5"
        n_total = n_total or 1_000_000
        shares = sum(s for _, s, _, _ in C5_TYPES)
        self.groups = []
        host_frames = []
        for case, share, param, fname in C5_TYPES:
            n = n_total * share // shares
            cd = SP.Codec(LY.case_layout(case), device=dev)
            src = SP.synth_batch(cd, case, n, C5_SEEDS[case], param, first=rank * n)
            plan = cd.get_needed_size(src, SP.MODE_MESSAGES)
            fid = RPC.func_id(fname)
            rq = RPC.req_frame(fid, seq_base=rank * n)
            rs = RPC.resp_frame(seq_base=0)  # seq_num copied from the requests
            req_len = plan.total_bytes + n * rq.prefix_len
            req = torch.empty(req_len + 64, dtype=torch.uint8, device=dev)
            req_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
            cd.serialize_to(req, src, SP.MODE_MESSAGES, req_offs, planned=True, frame=rq)
            host_frames.append((req[:req_len].cpu().numpy(), req_offs.cpu().numpy()))
            del req, req_offs
            elems = [int(h.numel()) // sp.elem.size for h, sp in zip(src.heaps, cd.L.dev.spans)]
            args_b = cd.alloc_batch(n, elems)
            resp_len = plan.total_bytes + n * rs.prefix_len
            resp = torch.empty(resp_len + 64, dtype=torch.uint8, device=dev)
            resp_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
            rec_bytes = src.recs.numel() + sum(int(h.numel()) for h in src.heaps)
            self.groups.append(dict(case=case, n=n, cd=cd, src=src, fid=fid, args=args_b,
                                    resp=resp, resp_offs=resp_offs, rq=rq, rs=rs,
                                    rec_bytes=rec_bytes, req_len=req_len, resp_len=resp_len))
        # the connection's byte stream: frames of all types in a seeded arrival order
        rng = np.random.default_rng(0x5EED000C5 + rank)
        tags = np.concatenate([np.full(g["n"], k, np.int8) for k, g in enumerate(self.groups)])
        rng.shuffle(tags)
        nxt = [0] * len(self.groups)
        lens = np.empty(len(tags), np.int64)
        for k, (_, offs) in enumerate(host_frames):
            lens[tags == k] = np.diff(offs)
        moffs = np.zeros(len(tags) + 1, np.int64)
        moffs[1:] = np.cumsum(lens)
        buf = np.empty(int(moffs[-1]), np.uint8)
        for j, k in enumerate(tags.tolist()):
            w, offs = host_frames[k]
            i = nxt[k]
            nxt[k] = i + 1
            buf[moffs[j]:moffs[j + 1]] = w[offs[i]:offs[i + 1]]
        del host_frames
        self.nframes = len(tags)
        self.wire = torch.from_numpy(buf).to(dev)
        self.offs = torch.from_numpy(moffs).to(dev)
        del buf
        self.router = RPC.FrameRouter([g["fid"] for g in self.groups], self.nframes, device=dev)
        self.counts_pinned = torch.empty(len(self.groups) + 1, dtype=torch.int64).pin_memory()
        self.sync = False
        # request frames in + records/heaps out (decode), records/heaps in +
        # response frames out (encode)
        self.algo_bytes = sum(g["req_len"] + 2 * g["rec_bytes"] + g["resp_len"] for g in self.groups)
        self.units = sum(g["n"] for g in self.groups)
        self.n = self.units
        self.data = "spk_synth seeded rpcrect/person/ints, frames interleaved in a seeded order"

    def phases(self):
        return ("route", "decode", "encode")

    def step(self, stream, marks=None):
        """sync=False (default): each type's decode and response encode take
        its frame count from the router's device counts (spk_decode_frames_dn,
        spk_plan_dn, spk_encode_framed_echo_dn), so the step is one
        stream-ordered sequence with no host read-back; sync=True: the host
        reads the counts after routing (one stream.synchronize per step)."""
        RPC = self.RPC
        if marks is not None:
            marks[0].record(stream)
        rt = self.router
        rt.route(self.wire, self.offs, self.nframes, stream=stream)
        counts = None
        if self.sync:
            self.counts_pinned.copy_(rt.counts, non_blocking=True)
            stream.synchronize()  # the per-type counts size the decode launches
            counts = self.counts_pinned.tolist()
        if marks is not None:
            marks[1].record(stream)
        for k, g in enumerate(self.groups):
            if counts is not None:
                g["cd"].deserialize_frames(g["args"], self.wire, rt.begins[k], rt.ends[k],
                                           int(counts[k]), g["rq"].prefix_len, stream=stream)
            else:  # capacity g["n"]: this type's buffers; the count stays on the device
                g["cd"].deserialize_frames(g["args"], self.wire, rt.begins[k], rt.ends[k],
                                           g["n"], g["rq"].prefix_len, stream=stream,
                                           d_count=rt.counts[k:k + 1])
        if marks is not None:
            marks[2].record(stream)
        for k, g in enumerate(self.groups):
            # responses carry their requests' seq_num (spk_encode_framed_echo)
            g["cd"].serialize_echo(g["resp"], g["args"], g["resp_offs"], g["rs"], self.wire,
                                   rt.begins[k], RPC.REQ_SEQ_OFF, stream=stream,
                                   d_count=None if counts is not None else rt.counts[k:k + 1])
        if marks is not None:
            marks[3].record(stream)

    def check(self):
        torch = self.torch
        counts = self.router.counts_host()
        for k, g in enumerate(self.groups):
            r = g["cd"].result()
            if (r.errc != 0 or r.count != g["n"] or counts[k] != g["n"]
                    or not torch.equal(g["args"].recs, g["src"].recs)
                    or int(g["resp_offs"][-1].item()) != g["resp_len"]):
                return f"c5 {g['case']}"
            for q, (h_in, h_out) in enumerate(zip(g["src"].heaps, g["args"].heaps)):
                used = int(r.heap_used[q]) * g["cd"].L.dev.spans[q].elem.size
                if not torch.equal(h_out[:used], h_in[:used]):
                    return f"c5 {g['case']} heap {q}"
            # response j echoes request j's seq_num (the request's rank*n + j)
            ro = g["resp_offs"][:-1]
            seq = torch.stack([g["resp"][ro + self.RPC.RESP_SEQ_OFF + b].to(torch.int64) << (8 * b)
                               for b in range(4)]).sum(0)
            if not torch.equal(seq, torch.arange(g["n"], device=seq.device) + g["rq"].seq_base):
                return f"c5 {g['case']} seq_num"
        if self.router.counts_host()[-1] != 0:
            return "c5 unrouted frames"
        return None

    def kernel_bytes(self):
        kb = {}

        def add(k, v):
            kb[k] = kb.get(k, 0) + v
        for g in self.groups:
            ob = 8 * (g["n"] + 1)
            if g["cd"].L.dev.trivial:
                add("fixed_msg_decode_lds", g["req_len"] + 2 * ob + g["rec_bytes"])
                add("fixed_msg_encode_lds", g["rec_bytes"] + g["resp_len"] + ob)
            else:
                add("var_msg_write", g["req_len"] + 2 * ob + g["rec_bytes"])
                add("var_encode_write", g["rec_bytes"] + g["resp_len"] + ob)
        # routing: frame offsets and keys in, begins / ends / arrival index out
        add("route_scatter", 8 * (self.nframes + 1) + self.nframes + 24 * self.nframes)
        return kb

    def config(self):
        return {"workload": "C5: coro_rpc server step, %d framed requests per GPU in arrival "
                            "order (rect / person / vector<int>~1K interleaved): route by "
                            "function id, decode [req_header][args] per type, encode "
                            "[resp_header][ret] with the request's seq_num" % self.units,
                "messages_per_gpu": self.units,
                "per_type": {g["case"]: g["n"] for g in self.groups},
                "algorithmic_bytes_per_step_per_gpu": self.algo_bytes}

    def cpu_case(self):
        return "c5"

    def host_path(self, torch, dev, reps=3):
        """C5 with the coro_rpc socket buffers in host memory: the
        connection's request bytes and frame offsets H2D from pinned buffers,
        route + decode + encode as in the device step, then every type's
        response frames and offsets D2H into pinned buffers. Serial, one
        stream; the per-type counts stay on the device as in the step."""
        stream = torch.cuda.current_stream(dev)
        h_wire = torch.empty_like(self.wire, device="cpu").pin_memory()
        h_wire.copy_(self.wire)
        h_offs = torch.empty_like(self.offs, device="cpu").pin_memory()
        h_offs.copy_(self.offs)
        h_resp = [torch.empty(g["resp_len"], dtype=torch.uint8).pin_memory() for g in self.groups]
        h_roff = [torch.empty_like(g["resp_offs"], device="cpu").pin_memory() for g in self.groups]
        torch.cuda.synchronize(dev)

        def one():
            self.wire.copy_(h_wire, non_blocking=True)
            self.offs.copy_(h_offs, non_blocking=True)
            self.step(stream)
            for g, hr, ho in zip(self.groups, h_resp, h_roff):
                hr.copy_(g["resp"][:g["resp_len"]], non_blocking=True)
                ho.copy_(g["resp_offs"], non_blocking=True)
        one()
        torch.cuda.synchronize(dev)
        bad = self.check()
        t0 = time.perf_counter()
        for _ in range(reps):
            one()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        moved = int(self.wire.numel()) + 8 * int(self.offs.numel()) + sum(
            g["resp_len"] + 8 * (g["n"] + 1) for g in self.groups)
        return {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(self.algo_bytes / dt / 2**30, 3),
                "pcie_bytes": moved, "check": bad or "ok",
                "note": "serial: H2D of the request stream + frame offsets (pinned), route, "
                        "decode per type, encode the echo responses, D2H of every type's "
                        "response frames + offsets (pinned); gib_s uses the device step's "
                        "algorithmic bytes"}


# ---------------------------------------------------------------------------
# timing
# ---------------------------------------------------------------------------
def pmc_traffic(cfg, pmc_dir):
    """PMC HBM bytes per launch per kernel from a rocprofv3 --pmc summary of
    this command (scripts/gpu_pmc.sh -> profiles/<round>/pmc_<config>.json)."""
    for d in ([pmc_dir] if pmc_dir else []) + [os.path.join(ROOT, "profiles", PROFILE_ROUND)]:
        p = os.path.join(d, f"pmc_{cfg}.json")
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f), os.path.relpath(p, ROOT)
    return {}, None


class ConfigFailed(RuntimeError):
    """A config failed on at least one rank; raised on EVERY rank (after the
    ranks agreed on it), so no rank is left waiting in a collective."""

    def __init__(self, msg, code=1):
        super().__init__(msg)
        self.code = code


def agree_ok(ok, torch, dist, world, dev):
    """True iff every rank passed `ok` (MIN over ranks; trivially ok at N=1).
    Every rank must call it at the same point: it is itself a collective."""
    if world <= 1:
        return bool(ok)
    on = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def measure(wl, args, torch, dist, world, dev, steps, warmup, settle):
    """Gate, settle, warmup, K timed steps (barrier + sync on both sides,
    max over ranks), then instrumented steps: phase events + per-kernel
    hipEvents (spk_trace) on the launch stream."""
    from yalantinglibs_amd import _capi as C
    stream = torch.cuda.current_stream(dev)
    bad = None
    try:
        wl.step(stream)
        torch.cuda.synchronize(dev)
        diag = os.environ.get("SPK_TILE_DBG", "0") not in ("", "0")  # (diagnostics builds)
        bad = None if diag else wl.check()  # diagnostics runs (wrong output by design): no gate
    except Exception as e:  # a local fault: report it, then fail on every rank together
        bad = f"{type(e).__name__}: {e}"
    if bad:
        print(json.dumps({"error": "round trip mismatch", "config": wl.cfg, "what": bad}),
              flush=True)
    if not agree_ok(not bad, torch, dist, world, dev):
        raise ConfigFailed(f"{wl.cfg}: first step failed on "
                           f"{'this rank' if bad else 'another rank'}", code=3)
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < settle:
        wl.step(stream)
        torch.cuda.synchronize(dev)
    for _ in range(warmup):
        wl.step(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        wl.step(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # instrumented steps (outside the timed region)
    n_inst = max(3, min(steps, 10))
    names = wl.phases()
    acc = [0.0] * len(names)
    C.trace_reset()
    C.trace_enable(True)
    try:
        for _ in range(n_inst):
            marks = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
            wl.step(stream, marks)
            torch.cuda.synchronize(dev)
            for i in range(len(names)):
                acc[i] += marks[i].elapsed_time(marks[i + 1])
        trace = C.trace_read()
    finally:
        C.trace_enable(False)
    phase_ms = {k: round(v / n_inst, 4) for k, v in zip(names, acc)}
    kernels = {k: {"launches_per_step": round(l / n_inst, 3), "ms_per_launch": round(ms / l, 5),
                   "ms_per_step": round(ms / n_inst, 5)} for k, (l, ms) in trace.items() if l}
    return dt, phase_ms, kernels


def _kbase(name):
    """A traced kernel's base name: "vec_tile_emit<NS>" and "(nest_emit<D, LU>)"
    (a template launched through SPK_LAUNCH in parentheses) -> the plain name."""
    return name.strip("() ").split("<")[0]


def roofline(wl, kernels, pmc, pmc_src):
    """Roofline of the dominant byte-moving kernel: algorithmic bytes per
    launch / average launch duration (HIP events), against the 8 TB/s HBM
    peak; `traffic` = PMC HBM bytes per launch of the same kernel."""
    kb = wl.kernel_bytes()
    for name, k in kernels.items():
        base = _kbase(name)
        if base in kb:
            k["bytes_per_step"] = kb[base]
            k["achieved_gbs"] = round(kb[base] / (k["ms_per_step"] * 1e-3) / 1e9, 1)
            k["frac"] = round(k["achieved_gbs"] / HBM_PEAK_GBS, 4)
    cand = [(k["ms_per_step"], name) for name, k in kernels.items() if "bytes_per_step" in k]
    if not cand:
        return None
    _, dom = max(cand)
    k = kernels[dom]
    launches = k["launches_per_step"]
    bpl = k["bytes_per_step"] / launches
    traffic = None
    for kname, v in pmc.items():
        if kname.split("(")[0].split("<")[0].replace("void ", "").replace("spk::", "") == \
                _kbase(dom):
            traffic = v.get("hbm_bytes_per_launch")
    return {"bound": "hbm", "kernel": dom, "launches_per_step": launches,
            "bytes_per_launch": int(bpl), "ms_per_launch": k["ms_per_launch"],
            "achieved": k["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": k["frac"], "traffic": traffic,
            "traffic_ratio": round(traffic / bpl, 3) if traffic else None,
            "traffic_source": pmc_src if traffic else None}


def run_config(cfg, args, torch, dist, world, rank, dev, steps, warmup, settle, cpu):
    n = args.records if cfg == args.config else 0
    wl, err = None, None
    try:  # build on every rank, then agree before the first collective
        wl = C5Workload(torch, n, rank, dev) if cfg == "c5" else VecWorkload(torch, cfg, n, rank,
                                                                             dev)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
        print(f"[bench] rank {rank}: {cfg} workload build failed: {err}", file=sys.stderr,
              flush=True)
    if not agree_ok(err is None, torch, dist, world, dev):
        wl = None
        torch.cuda.empty_cache()
        raise ConfigFailed(f"{cfg}: workload build failed on "
                           f"{'this rank: ' + err if err else 'another rank'}")
    dt, phase_ms, kernels = measure(wl, args, torch, dist, world, dev, steps, warmup, settle)
    ms_step = dt * 1e3 / steps
    sync_variant = None
    if cfg == "c5":  # the same step with the host reading the route counts
        wl.sync = True
        dts, _, _ = measure(wl, args, torch, dist, world, dev, steps, warmup, settle)
        wl.sync = False
        sync_variant = {"ms_per_step": round(dts * 1e3 / steps, 4),
                        "note": "host reads the per-type route counts before the decodes "
                                "(one stream.synchronize per step); the headline step "
                                "keeps them on the device (spk_*_dn)"}
    value = wl.algo_bytes * world * steps / dt / 2**30
    pmc, pmc_src = pmc_traffic(cfg, args.pmc_dir)
    out = {"config": cfg, "value": round(value, 3), "unit": "GiB/s", "steps": steps,
           "ms_per_step": round(ms_step, 4),
           ("mmsg_per_s" if cfg == "c5" else "mrec_per_s"):
               round(wl.units * world * steps / dt / 1e6, 3),
           "phase_ms": phase_ms, "kernels": kernels,
           "roofline": roofline(wl, kernels, pmc, pmc_src),
           "step_frac": round(wl.algo_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "detail": wl.config(), "data": wl.data}
    if sync_variant:
        out["with_host_sync"] = sync_variant
    host = None
    want_host = (args.host_path or (cfg in ("c2", "c5") and not args.no_host_path)) \
        and world == 1
    if want_host and rank == 0:
        host = wl.host_path(torch, dev) if cfg == "c5" else host_path(wl, torch, dev)
    if host:
        out["host_path"] = host
        try:
            hp = None if cfg == "c5" else host_path_pipelined(wl, torch, dev)
        except Exception as e:  # never lose the line
            hp = {"error": f"{type(e).__name__}: {e}"}
        if hp:
            out["host_path_pipelined"] = hp
    out["cpu_baseline"] = None
    if cpu and rank == 0 and world == 1 and not args.no_cpu_baseline and wl.cpu_case():
        out["cpu_baseline"] = cpu_baseline(wl.cpu_case(), wl.units,
                                           getattr(wl, "param", 0), wl.algo_bytes,
                                           "message" if cfg == "c5" else "record")
    del wl
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return out


def host_path(wl, torch, dev):
    """PCIe-inclusive rate: pinned host records (+ heaps) -> H2D -> encode ->
    D2H wire; pinned host wire -> H2D -> decode -> D2H records (+ heaps)
    (DESIGN.md). The coro_rpc socket buffers this models live in host memory."""
    SP = wl.SP
    stream = torch.cuda.current_stream(dev)
    srcs = [wl.batch.recs] + list(wl.batch.heaps)
    dsts = [wl.dec.recs] + list(wl.dec.heaps)
    h_in = [torch.empty_like(t, device="cpu").pin_memory() for t in srcs]
    for h, t in zip(h_in, srcs):
        h.copy_(t)
    total = wl.plan.total_bytes
    h_wire = torch.empty(total, dtype=torch.uint8).pin_memory()
    h_out = [torch.empty_like(t, device="cpu").pin_memory() for t in dsts]
    torch.cuda.synchronize(dev)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        for t, h in zip(srcs, h_in):
            t.copy_(h, non_blocking=True)
        wl.cd.plan(wl.batch, wl.mode, stream)
        wl.cd.serialize_to(wl.wire, wl.batch, wl.mode, wl.offs, stream=stream, planned=True)
        h_wire.copy_(wl.wire[:total], non_blocking=True)
        wl.wire[:total].copy_(h_wire, non_blocking=True)
        wl.cd.deserialize_to(wl.dec, wl.wire[:total], wl.mode, wl.offs,
                             wl.n if wl.mode == SP.MODE_MESSAGES else 0, stream=stream)
        for t, h in zip(dsts, h_out):
            h.copy_(t, non_blocking=True)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(wl.algo_bytes / dt / 2**30, 3),
            "note": "serial: H2D of records (+heaps), encode, D2H of wire, H2D of wire, decode, "
                    "D2H of decoded records (+heaps); pinned host buffers, one stream"}


def concat_bench(torch, dist, world, rank, dev, n, reps=3):
    """N>1 only: ONE serialize(vector<Rec64>) message over the records of all
    ranks (yalantinglibs_amd/parallel.py ShardedVectorEncoder), the data-path
    collective the weak-scaling headline does not have. Times, max over ranks,
    best of `reps`: the plan agreement (all-reduce SUM/MAX + all-gather of body
    sizes), each rank's body encode, and three concatenations of the bodies —
    P2P gather into rank 0's message buffer (grouped RCCL send/recv over
    xGMI), all-gather (every rank gets the whole message), and each rank's D2H
    of its body into pinned host memory (the coro_rpc destination). Checked
    once: rank 0 decodes the gathered message and compares it with the global
    synthetic batch."""
    from yalantinglibs_amd import layout as LY
    from yalantinglibs_amd import parallel as PAR
    from yalantinglibs_amd import struct_pack as SP
    err = None
    try:  # local setup on every rank, agreed on before the first collective
        cd = SP.Codec(LY.case_layout("rec64"), device=dev)
        batch = SP.synth_batch(cd, "rec64", n, SEEDS["rec64"], 0, first=rank * n)
        enc = PAR.ShardedVectorEncoder(cd)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    if not agree_ok(err is None, torch, dist, world, dev):
        raise ConfigFailed(f"concat: setup failed on {'this rank: ' + err if err else 'another rank'}")
    red_dev = torch.device("cpu") if dist.get_backend() == "gloo" else dev

    def timed(fn):
        best = None
        for i in range(reps + 1):
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            if i:  # the first run is a warmup
                best = dt.item() if best is None else min(best, dt.item())
        return best

    sp = enc.plan(batch)
    t_plan = timed(lambda: enc.plan(batch))
    mine = sp.body_bytes[rank]
    body = torch.empty(max(mine, 1), dtype=torch.uint8, device=dev)
    t_enc = timed(lambda: enc.encode_body(batch, sp.width, body))
    out = torch.empty(sp.total_bytes, dtype=torch.uint8, device=dev) if rank == 0 else None
    t_p2p = timed(lambda: enc.gather(sp, body, out))
    check = "skipped"
    if rank == 0:
        res, back, _ = cd.deserialize(out)
        want = SP.synth_batch(cd, "rec64", world * n, SEEDS["rec64"], 0, first=0)
        check = "ok" if (res.errc == 0 and res.count == world * n and
                         torch.equal(back.recs, want.recs)) else f"FAILED errc {res.errc}"
        del back, want
    del out
    torch.cuda.empty_cache()
    full = torch.empty(sp.total_bytes, dtype=torch.uint8, device=dev)
    slab = [None]

    def ag():
        slab[0] = enc.all_gather(sp, body, full, slab[0])
    t_ag = timed(ag)
    del full, slab
    host = torch.empty(max(mine, 1), dtype=torch.uint8).pin_memory()
    t_d2h = timed(lambda: host.copy_(body[:mine], non_blocking=True))
    total = sp.total_bytes
    gbs = lambda b, t: round(b / t / 1e9, 2)
    dec = None
    try:
        dec = sharded_decode_bench(torch, dist, world, rank, dev, timed)
    except ConfigFailed as e:  # raised on every rank together (other faults propagate:
        dec = {"error": str(e)}  # torch.distributed.run then ends every rank)
    return {
        "sharded_decode": dec,
        "workload": f"one serialize(vector<Rec64>) message of {world} x {n} records "
                    f"({total / 2**30:.2f} GiB), bodies encoded on their own ranks",
        "records_per_rank": n, "message_bytes": total, "width": sp.width,
        "plan_ms": round(t_plan * 1e3, 3), "encode_body_ms": round(t_enc * 1e3, 3),
        "p2p_gather_ms": round(t_p2p * 1e3, 3),
        "p2p_gather_gbs": gbs(total - sp.body_bytes[0], t_p2p),
        "all_gather_ms": round(t_ag * 1e3, 3), "all_gather_gbs": gbs(total * (world - 1), t_ag),
        "d2h_pinned_ms": round(t_d2h * 1e3, 3), "d2h_pinned_gbs_per_rank": gbs(mine, t_d2h),
        "check": check,
        "note": "p2p_gather_gbs = bytes received by rank 0 / time; all_gather_gbs = bytes "
                "received over all ranks / time; times are max over ranks, best of "
                f"{reps} after a warmup",
    }


def host_path_pipelined(wl, torch, dev, chunk_records=4_000_000, reps=3):
    """The host path of a trivially-serializable VECTOR config (C2) as a
    pipeline: the batch moves in record chunks over three HIP streams (H2D,
    compute, D2H) with pinned host buffers. Chunk c of the step's encode leg
    (H2D records -> spk_encode_body -> D2H wire) and of its decode leg (H2D
    wire -> spk_decode_body -> D2H records, header parsed on the host by
    spk_parse_vector_header) run beside chunk c+1's transfers, so both PCIe
    directions stay busy. Same bytes as host_path (the serial form)."""
    import ctypes as ct
    SP = wl.SP
    cd = wl.cd
    if not cd.L.dev.trivial or wl.mode != SP.MODE_VECTOR:
        return None
    n, stride = wl.n, cd.L.stride
    plan = cd.get_needed_size(wl.batch, SP.MODE_VECTOR)
    w, hl, total = plan.width, plan.header_bytes, plan.total_bytes
    hb = (ct.c_uint8 * 512)()
    k = cd.lib.spk_vector_header(cd.L.ptr, n, w, hb, 512)
    assert k == hl
    recs_b = n * stride
    h_recs = torch.empty(recs_b, dtype=torch.uint8).pin_memory()
    h_recs.copy_(wl.batch.recs.view(-1))
    h_wire_in = torch.empty(total, dtype=torch.uint8).pin_memory()   # decode input
    h_wire_out = torch.empty(total, dtype=torch.uint8).pin_memory()  # encode output
    h_out = torch.empty(recs_b, dtype=torch.uint8).pin_memory()
    cd.serialize_to(wl.wire, wl.batch, SP.MODE_VECTOR, planned=False)
    h_wire_in.copy_(wl.wire[:total])
    d_recs = wl.batch.recs.view(-1)
    d_wire_out = wl.wire
    d_wire_in = torch.empty(total, dtype=torch.uint8, device=dev)
    d_dec = wl.dec.recs.view(-1)
    s_in, s_cmp, s_out = (torch.cuda.Stream(dev) for _ in range(3))
    ws = cd.workspace(SP.MODE_VECTOR, max(chunk_records, 1), total)
    chunks = [(r, min(r + chunk_records, n)) for r in range(0, n, chunk_records)]
    nullh = (ct.c_void_p * 1)(0)
    caps0 = (ct.c_uint64 * 1)(0)

    def step():
        h_wire_out[:hl].copy_(torch.frombuffer(bytearray(bytes(hb[:hl])), dtype=torch.uint8))
        e, nn, ww, hh = cd.parse_vector_header(bytes(h_wire_in[:64].numpy()))
        assert e == 0 and nn == n and ww == w and hh == hl
        for r0, r1 in chunks:
            b0, b1 = r0 * stride, r1 * stride
            # encode leg
            with torch.cuda.stream(s_in):
                d_recs[b0:b1].copy_(h_recs[b0:b1], non_blocking=True)
                ev_in = torch.cuda.Event()
                ev_in.record(s_in)
                d_wire_in[hl + b0:hl + b1].copy_(h_wire_in[hl + b0:hl + b1], non_blocking=True)
                ev_win = torch.cuda.Event()
                ev_win.record(s_in)
            s_cmp.wait_event(ev_in)
            rc = cd.lib.spk_encode_body(cd.L.ptr, r1 - r0, SP._p(d_recs[b0:]), nullh, w,
                                        SP._p(d_wire_out[hl + b0:]), b1 - b0, SP._p(ws),
                                        ws.numel(), SP._stream(s_cmp))
            assert rc == 0
            ev_enc = torch.cuda.Event()
            ev_enc.record(s_cmp)
            s_cmp.wait_event(ev_win)
            rc = cd.lib.spk_decode_body(cd.L.ptr, SP._p(d_wire_in[hl + b0:]), b1 - b0, w,
                                        r1 - r0, SP._p(d_dec[b0:]), r1 - r0, nullh, caps0,
                                        SP._p(cd.res_buf), SP._p(ws), ws.numel(),
                                        SP._stream(s_cmp))
            assert rc == 0
            ev_dec = torch.cuda.Event()
            ev_dec.record(s_cmp)
            s_out.wait_event(ev_enc)
            with torch.cuda.stream(s_out):
                h_wire_out[hl + b0:hl + b1].copy_(d_wire_out[hl + b0:hl + b1], non_blocking=True)
            s_out.wait_event(ev_dec)
            with torch.cuda.stream(s_out):
                h_out[b0:b1].copy_(d_dec[b0:b1], non_blocking=True)
        for st in (s_in, s_cmp, s_out):
            st.synchronize()

    step()  # warmup
    ok = bool(torch.equal(h_out, h_recs)) and bool(torch.equal(h_wire_out, h_wire_in))
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    dt = (time.perf_counter() - t0) / reps
    return {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(wl.algo_bytes / dt / 2**30, 3),
            "chunk_records": chunk_records, "check": "ok" if ok else "FAILED",
            "note": "pipelined: per record chunk H2D records -> spk_encode_body -> D2H wire and "
                    "H2D wire -> spk_decode_body -> D2H records, three HIP streams, pinned "
                    "host buffers, header parsed on the host (spk_parse_vector_header)"}


def sharded_decode_bench(torch, dist, world, rank, dev, timed, per_rank=2_000_000):
    """N>1: ONE C4-shaped message (vector<Outer>, world x 2M records) that
    every rank holds, decoded by ShardedVectorDecoder (each rank indexes and
    emits the records starting in its 1/world of the body; one all-gather of
    summaries) vs the whole message decoded by one GPU (rank 0)."""
    from yalantinglibs_amd import layout as LY
    from yalantinglibs_amd import parallel as PAR
    from yalantinglibs_amd import struct_pack as SP
    n = per_rank * world
    err = None
    try:  # local setup on every rank, agreed on before the first collective
        cd = SP.Codec(LY.case_layout("outer"), device=dev)
        batch = SP.synth_batch(cd, "outer", n, SEEDS["outer"], 16)
        wire, _ = cd.serialize(batch, SP.MODE_VECTOR)
        del batch
        torch.cuda.empty_cache()
        dec = PAR.ShardedVectorDecoder(cd)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    if not agree_ok(err is None, torch, dist, world, dev):
        raise ConfigFailed(f"sharded decode: setup failed on "
                           f"{'this rank: ' + err if err else 'another rank'}")
    out = [None]

    def run():
        out[0] = dec.decode(wire)
    t_sh = timed(run)
    b, first, res = out[0]
    counts = torch.tensor([b.n, int(res.errc)], dtype=torch.int64,
                          device=torch.device("cpu") if dist.get_backend() == "gloo" else dev)
    dist.all_reduce(counts)
    del out, b
    torch.cuda.empty_cache()
    single = None
    if rank == 0:
        one = cd.alloc_batch(n, [int(wire.numel())])
        ts = []
        for _ in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            cd.deserialize_to(one, wire, SP.MODE_VECTOR)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        single = min(ts[1:])
        del one
    return {"records": n, "message_bytes": int(wire.numel()), "ms": round(t_sh * 1e3, 3),
            "exchange_rounds": dec.rounds, "records_decoded": int(counts[0].item()),
            "errc_sum": int(counts[1].item()),
            "single_gpu_ms": round(single * 1e3, 3) if single else None,
            "note": "sharded: header parse + index + summary all-gather + emit on every rank, "
                    "max over ranks; single_gpu_ms: rank 0 decodes the whole message"}


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def compact_roofline(rf):
    if not rf:
        return None
    keep = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "traffic_ratio",
            "bytes_per_launch", "ms_per_launch")
    out = {k: _r(rf.get(k)) for k in keep}
    out["kernel"] = (rf.get("kernel") or "").split("(")[0][:40]
    return out


def compact_cpu(cb):
    if not cb:
        return None
    return {"value": cb["value"], "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
            "sample": cb["sample"][:160], "single_thread_gib_s": cb.get("single_thread_gib_s")}


def compact_host(entry):
    """Host-inclusive (PCIe) rates of a config: the serial form and, for C2,
    the pipelined one (GiB/s of the device step's algorithmic bytes)."""
    h = {}
    if entry.get("host_path"):
        h["serial_gib_s"] = entry["host_path"].get("gib_s")
    hp = entry.get("host_path_pipelined")
    if hp and "gib_s" in hp:
        h["pipelined_gib_s"] = hp["gib_s"]
    return h or None


def compact_line(line, detail_path):
    """The stdout line: the contract fields, `roofline`, `cpu_baseline` and
    one short entry per extra config, well under 2 KB so a tail of the
    driver's stdout holds all of it; the per-kernel tables, phase times and
    CPU-baseline details go to the detail file."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "mrec_per_s",
            "mmsg_per_s", "step_frac")
    out = {k: line[k] for k in keep if k in line}
    cfg = line["config"]
    out["config"] = {"workload": cfg["workload"][:90], "records_per_gpu": cfg.get(
        "records_per_gpu", cfg.get("messages_per_gpu")), "mode": cfg.get("mode", "messages"),
        "parallelism": cfg.get("parallelism")}
    out["roofline"] = compact_roofline(line.get("roofline"))
    out["cpu_baseline"] = compact_cpu(line.get("cpu_baseline"))
    h = compact_host(line)
    if h:
        out["host_path"] = h
    if "concat" in line:
        c = line["concat"] or {}
        sd = c.get("sharded_decode") or {}
        out["concat"] = {k: c.get(k) for k in ("p2p_gather_ms", "p2p_gather_gbs",
                                               "all_gather_ms", "d2h_pinned_ms", "check")}
        out["concat"]["sharded_decode_ms"] = sd.get("ms")
        out["concat"]["sharded_single_gpu_ms"] = sd.get("single_gpu_ms")
        if "error" in c:
            out["concat"]["error"] = str(c["error"])[:120]
    ex = (line.get("extra") or {}).get("configs") or {}
    if ex:
        cc = {}
        for name, e in ex.items():
            if "error" in e:
                cc[name] = {"error": str(e["error"])[:100]}
                continue
            rf = e.get("roofline") or {}
            cb = e.get("cpu_baseline") or {}
            d = {"ms": e.get("ms_per_step"), "gib_s": e.get("value"),
                 "mrec_s": e.get("mrec_per_s", e.get("mmsg_per_s")),
                 "kernel": (rf.get("kernel") or "").strip("() ").split("(")[0][:28],
                 "frac": rf.get("frac"), "traffic_ratio": rf.get("traffic_ratio"),
                 "cpu_gib_s": cb.get("value")}
            h = compact_host(e)
            if h:
                d["host_gib_s"] = h.get("pipelined_gib_s", h.get("serial_gib_s"))
            cc[name] = d
        out["extra"] = {"configs": cc}
    out["detail"] = os.path.relpath(detail_path, ROOT) if detail_path else None
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(args.gpus, world)
    if args.spawn_probe:
        print(json.dumps({"rank": rank, "world": world, "local": local}), flush=True)
        return
    import torch
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # one rank per GPU; the modulo only matters when rehearsing several ranks
    # on fewer GPUs (BENCH_DIST_BACKEND=gloo: RCCL refuses two ranks per GPU)
    dev = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}")
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    try:
        head = run_config(args.config, args, torch, dist, world, rank, dev, args.steps,
                          args.warmup, args.settle, cpu=True)
    except ConfigFailed as e:  # every rank got here together: no rank waits in a collective
        if rank == 0:
            print(json.dumps({"error": str(e), "config": args.config}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(e.code)
    concat = None
    if world > 1 and not args.no_concat:
        try:
            concat = concat_bench(torch, dist, world, rank, dev, args.concat_records)
        except ConfigFailed as e:  # raised on every rank together; any other fault
            concat = {"error": str(e)}  # propagates and torch.distributed.run ends every rank
    if rank == 0:  # progress on stderr (the JSON line stays the only stdout line)
        print(f"[bench] {args.config}: {head['ms_per_step']} ms/step", file=sys.stderr, flush=True)
    extra = {}
    if world > 1 and not args.no_shard_extra and args.config == "c2":
        # the sharded BASELINE configs, weak scaling: every rank its own 10M
        # Outer (C4) / 1M request frames (C5), no data-path collective
        for cfg in ("c4", "c5"):
            try:
                extra[cfg] = run_config(cfg, args, torch, dist, world, rank, dev,
                                        args.extra_steps, 2, 0.5, cpu=False)
            except ConfigFailed as e:  # raised on every rank together: skip it everywhere
                extra[cfg] = {"error": str(e)}
            if rank == 0:
                print(f"[bench] {cfg} x{world}: {extra[cfg].get('ms_per_step')} ms/step",
                      file=sys.stderr, flush=True)
    if world == 1 and not args.no_extra and args.config == "c2":
        for cfg in EXTRA:
            extra[cfg] = run_config(cfg, args, torch, dist, world, rank, dev, args.extra_steps,
                                    2, 0.5, cpu=True)
            if rank == 0:
                print(f"[bench] {cfg}: {extra[cfg].get('ms_per_step')} ms/step", file=sys.stderr,
                      flush=True)

    if rank == 0:
        line = {
            "metric": "struct_pack encode+decode throughput, device-resident (GiB/s)",
            "value": head["value"], "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": f"synthetic ({head['data']})",
            "config": dict(head["detail"], parallelism=(
                f"record-range shards x{world}, no data-path collective"
                if args.config != "c5" else f"message-range shards x{world}, no data-path collective")),
            ("mmsg_per_s" if args.config == "c5" else "mrec_per_s"):
                head.get("mmsg_per_s", head.get("mrec_per_s")),
            "phase_ms": head["phase_ms"], "kernels": head["kernels"],
            "roofline": head["roofline"],
            "step_frac": head["step_frac"],
            "cpu_baseline": head["cpu_baseline"],
        }
        if "with_host_sync" in head:
            line["with_host_sync"] = head["with_host_sync"]
        if "host_path" in head:
            line["host_path"] = head["host_path"]
        if "host_path_pipelined" in head:
            line["host_path_pipelined"] = head["host_path_pipelined"]
        if concat is not None:
            line["concat_ms"] = concat.get("p2p_gather_ms")
            line["concat_gbs"] = concat.get("p2p_gather_gbs")
            line["concat"] = concat
        if extra:
            line["extra"] = {"configs": extra}
        path = args.detail_out or os.path.join(
            ROOT, "gpurun_out", f"bench_detail_{args.config}_n{world}.json")
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "w") as f:
                json.dump(line, f, indent=1)
        except OSError as e:
            print(f"[bench] detail not written: {e}", file=sys.stderr, flush=True)
            path = None
        out = line if args.full_line else compact_line(line, path)
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
