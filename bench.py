#!/usr/bin/env python3
"""bench.py — struct_pack encode+decode throughput on MI355X (device-resident).

A "step" = one serialize + one deserialize of this rank's whole record batch
through the C ABI (spk_plan + spk_encode + spk_decode), inputs already in HBM.
Default workload (BASELINE.json configs[1], "C2"): 100M 64-byte Rec64 records
per GPU as one struct_pack message, serialize(std::vector<Rec64>) and
deserialize_to back. Multi-GPU: each rank owns an independent 100M-record
shard (record-range partition, no data-path collective) => weak scaling.

value = algorithmic bytes of all ranks / max-over-ranks wall time, in GiB/s:
  per record: encode reads the record and writes its wire bytes, decode reads
  the wire bytes and writes the record: 4 x 64 B for C2.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2b|c3|c4]
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
    "c4": ("outer", 10_000_000, 16, "A",
           "C4: 10M Outer{int64, vector<Inner{int32,float}> n U[0,16]} per GPU, one vector message"),
    "cv": ("var", 10_000_000, 16, "A",
           "varint records: 10M Var{var_int32_t, std::string len U[0,16], var_uint64_t, double, "
           "var_int64_t, var_uint32_t} per GPU (LEB128 lengths 1-10 B), one vector message"),
}
# kernel the roofline object describes, per config (rocprof name prefix, for
# the PMC traffic lookup in profiles/r01/pmc_<config>.json)
DOMINANT = {"c2": "spk::shift_copy_kernel", "c2b": "void spk::fixed_msg_encode_lds<true>",
            "c3": "spk::var_encode_write", "c4": "spk::var_encode_write",
            "cv": "spk::var_encode_write"}
SEEDS = {"rec64": 0x5EED0002, "recs": 0x5EED0003, "outer": 0x5EED0004, "var": 0x5EED000C}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + ["c5"])
    ap.add_argument("--records", type=int, default=0, help="override records per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--settle", type=float, default=1.0,
                    help="seconds of untimed steps before the warmup (GPU clock ramp)")
    ap.add_argument("--host-path", action="store_true",
                    help="also time H2D + encode + decode + D2H from pinned host buffers")
    ap.add_argument("--pmc-json", default="", help="rocprofv3 PMC summary for roofline.traffic")
    return ap.parse_args()


def cpu_baseline(case, param):
    """Reference header-only struct_pack on the host cores (rank 0 only)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    if not os.path.exists(exe):
        return None
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    n = {"rec64": 20_000_000, "recs": 4_000_000, "outer": 4_000_000, "c5": 600_000,
         "var": 4_000_000}[case]
    out = {}
    for t in sorted({1, threads}):
        r = subprocess.run([exe, case, str(n), str(SEEDS.get(case, 0)), str(param), str(t), "10"],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            return None
        out[t] = json.loads(r.stdout.strip().splitlines()[-1])
    return out, n, threads


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from yalantinglibs_amd import _capi as C
    from yalantinglibs_amd import layout as LY
    from yalantinglibs_amd import struct_pack as SP

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    if args.config == "c5":
        return run_c5(args, torch, dist, world, rank, dev)

    case, n, param, modech, desc = CONFIGS[args.config]
    if args.records:
        n = args.records
    mode = SP.MODE_VECTOR if modech == "A" else SP.MODE_MESSAGES
    cd = SP.Codec(LY.case_layout(case), device=dev)
    # this rank's shard: global records [rank*n, (rank+1)*n)
    if case in ("rec64", "recs", "outer"):
        batch = SP.synth_batch(cd, case, n, SEEDS[case], param, first=rank * n)
    else:  # host generator (yalantinglibs_amd/synth.py), uploaded before timing;
        # every rank gets the same n records (same shape and bytes per rank)
        import numpy as np
        from yalantinglibs_amd import synth as SY
        _, recs_np, heaps_np = SY.make_batch(case, n, SEEDS[case], param)
        batch = SP.RecordBatch(
            cd.L, torch.from_numpy(recs_np.view(np.uint8).reshape(n, cd.L.stride)).to(dev),
            [torch.from_numpy(np.ascontiguousarray(h).view(np.uint8).reshape(-1)).to(dev)
             for h in heaps_np])
    plan = cd.get_needed_size(batch, mode)
    wire = torch.empty(plan.total_bytes + 64, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev) if mode == SP.MODE_MESSAGES else None
    elems = [int(h.numel()) // sp.elem.size for h, sp in zip(batch.heaps, cd.L.dev.spans)]
    dec = cd.alloc_batch(n, elems)
    stream = torch.cuda.current_stream(dev)

    rec_bytes = batch.recs.numel() + sum(int(h.numel()) for h in batch.heaps)
    if batch.heaps and any(e == 0 for e in elems):
        rec_bytes = batch.recs.numel()
    wire_bytes = plan.total_bytes
    algo_bytes = 2 * rec_bytes + 2 * wire_bytes  # enc in/out + dec in/out

    ev = []

    def step(record=False):
        e0 = torch.cuda.Event(enable_timing=True) if record else None
        if record:
            e0.record(stream)
        cd.plan(batch, mode, stream)
        e1 = torch.cuda.Event(enable_timing=True) if record else None
        if record:
            e1.record(stream)
        cd.serialize_to(wire, batch, mode, offs, stream=stream, planned=True)
        e2 = torch.cuda.Event(enable_timing=True) if record else None
        if record:
            e2.record(stream)
        cd.deserialize_to(dec, wire[:plan.total_bytes], mode, offs,
                          n if mode == SP.MODE_MESSAGES else 0, stream=stream)
        if record:
            e3 = torch.cuda.Event(enable_timing=True)
            e3.record(stream)
            ev.append((e0, e1, e2, e3))

    # correctness gate before timing: round trip must be exact
    step()
    torch.cuda.synchronize(dev)
    res = cd.result()
    ok = res.errc == 0 and res.count == n and torch.equal(dec.recs, batch.recs)
    if not ok:
        print(json.dumps({"error": "round trip mismatch", "errc": res.errc}), flush=True)
        sys.exit(3)

    # untimed settle: the GPU needs ~0.5-1 s of sustained load before its
    # clocks reach the steady state (a copy runs ~13 % slower in the first
    # few hundred ms: scripts/probes/copy_probe.hip before/after a bench in
    # one call), so keep stepping for --settle seconds before the warmup
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        step()
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # phase breakdown: separate event-instrumented steps (outside the timed region)
    for _ in range(max(3, min(args.steps, 10))):
        step(record=True)
    torch.cuda.synchronize(dev)
    plan_ms = sum(a.elapsed_time(b) for a, b, _, _ in ev) / len(ev)
    enc_ms = sum(b.elapsed_time(c) for _, b, c, _ in ev) / len(ev)
    dec_ms = sum(c.elapsed_time(d) for _, _, c, d in ev) / len(ev)
    ms_step = dt * 1e3 / args.steps
    total_bytes = algo_bytes * world * args.steps
    value = total_bytes / dt / 2**30
    mrec = n * world * args.steps / dt / 1e6

    # dominant kernel and its per-launch algorithmic bytes / duration:
    #   trivially serializable records in one vector message (C2): every
    #   step is two launches of shift_copy_kernel (encode: records -> wire
    #   body, decode: wire body -> records), each moving 2 x record bytes; its
    #   average duration is the mean of the encode and decode phases (HIP
    #   events on the launch stream; the decode phase also holds the ~4 us
    #   header kernel, so this slightly understates the kernel's rate);
    #   otherwise: the encode write pass (record + heap bytes in, wire out).
    if cd.L.dev.trivial and mode == SP.MODE_VECTOR:
        roof_kernel = "shift_copy_kernel (encode + decode launches)"
        launch_bytes = 2 * rec_bytes
        launch_ms = (enc_ms + dec_ms) / 2
    else:
        roof_kernel = ("fixed_msg_encode_lds" if cd.L.dev.trivial else "var_encode_write") \
            + " (encode phase)"
        launch_bytes = rec_bytes + wire_bytes
        launch_ms = enc_ms
    roof_ach = launch_bytes / (launch_ms * 1e-3) / 1e9
    # HBM bytes per launch of the same kernel from a separate rocprofv3 PMC run
    # of this command (scripts/gpu_pmc.sh -> profiles/r01/pmc_<config>.json;
    # FETCH_SIZE doubled per the gfx950 correction, WRITE_SIZE exact)
    traffic = None
    pmc = args.pmc_json or os.path.join(ROOT, "profiles", "r01", f"pmc_{args.config}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            for k, v in json.load(f).items():
                if k.startswith(DOMINANT.get(args.config, "~")):
                    traffic = v.get("hbm_bytes_per_launch")

    host = None
    if args.host_path and rank == 0:
        host = host_path(cd, batch, mode, plan, wire, dec, offs, n, stream, dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # N=1 only
        cb = cpu_baseline(case, param)
        if cb:
            runs, cn, threads = cb
            best = runs[threads]
            per_rec = algo_bytes / n
            tsec = best["encode_s"] + best["decode_s"]
            single = runs[1]
            cpu = {"value": round(per_rec * cn / tsec / 2**30, 3), "unit": "GiB/s",
                   "cores": threads, "kind": "reference",
                   "sample": f"{cn} {case} records, reference struct_pack serialize_to + "
                             f"deserialize_to (-O3 -DNDEBUG -DSTRUCT_PACK_OPTIMIZE), "
                             f"{threads} threads x contiguous slices, best of 10",
                   "single_thread_gib_s": round(per_rec * cn / (single["encode_s"] +
                                                                single["decode_s"]) / 2**30, 3),
                   "mrec_per_s": round(cn / tsec / 1e6, 2)}

    if rank == 0:
        line = {
            "metric": "struct_pack encode+decode throughput, device-resident (GiB/s)",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": (f"synthetic ({'spk_synth' if case in ('rec64', 'recs', 'outer') else 'host synth.py'} "
                                     f"seeded {case}, seed {SEEDS[case]:#x})"),
            "config": {"workload": desc, "records_per_gpu": n,
                       "mode": "vector" if modech == "A" else "messages",
                       "wire_bytes_per_gpu": wire_bytes, "record_bytes_per_gpu": rec_bytes,
                       "algorithmic_bytes_per_step_per_gpu": algo_bytes,
                       "parallelism": f"record-range shards x{world}, no data-path collective"},
            "mrec_per_s": round(mrec, 2),
            "phase_ms": {"plan": round(plan_ms, 4), "encode": round(enc_ms, 4),
                         "decode": round(dec_ms, 4)},
            "roofline": {"bound": "hbm", "kernel": roof_kernel,
                         "bytes_per_launch": launch_bytes, "ms_per_launch": round(launch_ms, 4),
                         "achieved": round(roof_ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(roof_ach / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "step_achieved": round(algo_bytes / (ms_step * 1e-3) / 1e9, 1),
                         "step_frac": round(algo_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "cpu_baseline": cpu,
        }
        if host:
            line["host_path"] = host
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


C5_TYPES = [  # (case, share of messages, param, rpc function name) — coro_rpc bench shapes
    ("rpcrect", 1, 0, "echo_rect"),          # rect{point p1, p2}   (api/Rect.h)
    ("person", 1, 48, "echo_person"),        # person{id, name, age, salary}
    ("ints", 1, 2000, "array_1K_int"),       # std::vector<int>, ~1K elements (data_gen.cpp:61)
]
C5_SEEDS = {"rpcrect": 0x5EED0007, "person": 0x5EED0008, "ints": 0x5EED0009}


def run_c5(args, torch, dist, world, rank, dev):
    """C5: a coro_rpc server step over a batch of framed requests of three
    record types (grouped by function id, one launch per type): decode every
    [req_header][args] frame, echo, encode every [resp_header][ret] frame.
    Device-resident `value`; the host-inclusive rate (H2D of the socket
    buffers + offsets, D2H of the responses) goes in `host_path`."""
    from yalantinglibs_amd import coro_rpc as RPC
    from yalantinglibs_amd import layout as LY
    from yalantinglibs_amd import struct_pack as SP
    n_total = args.records or 1_000_000
    shares = sum(s for _, s, _, _ in C5_TYPES)
    stream = torch.cuda.current_stream(dev)
    groups = []
    for case, share, param, fname in C5_TYPES:
        n = n_total * share // shares
        cd = SP.Codec(LY.case_layout(case), device=dev)
        src = SP.synth_batch(cd, case, n, C5_SEEDS[case], param, first=rank * n)
        plan = cd.get_needed_size(src, SP.MODE_MESSAGES)
        fid = RPC.func_id(fname)
        rq = RPC.req_frame(fid, seq_base=rank * n)
        rs = RPC.resp_frame(seq_base=rank * n)
        req_len = plan.total_bytes + n * rq.prefix_len
        req = torch.empty(req_len + 64, dtype=torch.uint8, device=dev)
        req_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cd.serialize_to(req, src, SP.MODE_MESSAGES, req_offs, planned=True, frame=rq)
        elems = [int(h.numel()) // sp.elem.size for h, sp in zip(src.heaps, cd.L.dev.spans)]
        args_b = cd.alloc_batch(n, elems)
        resp_len = plan.total_bytes + n * rs.prefix_len
        resp = torch.empty(resp_len + 64, dtype=torch.uint8, device=dev)
        resp_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        rec_bytes = src.recs.numel() + sum(int(h.numel()) for h in src.heaps)
        groups.append(dict(case=case, n=n, cd=cd, src=src, req=req[:req_len],
                           req_offs=req_offs, args=args_b, resp=resp, resp_offs=resp_offs,
                           rq=rq, rs=rs, rec_bytes=rec_bytes, req_len=req_len,
                           resp_len=resp_len))

    def step():
        for g in groups:
            cd = g["cd"]
            cd.deserialize_to(g["args"], g["req"], SP.MODE_MESSAGES, g["req_offs"], g["n"],
                              stream=stream, prefix=g["rq"].prefix_len)
            cd.serialize_to(g["resp"], g["args"], SP.MODE_MESSAGES, g["resp_offs"],
                            stream=stream, frame=g["rs"])

    step()
    torch.cuda.synchronize(dev)
    for g in groups:  # correctness gate: every request decoded, echo == source
        r = g["cd"].result()
        if (r.errc != 0 or r.count != g["n"] or not torch.equal(g["args"].recs, g["src"].recs)
                or int(g["resp_offs"][-1].item()) != g["resp_len"]):
            print(json.dumps({"error": "c5 round trip mismatch", "case": g["case"]}), flush=True)
            sys.exit(3)
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        step()
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # algorithmic bytes: request frames in + records/heaps out (decode),
    # records/heaps in + response frames out (encode)
    algo = sum(g["req_len"] + 2 * g["rec_bytes"] + g["resp_len"] for g in groups)
    n_msgs = sum(g["n"] for g in groups)
    ms_step = dt * 1e3 / args.steps
    value = algo * world * args.steps / dt / 2**30

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # N=1 only
        cb = cpu_baseline("c5", 0)
        if cb:
            runs, cn, threads = cb
            per_msg = algo / n_msgs
            best, single = runs[threads], runs[1]
            cpu = {"value": round(per_msg * cn / (best["encode_s"] + best["decode_s"]) / 2**30, 3),
                   "unit": "GiB/s", "cores": threads, "kind": "reference",
                   "sample": f"{cn} framed requests (rect/person/vector<int> thirds), reference "
                             "struct_pack deserialize_to of each request + resp_header/"
                             "serialize of each echo response (-O3 -DNDEBUG "
                             f"-DSTRUCT_PACK_OPTIMIZE), {threads} threads x message slices, "
                             "best of 10",
                   "single_thread_gib_s": round(per_msg * cn / (single["encode_s"] +
                                                                single["decode_s"]) / 2**30, 3),
                   "mmsg_per_s": round(cn / (best["encode_s"] + best["decode_s"]) / 1e6, 3)}

    host = None
    if rank == 0:
        # host-inclusive: socket buffers live in (pinned) host memory
        h_req = [torch.empty(g["req_len"], dtype=torch.uint8).pin_memory() for g in groups]
        h_ro = [torch.empty(g["n"] + 1, dtype=torch.int64).pin_memory() for g in groups]
        h_resp = [torch.empty(g["resp_len"], dtype=torch.uint8).pin_memory() for g in groups]
        h_so = [torch.empty(g["n"] + 1, dtype=torch.int64).pin_memory() for g in groups]
        for g, a, b in zip(groups, h_req, h_ro):
            a.copy_(g["req"])
            b.copy_(g["req_offs"])
        torch.cuda.synchronize(dev)
        reps = 3
        t1 = time.perf_counter()
        for _ in range(reps):
            for g, a, b in zip(groups, h_req, h_ro):
                g["req"].copy_(a, non_blocking=True)
                g["req_offs"].copy_(b, non_blocking=True)
            step()
            for g, a, b in zip(groups, h_resp, h_so):
                a.copy_(g["resp"][:g["resp_len"]], non_blocking=True)
                b.copy_(g["resp_offs"], non_blocking=True)
        torch.cuda.synchronize(dev)
        ht = (time.perf_counter() - t1) / reps
        host = {"ms_per_step": round(ht * 1e3, 3), "gib_s": round(algo / ht / 2**30, 3),
                "mmsg_per_s": round(n_msgs / ht / 1e6, 3),
                "note": "H2D of request frames + offsets, decode, echo encode, D2H of "
                        "response frames + offsets (pinned host buffers)"}
    if rank == 0:
        line = {
            "metric": "struct_pack encode+decode throughput, device-resident (GiB/s)",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic (spk_synth seeded rpcrect/person/ints)",
            "config": {"workload": "C5: coro_rpc server step, %d framed requests per GPU "
                                   "(rect / person / vector<int>~1K, one launch per type): "
                                   "decode [req_header][args], encode [resp_header][ret]"
                                   % n_msgs,
                       "messages_per_gpu": n_msgs,
                       "per_type": {g["case"]: g["n"] for g in groups},
                       "algorithmic_bytes_per_step_per_gpu": algo,
                       "parallelism": f"message-range shards x{world}, no data-path collective"},
            "mmsg_per_s": round(n_msgs * world * args.steps / dt / 1e6, 3),
            "roofline": {"bound": "hbm", "kernel": "whole step",
                         "achieved": round(algo / (ms_step * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None},
            "cpu_baseline": cpu,
            "host_path": host,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_path(cd, batch, mode, plan, wire, dec, offs, n, stream, dev):
    """PCIe-inclusive rate: pinned host records (+ heaps) -> H2D -> encode ->
    D2H wire; pinned host wire -> H2D -> decode -> D2H records (+ heaps)
    (DESIGN.md). The coro_rpc socket buffers this models live in host memory."""
    import torch
    from yalantinglibs_amd import struct_pack as SP
    srcs = [batch.recs] + list(batch.heaps)
    dsts = [dec.recs] + list(dec.heaps)
    h_in = [torch.empty_like(t, device="cpu").pin_memory() for t in srcs]
    for h, t in zip(h_in, srcs):
        h.copy_(t)
    h_wire = torch.empty(plan.total_bytes, dtype=torch.uint8).pin_memory()
    h_out = [torch.empty_like(t, device="cpu").pin_memory() for t in dsts]
    torch.cuda.synchronize(dev)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        for t, h in zip(srcs, h_in):
            t.copy_(h, non_blocking=True)
        cd.plan(batch, mode, stream)
        cd.serialize_to(wire, batch, mode, offs, stream=stream, planned=True)
        h_wire.copy_(wire[:plan.total_bytes], non_blocking=True)
        wire[:plan.total_bytes].copy_(h_wire, non_blocking=True)
        cd.deserialize_to(dec, wire[:plan.total_bytes], mode, offs,
                          n if mode == SP.MODE_MESSAGES else 0, stream=stream)
        for t, h in zip(dsts, h_out):
            h.copy_(t, non_blocking=True)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    algo = 2 * sum(int(t.numel()) for t in srcs) + 2 * plan.total_bytes
    return {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(algo / dt / 2**30, 3),
            "note": "includes H2D of records (+heaps) and wire, D2H of wire and decoded "
                    "records (+heaps); pinned host buffers"}


if __name__ == "__main__":
    main()
