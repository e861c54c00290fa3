"""Per-type timing of the C5 message kernels on the arrival-order batch:
decode (spk_decode_frames over the routed frame lists) and encode
(serialize_to with the response frame) of each C5 record type on its own,
HIP-event timed on one stream (diagnostic)."""
import sys
import torch
sys.path.insert(0, ".")
import bench
from yalantinglibs_amd import struct_pack as SP

dev = torch.device("cuda:0")
wl = bench.C5Workload(torch, 1_000_000, 0, dev)
s = torch.cuda.current_stream()
wl.step(s)
torch.cuda.synchronize()
print("check:", wl.check(), flush=True)
rt = wl.router


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


ms = timed(lambda: rt.route(wl.wire, wl.offs, wl.nframes, stream=s))
print(f"route: {ms:.4f} ms  n={wl.nframes}", flush=True)
for k, g in enumerate(wl.groups):
    dec = lambda: g["cd"].deserialize_frames(g["args"], wl.wire, rt.begins[k], rt.ends[k], g["m"],
                                             g["rq"].prefix_len, stream=s)
    enc = lambda: g["cd"].serialize_to(g["resp"], g["args"], SP.MODE_MESSAGES, g["resp_offs"],
                                       stream=s, frame=g["rs"])
    for name, fn in (("decode", dec), ("encode", enc)):
        ms = timed(fn)
        byt = g["req_len"] + g["rec_bytes"] if name == "decode" else g["rec_bytes"] + g["resp_len"]
        print(f"{g['case']:8s} {name}: {ms:.4f} ms  {byt / ms / 1e6:.1f} GB/s  n={g['n']}", flush=True)
