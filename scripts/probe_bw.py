"""Copy-bandwidth probe on the GPU box: torch D2D copy (hipMemcpy-class) vs
the codec's C2 encode/decode, to calibrate the achievable HBM rate."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps


nbytes = 6_400_000_000
a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
a.fill_(1)
out = {}
ms = timeit(lambda: b.copy_(a))
out["torch_copy_6.4GB"] = {"ms": round(ms, 3), "GBps": round(2 * nbytes / ms / 1e6, 1)}
ms = timeit(lambda: b[9:].copy_(a[:-9]))
out["torch_copy_shift9"] = {"ms": round(ms, 3), "GBps": round(2 * (nbytes - 9) / ms / 1e6, 1)}
a32 = a.view(torch.int32)
b32 = b.view(torch.int32)
ms = timeit(lambda: torch.add(a32, 0, out=b32))
out["torch_add_int32"] = {"ms": round(ms, 3), "GBps": round(2 * nbytes / ms / 1e6, 1)}
print(json.dumps(out))
