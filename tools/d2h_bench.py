"""Host-table fill rates for the drop-in's first query (experiments only): D2H of a
20 GB device buffer into fresh pageable memory, pre-faulted pageable memory, and
pinned memory (allocation time reported separately), and pre-faulted memory
registered with hipHostRegister (registration time reported separately)."""
import ctypes
import time

import torch

n = 2_500_000_000  # 20 GB of f64
d = torch.empty(n, dtype=torch.float64, device="cuda")
d.fill_(1.0)
torch.cuda.synchronize()
hip = ctypes.CDLL("libamdhip64.so")
for label in ("fresh pageable", "prefaulted pageable", "pinned", "prefaulted + registered"):
    t0 = time.perf_counter()
    if label == "pinned":
        h = torch.empty(n, dtype=torch.float64, pin_memory=True)
    else:
        h = torch.empty(n, dtype=torch.float64)
        if label.startswith("prefaulted"):
            h.fill_(0.0)
        if label.endswith("registered"):
            tr = time.perf_counter()
            rc = hip.hipHostRegister(ctypes.c_void_p(h.data_ptr()), ctypes.c_size_t(n * 8), ctypes.c_uint(0))
            print(f"  hipHostRegister rc={rc} {time.perf_counter() - tr:.2f} s", flush=True)
    t1 = time.perf_counter()
    h.copy_(d)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{label}: alloc/fault {t1 - t0:.2f} s, copy {t2 - t1:.2f} s = {n * 8 / (t2 - t1) / 1e9:.1f} GB/s", flush=True)
    if label.endswith("registered"):
        hip.hipHostUnregister(ctypes.c_void_p(h.data_ptr()))
    del h
