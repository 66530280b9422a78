"""CPU cost of the allocator / driver memory queries, and whether they wait for queued GPU work."""
import time

import torch

x = torch.randn(8192, 8192, device="cuda")
torch.cuda.synchronize()
for name, fn in (("memory_reserved", lambda: torch.cuda.memory_reserved(0)),
                 ("mem_get_info", lambda: torch.cuda.mem_get_info(0))):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        fn()
    idle = (time.perf_counter() - t0) * 1e4  # us per call
    for _ in range(20):
        y = x @ x  # ~10 ms of queued GPU work
    t0 = time.perf_counter()
    fn()
    busy = (time.perf_counter() - t0) * 1e6
    torch.cuda.synchronize()
    print(f"{name}: {idle:.1f} us idle, {busy:.1f} us with queued work")
