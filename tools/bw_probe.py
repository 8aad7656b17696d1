import time, torch, numpy as np, os
n = 512 << 20
src = torch.empty(n, dtype=torch.uint8).pin_memory()
dst = torch.empty(n, dtype=torch.uint8, device="cuda")
pageable = torch.empty(n, dtype=torch.uint8)
pageable.fill_(1); src.fill_(2)
for name, s in (("pinned", src), ("pageable", pageable)):
    for _ in range(2):
        torch.cuda.synchronize(); t = time.perf_counter(); dst.copy_(s, non_blocking=True); torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(name, "H2D GB/s", round(n / dt / 1e9, 1))
a = np.ones(n, np.uint8); b = np.empty(n, np.uint8)
for _ in range(2):
    t = time.perf_counter(); np.copyto(b, a); dt = time.perf_counter() - t
print("host memcpy 1 thread GB/s", round(n / dt / 1e9, 1), "cpus", os.sched_getaffinity(0).__len__())
