"""Host<->device copy probe: pinned allocation rate, host-register rate,
pageable vs pinned H2D / D2H bandwidth, and pageable copies from several
threads at once (is the runtime's staging path serialised?)."""
import threading
import time

import torch

GB = 1 << 30
dev = torch.device("cuda:0")
d = torch.empty(GB, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()


def t(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


pg = torch.empty(GB, dtype=torch.uint8)
pg.fill_(1)
print(f"pageable H2D 1 GiB: {GB / t(lambda: d.copy_(pg)) / 1e9:.1f} GB/s", flush=True)
print(f"pageable D2H 1 GiB: {GB / t(lambda: pg.copy_(d)) / 1e9:.1f} GB/s", flush=True)
t0 = time.perf_counter()
pn = torch.empty(GB, dtype=torch.uint8, pin_memory=True)
print(f"pinned alloc 1 GiB: {GB / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)
pn.fill_(1)
print(f"pinned H2D 1 GiB: {GB / t(lambda: d.copy_(pn, non_blocking=True)) / 1e9:.1f} GB/s", flush=True)
print(f"pinned D2H 1 GiB: {GB / t(lambda: pn.copy_(d, non_blocking=True)) / 1e9:.1f} GB/s", flush=True)
rt = torch.cuda.cudart()
pg2 = torch.empty(GB, dtype=torch.uint8)
pg2.fill_(2)
t0 = time.perf_counter()
rc = rt.cudaHostRegister(pg2.data_ptr(), GB, 0)
reg = time.perf_counter() - t0
print(f"host register 1 GiB: rc {rc}, {GB / reg / 1e9:.1f} GB/s", flush=True)
print(f"registered H2D 1 GiB: {GB / t(lambda: d.copy_(pg2, non_blocking=True)) / 1e9:.1f} GB/s", flush=True)
t0 = time.perf_counter()
rt.cudaHostUnregister(pg2.data_ptr())
print(f"host unregister 1 GiB: {GB / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)

# four threads, each a pageable 256 MiB H2D on its own stream
n = 4
parts = [torch.empty(GB // 4, dtype=torch.uint8) for _ in range(n)]
for p in parts:
    p.fill_(3)
dst = [torch.empty(GB // 4, dtype=torch.uint8, device=dev) for _ in range(n)]
streams = [torch.cuda.Stream() for _ in range(n)]
spans = [None] * n


def work(i):
    with torch.cuda.stream(streams[i]):
        t0 = time.perf_counter()
        dst[i].copy_(parts[i])
        streams[i].synchronize()
        spans[i] = (t0, time.perf_counter())


torch.cuda.synchronize()
th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
t0 = time.perf_counter()
for x in th:
    x.start()
for x in th:
    x.join()
wall = time.perf_counter() - t0
print(f"{n} threads x 256 MiB pageable H2D: wall {wall * 1e3:.1f} ms ({GB / wall / 1e9:.1f} GB/s), per-thread ms "
      + ", ".join(f"{(b - a) * 1e3:.1f}" for a, b in spans), flush=True)
