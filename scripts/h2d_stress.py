"""Background host->device copy load for the clock experiment (round 4, r4e):
pinned 1 GiB host buffer copied to the device in a loop at about --gbs GB/s
for --seconds.  usage: python scripts/h2d_stress.py [--gbs 8] [--seconds 20]"""
import argparse
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--gbs", type=float, default=8.0)
ap.add_argument("--seconds", type=float, default=20.0)
a = ap.parse_args()
h = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
t0 = time.perf_counter()
n = 0
while time.perf_counter() - t0 < a.seconds:
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    n += 1
    ahead = n * (1 << 30) / (a.gbs * 1e9) - (time.perf_counter() - t0)
    if ahead > 0:
        time.sleep(ahead)
el = time.perf_counter() - t0
print(f"h2d_stress: {n} GiB in {el:.1f} s = {n * (1 << 30) / el / 1e9:.1f} GB/s", flush=True)
