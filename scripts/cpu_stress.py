"""Host load for the clock experiment (round 4, r4f): --mode mem copies 512 MiB
arrays on every thread (host memory traffic, like the CLI's reader filling its
windows); --mode alu runs cache-resident arithmetic (host power, little memory
traffic).  numpy releases the GIL in both.  usage: python scripts/cpu_stress.py
--mode mem|alu [--threads 16] [--seconds 40]"""
import argparse
import threading
import time

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="mem")
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--seconds", type=float, default=40.0)
a = ap.parse_args()
moved = [0] * a.threads


def work(k):
    t0 = time.perf_counter()
    if a.mode == "mem":
        x = np.ones(512 << 20, np.uint8)
        y = np.empty_like(x)
        while time.perf_counter() - t0 < a.seconds:
            np.copyto(y, x)
            moved[k] += 2 * x.size
    else:
        x = np.random.default_rng(k).random(4096)
        while time.perf_counter() - t0 < a.seconds:
            for _ in range(200):
                x = np.sin(x) * 1.0001
            moved[k] += 200


th = [threading.Thread(target=work, args=(k,)) for k in range(a.threads)]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
el = time.perf_counter() - t0
print(f"cpu_stress {a.mode}: {a.threads} threads, {sum(moved) / el / 1e9:.1f} G units/s over {el:.1f} s", flush=True)
