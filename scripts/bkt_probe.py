"""Summary of SA_BKT_PROBE files (one line per k_replay_seq_bkt wave: block,
digit, start / end us on the 100 MHz clock, shader cycles, steps of 64
symbols, steps with a context shared by lanes, XCC).  Per launch (waves
grouped by start time): the span, the waves' cycles per step (median / p90),
the largest wave, and how many waves were alive on average.
usage: python scripts/bkt_probe.py probe.txt"""
import statistics
import sys

rows = []
for line in open(sys.argv[1]):
    f = line.split()
    if len(f) < 8:
        continue
    rows.append(dict(blk=int(f[0]), dig=int(f[1]), t0=float(f[2]), t1=float(f[3]), cyc=int(f[4]), steps=int(f[5]),
                     shared=int(f[6]), xcc=int(f[7])))
rows.sort(key=lambda r: r["t0"])
# launches: a new one starts when a wave starts after every earlier wave ended
launches, cur, end = [], [], -1.0
for r in rows:
    if cur and r["t0"] > end + 50.0:
        launches.append(cur)
        cur, end = [], -1.0
    cur.append(r)
    end = max(end, r["t1"])
if cur:
    launches.append(cur)
print(f"{len(rows)} waves, {len(launches)} launches")
for i, L in enumerate(launches):
    t0, t1 = min(r["t0"] for r in L), max(r["t1"] for r in L)
    span = t1 - t0
    cps = [r["cyc"] / r["steps"] for r in L if r["steps"]]
    us = [r["t1"] - r["t0"] for r in L]
    big = max(L, key=lambda r: r["t1"] - r["t0"])
    busy = sum(us) / span if span > 0 else 0.0
    steps = sum(r["steps"] for r in L)
    sh = sum(r["shared"] for r in L) / max(steps, 1)
    q = sorted(cps)
    print(f"launch {i}: {len(L)} waves, span {span / 1000:.2f} ms, waves alive {busy:.0f} on average, "
          f"cycles/step median {statistics.median(cps):.0f} p10 {q[len(q) // 10]:.0f} p90 {q[9 * len(q) // 10]:.0f}, "
          f"steps {steps} ({sh * 100:.0f} % shared), longest wave {(big['t1'] - big['t0']) / 1000:.2f} ms "
          f"({big['steps']} steps, digit {big['dig']}), median wave {statistics.median(us) / 1000:.3f} ms")
