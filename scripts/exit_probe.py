"""Runs micro_run/exit_probe (scripts/micro/exit_probe.hip) per mode and prints the time from its _Exit to its reaping (round 3 g4i)."""
import subprocess
import sys
import time

for mode, gb in (("pinned", 8), ("thp", 8), ("dev", 200), ("pinned", 2), ("dev", 50)):
    time.sleep(5)
    r = subprocess.run(["./micro_run/exit_probe", mode, str(gb)], capture_output=True, text=True, timeout=300)
    m1 = time.monotonic()
    out = r.stdout.strip().splitlines()
    ex = [float(l.split()[1]) for l in out if l.startswith("exit ")]
    print(f"rc {r.returncode}: {out[0] if out else r.stderr[-300:]}; exit -> reaped "
          f"{(m1 - ex[0]) if ex else float('nan'):.3f} s", flush=True)
