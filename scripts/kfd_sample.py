"""Samples, every 0.25 s until killed, what the kernel driver reports about
every process that has the GPU open: KFD's per-process, per-device
`evicted_ms` (time its user queues spent evicted: userptr invalidations by MMU
notifiers -- NUMA hinting, THP collapse, munmap of registered memory -- and
memory pressure) and `cu_occupancy`, beside /proc/vmstat's NUMA / THP
counters.  One line per sample:
  t <epoch> pid=<pid>:<gpu>:evicted_ms=<n>:cu_occ=<n>:<comm> ... vm <name>=<n> ...
Also prints, once, the host settings behind them (numa_balancing, THP).
Usage: python3 scripts/kfd_sample.py OUT [COMM ...]  (run in the background, kill it;
COMM: process names to keep, e.g. seqarc_amd python3)."""
import glob
import os
import sys
import time

VM = ("numa_hint_faults", "numa_hint_faults_local", "numa_pages_migrated", "numa_pte_updates",
      "thp_fault_alloc", "thp_fault_fallback", "thp_collapse_alloc", "thp_split_pmd", "pgmigrate_success")


def read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return None


def main():
    out = open(sys.argv[1], "a", buffering=1)
    only = set(sys.argv[2:])   # process names to keep (default: all)
    for p in ("/proc/sys/kernel/numa_balancing", "/sys/kernel/mm/transparent_hugepage/enabled",
              "/sys/kernel/mm/transparent_hugepage/defrag", "/sys/kernel/mm/transparent_hugepage/khugepaged/defrag",
              "/sys/kernel/mm/transparent_hugepage/khugepaged/scan_sleep_millisecs"):
        out.write(f"# {p}: {read(p)}\n")
    while True:
        parts = [f"t {time.time():.3f}"]
        for d in sorted(glob.glob("/sys/class/kfd/kfd/proc/*")):
            pid = os.path.basename(d)
            comm = (read(f"/proc/{pid}/comm") or "?").replace(" ", "_")
            if only and comm not in only:   # (the host's other GPUs run other jobs)
                continue
            for s in sorted(glob.glob(d + "/stats_*")):
                gpu = s.rsplit("_", 1)[1]
                ev = read(s + "/evicted_ms")
                occ = read(s + "/cu_occupancy")
                parts.append(f"pid={pid}:{gpu}:evicted_ms={ev}:cu_occ={occ}:{comm}")
        vm = {}
        for ln in (read("/proc/vmstat") or "").splitlines():
            k, _, v = ln.partition(" ")
            if k in VM:
                vm[k] = v
        parts.append("vm " + " ".join(f"{k}={vm.get(k)}" for k in VM))
        out.write(" ".join(parts) + "\n")
        time.sleep(0.25)


if __name__ == "__main__":
    main()
