"""Batch overlap from a rocprofv3 kernel trace CSV: for every pass-R launch
(k_coder_rv), which front kernels of other batches (other queues) ran while it
ran, and a kernel timeline (> 0.5 ms) of a window in the middle of the run.
usage: python scripts/overlap.py run_kernel_trace.csv [window_ms]"""
import csv
import sys

FRONT = ("k_prep", "k_emit", "k_sort_", "k_replay_seq", "k_replay_aux_short", "k_find_runs")
rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 1500.0


def name(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sa::", "")


ks = sorted(({"n": name(r), "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"]), "q": r.get("Queue_Id", "")}
             for r in rows), key=lambda k: k["s"])
t0 = ks[0]["s"]
passr = [k for k in ks if k["n"].startswith("k_coder_rv")]
print("pass R launches: %d" % len(passr))
for p in passr:
    inside = [k for k in ks if k["q"] != p["q"] and k["n"].startswith(FRONT) and k["s"] < p["e"] and k["e"] > p["s"]]
    busy = sum(min(k["e"], p["e"]) - max(k["s"], p["s"]) for k in inside)
    print("k_coder_rv q%-3s %9.1f-%9.1f ms (%6.1f ms): %3d front kernels of other batches overlap it, %6.1f ms of "
          "front kernel time inside" % (p["q"], (p["s"] - t0) / 1e6, (p["e"] - t0) / 1e6, (p["e"] - p["s"]) / 1e6,
                                        len(inside), busy / 1e6))
mid = passr[len(passr) // 2]["s"] if passr else ks[len(ks) // 2]["s"]
print("\ntimeline %.0f ms from %.1f ms (kernels > 0.5 ms): name, queue, start, end, duration" % (win, (mid - t0) / 1e6))
for k in ks:
    if mid <= k["s"] < mid + win * 1e6 and k["e"] - k["s"] > 5e5:
        print("%-26s q%-3s %9.1f %9.1f %7.1f" % (k["n"], k["q"], (k["s"] - t0) / 1e6, (k["e"] - t0) / 1e6,
                                                (k["e"] - k["s"]) / 1e6))
