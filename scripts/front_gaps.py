"""Front occupancy from a rocprofv3 kernel trace CSV of bench.py: the front
kernels (prep .. short SIMPLE_MODEL runs) of all batches
run one front at a time, so the share of wall time with no front kernel
running bounds what the front can still give.  Prints, over the timed region
(from the 3rd k_prep to the last k_replay_aux_short): the union of front
kernel intervals, the gaps between fronts (end of one front's last kernel to
the next front's first kernel) and within fronts (host syncs inside a front).
usage: python scripts/front_gaps.py run_kernel_trace.csv"""
import csv
import statistics
import sys

FRONT = ("k_prep", "k_scan_reads", "k_pad_keys", "k_emit", "k_sort_", "k_replay_seq", "k_find_runs", "k_sort_huge",
         "k_replay_aux_short", "__amd_rocclr_fill")


def name(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sa::", "")


rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(({"n": name(r), "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"])} for r in rows),
            key=lambda k: k["s"])
fr = [k for k in ks if k["n"].startswith(FRONT)]
preps = [i for i, k in enumerate(fr) if k["n"] in ("k_prep", "k_prep_sq16") and (i == 0 or not fr[i - 1]["n"].startswith("k_prep"))]
if len(preps) < 4:
    sys.exit("too few fronts in the trace")
# fronts: from one k_prep to the kernel before the next k_prep (fronts run one at a time)
fronts = []
for a, b in zip(preps, preps[1:] + [len(fr)]):
    seg = fr[a:b]
    fronts.append({"s": seg[0]["s"], "e": max(k["e"] for k in seg), "busy": 0, "kernels": seg})
for f in fronts:   # union of the front's kernel intervals
    cur_s = cur_e = None
    for k in sorted(f["kernels"], key=lambda k: k["s"]):
        if cur_e is None or k["s"] > cur_e:
            if cur_e is not None:
                f["busy"] += cur_e - cur_s
            cur_s, cur_e = k["s"], k["e"]
        else:
            cur_e = max(cur_e, k["e"])
    f["busy"] += cur_e - cur_s
sel = fronts[2:-1]   # the timed region roughly: skip warm-up fronts and the last
span = sel[-1]["e"] - sel[0]["s"]
busy = sum(f["busy"] for f in sel)
inside = sum(f["e"] - f["s"] for f in sel)
between = [b["s"] - a["e"] for a, b in zip(sel, sel[1:])]
print(f"fronts {len(sel)} over {span / 1e6:.1f} ms: {span / len(sel) / 1e6:.1f} ms per front (batch)")
print(f"front kernels busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f} %), front spans {inside / 1e6:.1f} ms "
      f"({100 * inside / span:.1f} %)")
print(f"per front: span median {statistics.median(f['e'] - f['s'] for f in sel) / 1e6:.1f} ms, "
      f"busy median {statistics.median(f['busy'] for f in sel) / 1e6:.1f} ms; "
      f"gap between fronts median {statistics.median(between) / 1e6:.2f} ms, max {max(between) / 1e6:.2f} ms")
# idle stretches inside fronts (host syncs)
gaps = []
for f in sel:
    ks_ = sorted(f["kernels"], key=lambda k: k["s"])
    end = ks_[0]["e"]
    for k in ks_[1:]:
        if k["s"] > end:
            gaps.append((k["s"] - end, k["n"]))
        end = max(end, k["e"])
by = {}
for g, n in gaps:
    by.setdefault(n, []).append(g)
print("idle before (inside fronts), per front:")
for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {n[:36]:36s} {sum(v) / len(sel) / 1e6:7.2f} ms  (n {len(v)}, median {statistics.median(v) / 1e6:.2f})")
