"""Front duty cycle from a rocprofv3 kernel trace of bench.py: per batch the
front's span (its k_prep start to its k_replay_aux_short end) and the idle
stretch before the next front starts, and per context (host thread) the cycle
front -> pass R -> L passes -> assembly -> next front, so it shows whether the
next front waited for a free front turn or for a context to come back from its
tail.  usage: python scripts/front_cycle.py run_kernel_trace.csv"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))


def nm(r):   # (template arguments dropped: k_coder_l1<32u> -> k_coder_l1)
    return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sa::", "").split("<")[0]


ks = sorted(({"n": nm(r), "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"]), "th": r["Thread_Id"]}
             for r in rows), key=lambda k: k["s"])
fronts = []
cur = None
for k in ks:
    if k["n"] == "k_prep" or (k["n"] == "k_prep_sq16" and (cur is None or cur.get("done"))):
        if cur is None or cur.get("done"):
            cur = {"s": k["s"], "th": k["th"]}
            fronts.append(cur)
    if cur is not None and k["n"] == "k_replay_aux_short" and k["th"] == cur["th"]:
        cur["e"] = k["e"]
        cur["done"] = True
fronts = [f for f in fronts if "e" in f]
# per host thread: the end of its previous batch's assembly before each front
asm_end = {}
for k in ks:
    if k["n"].startswith("k_assemble_copy"):
        asm_end.setdefault(k["th"], []).append(k["e"])
sel = fronts[2:-1]
span = [(f["e"] - f["s"]) / 1e6 for f in sel]
gap = [(b["s"] - a["e"]) / 1e6 for a, b in zip(sel, sel[1:])]
wait_tail = []
for a, b in zip(sel, sel[1:]):
    prev = [t for t in asm_end.get(b["th"], []) if t < b["s"]]
    wait_tail.append((b["s"] - max(prev)) / 1e6 if prev else float("nan"))
print(f"fronts {len(sel)}: span median {statistics.median(span):.1f} ms (min {min(span):.1f}, max {max(span):.1f})")
print(f"idle between fronts: median {statistics.median(gap):.1f} ms, mean {statistics.mean(gap):.1f}, "
      f"max {max(gap):.1f}; share of time {100 * sum(gap) / ((sel[-1]['e'] - sel[0]['s']) / 1e6):.1f} %")
print(f"next front start - that context's previous assembly end: median {statistics.median(wait_tail):.2f} ms")
print("batch  th     span   idle_after  ctx_back(ms before start)")
for f, g, w in zip(sel, gap + [0], wait_tail + [0]):
    print(f"  {f['th']:>6} {(f['e'] - f['s']) / 1e6:7.1f} {g:8.1f}   {w:8.2f}")

# per context (host thread), batch by batch: front -> pass R -> L passes ->
# assembly -> the same context's next front
by = {}
for k in ks:
    by.setdefault(k["th"], []).append(k)
acc = {}
for th, L in by.items():
    idx = [i for i, k in enumerate(L) if k["n"] == "k_prep"]
    for a, b in zip(idx, idx[1:]):
        d = {k["n"]: k for k in L[a:b]}
        try:
            fs, fe = L[a]["s"], d["k_replay_aux_short"]["e"]
            rs, re_ = d["k_coder_rv"]["s"], d["k_coder_rv"]["e"]
            l1, l3, ae = d["k_coder_l1"]["s"], d["k_coder_l3"]["e"], d["k_assemble_copy"]["e"]
        except KeyError:
            continue
        for name, v in (("front", fe - fs), ("front end -> pass R start", rs - fe), ("pass R", re_ - rs),
                        ("pass R end -> L1", l1 - re_), ("L1 .. L3", l3 - l1), ("L3 -> assembly end", ae - l3),
                        ("assembly end -> next front", L[b]["s"] - ae), ("cycle", L[b]["s"] - fs)):
            acc.setdefault(name, []).append(v / 1e6)
print("\nper context (host thread), batch by batch: the cycle front -> pass R -> L passes -> assembly -> next front (ms)")
for name, v in acc.items():
    print(f"  {name:28s} n {len(v):3d}  median {statistics.median(v):8.1f}  mean {statistics.mean(v):8.1f}  "
          f"min {min(v):8.1f}  max {max(v):8.1f}")
