"""Device timeline of a seqarc_amd -c run from its rocprofv3 kernel trace: busy
fraction per 100 ms (any kernel running) and the front kernels' share.
usage: e2e_timeline.py KERNEL_TRACE_CSV"""
import csv
import sys

FRONT = ("k_prep", "k_emit", "k_sort", "k_replay_seq", "k_find_runs", "k_replay_aux_short", "k_pad_keys",
         "k_scan_reads", "k_sort_huge")
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("sa::", "").replace("void ", "").split("<")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
rows.sort()
t0 = rows[0][0]
end = max(e for _, e, _ in rows)
W = 100_000_000
nb = (end - t0) // W + 1
busy = [0] * nb
front = [0] * nb
for kind, acc in (("any", busy), ("front", front)):
    iv = sorted((s, e) for s, e, n in rows if kind == "any" or n.startswith(FRONT))
    merged = []
    for s, e in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    for s, e in merged:
        while s < e:
            b = (s - t0) // W
            cut = min(e, t0 + (b + 1) * W)
            acc[b] += cut - s
            s = cut
for b in range(nb):
    print(f"{b * 0.1:6.1f} s  busy {busy[b] / W:5.2f}  front {front[b] / W:5.2f}")
tot = sum(busy) / (end - t0)
print(f"span {(end - t0) / 1e9:.2f} s, any-kernel busy {tot:.2f}, front busy {sum(front) / (end - t0):.2f}")
