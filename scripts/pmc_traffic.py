"""Per-launch HBM traffic per kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, then WRITE_SIZE; MI355X_MICROARCH.md "HBM": separate passes,
FETCH_SIZE doubled on gfx950 -- it tallies 128-B requests at 64 B).
usage: python scripts/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON
OUT_JSON maps bench phase names (and kernel names) to bytes per launch."""
import collections
import csv
import json
import sys

PHASE = {"k_coder_rv": "coder_r", "k_coder_r": "coder_r", "k_replay_aux_long": "replay_aux", "k_md5": "md5", "k_emit_sq": "emit",
         "k_replay_seq": "replay_seq", "k_assemble": "assemble", "k_prep": "prep+scan"}


def per_launch(path, counter):
    tot, n = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("sa::", "").replace("void ", "")
        tot[k] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(n[k]) for k in tot}


fetch = per_launch(sys.argv[1], "FETCH_SIZE")
write = per_launch(sys.argv[2], "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    b = 2 * fetch.get(k, 0.0) * 1024 + write.get(k, 0.0) * 1024   # KB -> B; FETCH doubled
    out[k] = {"bytes": round(b), "fetch_kb_raw": round(fetch.get(k, 0.0)), "write_kb": round(write.get(k, 0.0))}
    base = k.split("<")[0]   # (k_coder_rv<5>: a template instance)
    if base in PHASE:
        out[PHASE[base]] = round(b)
json.dump(out, open(sys.argv[3], "w"), indent=1)
for k, v in out.items():
    if isinstance(v, dict):
        print("%-28s %10.3f GB/launch" % (k, v["bytes"] / 1e9))
