"""Kernel timeline of the last bench step from a rocprofv3 kernel trace CSV.
usage: python scripts/timeline.py gpurun_out/prof_TAG/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
starts = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
rs = sorted(rows[starts[-1]:], key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rs[0]["Start_Timestamp"])
for r in rs:
    n = r["Kernel_Name"].split("(")[0].replace("sa::", "")
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s > 0.5:
        print("%-24s q%-3s %8.1f %8.1f %7.1f" % (n, r.get("Queue_Id", ""), s, e, e - s))
