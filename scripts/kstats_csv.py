"""Per-kernel summary of a rocprofv3 --stats kernel_stats.csv (calls, average and
total ms, share), sorted by total time.  usage: kstats_csv.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tot = sum(int(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:n]:
    name = r["Name"].split("(")[0].replace("void ", "").replace("sa::", "").replace("(anonymous namespace)::", "")
    print(f"{name[:40]:40s} {int(r['Calls']):6d} avg {int(float(r['AverageNs'])) / 1e6:9.3f} ms  "
          f"total {int(r['TotalDurationNs']) / 1e6:10.2f} ms  {100 * int(r['TotalDurationNs']) / tot:5.1f} %")
