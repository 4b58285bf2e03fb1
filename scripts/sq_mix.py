"""Per-kernel instruction mix and stall shares from rocprofv3 --pmc CSVs of the
SQ counters (scripts/gpu_r4j.sh): per wave, VALU / SALU / LDS / VMEM
instructions and the shares of the wave's cycles spent issuing, waiting on
memory (s_waitcnt) and stalled at issue.  usage: sq_mix.py CSV [CSV ...]"""
import collections
import csv
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sa::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r["Dispatch_Id"]))
rows = []
for k, c in tot.items():
    w = c.get("SQ_WAVES", 0.0)
    if w <= 0:
        continue
    cyc = c.get("SQ_WAVE_CYCLES", 0.0)
    rows.append((cyc, k, c, w))
print(f"{'kernel':32s} {'waves':>9s} {'VALU/w':>8s} {'SALU/w':>8s} {'LDS/w':>7s} {'VMRD/w':>7s} {'VMWR/w':>7s} "
      f"{'cyc/w':>9s} {'issue%':>6s} {'wait%':>6s} {'stall%':>6s}")
for cyc, k, c, w in sorted(rows, reverse=True)[:25]:
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    print(f"{k[:32]:32s} {w:9.0f} {c.get('SQ_INSTS_VALU', 0) / w:8.1f} {c.get('SQ_INSTS_SALU', 0) / w:8.1f} "
          f"{c.get('SQ_INSTS_LDS', 0) / w:7.1f} {c.get('SQ_INSTS_VMEM_RD', 0) / w:7.1f} "
          f"{c.get('SQ_INSTS_VMEM_WR', 0) / w:7.1f} {4 * wc / w:9.0f} "
          f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
          f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f}")
