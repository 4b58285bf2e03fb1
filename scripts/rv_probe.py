"""Pass-R placement and speed from SA_RV_PROBE files (k_coder_rv's per-wave
probe, sa_engine.hip write_rv_probe): per batch the launch's span, its waves'
durations and shader clock, and how often a chain wave shared its SIMD (or its
CU) with another pass-R wave that ran at the same time (of any batch).
usage: python scripts/rv_probe.py PROBE_FILE [more files...]"""
import collections
import statistics
import sys


def load(path):
    waves = []
    for ln in open(path):
        f = ln.split()
        if len(f) < 18:
            continue
        waves.append({"ctx": f[0], "batch": int(f[1]), "wave": int(f[2]), "t0": float(f[3]), "t1": float(f[4]),
                      "mhz": float(f[5]), "xcc": int(f[7]), "se": int(f[9]), "cu": int(f[11]), "simd": int(f[13]),
                      "slot": int(f[15]), "chains": int(f[17]), "sh": int(f[19]) if len(f) > 19 else 0})
    return waves


def report(path):
    ws = load(path)
    if not ws:
        print(f"{path}: no waves")
        return
    by_batch = collections.defaultdict(list)
    for w in ws:
        by_batch[w["batch"]].append(w)
    # SIMD / CU sharing: for each wave, the largest number of other pass-R waves
    # on its SIMD (CU) overlapping it, weighted by overlap time
    by_simd = collections.defaultdict(list)
    by_cu = collections.defaultdict(list)
    for w in ws:
        by_simd[(w["xcc"], w["se"], w["sh"], w["cu"], w["simd"])].append(w)
        by_cu[(w["xcc"], w["se"], w["sh"], w["cu"])].append(w)

    def shared_frac(w, group):
        ov = 0.0
        for o in group:
            if o is w:
                continue
            a, b = max(w["t0"], o["t0"]), min(w["t1"], o["t1"])
            if b > a:
                ov += b - a
        return ov / max(w["t1"] - w["t0"], 1e-9)

    print(f"== {path}: {len(by_batch)} batches, {len(ws)} waves, "
          f"{len(by_simd)} SIMDs, {len(by_cu)} CUs used")
    print("batch  span_ms  waves  long_ms(med/max)  MHz(med/min)  simd_shared  cu_waves(med)")
    for b in sorted(by_batch):
        bw = by_batch[b]
        t0, t1 = min(w["t0"] for w in bw), max(w["t1"] for w in bw)
        longs = [w for w in bw if w["chains"] == 1]
        d = [(w["t1"] - w["t0"]) / 1e3 for w in longs] or [0.0]
        mhz = [w["mhz"] for w in bw if w["mhz"] > 0] or [0.0]
        sh = [shared_frac(w, by_simd[(w["xcc"], w["se"], w["sh"], w["cu"], w["simd"])]) for w in longs] or [0.0]
        cuw = [len([o for o in by_cu[(w["xcc"], w["se"], w["sh"], w["cu"])] if o["t0"] < w["t1"] and o["t1"] > w["t0"]])
               for w in longs] or [0]
        print(f"{b:5d} {(t1 - t0) / 1e3:8.1f} {len(bw):6d}   {statistics.median(d):7.1f} / {max(d):7.1f}"
              f"   {statistics.median(mhz):6.0f} / {min(mhz):6.0f}   {statistics.mean(sh):8.3f}   "
              f"{statistics.median(cuw):5.1f}")


for p in sys.argv[1:]:
    report(p)
