"""amd-smi metric -v -c -p --json samples (scripts/gpu_r5b.sh's sampler: a
't <epoch>' line, then one JSON document per sample) -> one line per sample:
time, socket power, gfx clocks (min/max over the XCDs), and the throttle
record: PPT / thermal / PROCHOT / HBM violation activity and the per-XCD
"gfx clock below host limit" activities (power, thermal, total) and the
low-utilization activity (amd-smi's *_VIOLATION_ACTIVITY: % of the interval
since the previous read)."""
import json
import sys


def docs(path):
    t, buf = None, []
    for ln in open(path):
        if ln.startswith("t "):
            if buf and t is not None:
                try:
                    yield t, json.loads("".join(buf))
                except json.JSONDecodeError:
                    pass
            t, buf = float(ln.split()[1]), []
        else:
            buf.append(ln)
    if buf and t is not None:
        try:
            yield t, json.loads("".join(buf))
        except json.JSONDecodeError:
            pass


def val(x):
    if isinstance(x, dict):
        return x.get("value")
    return x


def main():
    for path in sys.argv[1:]:
        print(f"== {path}")
        print("   t_s  power_W  gfx_MHz(min/max)  ppt%  therm%  prochot%  hbm%  below_host_power%  "
              "below_host_thermal%  below_host_total%  low_util%")
        t0 = None
        for t, d in docs(path):
            g = d["gpu_data"][0] if "gpu_data" in d else d[0]
            t0 = t0 if t0 is not None else t
            clk = [val(v["clk"]) for k, v in g.get("clock", {}).items() if k.startswith("gfx_")]
            clk = [c for c in clk if isinstance(c, (int, float))]
            v = g.get("violation", g.get("throttle", {}))

            def pct(key):
                x = v.get(key)
                if isinstance(x, dict):   # per-XCP lists
                    x = list(x.values())[0]
                if isinstance(x, list):
                    xs = [val(e) for e in x]
                    xs = [e for e in xs if isinstance(e, (int, float))]
                    return f"{min(xs):.0f}-{max(xs):.0f}" if xs else "NA"
                x = val(x)
                return f"{x:.0f}" if isinstance(x, (int, float)) else "NA"
            print(f"{t - t0:6.1f}  {val(g['power']['socket_power']):>7}  "
                  f"{(min(clk) if clk else 0):>7}/{(max(clk) if clk else 0):<7}  "
                  f"{pct('ppt_violation_activity'):>4}  {pct('socket_thermal_violation_activity'):>6}  "
                  f"{pct('prochot_violation_activity'):>8}  {pct('hbm_thermal_violation_activity'):>4}  "
                  f"{pct('gfx_clk_below_host_limit_power_violation_activity'):>17}  "
                  f"{pct('gfx_clk_below_host_limit_thermal_violation_activity'):>19}  "
                  f"{pct('total_gfx_clk_below_host_limit_violation_activity'):>17}  "
                  f"{pct('low_utilization_violation_activity'):>9}")


if __name__ == "__main__":
    main()
