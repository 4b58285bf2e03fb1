"""Run seqarc_amd -c on one input several times under given environments and
report, per run: the wall clock around the process, the command line's own
clock, the exit -> reaped time (bench.py's exit_to_reaped_s) and the
exit-probe line (SA_CLI_EXIT_PROBE=1).  Round 6, call r6z.

    python3 scripts/cli_exit_ab.py DIR OUT_TXT name=ENV[,ENV...] ...
"""
import os
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(R, "fastqueeze_amd", "bin", "seqarc_amd")


def run(d, env_extra):
    cmd = [CLI, "-c", "-f", "-v", "-t", "16", "-1", "r1.fq", "-2", "r2.fq", "-o", "e2e", "--contexts", "5",
           "--batch", "69", "--slevel", "3", "--qlevel", "2", "--block-size", "50"]
    env = dict(os.environ, **env_extra)
    time.sleep(3)
    t0, m0 = time.perf_counter(), time.monotonic()
    r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=120)
    wall, m1 = time.perf_counter() - t0, time.monotonic()
    res = {"rc": r.returncode, "wall_s": round(wall, 3)}
    for ln in r.stderr.splitlines():
        if "MB/s" in ln and "block(s)" in ln:
            res["cli_s"] = float(ln.rsplit(",", 2)[1].split()[0])
        if "monotonic clock: main" in ln:
            mm, me = (float(x.split()[-1]) for x in ln.split(": ", 2)[2].split(", "))
            res["start_to_main_s"] = round(mm - m0, 3)
            res["exit_to_reaped_s"] = round(m1 - me, 3)
        if "exit probe" in ln or "contexts ready" in ln or "blocks written" in ln:
            res.setdefault("lines", []).append(ln.split(": ", 1)[1])
    if r.returncode == 0 and os.environ.get("AB_MD5"):
        import hashlib
        h = hashlib.md5()
        with open(os.path.join(d, "e2e.arc"), "rb") as f:
            for chunk in iter(lambda: f.read(64 << 20), b""):
                h.update(chunk)
        res["arc_md5"] = h.hexdigest()
    try:
        os.remove(os.path.join(d, "e2e.arc"))
    except OSError:
        pass
    if r.returncode != 0:
        res["stderr"] = r.stderr[-1500:]
    return res


def main():
    d, out = sys.argv[1], sys.argv[2]
    with open(out, "a") as f:
        for spec in sys.argv[3:]:
            name, _, envs = spec.partition("=")
            env = dict(e.split(":", 1) for e in envs.split(",") if e)
            res = run(d, env)
            f.write(f"{name} {env} {res}\n")
            f.flush()
            print(name, res, flush=True)
            if res["rc"] != 0:
                sys.exit(res["rc"])


if __name__ == "__main__":
    main()
