"""Per-kernel statistics from a rocprofv3 results database (the `kernels` view):
calls, average / total ms, VGPRs and LDS, sorted by total time.
usage: python scripts/kstats.py run_results.db [more.db ...] [--csv out.csv]"""
import sqlite3
import sys


def kernel_stats(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(duration), sum(duration), max(vgpr_count), max(lds_size) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    return [(n.split("(")[0].replace("void ", ""), k, a / 1e6, s / 1e6, v, l) for n, k, a, s, v, l in rows]


def main():
    args = sys.argv[1:]
    out = None
    if "--csv" in args:
        i = args.index("--csv")
        out = args[i + 1]
        args = args[:i] + args[i + 2:]
    lines = []
    for p in args:
        print(f"== {p}")
        for n, k, a, s, v, l in kernel_stats(p):
            print(f"{n[:48]:48s} {k:6d} avg {a:9.3f} ms  total {s:10.2f} ms  vgpr {v:4d} lds {l}")
            lines.append(f'"{p}","{n}",{k},{a:.4f},{s:.3f},{v},{l}')
    if out:
        with open(out, "w") as f:
            f.write("db,kernel,calls,avg_ms,total_ms,vgpr,lds\n" + "\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
