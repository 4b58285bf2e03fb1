"""Kernel statistics from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace -d DIR -o NAME` on ROCm 7.2: DIR/.../NAME_results.db):
per kernel name the launches, average / min / max and total duration and the
share of all kernel time (the --stats summary's columns), plus, when the trace
has them, the memory copies by direction.  Usage: kstats_db.py DB [--batches N]
(N: per-batch totals divided by N as well)."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    nb = int(sys.argv[sys.argv.index("--batches") + 1]) if "--batches" in sys.argv else 0
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[5] for r in rows) or 1
    for name, n, avg, mn, mx, s in rows:
        extra = f"  per batch {s / nb / 1e6:9.2f} ms" if nb else ""
        print(f"{name[:44]:44s} {n:6d} avg {avg / 1e6:9.3f} ms  min {mn / 1e6:9.3f}  max {mx / 1e6:9.3f}  "
              f"total {s / 1e6:10.2f} ms {100 * s / tot:5.1f} %{extra}")
    try:
        cp = c.execute("select src_agent_type, dst_agent_type, count(*), sum(size), sum(duration), avg(duration) "
                       "from memory_copies group by src_agent_type, dst_agent_type").fetchall()
        for src, dst, n, size, dur, avg in cp:
            print(f"copy {src}->{dst}: {n} copies, {size / 1e9:.2f} GB, {dur / 1e6:.1f} ms total, "
                  f"avg {avg / 1e3:.1f} us, {size / max(dur, 1):.1f} GB/s while active")
    except sqlite3.OperationalError:
        pass


if __name__ == "__main__":
    main()
