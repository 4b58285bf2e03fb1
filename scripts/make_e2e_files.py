"""Writes the bench's end-to-end FASTQ pair (bench.make_batch's generator, seeds
1000 + batch id) to DIR/r1.fq and DIR/r2.fq: BATCHES distinct batches, the
whole text repeated REPEAT times.  usage: make_e2e_files.py DIR BATCHES REPEAT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

if __name__ == "__main__":
    import synth
    d, nb, rep = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    os.makedirs(d, exist_ok=True)
    paths = [os.path.join(d, "r1.fq"), os.path.join(d, "r2.fq")]
    for p in paths:
        open(p, "wb").close()
    for g in range(nb):
        t1, t2 = synth.generate(5_000_000, read_len=150, paired=True, seed=1000 + g, workers=16, x_span=8)
        for p, t in zip(paths, (t1, t2)):
            with open(p, "ab") as f:
                f.write(t)
        print(f"batch {g} written", flush=True)
    for p in paths:
        size0 = os.path.getsize(p)
        with open(p, "ab") as dst:
            for _ in range(rep - 1):
                with open(p, "rb") as src:
                    left = size0
                    while left > 0:
                        chunk = src.read(min(left, 256 << 20))
                        dst.write(chunk)
                        left -= len(chunk)
    print("sizes", [os.path.getsize(p) for p in paths], flush=True)
