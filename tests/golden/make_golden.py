"""Regenerate tests/golden/golden.json: SHA-256 and per-block sizes of the CPU
restatement's output on the committed inputs (regression pins of the oracle;
the external pins are the reference-run sizes recorded in SURVEY.md section 6,
checked in tests/test_oracle.py).  Run: python tests/golden/make_golden.py"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import fastqueeze_amd as fq  # noqa: E402  (host cut/parse only; no GPU)
import oracle_py  # noqa: E402
import synth  # noqa: E402

CASES = {
    "test_pe": dict(files=("ERR2755197_test_1.fq", "ERR2755197_test_2.fq")),
    "test_se": dict(files=("ERR2755197_test_1.fq",)),
    "test_pe_600k": dict(files=("ERR2755197_test_1.fq", "ERR2755197_test_2.fq"), bs=600000),
    "synth_pe_4k": dict(synth=dict(n_reads=4000, paired=True, seed=7)),
    "synth_pe_4k_s4": dict(synth=dict(n_reads=4000, paired=True, seed=7), slevel=4),
    "synth_se_4k_q3": dict(synth=dict(n_reads=4000, seed=9), qlevel=3),
    "edge_se": dict(edge=True),
    "edge_se_s9": dict(edge=True, slevel=9),
    "test_pe_lossy_115": dict(files=("ERR2755197_test_1.fq", "ERR2755197_test_2.fq"), lossy=1.15),
    "synth_se_lossy_16": dict(synth=dict(n_reads=3000, seed=13), lossy=1.6),
    "synth_long_70k": dict(synth=dict(n_reads=12, seed=5, read_len=70000)),
}


def inputs(case):
    if "files" in case:
        ts = [open(os.path.join(HERE, f), "rb").read() for f in case["files"]]
        return ts[0], (ts[1] if len(ts) > 1 else None)
    if "synth" in case:
        return synth.generate(**case["synth"])
    return synth.edge_cases(), None


def run_case(case):
    t1, t2 = inputs(case)
    blocks = fq.blocks_from_fastq(t1, t2, case.get("bs", fq.BLOCK_SIZE))
    tmpl = oracle_py.analyze_ids(blocks[0], t2 is None)
    outs = [oracle_py.encode_block(b, case.get("slevel", 3), case.get("qlevel", 2), True, int(tmpl[0]),
                                   case.get("lossy", 0.0))
            for b in blocks]
    return blocks, tmpl, outs


def main():
    res = {}
    for name, case in CASES.items():
        blocks, tmpl, outs = run_case(case)
        res[name] = dict(case=case, bin_mode=int(tmpl[0]), petype=int(tmpl[1]),
                         blocks=[len(o) for o in outs],
                         sha256=hashlib.sha256(b"".join(outs)).hexdigest())
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v["blocks"] for k, v in res.items()}))


if __name__ == "__main__":
    main()
