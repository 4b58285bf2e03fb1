"""The compiled pass-R kernel keeps its SMEM operand buffers to itself.

k_coder_rv<6> (sa_kernels.hip, coder_rg_chain) loads each group of 16
symbols' (m, tf) pairs with s_load into fixed SGPRs, s[36:99], declared as
clobbers of its inline asm; the loads land while the previous group's steps
run.  Between two such asm blocks the compiler believes those registers free:
if code it generates there used one of them, an in-flight load would overwrite
it (or it the loaded operands).  This test compiles the library's device code
and checks that, in the layout of the kernel, every instruction outside the
asm that names s36..s99 lies in a region where no load is in flight: after the
"sa_rg_drained" marker (s_waitcnt lgkmcnt(0)) and before the next
"sa_rg_first" marker (the re-issued first load), i.e. seg_retry's code.
CPU only: hipcc cross-compiles for gfx950 here.
"""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "fastqueeze_amd", "csrc", "sa_engine.hip")


def _hipcc():
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    return None


def armed_uses(asm_text: str, kernel_re: str = r"k_coder_rvILi6E"):
    names = re.findall(r"^(_Z\w*" + kernel_re + r"\w*):", asm_text, re.M)
    assert names, "k_coder_rv<6> not in the device code"
    body = asm_text[asm_text.index(names[0] + ":"):]
    body = body[: body.index(".Lfunc_end")]
    inasm = armed = False
    bad, uses, firsts = [], 0, 0
    for line in body.split("\n"):
        s = line.strip()
        if "sa_rg_first" in s:
            armed = True
            firsts += 1
        if "sa_rg_drained" in s:
            armed = False
        if s.startswith(";;#ASMSTART"):
            inasm = True
            continue
        if s.startswith(";;#ASMEND"):
            inasm = False
            continue
        if inasm or not s or s.startswith((";", ".")):
            continue
        hit = any(int(b) >= 36 and int(a) <= 99 for a, b in re.findall(r"\bs\[(\d+):(\d+)\]", s))
        hit = hit or any(36 <= int(a) <= 99 for a in re.findall(r"\bs(\d+)\b", s))
        uses += hit
        if hit and armed:
            bad.append(s)
    return bad, uses, firsts


def test_pass_r_smem_buffers_untouched(tmp_path):
    hipcc = _hipcc()
    if hipcc is None:
        pytest.skip("hipcc not available")
    out = tmp_path / "sa_engine.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-o", str(out), SRC], check=True, capture_output=True)
    bad, uses, firsts = armed_uses(out.read_text())
    assert firsts >= 2   # the chain's first load and the one after a retry
    assert not bad, "compiler code uses the pass-R operand buffers while loads are in flight:\n" + "\n".join(bad[:10])


def test_checker_flags_a_use_in_flight():
    asm = """_ZN2sa10k_coder_rvILi6EEEvPKv:
\t;;#ASMSTART
\t; sa_rg_first
\ts_load_dwordx16 s[36:51], s[2:3], 0x0 glc
\t;;#ASMEND
\ts_mov_b32 s40, 0
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t; sa_rg_drained
\t;;#ASMEND
\ts_mov_b32 s41, 0
.Lfunc_end0:
"""
    bad, uses, firsts = armed_uses(asm)
    assert bad == ["s_mov_b32 s40, 0"] and uses == 2 and firsts == 1
