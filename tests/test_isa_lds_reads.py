"""Static check of the built library's machine code (no GPU): the kernels that issue LDS reads as
inline asm and wait for them later with a counted `s_waitcnt lgkmcnt(N)` (attention forward stages
5 / 7, the LDS-DMA dK/dV backward kernel) are only
correct if nothing reads or overwrites a read's destination registers before that wait. The
compiler does not know the data lands late: a spill store, a register copy or a branch placed
between the read and its wait would use stale values (round 4: a spill store of in-flight
transposed fragments in the pipelined forward's tail gave wrong rows). Disassembles the device
code of libcullavo_hip.so with llvm-objdump and scans every LDS read of those kernels forward to
the first lgkmcnt wait."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "causal-unified-language-vision_amd", "libcullavo_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
# kernels whose LDS reads are inline asm with deferred counted waits
ASM_READ_KERNELS = ("attn_fwd_pipe_k", "attn_fwd_kILi128ELb1ELi5E", "attn_fwd_kILi64ELb0ELi5E",
                    # round 5: the LDS-DMA dK/dV kernel's fragment reads (DMA = true instantiations)
                    "attn_bwd_dkdv8_kILi128ELb1ELb1ELb1E", "attn_bwd_dkdv8_kILi128ELb1ELb0ELb1E",
                    "attn_bwd_dkdv8_kILi128ELb0ELb1ELb1E", "attn_bwd_dkdv8_kILi128ELb0ELb0ELb1E",
                    "attn_bwd_dkdv8_kILi64ELb1ELb1ELb1E", "attn_bwd_dkdv8_kILi64ELb0ELb1ELb1E",
                    "attn_bwd_dkdv8_kILi64ELb1ELb0ELb1E", "attn_bwd_dkdv8_kILi64ELb0ELb0ELb1E")


def _regs(spec):
    m = re.match(r"v\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", spec)
    return {int(m.group(1))} if m else set()


def _operands(ins):
    parts = ins.replace(",", " ").split()
    return parts[0], parts[1:]


def _kernels():
    tmp = tempfile.mkdtemp()
    try:
        so = os.path.join(tmp, "lib.so")
        shutil.copy(LIB, so)
        subprocess.run([OBJDUMP, "--offloading", so], cwd=tmp, check=True, capture_output=True, timeout=300)
        out = {}
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            dis = subprocess.run([OBJDUMP, "-d", os.path.join(tmp, f)], check=True, capture_output=True, text=True,
                                 timeout=300).stdout
            if not any(k in dis for k in ASM_READ_KERNELS):
                continue
            name, body = None, []
            for line in dis.split("\n"):
                m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
                if m:
                    if name:
                        out[name] = body
                    name, body = m.group(1), []
                elif name and line.startswith("\t"):
                    body.append(line.split("//")[0].strip())
            if name:
                out[name] = body
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _early_uses(body, allow_branch=False):
    bad = []
    for i, ins in enumerate(body):
        if not ins.startswith("ds_read"):
            continue
        _, ops = _operands(ins)
        dest = _regs(ops[0])
        for j in range(i + 1, min(i + 600, len(body))):
            nxt = body[j]
            op, args = _operands(nxt)
            if op == "s_waitcnt" and "lgkmcnt" in nxt:
                break
            if op.startswith("s_cbranch") or op == "s_branch" or op == "s_setpc_b64":
                if not allow_branch:
                    bad.append((i, ins, j, nxt, "branch before the wait"))
                break
            srcs = set().union(*(_regs(a) for a in args[1:])) if len(args) > 1 else set()
            if op.startswith(("ds_", "buffer_", "global_", "scratch_")):
                # memory ops: every register operand is read except a load's destination
                srcs = set().union(*(_regs(a) for a in (args[1:] if "load" in op or "read" in op else args)))
            if dest & srcs:
                bad.append((i, ins, j, nxt, "read before the wait"))
                break
            if args and dest & _regs(args[0]) and not (op.startswith("ds_read") or "load" in op or op == "s_waitcnt"):
                bad.append((i, ins, j, nxt, "overwritten before the wait"))
                break
    return bad


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_inline_asm_lds_reads_not_used_before_their_wait():
    kernels = _kernels()
    checked = [n for n in kernels if any(k in n for k in ASM_READ_KERNELS)]
    assert any("attn_fwd_pipe_k" in n for n in checked) and any("attn_fwd_kILi128ELb1ELi5E" in n for n in checked)
    problems = {}
    for n in checked:
        bad = _early_uses(kernels[n], allow_branch=False)
        if bad:
            problems[n] = bad[:3]
    assert not problems, problems
