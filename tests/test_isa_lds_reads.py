"""Static check of the built library's machine code (no GPU): the kernels that issue LDS reads as
inline asm and wait for them later with a counted `s_waitcnt lgkmcnt(N)` (attention forward stages
5 / 7, the LDS-DMA dK/dV backward kernel) are only
correct if nothing reads or overwrites a read's destination registers before that wait. The
compiler does not know the data lands late: a spill store, a register copy or a branch placed
between the read and its wait would use stale values (round 4: a spill store of in-flight
transposed fragments in the pipelined forward's tail gave wrong rows). Disassembles the device
code of libcullavo_hip.so with llvm-objdump and scans every LDS read of those kernels forward to
the first lgkmcnt wait."""
import functools
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


@functools.lru_cache(maxsize=1)
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
                    am = re.search(r"//\s*([0-9A-Fa-f]+):", line)
                    body.append((int(am.group(1), 16) if am else -1, line.split("//")[0].strip()))
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


# the dK/dV kernels that store dS^T while the next tile's LDS-DMA is in flight (DS_OUT = DMA = true):
# their loop ends with a hand-counted `s_waitcnt vmcnt(4)` that lets exactly the tile's four dS^T stores
# stay outstanding (attention.hip, the DMA branch at the end of the tile loop)
DS_OUT_DMA_KERNELS = ("attn_bwd_dkdv8_kILi128ELb1ELb1ELb1E", "attn_bwd_dkdv8_kILi128ELb0ELb1ELb1E",
                      "attn_bwd_dkdv8_kILi64ELb1ELb1ELb1E", "attn_bwd_dkdv8_kILi64ELb0ELb1ELb1E")


def _counted_vmcnt_problems(body, n=4):
    """every `s_waitcnt vmcnt(n)` must have, on EVERY control-flow path into it, at least n
    vector-memory STORES issued after the last vector-memory load (the LDS-DMA pieces and the aux
    loads are then retired by the wait); a load among the n youngest (the compiler reordering a load
    behind the stores) is a silent race. Paths are followed backwards through fall-through edges and
    SOPP branches (target = pc + 4 + 4 * simm16)."""
    index = {addr: i for i, (addr, _) in enumerate(body)}
    preds = {i: [] for i in range(len(body))}
    for i, (addr, ins) in enumerate(body):
        op = ins.split()[0] if ins else ""
        if op.startswith("s_cbranch") or op == "s_branch":
            simm = int(ins.split()[1])
            simm = simm - 65536 if simm >= 32768 else simm
            t = index.get(addr + 4 + 4 * simm)
            if t is not None:
                preds[t].append(i)
        if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and i + 1 < len(body):
            preds[i + 1].append(i)

    def min_stores(start):
        best = None
        seen = set()
        stack = [(p, 0) for p in preds[start]]
        while stack:
            j, cnt = stack.pop()
            if (j, cnt) in seen or cnt > n:
                continue
            seen.add((j, cnt))
            op = body[j][1].split()[0] if body[j][1] else ""
            if op.startswith(("global_store", "buffer_store", "scratch_store", "flat_store")):
                cnt += 1
            elif op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load", "global_atomic",
                                "buffer_atomic")):
                best = cnt if best is None else min(best, cnt)
                continue
            if cnt >= n:
                continue  # enough stores on this path already
            stack.extend((p, cnt) for p in preds[j])
        return n if best is None else best

    bad = []
    for i, (_, ins) in enumerate(body):
        if re.match(rf"s_waitcnt vmcnt\({n}\)", ins):
            m = min_stores(i)
            if m < n:
                bad.append((i, ins, f"a path with {m} stores after its last load"))
    return bad


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_dkdv_dsout_counted_vmcnt_leaves_only_the_stores():
    """the LDS-DMA dK/dV kernel's `vmcnt(4)` assumes the four dS^T stores are the only
    vector-memory ops issued after the next tile's DMA and aux loads; checked on the built code."""
    kernels = _kernels()
    checked = [n for n in kernels if any(k in n for k in DS_OUT_DMA_KERNELS)]
    assert len(checked) == len(DS_OUT_DMA_KERNELS), checked
    problems = {}
    for n in checked:
        waits = [ins for _, ins in kernels[n] if re.match(r"s_waitcnt vmcnt\(4\)", ins)]
        assert waits, f"{n}: no vmcnt(4) wait found"
        bad = _counted_vmcnt_problems(kernels[n])
        if bad:
            problems[n] = bad[:3]
    assert not problems, problems


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_inline_asm_lds_reads_not_used_before_their_wait():
    kernels = _kernels()
    checked = [n for n in kernels if any(k in n for k in ASM_READ_KERNELS)]
    assert any("attn_fwd_pipe_k" in n for n in checked) and any("attn_fwd_kILi128ELb1ELi5E" in n for n in checked)
    problems = {}
    for n in checked:
        bad = _early_uses([ins for _, ins in kernels[n]], allow_branch=False)
        if bad:
            problems[n] = bad[:3]
    assert not problems, problems
