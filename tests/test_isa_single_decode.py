"""ISA check of the single-stream decoder's hand-scheduled scalar loads
(CPU test on the built libfsehip.so; no GPU needed).

single_decode_kernel (fse_decode.hip, fent_issue* / fent_wait* / fstep)
issues `s_load_dwordx2` in one asm statement and waits for it with
`s_waitcnt lgkmcnt(0)` in a later one.  The compiler does not track those
loads, so the output is right only if no instruction touches a load's
destination SGPRs while it is in flight: no copy, spill or reuse of them on
any control-flow path between the load and the wait.  `fstep` also
hard-codes s[98:99] as its bit-field temporary, so nothing else may use
s98/s99 in the kernel.  This test disassembles the shipped code object
and checks both on the control-flow graph, so a toolchain whose register
allocation breaks either assumption fails here instead of corrupting
decodes.
"""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "entropy_coders_amd", "libfsehip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

INSN = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):")
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def _code_objects(path):
    """The gfx950 code objects in a host binary's offload bundles."""
    data = open(path, "rb").read()
    out, i = [], data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode(errors="replace")
            p += tl
            if "gfx950" in triple and size:
                out.append(data[i + off:i + off + size])
        i = data.find(MAGIC, i + len(MAGIC))
    return out


def _sregs(ops):
    regs = set()
    for a, b, one in SREG.findall(ops):
        if one:
            regs.add(int(one))
        else:
            regs.update(range(int(a), int(b) + 1))
    return regs


def _functions(asm, name_part):
    """{symbol: [(addr, opcode, operands)]} for the functions matching name_part."""
    funcs, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1) if name_part in m.group(1) else None
            if cur:
                funcs[cur] = []
            continue
        if cur is None:
            continue
        m = INSN.match(line)
        if m:
            funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2)))
    return funcs


def _successors(insns, idx):
    addr, op, ops = insns[idx]
    nxt = [idx + 1] if idx + 1 < len(insns) else []
    if op == "s_endpgm":
        return []
    if op.startswith(("s_branch", "s_cbranch")):
        simm = int(ops.split()[0])
        if simm >= 1 << 15:
            simm -= 1 << 16
        target = addr + 4 + 4 * simm
        tgt = [j for j, (a, _, _) in enumerate(insns) if a == target]
        assert tgt, f"branch target {target:#x} not an instruction"
        return tgt if op == "s_branch" else sorted(set(tgt + nxt))
    return nxt


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.skip("libfsehip.so not built")
    if not shutil.which(OBJDUMP):
        pytest.skip("llvm-objdump not found")
    found = {}
    d = tmp_path_factory.mktemp("co")
    for k, co in enumerate(_code_objects(LIB)):
        if b"single_decode_kernel" not in co:
            continue
        f = d / f"co{k}.elf"
        f.write_bytes(co)
        asm = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(f)], check=True, capture_output=True,
                             text=True).stdout
        found.update(_functions(asm, "single_decode_kernel"))
    assert len(found) == 2, sorted(found)  # NS = 1 and NS = 2
    return found


def test_scalar_loads_untouched_until_waited(kernels):
    checked = 0
    for name, insns in kernels.items():
        for i, (addr, op, ops) in enumerate(insns):
            if op != "s_load_dwordx2":
                continue
            dst = _sregs(ops.split(",")[0])
            # walk every path from the load to a wait that drains lgkmcnt
            seen, todo = set(), list(_successors(insns, i))
            while todo:
                j = todo.pop()
                if j in seen:
                    continue
                seen.add(j)
                a, o, x = insns[j]
                if o == "s_waitcnt" and "lgkmcnt(0)" in x:
                    continue
                assert not (dst & _sregs(x)), (
                    f"{name}: {op} {ops} at {addr:#x} in flight while {o} {x} at {a:#x} touches its registers")
                todo.extend(_successors(insns, j))
            checked += 1
    assert checked >= 8, checked  # the hand-issued loads of both kernels


def test_fstep_scratch_pair_private(kernels):
    uses = 0
    for name, insns in kernels.items():
        for i, (addr, op, ops) in enumerate(insns):
            if not ({98, 99} & _sregs(ops)):
                continue
            if op == "s_bfe_u64" and ops.startswith("s[98:99],"):
                nxt = insns[i + 1]
                assert nxt[1] == "s_lshl3_add_u32" and re.match(r"s\d+, s98, ", nxt[2]), (
                    f"{name}: s_bfe_u64 into s[98:99] at {addr:#x} not consumed at once: {nxt}")
                assert not ({98, 99} & _sregs(nxt[2].split(",")[0])), nxt
                uses += 1
            elif op == "s_lshl3_add_u32" and insns[i - 1][1] == "s_bfe_u64":
                continue
            else:
                pytest.fail(f"{name}: {op} {ops} at {addr:#x} uses fstep's s[98:99]")
    assert uses >= 4, uses


def test_checker_flags_a_copy_in_flight():
    """The walk itself: a copy of an in-flight destination behind a branch is caught."""
    asm = """0000000000000000 <_Zsingle_decode_kernelX>:
	s_load_dwordx2 s[22:23], s[16:17], s37                     // 000000000000: C0040588 00000025
	s_cbranch_scc1 1                                           // 000000000008: BF850001
	s_nop 0                                                    // 00000000000C: BF800000
	s_mov_b64 s[40:41], s[22:23]                               // 000000000010: BEA80116
	s_waitcnt lgkmcnt(0)                                       // 000000000014: BF8CC07F
	s_endpgm                                                   // 000000000018: BF810000
"""
    insns = _functions(asm, "single_decode_kernel")["_Zsingle_decode_kernelX"]
    assert [op for _, op, _ in insns][:2] == ["s_load_dwordx2", "s_cbranch_scc1"]
    assert _successors(insns, 1) == [2, 3]
    dst, hit = _sregs("s[22:23]"), False
    seen, todo = set(), list(_successors(insns, 0))
    while todo:
        j = todo.pop()
        if j in seen:
            continue
        seen.add(j)
        _, o, x = insns[j]
        if o == "s_waitcnt" and "lgkmcnt(0)" in x:
            continue
        hit |= bool(dst & _sregs(x))
        todo.extend(_successors(insns, j))
    assert hit
