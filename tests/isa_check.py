"""Static check of the hand-counted memory waits in the gfx950 ISA of
usnetd_amd/csrc/usn_device.hip (test infrastructure, CPU only).

The rx hot path issues its table-slot, displacement and header loads as
inline asm and waits for them with explicit `s_waitcnt vmcnt(N)` counts
(hipcc's own waits would be vmcnt(0) and drain the header DMA in flight).
That is correct only while, on every path from a load to the wait meant for
it, at least N vector-memory instructions are issued after the load (vmcnt
completes in issue order), and no instruction touches the load's destination
registers before a wait that covers it.  A compiler change or an innocent
edit (a spill, a hoisted load, a copy of an in-flight register) breaks that
silently; this module re-derives both facts from the emitted assembly.

For every VGPR-destination load inside an inline-asm block it walks every
control-flow path forward from the load (both ways at each conditional
branch) counting the vector-memory instructions issued after it (Y), until
the first `s_waitcnt` whose vmcnt(N) has N <= Y (the load is then complete).
It reports
  * hazard: an instruction naming one of the load's destination registers
    before such a wait (a read, a copy, or a write the load's late return
    would clobber);
  * loose:  for the last load of an asm block (a block may issue a pair that
    one wait covers), the covering wait is an inline-asm wait with 0 < N < Y,
    i.e. the hand count no longer equals the instructions actually issued in
    between (the wait is then stricter than intended: slower, and a sign the
    count is stale).  vmcnt(0) is a drain and names no count to go stale.
A path through an instruction marked `; usn_rare` in its asm (a rare path's
extra store, which only makes the waits after it stricter) reports no loose
wait.  LDS-DMA loads (global_load_lds, builtins) have no register destination and
are only counted as issued instructions here.
"""
from __future__ import annotations

import re
import subprocess
from dataclasses import dataclass, field

VMEM_PREFIX = ("global_", "buffer_", "flat_", "scratch_")
REG_RE = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")
WAIT_RE = re.compile(r"vmcnt\((\d+)\)")


@dataclass
class Insn:
    line: int
    text: str
    op: str
    args: str
    in_asm: bool
    block: int = -1    # inline-asm block index (-1: compiler code)
    rare: bool = False # an inline-asm instruction marked `; usn_rare` (a rare path's extra store)


@dataclass
class Func:
    name: str
    insns: list = field(default_factory=list)
    labels: dict = field(default_factory=dict)   # label -> index of the next insn


@dataclass
class Finding:
    func: str
    kind: str          # "hazard" | "loose"
    load_line: int
    load: str
    at_line: int
    at: str
    detail: str

    def __str__(self):
        return "%s %s: load @%d `%s` -> @%d `%s` (%s)" % (
            self.kind, self.func[:60], self.load_line, self.load, self.at_line, self.at, self.detail)


def regs(args: str) -> set:
    out = set()
    for m in REG_RE.finditer(args):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(asm_text: str) -> list:
    """Functions of an assembly file, with instructions and labels."""
    funcs, cur, in_asm, nblock = [], None, False, 0
    for ln, raw in enumerate(asm_text.splitlines(), 1):
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            nblock += 1
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(_Z[\w.$]+):", raw)
        if m:
            cur = Func(m.group(1))
            funcs.append(cur)
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        rare = "usn_rare" in s
        s = s.split(";", 1)[0].strip()
        if not s:
            continue
        m = re.match(r"^(\.L\w+):", s)
        if m:
            cur.labels[m.group(1)] = len(cur.insns)
            continue
        if s.startswith("."):
            continue
        op, _, args = s.partition(" ")
        cur.insns.append(Insn(ln, s, op, args.strip(), in_asm, nblock if in_asm else -1, rare))
    return funcs


def is_vmem(op: str) -> bool:
    return op.startswith(VMEM_PREFIX)


def vmem_dest(ins: Insn) -> set:
    """VGPRs a load writes (its first operand); stores, LDS-DMA and atomics
    without a return value write none."""
    if not is_vmem(ins.op) or "_load" not in ins.op or "_lds" in ins.op:
        return set()
    first = ins.args.split(",", 1)[0]
    return regs(first)


def successors(f: Func, i: int) -> list:
    ins = f.insns[i]
    if ins.op in ("s_endpgm", "s_setpc_b64", "s_trap"):
        return []
    tgt = ins.args.split(",")[0].strip() if ins.op.startswith(("s_branch", "s_cbranch")) else None
    if ins.op == "s_branch":
        return [f.labels[tgt]] if tgt in f.labels else []
    nxt = [i + 1] if i + 1 < len(f.insns) else []
    if ins.op.startswith("s_cbranch") and tgt in f.labels:
        nxt.append(f.labels[tgt])
    return nxt


def check_load(f: Func, i: int, tight: bool, max_steps=20000) -> list:
    """Hazards of load i on every path; with `tight` (the last load of its asm
    block), also inline-asm covering waits whose count is below the
    instructions issued since (a drain, vmcnt(0), is exempt)."""
    load = f.insns[i]
    dest = vmem_dest(load)
    out = []
    # (instruction, issued since the load, a rare instruction on the path)
    stack = [(j, 0, False) for j in successors(f, i)]
    seen = set()
    steps = 0
    while stack and steps < max_steps:
        j, y, rare = stack.pop()
        if (j, y, rare) in seen:
            continue
        seen.add((j, y, rare))
        steps += 1
        ins = f.insns[j]
        if ins.op == "s_waitcnt":
            m = WAIT_RE.search(ins.args)
            n = int(m.group(1)) if m else None
            if n is None and ins.args.strip() == "0":
                n = 0
            if n is not None and n <= y:
                if tight and ins.in_asm and 0 < n < y and not rare:
                    out.append(Finding(f.name, "loose", load.line, load.text, ins.line, ins.text,
                                       "%d vector-memory instructions issued after the load, "
                                       "wait counts %d" % (y, n)))
                continue                     # the load is complete on this path
        elif dest & regs(ins.args):
            out.append(Finding(f.name, "hazard", load.line, load.text, ins.line, ins.text,
                               "destination v%s named before a covering wait (%d issued after)"
                               % (sorted(dest & regs(ins.args)), y)))
            continue
        if is_vmem(ins.op):
            y = min(y + 1, 63)
        rare = rare or ins.rare
        for k in successors(f, j):
            stack.append((k, y, rare))
    return out


def check(asm_text: str, func_filter=lambda name: True) -> tuple:
    """(findings, number of inline-asm VGPR loads checked)"""
    findings, n = [], 0
    for f in parse(asm_text):
        if not func_filter(f.name):
            continue
        for i, ins in enumerate(f.insns):
            if ins.in_asm and vmem_dest(ins):
                n += 1
                last = not any(vmem_dest(x) for x in f.insns[i + 1:i + 8] if x.block == ins.block)
                findings.extend(check_load(f, i, last))
    # one finding per (load, wait) pair
    uniq = {(x.func, x.kind, x.load_line, x.at_line): x for x in findings}
    return list(uniq.values()), n


def compile_asm(src: str, out: str, defines=()) -> str:
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "-S", "--offload-device-only", "-o", out, src] + ["-D" + d for d in defines]
    subprocess.run(cmd, check=True, capture_output=True)
    with open(out) as fh:
        return fh.read()
