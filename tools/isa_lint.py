#!/usr/bin/env python3
"""ISA lint for the counted-wait LDS kernels (gemm3.hip / gemm4.hip).

The wide dequant GEMMs issue their LDS reads as inline asm and retire them with their own counted
``s_waitcnt lgkmcnt(N)`` (csrc/kernels/gemm_lds.h).  The compiler believes an asm read's result
is available the moment the asm statement ends, so two things can go silently wrong:

  * **clobber** -- a VALU/VMEM/LDS instruction WRITES a VGPR that is still the destination of an
    in-flight LDS read (the compiler recycled a dead read's register, or copied into it): when the
    LDS data lands it overwrites the newer value;
  * **stale read** -- an instruction READS such a VGPR before the wait that retires the read (the
    compiler moved a use, or inserted a copy, above the counted wait);

Scalar-memory loads the compiler schedules inside a counted window (kernel-argument loads for the
epilogue) are reported as information only: lgkmcnt counts LDS and SMEM together and SMEM may
return out of order, but an outstanding SMEM op only adds to the count, so ``lgkmcnt(N)`` still
means at most N LDS ops are outstanding -- the counted waits can over-wait, never under-wait.

The lint walks every kernel's control-flow graph (labels and ``s_branch`` / ``s_cbranch_*``) and
carries the ordered queue of in-flight LDS operations to a fixed point; ``s_waitcnt lgkmcnt(N)``
retires all but the N most recent.  LDS reads that return in order may overwrite one another
(write-after-write by a later LDS read of the same register is allowed).  The ``-Winline-asm``
warnings of the same compile are counted too (the ``m0`` clobber of the LDS-DMA helper).

Usage:  python tools/isa_lint.py [--asm FILE.s ...] [--src csrc/kernels/gemm4.hip ...] [-v]
With ``--src`` it runs ``hipcc --cuda-device-only -S`` itself (2-3 min for gemm4.hip).
Exit status 1 when there is any finding.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REG_RANGE = re.compile(r"\b([va])\[(\d+):(\d+)\]")
REG_ONE = re.compile(r"\b([va])(\d+)\b")
LABEL = re.compile(r"^(\.LBB\d+_\d+):")
FUNC = re.compile(r"^(_Z\w+):")
WAIT = re.compile(r"lgkmcnt\((\d+)\)")

# LDS ops that write a VGPR destination (their first operand)
DS_DEST = ("ds_read", "ds_load", "ds_bpermute", "ds_permute", "ds_swizzle", "ds_consume", "ds_append")
SMEM = ("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_dcache", "s_scratch_load",
        "s_atc_probe", "s_sendmsg")


def regs(text: str) -> set:
    out = set()
    for m in REG_RANGE.finditer(text):
        for i in range(int(m.group(2)), int(m.group(3)) + 1):
            out.add(f"{m.group(1)}{i}")
    text = REG_RANGE.sub(" ", text)
    for m in REG_ONE.finditer(text):
        out.add(f"{m.group(1)}{m.group(2)}")
    return out


def split_operands(ops: str) -> list:
    out, depth, cur = [], 0, ""
    for ch in ops:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


class Insn:
    __slots__ = ("line", "op", "text", "dst", "src", "asm", "kind", "wait", "target")

    def __init__(self, line, op, rest, asm):
        self.line, self.op, self.text, self.asm = line, op, (op + " " + rest).strip(), asm
        self.dst, self.src, self.kind, self.wait, self.target = set(), set(), "other", None, None
        operands = split_operands(rest.split(";")[0])
        if op.startswith("ds_"):
            self.kind = "lds"
            if op.startswith(DS_DEST) or "_rtn" in op:
                self.dst = regs(operands[0]) if operands else set()
                self.src = regs(",".join(operands[1:]))
            else:
                self.src = regs(",".join(operands))
        elif op.startswith(SMEM):
            self.kind = "smem"
        elif op == "s_waitcnt":
            m = WAIT.search(rest)
            if m:
                self.kind, self.wait = "wait", int(m.group(1))
        elif op == "s_branch" or op.startswith("s_cbranch"):
            self.kind = "branch"
            self.target = operands[0] if operands else None
        elif op in ("s_endpgm", "s_setpc_b64", "s_endpgm_saved"):
            self.kind = "end"
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            store = "store" in op or "_lds" in op or (("atomic" in op) and not re.search(r"\b(glc|sc0)\b", rest))
            if store:
                self.src = regs(",".join(operands))
            else:
                self.dst = regs(operands[0]) if operands else set()
                self.src = regs(",".join(operands[1:]))
        elif op.startswith("v_"):
            if operands:
                self.dst = regs(operands[0])
                self.src = regs(",".join(operands[1:]))
                if op.startswith(("v_mac", "v_fmac", "v_dot2c", "v_writelane")):
                    self.src |= self.dst
        # s_* other: no VGPR traffic


def parse(path: str):
    """{kernel: (insns, blocks)}; blocks: list of (label, start, end) over insns."""
    kernels = {}
    name, insns, labels, asm = None, [], {}, False
    with open(path) as f:
        for ln, raw in enumerate(f, 1):
            s = raw.strip()
            if name is None:
                m = FUNC.match(s)
                if m:
                    name, insns, labels = m.group(1), [], {}
                continue
            if s.startswith(".Lfunc_end"):
                kernels[name] = (insns, labels)
                name = None
                continue
            if s == ";;#ASMSTART":
                asm = True
                continue
            if s == ";;#ASMEND":
                asm = False
                continue
            m = LABEL.match(s)
            if m:
                labels[m.group(1)] = len(insns)
                continue
            if not s or s.startswith((";", ".", "//")):
                continue
            parts = s.split(None, 1)
            insns.append(Insn(ln, parts[0], parts[1] if len(parts) > 1 else "", asm))
    return kernels


def analyse(insns, labels, max_states=256):
    """Fixed-point walk; returns (findings, counted waits with SMEM in flight, overflow)."""
    starts = sorted(set([0] + list(labels.values()) +
                        [i + 1 for i, x in enumerate(insns) if x.kind in ("branch", "end")]))
    starts = [s for s in starts if s < len(insns)]
    block_of = {s: k for k, s in enumerate(starts)}
    ends = starts[1:] + [len(insns)]
    succ = []
    for k, (a, b) in enumerate(zip(starts, ends)):
        last = insns[b - 1]
        nxt = []
        if last.kind == "branch":
            t = labels.get(last.target)
            if t is not None and t in block_of:
                nxt.append(block_of[t])
            if last.op != "s_branch" and b < len(insns):
                nxt.append(block_of[b])
        elif last.kind != "end" and b < len(insns):
            nxt.append(block_of[b])
        succ.append(nxt)

    seen = defaultdict(set)
    findings, infos = {}, set()
    work = [(0, ((), False))]
    seen[0].add(((), False))
    overflow = False
    while work:
        k, (queue, smem) = work.pop()
        q = list(queue)
        for i in range(starts[k], ends[k]):
            x = insns[i]
            inflight = set().union(*q) if q else set()
            if x.kind == "wait":
                if x.wait > 0 and smem and q:
                    infos.add(i)
                if x.wait == 0:
                    smem = False
                while len(q) > x.wait:
                    q.pop(0)
                continue
            if x.kind == "smem":
                smem = True
                continue
            if inflight:
                bad_r = x.src & inflight
                if bad_r:
                    findings.setdefault((i, "read"), f"reads in-flight LDS destination {sorted(bad_r)}")
                bad_w = x.dst & inflight
                if bad_w and x.kind != "lds":
                    findings.setdefault((i, "clobber"), f"writes in-flight LDS destination {sorted(bad_w)}")
            if x.kind == "lds":
                q.append(frozenset(x.dst))
        state = (tuple(q), smem)
        for n in succ[k]:
            if state not in seen[n]:
                if len(seen[n]) >= max_states:
                    overflow = True
                    continue
                seen[n].add(state)
                work.append((n, state))
    return findings, infos, overflow


def compile_asm(src: str, out_dir: str) -> tuple:
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, os.path.basename(src).replace(".hip", ".s"))
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "-I/opt/rocm/include",
           "-I" + os.path.join(ROOT, "csrc/runtime"), "--offload-arch=gfx950", "-munsafe-fp-atomics",
           "--cuda-device-only", "-S", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        raise SystemExit(f"isa_lint: compile of {src} failed")
    n_warn = r.stderr.count("[-Winline-asm]")
    return out, n_warn


def lint_file(path: str, pattern: str, verbose: bool) -> int:
    kernels = parse(path)
    total, n_kernels, n_info = 0, 0, 0
    for name, (insns, labels) in kernels.items():
        if pattern and not re.search(pattern, name):
            continue
        if not any(x.kind == "lds" and x.asm for x in insns):
            continue
        n_kernels += 1
        findings, infos, overflow = analyse(insns, labels)
        n_info += len(infos)
        if overflow:
            print(f"{os.path.basename(path)}: {name}: state overflow (analysis incomplete)")
            total += 1
        for (i, kind), msg in sorted(findings.items()):
            total += 1
            if verbose or total <= 40:
                print(f"{os.path.basename(path)}:{insns[i].line}: {name[:70]}: {kind}: {insns[i].text}  -- {msg}")
    print(f"isa_lint: {os.path.basename(path)}: {n_kernels} kernel(s) with asm LDS reads; info: {n_info} counted "
          f"wait(s) with an SMEM load in flight (safe: over-wait only)")
    return total


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--asm", nargs="*", default=[], help="device assembly files (hipcc -S output)")
    ap.add_argument("--src", nargs="*", default=[], help=".hip sources to compile with hipcc -S")
    ap.add_argument("--out-dir", default=os.path.join(ROOT, "build", "isa"))
    ap.add_argument("--kernels", default=r"gemm[34]_kernel", help="regex on the mangled kernel name")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    if not a.asm and not a.src:   # no arguments: the two kernels the CPU suite lints
        a.src = [os.path.join(ROOT, "csrc", "kernels", f) for f in ("gemm4.hip", "gemm3.hip")]
    files, warns = list(a.asm), 0
    for s in a.src:
        out, w = compile_asm(s, a.out_dir)
        warns += w
        files.append(out)
    total = 0
    for f in files:
        n = lint_file(f, a.kernels, a.verbose)
        print(f"isa_lint: {f}: {n} finding(s)")
        total += n
    if a.src:
        print(f"isa_lint: {warns} -Winline-asm warning(s)")
    return 1 if total or warns else 0


if __name__ == "__main__":
    sys.exit(main())
