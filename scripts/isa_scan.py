"""Scan the gfx950 code objects of a built library for a VALU -> packed-f32 read pattern.

Usage: python scripts/isa_scan.py [LIB_OR_CODE_OBJECT ...]   (default: the shipping library)

It extracts every gfx950 code object (llvm-objdump --offloading, into a temp dir), disassembles
it, and reports, per kernel, every `v_pk_*` instruction that reads as a 64-bit source a VGPR
pair one half of which was written by one of the N VALU instructions right before it while
the other half was not (a pair assembled from two writes just before the packed read).
DESIGN.md §5 ("The packed-f32 forwarding hazard") says why: that is the sequence config 5's
fused kernel ran when it returned wrong half-0 sums.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Tuple

LLVM = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin"
ROOT = Path(__file__).resolve().parent.parent
DEFAULT_LIB = ROOT / "decagon_amd" / "lib" / "libdecagon_hip.so"

_KERNEL = re.compile(r"^[0-9a-f]+ <([^>]+)>:")
_INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*//")
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


@dataclass
class Insn:
    op: str
    dst: Optional[Tuple[int, int]]      # (first VGPR, count) written, VALU only
    srcs: List[Tuple[int, int]]         # VGPR operands read
    text: str


@dataclass
class Finding:
    kernel: str
    index: int                          # instruction index in the kernel
    distance: int                       # 1: the writer is the instruction right before
    writer: str
    reader: str


@dataclass
class Kernel:
    name: str
    insns: List[Insn] = field(default_factory=list)


def _regs(s: str) -> List[Tuple[int, int]]:
    out = []
    for m in _VREG.finditer(s):
        if m.group(3) is not None:
            out.append((int(m.group(3)), 1))
        else:
            a, b = int(m.group(1)), int(m.group(2))
            out.append((a, b - a + 1))
    return out


def _is_valu(op: str) -> bool:
    return op.startswith("v_") and not op.startswith(("v_mfma", "v_smfma", "v_readlane", "v_readfirstlane",
                                                       "v_cmp", "v_cmpx"))


def parse(asm: str) -> List[Kernel]:
    kernels: List[Kernel] = []
    cur: Optional[Kernel] = None
    for line in asm.splitlines():
        m = _KERNEL.match(line)
        if m:
            cur = Kernel(m.group(1))
            kernels.append(cur)
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        op, args = m.group(1), (m.group(2) or "")
        regs = _regs(args.split(" op_sel")[0])
        dst = None
        srcs = regs
        if _is_valu(op) and regs and re.match(r"\s*v", args):
            dst, srcs = regs[0], regs[1:]
        cur.insns.append(Insn(op, dst, srcs, line.split("//")[0].strip()))
    return kernels


def scan_kernel(k: Kernel, window: int = 1) -> List[Finding]:
    """v_pk_* reads of a 64-bit VGPR pair one half of which a VALU instruction at most
    `window` instructions before wrote alone (32-bit destination)."""
    found = []
    for i, ins in enumerate(k.insns):
        if not ins.op.startswith("v_pk_"):
            continue
        for base, n in ins.srcs:
            if n != 2:
                continue
            for d in range(1, window + 1):
                if i - d < 0:
                    break
                w = k.insns[i - d]
                if w.dst is None or w.dst[1] != 1 or w.op.startswith("v_pk_"):
                    continue
                if w.dst[0] in (base, base + 1):
                    found.append(Finding(k.name, i, d, w.text, ins.text))
    return found


def extract_code_objects(lib: Path, workdir: Path) -> List[Path]:
    """gfx950 code objects inside a host library (or the file itself if it is one)."""
    head = lib.read_bytes()[:64]
    if head[:4] == b"\x7fELF" and head[18] == 0xE0:  # EM_AMDGPU
        return [lib]
    tmp = workdir / lib.name
    shutil.copy(lib, tmp)
    subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(tmp)], cwd=workdir, check=True,
                   capture_output=True)
    return sorted(p for p in workdir.iterdir() if "amdgcn" in p.name and "gfx950" in p.name)


def disassemble(co: Path) -> str:
    r = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                       capture_output=True, text=True)
    return r.stdout


def scan_library(lib: Path = DEFAULT_LIB, window: int = 1) -> Tuple[Dict[str, int], List[Finding]]:
    """(v_pk_* count per kernel, findings) over every gfx950 code object of `lib`."""
    counts: Dict[str, int] = {}
    findings: List[Finding] = []
    with tempfile.TemporaryDirectory() as td:
        for co in extract_code_objects(Path(lib), Path(td)):
            for k in parse(disassemble(co)):
                counts[k.name] = counts.get(k.name, 0) + sum(1 for x in k.insns if x.op.startswith("v_pk_"))
                findings += scan_kernel(k, window)
    return counts, findings


def main(argv: List[str]) -> int:
    libs = [Path(a) for a in argv] or [DEFAULT_LIB]
    bad = 0
    for lib in libs:
        counts, findings = scan_library(lib, window=int(os.environ.get("DG_ISA_WINDOW", "1")))
        print(f"{lib}: {len(counts)} kernels, {sum(counts.values())} v_pk_* instructions, "
              f"{len(findings)} findings")
        for f in findings:
            print(f"  {f.kernel}  [{f.index}] d={f.distance}\n    {f.writer}\n    {f.reader}")
        bad += len(findings)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
