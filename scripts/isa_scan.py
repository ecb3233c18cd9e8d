"""Disassemble the gfx950 code objects of a built library (or a code object) into kernels.

Usage: python scripts/isa_scan.py [LIB_OR_CODE_OBJECT ...]   (default: the shipping library)

It extracts every gfx950 code object (llvm-objdump --offloading, into a temp dir, never next
to the library), disassembles it and parses each kernel's instructions (mnemonic, VGPR
destination, VGPR sources).  tests/test_cpu_isa.py uses it to pin the config-5 kernel's
validated instruction selection ("The config-5 miscompile"); run as a script it
prints, per kernel, the MFMA and packed-fp32 instruction counts.
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
from typing import List, Optional, Tuple

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


def kernels(lib: Path = DEFAULT_LIB) -> List[Kernel]:
    """Every kernel of every gfx950 code object of `lib`."""
    out: List[Kernel] = []
    with tempfile.TemporaryDirectory() as td:
        for co in extract_code_objects(Path(lib), Path(td)):
            out += parse(disassemble(co))
    return out


def main(argv: List[str]) -> int:
    for lib in [Path(a) for a in argv] or [DEFAULT_LIB]:
        ks = kernels(lib)
        print(f"{lib}: {len(ks)} kernels")
        for k in ks:
            n_mfma = sum(x.op.startswith("v_mfma") for x in k.insns)
            n_pk = sum(x.op.startswith("v_pk_") for x in k.insns)
            print(f"  {len(k.insns):6d} insns  {n_mfma:4d} mfma  {n_pk:4d} v_pk  {k.name[:100]}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
