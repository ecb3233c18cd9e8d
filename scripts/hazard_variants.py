"""Build the code objects scripts/hazard_harness compares (DESIGN.md §5, config 5's hazard).

Run on the CPU container (needs git and the ROCm toolchain):  python scripts/hazard_variants.py
Writes scripts/hazard/*.hsaco (git-ignored; they travel to the GPU box with the tree):

  ref.hsaco          the round-4 source as shipped (commit 3b0d266: per-half sums kept
                     unpaired by an opaque copy)
  failing.hsaco      the same source without the opaque copy — the build that returned wrong
                     half-0 scores on ~2 % of tiles — assembled from its own .s, unchanged
  <site>.hsaco       that .s with ONE candidate site changed (wait states inserted, or one
                     register renamed), nothing else, so a build that stops failing names the
                     sequence
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "scripts" / "hazard"
LLVM = Path("/opt/rocm/lib/llvm/bin")
COMMIT = "3b0d266"
KERNEL = "_ZN12_GLOBAL__N_124decoder_bf16_cs16_kernelILi768ELb1EEEvNS_11Bf16DecArgsE"
FENCE = 'asm volatile("" : "+v"(pp[b]), "+v"(pn[b]));'


def git_show(path: str) -> str:
    return subprocess.run(["git", "-C", str(ROOT), "show", f"{COMMIT}:{path}"], check=True, capture_output=True,
                          text=True).stdout


def compile_s(src: str, inc: Path, work: Path, name: str) -> str:
    (work / f"{name}.hip").write_text(src)
    s = work / f"{name}.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                    f"-I{inc}", "-S", str(work / f"{name}.hip"), "-o", str(s)], check=True, capture_output=True)
    return s.read_text()


def assemble(asm: str, work: Path, name: str) -> Path:
    s = work / f"{name}.s"
    s.write_text(asm)
    o = work / f"{name}.o"
    subprocess.run([str(LLVM / "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    str(s), "-o", str(o)], check=True, capture_output=True)
    out = OUT / f"{name}.hsaco"
    subprocess.run([str(LLVM / "ld.lld"), "-shared", str(o), "-o", str(out)], check=True, capture_output=True)
    return out


def kernel_span(lines):
    a = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    b = next(i for i in range(a + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return a, b


_VR = re.compile(r"v\[(\d+):(\d+)\]")


def edit_pk(lines):
    """s_nop 1 between a v_mov_b32 that writes one VGPR and the v_pk_fma_f32 right after it
    reading that VGPR inside a 64-bit source pair (the failing build's four epilogue sites)."""
    a, b = kernel_span(lines)
    out, n = list(lines), 0
    for i in range(b, a, -1):
        cur, prev = lines[i].strip(), lines[i - 1].strip()
        m = re.match(r"v_mov_b32_e32 v(\d+),", prev)
        if not (cur.startswith("v_pk_fma_f32") and m):
            continue
        w = int(m.group(1))
        if any(int(x) <= w <= int(y) for x, y in _VR.findall(cur.split(",", 1)[1])):
            out.insert(i, "\ts_nop 1")
            n += 1
    return out, n


def edit_srcc(lines):
    """s_nop 7 before every ds_read whose destination is the SrcC of an MFMA at most 4
    instructions earlier (the failing build's one such site, in half 0's chain)."""
    a, b = kernel_span(lines)
    out, n = list(lines), 0
    for i in range(b, a, -1):
        cur = lines[i].strip()
        if not cur.startswith("ds_read_b128"):
            continue
        dst = _VR.match(cur.split()[1])
        if not dst:
            continue
        for j in range(i - 1, max(a, i - 5), -1):
            prev = lines[j].strip()
            if prev.startswith("v_mfma"):
                regs = _VR.findall(prev)
                if len(regs) >= 4 and regs[3] == dst.groups():
                    out.insert(i, "\ts_nop 7")
                    n += 1
                break
    return out, n


def _find(lines, text, start=0):
    return next(i for i in range(start, len(lines)) if lines[i].strip() == text)


def edit_addr_own(lines):
    """ep[0]'s load addressed through its own destination register (v114) instead of v66,
    which the next load (en[0]) overwrites with its returning data."""
    out = list(lines)
    i = _find(out, "v_add_u32_e32 v66, s6, v109")
    j = _find(out, "buffer_load_dwordx4 v[114:117], v66, s[44:47], 0 offen", i)
    out[i] = "\tv_add_u32_e32 v114, s6, v109"
    out[j] = "\tbuffer_load_dwordx4 v[114:117], v114, s[44:47], 0 offen"
    return out, 1


def edit_drain_ep0(lines):
    """s_waitcnt vmcnt(0) right after ep[0]'s load: en[0]'s load issues once ep[0]'s data is in."""
    out = list(lines)
    j = _find(out, "buffer_load_dwordx4 v[114:117], v66, s[44:47], 0 offen")
    out.insert(j + 1, "\ts_waitcnt vmcnt(0)")
    return out, 1


def edit_wait_all(lines):
    """The q loop's first row-load waits (vmcnt(3), vmcnt(1)) as vmcnt(0)."""
    out = list(lines)
    i = _find(out, "v_add_u32_e32 v66, s6, v109")
    a = _find(out, "s_waitcnt vmcnt(3)", i)
    b = _find(out, "s_waitcnt vmcnt(1)", a)
    out[a] = out[b] = "\ts_waitcnt vmcnt(0)"
    return out, 2


def _q_loop(lines):
    """(first, last) line of the fused kernel's q loop: from the row loads' address adds to
    the loop's back-edge branch."""
    i = _find(lines, "v_add_u32_e32 v66, s6, v109")
    j = next(k for k in range(i, len(lines)) if lines[k].strip().startswith("s_cbranch_scc0"))
    return i, j


def edit_pk_nop_all(lines):
    """s_nop 4 before every v_pk_* instruction of the q loop (the whole packed epilogue)."""
    a, b = _q_loop(lines)
    out, n = list(lines), 0
    for i in range(b, a, -1):
        if lines[i].strip().startswith("v_pk_"):
            out.insert(i, "\ts_nop 4")
            n += 1
    return out, n


def edit_bperm_nop(lines):
    """s_nop 7 before the first cross-lane shuffle of the sums after the q loop."""
    a, b = _q_loop(lines)
    out = list(lines)
    k = next(i for i in range(b, len(lines)) if lines[i].strip().startswith("ds_bpermute_b32"))
    out.insert(k, "\ts_nop 7")
    return out, 1


def edit_mfma_drain(lines):
    """24 wait states after the q loop's last MFMA, before the epilogue touches any register:
    every MFMA has finished writing its accumulator, even behind other waves' MFMAs."""
    a, b = _q_loop(lines)
    last = max(i for i in range(a, b) if lines[i].strip().startswith("v_mfma"))
    out = list(lines)
    out[last + 1:last + 1] = ["\ts_nop 7", "\ts_nop 7", "\ts_nop 7"]
    return out, 1


def main() -> int:
    OUT.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        work = Path(td)
        inc = work / "inc"
        inc.mkdir()
        for f in ("common.h", "decoder_tile.h", "dropout.h", "peer.h"):
            try:
                (inc / f).write_text(git_show(f"decagon_amd/csrc/{f}"))
            except subprocess.CalledProcessError:
                pass
        (inc / "decagon_hip.h").write_text(git_show("include/decagon_hip.h"))
        src = git_show("decagon_amd/csrc/decoder_bf16.hip")
        assert FENCE in src
        ref = compile_s(src, inc, work, "ref")
        assemble(ref, work, "ref")
        failing = compile_s(src.replace(FENCE, "/* opaque copy removed */"), inc, work, "failing")
        assemble(failing, work, "failing")
        lines = failing.splitlines()
        for name, fn in (("pk_nop", edit_pk), ("srcc_nop", edit_srcc), ("addr_own", edit_addr_own),
                         ("drain_ep0", edit_drain_ep0), ("wait_all", edit_wait_all),
                         ("pk_nop_all", edit_pk_nop_all), ("bperm_nop", edit_bperm_nop),
                         ("mfma_drain", edit_mfma_drain)):
            edited, n = fn(lines)
            assemble("\n".join(edited) + "\n", work, name)
            print(f"{name}: {n} site(s) edited")
    print("wrote", sorted(p.name for p in OUT.glob("*.hsaco")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
