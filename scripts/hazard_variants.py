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


def _reorder_loads(lines, order, waits):
    """The q loop's four row loads (ep[0], en[0], ep[1], en[1]) issued in `order` (ep[0]
    addressed through its own destination register, as in addr_own, so no load's returning
    data overwrites another's address), and its first two waits set to `waits`."""
    out = list(lines)
    i = _find(out, "v_add_u32_e32 v66, s6, v109")
    out[i] = "\tv_add_u32_e32 v114, s6, v109"
    loads = {"ep0": "\tbuffer_load_dwordx4 v[114:117], v114, s[44:47], 0 offen",
             "en0": "\tbuffer_load_dwordx4 v[66:69], v67, s[44:47], 0 offen",
             "ep1": "\tbuffer_load_dwordx4 v[82:85], v70, s[44:47], 0 offen",
             "en1": "\tbuffer_load_dwordx4 v[70:73], v71, s[44:47], 0 offen"}
    j = _find(out, "buffer_load_dwordx4 v[114:117], v66, s[44:47], 0 offen", i)
    assert [out[j + 2 * k].strip() for k in range(1, 4)] == [loads[n].strip() for n in ("en0", "ep1", "en1")]
    for k, n in enumerate(order):
        out[j + 2 * k] = loads[n]
    a = _find(out, "s_waitcnt vmcnt(3)", j)
    b = _find(out, "s_waitcnt vmcnt(1)", a)
    out[a], out[b] = (f"\ts_waitcnt vmcnt({w})" for w in waits)
    return out, 1


def edit_ep0_last(lines):
    """ep[0]'s row load issued last of the four instead of first (both waits vmcnt(0))."""
    return _reorder_loads(lines, ("en0", "ep1", "en1", "ep0"), (0, 0))


def edit_en0_first(lines):
    """en[0]'s row load issued first, ep[0]'s second (first wait vmcnt(2))."""
    return _reorder_loads(lines, ("en0", "ep0", "ep1", "en1"), (2, 1))


_PK = re.compile(r"(v_pk_(?:fma|mul|add)_f32) v\[(\d+):\d+\], (.*?)(?: op_sel:\[([01,]+)\])?(?: op_sel_hi:\[([01,]+)\])?$")


def _unpack(line):
    """One packed fp32 instruction as two scalar VOP3 ones with the same operands and half
    selects (lo result: op_sel, hi result: op_sel_hi), ordered so neither clobbers a source
    of the other."""
    m = _PK.match(line.strip())
    op, d, rest, sel, selhi = m.groups()
    srcs = [int(x) for x in re.findall(r"v\[(\d+):\d+\]", rest)]
    n = len(srcs)
    sel = [int(x) for x in sel.split(",")] if sel else [0] * n
    selhi = [int(x) for x in selhi.split(",")] if selhi else [1] * n
    sop = {"v_pk_fma_f32": "v_fma_f32", "v_pk_mul_f32": "v_mul_f32", "v_pk_add_f32": "v_add_f32"}[op]
    d = int(d)
    lo_src = [s + k for s, k in zip(srcs, sel)]
    hi_src = [s + k for s, k in zip(srcs, selhi)]
    lo = f"\t{sop} v{d}, " + ", ".join(f"v{r}" for r in lo_src)
    hi = f"\t{sop} v{d + 1}, " + ", ".join(f"v{r}" for r in hi_src)
    if d in hi_src:
        assert d + 1 not in lo_src, line
        return [hi, lo]
    return [lo, hi]


def _unpack_where(lines, pred):
    a, b = _q_loop(lines)
    out, n = list(lines), 0
    for i in range(b, a, -1):
        t = lines[i].strip()
        if t.startswith("v_pk_") and pred(t):
            out[i:i + 1] = _unpack(t)
            n += 1
    return out, n


def edit_unpack_all(lines):
    """Every packed fp32 instruction of the q loop as two scalar ones (same registers)."""
    return _unpack_where(lines, lambda t: True)


def edit_unpack_sel01(lines):
    """Only the v_pk_mul_f32 with op_sel:[0,1] (the low result reads src1's high dword)."""
    return _unpack_where(lines, lambda t: t.startswith("v_pk_mul_f32") and "op_sel:[0,1]" in t)


def edit_unpack_selhi10(lines):
    """Only the v_pk_mul_f32 with op_sel_hi:[1,0] (the high result reads src1's low dword)."""
    return _unpack_where(lines, lambda t: t.startswith("v_pk_mul_f32") and "op_sel_hi:[1,0]" in t)


def edit_swap_sel01(lines):
    """Each v_pk_mul_f32 D, A, B op_sel:[0,1] as v_pk_mul_f32 D, B, A op_sel:[1,0]: the same
    products (fp32 multiplication commutes exactly), the broadcast half read through src0."""
    a, b = _q_loop(lines)
    out, n = list(lines), 0
    for i in range(a, b):
        m = re.match(r"v_pk_mul_f32 (v\[\d+:\d+\]), (v\[\d+:\d+\]), (v\[\d+:\d+\]) op_sel:\[0,1\]$",
                     lines[i].strip())
        if m:
            out[i] = f"\tv_pk_mul_f32 {m.group(1)}, {m.group(3)}, {m.group(2)} op_sel:[1,0]"
            n += 1
    return out, n


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
                         ("mfma_drain", edit_mfma_drain), ("ep0_last", edit_ep0_last),
                         ("en0_first", edit_en0_first), ("unpack_all", edit_unpack_all),
                         ("unpack_sel01", edit_unpack_sel01), ("unpack_selhi10", edit_unpack_selhi10),
                         ("swap_sel01", edit_swap_sel01)):
            edited, n = fn(lines)
            assemble("\n".join(edited) + "\n", work, name)
            print(f"{name}: {n} site(s) edited")
    print("wrote", sorted(p.name for p in OUT.glob("*.hsaco")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
