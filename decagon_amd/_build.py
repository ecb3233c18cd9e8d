"""Build libdecagon_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

The library is the only native artefact of the package; it is git-ignored but travels to
the GPU box with the repository snapshot (decagon_amd/lib/).
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path
from .tuning import knob

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
LIBDIR = PKG / "lib"
LIBNAME = "libdecagon_hip.so"
ARCH = knob("DG_OFFLOAD_ARCH", "gfx950")


def lib_path() -> Path:
    return LIBDIR / LIBNAME


def _sources():
    return sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))


def _deps():
    return _sources() + sorted(CSRC.glob("*.h")) + sorted(INCLUDE.glob("*.h"))


def needs_build() -> bool:
    out = lib_path()
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(p.stat().st_mtime > t for p in _deps())


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libdecagon_hip.so)")


def build(force: bool = False, verbose: bool = False, defines=(), out: Path = None) -> Path:
    """Compile every csrc/*.hip into decagon_amd/lib/libdecagon_hip.so for gfx950 (or, with
    `defines` such as "DG_SLOT_ABL=1", a variant build into `out`: A/B and ablation runs load
    it through DG_LIB)."""
    out = lib_path() if out is None else Path(out)
    if not force and not defines and not needs_build():
        return out
    LIBDIR.mkdir(parents=True, exist_ok=True)
    tmp = out.with_suffix(".so.tmp")
    cmd = [
        hipcc(),
        "-O3",
        "-std=c++17",
        f"--offload-arch={ARCH}",
        "-fPIC",
        "-shared",
        "-Wall",
        "-Wno-pass-failed",
        f"-I{INCLUDE}",
        f"-I{CSRC}",
        *[d if d.startswith("-") else f"-D{d}" for d in defines],  # (variants: raw flags too)
        "-o",
        str(tmp),
        *[str(s) for s in _sources()],
    ]
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    if verbose and res.stderr.strip():
        print(res.stderr)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    import sys

    # python -m decagon_amd._build [NAME DEFINE ...]: a variant lib/var_NAME.so
    if len(sys.argv) > 2:
        print(build(force=True, defines=sys.argv[2:], out=LIBDIR / f"var_{sys.argv[1]}.so"))
    else:
        print(build(force=True, verbose=True))
