"""Variant builds of libdecagon_hip.so for A/B timing (profiling aid).
    python scripts/variants.py build NAME [-DFLAG ...]   -> scripts/prof_build/lib_NAME.so
    python scripts/variants.py run SCRIPT [args]         (GPU box: SCRIPT once per built variant,
                                                          DG_LIB pointing at it, then the default)"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "scripts" / "prof_build"


def build(name, flags):
    sys.path.insert(0, str(ROOT))
    from decagon_amd import _build
    OUT.mkdir(exist_ok=True)
    cmd = [_build.hipcc(), "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", "-Wno-pass-failed", *flags,
           f"-I{ROOT / 'include'}", f"-I{_build.CSRC}", "-o", str(OUT / f"lib_{name}.so"),
           *map(str, _build._sources())]
    subprocess.run(cmd, check=True)


def run(script, args):
    libs = sorted(OUT.glob("lib_*.so"))
    for lib in [None] + libs:
        env = dict(os.environ)
        if lib is not None:
            env["DG_LIB"] = str(lib)
        r = subprocess.run([sys.executable, str(ROOT / script), *args], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3:])
    else:
        run(sys.argv[2], sys.argv[3:])
