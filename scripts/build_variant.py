"""Build an A/B variant library from the current sources with textual edits applied to copies
(no A/B macros in the product code): decagon_amd/lib/var_NAME.so, loaded on the GPU box with
DG_LIB (scripts/ab.sh NAME).

    python scripts/build_variant.py NAME EDITS.py [DEFINE ...]

EDITS.py defines EDITS = [(file name under csrc/, old text, new text), ...]; each old text must
occur exactly once.  The edited files go to a temporary copy of csrc/ (the includes resolve
there first), the library is compiled from it exactly as decagon_amd/_build.py compiles the
product library."""
import runpy
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from decagon_amd import _build  # noqa: E402


def main():
    name, edits_py, defines = sys.argv[1], sys.argv[2], sys.argv[3:]
    edits = runpy.run_path(edits_py)["EDITS"]
    with tempfile.TemporaryDirectory() as tmp:
        src = Path(tmp) / "csrc"
        shutil.copytree(_build.CSRC, src)
        for fname, old, new in edits:
            p = src / fname
            text = p.read_text()
            if text.count(old) != 1:
                raise SystemExit(f"{fname}: the edit's old text occurs {text.count(old)} times")
            p.write_text(text.replace(old, new))
        out = _build.LIBDIR / f"var_{name}.so"
        cmd = [_build.hipcc(), "-O3", "-std=c++17", f"--offload-arch={_build.ARCH}", "-fPIC", "-shared", "-Wall",
               "-Wno-pass-failed", f"-I{_build.INCLUDE}", f"-I{src}",
               *[d if d.startswith("-") else f"-D{d}" for d in defines], "-o", str(out),
               *[str(s) for s in sorted(src.glob("*.hip")) + sorted(src.glob("*.cpp"))]]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode:
            raise SystemExit(res.stderr)
        print(out)


if __name__ == "__main__":
    main()
