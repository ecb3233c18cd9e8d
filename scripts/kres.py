"""Per-kernel resources of a built library's gfx950 code objects: VGPRs, AGPRs, SGPRs, spills,
static LDS and occupancy-relevant figures, read from the code object's metadata notes.

Usage: python scripts/kres.py [LIB] [NAME_SUBSTRING ...]   (default: the shipping library)
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import isa_scan  # noqa: E402

KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".group_segment_fixed_size", ".private_segment_fixed_size")


def resources(lib: Path):
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for co in isa_scan.extract_code_objects(lib, Path(td)):
            r = subprocess.run([str(isa_scan.LLVM / "llvm-readelf"), "--notes", str(co)], check=True,
                               capture_output=True, text=True).stdout
            cur = {}
            for line in r.splitlines():
                s = line.strip().lstrip("- ")
                for k in KEYS + (".name",):
                    if s.startswith(k + ":"):
                        cur[k] = s.split(":", 1)[1].strip()
                if s.startswith(".wavefront_size:") and ".name" in cur:
                    out[cur[".name"]] = dict(cur)
                    cur = {}
    return out


if __name__ == "__main__":
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else isa_scan.DEFAULT_LIB
    pats = [a for a in sys.argv[1:] if not a.endswith(".so")]
    for name, r in sorted(resources(lib).items()):
        if pats and not any(p in name for p in pats):
            continue
        print(f"{name[:90]:90s} vgpr {r.get('.vgpr_count')} agpr {r.get('.agpr_count')} "
              f"sgpr {r.get('.sgpr_count')} spill v{r.get('.vgpr_spill_count')}/s{r.get('.sgpr_spill_count')} "
              f"lds {r.get('.group_segment_fixed_size')} scratch {r.get('.private_segment_fixed_size')}")
