"""List short loops in the shipping library whose body waits vmcnt(0) on its own loads — the
pattern of a serial chain of memory round trips (one per iteration) that found round 5's
config-5 loss sum and the backward's index scans.  A heuristic: backward
branches within ~60 instructions whose body holds one or two vector loads and a full wait.
Peer polls (s_sleep loops) and rare fallback paths show up too; read each hit's source.

Usage (CPU container):  python scripts/serial_loads.py [filter]
"""
import re
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scripts"))

import isa_scan  # noqa: E402


def main(argv):
    filt = argv[1] if len(argv) > 1 else ""
    lib = ROOT / "decagon_amd" / "lib" / "libdecagon_hip.so"
    with tempfile.TemporaryDirectory() as td:
        for co in isa_scan.extract_code_objects(lib, Path(td)):
            for k in isa_scan.parse(isa_scan.disassemble(co)):
                if filt not in k.name:
                    continue
                ins = [i.text for i in k.insns]
                for i, t in enumerate(ins):
                    m = re.match(r"s_(?:cbranch_\w+|branch) (\d+)", t)
                    if not m or int(m.group(1)) < 32768:
                        continue  # forward branch
                    body = ins[max(0, i - (65536 - int(m.group(1)))):i]
                    if len(body) > 60:
                        continue
                    loads = sum(("global_load" in x or "buffer_load" in x) for x in body)
                    waits = sum("vmcnt(0)" in x for x in body)
                    sleeps = any("s_sleep" in x for x in body)
                    if 1 <= loads <= 2 and waits and not sleeps:
                        print(f"{k.name[:80]}  at {i}: body ~{len(body)}, loads {loads}, full waits {waits}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
