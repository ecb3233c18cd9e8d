# A/B: gcn_tab_kernel's round-5 finishing (per-group normalising waves, a second barrier, the
# nbuf hand-off to the row's wave) against round 6's single finishing wave — the segspmm.hip of
# commit 97a0bd5 (the host's descriptors carry both forms' fields).
import subprocess
from pathlib import Path

_root = Path(__file__).resolve().parents[2]
_cur = (_root / "decagon_amd/csrc/segspmm.hip").read_text()
_old = subprocess.run(["git", "-C", str(_root), "show", "97a0bd5:decagon_amd/csrc/segspmm.hip"],
                      capture_output=True, text=True, check=True).stdout
EDITS = [("segspmm.hip", _cur, _old)]
