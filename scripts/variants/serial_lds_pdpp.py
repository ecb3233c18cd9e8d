# (serial LDS sums adopted: this is proj_dpp.py)
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).resolve().parent / "proj_dpp.py"))["EDITS"]
