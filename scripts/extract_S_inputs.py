"""Write decagon_amd/data/synthetic_S_adj.npz: the INPUT arrays of config S (the
reference-normalised adjacency COO tuples, degrees, edge types, node counts, decoder kinds)
taken from tests/golden/synthetic_S.npz (made by tests/golden/make_golden.py with the
reference's own EdgeMinibatchIterator), so the bench and synthetic.load_S never read the
test fixtures.  No oracle output is copied.

    python3 scripts/extract_S_inputs.py
"""
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
z = np.load(ROOT / "tests" / "golden" / "synthetic_S.npz", allow_pickle=False)
keep = {k: z[k] for k in z.files
        if k in ("edge_types", "n_nodes", "decoders") or k.startswith(("adj_", "deg_"))}
out = ROOT / "decagon_amd" / "data" / "synthetic_S_adj.npz"
out.parent.mkdir(exist_ok=True)
np.savez_compressed(out, **keep)
print(out, len(keep), "arrays")
