"""Synthetic graphs of the benchmark configurations (BASELINE.json `configs`).

S  — main.py's 5-relation / 10-matrix toy graph (main.py:137-217).  Its exact
     reference-normalised train adjacencies (generated with the reference's own iterator by
     tests/golden/make_golden.py) are committed as package data, decagon_amd/data/
     synthetic_S_adj.npz (inputs only: scripts/extract_S_inputs.py); `load_S` reads them.
P  — polypharmacy-shaped: 19,085 proteins, 645 drugs; PPI with 715,612
     undirected edges; 18,596 drug–target edges as (0,1) and its transpose (1,0); 964
     drug–drug relations of Zipf sizes s_r = max(500, ⌊28,568·r^-0.31⌋), each symmetric,
     + their transposes ⇒ 1,932 matrices, ≈23 M nonzeros after normalisation (+I).
     Seeded (numpy default_rng); normalised with preprocess_graph (minibatch.py:80-93).
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import scipy.sparse as sp

from .sparse import HostCSR, coo_to_csr, preprocess_graph

EdgeType = Tuple[int, int]
ROOT = Path(__file__).resolve().parents[1]
GOLDEN_S = Path(__file__).resolve().parent / "data" / "synthetic_S_adj.npz"


@dataclass
class SyntheticGraph:
    name: str
    n_nodes: Dict[int, int]
    edge_types: Dict[EdgeType, int]
    decoders: Dict[EdgeType, str]
    adj: Dict[EdgeType, List[Tuple[np.ndarray, np.ndarray, Tuple[int, int]]]]  # COO tuples
    degrees: Dict[int, List[np.ndarray]]

    def csr(self) -> Dict[EdgeType, List[HostCSR]]:
        out: Dict[EdgeType, List[HostCSR]] = {}
        memo: Dict[int, HostCSR] = {}
        for et, rels in self.adj.items():
            lst = []
            for coo in rels:
                key = (id(coo[0]), id(coo[1]), tuple(coo[2]))  # one CSR per distinct tuple
                if key not in memo:
                    memo[key] = coo_to_csr(*coo)
                lst.append(memo[key])
            out[et] = lst
        return out

    @property
    def nnz(self) -> int:
        return int(sum(len(c[1]) for rels in self.adj.values() for c in rels))


def load_S(path: Path = GOLDEN_S) -> SyntheticGraph:
    z = np.load(path, allow_pickle=False)
    et_rows = z["edge_types"]
    edge_types = {(int(i), int(j)): int(k) for i, j, k in et_rows}
    decoders = {et: str(d) for et, d in zip(edge_types, z["decoders"])}
    adj, degrees = {}, {0: [], 1: []}
    for (i, j), K in edge_types.items():
        adj[i, j] = []
        for k in range(K):
            adj[i, j].append((z[f"adj_{i}_{j}_{k}_coords"], z[f"adj_{i}_{j}_{k}_values"],
                              tuple(int(s) for s in z[f"adj_{i}_{j}_{k}_shape"])))
    n = z["n_nodes"]
    return SyntheticGraph("S", {0: int(n[0]), 1: int(n[1])}, edge_types, decoders, adj,
                          _degrees_from(z, edge_types))


def _degrees_from(z, edge_types) -> Dict[int, List[np.ndarray]]:
    deg: Dict[int, List[np.ndarray]] = {}
    for (i, j), K in edge_types.items():
        for k in range(K):
            if i == j:
                deg.setdefault(i, []).append(z[f"deg_{i}_{j}_{k}"])
    return deg


def _sym_relation(rng, n: int, n_edges: int) -> sp.csr_matrix:
    """A symmetric 0/1 relation with n_edges distinct undirected edges, no self loops."""
    n_edges = min(n_edges, n * (n - 1) // 2)
    keys = np.zeros(0, np.int64)
    while keys.size < n_edges:
        need = n_edges - keys.size
        a = rng.integers(0, n, size=int(need * 1.2) + 16)
        b = rng.integers(0, n, size=a.size)
        lo, hi = np.minimum(a, b), np.maximum(a, b)
        cand = (lo * n + hi)[lo != hi]
        keys = np.unique(np.concatenate([keys, cand]))
    keys = rng.permutation(keys)[:n_edges]
    a, b = keys // n, keys % n
    r = np.concatenate([a, b])
    c = np.concatenate([b, a])
    return sp.csr_matrix((np.ones(r.size), (r, c)), shape=(n, n))


def make_P(seed: int = 0, n_proteins: int = 19085, n_drugs: int = 645, n_side_effects: int = 964,
           ppi_edges: int = 715612, target_edges: int = 18596) -> SyntheticGraph:
    rng = np.random.default_rng(seed)
    # PPI: uniform random undirected graph
    ppi = _sym_relation(rng, n_proteins, ppi_edges)
    # drug-target: bipartite, uniform
    flat = rng.choice(n_proteins * n_drugs, size=target_edges, replace=False)
    tgt = sp.csr_matrix((np.ones(target_edges), (flat // n_drugs, flat % n_drugs)),
                        shape=(n_proteins, n_drugs))
    ppi_n = preprocess_graph(ppi)
    # The transposed copies the reference trains with (DecagonDataSet.py:212-231) are the
    # flipped COO of the normalised matrix; for a symmetric relation that is the same matrix
    # (every stored value is d_r·d_c), so the same tuple object is reused.
    ppi_t = ppi_n
    g2d = preprocess_graph(tgt)
    d2g = (g2d[0][:, ::-1].copy(), g2d[1], (g2d[2][1], g2d[2][0]))
    dd, deg_d = [], []
    for r in range(1, n_side_effects + 1):
        size = max(500, int(28568 * r ** -0.31))
        m = _sym_relation(rng, n_drugs, size)
        deg_d.append(np.asarray(m.sum(axis=0)).ravel())
        dd.append(preprocess_graph(m))
    dd_t = list(dd)
    adj = {(0, 0): [ppi_n, ppi_t], (0, 1): [g2d], (1, 0): [d2g], (1, 1): dd + dd_t}
    edge_types = {et: len(v) for et, v in adj.items()}
    decoders = {(0, 0): "bilinear", (0, 1): "bilinear", (1, 0): "bilinear", (1, 1): "dedicom"}
    ppi_deg = np.asarray(ppi.sum(axis=0)).ravel()
    return SyntheticGraph("P", {0: n_proteins, 1: n_drugs}, edge_types, decoders, adj,
                          {0: [ppi_deg, ppi_deg], 1: deg_d + deg_d})


def replicate_sets(g: SyntheticGraph, copies: int) -> SyntheticGraph:
    """The weak-scaling graph: `copies` relation sets of g over the same nodes (relation
    set r is g's relations again, with its own weights) — edge type (i,j) then has
    copies·K_ij relations, set r at [r·K_ij, (r+1)·K_ij)."""
    adj = {et: list(rels) * copies for et, rels in g.adj.items()}
    deg = {t: list(v) * copies for t, v in g.degrees.items()}
    return SyntheticGraph(f"{g.name}x{copies}", dict(g.n_nodes), {et: len(v) for et, v in adj.items()},
                          dict(g.decoders), adj, deg)


@dataclass
class Config5:
    """BASELINE configs[4]'s scorer inputs (float32 here; the bench and tests round them to
    bf16): d = 256 drug embeddings, the global R, one D_k per drug-drug relation slot, B
    positive pairs per slot (slot-major, edges of the slot's relation) and each slot's drug
    degrees, which its negatives follow (optimizer.py:38-47 samples relation k's negatives
    from degrees[i][k])."""

    E: np.ndarray
    R: np.ndarray
    D: np.ndarray
    pos_rows: np.ndarray
    pos_cols: np.ndarray
    degrees: np.ndarray  # [n_slots, n_drugs]
    batch: int


def make_config5(seed: int = 5, n_drugs: int = 645, n_slots: int = 1928, d: int = 256, batch: int = 512) -> Config5:
    """Slots are config P's drug-drug relations: relation r (1-based, r <= n_slots/2) has
    max(500, ⌊28,568·r^-0.31⌋) undirected edges, slot r + n_slots/2 is its
    transpose (same degrees); each slot's positives are B of its edges."""
    rng = np.random.default_rng(seed)
    E = (rng.standard_normal((n_drugs, d)) / 4).astype(np.float32)
    r = np.sqrt(6.0 / (2 * d))
    R = rng.uniform(-r, r, (d, d)).astype(np.float32)
    r = np.sqrt(6.0 / (d + 1))
    D = rng.uniform(-r, r, (n_slots, d)).astype(np.float32)
    half = n_slots // 2 if n_slots > 1 else n_slots
    degrees = np.zeros((n_slots, n_drugs), np.float64)
    pos_rows = np.empty(n_slots * batch, np.int32)
    pos_cols = np.empty(n_slots * batch, np.int32)
    edges = {}
    for k in range(n_slots):
        rel = k % half
        if rel not in edges:
            size = max(500, int(28568 * (rel + 1) ** -0.31))
            a = rng.integers(0, n_drugs, size)
            b = rng.integers(0, n_drugs, size)
            keep = a != b
            edges[rel] = (a[keep], b[keep])
        src, dst = edges[rel] if k < half else edges[rel][::-1]  # slot k + half: the transpose
        degrees[k] = np.bincount(src, minlength=n_drugs) + np.bincount(dst, minlength=n_drugs)
        pick = rng.integers(0, src.size, batch)
        pos_rows[k * batch:(k + 1) * batch] = src[pick]
        pos_cols[k * batch:(k + 1) * batch] = dst[pick]
    return Config5(E, R, D, pos_rows, pos_cols, degrees, batch)
