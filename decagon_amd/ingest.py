"""Polypharmacy ingestion: the DecagonPublicData CSV files → node lists,
adjacency matrices and node features, laid out the way DecagonDataSet hands them to the model.

Restates (paths relative to the reference root):
  DecagonPublicDataNodeListsBuilder         main/DataSetParsers/NodeLists/DecagonPublicDataNodeListsBuilder.py:13-77
  DecagonPublicDataAdjacencyMatricesBuilder main/DataSetParsers/AdjacencyMatrices/DecagonPublicDataAdjacencyMatricesBuilder.py:17-152
  DecagonPublicDataNodeFeaturesBuilder      main/DataSetParsers/NodeFeatures/DecagonPublicDataNodeFeaturesBuilder.py:16-79
  BaseNodeId._formatStr                     main/Dtos/NodeIds.py:29-49
  DecagonDataSet._getAdjMtxDict / transposes / _getDegreesDict / _getFeaturesDict
                                            main/Trainable/Decagon/DecagonDataSet.py:189-292

The reference parses with networkx (read_edgelist into a MultiGraph / Graph) and fills dense
numpy matrices; here each file is tokenised once and everything after that is vectorised
numpy over integer ids, producing scipy CSR directly.  Behaviour kept exactly, defects
included:
  * node ids: every non-digit is dropped and leading zeros stripped — except that a raw id
    whose LAST character is '0' becomes 0 (NodeIds.py:40-41), so e.g. CID000002170 and
    CID000003000 both map to drug 0;
  * the combo file must be the preprocessed 3-column form `drug,drug,Cxxxxxxx` (networkx
    rejects other widths for a one-key data tuple); the relation id is int(token[1:]);
  * a side effect is kept when it has >= 500 combo LINES (MultiGraph edges: duplicate lines
    count); its matrix is the symmetric 0/1 adjacency of the distinct pairs (a self-loop is 1
    on the diagonal) over the sorted drug list;
  * drug-drug relations are ordered by their first edge in networkx's MultiGraph edge
    traversal (nodes in first-appearance order, each node's neighbours in first-link order,
    parallel edges in line order) — the order `list(drugDrugRelationMtxs.values())` gives;
  * drugs = sorted(combo drugs ∪ CID-prefixed target nodes), proteins = sorted(PPI nodes ∪
    the other target nodes); the drug-protein matrix is [protein × drug];
  * mono features: one-hot [drug × side effect] over np.unique of every side effect in the
    file (also those of drugs outside the drug list, whose rows are skipped);
  * with transposes (TrainWithTransposedAdjacencyMatrices) the edge types come out in the
    order (0,0): [PPI, PPIᵀ], (0,1): [DP], (1,1): [R_1..R_n, R_1ᵀ..R_nᵀ], (1,0): [DPᵀ].
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import scipy.sparse as sp

EdgeType = Tuple[int, int]
PPI, DRUG = 0, 1
MIN_RELATION_EDGES = 500  # DecagonPublicDataAdjacencyMatricesBuilder.py:124-125
CooTuple = Tuple[np.ndarray, np.ndarray, Tuple[int, int]]


def _format_id(t: str) -> int:
    if t == "0" or t[-1:] == "0":
        return 0
    d = "".join(ch for ch in t if "0" <= ch <= "9").lstrip("0")
    if not d:  # int('') in the reference
        raise ValueError(f"node id without digits: {t!r}")
    return int(d)


def format_ids(tokens) -> np.ndarray:
    """BaseNodeId(token) for an array of raw id strings (NodeIds.py:8-12, :29-49) → int64.
    Each distinct token is formatted once."""
    import pandas as pd

    codes, uniq = pd.factorize(np.asarray(list(tokens) if not isinstance(tokens, np.ndarray) else tokens,
                                          dtype=object))
    vals = np.fromiter((_format_id(str(u)) for u in uniq), dtype=np.int64, count=len(uniq))
    return vals[codes] if len(codes) else np.zeros(0, dtype=np.int64)


def _map_unique(col: np.ndarray, fn) -> np.ndarray:
    """fn applied to each distinct value of an object column."""
    import pandas as pd

    codes, uniq = pd.factorize(col)
    out = np.asarray([fn(u) for u in uniq], dtype=object)
    return out[codes] if len(codes) else col


def read_edgelist_tokens(path: str, n_cols: int) -> List[np.ndarray]:
    """networkx.read_edgelist's tokenisation (text after '#' dropped, blank lines skipped, the
    line stripped and split on ','): `n_cols` token columns (object arrays of str).  A line
    with a single field is skipped, as networkx does; a line with any other width than
    `n_cols` is an error."""
    import pandas as pd

    try:
        df = pd.read_csv(path, header=None, dtype=str, comment="#", skip_blank_lines=True,
                         na_filter=False, keep_default_na=False, engine="c")
    except pd.errors.EmptyDataError:
        return [np.zeros(0, dtype=object) for _ in range(n_cols)]
    except pd.errors.ParserError as e:
        raise ValueError(f"{path}: {e}") from None
    if df.shape[1] != n_cols:
        raise ValueError(f"{path}: expected {n_cols} comma-separated fields, got {df.shape[1]}")
    cols = [df[c].to_numpy(dtype=object) for c in df.columns]
    rest = np.zeros(len(df), dtype=bool)
    for c in cols[1:]:
        rest |= c != ""
    single = ~rest
    if n_cols > 2 and np.any(rest & (cols[-1] == "")):
        raise ValueError(f"{path}: expected {n_cols} comma-separated fields")
    if single.any():
        cols = [c[~single] for c in cols]
    cols[0] = _map_unique(cols[0], str.lstrip)  # line.strip() in read_edgelist
    cols[-1] = _map_unique(cols[-1], str.rstrip)
    return cols


def _sym_adjacency(a: np.ndarray, b: np.ndarray, n: int) -> sp.csr_matrix:
    """nx.adjacency_matrix of the undirected simple graph on the distinct pairs {a_i, b_i}
    (weight 1; a self-loop is 1 on the diagonal), float64 CSR with sorted columns."""
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    key = np.unique(lo * n + hi)
    lo, hi = key // n, key % n
    off = lo != hi
    rows = np.concatenate([lo, hi[off]])
    cols = np.concatenate([hi, lo[off]])
    m = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(n, n))
    m.sort_indices()
    return m


def multigraph_edge_order(u: np.ndarray, v: np.ndarray) -> np.ndarray:
    """Line indices of the edges (u_i, v_i) in networkx's MultiGraph edge traversal: nodes in
    insertion order (add_edge adds u, then v), at each node its not-yet-visited neighbours in
    first-link order, parallel edges in insertion order."""
    m = len(u)
    if m == 0:
        return np.zeros(0, dtype=np.int64)
    inter = np.empty(2 * m, dtype=np.int64)
    inter[0::2], inter[1::2] = u, v
    nodes, first = np.unique(inter, return_index=True)
    rank_of = np.empty(len(nodes), dtype=np.int64)
    rank_of[np.argsort(first, kind="stable")] = np.arange(len(nodes))
    ru = rank_of[np.searchsorted(nodes, u)]
    rv = rank_of[np.searchsorted(nodes, v)]
    lo, hi = np.minimum(ru, rv), np.maximum(ru, rv)  # emitted at the earlier-inserted endpoint
    _, pfirst, inv = np.unique(lo * len(nodes) + hi, return_index=True, return_inverse=True)
    line = np.arange(m, dtype=np.int64)
    return np.lexsort((line, pfirst[inv.reshape(-1)], lo))


@dataclass
class NodeLists:
    """main/Dtos/NodeLists.py: sorted protein and drug ids."""
    proteins: np.ndarray
    drugs: np.ndarray


@dataclass
class PublicData:
    """The DecagonDataSet view of the ingested files."""
    node_lists: NodeLists
    relation_ids: List[int]                       # drug-drug side effects, in model order
    adj: Dict[EdgeType, List[sp.csr_matrix]]      # edge type → raw 0/1 matrices, DecagonDataSet order
    features: Dict[int, CooTuple]                 # sparse_to_tuple of the node features
    degrees: Dict[int, List[np.ndarray]]          # column sums (DecagonDataSet.py:276-292)
    side_effects: np.ndarray                      # mono side-effect ids (feature columns)

    @property
    def edge_types(self) -> Dict[EdgeType, int]:
        return {et: len(v) for et, v in self.adj.items()}


def _split_targets(t0: np.ndarray, t1: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    toks = np.unique(np.concatenate([t0, t1]).astype(str))
    is_drug = np.char.startswith(toks, "CID")
    return toks[is_drug], toks[~is_drug]


def _node_lists(c0, c1, t0, t1, p0, p1) -> NodeLists:
    tdrug, tprot = _split_targets(t0, t1)
    drugs = np.unique(np.concatenate([format_ids(c0), format_ids(c1), format_ids(tdrug)]))
    proteins = np.unique(np.concatenate([format_ids(p0), format_ids(p1), format_ids(tprot)]))
    return NodeLists(proteins=proteins, drugs=drugs)


def node_lists(ppi_csv: str, targets_csv: str, combo_csv: str) -> NodeLists:
    """DecagonPublicDataNodeListsBuilder.build (NodeLists…Builder.py:37-77)."""
    c0, c1, _ = read_edgelist_tokens(combo_csv, 3)
    t0, t1 = read_edgelist_tokens(targets_csv, 2)
    p0, p1 = read_edgelist_tokens(ppi_csv, 2)
    return _node_lists(c0, c1, t0, t1, p0, p1)


def _index(ids: np.ndarray, sorted_ids: np.ndarray, what: str) -> np.ndarray:
    """Positions of ids in a sorted id list (the reference's dict lookups: KeyError if absent)."""
    if len(ids) == 0:
        return np.zeros(0, dtype=np.int64)
    pos = np.minimum(np.searchsorted(sorted_ids, ids), max(len(sorted_ids) - 1, 0))
    if len(sorted_ids) == 0 or np.any(sorted_ids[pos] != ids):
        raise KeyError(f"{what} id not in the node list")
    return pos.astype(np.int64)


def _drug_protein(t0: np.ndarray, t1: np.ndarray, nl: NodeLists) -> sp.csr_matrix:
    """_buildDrugProteinRelationMtx (AdjacencyMatricesBuilder.py:127-145): [protein × drug] 0/1
    over the distinct unordered token pairs; the CID-prefixed token of a pair is the drug."""
    pairs = sorted({(a, b) if a <= b else (b, a) for a, b in zip(t0.astype(str), t1.astype(str))})
    drug_tok = [a if a[:3] == "CID" else b for a, b in pairs]
    prot_tok = [b if a[:3] == "CID" else a for a, b in pairs]
    di = _index(format_ids(drug_tok), nl.drugs, "drug")
    pi = _index(format_ids(prot_tok), nl.proteins, "protein")
    m = sp.csr_matrix((np.ones(len(di)), (pi, di)), shape=(len(nl.proteins), len(nl.drugs)))
    m.sum_duplicates()
    m.data[:] = 1.0
    m.sort_indices()
    return m


def _mono_features(mono_csv: str, drugs: np.ndarray) -> Tuple[CooTuple, np.ndarray]:
    """_getDrugNodeFeatures (NodeFeaturesBuilder.py:34-79): one-hot [drug × side effect],
    coordinates in row-major order (coo of a dense matrix), values 1."""
    import pandas as pd

    mono = pd.read_csv(mono_csv, header=0, dtype=str, keep_default_na=False, na_filter=False)
    if mono.shape[1] < 2:
        raise ValueError(f"{mono_csv}: expected at least 2 columns")
    md, ms = format_ids(mono.iloc[:, 0].to_numpy()), format_ids(mono.iloc[:, 1].to_numpy())
    side_effects = np.unique(ms)
    ne = max(1, len(side_effects))
    inlist = np.isin(md, drugs)
    key = np.unique(np.searchsorted(drugs, md[inlist]) * ne + np.searchsorted(side_effects, ms[inlist]))
    coords = np.stack([key // ne, key % ne], axis=1).astype(np.int64)
    return (coords, np.ones(len(key)), (len(drugs), len(side_effects))), side_effects


def load_public_data(ppi_csv: str, targets_csv: str, combo_csv: str, mono_csv: str,
                     transpose: bool = True, min_edges: int = MIN_RELATION_EDGES) -> PublicData:
    """Node lists + adjacency matrices + node features of the four DecagonPublicData files,
    assembled as DecagonDataSet.fromDataSet does (DecagonDataSet.py:168-292)."""
    c0, c1, c2 = read_edgelist_tokens(combo_csv, 3)
    t0, t1 = read_edgelist_tokens(targets_csv, 2)
    p0, p1 = read_edgelist_tokens(ppi_csv, 2)
    nl = _node_lists(c0, c1, t0, t1, p0, p1)
    nd, npr = len(nl.drugs), len(nl.proteins)

    # ---- drug-drug relations (AdjacencyMatricesBuilder.py:54-125) ----
    du, dv = format_ids(c0), format_ids(c1)
    rel = _map_unique(c2, lambda t: int(t[1:])).astype(np.int64)
    rel_ids, rinv, counts = np.unique(rel, return_inverse=True, return_counts=True)
    pos = np.empty(len(rel), dtype=np.int64)
    pos[multigraph_edge_order(du, dv)] = np.arange(len(rel))
    first_pos = np.full(len(rel_ids), np.iinfo(np.int64).max, dtype=np.int64)
    np.minimum.at(first_pos, rinv.reshape(-1), pos)
    valid = counts >= min_edges
    rel_order = [int(r) for r in rel_ids[valid][np.argsort(first_pos[valid], kind="stable")]]
    ui, vi = _index(du, nl.drugs, "drug"), _index(dv, nl.drugs, "drug")
    by_rel = np.argsort(rinv.reshape(-1), kind="stable")  # lines grouped by relation
    bounds = np.concatenate([[0], np.cumsum(counts)])
    rel_slot = {int(r): s for s, r in enumerate(rel_ids)}
    rels = []
    for r in rel_order:
        sel = by_rel[bounds[rel_slot[r]]:bounds[rel_slot[r] + 1]]
        rels.append(_sym_adjacency(ui[sel], vi[sel], nd))

    dp = _drug_protein(t0, t1, nl)
    ppi = _sym_adjacency(_index(format_ids(p0), nl.proteins, "protein"),
                         _index(format_ids(p1), nl.proteins, "protein"), npr)
    feat_drug, side_effects = _mono_features(mono_csv, nl.drugs)
    eye = np.arange(npr, dtype=np.int64)
    feat_prot = (np.stack([eye, eye], axis=1), np.ones(npr), (npr, npr))  # sp.identity(coo)

    # ---- DecagonDataSet assembly (DecagonDataSet.py:189-231, 276-292) ----
    adj: Dict[EdgeType, List[sp.csr_matrix]] = {(PPI, PPI): [ppi], (PPI, DRUG): [dp], (DRUG, DRUG): rels}
    if transpose:
        def tr(m):
            t = m.T.tocsr(copy=True)
            t.sort_indices()
            return t
        adj[(PPI, PPI)] = [ppi, tr(ppi)]
        adj[(DRUG, DRUG)] = rels + [tr(m) for m in rels]
        adj[(DRUG, PPI)] = [tr(dp)]

    def deg(ms):
        return [np.asarray(m.sum(axis=0)).reshape(-1) for m in ms]

    return PublicData(node_lists=nl, relation_ids=rel_order, adj=adj,
                      features={PPI: feat_prot, DRUG: feat_drug},
                      degrees={PPI: deg(adj[(PPI, PPI)]), DRUG: deg(adj[(DRUG, DRUG)])},
                      side_effects=side_effects)


def normalized(data: PublicData) -> Dict[EdgeType, List[CooTuple]]:
    """The COO tuples the model is fed (`adj_mats_i,j,k`): preprocess_graph of every matrix
    (minibatch.py:80-93), without the iterator's train/val/test edge masking."""
    from .sparse import preprocess_graph

    return {et: [preprocess_graph(m) for m in ms] for et, ms in data.adj.items()}


def write_public_csvs(prefix: str, seed: int = 0, n_proteins: int = 2000, n_drugs: int = 120,
                      n_side_effects: int = 6, n_ppi: int = 8000, n_targets: int = 900,
                      n_mono: int = 3000, n_mono_effects: int = 400,
                      combo_sizes: Optional[List[int]] = None) -> Tuple[str, str, str, str]:
    """Seeded files in the DecagonPublicData formats — headerless edge lists for PPI and
    targets, the preprocessed 3-column combo list, the mono side-effect CSV with its header —
    for tests and benches (the real files are not in the image).  Ids are drawn so that some
    end in '0' (the NodeIds collapse is exercised).  Returns (ppi, targets, combo, mono)."""
    rng = np.random.default_rng(seed)
    prot = rng.choice(np.arange(1, 10 ** 6), n_proteins, replace=False)
    drug = rng.choice(np.arange(1, 10 ** 8), n_drugs, replace=False)
    se = rng.choice(np.arange(1, 10 ** 6), max(n_side_effects, 1), replace=False)
    sizes = combo_sizes or [int(max(300, 2500 * (r + 1) ** -0.6)) for r in range(n_side_effects)]
    paths = tuple(f"{prefix}-{n}.csv" for n in ("ppi", "targets", "combo", "mono"))
    with open(paths[0], "w") as f:
        a, b = rng.integers(0, n_proteins, (2, n_ppi))
        f.writelines(f"{prot[x]},{prot[y]}\n" for x, y in zip(a, b))
    with open(paths[1], "w") as f:
        a, b = rng.integers(0, n_drugs, n_targets), rng.integers(0, n_proteins, n_targets)
        for x, y, flip in zip(a, b, rng.random(n_targets) < 0.1):
            d, p = f"CID{drug[x]:09d}", f"{prot[y]}"
            f.write(f"{p},{d}\n" if flip else f"{d},{p}\n")
    with open(paths[2], "w") as f:
        lines = []
        for r, s in enumerate(sizes):
            a, b = rng.integers(0, n_drugs, (2, s))
            lines += [f"CID{drug[x]:09d},CID{drug[y]:09d},C{se[r % len(se)]:07d}\n" for x, y in zip(a, b)]
        f.writelines(lines[i] for i in rng.permutation(len(lines)))
    with open(paths[3], "w") as f:
        f.write("STITCH,Individual Side Effect,Side Effect Name\n")
        eff = rng.choice(np.arange(1, 10 ** 7), n_mono_effects, replace=False)
        a, b = rng.integers(0, n_drugs + 5, n_mono), rng.integers(0, n_mono_effects, n_mono)
        for x, y in zip(a, b):
            d = f"CID{drug[x]:09d}" if x < n_drugs else f"CID{900000001 + 2 * x:09d}"
            f.write(f"{d},C{eff[y]:07d},name {y}\n")
    return paths
