"""Generate the committed golden fixtures under tests/golden/.

RUNS ONLY IN THE BUILD CONTAINER: it imports the reference's own input pipeline from
/root/reference (read-only; bytecode writing disabled) — `decagon.deep.minibatch`
(EdgeMinibatchIterator, preprocess_graph) and `main/Utils/Sparse.py` (RelationCsrMatrix) —
which need only numpy/scipy.  TensorFlow (the reference's compute backend) is absent, so
expected OUTPUTS come from the float64 restatement in oracle/decagon_oracle.py.  Nothing
of the reference is copied: the fixtures hold numbers only.

Fixtures:
  synthetic_S.npz   config S (BASELINE configs[0/1]): main.py's 5-relation / 10-matrix toy
                    graph (main.py:137-217), train adjacencies exactly as the reference's
                    EdgeMinibatchIterator normalizes them (minibatch.py:80-93, 174-233,
                    transposes linked as DecagonDataSet does, DecagonDataSet.py:212-231),
                    seeded glorot weights, 4 minibatches from the reference iterator
                    (minibatch.py:278-313) with injected unigram negatives, and the
                    restated forward outputs.
  dedicom_kat.npz   the reference's trained DEDICOM parameters (ndarray-dumpGlobalRelations.npy,
                    ndarray-dumpEmbeddingImportance.npyz.npz arr_0) with seeded embeddings and
                    the NpPredictor formula's scores (main/Predictor/NpPredictor.py:304).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys
from itertools import combinations
from pathlib import Path

import numpy as np
import scipy.sparse as sp

sys.dont_write_bytecode = True
REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

from oracle import decagon_oracle as orc  # noqa: E402

H1, H2 = 64, 32
BATCH = 512
MARGIN = 0.1


def _load_reference():
    if not REF.exists():
        raise SystemExit("make_golden.py needs /root/reference (build container only)")
    sys.path.insert(0, str(REF))
    from decagon.deep import minibatch  # seeds np.random with 123 at import (minibatch.py:9)

    spec = importlib.util.spec_from_file_location("ref_sparse", REF / "main/Utils/Sparse.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return minibatch, mod.RelationCsrMatrix


def build_synthetic_graph(RelationCsrMatrix):
    """main.py:137-183 toy graph (after np.random.seed(0), main.py:31)."""
    import networkx as nx

    n_genes, n_drugs, n_rel = 500, 400, 3
    gene_net = nx.planted_partition_graph(50, 10, 0.2, 0.05, seed=42)
    gene_adj = sp.csr_matrix(nx.adjacency_matrix(gene_net), dtype=np.float64)
    gene_degrees = np.asarray(gene_adj.sum(axis=0)).ravel()
    gene_drug = sp.csr_matrix((10 * np.random.randn(n_genes, n_drugs) > 15).astype(int))
    common = (gene_drug.T @ gene_drug).toarray()
    drug_drug = []
    iu = np.array(list(combinations(range(n_drugs), 2)))
    for i in range(n_rel):
        mat = np.zeros((n_drugs, n_drugs))
        hit = iu[common[iu[:, 0], iu[:, 1]] == i + 4]
        mat[hit[:, 0], hit[:, 1]] = 1.0
        mat[hit[:, 1], hit[:, 0]] = 1.0
        drug_drug.append(sp.csr_matrix(mat))
    drug_degrees = [np.asarray(m.sum(axis=0)).ravel() for m in drug_drug]

    ppi = RelationCsrMatrix(gene_adj)
    g2d = RelationCsrMatrix(gene_drug)
    dd = [RelationCsrMatrix(m) for m in drug_drug]
    adj = {
        (0, 0): [ppi, ppi.transpose(copy=True, setId=True)],
        (0, 1): [g2d],
        (1, 0): [g2d.transpose(copy=True, setId=True)],
        (1, 1): dd + [m.transpose(copy=True, setId=True) for m in dd],
    }
    degrees = {0: [gene_degrees, gene_degrees], 1: drug_degrees + drug_degrees}
    return adj, degrees, (n_genes, n_drugs)


def glorot(rng, n_in, n_out):
    r = np.sqrt(6.0 / (n_in + n_out))  # inits.py:5-12
    return rng.uniform(-r, r, size=(n_in, n_out)).astype(np.float32)


def main():
    minibatch, RelationCsrMatrix = _load_reference()
    np.random.seed(0)  # main.py:31
    adj, degrees, (n0, n1) = build_synthetic_graph(RelationCsrMatrix)
    edge_types = {k: len(v) for k, v in adj.items()}
    decoders = {(0, 0): "bilinear", (0, 1): "bilinear", (1, 0): "bilinear", (1, 1): "dedicom"}
    nodes = {0: n0, 1: n1}
    feat = {0: (np.stack([np.arange(n0)] * 2, 1), np.ones(n0), (n0, n0)),
            1: (np.stack([np.arange(n1)] * 2, 1), np.ones(n1), (n1, n1))}

    it = minibatch.EdgeMinibatchIterator(adj_mats=adj, feat=feat, edge_types=edge_types,
                                         drug_drug_test_edges={}, batch_size=BATCH,
                                         val_test_size=0.05)
    out = {}
    et_list = list(edge_types)
    out["edge_types"] = np.array([[i, j, k] for (i, j), k in edge_types.items()], np.int32)
    out["decoders"] = np.array([decoders[et] for et in et_list])
    out["n_nodes"] = np.array([n0, n1], np.int32)
    adj_f64 = {}
    for (i, j) in et_list:
        adj_f64[i, j] = []
        for k in range(edge_types[i, j]):
            coords, values, shape = it.adj_train[i, j][k]
            out[f"adj_{i}_{j}_{k}_coords"] = np.asarray(coords, np.int32)
            out[f"adj_{i}_{j}_{k}_values"] = np.asarray(values, np.float64)
            out[f"adj_{i}_{j}_{k}_shape"] = np.asarray(shape, np.int64)
            out[f"deg_{i}_{j}_{k}"] = np.asarray(degrees[i][k], np.float64)
            adj_f64[i, j].append((np.asarray(coords), np.asarray(values, np.float64), shape))
            # raw (un-normalized) training adjacency: checks our preprocess_graph restatement
            tr = it.train_edges[i, j][k]
            out[f"train_{i}_{j}_{k}"] = np.asarray(tr, np.int32)

    rng = np.random.default_rng(20241015)
    w1, w2, dec = {}, {}, {}
    for (i, j) in et_list:
        w1[i, j] = [glorot(rng, nodes[j], H1) for _ in range(edge_types[i, j])]
        w2[i, j] = [glorot(rng, H1, H2) for _ in range(edge_types[i, j])]
        for k in range(edge_types[i, j]):
            out[f"w1_{i}_{j}_{k}"] = w1[i, j][k]
            out[f"w2_{i}_{j}_{k}"] = w2[i, j][k]
        p = {}
        if decoders[i, j] == "bilinear":
            for k in range(edge_types[i, j]):
                p["relation_%d" % k] = glorot(rng, H2, H2)
        elif decoders[i, j] == "dedicom":
            p["global_interaction"] = glorot(rng, H2, H2)
            for k in range(edge_types[i, j]):
                p["local_variation_%d" % k] = glorot(rng, H2, 1).reshape(-1)
        elif decoders[i, j] == "distmult":
            for k in range(edge_types[i, j]):
                p["relation_%d" % k] = glorot(rng, H2, 1).reshape(-1)
        for name, v in p.items():
            out[f"dec_{i}_{j}_{name}"] = v
        dec[i, j] = p

    feats64 = {t: (f[0], f[1].astype(np.float64), f[2]) for t, f in feat.items()}
    w1_64 = {k: [w.astype(np.float64) for w in v] for k, v in w1.items()}
    w2_64 = {k: [w.astype(np.float64) for w in v] for k, v in w2.items()}
    h1, emb = orc.decagon_forward(edge_types, adj_f64, feats64, w1_64, w2_64)
    out["hidden1_0"], out["hidden1_1"] = h1[0], h1[1]
    out["emb_0"], out["emb_1"] = emb[0], emb[1]
    dec64 = {k: {n: np.asarray(v, np.float64) for n, v in p.items()} for k, p in dec.items()}
    inters, varies = orc.latent_matrices(edge_types, decoders, dec64, H2)

    # four minibatches exactly as the reference iterator yields them (main.py:299-304)
    class _PH(dict):
        def __missing__(self, key):
            return key
    it.shuffle()
    for b in range(4):
        fd = it.next_minibatch_feed_dict(_PH())
        e = int(fd["batch_edge_type_idx"])
        rt, ct = int(fd["batch_row_edge_type"]), int(fd["batch_col_edge_type"])
        batch = np.asarray(fd["batch"], np.int32)
        i, j, k = it.idx2edge_type[e]
        probs = orc.unigram_distribution(degrees[i][k])
        neg = rng.choice(len(probs), size=batch.shape[0], p=probs).astype(np.int32)
        pos_s = orc.batch_predict(emb, rt, ct, inters[e], varies[e], batch[:, 0], batch[:, 1])
        neg_s = orc.batch_predict(emb, rt, ct, inters[e], varies[e], neg, batch[:, 1])
        out[f"batch{b}_edges"] = batch
        out[f"batch{b}_meta"] = np.array([e, rt, ct], np.int32)
        out[f"batch{b}_neg"] = neg
        out[f"batch{b}_outputs"] = pos_s
        out[f"batch{b}_neg_outputs"] = neg_s
        out[f"batch{b}_cost"] = np.array(orc.hinge_loss(pos_s, neg_s, MARGIN))
        out[f"batch{b}_xent"] = np.array(orc.xent_loss(pos_s, neg_s, 1.0))
    # full predictions for one bilinear and one dedicom relation (optimizer.py:87-106)
    for e, (rt, ct) in ((2, (0, 1)), (7, (1, 1))):  # (0,1,0) bilinear, (1,1,3) dedicom
        out[f"predictions_{e}"] = orc.predict(emb, rt, ct, inters[e], varies[e])
    np.savez_compressed(HERE / "synthetic_S.npz", **out)

    # DEDICOM known-answer test on the reference's trained parameters
    R = np.load(REF / "ndarray-dumpGlobalRelations.npy", allow_pickle=False)
    with np.load(REF / "ndarray-dumpEmbeddingImportance.npyz.npz", allow_pickle=False) as z:
        D = z["arr_0"]
    rng2 = np.random.default_rng(7)
    E = rng2.standard_normal((96, 32)).astype(np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    kat = {"R": R, "Ddiag": np.stack([np.diag(x) for x in D]).astype(np.float32), "E": E}
    for r in range(D.shape[0]):
        ref = orc.np_predictor_dedicom(E.astype(np.float64), E.astype(np.float64),
                                       D[r].astype(np.float64), R.astype(np.float64))
        ours = orc.predict([E.astype(np.float64)], 0, 0, R.astype(np.float64), D[r].astype(np.float64))
        assert np.allclose(ref, ours, rtol=1e-12, atol=1e-12)
        kat[f"scores_{r}"] = ref
    np.savez_compressed(HERE / "dedicom_kat.npz", **kat)
    print("wrote", HERE / "synthetic_S.npz", HERE / "dedicom_kat.npz")
    print({k: v for k, v in edge_types.items()},
          {f"{i}{j}{k}": len(out[f'adj_{i}_{j}_{k}_values']) for (i, j) in et_list for k in range(edge_types[i, j])})


if __name__ == "__main__":
    main()
