"""CPU: the oracle pinned against the golden vectors, and the product's host-side
preprocessing against the reference-generated inputs.

synthetic_S.npz holds the reference's own normalised training adjacencies (produced by
decagon.deep.minibatch.EdgeMinibatchIterator in tests/golden/make_golden.py) and the raw
training edges they came from; dedicom_kat.npz the reference's trained DEDICOM parameters.
"""
import numpy as np
import pytest

from conftest import rel_err
from oracle import decagon_oracle as orc


def _graph(z):
    edge_types = {(int(i), int(j)): int(k) for i, j, k in z["edge_types"]}
    adj = {et: [(z[f"adj_{et[0]}_{et[1]}_{k}_coords"], z[f"adj_{et[0]}_{et[1]}_{k}_values"],
                 tuple(int(s) for s in z[f"adj_{et[0]}_{et[1]}_{k}_shape"])) for k in range(K)]
           for et, K in edge_types.items()}
    return edge_types, adj


def test_fixture_matches_survey_counts(golden_S):
    """SURVEY §8a measured these nnz with the reference iterator."""
    z = golden_S
    want = {"0_0_0": 13065, "0_0_1": 13065, "0_1_0": 12572, "1_0_0": 12572, "1_1_0": 16860,
            "1_1_1": 7538, "1_1_2": 2952, "1_1_3": 16860, "1_1_4": 7538, "1_1_5": 2952}
    for k, n in want.items():
        assert z[f"adj_{k}_values"].shape[0] == n


def test_oracle_reproduces_golden_forward(golden_S):
    z = golden_S
    edge_types, adj = _graph(z)
    n = {0: int(z["n_nodes"][0]), 1: int(z["n_nodes"][1])}
    feats = {t: (np.stack([np.arange(n[t])] * 2, 1), np.ones(n[t]), (n[t], n[t])) for t in n}
    w1 = {et: [z[f"w1_{et[0]}_{et[1]}_{k}"].astype(np.float64) for k in range(K)] for et, K in edge_types.items()}
    w2 = {et: [z[f"w2_{et[0]}_{et[1]}_{k}"].astype(np.float64) for k in range(K)] for et, K in edge_types.items()}
    h1, emb = orc.decagon_forward(edge_types, adj, feats, w1, w2)
    assert rel_err(h1[0], z["hidden1_0"]) < 1e-12 and rel_err(h1[1], z["hidden1_1"]) < 1e-12
    assert rel_err(emb[0], z["emb_0"]) < 1e-12 and rel_err(emb[1], z["emb_1"]) < 1e-12
    # l2_normalize semantics: rows of each per-group output have unit norm or are zero
    assert np.all(h1[0] >= 0)


def test_scalar_c_oracle_agrees_with_float64(golden_S):
    """The timed CPU baseline (oracle/gcn_ref.c, fp32) computes the same forward."""
    from decagon_amd.synthetic import load_S
    from oracle import cpu_forward

    z = golden_S
    g = load_S()
    w1 = {et: np.stack([z[f"w1_{et[0]}_{et[1]}_{k}"] for k in range(K)]) for et, K in g.edge_types.items()}
    w2 = {et: np.stack([z[f"w2_{et[0]}_{et[1]}_{k}"] for k in range(K)]) for et, K in g.edge_types.items()}
    fwd = cpu_forward.Forward(cpu_forward.load(), g, 64, 32, w1=w1, w2=w2)
    h1, emb = fwd.run()
    assert rel_err(h1[1], z["hidden1_1"]) < 1e-5
    assert rel_err(emb[0], z["emb_0"]) < 1e-5 and rel_err(emb[1], z["emb_1"]) < 1e-5


def test_batches_and_losses(golden_S):
    z = golden_S
    for b in range(4):
        pos, neg = z[f"batch{b}_outputs"], z[f"batch{b}_neg_outputs"]
        assert abs(orc.hinge_loss(pos, neg, 0.1) - float(z[f"batch{b}_cost"])) < 1e-9
        assert z[f"batch{b}_edges"].shape == (512, 2)


def test_batch_predict_is_diag_of_predict(golden_S):
    z = golden_S
    emb = [z["emb_0"], z["emb_1"]]
    rng = np.random.default_rng(0)
    G = rng.standard_normal((32, 32))
    L = np.diag(rng.standard_normal(32))
    rows, cols = rng.integers(0, 400, 50), rng.integers(0, 400, 50)
    full = orc.predict(emb, 1, 1, G, L)
    assert np.allclose(orc.batch_predict(emb, 1, 1, G, L, rows, cols), full[rows, cols])


def test_dedicom_kat_against_np_predictor(golden_kat):
    """The reference's trained R (32x32) and D_r (6 diagonal 32x32), NpPredictor.py:304."""
    z = golden_kat
    R = z["R"].astype(np.float64)
    E = z["E"].astype(np.float64)
    assert R.shape == (32, 32) and z["Ddiag"].shape == (6, 32)
    for r in range(6):
        D = np.diag(z["Ddiag"][r].astype(np.float64))
        assert rel_err(orc.np_predictor_dedicom(E, E, D, R), z[f"scores_{r}"]) < 1e-12
        assert rel_err(orc.predict([E], 0, 0, R, D), z[f"scores_{r}"]) < 1e-12


def test_product_preprocess_graph_matches_reference(golden_S):
    """decagon_amd.preprocess_graph (the product's host normalisation) reproduces the
    reference's EdgeMinibatchIterator.preprocess_graph output (minibatch.py:80-93) on the
    reference's own training edges — same entries, float64 values equal."""
    import scipy.sparse as sp

    from decagon_amd.sparse import preprocess_graph

    z = golden_S
    for key, linked in (("0_0_0", None), ("0_1_0", None), ("1_1_0", None), ("1_1_2", None)):
        tr = z[f"train_{key}"]
        shape = tuple(int(s) for s in z[f"adj_{key}_shape"])
        adj = sp.csr_matrix((np.ones(tr.shape[0]), (tr[:, 0], tr[:, 1])), shape=shape)
        coords, vals, shp = preprocess_graph(adj)
        ref_c, ref_v = z[f"adj_{key}_coords"], z[f"adj_{key}_values"]
        assert shp == shape
        a = sp.coo_matrix((vals, (coords[:, 0], coords[:, 1])), shape=shape).tocsr()
        b = sp.coo_matrix((ref_v, (ref_c[:, 0], ref_c[:, 1])), shape=shape).tocsr()
        a.sort_indices()
        b.sort_indices()
        assert np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
        assert np.max(np.abs(a.data - b.data)) <= 1e-15 * np.max(np.abs(b.data))


def test_transposed_relations_are_flipped_copies(golden_S):
    """The reference links transposed relations to their originals (minibatch.py:137-172):
    relation (0,0,1) is (0,0,0) with coordinates flipped and the same values."""
    z = golden_S
    assert np.array_equal(z["adj_0_0_1_coords"], z["adj_0_0_0_coords"][:, ::-1])
    assert np.array_equal(z["adj_0_0_1_values"], z["adj_0_0_0_values"])
    assert np.array_equal(z["adj_1_0_0_coords"], z["adj_0_1_0_coords"][:, ::-1])


def test_unigram_distribution():
    p = orc.unigram_distribution(np.array([0.0, 1.0, 16.0]))
    assert p[0] == 0 and abs(p[2] / p[1] - 8.0) < 1e-12


def test_sigmoid_np114_saturation():
    """The reference's sigmoid forms saturate where numpy 1.14 + float32 logits put them:
    main.py (float32 exp, float64 1/(1+e)) at 1.0 above ≈36.7 and 0.0 below ≈-88.7 (float32
    exp overflow); MathUtils.sigmoid on the float32 array at 1.0 above ≈16.6."""
    from oracle.decagon_oracle import sigmoid_np114

    m = sigmoid_np114(np.array([37.0, 36.0, -88.0, -89.0, np.nan], np.float32), "main")
    assert m[0] == 1.0 and m[1] < 1.0 and m[2] > 0.0 and m[3] == 0.0 and m[4] == 0.0
    assert m.dtype == np.float64
    e = sigmoid_np114(np.array([17.0, 16.0, 0.0], np.float32), "evaluator")
    assert e.dtype == np.float32 and e[0] == 1.0 and e[1] < 1.0 and e[2] == np.float32(0.5)
