"""Polypharmacy ingestion (decagon_amd/ingest.py) against hand-derived known
answers and the loop-level restatement in oracle/ingest_oracle.py.

Parity unpinned against the reference itself: importing its DecagonPublicData builders to
generate fixtures was refused in this environment and the reference holds none for them
(DESIGN.md §Ingestion).  The known answers below are derived by hand from the reference's
code (file:line in each test)."""
import numpy as np
import pytest

from decagon_amd import ingest
from oracle import ingest_oracle


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


@pytest.fixture
def kat_files(tmp_path):
    combo = _write(tmp_path, "combo.csv",
                   "CID3,CID4,C7\n"
                   "CID1,CID2,C5\n"
                   "CID2,CID3,C0000008\n"
                   "# a comment line\n"
                   "CID3,CID4,C7\n"
                   "CID20,CID30,C5\n")
    targets = _write(tmp_path, "targets.csv", "CID1,11\n12,CID2\nCID1,11\nCID9,13\n")
    ppi = _write(tmp_path, "ppi.csv", "11,12\n12,11\n13,13\n\n14,15\n")
    mono = _write(tmp_path, "mono.csv",
                  "STITCH,Individual Side Effect,Side Effect Name\n"
                  "CID1,C001,a\nCID1,C002,b\nCID77,C003,c\nCID2,C002,b\nCID2,C002,b\n")
    return ppi, targets, combo, mono


def test_format_ids_kat():
    # NodeIds.py:39-49: a trailing '0' maps the whole id to 0; otherwise digits, no leading 0s
    toks = ["CID000002170", "CID000012314", "C00512341", "SID123", "0", "10", "CID003000", " 12"]
    assert ingest.format_ids(toks).tolist() == [0, 12314, 512341, 123, 0, 0, 0, 12]
    assert [ingest_oracle.format_id(t) for t in toks] == [0, 12314, 512341, 123, 0, 0, 0, 12]
    with pytest.raises(ValueError):
        ingest.format_ids(["CID"])


def test_multigraph_edge_order_kat():
    # nodes inserted 3, 4, 1, 2; node 3 visits 4 (line 0, 3) then 2 (line 2); node 1 visits 2
    u = np.array([3, 1, 2, 3])
    v = np.array([4, 2, 3, 4])
    assert ingest.multigraph_edge_order(u, v).tolist() == [0, 3, 2, 1]


def test_public_data_kat(kat_files):
    d = ingest.load_public_data(*kat_files, min_edges=2)
    assert d.node_lists.drugs.tolist() == [0, 1, 2, 3, 4, 9]          # CID20/CID30 -> 0, CID9 from targets
    assert d.node_lists.proteins.tolist() == [11, 12, 13, 14, 15]
    # C8 has one line (< 2); C7 precedes C5 in the MultiGraph traversal (node 3 is first)
    assert d.relation_ids == [7, 5]
    assert list(d.adj) == [(0, 0), (0, 1), (1, 1), (1, 0)]            # DecagonDataSet.py:196-229
    r7, r5 = (m.toarray() for m in d.adj[(1, 1)][:2])
    e7 = np.zeros((6, 6)); e7[3, 4] = e7[4, 3] = 1
    e5 = np.zeros((6, 6)); e5[1, 2] = e5[2, 1] = 1; e5[0, 0] = 1      # the collapsed pair is a self-loop
    np.testing.assert_array_equal(r7, e7)
    np.testing.assert_array_equal(r5, e5)
    np.testing.assert_array_equal(d.adj[(1, 1)][2].toarray(), e7.T)
    dp = np.zeros((5, 6)); dp[0, 1] = dp[1, 2] = dp[2, 5] = 1
    np.testing.assert_array_equal(d.adj[(0, 1)][0].toarray(), dp)
    np.testing.assert_array_equal(d.adj[(1, 0)][0].toarray(), dp.T)
    ppi = np.zeros((5, 5)); ppi[0, 1] = ppi[1, 0] = ppi[2, 2] = ppi[3, 4] = ppi[4, 3] = 1
    np.testing.assert_array_equal(d.adj[(0, 0)][0].toarray(), ppi)
    coords, vals, shape = d.features[1]
    assert shape == (6, 3) and d.side_effects.tolist() == [1, 2, 3]  # C003 of an unlisted drug still counts
    assert coords.tolist() == [[1, 0], [1, 1], [2, 1]] and vals.tolist() == [1, 1, 1]
    assert d.features[0][2] == (5, 5)
    np.testing.assert_array_equal(d.degrees[1][0], e7.sum(axis=0))
    assert d.edge_types == {(0, 0): 2, (0, 1): 1, (1, 1): 4, (1, 0): 1}
    assert ingest.load_public_data(*kat_files, min_edges=1).relation_ids == [7, 8, 5]
    assert list(ingest.load_public_data(*kat_files, min_edges=2, transpose=False).adj) == [(0, 0), (0, 1), (1, 1)]


def test_combo_width_is_checked(tmp_path, kat_files):
    bad = _write(tmp_path, "bad.csv", "CID1,CID2,C5,name\n")
    with pytest.raises(ValueError):
        ingest.load_public_data(kat_files[0], kat_files[1], bad, kat_files[3])


@pytest.mark.parametrize("seed,min_edges", [(0, 500), (1, 300), (2, 1)])
def test_public_data_matches_oracle(tmp_path, seed, min_edges):
    paths = ingest.write_public_csvs(str(tmp_path / f"s{seed}"), seed=seed, n_proteins=300, n_drugs=60,
                                     n_side_effects=8, n_ppi=1500, n_targets=200, n_mono=600,
                                     n_mono_effects=80)
    d = ingest.load_public_data(*paths, min_edges=min_edges)
    proteins, drugs, rel_ids, adj, fd, degrees = ingest_oracle.load_public_data(*paths, min_edges=min_edges)
    assert d.node_lists.proteins.tolist() == proteins
    assert d.node_lists.drugs.tolist() == drugs
    assert d.relation_ids == rel_ids and len(rel_ids) > 0
    assert list(d.adj) == list(adj)
    for et in adj:
        assert len(d.adj[et]) == len(adj[et])
        for m, ref in zip(d.adj[et], adj[et]):
            np.testing.assert_array_equal(m.toarray(), ref)
            assert m.has_sorted_indices
    coords, vals, shape = d.features[1]
    dense = np.zeros(shape)
    dense[coords[:, 0], coords[:, 1]] = vals
    np.testing.assert_array_equal(dense, fd)
    assert coords.tolist() == np.argwhere(fd).tolist()                  # row-major, as coo of a dense matrix
    for t in (0, 1):
        for a, b in zip(d.degrees[t], degrees[t]):
            np.testing.assert_array_equal(a, b)


def test_normalized_tuples(kat_files):
    from decagon_amd.sparse import preprocess_graph

    d = ingest.load_public_data(*kat_files, min_edges=2)
    nz = ingest.normalized(d)
    for et, ms in d.adj.items():
        for m, (c, v, s) in zip(ms, nz[et]):
            c2, v2, s2 = preprocess_graph(m)
            np.testing.assert_array_equal(c, c2)
            np.testing.assert_array_equal(v, v2)
            assert s == s2
