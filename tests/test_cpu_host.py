"""CPU: host-side logic of the product — sparse formats, the C-ABI library (loads, exports
every symbol include/decagon_hip.h declares, rejects bad arguments before touching the
GPU), the drop-in surface's construction contract, chunk policy and synthetic graphs."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = Path(__file__).resolve().parents[1]


def test_coo_to_csr_keeps_in_row_order():
    from decagon_amd.sparse import coo_to_csr

    coords = np.array([[2, 5], [0, 1], [2, 0], [0, 3]])
    vals = np.array([1.0, 2.0, 3.0, 4.0])
    h = coo_to_csr(coords, vals, (3, 6))
    assert h.rowptr.tolist() == [0, 2, 2, 4]
    assert h.col.tolist() == [1, 3, 5, 0]  # feed order kept inside each row
    assert h.val.dtype == np.float32 and h.val.tolist() == [2.0, 4.0, 1.0, 3.0]


def test_coo_to_csr_rejects_out_of_range():
    from decagon_amd.sparse import coo_to_csr

    with pytest.raises(ValueError):
        coo_to_csr(np.array([[0, 7]]), np.array([1.0]), (3, 6))


def test_stack_relations_offsets():
    from decagon_amd.sparse import coo_to_csr, sparse_to_tuple, stack_relations

    rng = np.random.default_rng(0)
    mats = [sp.random(7, 5, density=0.3, random_state=rng, format="csr") for _ in range(3)]
    st = stack_relations([coo_to_csr(*sparse_to_tuple(m)) for m in mats])
    assert st.rowptr.shape == (3 * 7 + 1,)
    for k, m in enumerate(mats):
        for r in range(7):
            a, b = st.rowptr[k * 7 + r], st.rowptr[k * 7 + r + 1]
            assert b - a == m.indptr[r + 1] - m.indptr[r]
            assert sorted(st.col[a:b].tolist()) == sorted(m.indices[m.indptr[r]:m.indptr[r + 1]].tolist())


def test_is_identity():
    from decagon_amd.sparse import is_identity, sparse_to_tuple

    assert is_identity(*sparse_to_tuple(sp.identity(9).tocoo()))
    assert not is_identity(*sparse_to_tuple((2 * sp.identity(9)).tocoo()))


def _declared_symbols():
    hdr = (ROOT / "include" / "decagon_hip.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t)\s+(dg_\w+)\s*\(", hdr, re.M)))


def test_library_exports_every_declared_symbol():
    from decagon_amd import _lib

    lib = _lib.load()
    syms = _declared_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} not bound in _lib.SIGNATURES"
    assert lib.dg_abi_version() == _lib.ABI_VERSION


def test_integration_doc_matches_abi():
    """INTEGRATION.md is the maintainer's binding guide: the ABI number it states and its
    stub asserts, the stubs' argtypes, and its table's coverage of every declared entry point
    must match the library (a stale doc fails here, not in a maintainer's first call)."""
    from decagon_amd import _lib

    doc = (ROOT / "INTEGRATION.md").read_text()
    stated = {int(x) for x in re.findall(r"`dg_abi_version\(\)` returns (\d+)", doc)}
    asserted = {int(x) for x in re.findall(r"dg_abi_version\(\) == (\d+)", doc)}
    assert stated == {_lib.ABI_VERSION} and asserted == {_lib.ABI_VERSION}, (stated, asserted)
    names = {"c_void_p": ctypes.c_void_p, "c_int32": ctypes.c_int32, "c_int64": ctypes.c_int64,
             "c_float": ctypes.c_float}
    stubs = re.findall(r"_lib\.(dg_\w+)\.argtypes = \[([^\]]*)\]", doc, re.S)
    assert len(stubs) >= 2
    for fn, body in stubs:
        got = [names[t.strip()] for t in body.replace("\n", " ").split(",") if t.strip()]
        assert got == list(_lib.SIGNATURES[fn][1]), fn
    table = set(re.findall(r"`(dg_\w+)`", doc))
    missing = [s for s in _declared_symbols() if s not in table and s != "dg_abi_version"]
    assert not missing, f"INTEGRATION.md's table does not list {missing}"


def test_abi_rejects_bad_arguments_without_a_device():
    """Argument checks run on the host before any HIP call, so they work here."""
    from decagon_amd import _lib

    lib = _lib.load()
    assert lib.dg_spmm_groups_f32(None, 1, 64, None) == _lib.DG_EINVAL
    g = (_lib.DgRelGroup * 1)()
    assert lib.dg_spmm_groups_f32(g, 1, 6, None) == _lib.DG_EINVAL  # d % 4 != 0
    assert lib.dg_spmm_groups_f32(g, 9, 64, None) == _lib.DG_ETOOMANY
    g[0].n_rows, g[0].n_chunks, g[0].x_rows = 10, 1, 10
    g[0].rowptr, g[0].x, g[0].out = 16, 17, 32  # misaligned x
    g[0].x_ld = 64
    assert lib.dg_spmm_groups_f32(g, 1, 64, None) == _lib.DG_EALIGN
    assert lib.dg_decoder_score_f32(None, 32, None, 32, None, None, 4, None, None, 33, None, None) == _lib.DG_EINVAL
    assert lib.dg_gemm_f32(None, 1, None) == _lib.DG_EINVAL
    assert lib.dg_decoder_hinge_f32(*([None, 32, None, 32, None, None, None, None, 0, 0, 0, 4, None, None, 32, 0.1] + [None] * 6)) == _lib.DG_EINVAL
    e = (_lib.DgEpiGroup * 1)()
    assert lib.dg_gcn_epilogue_f32(e, 1, None, 10, 64, 128, None) == _lib.DG_EINVAL  # bad flags
    assert lib.dg_unigram_sample(None, 0, 5, 0, 0, None, None) == _lib.DG_EINVAL
    # a pushed group sum needs a peer exchange descriptor (dg_gcn_epilogue_peer_f32), and the
    # bf16 scorers need the tables' row counts (ABI 34)
    t = (_lib.DgEpiTarget * 1)()
    assert lib.dg_gcn_epilogue_peer_f32(t, 1, 64, 1, None, None) == _lib.DG_EINVAL
    assert lib.dg_decoder_score_bf16_paired(*([None, 256, 0, None, 256, 0] + [None] * 3 + [1, None, None, 256, None, None])) == _lib.DG_EINVAL
    # ABI 37: dg_spmm_csr_f32's beta must be finite; dg_rownorm_l2_f32 takes relu only, d % 4 == 0
    f = ctypes.c_float
    assert lib.dg_spmm_csr_f32(16, 16, 16, 10, 10, 16, 64, 16, 64, 64, f(float("nan")), None) == _lib.DG_EINVAL
    assert lib.dg_spmm_csr_f32(16, 16, 16, 10, 10, 16, 64, 16, 64, 64, f(float("inf")), None) == _lib.DG_EINVAL
    assert lib.dg_spmm_csr_f32(16, 16, 16, 10, 10, 16, 64, 16, 32, 64, f(0.0), None) == _lib.DG_EINVAL  # ldy != d
    assert lib.dg_spmm_csr_f32(16, 16, 16, 0, 10, 16, 64, 16, 64, 64, f(1.0), None) == _lib.DG_OK  # no rows
    assert lib.dg_rownorm_l2_f32(16, 16, 10, 64, _lib.DG_EPI_L2NORM, None) == _lib.DG_EINVAL
    assert lib.dg_rownorm_l2_f32(16, 16, 10, 62, 0, None) == _lib.DG_EINVAL
    assert lib.dg_rownorm_l2_f32(None, None, 0, 64, 0, None) == _lib.DG_OK
    # ABI 38: a staged group's variable chunk table is checked before any launch
    for cs in ([0, 2, 2, 5], [1, 5], [0, 4], [0] + list(range(5, 70, 65)) + [70]):
        cs_arr = np.asarray(cs, np.int32)
        grp = (_lib.DgStagedGroup * 1)()
        g = grp[0]
        g.pairs = g.jm = g.jmoff = g.x = g.out = 4096
        g.x_ld, g.n_rows, g.n_cols, g.n_rels, g.out_chunk = 64, 10, 10, 5 if cs[-1] != 70 else 70, 4
        g.x_rows, g.jm_len = 640, 36 + 1024
        g.chunk_start, g.n_chunks = cs_arr.ctypes.data, len(cs) - 1
        if cs[-1] == 70:  # chunk of 65 relations
            cs_arr = np.asarray([0, 65, 70], np.int32)
            g.chunk_start, g.n_chunks = cs_arr.ctypes.data, 2
        assert lib.dg_spmm_staged_f32(grp, 1, 64, None) == _lib.DG_EINVAL, cs


def test_merge_chunks_layout():
    from decagon_amd.sparse import coo_to_csr, merge_chunks, sparse_to_tuple

    rng = np.random.default_rng(2)
    mats = [sp.random(8, 6, density=0.4, random_state=rng, format="csr") for _ in range(5)]
    slabs = [3, 0, 1, 6, 2]
    m = merge_chunks([coo_to_csr(*sparse_to_tuple(x)) for x in mats], slabs, 2, 7)
    assert m.n_chunks == 3 and m.rowptr.shape == (3 * 8 + 1,) and m.x_rows == 42
    X = rng.standard_normal((42, 4))
    for c in range(3):
        for r in range(8):
            a, b = m.rowptr[c * 8 + r], m.rowptr[c * 8 + r + 1]
            got = (m.val[a:b, None] * X[m.vcol[a:b]]).sum(0)
            want = sum((mats[k] @ X[slabs[k] * 6:(slabs[k] + 1) * 6])[r] for k in range(2 * c, min(5, 2 * c + 2)))
            assert np.allclose(got, want)


def test_choose_chunk_policy():
    from decagon_amd.engine import choose_chunk

    assert choose_chunk(6, 400, 55000, 64) == 6            # config S (1,1): one chunk
    c = choose_chunk(1928, 645, 20_100_000, 64)            # config P (1,1): many chunks
    assert 8 <= c <= 128
    assert choose_chunk(1, 100, 10, 64) == 1


def test_model_surface_constructs_like_the_reference():
    import decagon_amd as dg

    et = {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 6}
    dec = {(0, 0): "bilinear", (0, 1): "bilinear", (1, 0): "bilinear", (1, 1): "dedicom"}
    ph = dg.construct_placeholders(et)
    assert "adj_mats_1,1,5" in ph and "feat_1" in ph and ph["dropout"].has_default
    m = dg.DecagonModel(ph, {0: 500, 1: 400}, {0: 500, 1: 400}, et, dec)
    assert len(m.latent_inters) == len(m.latent_varies) == 10
    assert len(m.embeddings) == 2 and set(m.hidden1) == {0, 1}
    # variable layout of layers.py / model.py
    w = [n for n in m.vars if "graphconvolutionsparsemulti" in n and n.endswith("weights_0:0")]
    assert w and m.vars[w[0]].shape in {(500, 64), (400, 64)}
    assert any(n.endswith("global_interaction:0") for n in m.vars)
    assert sum(1 for n in m.vars if "local_variation_" in n) == 6
    with pytest.raises(AssertionError):
        dg.DecagonModel(ph, {0: 500, 1: 400}, {0: 500, 1: 400}, et, dec, bogus=1)
    with pytest.raises(ValueError):
        dg.DecagonModel(ph, {0: 500, 1: 400}, {0: 500, 1: 400}, et, {**dec, (1, 1): "nope"})
    opt = dg.DecagonOptimizer(m.embeddings, m.latent_inters, m.latent_varies,
                              {0: [np.ones(500)] * 2, 1: [np.ones(400)] * 6}, et,
                              {e: [(500 if e[0] == 0 else 400, 0)] * k for e, k in et.items()}, ph)
    for attr in ("outputs", "neg_outputs", "cost", "predictions", "opt_op", "batch_edge_type_idx", "preds"):
        assert hasattr(opt, attr)
    assert opt.obj_type2n == {0: 500, 1: 400}


def test_session_requires_a_device():
    import torch

    import decagon_amd as dg

    if torch.cuda.is_available():
        pytest.skip("device present")
    with pytest.raises(RuntimeError):
        dg.Session()


def test_act_kind_probe():
    from decagon_amd.layers import act_kind, relu

    assert act_kind(lambda x: x) == "identity"
    assert act_kind(relu) == "relu"
    with pytest.raises(ValueError):
        act_kind(lambda x: 2 * x)


def test_synthetic_P_shape_small():
    from decagon_amd.synthetic import make_P

    g = make_P(seed=1, n_proteins=500, n_drugs=60, n_side_effects=12, ppi_edges=2000, target_edges=300)
    assert g.edge_types == {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 24}
    c = g.csr()
    assert c[(1, 0)][0].shape == (60, 500) and c[(0, 1)][0].shape == (500, 60)
    # every drug-drug relation is symmetric and includes self loops (A + I)
    r = c[(1, 1)][0]
    dense = np.zeros((60, 60))
    for i in range(60):
        dense[i, r.col[r.rowptr[i]:r.rowptr[i + 1]]] = r.val[r.rowptr[i]:r.rowptr[i + 1]]
    assert np.allclose(dense, dense.T) and np.all(np.diag(dense) > 0)


def test_flags_defaults_match_main_py():
    from decagon_amd import FLAGS

    assert FLAGS.hidden1 == 64 and FLAGS.hidden2 == 32 and FLAGS.batch_size == 512
    assert FLAGS.max_margin == 0.1 and FLAGS.learning_rate == 0.001


def test_alias_table_encodes_the_unigram_distribution():
    from decagon_amd.sampling import alias_table, table_distribution
    from oracle.decagon_oracle import unigram_distribution

    rng = np.random.default_rng(3)
    for deg in (rng.integers(0, 100, 645).astype(float), np.array([0.0, 0.0, 5.0]), np.ones(7)):
        tab = alias_table(deg)
        assert tab.shape == (deg.shape[0], 2)
        assert np.max(np.abs(table_distribution(tab) - unigram_distribution(deg))) < 1e-7
    with pytest.raises(ValueError):
        alias_table(np.zeros(4))


@pytest.mark.parametrize("builder", ["feed", "library"])
def test_staged_layout_reproduces_every_relation(builder):
    """The staged layout (sparse.staged_layout) holds each relation exactly: rebuilding A_k
    from vinfo / woff / rlw / pairs gives the matrix back.  Long rows become groups of 2, 4 or
    8 equal-length segments (zero-column padding), groups sit on consecutive lanes starting at
    a multiple of their size (inside one 64-lane wave and one 16-lane DPP row), lanes are sorted by length, at most `lanes` of them, and every wave's block
    is dense: lane j's pair at diagonal m sits at woff + 64 m + j (holes are zero pairs).  With
    the library's block builder (kernels.staged_block) a lane's nonzeros may sit on any of its
    wave's diagonals and holes read one of the sixteen zero columns n_c .. n_c + 15."""
    import scipy.sparse as sp

    from decagon_amd.sparse import coo_to_csr, sparse_to_tuple, staged_layout

    rng = np.random.default_rng(3)
    n_r, n_c = 150, 30
    mats = [sp.random(n_r, n_c, density=dn, random_state=int(rng.integers(1 << 30)), format="csr",
                      dtype=np.float32) for dn in (0.3, 0.0, 0.05, 0.9)]
    lanes = 256
    block = None
    if builder == "library":
        from decagon_amd import kernels
        block = kernels.staged_block
    lay = staged_layout([coo_to_csr(*sparse_to_tuple(m)) for m in mats], block, lanes=lanes)
    vals = lay.pairs[:, 1].view(np.float32)
    covered = np.zeros(len(lay.pairs), bool)
    for k, m in enumerate(mats):
        jm = lay.jm[lay.jmoff[k]:lay.jmoff[k + 1]]
        n_w, big = int(jm[0]), int(jm[1])
        woff, rw = jm[4:20].astype(np.int64), jm[20:36].astype(np.int64)
        rlw, wbig = rw & 0xFFFF, rw >> 16                                 # per wave: diagonals, largest group
        vinfo = jm[36:].astype(np.int64)
        assert len(vinfo) == 64 * n_w and 64 * n_w <= lanes
        assert np.all(rlw[n_w:] == 0) and np.all(rlw % 4 == 0)
        row, seg, gsz, vlen = vinfo & 1023, (vinfo >> 10) & 7, ((vinfo >> 13) & 7) + 1, vinfo >> 16
        assert np.all(np.diff(vlen) <= 0)                                 # sorted by length
        assert big == (gsz.max() if n_w else 1)
        for w in range(n_w):
            assert wbig[w] == gsz[64 * w:64 * w + 64].max()
        for i in range(64 * n_w):                                         # groups inside a wave
            if row[i] != 1023 and seg[i] == 0:
                assert gsz[i] in (1, 2, 4, 8) and i % gsz[i] == 0           # aligned power-of-two group
                assert i // 64 == (i + gsz[i] - 1) // 64
                assert np.all(row[i:i + gsz[i]] == row[i]) and np.all(seg[i:i + gsz[i]] == np.arange(gsz[i]))
        got = np.zeros((n_r, n_c), np.float64)
        for w in range(n_w):
            assert woff[w] % 64 == 0 and vlen[64 * w] <= rlw[w]
            blk = slice(woff[w], woff[w] + 64 * rlw[w])
            assert not covered[blk].any()
            covered[blk] = True
            for j in range(64):
                i = 64 * w + j
                for mm in range(rlw[w]):
                    p = woff[w] + 64 * mm + j
                    c = lay.pairs[p, 0]
                    if c >= n_c:
                        assert c < n_c + (16 if block else 1) and vals[p] == 0.0   # padding pair
                        continue
                    # (the library's colouring may place a lane's nonzero on any of the
                    # wave's diagonals; feed order keeps them on the lane's first vlen)
                    assert (block is not None or mm < vlen[i]) and row[i] != 1023 and got[row[i], c] == 0
                    got[row[i], c] = vals[p]
        np.testing.assert_array_equal(got, m.toarray())
    assert covered.all()


def test_stageable_respects_the_lds_budget():
    """The engine only stages groups whose two slab buffers, accumulators and relation
    tables fit one workgroup's LDS (the launcher refuses the rest with DG_EINVAL)."""
    from decagon_amd import engine, kernels
    assert engine.stageable(1928, 645, 645)                   # polypharmacy drug x drug
    assert kernels.staged_lds_bytes(645, 645) <= kernels.STAGED_LDS_BYTES
    assert not engine.stageable(64, 64, 1024)                 # slabs alone overflow
    assert not engine.stageable(64, 1023, 16)                 # rows beyond the 10-bit row id
    assert not engine.stageable(8, 645, 645)                  # too few relations to pay off


# ---------------------------------------------------------------- session state (no GPU needed)
def test_byte_lru_evicts_oldest_by_bytes():
    from decagon_amd.runtime import ByteLRU

    gone = []
    c = ByteLRU(100, on_evict=lambda k, v: gone.append(k))
    c.put("a", 1, 40)
    c.put("b", 2, 40)
    assert c.get("a") == 1          # a is now the most recent
    c.put("c", 3, 40)               # over the cap: b (least recent) goes
    assert gone == ["b"] and "a" in c and "c" in c and c.bytes == 80
    c.put("huge", 4, 500)           # the entry just inserted is never evicted
    assert "huge" in c and len(c) == 1 and gone == ["b", "a", "c"]


def test_feed_keys_follow_the_fed_objects_and_freeze_them():
    from decagon_amd.runtime import _feed_key, _freeze

    coords = np.array([[0, 1], [1, 0]])
    vals = np.array([1.0, 2.0])
    k1, keep = _feed_key((coords, vals, (2, 2)))
    k2, _ = _feed_key([coords, vals, [2, 2]])      # a tuple re-built around the same arrays
    assert k1 == k2
    m = sp.csr_matrix(np.eye(3))
    assert _feed_key(m)[0] == _feed_key(m)[0] != _feed_key(sp.csr_matrix(np.eye(3)))[0]
    _freeze(*keep, m)
    with pytest.raises(ValueError):
        vals[0] = 5.0                               # cached by identity: must not change silently
    with pytest.raises(ValueError):
        m.data[0] = 2.0


def test_global_variables_initializer_redraws_in_place():
    """tf.global_variables_initializer (main.py:286): every variable re-drawn from its
    initializer into the same buffer; with the same seed the draws repeat construction's."""
    import decagon_amd as dg
    from decagon_amd import graph

    et = {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 3}
    dec = {(0, 0): "bilinear", (0, 1): "bilinear", (1, 0): "bilinear", (1, 1): "dedicom"}
    dg.set_random_seed(42)
    model = dg.DecagonModel(dg.construct_placeholders(et), {0: 30, 1: 20}, {0: 30, 1: 20}, et, dec)
    vs = graph.global_variables()
    mine = [v for v in vs if any(v is x for lay in list(model.layers1.values()) + list(model.layers2.values())
                                 + list(model.edge_type2decoder.values()) for x in lay.vars.values())]
    before = {id(v): (v.tensor.data_ptr(), v.eval().copy()) for v in mine}
    reset = []

    class _S:
        def reset_optimizer_slots(self):
            reset.append(1)

    class _Ctx:
        session = _S()

    dg.set_random_seed(7)
    dg.global_variables_initializer()._fn(_Ctx())
    changed = [not np.array_equal(before[id(v)][1], v.eval()) for v in mine]
    assert all(v.tensor.data_ptr() == before[id(v)][0] for v in mine)   # in place
    assert sum(changed) == len(mine) and reset == [1]


def test_global_variables_are_scoped_to_their_graph():
    """TF's GLOBAL_VARIABLES belong to one graph, and the initializer op groups the variables
    that existed when it was created: a model built in another graph (or after the op) is
    not re-drawn."""
    import decagon_amd as dg

    et = {(0, 0): 1, (0, 1): 1, (1, 0): 1, (1, 1): 2}
    dec = {(0, 0): "bilinear", (0, 1): "bilinear", (1, 0): "bilinear", (1, 1): "dedicom"}

    class _S:
        def reset_optimizer_slots(self):
            pass

    class _Ctx:
        session = _S()

    g_a, g_b = dg.Graph(), dg.Graph()
    with g_a.as_default():
        a = dg.DecagonModel(dg.construct_placeholders(et), {0: 12, 1: 8}, {0: 12, 1: 8}, et, dec)
        init_a = dg.global_variables_initializer()
        assert dg.get_default_graph() is g_a
    with g_b.as_default():
        b = dg.DecagonModel(dg.construct_placeholders(et), {0: 12, 1: 8}, {0: 12, 1: 8}, et, dec)
        vb = {k: v.eval().copy() for k, v in b.layers1[0, 0].vars.items()}
        assert all(any(v is x for x in dg.global_variables()) for v in b.layers1[0, 0].vars.values())
        assert not any(v is x for x in dg.global_variables() for v in a.layers1[0, 0].vars.values())
    va = {k: v.eval().copy() for k, v in a.layers1[0, 0].vars.items()}
    init_a._fn(_Ctx())
    assert all(not np.array_equal(va[k], v.eval()) for k, v in a.layers1[0, 0].vars.items())
    assert all(np.array_equal(vb[k], v.eval()) for k, v in b.layers1[0, 0].vars.items())


def test_c_library_reads_no_environment():
    """SURVEY §8b's ABI is arguments-only: no kernel or entry point of the C library consults the
    process environment (round-4 review item 7), in source or in the built library's imports."""
    csrc = Path(__file__).resolve().parent.parent / "decagon_amd" / "csrc"
    hits = [f"{f.name}:{n}" for f in sorted(csrc.iterdir()) if f.suffix in (".hip", ".h", ".cpp")
            for n, line in enumerate(f.read_text().splitlines(), 1) if re.search(r"\b(getenv|secure_getenv|environ)\b", line)]
    assert not hits, hits
    lib = Path(__file__).resolve().parent.parent / "decagon_amd" / "lib" / "libdecagon_hip.so"
    if lib.exists():
        import subprocess

        syms = subprocess.run(["nm", "-D", "--undefined-only", str(lib)], capture_output=True, text=True).stdout
        assert "getenv" not in syms, [l for l in syms.splitlines() if "getenv" in l]


def test_dg_environment_reads_go_through_tuning(monkeypatch):
    """Every DG_* knob of the package is read by decagon_amd.tuning.knob (so bench.py can list
    the non-default ones on its JSON line), none by a direct os.environ read; the C library
    reads none at all (test_c_library_reads_no_environment)."""
    import re

    from decagon_amd import tuning

    pkg = Path(__file__).resolve().parent.parent / "decagon_amd"
    direct = []
    for f in sorted(pkg.glob("*.py")):
        if f.name == "tuning.py":
            continue
        for n, line in enumerate(f.read_text().splitlines(), 1):
            if re.search(r"os\.environ|os\.getenv", line) and "DG_" in line:
                direct.append(f"{f.name}:{n}")
    assert not direct, direct
    monkeypatch.setenv("DG_WINDOWS", "4")
    assert tuning.knob("DG_WINDOWS", 2) == 4 and tuning.overrides().get("DG_WINDOWS") == 4
    monkeypatch.setenv("DG_STAGED", "0")
    assert tuning.knob("DG_STAGED", True) is False
    monkeypatch.delenv("DG_WINDOWS")
    assert tuning.knob("DG_WINDOWS", 2) == 2 and "DG_WINDOWS" not in tuning.overrides()


@pytest.mark.parametrize("raw,want", [("0", False), ("false", False), ("No", False), ("OFF", False),
                                      ("1", True), ("true", True), ("YES", True), ("on", True)])
def test_bool_knobs_parse_strictly(monkeypatch, raw, want):
    """A switch takes 0/false/no/off or 1/true/yes/on (DG_WAVE_TABLE=false used to
    leave the feature on and go unreported); the parsed value is what overrides() reports."""
    from decagon_amd import tuning

    monkeypatch.setenv("DG_WAVE_TABLE", raw)
    assert tuning.knob("DG_WAVE_TABLE", not want) is want
    assert tuning.overrides().get("DG_WAVE_TABLE") is want


def test_bool_knob_rejects_other_values(monkeypatch):
    from decagon_amd import tuning

    for raw in ("2", "enable", ""):
        monkeypatch.setenv("DG_STAGED", raw)
        with pytest.raises(ValueError):
            tuning.knob("DG_STAGED", True)


@pytest.mark.parametrize("proj", [False, True])
def test_balanced_wave_dealing_covers_every_pair_once(proj):
    """PreparedFusedTab(balance=True)'s host dealing (kernels._balanced_waves): every pair of every
    relation lands in exactly one wave, in relation order within a group; a reassociated wave
    (proj) holds one relation only; the waves fit the row's slots and the longest share shrinks."""
    from decagon_amd.kernels import _balanced_waves

    rng = np.random.default_rng(5)
    for trial in range(50):
        n_groups = int(rng.integers(1, 4))
        nr = [int(rng.integers(1, 4)) for _ in range(n_groups)]
        lens = {(g, k): int(rng.choice([0, 3, 7, 40, 81, 130])) for g in range(n_groups) for k in range(nr[g])}

        class TB:
            def seg_len(self, g, k, r):
                return lens[g, k]

        slots = sum(nr) + int(rng.integers(0, 6))
        waves = _balanced_waves(TB(), list(range(n_groups)), nr, 0, slots, proj)
        assert len(waves) == n_groups and sum(len(w) for w in waves) <= slots
        for g in range(n_groups):
            assert waves[g], "at least one wave a group"
            got = [(k, a, e) for w in waves[g] for (k, a, e) in w]
            if proj:
                assert all(len({k for k, _, _ in w}) <= 1 for w in waves[g])
            # the pieces, in wave order, tile each relation's segment from 0 to its end
            for k in range(nr[g]):
                pk = [(a, e) for kk, a, e in got if kk == k]
                pos = 0
                for a, e in pk:
                    assert a == pos and (e > a or lens[g, k] == 0)
                    pos = e
                assert pos == lens[g, k]
            assert [k for k, _, _ in got] == sorted(k for k, _, _ in got)
        longest = max(sum(e - a for _, a, e in w) for wg in waves for w in wg)
        assert longest <= max(lens.values()) if proj else longest <= max(
            sum(lens[g, k] for k in range(nr[g])) for g in range(n_groups))


def test_staged_var_chunks():
    """Variable staged output chunks (engine.staged_var_chunks): a permutation of the relations,
    sub-chunks nested in the top-level chunks, 1..64 relations a chunk, LPT balance."""
    from decagon_amd import engine

    rng = np.random.default_rng(3)
    for n, n_top in ((241, 64), (1928, 64), (60, 64), (5, 64), (128, 2)):
        costs = 1500 + (7500 * rng.zipf(1.6, n).clip(1, 8)).astype(float)
        order, tops, subs = engine.staged_var_chunks(costs, n_top)
        assert sorted(order.tolist()) == list(range(n))
        assert tops[0] == 0 and tops[-1] == n and subs[0] == 0 and subs[-1] == n
        assert set(tops.tolist()) <= set(subs.tolist())
        assert len(tops) - 1 == min(n_top, n)
        for st in (tops, subs):
            assert np.diff(st).min() >= 1 and np.diff(st).max() <= 64
        c = costs[order]
        loads = np.array([c[a:b].sum() for a, b in zip(tops[:-1], tops[1:])])
        assert loads.max() <= max(costs.max(), costs.sum() / len(loads) + costs.max()) + 1e-6

    class G:  # the fields staged_chunk_starts reads
        pass
    g = G()
    order, tops, subs = engine.staged_var_chunks(np.ones(241), 64)
    g.var_chunks = (tops, subs)
    assert engine.staged_chunk_starts(g, 64) is tops           # 4 slices: 64 chunks
    assert engine.staged_chunk_starts(g, 32) is subs           # 2 slices: 128 chunks
    st = engine.staged_chunk_starts(g, 128)                    # 8 slices: runs of two chunks
    assert list(st) == list(tops[::2]) and engine.staged_out_chunk(g, 128) == int(np.diff(st).max())
    g.var_chunks = None
    g.n_rels, g.out_chunk = 241, 2
    assert engine.staged_chunk_starts(g, 64) is None


def test_staged_pieces_partition_rows():
    """engine.staged_pieces: a heavy relation becomes row pieces whose sum is the relation, every
    row in exactly one piece; light relations pass through whole."""
    import scipy.sparse as sp

    from decagon_amd import engine
    from decagon_amd.sparse import HostCSR

    rng = np.random.default_rng(5)
    mats = [sp.random(120, 90, density=dd, random_state=i, format="csr", dtype=np.float32)
            for i, dd in enumerate([0.3, 0.02, 0.05, 0.01])]
    loc = [HostCSR(m.indptr.astype(np.int32), m.indices.astype(np.int32), m.data, m.shape) for m in mats]
    costs = [c.nnz + 100 for c in loc]
    pcs = engine.staged_pieces(loc, costs, 2, 0.5)
    mean = sum(costs) / 2
    for i, c in enumerate(loc):
        mine = [p for j, p in pcs if j == i]
        assert (len(mine) > 1) == (costs[i] > 0.5 * mean)
        tot = sum(sp.csr_matrix((p.val, p.col, p.rowptr), shape=p.shape) for p in mine)
        assert abs(tot - mats[i]).max() == 0
        rows = [set(np.nonzero(np.diff(p.rowptr))[0]) for p in mine]
        assert sum(len(r) for r in rows) == len(set().union(*rows))   # disjoint rows
        assert all(p.nnz <= c.nnz / len(mine) + max(np.diff(c.rowptr)) for p in mine)  # about equal
    assert engine.staged_pieces(loc, costs, 2, 0.0) == [(i, c) for i, c in enumerate(loc)]
    del rng


def test_row_dealt_group_partitions_rows():
    """RelationShard.split(deal_rows=...): every rank holds each relation of a dealt group over
    its own block of output rows (the others emptied, same shape); the blocks add up to the
    relation; polypharmacy deals config P's drug-target relation this way with DG_SHARD_DEAL_ROWS=1."""
    import scipy.sparse as sp

    from decagon_amd import synthetic
    from decagon_amd.sharding import RelationShard, _no_op, _no_op_reduce

    g = synthetic.make_P(seed=3, n_proteins=1500, n_drugs=150, n_side_effects=60, ppi_edges=12000,
                         target_edges=1200)
    nnz = {et: [len(c[1]) for c in rels] for et, rels in g.adj.items()}
    csr = g.csr()
    for world in (2, 3, 8):
        tot = None
        for r in range(world):
            sh = RelationShard.split(g.edge_types, g.n_nodes, nnz, r, world, _no_op_reduce, _no_op,
                                     row_split_min=1000, deal_rows=[(1, 0)])
            assert list(sh.dealt) == [(1, 0)] and sh.local[1, 0] == [0]
            c = sh.local_csr(csr)[1, 0][0]
            assert c.shape == csr[1, 0][0].shape
            a, b = sh.dealt[1, 0]
            m = sp.csr_matrix((c.val, c.col, c.rowptr), shape=c.shape)
            assert m[:a].nnz == 0 and m[b:].nnz == 0
            tot = m if tot is None else tot + m
        ref = csr[1, 0][0]
        assert abs(tot - sp.csr_matrix((ref.val, ref.col, ref.rowptr), shape=ref.shape)).max() == 0
    from decagon_amd import sharding
    gP = synthetic.make_P(seed=0)
    assert not RelationShard.polypharmacy(gP, 0, 8, comm=False).dealt    # default: LPT owner
    sharding.DEAL_ROWS = True
    try:
        shP = RelationShard.polypharmacy(gP, 0, 8, comm=False)
    finally:
        sharding.DEAL_ROWS = False
    assert list(shP.dealt) == [(1, 0)] and all(len(shP.local[et]) for et in [(1, 0), (0, 0), (0, 1)])
