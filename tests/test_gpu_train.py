"""GPU: the training step (opt_op, grads_vars — decagon/deep/optimizer.py:108-114) against
the oracle's float64 gradients (oracle/decagon_oracle.train_grads, itself checked against
torch.autograd on the CPU in test_cpu_train_oracle.py) and TF 1.8's Adam restated in
float32 (oracle.adam_tf); plus the backward kernels one by one.

Tolerance: per gradient tensor max|g − g_ref| ≤ 1e-4·max|g_ref| (fp32 path).
"""
import numpy as np
import pytest

from conftest import rel_err
from oracle import decagon_oracle as orc
from test_gpu_model import _setup

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TOL = 1e-4


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _oracle_inputs(z, model, edge_types):
    w1 = {et: [model.layers1[et].vars["weights_%d" % k].eval().astype(np.float64) for k in range(K)]
          for et, K in edge_types.items()}
    w2 = {et: [model.layers2[et].vars["weights_%d" % k].eval().astype(np.float64) for k in range(K)]
          for et, K in edge_types.items()}
    dec = {et: {n: v.eval().astype(np.float64) for n, v in model.edge_type2decoder[et].vars.items()}
           for et in edge_types}
    adj = {et: [(z[f"adj_{et[0]}_{et[1]}_{k}_coords"], z[f"adj_{et[0]}_{et[1]}_{k}_values"],
                 tuple(int(s) for s in z[f"adj_{et[0]}_{et[1]}_{k}_shape"])) for k in range(K)]
           for et, K in edge_types.items()}
    return w1, w2, dec, adj


def _batch_feed(z, ph, opt, feed, b):
    e, rt, ct = (int(v) for v in z[f"batch{b}_meta"])
    f = dict(feed)
    f.update({ph["batch"]: z[f"batch{b}_edges"], ph["batch_edge_type_idx"]: e, ph["batch_row_edge_type"]: rt,
              ph["batch_col_edge_type"]: ct, opt.neg_samples: z[f"batch{b}_neg"]})
    return f, e, rt, ct


def _sharded_grads_vars_rank(rank, world, b, split):
    """One rank of a sharded Session: `sess.shard` set, grads_vars fetched through the drop-in
    surface (optimizer.py:114's compute_gradients) — every variable's gradient on every rank."""
    from conftest import GOLDEN
    from decagon_amd.sharding import RelationShard, torch_allgather, torch_allreduce

    z = np.load(GOLDEN / "synthetic_S.npz", allow_pickle=False)
    dg, ph, model, opt, feed = _setup(z)
    f, e, rt, ct = _batch_feed(z, ph, opt, feed, b)
    nnz = {et: [len(z[f"adj_{et[0]}_{et[1]}_{k}_values"]) for k in range(K)] for et, K in model.edge_types.items()}
    n = {0: int(z["n_nodes"][0]), 1: int(z["n_nodes"][1])}
    sess = dg.Session()
    if split:  # the genes (500 rows) row-split, the drugs' relations LPT-sharded
        sess.shard = RelationShard.split(model.edge_types, n, nnz, rank, world, torch_allreduce(), torch_allgather(),
                                         row_split_min=450)
    else:
        sess.shard = RelationShard.lpt(model.edge_types, nnz, rank, world, torch_allreduce())
    gv = sess.run(opt.grads_vars, feed_dict=f)
    owned = {et: list(v) for et, v in sess.shard.local.items()}
    return [(np.asarray(g), np.asarray(v)) for g, v in gv], owned, sorted(sess.shard.row_block)


@pytest.mark.parametrize("b,split", [(0, False), (3, False), (1, True)])
def test_sharded_grads_vars_match_oracle(golden_S, b, split):
    """grads_vars on 2 gloo ranks sharing the GPU (relations LPT-sharded; or the genes
    row-split): every rank returns EVERY variable's gradient — each relation's gathered from
    its owner rank (TrainPlan.full_grads) — equal to the float64 oracle's TF gradients within
    1e-4, and the ranks' lists are identical bit for bit."""
    from conftest import run_ranks

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    z = golden_S
    got = run_ranks(_sharded_grads_vars_rank, 2, (b, split))
    dg, ph, model, opt, feed = _setup(z)
    e, rt, ct = (int(v) for v in z[f"batch{b}_meta"])
    w1, w2, dec, adj = _oracle_inputs(z, model, model.edge_types)
    cost, ref = orc.train_grads(model.edge_types, adj, {0: None, 1: None}, w1, w2, model.decoders, dec, 32,
                                z[f"batch{b}_edges"], z[f"batch{b}_neg"], e, rt, ct, 0.1)
    want = []
    for et, K in model.edge_types.items():
        want += [ref["w1"][et][k] for k in range(K)]
    for et, K in model.edge_types.items():
        want += [ref["w2"][et][k] for k in range(K)]
    for et in model.edge_types:
        want += [ref["dec"][et][n] for n in model.edge_type2decoder[et].vars]
    (gv0, owned0, rb0), (gv1, owned1, rb1) = got[0], got[1]
    assert rb0 == ([0] if split else [])
    if not split:  # the relations really are split between the ranks
        assert all(sorted(owned0[et] + owned1[et]) == list(range(K)) for et, K in model.edge_types.items())
        assert any(len(owned0[et]) < K for et, K in model.edge_types.items())
    assert len(gv0) == len(gv1) == len(want)
    nonzero = 0
    for (g0, v0), (g1, v1), w in zip(gv0, gv1, want):
        assert np.array_equal(g0, g1) and np.array_equal(v0, v1)
        scale = np.max(np.abs(w))
        if scale == 0:
            assert np.max(np.abs(g0)) == 0.0
        else:
            nonzero += 1
            assert np.max(np.abs(g0 - w)) <= TOL * scale, f"gradient off by {rel_err(g0, w):.2e}"
    assert nonzero > 0


@pytest.mark.parametrize("b", [0, 1, 2, 3])
def test_grads_vars_match_oracle(golden_S, b):
    """Every variable's gradient (all four decoder kinds of config S appear across batches)."""
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    edge_types = model.edge_types
    decoders = model.decoders
    f, e, rt, ct = _batch_feed(z, ph, opt, feed, b)
    sess = dg.Session()
    gv = sess.run(opt.grads_vars, feed_dict=f)
    w1, w2, dec, adj = _oracle_inputs(z, model, edge_types)
    cost, ref = orc.train_grads(edge_types, adj, {0: None, 1: None}, w1, w2, decoders, dec, 32,
                                z[f"batch{b}_edges"], z[f"batch{b}_neg"], e, rt, ct, 0.1)
    want = []
    for et, K in edge_types.items():
        want += [ref["w1"][et][k] for k in range(K)]
    for et, K in edge_types.items():
        want += [ref["w2"][et][k] for k in range(K)]
    for et in edge_types:
        want += [ref["dec"][et][n] for n in model.edge_type2decoder[et].vars]
    assert len(gv) == len(want)
    nonzero = 0
    for (g, v), w in zip(gv, want):
        assert g.shape == w.shape
        scale = np.max(np.abs(w))
        if scale == 0:
            assert np.max(np.abs(g)) == 0.0  # unreachable variables: exact zeros, as TF's
        else:
            nonzero += 1
            assert np.max(np.abs(g - w)) <= TOL * scale, f"gradient off by {rel_err(g, w):.2e}"
    assert nonzero > 0


def test_opt_op_is_one_tf_adam_step(golden_S):
    """opt_op = forward + backward + ApplyAdam: params after two steps equal adam_tf applied to
    the device's own gradients (fetched by grads_vars on the same state), and the cost
    fetched with opt_op is the pre-update cost."""
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    f, e, rt, ct = _batch_feed(z, ph, opt, feed, 3)
    sess = dg.Session()
    params = [v for v in model.vars.values()]
    m = [np.zeros(p.shape, np.float32) for p in params]
    v = [np.zeros(p.shape, np.float32) for p in params]
    for t in (1, 2):
        gv = sess.run(opt.grads_vars, feed_dict=f)
        before = [p.eval() for p in params]
        _, cost = sess.run([opt.opt_op, opt.cost], feed_dict=f)
        after = [p.eval() for p in params]
        for i, ((g, _), p0, p1) in enumerate(zip(gv, before, after)):
            pw, m[i], v[i] = orc.adam_tf(p0, g, m[i], v[i], t)
            assert np.max(np.abs(p1 - pw)) <= 1e-6 * max(1.0, np.max(np.abs(pw))), params[i].name
        if t == 1:
            assert abs(float(cost) - float(z["batch3_cost"])) <= TOL * abs(float(z["batch3_cost"]))
    # training moves the cost down on the batch it fits
    c_end = sess.run(opt.cost, feed_dict=f)
    assert float(c_end) < float(z["batch3_cost"])


def test_initializer_in_a_second_session_redraws_and_restarts_adam(golden_S):
    """A second Session running global_variables_initializer (GreedyActiveLearner.py:18,
    main.py:286): every variable re-drawn (not the trained values), and the next opt_op is
    TF-Adam step t = 1 (fresh m / v / beta powers) on the device's own gradients."""
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    f, e, rt, ct = _batch_feed(z, ph, opt, feed, 3)
    sess = dg.Session()
    for _ in range(3):
        sess.run(opt.opt_op, feed_dict=f)
    params = [v for v in model.vars.values()]
    trained = [p.eval() for p in params]
    sess2 = dg.Session()
    sess2.run(dg.global_variables_initializer())
    fresh = [p.eval() for p in params]
    assert all(not np.array_equal(a, b) for a, b in zip(trained, fresh) if a.size > 1)
    for q in (sess, sess2):  # the same in the first session: its Adam restarts as well
        if q is sess:
            sess.run(dg.global_variables_initializer())
        gv = q.run(opt.grads_vars, feed_dict=f)
        before = [p.eval() for p in params]
        q.run(opt.opt_op, feed_dict=f)
        for (g, _), p0, prm in zip(gv, before, params):
            pw, _, _ = orc.adam_tf(p0, g, np.zeros_like(p0), np.zeros_like(p0), 1)
            assert np.max(np.abs(prm.eval() - pw)) <= 1e-6 * max(1.0, np.max(np.abs(pw))), prm.name


def test_feed_cache_is_bounded_and_fed_arrays_read_only(golden_S, monkeypatch):
    """Re-masked graphs fed every run (new arrays each time) stay within the device cache
    cap (LRU by bytes; plans built on an evicted graph go with it), and a cached fed array
    refuses in-place changes."""
    from decagon_amd import runtime

    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    monkeypatch.setattr(runtime, "DEVICE_CACHE_BYTES", 3 << 20)  # ~2 graphs of config S
    sess = dg.Session()
    key = ph["adj_mats_1,1,0"]
    c, v, s = feed[key]
    for it in range(6):
        f = dict(feed)
        f[key] = (c.copy(), v.copy() * (1.0 + 0.01 * it), s)   # a new graph each run
        sess.run(model.embeddings[1], feed_dict=f)
        assert len(sess.caches["dgraph"]) <= 3 and sess.caches["dgraph"].bytes <= (3 << 20) + (2 << 20)
        assert len(sess.caches["plans"]) <= len(sess.caches["dgraph"])
    with pytest.raises(ValueError):
        f[key][1][0] = 0.5


def test_adam_kernel_matches_tf_restatement():
    from decagon_amd import kernels, train

    dev = _dev()
    rng = np.random.default_rng(1)
    sizes = [1, 3, 4, 4097, 5000]
    p = [rng.standard_normal(n).astype(np.float32) for n in sizes]
    g = [rng.standard_normal(n).astype(np.float32) for n in sizes]
    dp = [torch.from_numpy(x.copy()).to(dev) for x in p]
    dgr = [torch.from_numpy(x).to(dev) for x in g]
    st = train.AdamState(dp, lr=0.01)
    grads = [dgr[0], None, dgr[2], dgr[3], dgr[4]]  # None: a zero gradient
    op = st.prepared(grads)
    m = [np.zeros(n, np.float32) for n in sizes]
    v = [np.zeros(n, np.float32) for n in sizes]
    for t in (1, 2, 3):
        if t == 2:  # the host-alpha form of the same step
            op(train.adam_alpha(0.01, t), train.BETA1, train.BETA2, train.EPSILON)
            kernels.adam_advance(st.state, 0.01, train.BETA1, train.BETA2)
        else:  # device beta powers (graph-capturable)
            st.apply(op)
        for i in range(len(sizes)):
            gi = g[i] if grads[i] is not None else np.zeros_like(g[i])
            p[i], m[i], v[i] = orc.adam_tf(p[i], gi, m[i], v[i], t, lr=0.01)
    torch.cuda.synchronize()
    for i in range(len(sizes)):
        assert np.max(np.abs(dp[i].cpu().numpy() - p[i])) <= 1e-6
        assert np.max(np.abs(st.m[i].cpu().numpy() - m[i])) <= 1e-6
    assert abs(float(st.state[2]) - train.adam_alpha(0.01, 4)) <= 1e-7


@pytest.mark.parametrize("kind", ["dedicom", "distmult", "bilinear", "innerproduct"])
def test_decoder_grad_kernel(kind):
    from decagon_amd import kernels

    dev = _dev()
    rng = np.random.default_rng(2)
    d, n, nr, nc = 32, 300, 50, 40
    U = rng.standard_normal((nr, d)).astype(np.float32)
    V = rng.standard_normal((nc, d)).astype(np.float32)
    rows, cols, negs = rng.integers(0, nr, n), rng.integers(0, nc, n), rng.integers(0, nr, n)
    G = rng.standard_normal((d, d)).astype(np.float32) if kind in ("dedicom", "bilinear") else \
        (np.diag(rng.standard_normal(d)).astype(np.float32) if kind == "distmult" else np.eye(d, dtype=np.float32))
    l = rng.standard_normal(d).astype(np.float32) if kind == "dedicom" else None
    L = np.diag(l) if l is not None else np.eye(d)
    M = L @ G.astype(np.float64) @ L
    pos = np.sum((U[rows] @ M) * V[cols], 1)
    neg = np.sum((U[negs] @ M) * V[cols], 1)
    a = ((neg - (pos - 0.1)) > 0).astype(np.float64)
    T = lambda x, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(x)).to(dev, dt)  # noqa: E731
    dG = torch.zeros(d * d, device=dev) if kind in ("dedicom", "bilinear") else None
    dl = torch.zeros(d, device=dev) if kind == "dedicom" else None
    dgd = torch.zeros(d, device=dev) if kind == "distmult" else None
    op = kernels.PreparedDecoderGrad(T(U), T(V), T(rows, torch.int32), T(cols, torch.int32), T(negs, torch.int32),
                                     T(pos), T(neg), T(G), T(l) if l is not None else None, 0.1,
                                     dG=dG, dl=dl, dG_diag=dgd)
    op()
    torch.cuda.synchronize()
    gr = op.grad_rows.cpu().numpy()
    gc = op.grad_cols.cpu().numpy()
    mv = V[cols] @ M.T
    assert rel_err(gr[:n], -a[:, None] * mv) <= 1e-5
    assert rel_err(gr[n:], a[:, None] * mv) <= 1e-5
    assert rel_err(gc, a[:, None] * ((U[negs] - U[rows]) @ M)) <= 1e-5
    dM = (a[:, None] * (U[negs] - U[rows])).T @ V[cols]
    if dG is not None:
        assert rel_err(dG.cpu().numpy().reshape(d, d), L.T @ dM @ L.T) <= 1e-5
    if dl is not None:
        ref = np.diag(dM @ (G @ L).T + (L @ G).T @ dM)
        assert rel_err(dl.cpu().numpy(), ref) <= 1e-5
    if dgd is not None:
        assert rel_err(dgd.cpu().numpy(), np.diag(dM)) <= 1e-5


def test_scatter_rows_and_l2norm_grad():
    from decagon_amd import kernels

    dev = _dev()
    rng = np.random.default_rng(3)
    n, d, nrow = 700, 32, 90
    idx = rng.integers(0, nrow, n).astype(np.int32)
    src = rng.standard_normal((n, d)).astype(np.float32)
    out0 = rng.standard_normal((nrow, d)).astype(np.float32)
    out = torch.from_numpy(out0.copy()).to(dev)
    kernels.scatter_rows(torch.from_numpy(idx).to(dev), torch.from_numpy(src).to(dev), out)
    ref = out0.astype(np.float64)
    np.add.at(ref, idx, src)
    assert rel_err(out.cpu().numpy(), ref) <= 1e-6
    # l2 normalisation backward, with a relu mask and all-zero rows
    for dd in (32, 64, 12):
        S = rng.standard_normal((nrow, dd)).astype(np.float32)
        S[::7] = 0.0
        dy = rng.standard_normal((nrow, dd)).astype(np.float32)
        mask = rng.standard_normal((nrow, dd)).astype(np.float32)
        T = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
        ds = torch.empty((nrow, dd), device=dev)
        kernels.PreparedL2Grad([(T(S), ds)], T(dy), T(mask), nrow, dd)()
        torch.cuda.synchronize()
        want = orc.l2_normalize_rows_grad(S.astype(np.float64), dy * (mask > 0))
        assert rel_err(ds.cpu().numpy(), want) <= 1e-5


def test_gemm_batch_reduce():
    """dg_gemm_f32's batch-reduce mode: Σ over runs of R batches, run partials in order."""
    from decagon_amd import kernels

    dev = _dev()
    rng = np.random.default_rng(4)
    K, n_j, c, h = 70, 45, 32, 64
    dP = rng.standard_normal((K, n_j, c)).astype(np.float32)
    W = rng.standard_normal((K, h, c)).astype(np.float32)
    R = 32
    runs = -(-K // R)
    out = torch.zeros((runs, n_j, h), device=dev)
    kernels.PreparedGemm(torch.from_numpy(dP).to(dev), (n_j * c, c, 1), torch.from_numpy(W).to(dev), (h * c, 1, c),
                         out, (n_j * h, h, 1), n_j, h, c, K, reduce=R)()
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for q in range(runs):
        ref = sum(dP[b].astype(np.float64) @ W[b].T.astype(np.float64) for b in range(q * R, min(K, q * R + R)))
        assert rel_err(got[q], ref) <= 1e-5


@pytest.mark.parametrize("rows,split", [(645, 1024), (3001, 700), (1, 64)])
def test_gemm_tn_split(rows, split):
    """dg_gemm_tn_f32: c[b] = aᵀ·b[b] over a long row reduction, with split partials."""
    from decagon_amd import kernels

    dev = _dev()
    rng = np.random.default_rng(5)
    M, N, batch = 64, 32, 7
    A = rng.standard_normal((rows, M)).astype(np.float32)
    B = rng.standard_normal((batch, rows, N)).astype(np.float32)
    C = torch.empty((batch, M, N), device=dev)
    kernels.PreparedGemmTN(torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev), C, rows_per_split=split)()
    torch.cuda.synchronize()
    ref = np.einsum("rm,brn->bmn", A.astype(np.float64), B.astype(np.float64))
    assert rel_err(C.cpu().numpy(), ref) <= 1e-5


@pytest.mark.parametrize("d", [64, 32, 12])
def test_spmm_lds_shared_operand(d):
    """dg_spmm_groups_lds_f32 = dg_spmm_groups_f32 (partial mode) for a small shared operand:
    out[k] = Âᵀ_k·X with empty rows and a long row."""
    from decagon_amd import kernels
    from decagon_amd.sparse import coo_to_csr, merge_chunks
    from decagon_amd.train import transpose_csr

    dev = _dev()
    rng = np.random.default_rng(6)
    n_i, n_j, K = 300, 200, 5
    rels = []
    for k in range(K):
        nnz = 900
        r, c = rng.integers(0, n_i, nnz), rng.integers(0, n_j, nnz)
        c[:60] = 3  # a long column → a long row of Âᵀ
        c[c == 7] = 8  # an empty row of Âᵀ
        keys = np.unique(r * n_j + c)
        co = np.stack([keys // n_j, keys % n_j], 1)
        rels.append(coo_to_csr(co, rng.standard_normal(len(keys)), (n_i, n_j)))
    tr = [transpose_csr(x) for x in rels]
    m = merge_chunks(tr, [0] * K, 1, 1)
    X = rng.standard_normal((n_i, d)).astype(np.float32)
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    outs = []
    for lds in (True, False):
        out = torch.zeros((K, n_j, d), device=dev)
        spec = kernels.RelGroupSpec(T(m.rowptr), T(m.vcol), T(m.val), T(X), out, n_j, K, d, n_i,
                                    vcol_max=int(m.vcol.max()))
        kernels.PreparedSpmm([spec], d, lds=lds)()
        outs.append(out)
    torch.cuda.synchronize()
    for k, rel in enumerate(rels):
        dense = np.zeros((n_i, n_j))
        lens = np.diff(rel.rowptr)
        dense[np.repeat(np.arange(n_i), lens), rel.col] = rel.val
        ref = dense.T @ X.astype(np.float64)
        assert rel_err(outs[0][k].cpu().numpy(), ref) <= 1e-5
    assert rel_err(outs[0].cpu().numpy(), outs[1].cpu().numpy()) <= 1e-6


def _lds_case(rng, K, n_rows, n_x, per_row=2, long_row=True):
    """K relations' transposed CSR (n_rows × n_x) merged one chunk per relation over a
    shared operand of n_x rows (the Âᵀ·dS form), with an empty row and a long row."""
    from decagon_amd.sparse import coo_to_csr, merge_chunks

    rels = []
    for k in range(K):
        nnz = per_row * n_rows
        r, c = rng.integers(0, n_rows, nnz), rng.integers(0, n_x, nnz)
        r[r == 5] = 6  # an empty row
        if long_row:
            r[:300] = 11  # a long row (> 4 batches of 64 for its lanes)
        keys = np.unique(r.astype(np.int64) * n_x + c)
        co = np.stack([keys // n_x, keys % n_x], 1)
        rels.append(coo_to_csr(co, rng.standard_normal(len(keys)), (n_rows, n_x)))
    return rels, merge_chunks(rels, [0] * K, 1, 1)


@pytest.mark.parametrize("cases,d", [
    ([(64, 30000)], 32),                 # ≈1.9 M items: 64 items per wave
    ([(64, 60000)], 36),                 # ≈3.8 M items: 128 per wave (rp2 at 128), partial d slice
    ([(4, 500), (64, 30000)], 64),       # two groups in one launch: block_begin dispatch, persist > 1
])
def test_spmm_lds_per_wave_and_groups(cases, d):
    """dg_spmm_groups_lds_f32 at the items-per-wave settings config P's training hits (64 /
    128, the 64-item boundary), several groups per launch and a partial column slice (d = 36)
    — against float64 Âᵀ·X per relation and the gather kernel (dg_spmm_groups_f32)."""
    import scipy.sparse as sps

    from decagon_amd import kernels

    dev = _dev()
    rng = np.random.default_rng(sum(k * n for k, n in cases) + d)
    n_x = 1000
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    groups = []
    for K, n_rows in cases:
        rels, m = _lds_case(rng, K, n_rows, n_x)
        X = rng.standard_normal((n_x, d)).astype(np.float32)
        groups.append((rels, m, X, K, n_rows))
    outs = {}
    for lds in (True, False):
        specs, bufs = [], []
        for rels, m, X, K, n_rows in groups:
            out = torch.full((K, n_rows, d), float("nan"), device=dev)
            specs.append(kernels.RelGroupSpec(T(m.rowptr), T(m.vcol), T(m.val), T(X), out, n_rows, K, d, n_x,
                                              vcol_max=int(m.vcol.max())))
            bufs.append(out)
        kernels.PreparedSpmm(specs, d, lds=lds)()
        torch.cuda.synchronize()
        outs[lds] = [b.cpu().numpy() for b in bufs]
    for gi, (rels, m, X, K, n_rows) in enumerate(groups):
        got = outs[True][gi]
        assert np.array_equal(got, outs[False][gi]) or rel_err(got, outs[False][gi]) <= 1e-6
        for k in (0, K // 2, K - 1):
            rel = rels[k]
            a = sps.csr_matrix((rel.val.astype(np.float64), rel.col, rel.rowptr), shape=rel.shape)
            assert rel_err(got[k], a @ X.astype(np.float64)) <= 1e-5, (gi, k)
        assert not np.isnan(got).any()


def test_dropout_masks_match_restatement():
    """dg_dropout_rows_f32 / dg_dropout_elems_f32 draw exactly oracle.dropout_scale's masks."""
    from decagon_amd import kernels

    dev = _dev()
    state = torch.tensor([123456789012, 5], dtype=torch.int64, device=dev)
    rows = torch.ones((3000, 8), device=dev)
    out = torch.empty_like(rows)
    kernels.dropout_rows(rows, out, state, 77, 0.8)
    src = torch.ones((50, 64), device=dev)
    el = torch.empty((7, 50, 64), device=dev)
    kernels.dropout_elems(src, el, state, 78, 0.8)
    torch.cuda.synchronize()
    want_r = orc.dropout_scale(123456789012, 5, 77, 3000, 0.8)
    want_e = orc.dropout_scale(123456789012, 5, 78, 7 * 50 * 64, 0.8)
    assert np.array_equal(out.cpu().numpy(), np.repeat(want_r[:, None], 8, 1))
    assert np.array_equal(el.cpu().numpy().reshape(-1), want_e)
    kernels.dropout_advance(state)
    torch.cuda.synchronize()
    assert int(state[1]) == 6


def test_gemm_batch_reduce_with_dropout_mask():
    from decagon_amd import kernels

    dev = _dev()
    rng = np.random.default_rng(8)
    K, n_j, c, h = 40, 37, 32, 64
    dP = rng.standard_normal((K, n_j, c)).astype(np.float32)
    W = rng.standard_normal((K, h, c)).astype(np.float32)
    state = torch.tensor([99, 3], dtype=torch.int64, device=dev)
    R = 16
    runs = -(-K // R)
    out = torch.zeros((runs, n_j, h), device=dev)
    kernels.PreparedGemm(torch.from_numpy(dP).to(dev), (n_j * c, c, 1), torch.from_numpy(W).to(dev), (h * c, 1, c),
                         out, (n_j * h, h, 1), n_j, h, c, K, reduce=R, drop=(state, 5, 0.7))()
    torch.cuda.synchronize()
    m = orc.dropout_scale(99, 3, 5, K * n_j * h, 0.7).reshape(K, n_j, h).astype(np.float64)
    got = out.cpu().numpy()
    for q in range(runs):
        ref = sum(m[b] * (dP[b].astype(np.float64) @ W[b].T.astype(np.float64)) for b in range(q * R, min(K, q * R + R)))
        assert rel_err(got[q], ref) <= 1e-5


def test_mapped_dropout_masks_and_reduce_gemm():
    """A relation shard's masks (dg_dropout_rows_map_f32 / dg_dropout_elems_map_f32 and the
    batch-mapped batch-reduce GEMM): local slab b carries global relation map[b]'s bits, the
    bits the unmapped kernels (and oracle.dropout_scale) draw for it."""
    from decagon_amd import kernels

    dev = _dev()
    state = torch.tensor([4242, 2], dtype=torch.int64, device=dev)
    K, F, d = 9, 37, 8
    ids = np.array([1, 4, 5, 8], np.int32)
    m = torch.from_numpy(ids).to(dev)
    W = torch.from_numpy(np.random.default_rng(3).standard_normal((K, F, d)).astype(np.float32)).to(dev)
    full = torch.empty_like(W)
    kernels.dropout_rows(W, full, state, 31, 0.7)
    glob = torch.zeros_like(W)
    kernels.dropout_rows_map(W, glob, m, F, state, 31, 0.7, True, True)
    loc = W[m.long()].clone()
    kernels.dropout_rows_map(loc, loc, m, F, state, 31, 0.7, False, False)
    src = torch.from_numpy(np.random.default_rng(4).standard_normal((F, 64)).astype(np.float32)).to(dev)
    el_full = torch.empty((K, F, 64), device=dev)
    kernels.dropout_elems(src, el_full, state, 32, 0.7)
    el_loc = torch.empty((len(ids), F, 64), device=dev)
    kernels.dropout_elems_map(src, el_loc, m, state, 32, 0.7)
    # batch-reduce GEMM over the local relations, W2 read at their global slabs, masks mapped
    rng = np.random.default_rng(5)
    dP = torch.from_numpy(rng.standard_normal((len(ids), F, 32)).astype(np.float32)).to(dev)
    W2 = torch.from_numpy(rng.standard_normal((K, 64, 32)).astype(np.float32)).to(dev)
    out = torch.zeros((1, F, 64), device=dev)
    kernels.PreparedGemm(dP, (F * 32, 32, 1), W2, (64 * 32, 1, 32), out, (F * 64, 64, 1), F, 64, 32, len(ids),
                         reduce=len(ids), drop=(state, 32, 0.7), b_map=m, b_batches=K, b_map_max=8)()
    torch.cuda.synchronize()
    assert np.array_equal(glob.cpu().numpy()[ids], full.cpu().numpy()[ids])
    assert np.array_equal(loc.cpu().numpy(), full.cpu().numpy()[ids])
    assert np.array_equal(el_loc.cpu().numpy(), el_full.cpu().numpy()[ids])
    mk = orc.dropout_scale(4242, 2, 32, K * F * 64, 0.7).reshape(K, F, 64).astype(np.float64)
    want = sum(mk[k] * (dP[b].cpu().numpy().astype(np.float64) @ W2[k].cpu().numpy().T.astype(np.float64))
               for b, k in enumerate(ids))
    assert rel_err(out.cpu().numpy()[0], want) <= 1e-5


def test_grads_vars_with_dropout_match_oracle(golden_S):
    """The training step at FLAGS.dropout = 0.1 (main.py:235, :307): every gradient against the
    oracle on the same masks (the device's draw for step 1, regenerated by the oracle)."""
    from test_cpu_train_oracle import _masks

    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    edge_types, decoders = model.edge_types, model.decoders
    f, e, rt, ct = _batch_feed(z, ph, opt, feed, 3)
    f[ph["dropout"]] = 0.1
    sess = dg.Session()
    gv = sess.run(opt.grads_vars, feed_dict=f)
    w1, w2, dec, adj = _oracle_inputs(z, model, edge_types)
    drop1, drop2 = _masks(edge_types, adj, 0.9, step=1)
    cost, ref = orc.train_grads(edge_types, adj, {0: None, 1: None}, w1, w2, decoders, dec, 32,
                                z["batch3_edges"], z["batch3_neg"], e, rt, ct, 0.1, drop1=drop1, drop2=drop2)
    want = []
    for et, K in edge_types.items():
        want += [ref["w1"][et][k] for k in range(K)]
    for et, K in edge_types.items():
        want += [ref["w2"][et][k] for k in range(K)]
    for et in edge_types:
        want += [ref["dec"][et][n] for n in model.edge_type2decoder[et].vars]
    for (g, v), w in zip(gv, want):
        scale = np.max(np.abs(w))
        if scale == 0:
            assert np.max(np.abs(g)) == 0.0
        else:
            assert np.max(np.abs(g - w)) <= TOL * scale, f"gradient off by {rel_err(g, w):.2e}"
    # the cost with dropout differs from the dropout-free one, and a second run draws new masks
    c1 = sess.run(opt.cost, feed_dict=f)
    assert abs(float(c1) - cost) > 1e-6 * abs(cost)
    st = model.dropout_state(type("C", (), {"session": sess})())
    assert int(st[1]) == 2
    # opt_op with dropout trains (the reference's main.py loop)
    for _ in range(5):
        sess.run([opt.opt_op, opt.cost], feed_dict=f)
    f0 = dict(f)
    f0[ph["dropout"]] = 0.0
    assert float(sess.run(opt.cost, feed_dict=f0)) < float(z["batch3_cost"])


@pytest.mark.parametrize("P,N,k,ties", [(1000, 1000, 50, True), (700, 1500, 50, False), (10, 3, 50, True),
                                        (60, 40, 50, True)])
def test_rank_metrics_match_sklearn(P, N, k, ties):
    """dg_rank_metrics_f32 = roc_auc_score / average_precision_score / rank_metrics.apk."""
    from decagon_amd.evaluate import rank_metrics

    dev = _dev()
    rng = np.random.default_rng(P + N)
    if ties:
        pos = rng.integers(0, 20, P).astype(np.float32) + 2.0
        neg = rng.integers(0, 20, N).astype(np.float32)
    else:
        pos = (rng.standard_normal(P) + 0.7).astype(np.float32)
        neg = rng.standard_normal(N).astype(np.float32)
    got = rank_metrics(torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), k)
    want = orc.accuracy_scores(pos, neg, k)
    for g, w in zip(got, want):
        assert abs(g - w) <= 1e-12, (got, want)


@pytest.mark.parametrize("mode", ["main", "evaluator", None])
def test_rank_metrics_saturating_logits(mode):
    """Logits spanning [-120, 120]: the reference ranks sigmoid scores that saturate (main.py
    under numpy 1.14: float32 exp, float64 1/(1+e) — ties at exactly 1.0 above ≈36.7 and 0.0
    below ≈-88.7; DecagonAccuracyEvaluator: all float32, ties above ≈16.6).  The device ranks
    the same scores: AUROC / AUPRC / AP@50 equal the restated sklearn / rank_metrics values
    within 1e-12, and (main, evaluator) differ from the logit ranking — the ties matter."""
    from decagon_amd.evaluate import rank_metrics

    dev = _dev()
    rng = np.random.default_rng(120)
    pos = rng.uniform(-60, 100, 1500).astype(np.float32)
    neg = rng.uniform(-120, 110, 1300).astype(np.float32)
    if mode == "main":
        neg[:7] = np.nan  # nan_to_num (main.py:81) scores a NaN logit 0.0
    got = rank_metrics(torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), 50, sigmoid=mode)
    want = orc.accuracy_scores(pos, neg, 50, sigmoid=mode)
    for g, w in zip(got, want):
        assert abs(g - w) <= 1e-12, (mode, got, want)
    if mode is not None:
        raw = orc.accuracy_scores(pos, np.nan_to_num(neg, nan=-200.0), 50, sigmoid=None)
        assert abs(raw[0] - want[0]) > 1e-4 and abs(raw[2] - want[2]) > 1e-3, (raw, want)


def test_accuracy_scores_through_the_model(golden_S):
    """evaluate.accuracy_scores (main.py:38-80 on the device) against sklearn on the oracle's
    predictions of the same sampled edges."""
    from decagon_amd import evaluate

    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    edge_types = model.edge_types
    sess = dg.Session()
    rng = np.random.default_rng(11)
    et = (1, 1, 2)
    pos = z["adj_1_1_2_coords"][rng.choice(len(z["adj_1_1_2_coords"]), 300, replace=False)]
    neg = rng.integers(0, 400, (300, 2))
    edges_pos = {(1, 1): {2: pos}}
    edges_neg = {(1, 1): {2: neg}}
    flat = {}
    for i, j in edge_types:
        for k in range(edge_types[i, j]):
            flat[i, j, k] = len(flat)
    got = evaluate.accuracy_scores(sess, opt, ph, feed, edges_pos, edges_neg, et, flat, k=50)
    emb = [z["emb_0"], z["emb_1"]]
    R = z["dec_1_1_global_interaction"].astype(np.float64)
    D = np.diag(z["dec_1_1_local_variation_2"].astype(np.float64))
    pred = orc.predict(emb, 1, 1, R, D)
    want = orc.accuracy_scores(pred[pos[:, 0], pos[:, 1]], pred[neg[:, 0], neg[:, 1]], 50)
    for g, w in zip(got, want):
        assert abs(g - w) <= 1e-3, (got, want)  # fp32 scores vs float64: near-ties may swap
