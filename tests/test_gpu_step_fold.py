"""The decoder step inside the fused layer's launch (dg_gcn_fused_hinge_f32, config S's layer 2
+ DEDICOM scores + hinge loss, optimizer.py:37-57 and :116-120 on the embeddings of
model.py:85-88): the same buffers and results as the two launches it replaces — embeddings,
sampled negatives and both score vectors bit for bit, the loss within float rounding (another
fixed summation order) — across repeated launches (the in-launch counters re-arm themselves),
inside a hipGraph replayed back to back, and against the float64 oracle.
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _plan_S():
    from decagon_amd import synthetic
    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = synthetic.load_S()
    rng = np.random.default_rng(1234)

    def glorot(k, a, b):
        r = np.sqrt(6.0 / (a + b))
        return torch.from_numpy(rng.uniform(-r, r, size=(k, a, b)).astype(np.float32)).cuda()

    dgr = DeviceGraph(g.edge_types, g.csr(), torch.device("cuda"), None)
    w1 = LayerWeights({et: glorot(K, g.n_nodes[et[1]], 64) for et, K in g.edge_types.items()})
    w2 = LayerWeights({et: glorot(K, 64, 32) for et, K in g.edge_types.items()})
    plan = ForwardPlan(dgr, {j: None for j in g.n_nodes}, w1, w2, 64, 32)
    return g, plan, rng


def _hinge(K, g, rng, row_t, col_t, d, n, given=False, row_node=1):
    rows = torch.from_numpy(rng.integers(0, row_t.shape[0], n).astype(np.int32)).cuda()
    cols = torch.from_numpy(rng.integers(0, col_t.shape[0], n).astype(np.int32)).cuda()
    G = torch.from_numpy((rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)).cuda()
    l = torch.from_numpy(rng.standard_normal(d).astype(np.float32)).cuda()
    if given:
        negs = torch.from_numpy(rng.integers(0, row_t.shape[0], n).astype(np.int32)).cuda()
        return K.PreparedDecoderHinge(row_t, col_t, rows, cols, G, l, 0.1, neg_rows=negs)
    alias = K.upload_alias(g.degrees[row_node][0], "cuda")
    return K.PreparedDecoderHinge(row_t, col_t, rows, cols, G, l, 0.1, alias=alias, seed=7, offset=5)


def _snap(tensors, op):
    torch.cuda.synchronize()
    return [t.detach().clone().cpu().numpy() for t in tensors] + [
        op.pos.cpu().numpy().copy(), op.neg.cpu().numpy().copy(), op.neg_rows.cpu().numpy().copy(),
        float(op.loss[0])]


def _check_oracle(op, row_t, col_t):
    import oracle.decagon_oracle as orc

    U = row_t.cpu().numpy().astype(np.float64)
    V = col_t.cpu().numpy().astype(np.float64)
    G = op._keep[4].cpu().numpy().astype(np.float64)
    L = np.diag(op._keep[5].cpu().numpy().astype(np.float64))
    rows = op._keep[2].cpu().numpy()
    cols = op._keep[3].cpu().numpy()
    negs = op.neg_rows.cpu().numpy()
    pos = orc.batch_predict([U, V], 0, 1, G, L, rows, cols)
    neg = orc.batch_predict([U, V], 0, 1, G, L, negs, cols)
    assert rel_err(op.pos.cpu().numpy(), pos) <= 1e-5
    assert rel_err(op.neg.cpu().numpy(), neg) <= 1e-5
    want = orc.hinge_loss(pos, neg, 0.1)
    assert abs(float(op.loss[0]) - want) <= 1e-4 * max(1.0, abs(want))


@pytest.mark.parametrize("given", [False, True])
@pytest.mark.parametrize("n", [512, 100, 1300])
def test_layer2_with_decoder_in_one_launch(n, given):
    """Config S's layer 2 + the decoder step: folded == unfolded, then vs the oracle."""
    from decagon_amd import kernels as K

    g, plan, rng = _plan_S()
    E = plan.embeddings
    op = _hinge(K, g, rng, E[1], E[0], 32, n, given)
    plan.run()
    op()
    ref = _snap([E[0], E[1]], op)
    assert plan.fold_hinge(op)
    folded = plan.folded_hinge
    for _ in range(3):  # the counters re-arm: every launch waits for its own layer
        for t in (E[0], E[1], op.pos, op.neg, op.loss):
            t.fill_(float("nan"))
        plan.run()
        got = _snap([E[0], E[1]], op)
        for a, b in zip(ref[:-1], got[:-1]):
            assert np.array_equal(a, b)
        assert abs(got[-1] - ref[-1]) <= 1e-6 * max(1.0, abs(ref[-1]))
    assert folded.timeouts() == 0
    _check_oracle(op, E[1], E[0])


def test_layer2_with_decoder_hipgraph_replays():
    """The folded step captured with layer 1 into one hipGraph of several steps and replayed
    back to back (the bench's form): every replay equals the eager two-launch result."""
    from decagon_amd import kernels as K

    g, plan, rng = _plan_S()
    E = plan.embeddings
    op = _hinge(K, g, rng, E[1], E[1], 32, 512)
    plan.run()
    op()
    ref = _snap([E[0], E[1]], op)
    assert plan.fold_hinge(op)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        plan.run()
        s.synchronize()
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg, stream=s, capture_error_mode="thread_local"):
            for _ in range(5):
                plan.run()
        for _ in range(4):
            op.pos.fill_(float("nan"))
            cg.replay()
    s.synchronize()
    got = _snap([E[0], E[1]], op)
    for a, b in zip(ref[:-1], got[:-1]):
        assert np.array_equal(a, b)
    assert abs(got[-1] - ref[-1]) <= 1e-6 * max(1.0, abs(ref[-1]))
    assert plan.folded_hinge.timeouts() == 0


@pytest.mark.parametrize("n", [512, 777])
def test_layer1_with_decoder_d64(n):
    """The general decoder path (d = 64: two k-blocks, two n-blocks) on layer 1's fused launch,
    which also writes the layer-2 projections: hidden1, the projections and the decoder
    outputs equal the two launches'."""
    from decagon_amd import kernels as K

    g, plan, rng = _plan_S()
    H = plan.hidden1
    f = plan._layer1.launches[0]
    assert isinstance(f, K.PreparedFused)
    op = _hinge(K, g, rng, H[0], H[1], 64, n, row_node=0)
    projs = [pj.out for pj in f._keep[2]]
    f()
    op()
    ref = _snap([H[0], H[1]] + projs, op)
    fh = K.PreparedFusedHinge(f, op)
    for _ in range(2):
        for t in [H[0], H[1], op.pos, op.neg] + projs:
            t.fill_(float("nan"))
        fh()
        got = _snap([H[0], H[1]] + projs, op)
        for a, b in zip(ref[:-1], got[:-1]):
            assert np.array_equal(a, b)
        assert abs(got[-1] - ref[-1]) <= 1e-6 * max(1.0, abs(ref[-1]))
    assert fh.timeouts() == 0
    _check_oracle(op, H[0], H[1])


def test_fold_refused_where_it_does_not_apply():
    """A plan whose layer 2 is not one fused launch (partial mode + epilogue) keeps the
    decoder as its own launch."""
    from decagon_amd import kernels as K
    from decagon_amd import synthetic
    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = synthetic.make_P(seed=3, n_proteins=5000, n_drugs=60, n_side_effects=6)
    rng = np.random.default_rng(0)
    dgr = DeviceGraph(g.edge_types, g.csr(), torch.device("cuda"), None)
    mk = lambda K_, a, b: torch.from_numpy(rng.uniform(-0.1, 0.1, (K_, a, b)).astype(np.float32)).cuda()
    w1 = LayerWeights({et: mk(K_, g.n_nodes[et[1]], 64) for et, K_ in g.edge_types.items()})
    w2 = LayerWeights({et: mk(K_, 64, 32) for et, K_ in g.edge_types.items()})
    plan = ForwardPlan(dgr, {j: None for j in g.n_nodes}, w1, w2, 64, 32)
    E = plan.embeddings
    op = _hinge(K, g, rng, E[1], E[1], 32, 64, given=True)
    assert not plan.fold_hinge(op)


def _step_ref(plan, op):
    plan.run()
    op()
    projs = [pj.out for pj in plan._layer1.launches[0]._keep[2]]
    outs = [plan.hidden1[0], plan.hidden1[1], plan.embeddings[0], plan.embeddings[1]] + projs
    return outs, _snap(outs, op)


@pytest.mark.parametrize("given", [False, True])
@pytest.mark.parametrize("n", [512, 1300])
def test_whole_step_in_one_launch(n, given):
    """dg_gcn_step_f32: layer 1 (+ the layer-2 projections), layer 2 and the decoder step in
    one launch equal the three launches — hidden1, the projections, the embeddings, negatives
    and scores bit for bit — launch after launch, and the scores match the oracle."""
    from decagon_amd import kernels as K

    g, plan, rng = _plan_S()
    E = plan.embeddings
    op = _hinge(K, g, rng, E[1], E[0], 32, n, given)
    outs, ref = _step_ref(plan, op)
    assert plan.fold_step(op)
    for _ in range(3):
        for t in outs + [op.pos, op.neg, op.loss]:
            t.fill_(float("nan"))
        plan.run()
        got = _snap(outs, op)
        for a, b in zip(ref[:-1], got[:-1]):
            assert np.array_equal(a, b)
        assert abs(got[-1] - ref[-1]) <= 1e-6 * max(1.0, abs(ref[-1]))
    assert plan.folded_step.timeouts() == 0
    _check_oracle(op, E[1], E[0])


def test_whole_step_hipgraph_replays():
    """The one-launch step captured G times into a hipGraph and replayed back to back."""
    from decagon_amd import kernels as K

    g, plan, rng = _plan_S()
    E = plan.embeddings
    op = _hinge(K, g, rng, E[1], E[1], 32, 512)
    outs, ref = _step_ref(plan, op)
    assert plan.fold_step(op)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        plan.run()
        s.synchronize()
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg, stream=s, capture_error_mode="thread_local"):
            for _ in range(10):
                plan.run()
        for _ in range(5):
            for t in outs:
                t.fill_(float("nan"))
            cg.replay()
    s.synchronize()
    got = _snap(outs, op)
    for a, b in zip(ref[:-1], got[:-1]):
        assert np.array_equal(a, b)
    assert abs(got[-1] - ref[-1]) <= 1e-6 * max(1.0, abs(ref[-1]))
    assert plan.folded_step.timeouts() == 0
