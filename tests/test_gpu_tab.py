"""GPU: the wave-table fused launch (dg_gcn_fused_tab_f32) against the fused-seg launch it
replaces (dg_gcn_fused_seg_f32) — the same workgroups, waves, batches of 64 and summation order,
so the rows must agree bit for bit — on config S's two layers (the benched form: layer 1 and
the reassociated layer 2) and on a graph of config S's shape whose rows carry relation segments
of 0 to 300 pairs, so the first-batch slot, one and several overflow batches and empty waves
all occur.  Parity with the oracle goes through test_gpu_model.py's golden forward, which runs
this form by default.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _plan(graph, balance=False):
    import bench
    from decagon_amd import engine

    engine.TAB_BALANCE = 2 if balance else 0  # (module policy read at plan build; restored by the fixture)
    args = bench.parse(["--config", "S"])
    args.chunk = dict(graph.edge_types)  # one chunk per group (the fused form's layout)
    plan, _ = bench.make_plan(args, graph, None, torch.device("cuda", 0))
    return plan


@pytest.fixture(autouse=True)
def _restore_balance():
    from decagon_amd import engine

    saved = engine.TAB_BALANCE
    yield
    engine.TAB_BALANCE = saved


def _check(plan, exact=True):
    """Each wave-table launch against its seg form: bit for bit (one wave per relation), or —
    balanced (pairs dealt over every wave slot: a group's sum re-associated) — within fp32
    re-association of a few dozen terms, max|Δ| ≤ 1e-6·max|y| per output."""
    from decagon_amd import kernels

    plan.run()
    torch.cuda.synchronize()
    n = 0
    for layer in plan.spmm_launches:
        for launch in layer:
            if not isinstance(launch, kernels.PreparedFusedTab):
                continue
            outs = launch._keep[1]
            launch()
            torch.cuda.synchronize()
            tab = [o.clone() for o in outs]
            for o in outs:
                o.fill_(float("nan"))
            launch.seg_form()
            torch.cuda.synchronize()
            for a, b in zip(tab, outs):
                assert torch.isfinite(a).all()
                if exact:
                    assert torch.equal(a, b)
                else:
                    assert launch.balance
                    assert float((a - b).abs().max()) <= 1e-6 * float(b.abs().max())
            n += 1
    assert n == 2, "both layers run the wave-table form"


def test_config_S_wave_table_equals_seg_form_bitwise():
    from decagon_amd import synthetic

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    _check(_plan(synthetic.load_S()))


def test_config_S_balanced_wave_table_matches_seg_form():
    """The shipped form (round 6: each row's pairs dealt over every wave slot of its workgroup)
    against the one-wave-per-relation seg form; parity with the float64 oracle is
    test_gpu_model.py's golden forward, which runs this form."""
    from decagon_amd import synthetic

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    _check(_plan(synthetic.load_S(), balance=True), exact=False)


def test_long_segments_wave_table_equals_seg_form_bitwise():
    """Rows whose per-relation segments run to 300 pairs (first batch + up to 4 overflow
    batches), rows with none, on config S's edge types and node counts."""
    from decagon_amd import synthetic

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    base = synthetic.load_S()
    rng = np.random.default_rng(3)
    adj = {}
    for (i, j), K in base.edge_types.items():
        n_r, n_c = base.n_nodes[i], base.n_nodes[j]
        rels = []
        for k in range(K):
            lens = rng.choice([0, 3, 17, 63, 64, 65, 129, 300], size=n_r, p=[.1, .2, .2, .1, .1, .1, .1, .1])
            lens = np.minimum(lens, n_c)
            rows = np.repeat(np.arange(n_r), lens)
            cols = np.concatenate([rng.choice(n_c, size=m, replace=False) for m in lens]) if lens.sum() else \
                np.zeros(0, np.int64)
            vals = rng.standard_normal(rows.size).astype(np.float32) * 0.1
            rels.append((np.stack([rows, cols], 1).astype(np.int64), vals, (n_r, n_c)))
        adj[i, j] = rels
    g = synthetic.SyntheticGraph("S-long", dict(base.n_nodes), dict(base.edge_types), dict(base.decoders), adj,
                                 base.degrees)
    _check(_plan(g))
    _check(_plan(g, balance=True), exact=False)  # slices crossing relations and overflow batches


@pytest.mark.parametrize("world", [4, 8])
def test_row_split_seg_wave_table_equals_seg_form_bitwise(world):
    """Config S's N-GPU row blocks (weak scaling: N relation sets, every node type row-split,
    dg_spmm_seg_f32 partials + the epilogue): every rank's seg launches of both layers in the
    wave-table form equal dg_spmm_seg_f32's chunk partials bit for bit (collectives as no-ops:
    the inputs need not be exchanged for the comparison)."""
    import bench
    from decagon_amd import kernels, synthetic
    from decagon_amd.sharding import RelationShard

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    graph = synthetic.replicate_sets(synthetic.load_S(), world)
    noop = lambda *a, **k: None  # noqa: E731
    for rank in (0, world - 1):
        shard = RelationShard.weak_sets(graph.edge_types, graph.n_nodes, rank, world, noop, noop)
        args = bench.parse(["--config", "S"])
        plan, _ = bench.make_plan(args, graph, shard, torch.device("cuda", 0))
        plan.run()
        torch.cuda.synchronize()
        n = 0
        for layer in plan.spmm_launches:
            for launch in layer:
                if not isinstance(launch, kernels.PreparedSegTab):
                    continue
                outs = [s.out for s in launch.specs]
                launch()
                torch.cuda.synchronize()
                tab = [o.clone() for o in outs]
                for o in outs:
                    o.fill_(float("nan"))
                launch.seg_form()
                torch.cuda.synchronize()
                for a, b in zip(tab, outs):
                    assert torch.equal(a, b)
                n += 1
        assert n >= 2, "both layers run the wave-table seg form"


@pytest.mark.parametrize("world", [4, 8])
def test_row_split_epilogue_table_equals_multi_form_bitwise(world):
    """The finishing launch of config S's N-GPU row blocks (Σ over the N set partials, L2 norm,
    Σ over edge types, relu) in its row-table form equals dg_gcn_epilogue_multi_f32's rows bit
    for bit, both layers, first and last rank."""
    import bench
    from decagon_amd import kernels, synthetic
    from decagon_amd.sharding import RelationShard

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    graph = synthetic.replicate_sets(synthetic.load_S(), world)
    noop = lambda *a, **k: None  # noqa: E731
    for rank in (0, world - 1):
        shard = RelationShard.weak_sets(graph.edge_types, graph.n_nodes, rank, world, noop, noop)
        args = bench.parse(["--config", "S"])
        plan, _ = bench.make_plan(args, graph, shard, torch.device("cuda", 0))
        plan.run()
        torch.cuda.synchronize()
        n = 0
        for layer in (plan._layer1, plan._layer2):
            for e in layer.local_epilogues:
                if not isinstance(e, kernels.PreparedEpilogueTab):
                    continue
                outs = [t for t in e._keep if t.dtype == torch.float32]
                e()
                torch.cuda.synchronize()
                tab = [o.clone() for o in outs]
                e.multi_form()
                torch.cuda.synchronize()
                for a, b in zip(tab, outs):
                    assert torch.equal(a, b)
                n += 1
        assert n == 2, "both layers' finishing launches run the row-table form"


@pytest.mark.parametrize("d", [32, 64])
@pytest.mark.parametrize("flags", [1, 3, 4 | 1, 4 | 3])
def test_epilogue_table_equals_multi_form_long_chunk_runs(d, flags):
    """the row-table epilogue against the multi form, bit for bit, with chunk counts
    that run its four-loads-in-flight loop and its tail loop — 2·CG+1, 3·CG+2 and 255 chunks a
    group (CG = 64/(d/4) lane groups a wave), 1 to 4 groups a row, several targets in one launch,
    and every flag combination the finishing launches use (L2NORM, RELU, CHUNK_RELU)."""
    from decagon_amd import kernels

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cg = 64 // (d // 4)
    runs = [2 * cg + 1, 3 * cg + 2, 255, 1]
    rng = np.random.default_rng(d * 10 + flags)
    targets = []
    for t, n_groups in enumerate((1, 2, 3, 4)):
        n_rows = 37 + 11 * t
        parts = []
        for g in range(n_groups):
            nc = runs[(t + g) % len(runs)]
            p = torch.from_numpy(rng.standard_normal((nc, n_rows, d)).astype(np.float32)).cuda()
            parts.append((p, nc))
        targets.append((parts, torch.empty((n_rows, d), device="cuda"), n_rows))
    tgt_a = [(parts, out, n) for parts, out, n in targets[:2]]
    tgt_b = [(parts, out, n) for parts, out, n in targets[2:]]
    for tg in (tgt_a, tgt_b):
        launch = kernels.PreparedEpilogueTab(tg, d, flags)
        for _, out, _ in tg:
            out.fill_(float("nan"))
        launch()
        torch.cuda.synchronize()
        tab = [out.clone() for _, out, _ in tg]
        for _, out, _ in tg:
            out.fill_(float("nan"))
        launch.multi_form()
        torch.cuda.synchronize()
        for a, (_, out, _) in zip(tab, tg):
            assert torch.equal(a, out)
            assert not torch.isnan(a).any()
