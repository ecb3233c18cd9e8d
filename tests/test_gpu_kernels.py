"""Kernel-level parity: every C-ABI entry point against the float64 oracle on seeded inputs,
including the edge cases the reference's data produce (empty rows — genes without drug
targets in (0,1); empty relations; single-relation groups; rectangular Â; d in
{4..256}).  Tolerance: max|y − y_ref| / max|y_ref| ≤ 1e-4 for fp32 outputs;
integer outputs bit-exact.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import rel_err, alias_draws
from oracle import decagon_oracle as orc

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def K():
    from decagon_amd import kernels

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return kernels


def _rand_csr(rng, n_r, n_c, density, empty_rows=0.0):
    m = sp.random(n_r, n_c, density=density, random_state=rng, format="csr", dtype=np.float64)
    if empty_rows:
        drop = rng.random(n_r) < empty_rows
        m = sp.diags((~drop).astype(np.float64)) @ m
        m = m.tocsr()
    m.eliminate_zeros()
    m.sort_indices()
    return m


def _dev_csr(m):
    from decagon_amd.sparse import coo_to_csr, sparse_to_tuple

    h = coo_to_csr(*sparse_to_tuple(m))
    return (torch.from_numpy(h.rowptr).cuda(), torch.from_numpy(h.col).cuda(),
            torch.from_numpy(h.val).cuda(), h)


@pytest.mark.parametrize("d", [4, 8, 16, 32, 48, 64, 128, 256])
def test_spmm_csr_matches_oracle(K, d):
    rng = np.random.default_rng(d)
    m = _rand_csr(rng, 301, 257, 0.05, empty_rows=0.2)
    x = rng.standard_normal((257, d)).astype(np.float32)
    rp, cl, vl, h = _dev_csr(m)
    y = K.spmm_csr(rp, cl, vl, torch.from_numpy(x).cuda(), 301)
    want = orc.sparse_dense_matmul((np.stack(m.nonzero(), 1), m.data, m.shape), x.astype(np.float64))
    # (nonzero order differs from CSR order only by summation order)
    assert rel_err(y.cpu().numpy(), want) <= 1e-5
    zero_rows = np.diff(m.indptr) == 0
    assert np.all(y.cpu().numpy()[zero_rows] == 0)


def test_spmm_long_rows(K):
    """Rows longer than one 64-nonzero batch, and a dense row."""
    rng = np.random.default_rng(3)
    m = _rand_csr(rng, 40, 3000, 0.2).tolil()
    m[5, :] = rng.random(3000)
    m = m.tocsr()
    m.sort_indices()
    x = rng.standard_normal((3000, 64)).astype(np.float32)
    rp, cl, vl, _ = _dev_csr(m)
    y = K.spmm_csr(rp, cl, vl, torch.from_numpy(x).cuda(), 40).cpu().numpy()
    want = m @ x.astype(np.float64)
    assert rel_err(y, want) <= 1e-5


def test_spmm_empty_matrix(K):
    m = sp.csr_matrix((17, 9))
    rp, cl, vl, _ = _dev_csr(m)
    x = torch.ones((9, 32), device="cuda")
    y = K.spmm_csr(rp, cl, vl, x, 17)
    assert torch.count_nonzero(y) == 0


@pytest.mark.parametrize("d", [32, 64])
def test_spmm_csr_beta_accumulates_add_n(K, d):
    """dg_spmm_csr_f32's beta: beta = 1 adds each relation's Â_k·X_k into a running
    sum — tf.add_n of layers.py:92 one relation at a time — bit for bit fmaf(1, Y, Â_k·X_k);
    beta = 0 overwrites a NaN-filled out without reading it; beta = 0.5 scales the old sum."""
    rng = np.random.default_rng(40 + d)
    mats = [_rand_csr(rng, 203, 150, 0.06, empty_rows=0.1) for _ in range(3)]
    xs = [rng.standard_normal((150, d)).astype(np.float32) for _ in mats]
    out = torch.full((203, d), float("nan"), device="cuda")
    parts = []
    for k, (m, x) in enumerate(zip(mats, xs)):
        rp, cl, vl, _ = _dev_csr(m)
        xd = torch.from_numpy(x).cuda()
        parts.append(K.spmm_csr(rp, cl, vl, xd, 203))
        K.spmm_csr(rp, cl, vl, xd, 203, out=out, beta=0.0 if k == 0 else 1.0)
    # add_n order: ((P0 + P1) + P2), each add one fp32 rounding — what fmaf(1, y, p) gives
    assert torch.equal(out, (parts[0] + parts[1]) + parts[2])
    want = sum(orc.sparse_dense_matmul((np.stack(m.nonzero(), 1), m.data, m.shape), x.astype(np.float64))
               for m, x in zip(mats, xs))
    assert rel_err(out.cpu().numpy(), want) <= 1e-5
    rp, cl, vl, _ = _dev_csr(mats[0])
    old = out.clone()
    K.spmm_csr(rp, cl, vl, torch.from_numpy(xs[0]).cuda(), 203, out=out, beta=0.5)
    want_half = torch.addcmul(parts[0], old, torch.full_like(old, 0.5))  # fmaf(0.5, old, p): exact scale
    assert torch.allclose(out, want_half, rtol=1e-6, atol=1e-6)
    with pytest.raises(ValueError):
        K.spmm_csr(rp, cl, vl, torch.from_numpy(xs[0]).cuda(), 203, beta=1.0)  # no running sum given


@pytest.mark.parametrize("d", [8, 32, 64, 256])
@pytest.mark.parametrize("relu", [False, True])
def test_rownorm_l2_matches_oracle(K, d, relu):
    """dg_rownorm_l2_f32 against oracle.l2_normalize_rows (TF 1.8: x·rsqrt(max(Σx², 1e-12)),
    layers.py:93, :117), including all-zero rows (which stay 0), in place and out of place, and
    bit for bit the fused epilogue's normalisation of the same rows."""
    rng = np.random.default_rng(7 * d + relu)
    x = rng.standard_normal((517, d)).astype(np.float32)
    x[rng.random(517) < 0.1] = 0.0
    x[3] *= 1e-7  # tiny but nonzero: Σx² below the 1e-12 floor
    xd = torch.from_numpy(x).cuda()
    y = K.rownorm_l2(xd, relu=relu)
    want = orc.l2_normalize_rows(x.astype(np.float64))
    if relu:
        want = np.maximum(want, 0.0)
    assert rel_err(y.cpu().numpy(), want) <= 1e-5
    assert np.all(y.cpu().numpy()[~x.any(axis=1)] == 0)
    ref = torch.empty_like(xd)
    K.PreparedEpilogue([(xd, 1)], ref, 517, d, 1 | (2 if relu else 0))()
    assert torch.equal(y, ref)
    z = xd.clone()
    K.rownorm_l2(z, out=z, relu=relu)
    assert torch.equal(z, y)


@pytest.mark.parametrize("chunk", [1, 2, 3, 7])
@pytest.mark.parametrize("d", [32, 64])
def test_spmm_groups_chunks_and_slabs(K, chunk, d):
    """Chunk-merged relations, chunked partial sums, relations living in arbitrary slabs of
    a bigger stacked operand (a rank's shard), and two groups in one launch."""
    from decagon_amd.sparse import coo_to_csr, merge_chunks, sparse_to_tuple

    rng = np.random.default_rng(chunk * 100 + d)
    wants, specs = [], []
    for (n_r, n_c, nrel) in ((120, 90, 7), (90, 120, 3)):
        mats = [_rand_csr(rng, n_r, n_c, 0.04, empty_rows=0.1) for _ in range(nrel)]
        total = nrel + 4
        slabs = rng.choice(total, size=nrel, replace=False).astype(np.int32)
        m = merge_chunks([coo_to_csr(*sparse_to_tuple(x)) for x in mats], slabs, chunk, total)
        X = rng.standard_normal((total, n_c, d)).astype(np.float32)
        nch = m.n_chunks
        out = torch.zeros((nch, n_r, d), device="cuda")
        spec = K.RelGroupSpec(torch.from_numpy(m.rowptr).cuda(), torch.from_numpy(m.vcol).cuda(),
                              torch.from_numpy(m.val).cuda(), torch.from_numpy(X).cuda(), out, n_r, nch, d,
                              total * n_c, vcol_max=int(m.vcol.max()))
        specs.append(spec)
        want = np.zeros((nch, n_r, d))
        for k, x in enumerate(mats):
            want[k // m.chunk] += x @ X[slabs[k]].astype(np.float64)
        wants.append(want)
    K.spmm_groups(specs, d)
    for s, w in zip(specs, wants):
        assert rel_err(s.out.cpu().numpy(), w) <= 1e-5


@pytest.mark.parametrize("chunk", [1, 3, 6, 16])
@pytest.mark.parametrize("form", [(32, 32), (64, 64), (64, 32)])
def test_spmm_seg_chunks_and_reassociated_projection(K, chunk, form):
    """dg_spmm_seg_f32 (one wave per (row, relation)): chunk partials of the chunk-merged layout
    with relations in arbitrary slabs, two groups (one with a short last chunk) in one launch;
    with a weight stack (d_in 64 → d_out 32) the reassociated layer 2, Σ_k (Â_k·H)·W[slab_k]
    (layers.py:113-114 with the sum regrouped), against the float64 products."""
    from decagon_amd.sparse import chunk_segments, coo_to_csr, merge_chunks, sparse_to_tuple

    d_in, d_out = form
    proj = d_in != d_out
    rng = np.random.default_rng(chunk * 1000 + d_in + d_out)
    wants, specs = [], []
    for (n_r, n_c, nrel, dens) in ((57, 90, 2 * chunk, 0.05), (40, 33, chunk + max(1, chunk // 2), 0.3)):
        mats = [_rand_csr(rng, n_r, n_c, dens, empty_rows=0.2) for _ in range(nrel)]
        mats[0] = sp.csr_matrix((n_r, n_c))  # an empty relation
        total = nrel + 3
        slabs = rng.choice(total, size=nrel, replace=False).astype(np.int32)
        hs = [coo_to_csr(*sparse_to_tuple(x)) for x in mats]
        m = merge_chunks(hs, slabs, chunk, total)
        seg = chunk_segments(hs, m)
        nch = m.n_chunks
        out = torch.full((nch, n_r, d_out), float("nan"), device="cuda")
        want = np.zeros((nch, n_r, d_out))
        if proj:
            H = rng.standard_normal((n_c, 64)).astype(np.float32)
            W = (0.2 * rng.standard_normal((total, 64, 32))).astype(np.float32)
            x, w = torch.from_numpy(H).cuda(), torch.from_numpy(W).cuda()
            for k, a in enumerate(mats):
                want[k // chunk] += (a @ H.astype(np.float64)) @ W[slabs[k]].astype(np.float64)
        else:
            X = rng.standard_normal((total * n_c, d_in)).astype(np.float32)
            x, w = torch.from_numpy(X).cuda(), None
            for k, a in enumerate(mats):
                want[k // chunk] += a @ X[slabs[k] * n_c:(slabs[k] + 1) * n_c].astype(np.float64)
        specs.append(K.SegSpec(torch.from_numpy(m.rowptr).cuda(), torch.from_numpy(seg).cuda(),
                               torch.from_numpy(m.vcol).cuda(), torch.from_numpy(m.val).cuda(), x, out, n_r, n_c,
                               nch, chunk, nrel, d_in, total * n_c, vcol_max=int(m.vcol.max()), w=w,
                               slab=torch.from_numpy(slabs).cuda(), slab_max=int(slabs.max())))
        wants.append(want)
    K.PreparedSeg(specs, d_in, d_out)()
    for s, w in zip(specs, wants):
        got = s.out.cpu().numpy()
        assert rel_err(got, w) <= 1e-5
        assert np.all(got[:, np.all(w == 0, axis=(0, 2))] == 0)  # rows without nonzeros: exact zeros


@pytest.mark.parametrize("form", [(32, 32, True), (64, 64, True), (64, 32, False)])
def test_gcn_fused_seg_layer(K, form):
    """dg_gcn_fused_seg_f32: two node types, each with two groups of one chunk holding all their
    relations (one with an empty relation, rows without nonzeros), finished in one launch —
    act(Σ_g l2norm(Σ_k Â_k·X_k)) (layers.py:85-94, model.py:74-75), and with weight stacks the
    reassociated layer 2, Σ_g l2norm(Σ_k (Â_k·H_j)·W[slab_k]) (layers.py:109-118, model.py:85-88)."""
    from decagon_amd.sparse import chunk_segments, coo_to_csr, merge_chunks, sparse_to_tuple

    d_in, d_out, relu = form
    proj = d_in != d_out
    rng = np.random.default_rng(d_in * 7 + d_out)
    n = {0: 61, 1: 45}
    ets = {(0, 0): 3, (0, 1): 2, (1, 0): 1, (1, 1): 6}
    H = {j: rng.standard_normal((n[j], 64)).astype(np.float32) for j in n}
    outs, targets, want = {}, [], {}
    for i in (0, 1):
        specs, tot = [], np.zeros((n[i], d_out))
        for (ti, j), nrel in ets.items():
            if ti != i:
                continue
            mats = [_rand_csr(rng, n[i], n[j], 0.1, empty_rows=0.2) for _ in range(nrel)]
            if nrel > 2:
                mats[1] = sp.csr_matrix((n[i], n[j]))
            total = nrel + 2
            slabs = rng.permutation(total)[:nrel].astype(np.int32)
            hs = [coo_to_csr(*sparse_to_tuple(x)) for x in mats]
            m = merge_chunks(hs, slabs, nrel, total)
            seg = torch.from_numpy(chunk_segments(hs, m)).cuda()
            ssum = np.zeros((n[i], d_out))
            if proj:
                W = (0.2 * rng.standard_normal((total, 64, 32))).astype(np.float32)
                x, w = torch.from_numpy(H[j]).cuda(), torch.from_numpy(W).cuda()
                for k, a in enumerate(mats):
                    ssum += (a @ H[j].astype(np.float64)) @ W[slabs[k]].astype(np.float64)
            else:
                X = rng.standard_normal((total * n[j], d_in)).astype(np.float32)
                x, w = torch.from_numpy(X).cuda(), None
                for k, a in enumerate(mats):
                    ssum += a @ X[slabs[k] * n[j]:(slabs[k] + 1) * n[j]].astype(np.float64)
            tot += ssum / np.sqrt(np.maximum((ssum ** 2).sum(1, keepdims=True), 1e-12))
            specs.append(K.SegSpec(torch.from_numpy(m.rowptr).cuda(), seg, torch.from_numpy(m.vcol).cuda(),
                                   torch.from_numpy(m.val).cuda(), x, None, n[i], n[j], 1, nrel, nrel,
                                   x.stride(0), total * n[j], vcol_max=int(m.vcol.max()), w=w,
                                   slab=torch.from_numpy(slabs).cuda(), slab_max=int(slabs.max())))
        outs[i] = torch.full((n[i], d_out), float("nan"), device="cuda")
        targets.append((outs[i], n[i], specs, relu))
        want[i] = np.maximum(tot, 0) if relu else tot
    K.PreparedFusedSeg(targets, d_in, d_out)()
    for i in (0, 1):
        assert rel_err(outs[i].cpu().numpy(), want[i]) <= 1e-5


@pytest.mark.parametrize("d", [12, 64])
def test_spmm_shared_pattern(K, d):
    """DG_GROUP_SHARED_PATTERN: one CSR (X_j's) for every chunk, chunk k over its own slab
    (X_j·W_k for all k, layers.py:89) — bit-identical to the merged layout that repeats the
    pattern K times, beside a merged group in the same launch; rejected by the fused and LDS
    entry points."""
    from decagon_amd import _lib
    from decagon_amd.sparse import coo_to_csr, merge_chunks, sparse_to_tuple

    rng = np.random.default_rng(d)
    n_r, F, nrel = 77, 130, 5
    m = _rand_csr(rng, n_r, F, 0.06, empty_rows=0.15)
    h = coo_to_csr(*sparse_to_tuple(m))
    W = torch.from_numpy(rng.standard_normal((nrel, F, d)).astype(np.float32)).cuda()
    out_s = torch.zeros((nrel, n_r, d), device="cuda")
    out_m = torch.zeros((nrel, n_r, d), device="cuda")
    shared = K.RelGroupSpec(torch.from_numpy(h.rowptr).cuda(), torch.from_numpy(h.col).cuda(),
                            torch.from_numpy(h.val).cuda(), W, out_s, n_r, nrel, d, F,
                            vcol_max=int(h.col.max()), shared=True)
    mm = merge_chunks([h] * nrel, np.arange(nrel), 1, nrel)
    merged = K.RelGroupSpec(torch.from_numpy(mm.rowptr).cuda(), torch.from_numpy(mm.vcol).cuda(),
                            torch.from_numpy(mm.val).cuda(), W, out_m, n_r, nrel, d, nrel * F,
                            vcol_max=int(mm.vcol.max()))
    K.spmm_groups([shared, merged], d)
    assert torch.equal(out_s, out_m)
    want = np.stack([m @ W[k].cpu().numpy().astype(np.float64) for k in range(nrel)])
    assert rel_err(out_s.cpu().numpy(), want) <= 1e-5
    with pytest.raises(_lib.KernelError):
        K.PreparedSpmm([shared], d, lds=True)()
    # an unknown flag bit is refused before launch
    arr = (_lib.DgRelGroup * 1)()
    K._fill_group(arr[0], shared)
    arr[0].flags = 2
    assert _lib.load().dg_spmm_groups_f32(arr, 1, d, None) != 0


def test_fused_kernel_matches_oracle(K):
    """dg_gcn_fused_f32 with two targets, several groups each, waves_per_group 1..3 and a
    projection epilogue against the float64 restatement."""
    from decagon_amd.sparse import coo_to_csr, merge_chunks, sparse_to_tuple

    rng = np.random.default_rng(42)
    n = {0: 150, 1: 90}
    ets = {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 3}
    mats, X, specs_by_t, want = {}, {}, {0: [], 1: []}, {}
    for et, Kr in ets.items():
        mats[et] = [_rand_csr(rng, n[et[0]], n[et[1]], 0.08, empty_rows=0.1) for _ in range(Kr)]
        X[et] = rng.standard_normal((Kr, n[et[1]], 64)).astype(np.float32)
        m = merge_chunks([coo_to_csr(*sparse_to_tuple(x)) for x in mats[et]], np.arange(Kr), Kr, Kr)
        specs_by_t[et[0]].append(K.RelGroupSpec(
            torch.from_numpy(m.rowptr).cuda(), torch.from_numpy(m.vcol).cuda(), torch.from_numpy(m.val).cuda(),
            torch.from_numpy(X[et]).cuda(), None, n[et[0]], 1, 64, Kr * n[et[1]], vcol_max=int(m.vcol.max())))
    for t in (0, 1):
        tot = 0
        for et in ets:
            if et[0] == t:
                s = sum(mats[et][k] @ X[et][k].astype(np.float64) for k in range(ets[et]))
                tot = tot + orc.l2_normalize_rows(s)
        want[t] = np.maximum(tot, 0)
    W2 = rng.standard_normal((5, 64, 32)).astype(np.float32)
    P = torch.zeros((5, n[1], 32), device="cuda")
    rmap = torch.tensor([4, 0, 2], dtype=torch.int32, device="cuda")
    for wpg in (1, 2, 3):
        outs = {t: torch.empty((n[t], 64), device="cuda") for t in (0, 1)}
        proj = K.ProjSpec(torch.from_numpy(W2).cuda(), P, 3, 1, rel_map=rmap, rel_map_max=4)
        K.PreparedFused([(outs[t], n[t], specs_by_t[t], True) for t in (0, 1)], 64, [proj], wpg)()
        for t in (0, 1):
            assert rel_err(outs[t].cpu().numpy(), want[t]) <= 1e-5
        for kk, rel in enumerate([4, 0, 2]):
            assert rel_err(P[rel].cpu().numpy(), want[1] @ W2[rel].astype(np.float64)) <= 1e-5


@pytest.mark.parametrize("flags", [0, 1, 2, 3, 5])
def test_epilogue(K, flags):
    from decagon_amd._lib import DG_EPI_CHUNK_RELU, DG_EPI_L2NORM, DG_EPI_RELU

    rng = np.random.default_rng(flags)
    n, d = 333, 64
    parts = []
    for nch in (3, 1, 2):
        p = rng.standard_normal((nch, n, d)).astype(np.float32)
        p[:, ::7] = 0.0  # all-zero rows: l2_normalize keeps them 0
        parts.append(p)
    out = torch.empty((n, d), device="cuda")
    K.gcn_epilogue([(torch.from_numpy(p).cuda(), p.shape[0]) for p in parts], out, n, d, flags)
    tot = np.zeros((n, d))
    for p in parts:
        p = p.astype(np.float64)
        if flags & DG_EPI_CHUNK_RELU:
            p = np.maximum(p, 0)
        s = p.sum(0)
        if flags & DG_EPI_L2NORM:
            s = orc.l2_normalize_rows(s)
        tot += s
    if flags & DG_EPI_RELU:
        tot = np.maximum(tot, 0)
    assert rel_err(out.cpu().numpy(), tot) <= 1e-5
    assert np.all(out.cpu().numpy()[::7] == 0)


@pytest.mark.parametrize("d", [32, 64])
def test_epilogue_multi_target(K, d):
    """dg_gcn_epilogue_multi_f32: three node types (one of them empty) in one launch, bit for
    bit what one dg_gcn_epilogue_f32 per node type writes."""
    from decagon_amd._lib import DG_EPI_L2NORM, DG_EPI_RELU

    rng = np.random.default_rng(d)
    flags = DG_EPI_L2NORM | DG_EPI_RELU
    targets, singles = [], []
    for n, chunks in ((1001, (2, 1)), (0, (1,)), (645, (3, 1, 1))):
        parts = [(torch.from_numpy(rng.standard_normal((c, n, d)).astype(np.float32)).cuda(), c) for c in chunks]
        out, ref = torch.zeros((n, d), device="cuda"), torch.zeros((n, d), device="cuda")
        targets.append((parts, out, n))
        singles.append((parts, ref, n))
    K.PreparedEpilogueMulti(targets, d, flags)()
    for parts, ref, n in singles:
        K.gcn_epilogue(parts, ref, n, d, flags)
    for (_, out, _), (_, ref, _) in zip(targets, singles):
        assert torch.equal(out, ref)


@pytest.mark.parametrize("m,n,k,batch", [(645, 32, 64, 5), (37, 70, 19, 3), (1, 1, 1, 1), (500, 32, 32, 2),
                                         (64, 96, 0, 1)])
def test_gemm(K, m, n, k, batch):
    rng = np.random.default_rng(m * n + k)
    A = rng.standard_normal((m, k)).astype(np.float32)
    B = rng.standard_normal((batch + 2, k, n)).astype(np.float32)
    bmap = rng.permutation(batch + 2)[:batch].astype(np.int32)
    sa = rng.standard_normal(k).astype(np.float32)
    sc = rng.standard_normal(n).astype(np.float32)
    C = torch.zeros((batch + 2, m, n), device="cuda")  # C is indexed by the map too
    K.PreparedGemm(torch.from_numpy(A).cuda(), (0, k, 1), torch.from_numpy(B).cuda(), (k * n, n, 1), C,
                   (m * n, n, 1), m, n, k, batch, torch.from_numpy(sa).cuda(), torch.from_numpy(sc).cuda(),
                   b_map=torch.from_numpy(bmap).cuda(), b_batches=batch + 2, b_map_max=int(bmap.max()))()
    for b in range(batch):
        want = ((A.astype(np.float64) * sa) @ B[bmap[b]].astype(np.float64)) * sc
        got = C[bmap[b]].cpu().numpy()
        if k == 0:
            assert np.all(got == 0)
        else:
            assert rel_err(got, want) <= 1e-5


@pytest.mark.parametrize("m,n,k,batch", [(645, 32, 64, 37), (100, 32, 32, 5), (33, 16, 64, 300),
                                         (1000, 32, 64, 1)])
def test_gemm_projection(K, m, n, k, batch):
    """The relation-batched projection path (shared A, n <= 32, unscaled): C[bmap[b]] =
    A · B[bmap[b]], float4 stores of the transposed MFMA product, partial row tiles."""
    rng = np.random.default_rng(m + n + k + batch)
    A = rng.standard_normal((m, k)).astype(np.float32)
    B = rng.standard_normal((batch + 3, k, n)).astype(np.float32)
    bmap = rng.permutation(batch + 3)[:batch].astype(np.int32)
    C = torch.full((batch + 3, m, n), 7.0, device="cuda")
    K.PreparedGemm(torch.from_numpy(A).cuda(), (0, k, 1), torch.from_numpy(B).cuda(), (k * n, n, 1), C,
                   (m * n, n, 1), m, n, k, batch, b_map=torch.from_numpy(bmap).cuda(), b_batches=batch + 3,
                   b_map_max=int(bmap.max()))()
    got = C.cpu().numpy()
    for b in range(batch):
        want = A.astype(np.float64) @ B[bmap[b]].astype(np.float64)
        assert rel_err(got[bmap[b]], want) <= 1e-5
    untouched = np.setdiff1d(np.arange(batch + 3), bmap)
    assert np.all(got[untouched] == 7.0)


def test_gemm_transposed_strides(K):
    rng = np.random.default_rng(11)
    A = rng.standard_normal((50, 32)).astype(np.float32)
    E = rng.standard_normal((70, 32)).astype(np.float32)
    Ad, Ed = torch.from_numpy(A).cuda(), torch.from_numpy(E).cuda()
    out = K.matmul(Ad, Ed.t())
    assert rel_err(out.cpu().numpy(), A.astype(np.float64) @ E.T.astype(np.float64)) <= 1e-5


@pytest.mark.parametrize("d", [32, 64, 256])
@pytest.mark.parametrize("diag", [False, True])
def test_decoder_score(K, d, diag):
    rng = np.random.default_rng(d + diag)
    n_r, n_c, npairs = 300, 200, 1000 + 17
    U = rng.standard_normal((n_r, d)).astype(np.float32)
    V = rng.standard_normal((n_c, d)).astype(np.float32)
    G = (rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)
    l = rng.standard_normal(d).astype(np.float32) if diag else None
    ri = rng.integers(0, n_r, npairs).astype(np.int32)
    ci = rng.integers(0, n_c, npairs).astype(np.int32)
    got = K.decoder_score(torch.from_numpy(U).cuda(), torch.from_numpy(V).cuda(), torch.from_numpy(ri).cuda(),
                          torch.from_numpy(ci).cuda(), torch.from_numpy(G).cuda(),
                          None if l is None else torch.from_numpy(l).cuda()).cpu().numpy()
    L = np.eye(d) if l is None else np.diag(l.astype(np.float64))
    want = orc.batch_predict([U.astype(np.float64), V.astype(np.float64)], 0, 1, G.astype(np.float64), L, ri, ci)
    assert rel_err(got, want) <= 1e-5


@pytest.mark.parametrize("d", [64, 128, 256])
def test_decoder_score_bf16(K, d):
    """Config 5's bf16 DEDICOM scorer against float64 on the same bf16 inputs: the kernel
    rounds u∘D_k to bf16 (the MFMA operand) and accumulates in fp32 — tolerance 1e-4 against
    a reference that applies the same operand rounding.  Pairs mix relations; ragged tail."""
    rng = np.random.default_rng(d)
    n_r, n_c, n_rel, n = 300, 200, 7, 32 * 40 + 13
    bf = torch.bfloat16
    E_r = torch.from_numpy(rng.standard_normal((n_r, d)).astype(np.float32)).to(bf)
    E_c = torch.from_numpy(rng.standard_normal((n_c, d)).astype(np.float32)).to(bf)
    R = torch.from_numpy((rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)).to(bf)
    Dk = torch.from_numpy(rng.standard_normal((n_rel, d)).astype(np.float32)).to(bf)
    rows = rng.integers(0, n_r, n).astype(np.int32)
    cols = rng.integers(0, n_c, n).astype(np.int32)
    rel = rng.integers(0, n_rel, n).astype(np.int32)
    got = K.decoder_score_bf16(E_r.cuda(), E_c.cuda(), torch.from_numpy(rows).cuda(), torch.from_numpy(cols).cuda(),
                               R.cuda(), Dk.cuda(), torch.from_numpy(rel).cuda()).cpu().numpy()
    u = E_r.float().numpy()[rows]
    v = E_c.float().numpy()[cols]
    dk = Dk.float().numpy()[rel]
    a = torch.from_numpy((u * dk).astype(np.float32)).to(bf).double().numpy()  # the bf16 operand
    want = np.einsum("pi,in,pn->p", a, R.double().numpy(), dk.astype(np.float64) * v.astype(np.float64))
    assert rel_err(got, want) <= 1e-4
    # identity diagonal, single relation
    got2 = K.decoder_score_bf16(E_r.cuda(), E_c.cuda(), torch.from_numpy(rows).cuda(), torch.from_numpy(cols).cuda(),
                                R.cuda()).cpu().numpy()
    want2 = np.einsum("pi,in,pn->p", u.astype(np.float64), R.double().numpy(), v.astype(np.float64))
    assert rel_err(got2, want2) <= 1e-4


@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("n_half", [32 * 40 + 13, 7, 4096])
def test_decoder_score_bf16_paired(K, d, n_half):
    """dg_decoder_score_bf16_paired (config 5's positive / negative layout: pair p and p + n_half
    share the column and the relation) against the float64 restatement of its association,
    (u∘D_k)ᵀ·(R·bf16(D_k∘v)) — T = R·(D_k∘v) once per positive / negative pair, the bf16
    operand rounding on D_k∘v — and against the row-side kernel (operand rounding on u∘D_k:
    the two agree to bf16 operand rounding); ragged tails, relations mixed within a tile, with
    and without the diagonals."""
    rng = np.random.default_rng(d + n_half)
    n_r, n_c, n_rel = 300, 200, 7
    bf = torch.bfloat16
    E_r = torch.from_numpy(rng.standard_normal((n_r, d)).astype(np.float32)).to(bf)
    E_c = torch.from_numpy(rng.standard_normal((n_c, d)).astype(np.float32)).to(bf)
    R = torch.from_numpy((rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)).to(bf)
    Dk = torch.from_numpy(rng.standard_normal((n_rel, d)).astype(np.float32)).to(bf)
    rows = rng.integers(0, n_r, 2 * n_half).astype(np.int32)
    c1 = rng.integers(0, n_c, n_half).astype(np.int32)
    r1 = rng.integers(0, n_rel, n_half).astype(np.int32)
    cols, rel = np.concatenate([c1, c1]), np.concatenate([r1, r1])
    dv = lambda x: torch.from_numpy(x).cuda()
    for L in (Dk, None):
        args = (E_r.cuda(), E_c.cuda(), dv(rows), dv(cols), R.cuda(), None if L is None else L.cuda(), dv(rel))
        got = K.decoder_score_bf16(*args, paired=True).cpu().numpy()
        ref = K.decoder_score_bf16(*args).cpu().numpy()
        assert rel_err(got, ref) <= 2e-2  # bf16 operand rounding on the other side
        u = E_r.float().numpy()[rows]
        v = E_c.float().numpy()[cols]
        dk = L.float().numpy()[rel] if L is not None else np.ones_like(u)
        b = torch.from_numpy((dk * v).astype(np.float32)).to(bf).double().numpy()  # the bf16 operand
        want = np.einsum("pi,in,pn->p", u.astype(np.float64) * dk.astype(np.float64), R.double().numpy(), b)
        assert rel_err(got, want) <= 1e-4
    with pytest.raises(ValueError):
        K.decoder_score_bf16(E_r.cuda(), E_c.cuda(), dv(rows[:-1]), dv(cols[:-1]), R.cuda(), paired=True)


@pytest.mark.parametrize("range_,batch,slot0,n_slots,per_slot", [
    (645, 512, 0, 7, True),      # config 5's tables
    (33, 37, 3, 5, True),        # odd batch, a slot sub-range
    (1, 3, 0, 2, True),          # one row
    (200, 64, 2, 3, False),      # one shared table (= dg_unigram_sample at offset slot0·batch)
])
def test_unigram_sample_slots(K, range_, batch, slot0, n_slots, per_slot):
    """dg_unigram_sample_slots: draw i of slot slot0 + i // batch is exactly the restated alias
    draw (conftest.alias_draws) of THAT slot's table at counter slot0·batch + i — per-relation
    degree distributions (optimizer.py:38-47), independent of how slots are dealt to ranks."""
    from decagon_amd.sampling import alias_table

    rng = np.random.default_rng(range_ + batch)
    total = slot0 + n_slots
    degs = [rng.integers(0, 40, range_).astype(np.float64) for _ in range(total)]
    for x in degs:
        x[rng.integers(0, range_)] += 1  # a positive sum
    tabs = np.stack([alias_table(x) for x in degs]) if per_slot else alias_table(degs[0])
    n = n_slots * batch
    got = K.unigram_sample_slots(torch.from_numpy(tabs.view(np.int32)).cuda(), slot0, batch, n, 1234).cpu().numpy()
    for s in range(n_slots):
        tab = tabs[slot0 + s] if per_slot else tabs
        idx = slot0 * batch + s * batch + np.arange(batch)
        assert np.array_equal(got[s * batch:(s + 1) * batch], alias_draws(tab, 1234, idx)), s
    if not per_slot:  # the shared-table form is dg_unigram_sample's stream
        one = K.unigram_sample(torch.from_numpy(tabs.view(np.int32)).cuda(), n, 1234, slot0 * batch).cpu().numpy()
        assert np.array_equal(got, one)


def test_losses(K):
    rng = np.random.default_rng(5)
    pos = rng.standard_normal(1000).astype(np.float32)
    neg = rng.standard_normal(1000).astype(np.float32)
    P, N = torch.from_numpy(pos).cuda(), torch.from_numpy(neg).cuda()
    h = float(K.hinge_loss(P, N, 0.1)[0])
    x = float(K.xent_loss(P, N, 1.0)[0])
    assert abs(h - orc.hinge_loss(pos, neg, 0.1)) <= 1e-4 * abs(orc.hinge_loss(pos, neg, 0.1))
    assert abs(x - orc.xent_loss(pos, neg, 1.0)) <= 1e-4 * abs(orc.xent_loss(pos, neg, 1.0))
    # deterministic: same bits twice
    assert float(K.hinge_loss(P, N, 0.1)[0]) == h


def test_unigram_sampler_distribution(K):
    from decagon_amd.sampling import alias_table, table_distribution

    rng = np.random.default_rng(9)
    deg = rng.integers(0, 50, 400).astype(np.float64)
    deg[:10] = 0
    p = orc.unigram_distribution(deg)
    tab = alias_table(deg)
    assert np.max(np.abs(table_distribution(tab) - p)) < 1e-7  # the table encodes p exactly
    dt = torch.from_numpy(tab.view(np.int32)).cuda()
    n = 400000
    s = K.unigram_sample(dt, n, seed=1, offset=0).cpu().numpy()
    assert s.min() >= 0 and s.max() < 400
    assert np.all(np.bincount(s, minlength=400)[:10] == 0)  # zero degree never drawn
    freq = np.bincount(s, minlength=400) / n
    assert np.max(np.abs(freq - p)) < 5e-3
    s2 = K.unigram_sample(dt, n, seed=1, offset=0).cpu().numpy()
    assert np.array_equal(s, s2)  # counter-based: reproducible


def test_shape_checks_fail_before_launch(K):
    """Host checks reject buffers too small for the indices the kernel would form."""
    m = sp.random(10, 10, density=0.3, random_state=0, format="csr")
    rp, cl, vl, _ = _dev_csr(m)
    x = torch.zeros((5, 32), device="cuda")  # fewer rows than n_cols
    with pytest.raises(ValueError):
        K.RelGroupSpec(rp, cl, vl, x, torch.zeros((1, 10, 32), device="cuda"), 10, 1, 32, 10,
                       vcol_max=int(cl.max())).validate(32)


@pytest.mark.parametrize("n,scale", [(512, 1), (100, 1), (1300, 1), (9000, 1), (512, 40), (9000, 40)])
def test_decoder_hinge_fused(K, n, scale):
    """dg_decoder_hinge_f32: sampled negatives are exactly dg_unigram_sample's draws, both
    score vectors match the oracle, the loss is the hinge of optimizer.py:116-120 — through the
    packed fixed-point atomic (≤ 255 blocks), with block partials ≥ 256 (scale 40: the
    write-through fallback inside it), and through the ticket (9,000 pairs: 282 blocks)."""
    rng = np.random.default_rng(n + scale)
    d, n_r, n_c = 32, 400, 300
    U = (scale * rng.standard_normal((n_r, d))).astype(np.float32)
    V = rng.standard_normal((n_c, d)).astype(np.float32)
    G = (rng.standard_normal((d, d)) / 6).astype(np.float32)
    l = rng.standard_normal(d).astype(np.float32)
    rows = rng.integers(0, n_r, n).astype(np.int32)
    cols = rng.integers(0, n_c, n).astype(np.int32)
    deg = rng.integers(0, 30, n_r).astype(np.float64)
    tab = K.upload_alias(deg, "cuda")
    dv = lambda a: torch.from_numpy(a).cuda()
    op = K.PreparedDecoderHinge(dv(U), dv(V), dv(rows), dv(cols), dv(G), dv(l), 0.1, alias=tab, seed=3, offset=77)
    op()
    negs = op.neg_rows.cpu().numpy()
    assert np.array_equal(negs, K.unigram_sample(tab, n, 3, 77).cpu().numpy())
    op()  # a second launch reuses the word / ticket the first one reset (checked below)
    L = np.diag(l.astype(np.float64))
    emb = [U.astype(np.float64), V.astype(np.float64)]
    pos = orc.batch_predict(emb, 0, 1, G.astype(np.float64), L, rows, cols)
    neg = orc.batch_predict(emb, 0, 1, G.astype(np.float64), L, negs, cols)
    assert rel_err(op.pos.cpu().numpy(), pos) <= 1e-5
    assert rel_err(op.neg.cpu().numpy(), neg) <= 1e-5
    want = orc.hinge_loss(pos, neg, 0.1)
    assert abs(float(op.loss[0]) - want) <= 1e-4 * abs(want)
    # the hand-off itself, on the device's own scores: the float64 sum within fp32 rounding,
    # the same bits on every launch
    own = orc.hinge_loss(op.pos.cpu().numpy().astype(np.float64), op.neg.cpu().numpy().astype(np.float64), 0.1)
    first = float(op.loss[0])
    assert abs(first - own) <= 1e-6 * abs(own)
    if n <= 255 * 32 and scale == 1:
        # the packed form: each block partial rounded to the nearest 2^-32 (decoder.hip), so the
        # sum of the fp32 block partials is met within 255·2^-33 absolute, without bias
        pos_d, neg_d = op.pos.cpu().numpy(), op.neg.cpu().numpy()
        parts = [np.float32(0)] * -(-n // 32)
        for b in range(len(parts)):
            t = np.maximum(neg_d[32 * b:32 * b + 32] - (pos_d[32 * b:32 * b + 32] - np.float32(0.1)), 0)
            parts[b] = np.float64(t.astype(np.float32).sum(dtype=np.float32))
        assert abs(first - sum(parts)) <= len(parts) * 2.0 ** -33 + 1e-6 * abs(own)
    for _ in range(2):
        op()
        assert float(op.loss[0]) == first
    # given negatives
    op2 = K.PreparedDecoderHinge(dv(U), dv(V), dv(rows), dv(cols), dv(G), dv(l), 0.1, neg_rows=dv(negs))
    op2()
    assert np.array_equal(op2.neg.cpu().numpy(), op.neg.cpu().numpy())


@pytest.mark.parametrize("d", [16, 32, 64, 40])
@pytest.mark.parametrize("n_rows,n_cols,density,out_chunk", [
    (150, 137, 0.03, 5),     # several relations per output chunk, empty rows
    (1000, 137, 0.03, 7),    # rows up to the 1024-thread workgroup
    (300, 137, 0.45, 4),     # long rows, split into segments
    (645, 645, 0.3, 3),      # ~125k nonzeros per relation
    (900, 50, 0.9, 2),       # 45 nonzeros per row: many segments per row
    (64, 880, 0.01, 23),     # widest column space that fits LDS at 64 rows, one output chunk
])
def test_spmm_staged(K, d, n_rows, n_cols, density, out_chunk):
    """LDS-staged SpMM against the float64 product: relations in permuted slabs, output
    chunks, split rows, a partial last column slice (d=40), an empty relation."""
    from decagon_amd.sparse import coo_to_csr, sparse_to_tuple, staged_layout

    rng = np.random.default_rng(d + n_rows + n_cols)
    nrel, total = 23, 30
    mats = [_rand_csr(rng, n_rows, n_cols, density, empty_rows=0.1) for _ in range(nrel)]
    mats[3] = sp.csr_matrix((n_rows, n_cols), dtype=np.float32)  # an empty relation
    slabs = rng.choice(total, size=nrel, replace=False).astype(np.int32)
    lay = staged_layout([coo_to_csr(*sparse_to_tuple(x)) for x in mats], K.staged_block)
    dev = K.StagedDevice.upload(lay, "cuda")
    X = rng.standard_normal((total, n_cols, d)).astype(np.float32)
    n_out = -(-nrel // out_chunk)
    out = torch.zeros((n_out, n_rows, d), device="cuda")
    spec = K.StagedSpec(dev, torch.from_numpy(slabs).cuda(), torch.from_numpy(X).cuda(), out, out_chunk, d,
                        total * n_cols, slab_max=int(slabs.max()))
    K.PreparedStaged([spec], d)()
    want = np.zeros((n_out, n_rows, d))
    for k, x in enumerate(mats):
        want[k // out_chunk] += x @ X[slabs[k]].astype(np.float64)
    assert rel_err(out.cpu().numpy(), want) <= 1e-5
    # bitwise reproducible
    out2 = torch.zeros_like(out)
    spec.out = out2
    K.PreparedStaged([spec], d)()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("d", [32, 64, 40])
@pytest.mark.parametrize("n_rows,n_cols,density,out_chunk", [
    (150, 137, 0.03, 5),     # a partial last 16-row projection tile, empty rows
    (300, 137, 0.45, 4),     # long rows, split into segments
    (645, 645, 0.3, 3),      # config P's shape: 41 tiles over 16 waves
    (64, 880, 0.01, 23),     # 55 tiles (up to 4 per wave)
])
def test_spmm_staged_projected(K, d, n_rows, n_cols, density, out_chunk):
    """dg_spmm_staged_proj_f32: relation k's operand H·W[slab(k)] made on the MFMA inside the
    kernel, against the float64 Σ_k A_k·(H·W_slab(k)); H with a padded leading dimension."""
    from decagon_amd.sparse import coo_to_csr, sparse_to_tuple, staged_layout

    rng = np.random.default_rng(7 * d + n_rows + n_cols)
    nrel, total = 23, 30
    mats = [_rand_csr(rng, n_rows, n_cols, density, empty_rows=0.1) for _ in range(nrel)]
    mats[5] = sp.csr_matrix((n_rows, n_cols), dtype=np.float32)
    slabs = rng.choice(total, size=nrel, replace=False).astype(np.int32)
    lay = staged_layout([coo_to_csr(*sparse_to_tuple(x)) for x in mats], K.staged_block)
    dev = K.StagedDevice.upload(lay, "cuda")
    Hp = rng.standard_normal((n_cols, 68)).astype(np.float32)   # leading dimension 68
    W = rng.standard_normal((total, 64, d)).astype(np.float32)
    h = torch.from_numpy(Hp).cuda()[:, :64]
    n_out = -(-nrel // out_chunk)
    out = torch.zeros((n_out, n_rows, d), device="cuda")
    proj = (h, torch.from_numpy(W).cuda())
    spec = K.StagedSpec(dev, torch.from_numpy(slabs).cuda(), None, out, out_chunk, d, 0,
                        slab_max=int(slabs.max()), proj=proj)
    K.PreparedStaged([spec], d)()
    H = Hp[:, :64].astype(np.float64)
    want = np.zeros((n_out, n_rows, d))
    for k, x in enumerate(mats):
        want[k // out_chunk] += x @ (H @ W[slabs[k]].astype(np.float64))
    assert rel_err(out.cpu().numpy(), want) <= 1e-5
    out2 = torch.zeros_like(out)
    spec.out = out2
    K.PreparedStaged([spec], d)()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("proj", [False, True])
@pytest.mark.parametrize("d", [32, 64])
@pytest.mark.parametrize("n_rows,n_cols,density", [(150, 137, 0.03), (645, 645, 0.05)])
def test_spmm_staged_var_chunks(K, proj, d, n_rows, n_cols, density):
    """Variable output chunks (dg_staged_group.chunk_start, ABI 38): chunk c sums relations
    [cs[c], cs[c+1]) — single-relation chunks, a long chunk, the empty relation alone — and a
    table of fixed runs is bitwise the fixed out_chunk launch."""
    from decagon_amd.sparse import coo_to_csr, sparse_to_tuple, staged_layout

    rng = np.random.default_rng(11 * d + n_rows + proj)
    nrel, total = 23, 30
    mats = [_rand_csr(rng, n_rows, n_cols, density, empty_rows=0.1) for _ in range(nrel)]
    mats[4] = sp.csr_matrix((n_rows, n_cols), dtype=np.float32)
    slabs = rng.choice(total, size=nrel, replace=False).astype(np.int32)
    lay = staged_layout([coo_to_csr(*sparse_to_tuple(x)) for x in mats], K.staged_block)
    dev = K.StagedDevice.upload(lay, "cuda")
    X = rng.standard_normal((total, n_cols, d)).astype(np.float32)
    Hp = rng.standard_normal((n_cols, 64)).astype(np.float32)
    W = rng.standard_normal((total, 64, d)).astype(np.float32)
    if proj:
        ops = [Hp.astype(np.float64) @ W[s].astype(np.float64) for s in range(total)]
    else:
        ops = [X[s].astype(np.float64) for s in range(total)]

    def run(out_chunk, cs):
        n_out = len(cs) - 1 if cs is not None else -(-nrel // out_chunk)
        out = torch.zeros((n_out, n_rows, d), device="cuda")
        kw = dict(slab_max=int(slabs.max()), chunk_start=None if cs is None else np.asarray(cs, np.int32))
        if proj:
            kw["proj"] = (torch.from_numpy(Hp).cuda(), torch.from_numpy(W).cuda())
            spec = K.StagedSpec(dev, torch.from_numpy(slabs).cuda(), None, out, out_chunk, d, 0, **kw)
        else:
            spec = K.StagedSpec(dev, torch.from_numpy(slabs).cuda(), torch.from_numpy(X).cuda(), out, out_chunk, d,
                                total * n_cols, **kw)
        K.PreparedStaged([spec], d)()
        torch.cuda.synchronize()
        return out

    cs = [0, 1, 4, 5, 6, 19, 21, 23]
    out = run(13, cs)
    want = np.zeros((len(cs) - 1, n_rows, d))
    for c in range(len(cs) - 1):
        for k in range(cs[c], cs[c + 1]):
            want[c] += mats[k] @ ops[slabs[k]]
    assert rel_err(out.cpu().numpy(), want) <= 1e-5
    assert torch.equal(out, run(13, cs))
    # fixed runs of 5 as a table: bitwise the fixed launch
    assert torch.equal(run(5, list(range(0, nrel, 5)) + [nrel]), run(5, None))
