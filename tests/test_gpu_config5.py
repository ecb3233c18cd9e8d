"""GPU: config 5 (BASELINE configs[4]) on the benched workload — every one of the 1,928
drug-drug relation slots scoring 512 positives and 512 device-sampled negatives with the
d = 256 bf16 DEDICOM decoder, then the hinge loss (decagon_amd.scorer.SlotScorer, as
bench.py runs it) — against a float64 restatement of the reference's scores
(decagon/deep/optimizer.py:51-57, 63-85 with G = R, L = D_k: model.py:130-134) and hinge
(optimizer.py:116-120) over EVERY pair, with the same bf16 operand rounding as the kernel
(inputs rounded to bf16; D_k∘v rounded to bf16 as the MFMA's operand; fp32 accumulation).

The negatives are read back from the device: each slot's are exactly the restated alias draws
of THAT slot's degree^0.75 table (fixed_unigram_candidate_sampler over degrees[i][k],
optimizer.py:38-47), their pooled counts match the slots' distributions, and they do not
depend on how the slots are sharded: the 2-rank slot-sharded run (gloo on the one GPU, loss
all-reduced) at 2 and 8 ranks reproduces the one-rank draws and scores bit for bit.
"""
import numpy as np
import pytest

from conftest import alias_draws, rel_err, run_ranks

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _scorer(device, slots=None, allreduce=None, fused=True):
    from decagon_amd import kernels, synthetic
    from decagon_amd.scorer import SlotScorer

    c5 = synthetic.make_config5()
    bf = torch.bfloat16
    E = torch.from_numpy(c5.E).to(bf).to(device)
    sc = SlotScorer(E, E, torch.from_numpy(c5.R).to(bf).to(device), torch.from_numpy(c5.D).to(bf).to(device),
                    torch.from_numpy(c5.pos_rows).to(device), torch.from_numpy(c5.pos_cols).to(device),
                    kernels.upload_alias(c5.degrees, device), c5.batch, 0.1, seed=11, slots=slots,
                    allreduce=allreduce, fused=fused)
    return c5, sc


def _restated_scores(c5, rows, cols):
    """float64 (u∘D_k)ᵀ·R·(D_k∘v) on the bf16-rounded inputs, D_k∘v rounded to bf16 (the MFMA
    operand of the column-shared paired kernel); pairs slot-major, B per slot."""
    bf = torch.bfloat16
    E = torch.from_numpy(c5.E).to(bf).float().numpy()
    R = torch.from_numpy(c5.R).to(bf).double().numpy()
    D = torch.from_numpy(c5.D).to(bf).float().numpy()
    rel = np.repeat(np.arange(D.shape[0]), c5.batch)
    out = np.empty(len(rows))
    step = 1 << 16
    for s in range(0, len(rows), step):
        r, c, k = rows[s:s + step], cols[s:s + step], rel[s:s + step]
        a = D[k].astype(np.float64) * E[r].astype(np.float64)
        b = torch.from_numpy(D[k] * E[c]).to(bf).double().numpy()          # the MFMA operand
        out[s:s + step] = np.einsum("pn,pn->p", a, b @ R.T)
    return out


def test_config5_full_workload_matches_restatement():
    from oracle import decagon_oracle as orc

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    c5, sc = _scorer(torch.device("cuda"))
    sc()
    torch.cuda.synchronize()
    n = sc.n
    slots = c5.D.shape[0]
    assert n == slots * c5.batch == 1928 * 512
    neg_rows = sc.neg_rows.cpu().numpy()
    pos, neg, loss = sc.pos.cpu().numpy(), sc.neg.cpu().numpy(), float(sc.loss[0])
    # device-sampled negatives: slot k's are the draws of slot k's own table, bit for bit
    from decagon_amd.sampling import alias_table

    B = c5.batch
    assert neg_rows.min() >= 0 and neg_rows.max() < c5.E.shape[0]
    for k in range(0, slots, 97):
        want = alias_draws(alias_table(c5.degrees[k]), 11, k * B + np.arange(B))
        assert np.array_equal(neg_rows[k * B:(k + 1) * B], want), k
    # ... and their pooled counts follow the slots' degree^0.75 distributions
    exp = sum(orc.unigram_distribution(c5.degrees[k]) * B for k in range(slots))
    obs = np.bincount(neg_rows, minlength=len(exp))
    assert np.all(np.abs(obs - exp) <= 6 * np.sqrt(exp) + 1)
    want_pos = _restated_scores(c5, c5.pos_rows, c5.pos_cols)
    want_neg = _restated_scores(c5, neg_rows, c5.pos_cols)
    assert rel_err(pos, want_pos) <= 1e-4
    assert rel_err(neg, want_neg) <= 1e-4
    # SURVEY §8c's elementwise form too: |y − y_ref| <= 1e-4·|y_ref| + 1e-6·max|y_ref| for every pair
    for got_, want_ in ((pos, want_pos), (neg, want_neg)):
        tol = 1e-4 * np.abs(want_) + 1e-6 * np.max(np.abs(want_))
        assert np.mean(np.abs(got_ - want_) <= tol) >= 0.999
    want_loss = orc.hinge_loss(want_pos, want_neg, 0.1)
    assert abs(loss - want_loss) <= 1e-4 * abs(want_loss)
    # the loss kernel itself, on the device's own scores (float64 sum): fp32-accumulation tight
    own = orc.hinge_loss(pos.astype(np.float64), neg.astype(np.float64), 0.1)
    assert abs(loss - own) <= 1e-5 * abs(own)


def _rank(rank, world):
    from decagon_amd.sharding import slot_range, torch_allreduce

    s0, s1 = slot_range(1928, rank, world)
    _, sc = _scorer(torch.device("cuda", 0), (s0, s1), torch_allreduce())
    sc()
    torch.cuda.synchronize()
    return s0, s1, sc.neg_rows.cpu().numpy(), sc.out.cpu().numpy(), float(sc.loss[0])


@pytest.mark.parametrize("world", [2, 8])
def test_config5_slot_sharded_ranks_equal_one_rank(world):
    """north_star configs[4] at 8 GPUs: the 1,928 slots dealt in contiguous blocks over `world`
    gloo ranks (sharing the one GPU), each rank's draws and scores bit for bit the one-rank
    run's, the blocks covering every slot once, the loss all-reduced to the one-rank sum."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    c5, sc = _scorer(torch.device("cuda"))
    sc()
    torch.cuda.synchronize()
    B = c5.batch
    full_neg, full_pos, full_negs = sc.neg_rows.cpu().numpy(), sc.pos.cpu().numpy(), sc.neg.cpu().numpy()
    full_loss = float(sc.loss[0])
    got = list(run_ranks(_rank, world).values())
    assert sorted((s0, s1) for s0, s1, *_ in got) == [(a, b) for a, b in zip(
        sorted(x[0] for x in got), sorted(x[0] for x in got)[1:] + [1928])]  # contiguous, no gap
    assert min(x[0] for x in got) == 0 and max(x[1] for x in got) == 1928
    for s0, s1, negr, out, loss in got:
        m = (s1 - s0) * B
        assert np.array_equal(negr, full_neg[s0 * B:s1 * B])
        assert np.array_equal(out[:m], full_pos[s0 * B:s1 * B])
        assert np.array_equal(out[m:], full_negs[s0 * B:s1 * B])
        assert abs(loss - full_loss) <= 1e-5 * abs(full_loss)  # all-reduced per-rank sums


@pytest.mark.parametrize("slots", [None, (5, 9), (1927, 1928)])
def test_config5_one_launch_equals_three(slots):
    """dg_slot_score_hinge_bf16 (sampler + scores + hinge in one launch, the benched step) against
    the three-launch form (dg_unigram_sample_slots, dg_decoder_score_bf16_paired,
    dg_hinge_loss_ws_f32): the same draws and the same score bits; the loss is summed in another
    fixed order (fp32 rounding); the fused loss is the same on every launch; slot sub-ranges
    (a rank's share) included."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    _, one = _scorer(dev, slots)
    _, three = _scorer(dev, slots, fused=False)
    one()
    three()
    torch.cuda.synchronize()
    assert torch.equal(one.neg_rows, three.neg_rows)
    assert torch.equal(one.out, three.out)
    l1, l3 = float(one.loss[0]), float(three.loss[0])
    assert abs(l1 - l3) <= 1e-5 * abs(l3)
    for _ in range(3):  # (a wrong sum that came and went once showed up in ≈ 2 % of tiles per launch)
        one()
        torch.cuda.synchronize()
        assert float(one.loss[0]) == l1
        assert torch.equal(one.out, three.out)
