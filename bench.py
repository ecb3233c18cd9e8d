"""Benchmark: GCN-layer edges/s + achieved HBM GB/s of the Decagon forward on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config S|P]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

A step is one full forward of the hot path over one batch: GCN layer 1 + layer 2 over every
relation (SpMM, projection, add_n, L2-norm, ReLU) + the DEDICOM decoder on B=512 positive
and 512 device-sampled negative pairs + the hinge loss.  Edges per step = 2 × Σ nnz (each
layer visits every stored nonzero of every normalised Â_r, self-loops and transposed copies
included — SURVEY §8d).  Inputs are resident in HBM before timing (uploaded once).

Workloads (BASELINE.json configs):
  S (default, configs[1]): main.py's 5-relation / 10-matrix synthetic, the exact
     reference-normalised adjacencies (tests/golden/synthetic_S.npz), d = 64/32, fp32.
     At N GPUs the graph holds N relation sets, one per GPU (weak scaling); each layer
     all-reduces the per-(i,j) pre-normalisation sums over RCCL.
  P (configs[2]/[3]): polypharmacy-shaped 19,085 + 645 nodes, 964 side effects ⇒ 1,932
     drug-drug matrices, ≈23 M nnz; at N GPUs the relations are LPT-sharded (strong scaling).

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "GCN-layer edges/sec + achieved HBM GB/s, 5-relation synthetic, 1/2/4/8 GPU"
JSON_OUT = sys.stdout
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md §Chip-level parameters)
H1, H2, BATCH, MARGIN = 64, 32, 512, 0.1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=["S", "P", "D"], default="S",
                    help="S / P: the GCN forward step (metric: edges/s); D: config 5, bf16 DEDICOM "
                         "scoring of every drug-drug slot's batch (metric: scored pairs/s)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=200)
    ap.add_argument("--graph-steps", type=int, default=10,
                    help="steps captured back to back in one hipGraph (must divide --steps and --warmup)")
    ap.add_argument("--target-waves", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--train", action="store_true",
                    help="S / P: time the TRAINING step (forward + hinge-cost backward + Adam on every "
                         "variable, optimizer.py:108-114) instead of the forward step; one GPU")
    ap.add_argument("--dropout", type=float, default=0.0,
                    help="--train: dropout rate of both GCN layers (main.py trains at FLAGS.dropout = 0.1)")
    ap.add_argument("--force-shard", action="store_true",
                    help="run the relation-sharded (N > 1) plan and its collectives even at N = 1 "
                         "(launch under torchrun: a rehearsal of the multi-GPU step on one GPU)")
    ap.add_argument("--collectives", choices=["graph", "eager"], default="graph",
                    help="N > 1 over RCCL: capture the whole step, all-reduces included, in one "
                         "hipGraph (graph), or replay the compute phases between eager collectives")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL; "
                    "gloo only to exercise the multi-rank path on a single-GPU box)")
    return ap.parse_args()


def glorot_stack(rng, k, d_in, d_out):
    r = np.sqrt(6.0 / (d_in + d_out))
    return rng.uniform(-r, r, size=(k, d_in, d_out)).astype(np.float32)


def build_workload(args, rank, world, sharded):
    import torch

    from decagon_amd import synthetic
    from decagon_amd.sharding import RelationShard, torch_allreduce

    allreduce = torch_allreduce() if sharded else None
    if args.config == "S":
        base = synthetic.load_S()
        graph = synthetic.replicate_sets(base, world) if world > 1 else base
        shard = RelationShard.blocks(base.edge_types, rank, world, allreduce) if sharded else None
        scaling = "weak"
        workload = ("S: main.py 5-relation / 10-matrix synthetic (reference-normalised, 105,974 nnz "
                    "per relation set), 2 GCN layers d=64/32 + DEDICOM decoder B=512+512")
    else:
        graph = synthetic.make_P(seed=0)
        shard = None
        if sharded:
            nnz = {et: [len(c[1]) for c in rels] for et, rels in graph.adj.items()}
            shard = RelationShard.lpt(graph.edge_types, nnz, rank, world, allreduce)
        scaling = "strong"
        workload = ("P: polypharmacy-shaped 19,085 proteins + 645 drugs, 964 side effects "
                    "(1,932 drug-drug matrices), 2 GCN layers d=64/32 + DEDICOM decoder B=512+512")
    return graph, shard, scaling, workload


def make_plan(args, graph, shard, device, keep_sums=False, dropout=None):
    import torch

    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights

    csr = graph.csr()
    if shard is not None:  # only local relations need host CSR / upload
        csr = {et: [c if k in set(shard.local[et]) else None for k, c in enumerate(v)] for et, v in csr.items()}
    dg = DeviceGraph(graph.edge_types, csr, device, None if shard is None else shard.local,
                     chunk=args.chunk, target_waves=args.target_waves)
    rng = np.random.default_rng(1234)
    n = graph.n_nodes
    w1 = LayerWeights({et: torch.from_numpy(glorot_stack(rng, K, n[et[1]], H1)).to(device)
                       for et, K in graph.edge_types.items()})
    w2 = LayerWeights({et: torch.from_numpy(glorot_stack(rng, K, H1, H2)).to(device)
                       for et, K in graph.edge_types.items()})
    plan = ForwardPlan(dg, {j: None for j in n}, w1, w2, H1, H2,
                       allreduce=None if shard is None else shard.allreduce, keep_sums=keep_sums,
                       dropout=dropout)
    plan.w1, plan.w2 = w1, w2
    return plan, dg


class Decoder:
    """DEDICOM scoring of B positive + B sampled negative pairs of one drug-drug relation,
    then the hinge loss — one dg_decoder_hinge_f32 launch (sampler + scores + loss)."""

    def __init__(self, graph, plan, device, rank):
        import torch

        from decagon_amd import kernels

        self.k = kernels
        et = (1, 1)
        coords = graph.adj[et][0][0]
        rng = np.random.default_rng(99 + rank)
        pick = coords[rng.choice(len(coords), BATCH, replace=False)]
        self.rows = torch.from_numpy(pick[:, 0].astype(np.int32)).to(device)
        self.cols = torch.from_numpy(pick[:, 1].astype(np.int32)).to(device)
        deg = graph.degrees[1][0]
        self.alias = kernels.upload_alias(deg, device)
        self.R = torch.from_numpy(glorot_stack(rng, 1, H2, H2)[0]).to(device)
        self.l = torch.from_numpy(glorot_stack(rng, 1, H2, 1).reshape(-1)).to(device)
        self.E = plan.embeddings[1]
        self.fused = kernels.PreparedDecoderHinge(self.E, self.E, self.rows, self.cols, self.R, self.l,
                                                  MARGIN, alias=self.alias, seed=7)

    def __call__(self):
        self.fused()


def time_kernel(fn, reps, stream):
    """Average device duration of one launch of `fn`, from HIP events on the stream the
    kernel runs on, over `reps` back-to-back launches captured in one hipGraph."""
    import torch

    with torch.cuda.stream(stream):
        fn()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(reps):
                fn()
        g.replay()
        stream.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(5):
            t0.record(stream)
            g.replay()
            t1.record(stream)
            t1.synchronize()
            ms = t0.elapsed_time(t1) / reps
            best = ms if best is None else min(best, ms)
    return best


KERNEL_NAMES = {"PreparedFused": "gcn_fused_kernel<{lp}>", "PreparedSpmm": "spmm_groups_kernel<{lp}>",
                "PreparedStaged": "spmm_staged_kernel"}


PreparedStagedT = type(None)  # set in main() once decagon_amd is imported


def pmc_traffic(config, launches, d):
    """HBM bytes per launch of `launches` from the newest committed PMC pass
    (profiles/rNN_traffic.json, written by scripts/prof_summary.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE runs of this bench): FETCH_SIZE × 2 (gfx950 counts half of a
    wide streaming read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KiB → bytes.  Returns
    (bytes or None, source, the profiled kernels' mean duration in ms)."""
    files = sorted(ROOT.glob("profiles/r*_traffic.json"))
    if not files:
        return None, None, None
    src = str(files[-1].relative_to(ROOT))
    rec = json.load(open(files[-1])).get(config, {})
    lp = 1 << max(0, (max(1, d // 4) - 1).bit_length())
    tot, us = 0.0, 0.0
    for l in launches:
        pat = KERNEL_NAMES.get(type(l).__name__, "?").format(lp=lp)
        hit = [v for k, v in rec.items() if k.replace("void ", "").startswith(pat)]
        if not hit or "fetch_size_kib" not in hit[0] or "write_size_kib" not in hit[0]:
            return None, src, None
        e = hit[0]
        if isinstance(l, PreparedStagedT) and e.get("by_grid"):
            # both layers launch this kernel; layer 1 (d=64: 4 column slices) has the largest grid
            e = e["by_grid"][max(e["by_grid"], key=int)]
            if "fetch_size_kib" not in e or "write_size_kib" not in e:
                return None, src, None
        tot += (2.0 * e["fetch_size_kib"] + e["write_size_kib"]) * 1024.0
        us += hit[0].get("avg_us", 0.0)
    return tot, src, us * 1e-3


def cpu_baseline(graph, seconds):
    """The oracle's scalar C restatement (fp32, one thread; oracle/gcn_ref.c) of the same
    two-layer forward in TF's op order, on a bounded number of repetitions."""
    import ctypes

    from oracle import cpu_forward

    lib = cpu_forward.load()
    fwd = cpu_forward.Forward(lib, graph, H1, H2)
    reps, t0 = 0, time.perf_counter()
    while True:
        fwd.run()
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or (reps >= 3 and el * (reps + 1) / reps > seconds * 1.5):
            break
    edges = 2 * graph.nnz * reps
    return {"value": edges / el, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"{reps} full 2-layer forwards of config {graph.name} ({graph.nnz} nnz/layer) in "
                      f"{el:.1f} s, oracle/gcn_ref.c fp32 scalar, 1 thread"}


BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: no sparsity)


def main_decoder(args):
    """Config 5 (BASELINE configs[4]): d = 256 bf16 embeddings / R / D_k, DEDICOM decoder on
    MFMA, every one of the 1,928 drug-drug relation slots scoring B = 512 positives and 512
    negatives drawn on the device from the degree^0.75 alias table, in one launch per step.
    One GPU; the 8-GPU form shards the slots (no collective but the scalar loss)."""
    import torch

    from decagon_amd import kernels

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    d, n_drugs, slots, B = 256, 645, 1928, BATCH
    rng = np.random.default_rng(5)
    bf = torch.bfloat16
    E = torch.from_numpy(rng.standard_normal((n_drugs, d)).astype(np.float32) / 4).to(bf).to(dev)
    R = torch.from_numpy(glorot_stack(rng, 1, d, d)[0]).to(bf).to(dev)
    Dk = torch.from_numpy(glorot_stack(rng, slots, d, 1).reshape(slots, d)).to(bf).to(dev)
    n = slots * B
    # positives: synthetic drug pairs of the P shape (uniform ids); negatives: device draws
    rows = torch.empty(2 * n, dtype=torch.int32, device=dev)
    rows[:n] = torch.from_numpy(rng.integers(0, n_drugs, n).astype(np.int32)).to(dev)
    cols1 = torch.from_numpy(rng.integers(0, n_drugs, n).astype(np.int32)).to(dev)
    cols = torch.cat([cols1, cols1])
    rel1 = torch.arange(slots, dtype=torch.int32, device=dev).repeat_interleave(B)
    rel = torch.cat([rel1, rel1])
    alias = kernels.upload_alias(rng.integers(1, 200, n_drugs).astype(np.float64), dev)
    out = torch.empty(2 * n, dtype=torch.float32, device=dev)
    neg_rows = rows[n:]

    def sample():
        kernels.unigram_sample(alias, n, 11, 0, out=neg_rows)

    def score():
        kernels.decoder_score_bf16(E, E, rows, cols, R, Dk, rel, out=out)

    def step():
        sample()
        score()

    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        step()
        stream.synchronize()
        if args.no_graph:  # eager launches (PMC passes attribute counters per dispatch)
            for _ in range(args.warmup):
                step()
            stream.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            stream.synchronize()
            el = time.perf_counter() - t0
        else:
            G = args.graph_steps if args.steps % max(1, args.graph_steps) == 0 and args.warmup % max(1, args.graph_steps) == 0 else 1
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg, stream=stream):
                for _ in range(G):
                    step()
            for _ in range(args.warmup // G):
                cg.replay()
            stream.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps // G):
                cg.replay()
            stream.synchronize()
            el = time.perf_counter() - t0
    k_ms = time_kernel(score, args.kernel_reps, stream)
    flop_pair = 2 * d * d + 4 * d
    tflops = 2 * n * flop_pair / (k_ms * 1e-3) / 1e12
    rec = {
        "metric": "DEDICOM scored pairs/sec (config 5: d=256 bf16, all 1,928 drug-drug slots)",
        "value": 2 * n * args.steps / el,
        "unit": "pairs/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 (fp32 accumulation)",
        "data": "synthetic drug pairs (uniform ids, 645 drugs), device-sampled negatives, random bf16 R / D_k",
        "config": {"workload": f"config 5: {slots} relation slots x ({B} pos + {B} neg) pairs, d={d}, "
                               "DEDICOM uT.D_k.R.D_k.v on v_mfma_f32_32x32x16_bf16",
                   "pairs_per_step": 2 * n, "hipgraph": not args.no_graph},
        "roofline": {"bound": "mfma", "achieved": tflops, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tflops / BF16_PEAK_TFLOPS, "traffic": None,
                     "kernel": "decoder_bf16_kernel<256, true>", "kernel_ms": k_ms,
                     "algorithmic_flops": 2 * n * flop_pair},
        "cpu_baseline": None,
    }
    print(json.dumps(rec), file=JSON_OUT, flush=True)


def main_train(args):
    """The training step of DecagonOptimizer.opt_op (optimizer.py:108-114) on one GPU: the
    forward in flat mode (pre-normalisation sums kept), the DEDICOM decoder + hinge on B
    positives / B device-sampled negatives, the backward through the decoder, both GCN
    layers (every relation's W1/W2 gradient) and ApplyAdam on every variable — one hipGraph
    per step group, Adam's beta powers advanced on the device."""
    import torch

    from decagon_amd import kernels, train

    torch.cuda.set_device(0)
    device = torch.device("cuda", 0)
    graph, shard, scaling, workload = build_workload(args, 0, 1, False)
    drop = None
    if args.dropout > 0:
        drop = (1.0 - args.dropout, torch.tensor([20180701, 0], dtype=torch.int64, device=device))
        workload += f"; dropout {args.dropout}"
    plan, dg = make_plan(args, graph, None, device, keep_sums=True, dropout=drop)
    dec = Decoder(graph, plan, device, 0)
    tp = train.TrainPlan(plan, plan.w1, plan.w2, {j: None for j in graph.n_nodes})
    dR = torch.zeros_like(dec.R)
    dl = torch.zeros_like(dec.l)
    f = dec.fused
    dgrad = kernels.PreparedDecoderGrad(dec.E, dec.E, dec.rows, dec.cols, f.neg_rows, f.pos, f.neg, dec.R, dec.l,
                                        MARGIN, dG=dR.view(-1), dl=dl)

    def decoder_grad(dE):
        dgrad()
        kernels.scatter_rows(dgrad.row_idx, dgrad.grad_rows, dE[1])
        kernels.scatter_rows(dec.cols, dgrad.grad_cols, dE[1])

    ets = list(graph.edge_types)
    params = [plan.w1.stacks[et] for et in ets] + [plan.w2.stacks[et] for et in ets] + [dec.R, dec.l]
    grads = [tp.gW1[et] for et in ets] + [tp.gW2[et] for et in ets] + [dR, dl]
    adam = train.AdamState(params, lr=0.001)
    prep = adam.prepared(grads)

    def step():
        plan.run()
        dec()
        tp.backward(decoder_grad)
        adam.apply(prep)

    stream = torch.cuda.Stream(device)
    G = args.graph_steps if args.steps % max(1, args.graph_steps) == 0 and args.warmup % max(1, args.graph_steps) == 0 else 1
    with torch.cuda.stream(stream):
        step()
        stream.synchronize()
        loss0 = float(f.loss[0])
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg, stream=stream):
            for _ in range(G):
                step()
        for _ in range(args.warmup // G):
            cg.replay()
        stream.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps // G):
            cg.replay()
        stream.synchronize()
        el = time.perf_counter() - t0
        loss1 = float(f.loss[0])
    params_n = int(sum(p.numel() for p in params))
    rec = {
        "metric": "GCN training-step edges/sec (forward + backward + Adam), " + ("5-relation synthetic" if args.config == "S" else "polypharmacy-shaped"),
        "value": 2 * dg.total_nnz * args.steps / el,
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (as the forward bench), random glorot weights, device-sampled negatives",
        "config": {"workload": workload + "; training step: backward + TF-Adam on %d parameters" % params_n,
                   "nnz_per_layer_total": dg.total_nnz, "parallelism": "1 GPU", "hipgraph": True,
                   "steps_per_graph": G},
        "loss_first_step": loss0,
        "loss_last_step": loss1,
        "roofline": None,
        "cpu_baseline": None,
    }
    print(json.dumps(rec), file=JSON_OUT, flush=True)


def main():
    args = parse()
    # stdout carries exactly one JSON line: libraries that print to fd 1 (RCCL prints its
    # version banner at communicator init) are sent to stderr instead
    global JSON_OUT
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.config == "D":
        return main_decoder(args)
    if args.train:
        return main_train(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torchrun --nproc-per-node N")
    dev_index = local_rank % max(1, torch.cuda.device_count())  # ranks share a GPU only in a gloo rehearsal
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    sharded = world > 1 or args.force_shard
    if sharded:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)

    graph, shard, scaling, workload = build_workload(args, rank, world, sharded)
    plan, dg = make_plan(args, graph, shard, device)
    dec = Decoder(graph, plan, device, rank)

    def step():
        plan.run()
        dec()

    stream = torch.cuda.Stream(device)
    use_graph = not args.no_graph
    # One GPU, or N > 1 over RCCL (--collectives graph): G complete steps per hipGraph replay,
    # the per-layer all-reduces captured with the compute (each replay runs exactly G steps, so
    # the timed region still runs exactly --steps steps; G = 1 when it does not divide both
    # counts).  Otherwise (gloo, or --collectives eager): the compute between the two per-layer
    # all-reduces is captured (one hipGraph per phase) and the collectives run eagerly between
    # the replays.
    full = use_graph and (not sharded or (args.backend == "nccl" and args.collectives == "graph"))
    G = args.graph_steps if full else 1
    if G < 1 or args.steps % G or args.warmup % G:
        G = 1
    mode = "eager"
    with torch.cuda.stream(stream):
        step()
        stream.synchronize()
        if sharded:
            dist.barrier()
        run = step
        if full:
            try:
                cg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(cg, stream=stream):
                    for _ in range(G):
                        step()
                run = cg.replay
                mode = "one hipGraph per %d steps%s" % (G, ", all-reduces captured" if sharded else "")
            except RuntimeError as e:  # a collective that refuses capture: per-phase graphs
                if not sharded:
                    raise
                print(f"bench: capturing the all-reduces failed ({e}); eager collectives", file=sys.stderr)
                torch.cuda.synchronize()
                full, G = False, 1
        if not full and use_graph:
            phases = plan.phases()
            last = max(i for i, (kind, _) in enumerate(phases) if kind == "compute")
            seq = []
            for i, (kind, fn) in enumerate(phases):
                if kind == "exchange":
                    seq.append(fn)
                    continue
                body = (lambda fn=fn: (fn(), dec())) if i == last else fn
                body()
                stream.synchronize()
                gph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gph, stream=stream):
                    body()
                seq.append(gph.replay)

            def run():
                for f in seq:
                    f()
            mode = "hipGraph per compute phase, eager collectives"
        for _ in range(args.warmup // G):
            run()
        stream.synchronize()
        if sharded:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps // G):
            run()
        stream.synchronize()
        torch.cuda.synchronize()
        if sharded:
            dist.barrier()
        el = time.perf_counter() - t0

    local_edges = 2 * dg.total_nnz
    el_max = el
    tot_edges = local_edges
    if sharded:
        t = torch.tensor([el, float(local_edges)], dtype=torch.float64, device=device)
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        el_max, tot_edges = float(tm[0]), float(t[1])
    value = tot_edges * args.steps / el_max

    # the roofline covers the dominant kernel: the longest layer-1 SpMM launch (config S: the
    # one fused launch; config P: the staged drug x drug SpMM), its algorithmic bytes over its
    # own duration; the whole layer-1 SpMM (launches as the forward runs them — concurrent
    # streams at P) is reported beside it
    l1, l2 = plan.spmm_launches
    per = [(time_kernel(lambda l=l: l(), args.kernel_reps, stream), i) for i, l in enumerate(l1)]
    k_ms, di = max(per)
    dom = l1[di]
    k_bytes = plan.launch_bytes(dom, 1)
    achieved = k_bytes / (k_ms * 1e-3) / 1e9
    l1_ms = time_kernel(plan._layer1.run_spmm, args.kernel_reps, stream)
    l1_bytes = plan.layer_bytes(1)
    k2_ms = time_kernel(plan._layer2.run_spmm, args.kernel_reps, stream)
    global PreparedStagedT
    from decagon_amd.kernels import PreparedStaged
    PreparedStagedT = PreparedStaged
    traffic, traffic_src, traffic_ms = pmc_traffic(args.config, [dom], H1)
    lp = 1 << max(0, (max(1, H1 // 4) - 1).bit_length())

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(graph, args.cpu_seconds)
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference-normalised adjacencies (config S) / seeded generator (P); "
                    "random glorot weights",
            "config": {"workload": workload, "nnz_per_layer_total": int(tot_edges // 2),
                       "parallelism": (f"relation-sharded x{world}, "
                                       f"{'RCCL' if args.backend == 'nccl' else args.backend} all-reduce per layer"
                                       if sharded else "1 GPU"),
                       "hipgraph": use_graph, "launch": mode, "steps_per_graph": G},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "traffic_profiled_kernel_ms": traffic_ms,
                         "kernel": KERNEL_NAMES.get(type(dom).__name__, "?").format(lp=lp) + " (layer 1)",
                         "kernel_ms": k_ms,
                         "algorithmic_bytes": k_bytes},
            "spmm_layer1": {"launches": [type(x).__name__ for x in l1], "ms": l1_ms,
                            "algorithmic_bytes": l1_bytes, "GB_s": l1_bytes / (l1_ms * 1e-3) / 1e9,
                            "frac": l1_bytes / (l1_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                            "edges_per_s": dg.total_nnz / (l1_ms * 1e-3)},
            "spmm_layer2_ms": k2_ms,
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), file=JSON_OUT, flush=True)
    if sharded:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
