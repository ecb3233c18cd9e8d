"""Benchmark: GCN-layer edges/s + achieved HBM GB/s of the Decagon forward on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config S|P|D] [--train]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

A step is one full forward of the hot path over one batch: GCN layer 1 + layer 2 over every
relation (SpMM, projection, add_n, L2-norm, ReLU) + the DEDICOM decoder on B=512 positive
and 512 device-sampled negative pairs + the hinge loss.  Edges per step = 2 × Σ nnz (each
layer visits every stored nonzero of every normalised Â_r, self-loops and transposed copies
included — SURVEY §8d).  Inputs are resident in HBM before timing (uploaded once).

Workloads (BASELINE.json configs):
  S (default, configs[1]): main.py's 5-relation / 10-matrix synthetic, the exact
     reference-normalised adjacencies (decagon_amd/data/synthetic_S_adj.npz), d = 64/32,
     fp32.  At N GPUs the graph holds N relation sets, one per GPU (weak scaling); every node
     type is row-split — each rank finishes its row block over all N sets in the fused kernel
     and the blocks are all-gathered over RCCL (two all-gathers per step, no all-reduce).
  P (configs[2]/[3]): polypharmacy-shaped 19,085 + 645 nodes, 964 side effects ⇒ 1,932
     drug-drug matrices, ≈23 M nnz; at N GPUs the drug×drug relations are LPT-sharded and the
     protein rows row-split (strong scaling, sharding.py).
  D (configs[4]): d = 256 bf16 DEDICOM scoring of every drug-drug slot's 512 + 512 pairs.

The default line (config S) also carries a "P" block (config P's forward step, the staged
SpMM's roofline, its CPU baseline) and a "D" block (config 5's scorer), at every N, so the
driver's own runs record every north-star number; --no-extra drops them.

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from decagon_amd.tuning import knob, overrides  # noqa: E402

METRIC = "GCN-layer edges/sec + achieved HBM GB/s, 5-relation synthetic, 1/2/4/8 GPU"
JSON_OUT = sys.stdout
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md §Chip-level parameters)
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: no sparsity)
H1, H2, BATCH, MARGIN = 64, 32, 512, 0.1


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=["S", "P", "D"], default="S",
                    help="S / P: the GCN forward step (metric: edges/s); D: config 5, bf16 DEDICOM "
                         "scoring of every drug-drug slot's batch (metric: scored pairs/s)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline time budget per form")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="config S: omit the P / D blocks of the default line")
    ap.add_argument("--p-steps", type=int, default=100, help="timed steps of the P block")
    ap.add_argument("--d-steps", type=int, default=100, help="timed steps of the D block")
    ap.add_argument("--kernel-reps", type=int, default=200)
    # (each hipGraph replay boundary costs ≈ 5-20 µs of host launch + GPU ramp, measured by
    # scripts/steps_sweep.sh: config S 20.8 µs a step at 20 steps in graphs of 10, 19.2 at 200
    # in graphs of 50; so whole runs of up to 50 steps are one graph)
    ap.add_argument("--graph-steps", type=int, default=50,
                    help="steps captured back to back in one hipGraph (the largest divisor of "
                         "--steps not above it is used)")
    ap.add_argument("--target-waves", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--train", action="store_true",
                    help="S / P: time the TRAINING step (forward + hinge-cost backward + Adam on every "
                         "variable, optimizer.py:108-114) instead of the forward step")
    ap.add_argument("--dropout", type=float, default=0.0,
                    help="--train: dropout rate of both GCN layers (main.py trains at FLAGS.dropout = 0.1)")
    ap.add_argument("--force-shard", action="store_true",
                    help="run the sharded (N > 1) plan and its collectives even at N = 1 "
                         "(launch under torchrun: a rehearsal of the multi-GPU step on one GPU)")
    ap.add_argument("--collectives", choices=["graph", "eager"], default="graph",
                    help="N > 1 over RCCL: capture the whole step, collectives included, in one "
                         "hipGraph (graph), or replay the compute phases between eager collectives")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="config P / S: time each rank's share of an N-GPU sharded step on this one GPU, "
                         "collectives replaced by no-ops (prints per-rank step times and the bytes each "
                         "collective would move)")
    ap.add_argument("--simulate-rank", type=int, default=-1,
                    help="--simulate-world: time only this rank (default: every rank)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL; "
                    "gloo only to exercise the multi-rank path on a single-GPU box)")
    ap.add_argument("--exchange", choices=["rccl", "peer", "peer-kernel"], default="rccl",
                    help="N > 1 (and --simulate-world): the row-split blocks' all-gather over RCCL, or by peer "
                         "stores over xGMI (peer.py) fused into the finishing launches (peer) or as a "
                         "stand-alone launch (peer-kernel); the line's \"peer\" block times the peer form "
                         "beside the RCCL default at N > 1 either way")
    return ap.parse_args(argv)


def steps_per_graph(steps: int, want: int) -> int:
    """The largest G <= want dividing `steps` (each hipGraph replay runs exactly G steps, so
    the timed region runs exactly `steps` steps)."""
    want = max(1, min(want, steps))
    return next(g for g in range(want, 0, -1) if steps % g == 0)


def glorot_stack(rng, k, d_in, d_out):
    r = np.sqrt(6.0 / (d_in + d_out))
    return rng.uniform(-r, r, size=(k, d_in, d_out)).astype(np.float32)


def collectives(backend):
    """(allreduce, allgather) of the sharded step: RCCL called directly on the capturing
    stream (decagon_amd/rccl.py) for backend nccl, torch.distributed's otherwise (gloo)."""
    from decagon_amd.sharding import torch_allgather, torch_allreduce

    if backend == "nccl":
        from decagon_amd.rccl import world_comm

        return world_comm().collectives()
    return torch_allreduce(), torch_allgather()


def peer_config(exchange, loopback=False):
    """The RelationShard.peer of an --exchange choice (None: RCCL / the backend's all-gather)."""
    if exchange == "rccl":
        return None
    from decagon_amd.peer import PeerConfig, dist_gather

    mode = "fused" if exchange == "peer" else "kernel"
    kind = knob("DG_PEER_REGION_KIND", 2)  # the exchange region's memory kind (2: uncached)
    if loopback:
        return PeerConfig(mode=mode, loopback=True, region_kind=kind)
    return PeerConfig(mode=mode, gather=dist_gather(), region_kind=kind)


def build_workload(config, rank, world, sharded, backend="nccl", exchange="rccl"):
    from decagon_amd import synthetic
    from decagon_amd.sharding import RelationShard

    coll = collectives(backend) if sharded else None
    allreduce = coll[0] if sharded else None
    if config == "S":
        base = synthetic.load_S()
        graph = synthetic.replicate_sets(base, world) if world > 1 else base
        shard = None
        if sharded:
            # weak scaling: the graph holds one relation set per GPU; every node type is
            # row-split (each rank finishes its row block over every set's relations —
            # dg_spmm_seg_f32 + the epilogue, layer 2 reassociated — then the blocks are
            # all-gathered: no all-reduce of sums)
            shard = RelationShard.weak_sets(graph.edge_types, graph.n_nodes, rank, world, allreduce, coll[1])
        scaling = "weak"
        workload = ("S: main.py 5-relation / 10-matrix synthetic (reference-normalised, 105,974 nnz "
                    "per relation set), 2 GCN layers d=64/32 + DEDICOM decoder B=512+512")
    else:
        graph = synthetic.make_P(seed=0)
        shard = None
        if sharded:
            shard = RelationShard.polypharmacy(graph, rank, world, collectives=coll)
        scaling = "strong"
        workload = ("P: polypharmacy-shaped 19,085 proteins + 645 drugs, 964 side effects "
                    "(1,932 drug-drug matrices), 2 GCN layers d=64/32 + DEDICOM decoder B=512+512")
    if shard is not None:
        shard.peer = peer_config(exchange)
    return graph, shard, scaling, workload


def make_plan(args, graph, shard, device, keep_sums=False, dropout=None):
    import torch

    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights

    csr = graph.csr()
    if shard is not None:  # only local relations need host CSR / upload
        csr = shard.local_csr(csr)
    chunk = args.chunk if shard is None or shard.chunks is None else shard.chunks
    dg = DeviceGraph(graph.edge_types, csr, device, None if shard is None else shard.local,
                     chunk=chunk, target_waves=args.target_waves,
                     row_block=None if shard is None else shard.row_block)
    rng = np.random.default_rng(1234)
    n = graph.n_nodes
    w1 = LayerWeights({et: torch.from_numpy(glorot_stack(rng, K, n[et[1]], H1)).to(device)
                       for et, K in graph.edge_types.items()})
    w2 = LayerWeights({et: torch.from_numpy(glorot_stack(rng, K, H1, H2)).to(device)
                       for et, K in graph.edge_types.items()})
    plan = ForwardPlan(dg, {j: None for j in n}, w1, w2, H1, H2, shard=shard, keep_sums=keep_sums,
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
    kernel runs on, over `reps` back-to-back launches captured in one hipGraph (best of 5
    replays)."""
    import torch

    with torch.cuda.stream(stream):
        fn()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
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


WARM_REPLAYS = knob("DG_WARM_REPLAYS", 1)  # untimed replays after capture
LAST_TIMING = {}  # timed_steps: the last timed region's device-side span (HIP events), untimed rerun


def timed_steps(step, steps, warmup, G, stream, use_graph=True, barrier=None):
    """W eager warm-up steps, then `steps` steps as steps/G replays of one hipGraph of G
    steps (one untimed replay first: graph upload), bracketed by barrier + synchronize."""
    import torch

    with torch.cuda.stream(stream):
        step()
        for _ in range(max(0, warmup - 1)):
            step()
        stream.synchronize()
        run = step
        if use_graph:
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg, stream=stream, capture_error_mode="thread_local"):
                for _ in range(G):
                    step()
            for _ in range(WARM_REPLAYS):
                cg.replay()
            run = cg.replay
        else:
            G = 1
        stream.synchronize()
        if barrier:
            barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps // G):
            run()
        stream.synchronize()
        torch.cuda.synchronize()
        if barrier:
            barrier()
        el = time.perf_counter() - t0
        # (untimed) the same replays once more between HIP events on the stream: the device's
        # own span, against which the wall-clock figure above shows the host's launch and
        # completion-wait cost of the timed region
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        h0 = time.perf_counter()
        for _ in range(steps // G):
            run()
        h1 = time.perf_counter()
        e1.record(stream)
        e1.synchronize()
        LAST_TIMING.clear()
        LAST_TIMING.update({"device_ms_per_step": e0.elapsed_time(e1) / steps,
                            "host_enqueue_ms": (h1 - h0) * 1e3, "wall_ms_per_step": el * 1e3 / steps})
        return el


KERNEL_NAMES = {"PreparedFused": "gcn_fused_kernel<{lp}>", "PreparedSpmm": "spmm_groups_kernel<{lp}>",
                "PreparedStaged": "spmm_staged_kernel", "PreparedFusedSeg": "gcn_fused_seg_kernel<{lp}, {proj}",
                "PreparedSeg": "spmm_seg_kernel<{lp}, {proj}", "PreparedFusedTab": "gcn_tab_kernel<{proj}",
                "PreparedSegTab": "seg_tab_kernel<{proj}"}


def _kernel_pat(launch, d):
    """The kernel-name prefix of a launch at layer width d (the reassociated seg forms — d_in 64
    → d_out 32 — are their <16, true> instances)."""
    proj = getattr(launch, "d_in", None) is not None and launch.d_in != launch.d_out
    lp = 16 if proj else 1 << max(0, (max(1, d // 4) - 1).bit_length())
    return KERNEL_NAMES.get(type(launch).__name__, "?").format(lp=lp, proj="true" if proj else "false")


def _kernel_label(launch, d):
    pat = _kernel_pat(launch, d)
    return pat if pat.endswith(">") or pat == "spmm_staged_kernel" else pat + ", …>"


def pmc_traffic(config, launch, d, layer=1):
    """HBM bytes per launch of `launch` from the newest committed PMC pass
    (profiles/rNN_traffic.json, written by scripts/prof_summary.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE runs of this bench): FETCH_SIZE × 2 (gfx950 counts half of a
    wide streaming read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KiB → bytes.  A kernel
    launched by both layers is split by launch class (grid / workgroup / LDS bytes; layer 1,
    at d = 64, is the class with the larger fetch).  Returns
    (bytes or None, source, the profiled launch's mean duration in ms)."""
    files = sorted(ROOT.glob("profiles/r*_traffic.json"))
    if not files:
        return None, None, None
    src = str(files[-1].relative_to(ROOT))
    rec = json.load(open(files[-1])).get(config, {})
    pat = _kernel_pat(launch, d)
    hit = [v for k, v in rec.items() if k.replace("void ", "").startswith(pat)]
    if not hit:
        return None, src, None
    e = hit[0]
    us = e.get("avg_us", 0.0)
    if e.get("by_grid") and len(e["by_grid"]) > 1:
        # launch classes (grid/workgroup/LDS): layer 1 (d = 64) fetches the most bytes
        keys = sorted(e["by_grid"], key=lambda c: e["by_grid"][c].get("fetch_size_kib", 0.0))
        key = keys[-1] if layer == 1 else keys[0]
        cls = (e.get("by_launch") or {}).get(key) or {}
        # the kernel-trace mean of that class's launches that ran alone (as bench.py times it)
        us = cls.get("alone_avg_us") or cls.get("overlapped_avg_us") or us
        e = e["by_grid"][key]
    if "fetch_size_kib" not in e or "write_size_kib" not in e:
        return None, src, None
    return (2.0 * e["fetch_size_kib"] + e["write_size_kib"]) * 1024.0, src, us * 1e-3


def cpu_baseline(graph, seconds):
    """torch-CPU on every host CPU this process may use (the reference's TF runs cpu_count()
    threads, DecagonTrainer.py:35-42) and scipy single-thread, same two-layer forward in TF's
    op order (oracle/cpu_baseline.py)."""
    from oracle import cpu_baseline as cb

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return cb.measure(graph, H1, H2, seconds)


# ----------------------------------------------------------------------------- forward step
def forward_bench(args, config, rank, world, sharded, device, dist, steps, warmup, kernel_reps):
    """One config's forward step: value (edges/s over every rank), the dominant layer-1
    kernel's roofline, the whole layer-1 SpMM.  Returns (record fields, graph)."""
    import torch

    graph, shard, scaling, workload = build_workload(config, rank, world, sharded, args.backend, args.exchange)
    plan, dg = make_plan(args, graph, shard, device)
    dec = Decoder(graph, plan, device, rank)
    if sharded:
        dist.barrier()  # (a peer exchange's first wait is bounded: start the ranks together)

    def step():
        plan.run()
        dec()

    stream = torch.cuda.Stream(device)
    use_graph = not args.no_graph
    # One GPU, or N > 1 over RCCL (--collectives graph): G complete steps per hipGraph replay,
    # the per-layer collectives captured with the compute.  Otherwise (gloo, or --collectives
    # eager): each compute phase between collectives is captured and the collectives run
    # eagerly between the replays.
    full = use_graph and (not sharded or (args.backend == "nccl" and args.collectives == "graph"))
    G = steps_per_graph(steps, args.graph_steps) if full else 1
    barrier = dist.barrier if sharded else None
    mode = "eager"
    el = None
    if full:
        try:
            el = timed_steps(step, steps, warmup, G, stream, True, barrier)
            mode = "one hipGraph per %d steps%s" % (G, ", collectives captured" if sharded else "")
        except RuntimeError as e:  # a collective that refuses capture: per-phase graphs
            if not sharded:
                raise
            print(f"bench: capturing the collectives failed ({e}); eager collectives", file=sys.stderr)
            torch.cuda.synchronize()
            full, G = False, 1
    if el is None:
        if use_graph:
            phases = plan.phases()
            last = max(i for i, (kind, _) in enumerate(phases) if kind == "compute")
            seq = []
            with torch.cuda.stream(stream):
                for i, (kind, fn) in enumerate(phases):
                    if kind == "exchange":
                        seq.append(fn)
                        continue
                    body = (lambda fn=fn: (fn(), dec())) if i == last else fn
                    body()
                    stream.synchronize()
                    gph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gph, stream=stream, capture_error_mode="thread_local"):
                        body()
                    seq.append(gph.replay)

            def run_seq():
                for f in seq:
                    f()
            el = timed_steps(run_seq, steps, warmup, 1, stream, False, barrier)
            mode = "hipGraph per compute phase, eager collectives"
        else:
            el = timed_steps(step, steps, warmup, 1, stream, False, barrier)

    split = dict(LAST_TIMING)
    local_edges = 2 * dg.total_nnz
    el_max, tot_edges = el, local_edges
    if sharded:
        t = torch.tensor([el, float(local_edges)], dtype=torch.float64, device=device)
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        el_max, tot_edges = float(tm[0]), float(t[1])
    value = tot_edges * steps / el_max

    # the roofline covers the dominant kernel: the longest SpMM launch of either layer (config
    # S: layer 2's fused, reassociated launch; config P: layer 1's staged drug x drug SpMM), its
    # algorithmic bytes over its own duration; each whole layer's SpMM (launches as the forward
    # runs them) is reported beside it
    l1, l2 = plan.spmm_launches
    per = [(time_kernel(lambda l=l: l(), kernel_reps, stream), 1, i) for i, l in enumerate(l1)]
    per += [(time_kernel(lambda l=l: l(), kernel_reps, stream), 2, i) for i, l in enumerate(l2)]
    k_ms, dom_layer, di = max(per)
    dom = (l1 if dom_layer == 1 else l2)[di]
    dom_d = H1 if dom_layer == 1 else H2
    k_bytes = plan.launch_bytes(dom, dom_layer)
    achieved = k_bytes / (k_ms * 1e-3) / 1e9
    l1_ms = time_kernel(plan._layer1.run_spmm, kernel_reps, stream)
    l1_bytes = plan.layer_bytes(1)
    k2_ms = time_kernel(plan._layer2.run_spmm, kernel_reps, stream)
    l2_bytes = plan.layer_bytes(2)
    traffic, traffic_src, traffic_ms = pmc_traffic(config if world == 1 else None, dom, dom_d, dom_layer)
    rec = {
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": el_max * 1e3 / steps,
        "timing_split": split,
        "scaling": scaling,
        "config": {"workload": workload, "nnz_per_layer_total": int(tot_edges // 2),
                   "parallelism": (plan.parallelism(args.backend) if sharded else "1 GPU"),
                   "hipgraph": use_graph, "launch": mode, "steps_per_graph": G},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "traffic_profiled_kernel_ms": traffic_ms,
                     "kernel": _kernel_label(dom, dom_d) + f" (layer {dom_layer})",
                     "kernel_ms": k_ms, "algorithmic_bytes": k_bytes,
                     "launches_us": {f"layer{ly} {_kernel_label((l1 if ly == 1 else l2)[i], H1 if ly == 1 else H2)}":
                                     ms * 1e3 for ms, ly, i in per}},
        "spmm_layer1": {"launches": [type(x).__name__ for x in l1], "ms": l1_ms,
                        "algorithmic_bytes": l1_bytes, "GB_s": l1_bytes / (l1_ms * 1e-3) / 1e9,
                        "frac": l1_bytes / (l1_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "edges_per_s": dg.total_nnz / (l1_ms * 1e-3)},
        # layer 2's compulsory bytes: the CSR once, H1_j (reassociated / staged forms) or P_k
        # once, W2 once where the launch reads it, the output once (ForwardPlan.layer_bytes)
        "spmm_layer2": {"launches": [type(x).__name__ for x in l2], "ms": k2_ms,
                        "algorithmic_bytes": l2_bytes, "GB_s": l2_bytes / (k2_ms * 1e-3) / 1e9,
                        "frac": l2_bytes / (k2_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "edges_per_s": dg.total_nnz / (k2_ms * 1e-3)},
        "spmm_layer2_ms": k2_ms,
    }
    if sharded:
        rec["rank_ms_per_step"] = el * 1e3 / steps
        if plan.peer is not None:
            rec["peer_error_word"] = plan.peer.error()
        if args.backend == "nccl" and use_graph:
            rec["phases"] = phase_times(plan, dec, stream, dist, min(kernel_reps, 20))
        if plan.xregion is not None and use_graph:
            rec["peer_probe"] = peer_probe(plan, stream, dist, min(kernel_reps, 20), rank, world)
        rec["_outputs"] = [{t: h.cpu().numpy() for t, h in plan.hidden1.items()},
                           {t: e.cpu().numpy() for t, e in plan.embeddings.items()}]
        if plan.peer is not None:
            dist.barrier()
            plan.peer.close()
    del plan, dec
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return rec, graph


def phase_times(plan, dec, stream, dist, reps):
    """The sharded step taken apart on this rank (every rank runs the same sequence): each
    compute phase between two collectives and each exchange (the layer's RCCL all-reduce /
    all-gather), each timed alone as `reps` back-to-back launches in one hipGraph; and the
    bytes each exchange moves.  compute + exchange ≈ the step (the step also pays the
    boundaries between them); the max over ranks of each is reported."""
    import torch

    phases = plan.phases()
    last = max(i for i, (kind, _) in enumerate(phases) if kind == "compute")
    out = {"compute_us": [], "exchange_us": [], "exchange_bytes": []}
    layers = [L for L in (plan._layer1, plan._layer2) if L.has_exchange]
    for i, (kind, fn) in enumerate(phases):
        body = (lambda fn=fn: (fn(), dec())) if i == last else fn
        out["compute_us" if kind == "compute" else "exchange_us"].append(time_kernel(body, reps, stream) * 1e3)
    for L in layers:
        nb = 0 if L.flat is None or L.allreduce is None else 4 * L.flat.numel()
        out["exchange_bytes"].append({"allreduce": nb, "allgather": sum(4 * o.numel() for o, _ in L.gathers)})
    t = torch.tensor(out["compute_us"] + out["exchange_us"], dtype=torch.float64, device=stream.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n_c = len(out["compute_us"])
    out["compute_us"], out["exchange_us"] = t[:n_c].tolist(), t[n_c:].tolist()
    out["compute_total_us"] = sum(out["compute_us"])
    out["exchange_total_us"] = sum(out["exchange_us"])
    return out


def peer_probe(plan, stream, dist, reps, rank, world):
    """Each layer's row-split all-gather as ONE stand-alone peer-store exchange launch
    (dg_peer_allgather, peer.py: IPC-mapped peer regions, write-through stores, bounded flag
    waits), timed alone like the phases — so the driver's N-GPU run records what the peer
    exchange costs on xGMI beside whatever exchange the step ran.  Never raises: an IPC or
    timeout failure is reported in the block."""
    import torch

    from decagon_amd.peer import PeerConfig, PeerExchange, dist_gather

    out = {"kernel": "peer_push_kernel (dg_peer_allgather)", "layers_us": [], "bytes_per_rank": []}
    ex = plan.peer
    own = ex is None
    try:
        if own:
            ex = PeerExchange(plan.xregion, rank, world, PeerConfig(mode="kernel", gather=dist_gather()))
            plan.peer = ex
        fns = plan.peer_probe()
        dist.barrier()
        for fn in fns:
            out["layers_us"].append(time_kernel(fn, reps, stream) * 1e3)
        out["bytes_per_rank"] = [sum(4 * plan._pad[i, layer].shape[1] * plan.row_block[i][2]
                                     for i in plan.row_block) for layer in (1, 2)]
        out["error_word"] = ex.error()
    except Exception as e:  # IPC refused / a peer failed: record it, keep the bench line
        out["error"] = f"{type(e).__name__}: {e}"
    t = torch.tensor(out["layers_us"] or [0.0], dtype=torch.float64, device=stream.device)
    try:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if out["layers_us"]:
            out["layers_us"] = t.tolist()
    except Exception as e:
        out["error"] = out.get("error", "") + f"; max-reduce: {e}"
    if own and ex is not None:
        plan.peer = None
        try:
            dist.barrier()
            ex.close()
        except Exception:
            pass
    return out


def peer_step(args, rank, world, device, dist, steps, warmup, ref_outputs, config="S"):
    """The step with its exchanges done by peer stores fused into the finishing launches
    (--exchange peer), timed as the default step is — beside the RCCL default, which stays
    `value` — and checked against the RCCL step's outputs: bit for bit for config S (only
    all-gathers), within 1e-4 of the largest value for config P, whose drug sums the peer
    all-reduce adds in rank order and RCCL in its ring's order."""
    import torch

    rec = {"exchange": "peer (fused into the finishing launches)"}
    try:
        graph, shard, _, _ = build_workload(config, rank, world, True, args.backend, "peer")
        plan, dg = make_plan(args, graph, shard, device)
        dec = Decoder(graph, plan, device, rank)

        def step():
            plan.run()
            dec()

        stream = torch.cuda.Stream(device)
        dist.barrier()
        G = steps_per_graph(steps, args.graph_steps)
        el = timed_steps(step, steps, warmup, G, stream, True, dist.barrier)
        err = plan.peer.error()
        rel = 0.0
        for t in plan.hidden1:
            for got, want in ((plan.hidden1[t].cpu().numpy(), ref_outputs[0][t]),
                              (plan.embeddings[t].cpu().numpy(), ref_outputs[1][t])):
                rel = max(rel, float(np.max(np.abs(got - want))) / max(float(np.max(np.abs(want))), 1e-30))
        ok = err == 0 and (rel == 0.0 if config == "S" else rel <= 1e-4)
        t = torch.tensor([el, float(2 * dg.total_nnz), 0.0 if ok else 1.0], dtype=torch.float64, device=device)
        tm = t.clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        r = torch.tensor([rel], dtype=torch.float64, device=device)
        dist.all_reduce(r, op=dist.ReduceOp.MAX)
        rec.update({"ms_per_step": float(tm[0]) * 1e3 / steps, "value": float(t[1]) * steps / float(tm[0]),
                    "unit": "edges/s", "steps": steps, "steps_per_graph": G,
                    ("bitwise_equal_to_rccl_and_no_timeout_all_ranks" if config == "S"
                     else "within_1e-4_of_rccl_and_no_timeout_all_ranks"): float(tm[2]) == 0.0,
                    "max_rel_err_vs_rccl": float(r[0]), "error_word": err})
        dist.barrier()
        plan.peer.close()
        del plan, dec
        torch.cuda.synchronize()
    except Exception as e:
        rec["error"] = f"{type(e).__name__}: {e}"
    return rec


# ----------------------------------------------------------------------------- config 5
def decoder_bench(args, device, steps, warmup, rank=0, world=1, dist=None):
    """Config 5 (BASELINE configs[4]): d = 256 bf16 embeddings / R / D_k, DEDICOM decoder on
    MFMA, every one of the 1,928 drug-drug relation slots scoring B = 512 positives and 512
    negatives drawn on the device from THAT slot's degree^0.75 alias table, then the hinge loss
    (scorer.SlotScorer: sampler + scorer + hinge in one launch per step).  At N ranks the
    slots are dealt in contiguous blocks and the scalar loss is all-reduced — the only
    collective.  Returns the record fields."""
    import torch

    from decagon_amd import kernels, synthetic
    from decagon_amd.scorer import SlotScorer
    from decagon_amd.sharding import slot_range

    c5 = synthetic.make_config5()
    bf = torch.bfloat16
    up = lambda a, dt=None: torch.from_numpy(a).to(device) if dt is None else torch.from_numpy(a).to(dt).to(device)
    E, R, Dk = up(c5.E, bf), up(c5.R, bf), up(c5.D, bf)
    slots, B, d = Dk.shape[0], c5.batch, E.shape[1]
    s0, s1 = slot_range(slots, rank, world)
    # (dist None at world > 1: a --simulate-world rank share, the loss all-reduce a no-op)
    sc = SlotScorer(E, E, R, Dk, up(c5.pos_rows), up(c5.pos_cols), kernels.upload_alias(c5.degrees, device), B,
                    MARGIN, seed=11, slots=(s0, s1),
                    allreduce=collectives(args.backend)[0] if world > 1 and dist is not None else None)
    stream = torch.cuda.Stream(device)
    G = steps_per_graph(steps, args.graph_steps)
    el = timed_steps(sc, steps, warmup, G, stream, not args.no_graph,
                     dist.barrier if dist is not None and world > 1 else None)
    if world > 1 and dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    reps = args.kernel_reps if steps >= 50 else 20
    # the step's one launch (sampler + scores + hinge: dg_slot_score_hinge_bf16), alone
    k_ms = time_kernel(lambda: kernels.slot_score_hinge_bf16(
        sc.E_row, sc.E_col, sc.rows[:sc.n], sc.cols[:sc.n], sc.alias, sc.s0, sc.s1 - sc.s0, sc.batch, sc.seed, sc.R,
        sc.D, sc.margin, sc.out, sc.neg_rows, sc.loss, sc._ws), reps, stream)
    # flops the column-shared paired kernel issues per (positive, negative) pair: T = R·(D_k∘v)
    # on the MFMA (2d²) once for both, the B operand (d) and two dots with u∘D_k (2·3d) on the
    # VALU — against 2·(2d² + 4d) when each pair is contracted on its own
    flop_pp = 2 * d * d + 7 * d
    n = 2 * sc.n
    tflops = sc.n * flop_pp / (k_ms * 1e-3) / 1e12
    mfma_tflops = sc.n * 2 * d * d / (k_ms * 1e-3) / 1e12
    return {
        "metric": "DEDICOM scored pairs/sec (config 5: d=256 bf16, all 1,928 drug-drug slots)",
        "value": 2 * slots * B * steps / el,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": el * 1e3 / steps,
        "timing_split": dict(LAST_TIMING),
        "scaling": "strong",
        "dtype": "bf16 (fp32 accumulation)",
        "data": "synthetic: per-slot relations (Zipf sizes, SURVEY §8d), positives = slot edges, negatives "
                "device-sampled from each slot's own degree^0.75 table, random bf16 E / R / D_k",
        "config": {"workload": f"config 5: {slots} relation slots x ({B} pos + {B} neg) pairs, d={d}, "
                               "DEDICOM uT.D_k.R.D_k.v on v_mfma_f32_16x16x32_bf16 + hinge loss",
                   "pairs_per_step": 2 * slots * B, "slots_this_rank": s1 - s0, "hipgraph": not args.no_graph,
                   "steps_per_graph": G},
        "loss": float(sc.loss[0]),
        "roofline": {"bound": "mfma", "achieved": tflops, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tflops / BF16_PEAK_TFLOPS, "traffic": None,
                     "kernel": "decoder_bf16_cs16_kernel<768, true> (sampler + scores + hinge)",
                     "kernel_ms": k_ms,
                     "algorithmic_flops": sc.n * flop_pp, "mfma_tflops": mfma_tflops,
                     "per_pair_form_tflops": n * (2 * d * d + 4 * d) / (k_ms * 1e-3) / 1e12},
    }


def main_decoder(args):
    import torch

    torch.cuda.set_device(0)
    if args.simulate_world:
        # config 5 at N GPUs, each rank's share timed on this one GPU (its contiguous block of
        # slots; the scalar loss all-reduce — the only collective — a no-op)
        N = args.simulate_world
        ranks = []
        for r in (range(N) if args.simulate_rank < 0 else [args.simulate_rank]):
            x = decoder_bench(args, torch.device("cuda", 0), args.steps, args.warmup, r, N, None)
            ranks.append({"rank": r, "ms_per_step": x["ms_per_step"], "kernel_ms": x["roofline"]["kernel_ms"],
                          "slots": x["config"]["slots_this_rank"]})
            print(f"rank {r}/{N}: {ranks[-1]['ms_per_step'] * 1e3:.1f} us/step", file=sys.stderr, flush=True)
        rec = {"metric": "config D sharded-step rehearsal on one GPU (the loss all-reduce not run)", "world": N,
               "steps": args.steps, "warmup": args.warmup,
               "max_rank_ms_per_step": max(x["ms_per_step"] for x in ranks), "ranks": ranks,
               "policy_overrides": overrides()}
        print(json.dumps(rec), file=JSON_OUT, flush=True)
        return
    rec = decoder_bench(args, torch.device("cuda", 0), args.steps, args.warmup)
    rec.update({"higher_is_better": True, "vs_baseline": None, "cpu_baseline": None})
    rec["policy_overrides"] = overrides()  # DG_* knobs that differed from the defaults
    print(json.dumps(rec), file=JSON_OUT, flush=True)


# ----------------------------------------------------------------------------- training step
def main_train(args):
    """The training step of DecagonOptimizer.opt_op (optimizer.py:108-114) on one GPU: the
    forward with the pre-normalisation sums kept, the DEDICOM decoder + hinge on B positives /
    B device-sampled negatives, the backward through the decoder, both GCN layers (every
    relation's W1/W2 gradient) and ApplyAdam on every variable — one hipGraph per step group,
    Adam's beta powers advanced on the device."""
    import torch

    from decagon_amd import kernels, train

    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev_index = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    sharded = world > 1 or args.force_shard
    shard = None
    if sharded:
        # sharded training (train.py) on the forward bench's partition: config S one relation set
        # per GPU with every node type row-split, config P proteins row-split + drug×drug
        # relations LPT-sharded — the forward's exchanges, the backward's dH1 all-reduce and the
        # row-split groups' gradient all-reduce
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)
        graph, shard, scaling, workload = build_workload(args.config, rank, world, True, args.backend)
    else:
        graph, _, scaling, workload = build_workload(args.config, 0, 1, False)
    drop = None
    if args.dropout > 0:
        drop = (1.0 - args.dropout, torch.tensor([20180701, 0], dtype=torch.int64, device=device))
        workload += f"; dropout {args.dropout}"
    plan, dg = make_plan(args, graph, shard, device, keep_sums=True, dropout=drop)
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

    pairs = tp.adam_pairs(plan.w1, plan.w2)
    params = [p for p, _ in pairs] + [dec.R, dec.l]
    grads = [g for _, g in pairs] + [dR, dl]
    adam = train.AdamState(params, lr=0.001)
    prep = adam.prepared(grads)

    def step():
        plan.run()
        dec()
        tp.backward(decoder_grad)
        adam.apply(prep)

    stream = torch.cuda.Stream(device)
    G = steps_per_graph(args.steps, args.graph_steps)
    with torch.cuda.stream(stream):
        step()
        stream.synchronize()
        loss0 = float(f.loss[0])
    el = timed_steps(step, args.steps, max(0, args.warmup - 1), G, stream, not args.no_graph,
                     dist.barrier if sharded else None)
    loss1 = float(f.loss[0])
    params_n = int(sum(p.numel() for p in params))
    edges = 2 * dg.total_nnz
    if sharded:
        t = torch.tensor([el, float(edges), float(params_n)], dtype=torch.float64, device=device)
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        el, edges, params_n = float(tm[0]), float(t[1]), int(t[2])
    rec = {
        "metric": "GCN training-step edges/sec (forward + backward + Adam), " + ("5-relation synthetic" if args.config == "S" else "polypharmacy-shaped"),
        "value": edges * args.steps / el,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (as the forward bench), random glorot weights, device-sampled negatives",
        "config": {"workload": workload + "; training step: backward + TF-Adam on %d parameters" % params_n,
                   "nnz_per_layer_total": int(edges // 2),
                   "parallelism": (shard.describe(args.backend) + " + all-reduce of dH1 (and of the row-split "
                                   "groups' weight gradients) in the backward" if sharded else "1 GPU"),
                   "hipgraph": not args.no_graph, "steps_per_graph": G},
        "loss_first_step": loss0,
        "loss_last_step": loss1,
        "roofline": None,
        "cpu_baseline": None,
    }
    if rank == 0:
        rec["policy_overrides"] = overrides()  # DG_* knobs that differed from the defaults
        print(json.dumps(rec), file=JSON_OUT, flush=True)
    if sharded:
        dist.barrier()
        from decagon_amd import rccl

        if rccl._COMM is not None:
            rccl._COMM.destroy()
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- rehearsal
def main_simulate(args):
    """One GPU standing in for each rank of an N-GPU step in turn: the rank's shard (config P:
    proteins row-split, drug×drug relations LPT-sharded; config S: N relation sets, every node
    type row-split — RelationShard.weak_sets) with the collectives replaced by no-ops,
    timed as the bench times a step.  max over ranks + the collectives' time is the N-GPU step
    (DESIGN §6); the bytes each collective moves are printed beside it."""
    import torch

    from decagon_amd import synthetic
    from decagon_amd.sharding import RelationShard, _no_op, _no_op_reduce

    torch.cuda.set_device(0)
    device = torch.device("cuda", 0)
    N = args.simulate_world
    if args.config == "S":
        graph = synthetic.replicate_sets(synthetic.load_S(), N)
    else:
        graph = synthetic.make_P(seed=0)
    stream = torch.cuda.Stream(device)
    G = steps_per_graph(args.steps, args.graph_steps)
    ranks = []
    for r in (range(N) if args.simulate_rank < 0 else [args.simulate_rank]):
        if args.config == "S":
            shard = RelationShard.weak_sets(graph.edge_types, graph.n_nodes, r, N, _no_op_reduce, _no_op)
        else:
            shard = RelationShard.polypharmacy(graph, r, N, comm=False)
        # --exchange peer / peer-kernel: the loopback rehearsal of the peer exchange — every
        # "peer" copy local scratch, every flag raised by the rank itself (peer.py)
        shard.peer = peer_config(args.exchange, loopback=True)
        plan, dg = make_plan(args, graph, shard, device)
        dec = Decoder(graph, plan, device, r)

        def step():
            plan.run()
            dec()
        el = timed_steps(step, args.steps, args.warmup, G, stream)
        l1, _ = plan.spmm_launches
        phases = {"layer1_spmm_ms": time_kernel(plan._layer1.run_spmm, 20, stream),
                  "layer2_spmm_ms": time_kernel(plan._layer2.run_spmm, 20, stream)}
        coll = []
        for L in (plan._layer1, plan._layer2):
            coll.append({"allreduce_bytes": 0 if L.flat is None else 4 * L.flat.numel(),
                         "allgather_bytes": sum(4 * o.numel() for o, _ in L.gathers)})
        if plan.peer is not None:
            phases["peer_error_word"] = plan.peer.error()
            plan.peer.close()
        ranks.append({"rank": r, "ms_per_step": el * 1e3 / args.steps, "nnz_per_layer": dg.total_nnz,
                      "collectives_per_layer": coll, **phases})
        print(f"rank {r}/{N}: {ranks[-1]['ms_per_step'] * 1e3:.1f} us/step, {dg.total_nnz} nnz", file=sys.stderr,
              flush=True)
        del plan, dec, dg
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    what = ("collectives not run" if args.exchange == "rccl" else
            f"exchange {args.exchange} in loopback: the peer stores, arrivals, flags and polls run, "
            "the xGMI wire latency does not")
    rec = {"metric": f"config {args.config} sharded-step rehearsal on one GPU ({what})", "world": N,
           "steps": args.steps, "warmup": args.warmup, "steps_per_graph": G,
           "max_rank_ms_per_step": max(x["ms_per_step"] for x in ranks), "ranks": ranks}
    rec["policy_overrides"] = overrides()  # DG_* knobs that differed from the defaults
    print(json.dumps(rec), file=JSON_OUT, flush=True)


# ----------------------------------------------------------------------------- main
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
    if args.simulate_world:
        return main_simulate(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
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

    rec, graph = forward_bench(args, args.config, rank, world, sharded, device, dist, args.steps, args.warmup,
                               args.kernel_reps)
    ref_outputs = rec.pop("_outputs", None)
    if sharded and args.config == "S" and args.exchange == "rccl" and args.backend == "nccl":
        # the peer-store form of the same step beside the RCCL default
        rec["peer"] = peer_step(args, rank, world, device, dist, args.steps, args.warmup, ref_outputs)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(graph, args.cpu_seconds)
    extra = {}
    if args.config == "S" and not args.no_extra:
        # config P's forward step (configs[2]; sharded over the same ranks: configs[3]) and
        # config 5's scorer (configs[4]; slot-sharded) — the north-star numbers, on the
        # driver's own run
        p, pgraph = forward_bench(args, "P", rank, world, sharded, device, dist, args.p_steps, 3,
                                  min(args.kernel_reps, 20))
        p_ref = p.pop("_outputs", None)
        if sharded and args.exchange == "rccl" and args.backend == "nccl":
            # config P's step with both exchanges by peer stores (the drug sums' all-reduce too)
            p["peer"] = peer_step(args, rank, world, device, dist, args.p_steps, 3, p_ref, "P")
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            p["cpu_baseline"] = cpu_baseline(pgraph, args.cpu_seconds)
        del pgraph
        extra["P"] = p
        extra["D"] = decoder_bench(args, device, args.d_steps, 3, rank, world, dist if sharded else None)
    if rank == 0:
        out = {"metric": METRIC}
        out.update(rec)
        out.update({"higher_is_better": True, "vs_baseline": None, "dtype": "f32",
                    "data": "synthetic: reference-normalised adjacencies (config S) / seeded generator (P); "
                            "random glorot weights",
                    "cpu_baseline": cpu})
        out.update(extra)
        out["policy_overrides"] = overrides()  # DG_* knobs that differed from the defaults
        print(json.dumps(out), file=JSON_OUT, flush=True)
    if sharded:
        dist.barrier()
        from decagon_amd import rccl

        if rccl._COMM is not None:
            rccl._COMM.destroy()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
