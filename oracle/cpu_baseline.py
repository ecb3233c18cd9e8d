"""ORACLE — test infrastructure only: the CPU baseline that bench.py times beside the GPU
(BASELINE.md "CPU-baseline plan").  Only bench.py's cpu_baseline leg imports it.

The reference's own path is TensorFlow 1.8 on the host CPU, with `cpu_count()` intra- and
inter-op threads (main/Trainer/DecagonTrainer.py:35-42).  TF 1.8 is not installable here
or on the GPU box, so the same two-layer forward is timed in TF's op order — per relation
X·W (identity features: W itself), sparse·dense matmul, add_n over k, l2_normalize,
Σ over edge types, relu (decagon/deep/layers.py:85-118, decagon/deep/model.py:64-88) — in
two CPU forms:

  torch   torch-CPU, CSR tensors, `torch.set_num_threads(<host CPUs this process may use>)`
  scipy   scipy.sparse CSR, one thread (scipy's sparse·dense product is single-threaded)

Both are fp32, on the same normalised adjacencies the GPU runs.
"""
from __future__ import annotations

import os
import platform
import time
from typing import Callable, Dict, Tuple

import numpy as np
import scipy.sparse as sp

EPS_L2 = 1e-12


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_threads() -> Tuple[int, str]:
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota (the GPU
    box gives a job a share of a larger machine; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = f"affinity {n} of os.cpu_count() {os.cpu_count()}"
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            cap = max(1, int(int(q) // int(p)))
            if cap < n:
                n, why = cap, why + f", cgroup quota {cap}"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < n:
        n, why = int(omp), why + f", OMP_NUM_THREADS {omp}"
    return n, why


def _glorot(rng, k, a, b):
    r = np.sqrt(6.0 / (a + b))
    return rng.uniform(-r, r, size=(k, a, b)).astype(np.float32)


def _csr_lists(graph):
    memo: Dict[int, sp.csr_matrix] = {}
    out = {}
    for et, rels in graph.adj.items():
        lst = []
        for coo in rels:
            key = id(coo[0])
            if key not in memo:
                c, v, s = coo
                memo[key] = sp.csr_matrix((np.asarray(v, np.float32), (c[:, 0], c[:, 1])), shape=s)
            lst.append(memo[key])
        out[et] = lst
    return out


class _Forward:
    def __init__(self, graph, h1: int, h2: int, seed: int):
        rng = np.random.default_rng(seed)
        self.et = dict(graph.edge_types)
        self.n = dict(graph.n_nodes)
        self.csr = _csr_lists(graph)
        self.w1 = {et: _glorot(rng, K, self.n[et[1]], h1) for et, K in self.et.items()}
        self.w2 = {et: _glorot(rng, K, h1, h2) for et, K in self.et.items()}
        self.nnz = int(sum(len(c[1]) for rels in graph.adj.values() for c in rels))


class ScipyForward(_Forward):
    def _layer(self, xs: Callable, relu: bool):
        out = {}
        for et in self.et:
            acc = None
            for k, a in enumerate(self.csr[et]):
                y = a @ xs(et, k)
                acc = y if acc is None else acc + y
            acc = acc / np.sqrt(np.maximum((acc * acc).sum(1, keepdims=True), EPS_L2))
            out[et[0]] = acc if et[0] not in out else out[et[0]] + acc
        return {i: np.maximum(v, 0) for i, v in out.items()} if relu else out

    def run(self):
        h1 = self._layer(lambda et, k: self.w1[et][k], True)
        return h1, self._layer(lambda et, k: h1[et[1]] @ self.w2[et][k], False)


class TorchForward(_Forward):
    def __init__(self, graph, h1, h2, seed):
        import torch

        super().__init__(graph, h1, h2, seed)
        self.t = torch
        memo = {}
        self.tcsr = {}
        for et, lst in self.csr.items():
            self.tcsr[et] = []
            for a in lst:
                if id(a) not in memo:
                    memo[id(a)] = torch.sparse_csr_tensor(
                        torch.from_numpy(a.indptr.astype(np.int64)), torch.from_numpy(a.indices.astype(np.int64)),
                        torch.from_numpy(a.data), size=a.shape)
                self.tcsr[et].append(memo[id(a)])
        self.w1 = {et: torch.from_numpy(w) for et, w in self.w1.items()}
        self.w2 = {et: torch.from_numpy(w) for et, w in self.w2.items()}

    def _layer(self, xs: Callable, relu: bool):
        t = self.t
        out = {}
        for et in self.et:
            acc = None
            for k, a in enumerate(self.tcsr[et]):
                y = t.sparse.mm(a, xs(et, k))
                acc = y if acc is None else acc.add_(y)
            acc = acc * t.rsqrt(t.clamp_min((acc * acc).sum(1, keepdim=True), EPS_L2))
            out[et[0]] = acc if et[0] not in out else out[et[0]].add_(acc)
        return {i: t.relu(v) for i, v in out.items()} if relu else out

    def run(self):
        with self.t.no_grad():
            h1 = self._layer(lambda et, k: self.w1[et][k], True)
            return h1, self._layer(lambda et, k: h1[et[1]] @ self.w2[et][k], False)


def _time(fwd, seconds: float, min_reps: int = 50, max_seconds: float = 30.0):
    """Per-forward wall times: at least `seconds` and at least `min_reps` forwards (BASELINE.md:
    the median of >= 50 runs), unless `max_seconds` run out first."""
    fwd.run()  # warm-up (allocator, thread pool)
    times, t0 = [], time.perf_counter()
    while True:
        t = time.perf_counter()
        fwd.run()
        times.append(time.perf_counter() - t)
        el = time.perf_counter() - t0
        if (el >= seconds and len(times) >= min_reps) or el >= max_seconds:
            return times, el


def measure(graph, h1: int, h2: int, seconds: float = 10.0, seed: int = 1234) -> dict:
    """bench.py's cpu_baseline object for one graph: torch-CPU on every CPU this process may
    use ("value"), scipy single-thread beside it, with the CPU model."""
    import torch

    threads, why = host_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        tf = TorchForward(graph, h1, h2, seed)
        times_t, el_t = _time(tf, seconds)
    finally:
        torch.set_num_threads(prev)
    sf = ScipyForward(graph, h1, h2, seed)
    times_s, el_s = _time(sf, seconds)
    edges = 2 * sf.nnz
    model = cpu_model()
    med_t, med_s = float(np.median(times_t)), float(np.median(times_s))
    return {
        "value": edges / med_t, "unit": "edges/s", "cores": threads, "kind": "port",
        "cpu_model": model, "threads_rule": why,
        "sample": (f"median of {len(times_t)} full 2-layer forwards of config {graph.name} ({sf.nnz} nnz/layer, "
                   f"{el_t:.1f} s), torch-CPU fp32 CSR, {threads} threads on {model}"),
        "ms_per_forward": med_t * 1e3, "ms_per_forward_mean": el_t * 1e3 / len(times_t),
        "scipy_1thread": {"value": edges / med_s, "unit": "edges/s", "cores": 1, "ms_per_forward": med_s * 1e3,
                          "sample": f"median of {len(times_s)} forwards ({el_s:.1f} s), scipy.sparse CSR fp32, 1 thread"},
    }
