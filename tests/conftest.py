"""Test configuration: the `gpu` marker, repo-root import path and shared fixtures.

`-m "not gpu"` tests run on the CPU container (oracle vs golden vectors, host logic, C-ABI
symbol checks, gloo multi-process sharding).  `-m gpu` tests are the parity tests proper:
they call the HIP kernels through the C ABI and compare with the oracle / golden fixtures.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests")


@pytest.fixture(scope="session")
def golden_S():
    return np.load(GOLDEN / "synthetic_S.npz", allow_pickle=False)


@pytest.fixture(scope="session")
def golden_kat():
    return np.load(GOLDEN / "dedicom_kat.npz", allow_pickle=False)


def rel_err(got, want) -> float:
    """max|got - want| / max|want| — the SURVEY §8c tolerance metric."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    den = np.max(np.abs(want))
    if den == 0:
        return float(np.max(np.abs(got)))
    return float(np.max(np.abs(got - want)) / den)


def alias_draws(table, seed, idx):
    """Host restatement of the device's counter-based alias draw (decoder_tile.h unigram_draw):
    h = splitmix64(seed ^ splitmix64(idx)); column j = ((h >> 32)·range) >> 32; accept j when
    the 24-bit uniform of h's low bits is below its probability, else its alias."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def sm(z):
        z = (z + np.uint64(0x9E3779B97F4A7C15)) & M
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M
        return z ^ (z >> np.uint64(31))

    with np.errstate(over="ignore"):
        h = sm(np.uint64(seed) ^ sm(np.asarray(idx, np.uint64)))
    rng_ = np.uint64(table.shape[0])
    j = (((h >> np.uint64(32)) * rng_) >> np.uint64(32)).astype(np.int64)
    u = (h & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    q = table[:, 0].view(np.float32)
    return np.where(u < q[j], j, table[j, 1].astype(np.int64)).astype(np.int32)


# ---------------------------------------------------------------- multi-rank tests (gloo)
def _rank_entry(fn, rank, world, port, q, args):
    """Child process of run_ranks: gloo group, fn(rank, world, *args) -> payload, reported
    as (rank, "ok", payload) or (rank, "err", traceback) — a failing rank is seen at once."""
    import datetime
    import traceback

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=180))
        q.put((rank, "ok", fn(rank, world, *args)))
        dist.barrier()
    except BaseException:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_ranks(fn, world, args=(), timeout=400):
    """Run fn(rank, world, *args) in `world` spawned processes over gloo (127.0.0.1) and return
    {rank: payload}.  Polls every few seconds (printing a heartbeat), fails as soon as a rank
    reports an error or dies, kills the others."""
    import socket
    import sys
    import time

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_rank_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    got, t0 = {}, time.time()
    try:
        while len(got) < world:
            try:
                r, status, payload = q.get(timeout=5)
            except Exception:
                dead = [p for p in procs if p.exitcode not in (None, 0)]
                if dead:
                    raise AssertionError(f"rank process died with exit code {dead[0].exitcode}")
                if time.time() - t0 > timeout:
                    raise AssertionError(f"ranks did not finish within {timeout} s")
                print(f"[run_ranks] waiting: {len(got)}/{world} ranks done, {time.time() - t0:.0f} s",
                      file=sys.stderr, flush=True)
                continue
            if status != "ok":
                raise AssertionError(f"rank {r} failed:\n{payload}")
            got[r] = payload
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return got
