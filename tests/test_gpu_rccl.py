"""GPU: the RCCL path of the multi-GPU step (decagon_amd/rccl.py), in a fresh process.

bench.py at N > 1 captures each whole step — kernels and the RCCL all-reduce / all-gather of
the exchange — into one hipGraph.  Issued through torch.distributed's ProcessGroupNCCL
inside a capture, a collective once aborted the process from the watchdog thread
(hipErrorCapturedEvent), which is why the collectives go straight to RCCL on a
communicator of their own.  This test launches tests/_rccl_child.py under
`python -m torch.distributed.run --nproc-per-node 1` (a child started before any GPU call in
it) and requires it to replay captured sharded steps of config S's row-split form and of the
scaled-down config P, match the float64 oracle at 1e-4, outlive the watchdog period, and
exit 0.  (The 8-rank partitions themselves are checked over gloo in test_gpu_sharded.py; a
multi-GPU RCCL run is the driver's.)
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_captured_rccl_step_in_fresh_process():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "tests" / "_rccl_child.py")]
    res = subprocess.run(cmd, cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=240)
    tail = (res.stdout[-3000:] + "\n---- stderr ----\n" + res.stderr[-3000:])
    assert res.returncode == 0, tail
    assert "RCCL_CHILD_OK" in res.stdout, tail
