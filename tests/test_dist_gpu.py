"""The multi-rank path through libdpg on the GPU (tools/dist_check.py): two ranks sharing the
card over gloo run bench.py's sharded step -- ICP shard, factor shard, one all-reduce of the packed
system per Gauss-Newton iteration -- and must reproduce the single-process ICP results byte for
byte and its poses within 1e-9.  (The 8-GPU RCCL run is the driver's; this pins the orchestration
and libdpg's sharded assembly on real hardware.)  A one-rank run on the "nccl" backend puts the
RCCL communicator and its device all-reduce of the packed system on the same path (RCCL needs a GPU
per rank, so more ranks than cards only run over gloo here)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,nproc,backend", [("config3", 2, "gloo"), ("config3", 1, "nccl")])
def test_ranks_match_single_process(cfg, nproc, backend):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "dpg-slam_amd")]),
               DIST_BACKEND=backend)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "tools", "dist_check.py"), cfg],
                       capture_output=True, text=True, timeout=240, env=env)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "dist check ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
