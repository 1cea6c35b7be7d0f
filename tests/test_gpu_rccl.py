"""GPU: RCCL from this code on hardware. One GPU per box, and RCCL refuses two ranks on one device, so a child
process runs a ONE-rank "nccl" process group (the communicator bootstrap, all_gather_into_tensor and all_reduce
through RCCL) and StatsGather's side-stream branch with the RCCL collective inside its test seam
(tests/helpers/rccl_world1.py). The N > 1 rank launch itself is rehearsed with gloo (tests/test_distributed_cpu.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_one_rank_group_and_side_stream_gather():
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rccl_world1.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-u", script], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["ok"], res["checks"]
