"""C5 (BASELINE.json configs[4]) rehearsed on the visible GPUs: world_size 2 through torch.distributed.run, one cell
per rank (device = cell_id mod G; on a one-GPU box both ranks share GPU 0), each rank's full C4 slot bit-exact vs the
oracle flow (tests/multi_cell_worker.py)."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_cells_two_ranks_bit_exact():
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        str(ROOT / "tests" / "multi_cell_worker.py")],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    assert res["ranks"] == 2 and res["mismatches"] == 0 and res["tb_crc_ok"] == 48
