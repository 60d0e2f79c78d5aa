"""GPU test of the device work queue's timed-out-wait fallback (ldpc_hip_dwq.cpp dwq_wait): a stalled queue
is made on demand (LDPC_HIP_DWQ_POLL_FLAGS=2, DWQ_POLL_TEST_NO_CLAIM: its grid polls but claims nothing) with a 50 ms
wait limit (LDPC_HIP_DWQ_WAIT_MS). The first one-codeblock call must fail loudly with the work-queue error and a stderr
line, the grid must be stopped and gone (so the context's staging stays usable), and the next calls of the same graph
must take the launch path and be bit-exact against the oracle. Run in a child process: the knobs are read once per
process."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import oracle as O
from srsran_projectvtlmo_amd import _lib
from srsran_projectvtlmo_amd import channel_coding as cc
ctx = _lib.Context(0)
dec = cc.ldpc_decoder_hip(ctx)
rng = np.random.default_rng(5)
out = {"first_error": None, "later": []}
for k in range(3):
    bg, Z, it = 2, 36, 4
    llr = (rng.integers(0, 2, O.BG_N_SHORT[bg] * Z) * 20 - 10).astype(np.int8)
    ref, _ = O.ldpc_decode(bg, Z, llr, it)
    cfg = cc.configuration()
    cfg.block_conf.tb_common.base_graph = bg
    cfg.block_conf.tb_common.lifting_size = Z
    cfg.algorithm_conf.max_iterations = it
    msg = np.zeros(cc.message_bytes(bg, Z), np.uint8)
    try:
        dec.decode(msg, llr, None, cfg)
    except Exception as e:
        if k == 0:
            out["first_error"] = str(e)
            continue
        raise
    out["later"].append(bool(np.array_equal(msg[:ref.size], ref)))
ctx.close()
print(json.dumps(out))
"""


def test_stalled_queue_times_out_then_launch_path_is_exact():
    env = dict(os.environ, LDPC_HIP_DWQ_POLL_FLAGS="2", LDPC_HIP_DWQ_WAIT_MS="50")
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], capture_output=True, text=True, timeout=120,
                       env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["first_error"] is not None and "work queue" in res["first_error"], res
    assert "queue disabled" in r.stderr and "stopped and gone" in r.stderr, r.stderr[-1000:]
    assert res["later"] == [True, True], res
