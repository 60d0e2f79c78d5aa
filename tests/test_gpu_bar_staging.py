"""GPU test of the one-codeblock calls' LLR staging (ldpc_hip_buffers.h bar_buffer). The default stages the LLRs of
ldpc_decoder_hip::decode and ldpc_rate_dematcher_hip::rate_dematch in device memory written through the PCIe BAR;
the rest of the suite runs that path. Here the same decode and dematch cases run in a child process with
LDPC_HIP_BAR_STAGING=0, the pinned staging every context falls back to when the BAR allocation or the CPU access
grant fails. Each case is compared bit for bit with the oracle: trailing-zero soft buffers, new data and combining,
limited buffers, and E beyond the LDS staging, on the work queue and on the launch path. The knob is read once per
process, hence the child."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu

CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from tests import test_gpu_dwq as T
for flags in (0, "no_dwq"):
    T.test_one_cb_decode_trailing_zeros(flags)
    T.test_one_cb_rate_dematch_threads(flags)
print("pinned staging exact")
"""


def test_pinned_staging_fallback_is_exact():
    env = dict(os.environ, LDPC_HIP_BAR_STAGING="0")
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], capture_output=True, text=True, timeout=110,
                       env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "pinned staging exact" in r.stdout
