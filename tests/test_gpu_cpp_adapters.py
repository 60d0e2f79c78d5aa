"""Runs the C++ adapter test program (tests/cpp/test_adapters.cpp): the srsRAN-side classes ldpc_decoder_hip,
ldpc_rate_dematcher_hip and hal::hw_accelerator_pusch_dec_hip, through the C ABI, checked against the oracle."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.gpu
def test_cpp_adapters_against_oracle():
    subprocess.run(["make", "-s", "-C", str(ROOT / "srsran_projectvtlmo_amd" / "adapters"), "test"], check=True)
    r = subprocess.run([str(ROOT / "tests" / "cpp" / "build" / "test_adapters")], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


def test_cpp_adapters_build():
    """CPU: the adapters and the test program compile and link against the C ABI library."""
    subprocess.run(["make", "-s", "-C", str(ROOT / "srsran_projectvtlmo_amd" / "adapters"), "test"], check=True)
    assert (ROOT / "tests" / "cpp" / "build" / "test_adapters").exists()
