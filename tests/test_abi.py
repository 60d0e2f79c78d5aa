"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol include/*.h declares; the
host-only entry points (schedule construction) work without a GPU. No compute calls are made here."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"\b(ldpc_hip_[a-z_0-9]+)\s*\(", text):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_the_boundary():
    names = _declared_functions()
    for required in ("ldpc_hip_open", "ldpc_hip_close", "ldpc_hip_decode_plan_create", "ldpc_hip_decode_launch",
                     "ldpc_hip_decode_sync", "ldpc_hip_rate_dematch_sync", "ldpc_hip_enqueue", "ldpc_hip_dequeue",
                     "ldpc_hip_read_outputs", "ldpc_hip_harq_free", "ldpc_hip_external_harq_supported",
                     "ldpc_hip_queue_reserve", "ldpc_hip_queue_free"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from srsran_projectvtlmo_amd import _lib
    L = _lib.load()
    for name in _declared_functions():
        assert hasattr(L, name), f"{name} declared in include/ but not exported"
    assert set(_lib.EXPORTED_SYMBOLS) <= set(_declared_functions())


def test_library_is_gfx950_code_object():
    from srsran_projectvtlmo_amd import _lib
    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_struct_layouts_match_header():
    from srsran_projectvtlmo_amd import _lib
    assert ctypes.sizeof(_lib.DecDesc) == 32
    assert ctypes.sizeof(_lib.CbResult) == 4
    assert ctypes.sizeof(_lib.HwConfig) == 44
    assert ctypes.sizeof(_lib.DematchDesc) == 20
    assert ctypes.sizeof(_lib.TbDesc) == 40
    assert ctypes.sizeof(_lib.TbResult) == 4
    assert ctypes.sizeof(_lib.EncDesc) == 24
    assert ctypes.sizeof(_lib.RmDesc) == 32
    assert ctypes.sizeof(_lib.DemodDesc) == 32


@pytest.mark.parametrize("bg,Z,expect", [(1, 384, 32), (2, 384, 28), (1, 2, 32), (2, 52, 28)])
def test_schedule_groups_host_only(bg, Z, expect):
    """Row groups of pairwise column-disjoint consecutive layers (host-side schedule; no GPU call)."""
    from srsran_projectvtlmo_amd import channel_coding as cc
    assert cc.schedule_groups(bg, Z) == expect
    assert cc.schedule_groups(1, 17) < 0  # invalid lifting size


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle or a CPU decoder."""
    pkg = ROOT / "srsran_projectvtlmo_amd"
    for py in pkg.rglob("*.py"):
        text = py.read_text()
        assert "import oracle" not in text and "from oracle" not in text, py


def test_specialised_kernel_selection_host_only():
    """The compile-time schedules of the specialised kernels equal build_graph's for every (BG, Z) of both base graphs
    (ldpc_spec.h: core, mid and small lifting sizes; checked on the host, no GPU call). (A context's
    LDPC_HIP_LAUNCH_NO_SPEC flag turns them off: tests/test_gpu_decoder.py::test_every_lifted_graph_generic_kernel.)"""
    from srsran_projectvtlmo_amd import channel_coding as cc
    import oracle as O
    for bg in (1, 2):
        for z in O.LIFTING_SIZES:
            assert cc.specialised(bg, z) == 1, (bg, z)
    assert cc.specialised(1, 17) < 0


def test_default_stream_is_the_context_stream():
    """0 / None reaches the C ABI as NULL (the context's stream); explicit handles pass through."""
    from srsran_projectvtlmo_amd import _lib
    assert _lib.stream_arg(0) is None and _lib.stream_arg(None) is None
    assert _lib.stream_arg(0x7f00dead0000) == 0x7f00dead0000


def test_decode_work_host_only():
    """ldpc_hip_decode_work (the "auto" type's CPU/GPU split): edges of the layers a codeblock decodes x Z x
    max_iterations, the layer count from the last non-zero LLR as ldpc_decoder_impl.cpp:97-114; 0 for all-zero or
    invalid inputs. Checked against the oracle's base-graph rows. Host only (no GPU call)."""
    import numpy as np

    import oracle as O
    from srsran_projectvtlmo_amd import channel_coding as cc
    rng = np.random.default_rng(4)
    for bg, Z in ((1, 384), (2, 36), (1, 7), (2, 208)):
        K = O.BG_K[bg]
        degs = [len(O.graph_row(bg, Z, m)[0]) for m in range(O.BG_M[bg])]
        for L in (K * Z + 2 * Z, (K + 5) * Z + 3, O.BG_N_SHORT[bg] * Z):
            llr = np.zeros(O.BG_N_SHORT[bg] * Z, np.int8)
            llr[:L] = rng.integers(1, 20, L)
            last = L
            cb_len = max(last + 2 * Z, (K + 4) * Z)
            nl = -(-cb_len // Z) - K
            for it in (1, 6):
                assert cc.decode_work(bg, Z, llr, it) == sum(degs[:nl]) * Z * it, (bg, Z, L, it)
        assert cc.decode_work(bg, Z, np.zeros(100, np.int8), 8) == 0
    assert cc.decode_work(3, 384, np.ones(10, np.int8), 8) == 0
    assert cc.decode_work(1, 385, np.ones(10, np.int8), 8) == 0
    # with CRC early stop the work counts min(max_iterations, 2) iterations
    llr = np.ones(O.BG_N_SHORT[1] * 384, np.int8)
    assert cc.decode_work(1, 384, llr, 8, early_stop=True) == 316 * 384 * 2
    assert cc.decode_work(1, 384, llr, 1, early_stop=True) == 316 * 384
    # the default crossover (measured): C4's codeblocks with early stop stay on the CPU, a full
    # BG1 Z=384 codeblock at 8 iterations without it goes to the GPU
    c4_big = np.ones(28 * 384 - 2 * 384, np.int8)          # BG1 Z=384, 6 layers
    c4_small = np.ones(1248 + 72, np.int8)                 # BG2 Z=36 one-CB TB
    assert not cc.auto_prefers_gpu(1, 384, c4_big, 8, True) and not cc.auto_prefers_gpu(2, 36, c4_small, 8, True)
    assert cc.auto_prefers_gpu(1, 384, llr, 8, False)


def test_stream_arg_host_only():
    """The launch wrappers' stream argument without a GPU in use: an explicit handle as given, 0 / None the context's
    own stream (None); with torch's CUDA initialised, 0 / None become torch's current stream (or hipStreamLegacy, 1,
    for its default stream) -- tests/test_gpu_streams.py."""
    from srsran_projectvtlmo_amd import _lib
    assert _lib.stream_arg(0x1234) == 0x1234
    assert _lib.stream_arg(_lib.STREAM_LEGACY) == 1
    import torch
    if not torch.cuda.is_initialized():
        assert _lib.stream_arg(None) is None and _lib.stream_arg(0) is None
