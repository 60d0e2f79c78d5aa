"""GPU tests of the PDSCH encoder plugin (hal::hw_accelerator_pdsch_enc on the MI355X, ldpc_hip_enc_* C ABI) driven in
pdsch_encoder_hw_impl's call order (tests/pdsch_flow.py), bit-exact against the oracle's TB CRC -> segmentation ->
CB CRC -> LDPC encoder -> rate matcher chain. Mirrors the reference's pdsch_encoder_test.cpp (which checks the HW
encoder against the same software chain) and pdsch_encoder_hwacc_benchmark.cpp's TB / CB modes."""
import numpy as np
import pytest

from tests.pdsch_flow import encode_hw, expected_codeword

pytestmark = pytest.mark.gpu

# (tbs, bg, nof_ch_symbols, modulation, layers, rv, Nref)
CASES = [
    (256, 2, 156 * 4, "QPSK", 4, 0, 0),                 # C4's small UEs: one BG2 Z=36 codeblock, CRC16, filler
    (1078248, 1, 250 * 156 * 4, "QAM256", 4, 0, 0),     # C4's UE0: 128 BG1 Z=384 codeblocks
    (40000, 2, 52 * 156, "QAM64", 2, 2, 0),             # 11 BG2 codeblocks, rv 2 (ldpc_segmenter_test_data.h case)
    (8456, 1, 24 * 156 + 2, "QPSK", 1, 3, 0),           # 2 BG1 codeblocks, rv 3, E = 3746 (not a multiple of 8)
    (30000, 1, 40 * 156, "QPSK", 2, 1, 25344 // 2),     # limited buffer (Nref), rv 1
    (1024, 2, 12 * 156, "BPSK", 1, 0, 0),               # BPSK, one codeblock, CRC16
]


@pytest.fixture(scope="module")
def ctx():
    from srsran_projectvtlmo_amd import _lib
    c = _lib.Context(0)
    yield c
    c.close()


def _tb(rng, tbs):
    return rng.integers(0, 256, tbs // 8).astype(np.uint8)


@pytest.mark.parametrize("cb_mode", [False, True])
@pytest.mark.parametrize("case", CASES, ids=[f"tbs{c[0]}_bg{c[1]}_{c[3]}" for c in CASES])
def test_pdsch_encoder_plugin_bit_exact(ctx, case, cb_mode):
    from srsran_projectvtlmo_amd import hal
    tbs, bg, nsym, mod, layers, rv, Nref = case
    rng = np.random.default_rng(tbs + 7 * bg + rv)
    tb = _tb(rng, tbs)
    enc = hal.hw_accelerator_pdsch_enc_hip(ctx, cb_mode=cb_mode)
    try:
        assert enc.get_cb_mode() == cb_mode
        got, stats = encode_hw(enc, tb, bg, nsym, mod, layers, rv, Nref)
    finally:
        enc.close()
    want = expected_codeword(tb, bg, nsym, mod, layers, rv, Nref)
    assert stats["enqueue_false"] == 0
    np.testing.assert_array_equal(got, want)


def test_pdsch_encoder_queue_full_and_tb_size_limit(ctx):
    """A batch of 16 codeblocks: a 41-CB TB in CB mode fills it (enqueue_operation returns False, the caller dequeues
    and enqueues the rest: three batches); in TB mode a TB above get_max_tb_size() is encoded in CB mode
    (pdsch_encoder_hw_impl.cpp:35-40). Both bit-exact."""
    from srsran_projectvtlmo_amd import hal
    rng = np.random.default_rng(40)
    tbs, bg, nsym, mod, layers = 337920, 1, 200 * 156, "QAM64", 4   # 41 BG1 codeblocks
    tb = _tb(rng, tbs)
    want = expected_codeword(tb, bg, nsym, mod, layers, 0, 0)
    enc = hal.hw_accelerator_pdsch_enc_hip(ctx, cb_mode=True, max_queue_cbs=16)
    try:
        got, stats = encode_hw(enc, tb, bg, nsym, mod, layers, 0, 0)
    finally:
        enc.close()
    np.testing.assert_array_equal(got, want)
    assert stats["enqueue_false"] == 2 and stats["batches"] == 3
    enc = hal.hw_accelerator_pdsch_enc_hip(ctx, cb_mode=False, max_tb_bytes=4096)
    try:
        assert enc.get_max_tb_size() == 4096 and not enc.get_cb_mode()
        got, _ = encode_hw(enc, tb, bg, nsym, mod, layers, 0, 0)
    finally:
        enc.close()
    np.testing.assert_array_equal(got, want)


def test_pdsch_encoder_factory_and_contract(ctx):
    """The factory selects the plugin by acc_type (hw_accelerator_factories.cpp); calls out of order and invalid
    configurations are refused, as the reference asserts."""
    from srsran_projectvtlmo_amd import _lib, hal
    assert hal.create_hw_accelerator_pdsch_enc_factory(hal.hw_accelerator_pdsch_enc_configuration(acc_type="acc100")) \
        is None
    f = hal.create_hw_accelerator_pdsch_enc_factory(hal.hw_accelerator_pdsch_enc_configuration(cb_mode=True))
    enc = f.create()
    try:
        assert enc.get_cb_mode() and enc.get_max_tb_size() == 159749
        cfg = hal.hw_pdsch_encoder_configuration(nof_tb_bits=256, base_graph_index=2, modulation="QPSK",
                                                 nof_segments=1, lifting_size=36, Ncb=1800, nof_filler_bits=88,
                                                 rm_length=1248, cb_mode=True)
        with pytest.raises(_lib.LdpcHipError):          # enqueue before reserve_queue
            enc.configure_operation(cfg, 0)
            enc.enqueue_operation(np.zeros((360 - 88 + 7) // 8, np.uint8), None, 0)
        enc.reserve_queue()
        bad = hal.hw_pdsch_encoder_configuration(**{**cfg.__dict__, "rm_length": 1249})  # E not a multiple of Qm
        with pytest.raises(_lib.LdpcHipError):
            enc.configure_operation(bad, 0)
        enc.configure_operation(cfg, 0)
        with pytest.raises(_lib.LdpcHipError):          # wrong data size
            enc.enqueue_operation(np.zeros(5, np.uint8), None, 0)
        assert enc.enqueue_operation(np.zeros((360 - 88 + 7) // 8, np.uint8), None, 0)
        out = np.zeros(1248, np.uint8)
        while not enc.dequeue_operation(out, None, 0):
            pass
        enc.free_queue()
    finally:
        enc.close()
        enc.ctx.close()


# Small batches (<= 8 codeblocks) take the encoder's device work queue (ldpc_dwq_encode_kernel); a context with
# LDPC_HIP_LAUNCH_NO_DWQ launches ldpc_pdsch_encode_kernel instead. Both routes, both modes, against the oracle chain;
# the 6-CB BG2 TB has segments of 3,338 bits, so TB mode reads them at bit offsets and attaches their CRC24B on the
# device.
SMALL_CASES = [
    (256, 2, 156 * 4, "QPSK", 4, 0, 0),        # one BG2 Z=36 codeblock, CRC16, filler
    (8456, 1, 24 * 156 + 2, "QPSK", 1, 3, 0),  # 2 BG1 codeblocks, rv 3
    (20000, 2, 52 * 156, "QAM64", 2, 1, 0),    # 6 BG2 codeblocks, segments not byte aligned, rv 1
]


@pytest.mark.parametrize("route", ["work_queue", "launch"])
@pytest.mark.parametrize("cb_mode", [False, True])
@pytest.mark.parametrize("case", SMALL_CASES, ids=[f"tbs{c[0]}_bg{c[1]}_{c[3]}" for c in SMALL_CASES])
def test_pdsch_encoder_small_batches_both_routes(case, cb_mode, route):
    from srsran_projectvtlmo_amd import _lib, hal
    tbs, bg, nsym, mod, layers, rv, Nref = case
    rng = np.random.default_rng(tbs + 11 * bg + rv)
    tb = _tb(rng, tbs)
    c = _lib.Context(0, launch_flags=_lib.LAUNCH_NO_DWQ if route == "launch" else 0)
    try:
        enc = hal.hw_accelerator_pdsch_enc_hip(c, cb_mode=cb_mode)
        try:
            got, stats = encode_hw(enc, tb, bg, nsym, mod, layers, rv, Nref)
        finally:
            enc.close()
    finally:
        c.close()
    assert stats["enqueue_false"] == 0
    np.testing.assert_array_equal(got, expected_codeword(tb, bg, nsym, mod, layers, rv, Nref))
