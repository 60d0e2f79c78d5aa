"""GPU parity tests of the rate dematcher and of the hw_accelerator_pusch_dec plugin (HAL) against the CPU oracle.

Procedures follow the reference's tests: ldpc_rm_test.cpp:124-212 (rate dematch incl. combining) and
pusch_decoder_vectortest.cpp:279-395 (TB decode through the SW or HW decoder with the RV sequence {0, 2, 3, 1},
early stop on/off). Bit-exact: per-CB packed messages, CRC flags, iteration counts and (host HARQ) soft buffers."""
import numpy as np
import pytest

import oracle as O
from tests.tb_chain import HwFlow, SwFlow, TransportBlock

pytestmark = pytest.mark.gpu


def _dm():
    from srsran_projectvtlmo_amd import channel_coding as cc
    return cc


DM_CASES = [  # (bg, Z, E, rv, Qm, F, Nref)
    (1, 384, 9728, 0, 8, 0, 0), (1, 384, 9760, 2, 8, 0, 0), (2, 36, 1248, 0, 2, 88, 0), (2, 36, 1248, 3, 2, 88, 0),
    (2, 52, 3000, 2, 4, 20, 0), (1, 52, 1500, 3, 6, 0, 2000), (2, 208, 4000, 1, 1, 100, 0),
    (1, 20, 3000, 0, 2, 0, 0), (2, 8, 1400, 1, 2, 8, 0), (1, 384, 60000, 0, 4, 0, 0), (2, 104, 300, 3, 6, 0, 3000),
    (1, 120, 4000, 1, 8, 64, 5000), (2, 384, 20000, 2, 4, 400, 0),
]


@pytest.mark.parametrize("bg,Z,E,rv,Qm,F,Nref", DM_CASES)
def test_rate_dematch_bit_exact(bg, Z, E, rv, Qm, F, Nref):
    cc = _dm()
    dm = cc.create_ldpc_rate_dematcher_factory_sw("hip").create()
    rng = np.random.default_rng(E + 7 * rv + Z)
    N = O.BG_N_SHORT[bg] * Z
    meta = cc.codeblock_metadata()
    meta.tb_common.rv = rv
    meta.tb_common.mod = {1: "BPSK", 2: "QPSK", 4: "QAM16", 6: "QAM64", 8: "QAM256"}[Qm]
    meta.tb_common.Nref = Nref
    meta.cb_specific.nof_filler_bits = F
    for new_data in (True, False):
        for _ in range(2):
            start = rng.integers(-120, 121, N).astype(np.int8)        # stale / previous HARQ content
            llr = rng.integers(-120, 121, E).astype(np.int8)
            llr[rng.random(E) < 0.03] = 127
            a, b = start.copy(), start.copy()
            dm.rate_dematch(a, llr, new_data, meta)
            O.rate_dematch(b, llr, new_data, rv, Qm, Nref, F)
            np.testing.assert_array_equal(a, b, err_msg=f"new_data={new_data}")


def _acc(ext, max_queue_cbs: int = 162):
    """ext: True (external HARQ; small batches zero-copy), "copy" (external HARQ, every batch through device copies:
    launch flag LDPC_HIP_LAUNCH_HAL_COPY), False (host HARQ)."""
    from srsran_projectvtlmo_amd import _lib, hal
    cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=bool(ext), nof_harq_slots=256,
                                                     max_queue_cbs=max_queue_cbs,
                                                     launch_flags=_lib.LAUNCH_HAL_COPY if ext == "copy" else 0)
    return hal.create_hw_accelerator_pusch_dec_factory(cfg).create()


TB_CASES = [  # (tbs, bg, nof_ch_symbols, mod, nof_layers, noise)
    (25000, 1, 2496 * 4, "QAM16", 2, 0.95),     # 3 CBs BG1
    (256, 2, 156 * 4, "QPSK", 4, 1.7),         # C4 small UE: BG2 Z=36, F=88, CRC16
    (2000, 2, 1872, "QPSK", 1, 1.1),           # 1 CB BG2, CRC16
    (6000, 1, 4000, "QPSK", 2, 1.0),           # 1 CB BG1, CRC24A
]


@pytest.mark.parametrize("ext", [True, "copy", False])
@pytest.mark.parametrize("early_stop", [True, False])
@pytest.mark.parametrize("case", TB_CASES)
def test_hal_tb_rv_sequence(case, early_stop, ext):
    tbs, bg, nsym, mod, nl, noise = case
    rng = np.random.default_rng(tbs + int(early_stop) + 2 * int(bool(ext)))
    tb = TransportBlock(rng, tbs, bg, nsym, mod, nl)
    acc = _acc(ext)
    sw = SwFlow(tb, nof_iters=6, early_stop=early_stop)
    hw = HwFlow(tb, acc, nof_iters=6, early_stop=early_stop)
    for i, rv in enumerate((0, 2, 3, 1)):
        llrs = tb.llrs(rng, rv, 1.0, noise)
        ok_sw, bits_sw = sw.transmission(llrs, rv, new_data=(i == 0))
        ok_hw, bits_hw = hw.transmission(llrs, rv, new_data=(i == 0))
        assert ok_sw == ok_hw, f"rv {rv}"
        assert sw.crc_ok == hw.crc_ok, f"rv {rv}"
        assert sw.iters_used == hw.iters_used, f"rv {rv}"
        for r in range(tb.C):
            np.testing.assert_array_equal(sw.msgs[r], hw.msgs[r], err_msg=f"rv {rv} cb {r}")
            if not ext and not sw.crc_ok[r]:
                np.testing.assert_array_equal(sw.soft[r], hw.soft[r], err_msg=f"rv {rv} cb {r} soft")
        if ok_sw:
            assert np.array_equal(bits_sw[:tbs], tb.data)
            break
        if not early_stop:
            # pusch_decoder_vectortest.cpp:388-390: without early stop, failed/finished CBs report max iterations
            assert all(it == 6 for it in hw.iters_used)


@pytest.mark.parametrize("ext", [True, False])
def test_hal_small_batches_retry(ext):
    """A batch that holds 2 CBs and a 5-CB TB: with external HARQ enqueue_operation returns False when the batch is
    full, pusch_decoder_hw_impl dequeues what it enqueued and enqueues the rest into the next batch of the same
    reservation (pusch_decoder_hw_impl.cpp:237-241, 246-249); with host HARQ it alternates enqueue and dequeue. Same
    bit-exact results as the CPU flow."""
    rng = np.random.default_rng(77 + int(ext))
    tb = TransportBlock(rng, 40000, 1, 2496 * 4, "QAM64", 2)
    assert tb.C >= 5
    acc = _acc(ext, max_queue_cbs=2)
    sw = SwFlow(tb, nof_iters=6, early_stop=True)
    hw = HwFlow(tb, acc, nof_iters=6, early_stop=True)
    for i, rv in enumerate((0, 2)):
        llrs = tb.llrs(rng, rv, 1.0, 1.05)
        ok_sw, _ = sw.transmission(llrs, rv, new_data=(i == 0))
        ok_hw, _ = hw.transmission(llrs, rv, new_data=(i == 0))
        assert ok_sw == ok_hw and sw.crc_ok == hw.crc_ok and sw.iters_used == hw.iters_used
        for r in range(tb.C):
            np.testing.assert_array_equal(sw.msgs[r], hw.msgs[r], err_msg=f"rv {rv} cb {r}")
        if ext and i == 0:
            assert hw.nof_enqueue_false >= 2       # the batch filled up and the retry path ran
        if ok_sw:
            break


def _small_tb_op(hal, tb, llr, abs_id, new_data=True):
    return hal.hw_pusch_decoder_configuration(base_graph_index=2, modulation="QPSK", nof_segments=1, rv=0,
                                              cw_length=llr.size, lifting_size=tb.Z, Ncb=tb.N,
                                              nof_filler_bits=tb.F, max_nof_ldpc_iterations=6, use_early_stop=True,
                                              new_data=new_data, cb_crc_len=16, cb_crc_type=hal.CRC16,
                                              absolute_cb_id=abs_id)


def test_hal_arena_full_drops_operation():
    """An operation that cannot get a HARQ entry is dropped as acc100 drops it: enqueue_operation still returns True
    (the caller carries on), and the operation dequeues as a CRC failure with the maximum number of iterations
    (hw_accelerator_pusch_dec_acc100_impl.cpp:179-186, 233-247)."""
    from srsran_projectvtlmo_amd import hal
    cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=True, nof_harq_slots=1)
    acc = hal.create_hw_accelerator_pusch_dec_factory(cfg).create()
    rng = np.random.default_rng(5)
    tb = TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)
    llr = tb.llrs(rng, 0, 1.0, 0.1)[0]
    acc.reserve_queue()
    acc.configure_operation(_small_tb_op(hal, tb, llr, 10), 0)
    assert acc.enqueue_operation(llr, None, 0)
    acc.configure_operation(_small_tb_op(hal, tb, llr, 11), 1)
    assert acc.enqueue_operation(llr, None, 1)             # accepted as dropped
    msg = np.zeros((10 * tb.Z + 7) // 8, np.uint8)
    while not acc.dequeue_operation(msg, None, 0):
        pass
    out = hal.hw_pusch_decoder_outputs()
    acc.read_operation_outputs(out, 0, 10)
    assert out.CRC_pass
    assert acc.dequeue_operation(msg, None, 1)
    acc.read_operation_outputs(out, 1, 11)
    assert not out.CRC_pass and out.nof_ldpc_iterations == 6
    acc.free_queue()
    acc.free_harq_context_entry(10)


def test_hal_retransmission_without_soft_data_is_dropped():
    """A retransmission (new_data = 0) of an absolute_cb_id the HARQ arena does not hold is dropped, as acc100 drops
    it when soft_data_len is 0 (hw_accelerator_pusch_dec_acc100_impl.cpp:120-130): CRC failure, max iterations."""
    from srsran_projectvtlmo_amd import hal
    acc = _acc(True)
    rng = np.random.default_rng(6)
    tb = TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)
    llr = tb.llrs(rng, 0, 1.0, 0.1)[0]
    acc.reserve_queue()
    acc.configure_operation(_small_tb_op(hal, tb, llr, 1234, new_data=False), 0)
    assert acc.enqueue_operation(llr, None, 0)
    msg = np.zeros((10 * tb.Z + 7) // 8, np.uint8)
    while not acc.dequeue_operation(msg, None, 0):
        pass
    out = hal.hw_pusch_decoder_outputs()
    acc.read_operation_outputs(out, 0, 1234)
    assert not out.CRC_pass and out.nof_ldpc_iterations == 6
    acc.free_queue()


def test_hal_factory_selects_by_acc_type():
    from srsran_projectvtlmo_amd import hal
    assert hal.create_hw_accelerator_pusch_dec_factory(hal.hw_accelerator_pusch_dec_configuration("acc100")) is None
    acc = _acc(True)
    assert acc.is_external_harq_supported()
    assert not _acc(False).is_external_harq_supported()
