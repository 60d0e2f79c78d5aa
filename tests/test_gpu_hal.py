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


def _repo(nof=1024, debug=False):
    """create_ext_harq_buffer_context_repository as pusch_decoder_vectortest.cpp:208-211 calls it (the capacity argument
    is the accelerator's HARQ memory size; the GPU's grows on demand)."""
    from srsran_projectvtlmo_amd import hal
    return hal.create_ext_harq_buffer_context_repository(nof, nof * hal.HARQ_INCR, debug)


def _acc(ext, max_queue_cbs: int = 162, dedicated_queue: bool = True):
    """ext: True (external HARQ; small batches zero-copy), "copy" (external HARQ, every batch through device copies:
    launch flag LDPC_HIP_LAUNCH_HAL_COPY), "separate" (external HARQ, the dematcher as its own kernel instead of fused
    into the decode kernels: LDPC_HIP_LAUNCH_SEPARATE_DEMATCH), False (host HARQ). Built from the reference's
    hw_accelerator_pusch_dec_configuration with acc_type "mi355x"."""
    from srsran_projectvtlmo_amd import _lib, hal
    cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=bool(ext),
                                                     harq_buffer_context=_repo(), dedicated_queue=dedicated_queue,
                                                     max_queue_cbs=max_queue_cbs,
                                                     launch_flags={"copy": _lib.LAUNCH_HAL_COPY,
                                                                   "separate": _lib.LAUNCH_SEPARATE_DEMATCH,
                                                                   "early": _lib.LAUNCH_HAL_EARLY_COPY}.get(ext, 0))
    return hal.create_hw_accelerator_pusch_dec_factory(cfg).create()


TB_CASES = [  # (tbs, bg, nof_ch_symbols, mod, nof_layers, noise)
    (25000, 1, 2496 * 4, "QAM16", 2, 0.95),     # 3 CBs BG1
    (256, 2, 156 * 4, "QPSK", 4, 1.7),         # C4 small UE: BG2 Z=36, F=88, CRC16
    (2000, 2, 1872, "QPSK", 1, 1.1),           # 1 CB BG2, CRC16
    (6000, 1, 4000, "QPSK", 2, 1.0),           # 1 CB BG1, CRC24A
]


@pytest.mark.parametrize("ext", [True, "copy", "separate", False, "shared_queue"])
@pytest.mark.parametrize("early_stop", [True, False])
@pytest.mark.parametrize("case", TB_CASES)
def test_hal_tb_rv_sequence(case, early_stop, ext):
    """ext "shared_queue": external HARQ with dedicated_queue = False (the queue is one of the device's shared HIP
    streams, borrowed per TB)."""
    tbs, bg, nsym, mod, nl, noise = case
    rng = np.random.default_rng(tbs + int(early_stop) + 2 * int(bool(ext)))
    tb = TransportBlock(rng, tbs, bg, nsym, mod, nl)
    acc = _acc(True, dedicated_queue=False) if ext == "shared_queue" else _acc(ext)
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


def test_hal_absolute_cb_id_out_of_repository_bounds():
    """The caller's repository is direct-indexed by absolute_cb_id and holds nof_codeblocks entries; an id beyond that
    is a contract violation (ext_harq_buffer_context_repository.h:70-73 asserts, when acc100's hw_config takes the
    entry), reported as an error, not a drop."""
    from srsran_projectvtlmo_amd import _lib, hal
    cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=True,
                                                     harq_buffer_context=_repo(4))
    acc = hal.create_hw_accelerator_pusch_dec_factory(cfg).create()
    rng = np.random.default_rng(5)
    tb = TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)
    llr = tb.llrs(rng, 0, 1.0, 0.1)[0]
    acc.reserve_queue()
    acc.configure_operation(_small_tb_op(hal, tb, llr, 3), 0)
    assert acc.enqueue_operation(llr, None, 0)
    with pytest.raises(_lib.LdpcHipError):
        acc.configure_operation(_small_tb_op(hal, tb, llr, 4), 1)
    msg = np.zeros((10 * tb.Z + 7) // 8, np.uint8)
    while not acc.dequeue_operation(msg, None, 0):
        pass
    out = hal.hw_pusch_decoder_outputs()
    acc.read_operation_outputs(out, 0, 3)
    assert out.CRC_pass
    acc.free_queue()
    with pytest.raises(_lib.LdpcHipError):
        acc.free_harq_context_entry(4)
    acc.free_harq_context_entry(3)


def test_hal_retransmission_without_soft_data_is_dropped():
    """A retransmission (new_data = 0) of an absolute_cb_id whose repository entry holds no soft data is dropped, as
    acc100 drops it when soft_data_len is 0 (hw_accelerator_pusch_dec_acc100_impl.cpp:120-130): enqueue_operation
    still returns True and the operation reads as a CRC failure with the maximum number of iterations (:179-186,
    233-247)."""
    from srsran_projectvtlmo_amd import hal
    acc = _acc(True)
    rng = np.random.default_rng(6)
    tb = TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)
    llr = tb.llrs(rng, 0, 1.0, 0.1)[0]
    acc.reserve_queue()
    acc.configure_operation(_small_tb_op(hal, tb, llr, 200, new_data=False), 0)
    assert acc.enqueue_operation(llr, None, 0)
    msg = np.zeros((10 * tb.Z + 7) // 8, np.uint8)
    while not acc.dequeue_operation(msg, None, 0):
        pass
    out = hal.hw_pusch_decoder_outputs()
    acc.read_operation_outputs(out, 0, 200)
    assert not out.CRC_pass and out.nof_ldpc_iterations == 6
    acc.free_queue()


def test_hal_factory_selects_by_acc_type():
    from srsran_projectvtlmo_amd import hal
    assert hal.create_hw_accelerator_pusch_dec_factory(hal.hw_accelerator_pusch_dec_configuration("acc100")) is None
    assert hal.hip_device_of_acc_type("mi355x:3") == 3 and hal.hip_device_of_acc_type("mi355x:") == -1
    acc = _acc(True)
    assert acc.is_external_harq_supported()
    assert not _acc(False).is_external_harq_supported()


def _entry(repo, i):
    e = repo.repo[i]
    return e.empty, e.soft_data_len


def _shared_factory(nof=512, debug=False, max_queue_cbs=162, dedicated_queue=True):
    from srsran_projectvtlmo_amd import hal
    repo = _repo(nof, debug)
    cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=True, harq_buffer_context=repo,
                                                     dedicated_queue=dedicated_queue, max_queue_cbs=max_queue_cbs)
    return repo, hal.create_hw_accelerator_pusch_dec_factory(cfg)


@pytest.mark.parametrize("case", TB_CASES[:3])
def test_hal_shared_repository_across_instances(case):
    from srsran_projectvtlmo_amd import hal
    """One external HARQ repository shared by two accelerators (the reference gives every hw_accelerator_pusch_dec a
    factory creates the same ext_harq_buffer_context_repository, hw_accelerator_factories.cpp:46-65): accelerator A
    decodes RV 0 of a TB, accelerator B (another PUSCH decoder thread) RV 2, 3 and 1 of it and combines with A's soft
    bits. Bit-exact with the oracle flow: messages, CRC flags, iteration counts, and the HBM soft buffers of every CB
    still being decoded (read back from the repository)."""
    tbs, bg, nsym, mod, nl, noise = case
    rng = np.random.default_rng(tbs + 11)
    tb = TransportBlock(rng, tbs, bg, nsym, mod, nl)
    repo, fac = _shared_factory()
    acc_a, acc_b = fac.create(), fac.create()
    sw = SwFlow(tb, nof_iters=6, early_stop=True)
    hw = HwFlow(tb, acc_a, nof_iters=6, early_stop=True, abs_base=100)
    combined = False
    for i, rv in enumerate((0, 2, 3, 1)):
        hw.acc = acc_a if i == 0 else acc_b
        llrs = tb.llrs(rng, rv, 1.0, noise + 0.25)
        ok_sw, bits_sw = sw.transmission(llrs, rv, new_data=(i == 0))
        ok_hw, _ = hw.transmission(llrs, rv, new_data=(i == 0))
        assert ok_sw == ok_hw and sw.crc_ok == hw.crc_ok and sw.iters_used == hw.iters_used, f"rv {rv}"
        for r in range(tb.C):
            np.testing.assert_array_equal(sw.msgs[r], hw.msgs[r], err_msg=f"rv {rv} cb {r}")
            if not ok_sw and not sw.crc_ok[r]:
                np.testing.assert_array_equal(hal.read_harq_soft_bits(0, 100 + r, tb.N), sw.soft[r],
                                              err_msg=f"rv {rv} cb {r} soft")
                assert _entry(repo, 100 + r) == (False, tb.N)
        if ok_sw:
            assert np.array_equal(bits_sw[:tbs], tb.data)
            # the TB passed: pusch_decoder_hw_impl frees its entries (pusch_decoder_hw_impl.cpp:372-389)
            assert all(_entry(repo, 100 + r)[0] for r in range(tb.C))
            break
        combined = combined or i > 0
    assert combined, "the case must need a retransmission to exercise the shared soft buffers"


@pytest.mark.parametrize("debug", [False, True])
def test_hal_repository_debug_mode_keeps_entries(debug):
    """free() empties an entry, so a later retransmission of it is dropped; in debug mode
    (ext_harq_buffer_context_repository.h:92-95, the reference's HARQ unit-test mode) the entry and its soft bits are
    kept, and the retransmission combines with them."""
    from srsran_projectvtlmo_amd import hal
    rng = np.random.default_rng(21)
    tb = TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)
    repo, fac = _shared_factory(8, debug)
    acc = fac.create()
    llr0 = tb.llrs(rng, 0, 1.0, 0.3)[0]
    llr2 = tb.llrs(rng, 0, 1.0, 0.3)[0]            # _small_tb_op configures rv 0
    msg = np.zeros((10 * tb.Z + 7) // 8, np.uint8)
    out = hal.hw_pusch_decoder_outputs()
    for new_data, llr in ((True, llr0), (False, llr2)):
        acc.reserve_queue()
        acc.configure_operation(_small_tb_op(hal, tb, llr, 5, new_data=new_data), 0)
        assert acc.enqueue_operation(llr, None, 0)
        while not acc.dequeue_operation(msg, None, 0):
            pass
        acc.read_operation_outputs(out, 0, 5)
        acc.free_queue()
        if new_data:
            assert out.CRC_pass
            soft = hal.read_harq_soft_bits(0, 5, tb.N)
            acc.free_harq_context_entry(5)
            assert _entry(repo, 5) == ((False, tb.N) if debug else (True, tb.N))
    if debug:
        assert out.CRC_pass                       # combined with the kept soft bits
        expect = soft.copy()
        O.rate_dematch(expect, llr2, False, 0, tb.Qm, 0, tb.F)
        np.testing.assert_array_equal(hal.read_harq_soft_bits(0, 5, tb.N), expect)
    else:
        assert not out.CRC_pass and out.nof_ldpc_iterations == 6   # dropped: no soft data


@pytest.mark.parametrize("dedicated_queue", [True, False])
def test_hal_concurrent_instances_shared_repository(dedicated_queue):
    """Eight accelerators from one factory (one shared repository), one per host thread, decode a slot's worth of
    TBs at once -- the shape of pusch_processor_benchmark.cpp:434-466 -- and the retransmission of every failed TB is
    decoded by a different thread than its first transmission. Every TB, CB flag and iteration count equals the
    oracle flow's."""
    import threading
    rng = np.random.default_rng(31)
    cases = [(25000, 1, 2496 * 4, "QAM16", 2)] + [(256, 2, 156 * 4, "QPSK", 4)] * 10 + \
        [(2000, 2, 1872, "QPSK", 1), (6000, 1, 4000, "QPSK", 2)] * 2
    tbs = [TransportBlock(rng, *c) for c in cases]
    noise = [0.9, 1.2, 1.4, 1.6, 1.7, 1.8, 1.3, 1.5, 1.65, 1.75, 1.85, 0.9, 0.8, 1.12, 1.02]
    llrs = [[tb.llrs(rng, rv, 1.0, nz) for rv in (0, 2)] for tb, nz in zip(tbs, noise)]
    sw = [SwFlow(tb, nof_iters=6, early_stop=True) for tb in tbs]
    expect = [[f.transmission(l[0], 0, True)] for f, l in zip(sw, llrs)]
    sw_state = [(list(f.crc_ok), list(f.iters_used), [m.copy() for m in f.msgs]) for f in sw]
    for f, l, e in zip(sw, llrs, expect):
        e.append(f.transmission(l[1], 2, False) if not e[0][0] else None)
    repo, fac = _shared_factory(1024, dedicated_queue=dedicated_queue)
    accs = [fac.create() for _ in range(8)]
    bases = np.cumsum([0] + [tb.C for tb in tbs])
    hw = [HwFlow(tb, accs[0], nof_iters=6, early_stop=True, abs_base=int(b)) for tb, b in zip(tbs, bases)]
    got = [[None, None] for _ in tbs]
    errors = []

    def worker(w, tx):
        try:
            for i in range(len(tbs)):
                if (i + tx) % 8 != w or (tx == 1 and got[i][0][0]):
                    continue
                hw[i].acc = accs[w]
                got[i][tx] = hw[i].transmission(llrs[i][tx], 0 if tx == 0 else 2, tx == 0)
                if tx == 0:
                    got[i].append((list(hw[i].crc_ok), list(hw[i].iters_used), [m.copy() for m in hw[i].msgs]))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    for tx in (0, 1):
        th = [threading.Thread(target=worker, args=(w, tx)) for w in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join(120)
        assert not errors, errors
    n_retx = 0
    for i, tb in enumerate(tbs):
        crc0, it0, msgs0 = got[i][2]
        assert got[i][0][0] == expect[i][0][0] and crc0 == sw_state[i][0] and it0 == sw_state[i][1], f"tb {i} tx 0"
        for r in range(tb.C):
            np.testing.assert_array_equal(msgs0[r], sw_state[i][2][r], err_msg=f"tb {i} cb {r} tx 0")
        if expect[i][1] is not None:
            n_retx += 1
            assert got[i][1][0] == expect[i][1][0], f"tb {i} tx 1"
            assert hw[i].crc_ok == sw[i].crc_ok and hw[i].iters_used == sw[i].iters_used, f"tb {i} tx 1"
            for r in range(tb.C):
                np.testing.assert_array_equal(hw[i].msgs[r], sw[i].msgs[r], err_msg=f"tb {i} cb {r} tx 1")
    assert n_retx >= 3, "the noise levels must leave some TBs for a retransmission"


def test_hal_harq_memory_grows_to_any_absolute_cb_id():
    """The GPU's HARQ memory starts at LDPC_HIP_HARQ_CODEBLOCKS entries and grows to hold whatever absolute_cb_id the
    caller's repository hands out (the reference sizes the accelerator memory, not the GPU): a TB whose CBs sit
    beyond the initial capacity decodes and combines bit-exactly."""
    from srsran_projectvtlmo_amd import _lib
    mem = _lib.HarqDeviceMemory(0)
    base = mem.nof_codeblocks + 700
    mem.close()
    rng = np.random.default_rng(44)
    tb = TransportBlock(rng, 25000, 1, 2496 * 4, "QAM16", 2)
    repo, fac = _shared_factory(base + tb.C + 1)
    acc = fac.create()
    sw = SwFlow(tb, nof_iters=6, early_stop=True)
    hw = HwFlow(tb, acc, nof_iters=6, early_stop=True, abs_base=base)
    for i, rv in enumerate((0, 2, 3, 1)):
        llrs = tb.llrs(rng, rv, 1.0, 1.25)
        ok_sw, _ = sw.transmission(llrs, rv, new_data=(i == 0))
        ok_hw, _ = hw.transmission(llrs, rv, new_data=(i == 0))
        assert ok_sw == ok_hw and sw.crc_ok == hw.crc_ok and sw.iters_used == hw.iters_used, f"rv {rv}"
        for r in range(tb.C):
            np.testing.assert_array_equal(sw.msgs[r], hw.msgs[r], err_msg=f"rv {rv} cb {r}")
        if ok_sw:
            break
    mem = _lib.HarqDeviceMemory(0)
    assert mem.nof_codeblocks > base
    mem.close()


@pytest.mark.parametrize("ext", [True, "early", "copy"])
def test_hal_large_tb_early_copy(ext):
    """A TB of more codeblocks than the work queue takes (36 BG1 CBs, 256QAM): by default its kernel reads the LLRs
    from the pinned staging buffer (zero-copy); "early" (LDPC_HIP_LAUNCH_HAL_EARLY_COPY) copies them to HBM in chunks
    while the caller is still enqueueing and the kernel reads HBM; "copy" is the device-copy path. RV 0 then RV 2 combining: every message, CB flag
    and iteration count equals the oracle flow's."""
    rng = np.random.default_rng(83)
    tb = TransportBlock(rng, 300000, 1, 156 * 273 * 12 // 14 * 2, "QAM256", 4)
    assert tb.C > 16
    acc = _acc(ext)
    sw = SwFlow(tb, nof_iters=8, early_stop=True)
    hw = HwFlow(tb, acc, nof_iters=8, early_stop=True)
    for i, (rv, noise) in enumerate(((0, 1.35), (2, 1.35))):
        llrs = tb.llrs(rng, rv, 2.0, noise)
        ok_sw, _ = sw.transmission(llrs, rv, new_data=(i == 0))
        ok_hw, _ = hw.transmission(llrs, rv, new_data=(i == 0))
        assert ok_sw == ok_hw and sw.crc_ok == hw.crc_ok and sw.iters_used == hw.iters_used, f"rv {rv}"
        for r in range(tb.C):
            np.testing.assert_array_equal(sw.msgs[r], hw.msgs[r], err_msg=f"rv {rv} cb {r}")
        if ok_sw:
            break
