"""GPU parity tests of the device work queue (csrc/ldpc_hip_dwq.{h,cpp}): the software route's one-codeblock calls
(ldpc_decoder::decode, ldpc_rate_dematcher::rate_dematch; pusch_codeblock_decoder.cpp:35-71) handed to the resident
grid of their graph's unit instead of a kernel launch each. Bit-exact against the CPU oracle: packed messages,
iteration counts / CRC status and soft buffers, from concurrent host threads (one context per thread, as one decoder
object per worker thread), across graphs of every kind of unit, with the queue's grid exiting and being relaunched
between calls, and against the launch path (LDPC_HIP_LAUNCH_NO_DWQ) of the same calls."""
import threading
import time

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

# graphs of the core unit, mid units and small units of both base graphs (spec_unit)
GRAPHS = [(1, 384), (2, 384), (1, 256), (2, 208), (1, 120), (2, 96), (1, 52), (2, 36), (2, 12), (1, 2), (2, 2)]


def _cb(rng, bg, Z, codeword, crc):
    """LLRs of a full-length codeblock: a CRC24B codeword plus noise, or random +-10 (the reference benchmark)."""
    K, N = O.BG_K[bg] * Z, O.BG_N_SHORT[bg] * Z
    if not codeword:
        return (rng.integers(0, 2, N) * 20 - 10).astype(np.int8)
    msg = rng.integers(0, 2, K).astype(np.uint8)
    if crc:
        c = O.crc_bits(O.CRC24B, msg[:K - 24])
        msg[K - 24:] = [(c >> (23 - i)) & 1 for i in range(24)]
    cw = O.ldpc_encode(bg, Z, msg)
    x = np.where(cw == 1, -2.0, 2.0) + rng.standard_normal(cw.size) * 0.9
    return O.quantize_array(x.astype(np.float32), 8.0)


def _decode_case(rng, bg, Z, it, codeword, crc):
    """One case and its oracle result (computed on the calling thread: the oracle's encoder caches state globally)."""
    crc = crc and O.BG_K[bg] * Z >= 64          # a CRC24B needs a message longer than its checksum
    llr = _cb(rng, bg, Z, codeword, crc)
    ref, ref_it = O.ldpc_decode(bg, Z, llr, it, O.CRC24B if crc else O.NO_CRC)
    return (bg, Z, it, crc, llr), (ref, ref_it)


def _run_decode(dec, cc, case):
    bg, Z, it, crc, llr = case
    cfg = cc.configuration()
    cfg.block_conf.tb_common.base_graph = bg
    cfg.block_conf.tb_common.lifting_size = Z
    cfg.algorithm_conf.max_iterations = it
    out = np.zeros(cc.message_bytes(bg, Z), np.uint8)
    got = dec.decode(out, llr, cc.crc_calculator("CRC24B") if crc else None, cfg)
    return out, got


@pytest.mark.parametrize("flags", [0, "no_dwq"])
def test_one_cb_decode_threads(flags):
    """8 host threads x every graph kind, codewords with CRC early stop and random inputs without CRC; each thread
    only calls the product (the cases and their oracle results are made beforehand)."""
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    lf = _lib.LAUNCH_NO_DWQ if flags == "no_dwq" else 0
    cases = []
    for w in range(8):
        rng = np.random.default_rng(100 + w)
        cases.append([_decode_case(rng, *GRAPHS[(w + k) % len(GRAPHS)], 1 + (k % 8), (k % 3) != 2, (k % 2) == 0)
                      for k in range(12)])
    errors, got = [], [[None] * 12 for _ in range(8)]

    def worker(w):
        ctx = _lib.Context(0, launch_flags=lf)
        try:
            dec = cc.ldpc_decoder_hip(ctx)
            for k, (case, _) in enumerate(cases[w]):
                got[w][k] = _run_decode(dec, cc, case)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)
        finally:
            ctx.close()

    th = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors[:4]
    for w in range(8):
        for k, (case, (ref, ref_it)) in enumerate(cases[w]):
            out, it = got[w][k]
            assert it == ref_it and np.array_equal(out, ref), (w, k, case[:4])


def test_one_cb_decode_grid_relaunch():
    """Calls further apart than the grid's idle period (2 ms): each finds the grid gone and relaunches it."""
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    ctx = _lib.Context(0)
    try:
        dec = cc.ldpc_decoder_hip(ctx)
        rng = np.random.default_rng(7)
        for k in range(6):
            case, (ref, ref_it) = _decode_case(rng, *GRAPHS[k * 2 % len(GRAPHS)], 8, True, True)
            out, it = _run_decode(dec, cc, case)
            assert it == ref_it and np.array_equal(out, ref), case[:2]
            time.sleep(0.02)
    finally:
        ctx.close()


DM = [  # (bg, Z, E, rv, Qm, F, Nref, new_data)
    (1, 384, 9728, 0, 8, 0, 0, True), (1, 384, 9760, 2, 8, 0, 0, False), (2, 36, 1248, 0, 2, 88, 0, True),
    (2, 36, 1248, 3, 2, 88, 0, False), (1, 52, 1500, 3, 6, 0, 2000, True), (2, 208, 4000, 1, 1, 100, 0, False),
    (1, 384, 60000, 0, 4, 0, 0, True), (2, 104, 300, 3, 6, 0, 3000, True),
]


@pytest.mark.parametrize("flags", [0, "no_dwq"])
def test_one_cb_rate_dematch_threads(flags):
    """ldpc_rate_dematcher::rate_dematch of one codeblock (dematch-only work items of the core unit's queue), 8
    threads, new data and combining, limited buffers and E beyond the LDS staging."""
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    lf = _lib.LAUNCH_NO_DWQ if flags == "no_dwq" else 0
    cases = []
    for w in range(8):
        rng = np.random.default_rng(200 + w)
        per = []
        for k in range(len(DM)):
            bg, Z, E, rv, Qm, F, Nref, nd = DM[(w + k) % len(DM)]
            start = rng.integers(-120, 121, O.BG_N_SHORT[bg] * Z).astype(np.int8)
            llr = rng.integers(-120, 121, E).astype(np.int8)
            ref = O.rate_dematch(start.copy(), llr, nd, rv, Qm, Nref, F)
            per.append(((bg, Z, E, rv, Qm, F, Nref, nd), start, llr, ref))
        cases.append(per)
    errors, got = [], [[None] * len(DM) for _ in range(8)]

    def worker(w):
        ctx = _lib.Context(0, launch_flags=lf)
        try:
            dm = cc.ldpc_rate_dematcher_hip(ctx)
            for k, ((bg, Z, E, rv, Qm, F, Nref, nd), start, llr, _) in enumerate(cases[w]):
                meta = cc.codeblock_metadata()
                meta.tb_common.rv = rv
                meta.tb_common.mod = {1: "BPSK", 2: "QPSK", 4: "QAM16", 6: "QAM64", 8: "QAM256"}[Qm]
                meta.tb_common.Nref = Nref
                meta.cb_specific.nof_filler_bits = F
                a = start.copy()
                dm.rate_dematch(a, llr, nd, meta)
                got[w][k] = a
        except Exception as e:  # pragma: no cover
            errors.append(e)
        finally:
            ctx.close()

    th = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors[:4]
    for w in range(8):
        for k, (params, _, _, ref) in enumerate(cases[w]):
            np.testing.assert_array_equal(got[w][k], ref, err_msg=f"{w} {k} {params}")


@pytest.mark.parametrize("flags", [0, "no_dwq"])
def test_one_cb_decode_trailing_zeros(flags):
    """ldpc_decoder::decode of a soft buffer of full length N whose tail is zero (a codeblock rate-dematched from
    E < N LLRs, the software route's usual input): the call stages only up to the last non-zero block, which must
    decode exactly as the whole buffer (ldpc_decoder_impl.cpp:85-112 works up to the last non-zero LLR); including
    tails ending inside the last 32-byte block, a non-zero LLR at the very end and an all-zero buffer."""
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    lf = _lib.LAUNCH_NO_DWQ if flags == "no_dwq" else 0
    rng = np.random.default_rng(11)
    cases = []
    for bg, Z, keep in ((1, 384, 9728), (1, 384, 9731), (2, 36, 700), (2, 52, 50 * 52), (1, 13, 24 * 13 + 1),
                        (2, 208, 3000), (1, 64, 0)):
        N = O.BG_N_SHORT[bg] * Z
        llr = np.zeros(N, np.int8)
        if keep:
            full = _cb(rng, bg, Z, True, O.BG_K[bg] * Z >= 64)
            llr[:keep] = full[:keep]
        crc = O.BG_K[bg] * Z >= 64 and keep != 0
        ref, ref_it = O.ldpc_decode(bg, Z, llr, 8, O.CRC24B if crc else O.NO_CRC)
        cases.append(((bg, Z, 8, crc, llr), (ref, ref_it)))
    ctx = _lib.Context(0, launch_flags=lf)
    try:
        dec = cc.ldpc_decoder_hip(ctx)
        for case, (ref, ref_it) in cases:
            out, it = _run_decode(dec, cc, case)
            assert it == ref_it and np.array_equal(out, ref), case[:4]
    finally:
        ctx.close()


# 14 graphs: more keys than the pool has streams (at most LDPC_HIP_DWQ_MAX_QUEUES = 3 resident grids, within the
# LDPC_HIP_DWQ_BUDGET of 128 workgroups), so most calls find every stream held and take the launch path while others
# ride the queues
GRAPHS14 = GRAPHS + [(1, 64), (2, 160), (1, 288)]


def test_many_graphs_beside_a_batch_launch():
    """8 host threads over 14 graphs (more queue keys than the device's stream pool holds grids) while the main
    thread launches 128-CB BG1 Z=384 batches (C2's plan) on its own stream: every one-CB call and every batch
    codeblock is bit-exact vs the oracle. Reports the worst call latency (a call refused by the budget launches
    instead of waiting for a grid to leave)."""
    import torch
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    cases = []
    for w in range(8):
        rng = np.random.default_rng(300 + w)
        cases.append([_decode_case(rng, *GRAPHS14[(w * 3 + k) % len(GRAPHS14)], 1 + (k % 6), True, (k % 2) == 0)
                      for k in range(14)])
    # the batch: 128 CBs of C2's graph, oracle results for a sample
    rng = np.random.default_rng(77)
    n = 128
    specs, ls, os_ = cc.uniform_batch_specs(n, 1, 384, 8)
    h = (rng.integers(0, 2, (n, ls)) * 20 - 10).astype(np.int8)
    ref = [O.ldpc_decode(1, 384, h[i, :66 * 384], 8)[0] for i in (0, 77, 127)]
    bctx = _lib.Context(0)
    plan = cc.DecodePlan(bctx, specs)
    d_llr = torch.from_numpy(h).cuda()
    d_out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    errors, got, lat = [], [[None] * 14 for _ in range(8)], []
    done = threading.Event()

    def worker(w):
        ctx = _lib.Context(0)
        try:
            dec = cc.ldpc_decoder_hip(ctx)
            for k, (case, _) in enumerate(cases[w]):
                t0 = time.perf_counter()
                got[w][k] = _run_decode(dec, cc, case)
                lat.append(time.perf_counter() - t0)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)
        finally:
            ctx.close()

    th = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in th:
        t.start()
    launches = 0
    while any(t.is_alive() for t in th) and launches < 400:
        plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, stream.cuda_stream)
        launches += 1
        if launches % 8 == 0:
            stream.synchronize()
    for t in th:
        t.join(120)
    stream.synchronize()
    done.set()
    assert not errors, errors[:4]
    out = d_out.cpu().numpy().reshape(n, os_)
    for i, r in zip((0, 77, 127), ref):
        np.testing.assert_array_equal(out[i, :r.size], r, err_msg=f"batch cb {i}")
    for w in range(8):
        for k, (case, (refm, ref_it)) in enumerate(cases[w]):
            o, it = got[w][k]
            assert it == ref_it and np.array_equal(o, refm), (w, k, case[:4])
    plan.close()
    bctx.close()
    print(f"one-CB calls: {len(lat)}, max latency {max(lat) * 1e6:.0f} us, p50 {np.median(lat) * 1e6:.0f} us; "
          f"{launches} batch launches beside them")
    assert max(lat) < 0.5, "a call waited for a grid to leave"


def test_harq_memory_grows_while_work_queue_batches_run():
    """Small HAL TBs (work-queue batches) decode and retransmit on one thread while another thread's accelerator
    keeps growing the GPU's HARQ memory (each growth moves the soft bits to a new allocation): growth waits for every
    issued work-queue item and launch that uses the old memory (ldpc_hip_harq_repo::wait_users), so every first
    transmission, every combined retransmission and every soft buffer stays bit-exact vs the oracle flow."""
    from srsran_projectvtlmo_amd import _lib, hal
    from tests.tb_chain import HwFlow, SwFlow, TransportBlock
    mem = _lib.HarqDeviceMemory(0)
    cap0 = mem.nof_codeblocks
    mem.close()
    repo = hal.create_ext_harq_buffer_context_repository(cap0 + 40000, (cap0 + 40000) * hal.HARQ_INCR, False)
    cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=True, harq_buffer_context=repo)
    fac = hal.create_hw_accelerator_pusch_dec_factory(cfg)
    rng = np.random.default_rng(91)
    tbs = [TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4) for _ in range(12)] + \
        [TransportBlock(rng, 2000, 2, 1872, "QPSK", 1) for _ in range(4)]
    llrs = [[tb.llrs(rng, rv, 1.0, 1.75) for rv in (0, 2)] for tb in tbs]
    sw = [SwFlow(tb, nof_iters=6, early_stop=True) for tb in tbs]
    expect = []
    for f, l in zip(sw, llrs):
        e0 = f.transmission(l[0], 0, True)
        expect.append((e0, f.transmission(l[1], 2, False) if not e0[0] else None, list(f.crc_ok)))
    acc = fac.create()
    hw = [HwFlow(tb, acc, nof_iters=6, early_stop=True, abs_base=10 * i) for i, tb in enumerate(tbs)]
    stop, errors = threading.Event(), []

    def grower():
        try:
            acc2 = fac.create()
            big = TransportBlock(np.random.default_rng(5), 256, 2, 156 * 4, "QPSK", 4)
            l2 = big.llrs(np.random.default_rng(6), 0, 2.0, 0.5)
            k = 0
            while not stop.is_set() and k < 4:  # 4 doublings from the initial capacity (16x, under 1 GB)
                # an absolute_cb_id beyond the current capacity: enqueue grows the memory (doubling)
                mem = _lib.HarqDeviceMemory(0)
                cap = mem.nof_codeblocks
                mem.close()
                HwFlow(big, acc2, nof_iters=6, early_stop=True, abs_base=cap + 5).transmission(l2, 0, True)
                k += 1
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    g = threading.Thread(target=grower)
    g.start()
    try:
        for i, (tb, f) in enumerate(zip(tbs, hw)):
            ok0, _ = f.transmission(llrs[i][0], 0, True)
            assert ok0 == expect[i][0][0], f"tb {i} tx 0"
            if not ok0:
                ok1, _ = f.transmission(llrs[i][1], 2, False)
                assert ok1 == expect[i][1][0], f"tb {i} tx 1 (combined)"
            assert f.crc_ok == expect[i][2], f"tb {i} CB flags"
    finally:
        stop.set()
        g.join(120)
    assert not errors, errors
