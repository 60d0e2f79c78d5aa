"""Full-size C4 (BASELINE.json configs[3]) on the GPU against the oracle: the n78 100 MHz
4-layer slot with UE0 (PRB 0-249, 256QAM, TBS 1,078,248: 128 BG1 CBs of Z=384, E = 9,728 / 9,760, CRC24B, a
33-chunk TB join with CRC24A) and 23 one-PRB QPSK UEs (TBS 256: BG2, Z=36, F=88, CRC16), 151 CBs in all, rv 0,
8 iterations with CRC early stop, through the device-resident slot pipeline (srsran_projectvtlmo_amd.pusch
.SlotPipeline: dematch -> decode -> TB join).

The checker is tests/tb_chain.SwFlow: pusch_decoder_impl + pusch_codeblock_decoder restated with the CPU oracle
(pusch_decoder_impl.cpp:309-497, pusch_codeblock_decoder.cpp:35-71), the per-TB flow of the reference's
pusch_decoder_vectortest.cpp:279-395. Compared bit for bit: every CB's CRC flag and iteration count, every TB's CRC
flag, and every TB's bytes. Run twice: from LLRs, and from equalised symbols with the soft demodulation fused into the
dematcher (ldpc_hip_demod_dematch_launch), where the oracle demodulates the same symbols (demodulation_mapper)."""
import numpy as np
import pytest

import oracle as O
from tests.tb_chain import SwFlow, TransportBlock
from tests.vectors import modulate

pytestmark = pytest.mark.gpu

C4_UES = [(1078248, 1, 250 * 156 * 4, "QAM256", 4)] + [(256, 2, 156 * 4, "QPSK", 4)] * 23
MODS = {"QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


def _c4_tbs(seed):
    rng = np.random.default_rng(seed)
    tbs = [TransportBlock(rng, *ue) for ue in C4_UES]
    assert [tb.C for tb in tbs] == [128] + [1] * 23
    assert tbs[0].Z == 384 and tbs[0].F == 0 and {m["rm_length"] for m in tbs[0].metas} == {9728, 9760}
    assert all(tb.Z == 36 and tb.F == 88 and tb.metas[0]["rm_length"] == 1248 for tb in tbs[1:])
    return rng, tbs


def _pipeline(hip_ctx, tbs, iters):
    from srsran_projectvtlmo_amd import pusch
    specs = [pusch.tb_slot_spec(tb.tbs, tb.bg, tb.Z, tb.F, [m["rm_length"] for m in tb.metas], tb.Qm, 0, True, 0,
                                iters, True) for tb in tbs]
    return pusch.SlotPipeline(hip_ctx, specs)


def _compare(tbs, flows, expect, got, cbres):
    i = 0
    n_ok = 0
    for t, (tb, f, (ok, _bits), (tb_bytes, g_ok, _written)) in enumerate(zip(tbs, flows, expect, got)):
        for r in range(tb.C):
            assert bool(cbres[i + r, 0]) == f.crc_ok[r], f"tb {t} cb {r} crc"
            assert cbres[i + r, 1] == f.iters_used[r], f"tb {t} cb {r} iterations"
        i += tb.C
        assert g_ok == ok, f"tb {t}: tb_crc_ok"
        if ok:
            n_ok += 1
            assert np.array_equal(np.unpackbits(tb_bytes)[: tb.tbs], tb.data), f"tb {t}: data"
    return n_ok


@pytest.mark.parametrize("noise", [0.7, 1.0])
def test_c4_full_slot_from_llrs(hip_ctx, noise):
    """Soft bits quantize(2 (1 - 2b) + N(0, s^2), 8), 8 iterations with early stop. s = 0.7: every TB passes (the
    128-CB TB joins its 33 chunks with a passing CRC24A); s = 1.0 is SURVEY 8d's C4 recipe, at which the rate-0.87
    256QAM TB fails (some of its CBs run all 8 iterations). Both bit-exact vs the oracle flow."""
    import torch
    iters = 8
    rng, tbs = _c4_tbs(3)
    llrs = [tb.llrs(rng, 0, 2.0, noise) for tb in tbs]
    flows = [SwFlow(tb, nof_iters=iters, early_stop=True) for tb in tbs]
    expect = [f.transmission(l, 0, True) for f, l in zip(flows, llrs)]
    pipe = _pipeline(hip_ctx, tbs, iters)
    pipe.upload(llrs)
    pipe.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got, cbres = pipe.results()
    assert cbres.shape[0] == 151
    n_ok = _compare(tbs, flows, expect, got, cbres)
    if noise < 1.0:
        assert n_ok == 24 and expect[0][0]          # the 128-CB TB joins (33 chunks) with a passing CRC24A
    else:
        assert not expect[0][0] and sum(flows[0].crc_ok) < 128


def test_c4_full_slot_from_symbols(hip_ctx):
    """The same slot fed with equalised symbols (TS 38.211 modulation + complex AWGN, noise variance 0.0015 for
    256QAM and 0.1 for QPSK): fused demodulation + dematch + decode + TB join on the GPU vs oracle demodulation
    (demodulation_mapper_qam256.cpp / _qpsk.cpp restated) + the oracle flow."""
    import torch
    iters = 8
    rng, tbs = _c4_tbs(4)
    syms, nvs, llrs = [], [], []
    for tb in tbs:
        mod = MODS[tb.mod]
        bits = np.concatenate(tb.rm_bits(0))
        z = modulate(bits, mod)
        nv_val = 0.0015 if mod == 8 else 0.1
        w = (rng.standard_normal(z.size) + 1j * rng.standard_normal(z.size)) * np.sqrt(nv_val / 2)
        sym = (z + w).astype(np.complex64)
        nv = np.full(sym.size, nv_val, np.float32)
        syms.append(sym)
        nvs.append(nv)
        per_cb, o = [], 0
        for m in tb.metas:
            ns = m["rm_length"] // tb.Qm
            per_cb.append(O.demodulate_soft(mod, sym[o:o + ns], nv[o:o + ns]))
            o += ns
        llrs.append(per_cb)
    flows = [SwFlow(tb, nof_iters=iters, early_stop=True) for tb in tbs]
    expect = [f.transmission(l, 0, True) for f, l in zip(flows, llrs)]
    pipe = _pipeline(hip_ctx, tbs, iters)
    pipe.upload_symbols(syms, nvs)
    assert pipe.fuse_demod
    pipe.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got, cbres = pipe.results()
    n_ok = _compare(tbs, flows, expect, got, cbres)
    assert n_ok >= 20
