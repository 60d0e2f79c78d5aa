"""The HAL plugin over the reference's own PUSCH decoder case table (pusch_decoder_test_data.h:40-217, extracted by
tests/golden/make_pusch_cases.py into tests/golden/pusch_decoder_cases.json): all 174 (base graph, modulation,
nof_ch_symbols) configurations, each with its RV sequence {0, 2, 3, 1}, through hw_accelerator_pusch_dec in
pusch_decoder_hw_impl's call order (tests/tb_chain.HwFlow, the flow test_hal_vectortest_setup drives in C++), with
external (HBM) and host soft buffers and early stop on and off across the table. Every transmission's CB CRC flags,
iteration counts, messages and TB CRC equal the oracle flow's (tests/tb_chain.SwFlow, pusch_decoder_impl restated).

The table's .dat payloads are absent, so each case's TB is self-generated (parity unpinned for the payloads; the
configuration space is the reference's). TB size rule: G = nof_ch_symbols x Qm x nof_layers channel bits, TBS = the
largest multiple of 8 not above R G with R = 0.45 for BG2 (at most 3824 bits, the BG2 limit of TS 38.212 7.2.2) and
R = 0.6 for BG1, at least 24 bits; soft bits amp (1 - 2b) + N(0, sigma^2) quantised with amp 1 and sigma in
[1.1, 1.6] by case, so that some first transmissions fail and the retransmissions combine."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.tb_chain import HwFlow, SwFlow, TransportBlock

pytestmark = pytest.mark.gpu

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "pusch_decoder_cases.json").read_text())["cases"]


def tbs_of(c):
    G = c["nof_ch_symbols"] * c["Qm"] * c["nof_layers"]
    if c["bg"] == 2:
        return max(24, min(3824, int(0.45 * G) // 8 * 8))
    return max(24, int(0.6 * G) // 8 * 8)


def test_tbs_rule_covers_the_table():
    assert len(CASES) == 174
    assert all(c["rv_sequence"] == [0, 2, 3, 1] for c in CASES)


def test_hal_over_reference_case_table():
    from srsran_projectvtlmo_amd import hal
    repo = hal.create_ext_harq_buffer_context_repository(4096, 4096 * hal.HARQ_INCR, False)
    accs = {}
    for ext in (True, False):
        cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=ext,
                                                         harq_buffer_context=repo)
        accs[ext] = hal.create_hw_accelerator_pusch_dec_factory(cfg).create()
    abs_base, n_tx, n_combined, n_fail_first = 0, 0, 0, 0
    for k, c in enumerate(CASES):
        rng = np.random.default_rng(1000 + c["index"])
        ext, es = (k % 2) == 0, (k % 4) < 2
        tb = TransportBlock(rng, tbs_of(c), c["bg"], c["nof_ch_symbols"], c["mod"], c["nof_layers"])
        sigma = 1.1 + 0.5 * (c["index"] % 5) / 4
        sw = SwFlow(tb, nof_iters=6, early_stop=es)
        hw = HwFlow(tb, accs[ext], nof_iters=6, early_stop=es, abs_base=abs_base)
        abs_base += tb.C
        for i, rv in enumerate(c["rv_sequence"]):
            llrs = tb.llrs(rng, rv, 1.0, sigma)
            ok_sw, _ = sw.transmission(llrs, rv, new_data=(i == 0))
            ok_hw, _ = hw.transmission(llrs, rv, new_data=(i == 0))
            where = f"case {c['index']} (BG{c['bg']} {c['mod']} {c['nof_ch_symbols']} sym, TBS {tb.tbs}, C {tb.C}, " \
                    f"ext {ext}, ET {es}) rv {rv}"
            assert ok_sw == ok_hw, where + ": TB CRC"
            assert sw.crc_ok == hw.crc_ok and sw.iters_used == hw.iters_used, where + ": CB flags / iterations"
            for r in range(tb.C):
                np.testing.assert_array_equal(sw.msgs[r], hw.msgs[r], err_msg=where + f" cb {r}")
            n_tx += 1
            n_combined += i > 0
            n_fail_first += (i == 0 and not ok_sw)
            if ok_sw:
                break
        if ext:
            for r in range(tb.C):
                accs[True].free_harq_context_entry(hw.abs_ids[r])
    print(f"{len(CASES)} cases, {n_tx} transmissions, {n_combined} retransmissions combined, "
          f"{n_fail_first} first transmissions failed")
    assert n_combined >= 20, "the noise levels must leave retransmissions to combine"
