"""CPU tests of the host-side TB bookkeeping (srsran_projectvtlmo_amd.segmentation) against the oracle restatements:
RX segmentation metadata (ldpc_segmenter_impl.cpp:254-331), CRC (crc_calculator_generic_impl.cpp) and TX segmentation
(TS 38.212 5.1-5.2 as built by tests/tb_chain.TransportBlock)."""
import numpy as np

import oracle as O
from srsran_projectvtlmo_amd import segmentation as S
from tests.tb_chain import TransportBlock

ORC_CRC = {"CRC24A": O.CRC24A, "CRC24B": O.CRC24B, "CRC16": O.CRC16}


def test_crc_matches_oracle():
    rng = np.random.default_rng(3)
    for name, poly in ORC_CRC.items():
        for n in (1, 7, 8, 9, 100, 2056, 8424):
            bits = rng.integers(0, 2, n).astype(np.uint8)
            assert S.crc_bits(name, bits) == O.crc_bits(poly, bits), (name, n)


def test_segment_rx_matches_oracle():
    rng = np.random.default_rng(4)
    for _ in range(300):
        bg = int(rng.integers(1, 3))
        tbs = int(rng.integers(3, 40000)) * 8
        layers = int(rng.integers(1, 5))
        Qm = int(rng.choice([2, 4, 6, 8]))
        syms = layers * int(rng.integers(100, 20000))
        ref = O.segment_rx(tbs, bg, syms, Qm, layers)
        got = S.segment_rx(tbs, bg, syms, Qm, layers)
        assert len(got) == len(ref)
        for g, r in zip(got, ref):
            assert (g.lifting_size, g.nof_filler_bits, g.rm_length, g.cw_offset, g.full_length, g.nof_crc_bits) == (
                r["Z"], r["nof_filler_bits"], r["rm_length"], r["cw_offset"], r["full_length"], r["nof_crc_bits"])


def test_segment_tx_matches_transport_block():
    rng = np.random.default_rng(5)
    for tbs, bg, syms in ((60000, 1, 30000), (3000, 2, 1500), (256, 2, 624)):
        tb = TransportBlock(rng, tbs, bg, syms, "QAM16", 2)
        msgs = S.segment_tx(tb.data, S.segment_rx(tbs, bg, syms, 4, 2))
        for r in range(tb.C):
            assert np.array_equal(msgs[r], np.where(tb.msgs[r] == O.FILLER_BIT, 0, tb.msgs[r]))
