"""The software route's CPU leg (bench.py cpu_baseline_sw_route, oracle/ldpc_cpu_slot.c) on a small self-generated
slot: every codeblock's CRC passes in both modes, on one and two worker threads, and the slot blob parser round-trips
the format bench_hal / bench_sw read. CPU only."""
import struct

import numpy as np

import bench
from tests.tb_chain import TransportBlock


def _blob(tbs_list, rng):
    parts = [struct.pack("<I", len(tbs_list))]
    expect = []
    for tb in tbs_list:
        llrs = tb.llrs(rng, 0, amp=3.0, noise=0.5)
        parts.append(struct.pack("<8I", tb.tbs, tb.bg, tb.Z, tb.F, tb.C, tb.Qm, 0, 8))
        for a in llrs:
            parts.append(struct.pack("<I", a.size) + a.astype(np.int8).tobytes())
            expect.append(a)
    return b"".join(parts), expect


def test_cpu_slot_leg_decodes_every_codeblock():
    rng = np.random.default_rng(5)
    tbs = [TransportBlock(rng, 20496, 1, 156 * 24, "QAM64", 2), TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)]
    blob, expect = _blob(tbs, rng)
    cbs = bench.slot_blob_cbs(blob)
    assert len(cbs) == sum(tb.C for tb in tbs)
    for c, e in zip(cbs, expect):
        assert np.array_equal(c[7], e)
    assert cbs[0][6] == 1 and cbs[-1][6] == 3  # CRC24B for the multi-CB TB, CRC16 for the 256-bit one
    out = bench.cpu_baseline_sw_route(blob, reps=2, threads=(1, 2))
    for mode in ("decoder_only", "dematch_decode"):
        for t, r in out[mode].items():
            assert r["cbs_crc_ok"] == len(cbs), (mode, t, r)
            assert r["slot_us_p50"] > 0
