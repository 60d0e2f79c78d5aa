"""CPU tests pinning the oracle (oracle/ldpc_oracle.c) to the reference's own known-answer tests and to
independent properties. The reference's golden .dat fixtures are absent and the reference may not be built or run
(SURVEY.md §8c), so these are the pins; see DESIGN.md "Oracle"."""
import numpy as np
import pytest

import oracle as O


# ---- log_likelihood_ratio_test.cpp:32-87 --------------------------------------------------------------------------
def test_llr_known_answers():
    llr0, llr1 = 0, 2
    assert O.llr_add(llr0, llr1) == 2                      # :45
    assert O.llr_sub(llr0, llr1) == -2                     # :46
    assert O.llr_promotion_sum(llr0, llr1) == 2            # :47
    assert O.llr_add(llr1, 119) == 120                     # LLR_MAX == llr1 + 119, :48
    llr0 = O.llr_add(llr0, llr1)                           # :50
    assert llr0 == 2
    assert O.llr_sub(llr0, llr1) == 0                      # special case 0, :52
    assert O.llr_sub(127, llr1) == 127                     # INFTY - finite, :53
    assert O.llr_add(llr0, 127) == 127                     # finite + INFTY, :54
    assert O.llr_sub(127, 127) == 0                        # INFTY - INFTY, :55
    assert O.llr_sub(-100, 100) == -120                    # negative saturation, :63
    assert O.llr_promotion_sum(120, 120) == 127            # :64
    assert O.llr_promotion_sum(127, 120) == 127            # :65


def test_llr_arithmetic_exhaustive_properties():
    """Over valid LLR values ([-120, 120] and +-127, log_likelihood_ratio.h constructor): the special-case rules of
    log_likelihood_ratio.cpp:39-86."""
    valid = list(range(-120, 121, 3)) + [-127, 127, 120, -120]
    for a in valid:
        for b in valid:
            s = O.llr_add(a, b)
            p = O.llr_promotion_sum(a, b)
            if a == -b:
                assert s == 0 and p == 0
            elif abs(a) > 120:
                assert s == a and p == a
            elif abs(b) > 120:
                assert s == b and p == b
            else:
                assert s == max(-120, min(120, a + b))
                assert p == (a + b if abs(a + b) <= 120 else (127 if a + b > 0 else -127))
            assert O.llr_add(a, b) == O.llr_add(b, a)


def test_quantize():
    """log_likelihood_ratio::quantize (log_likelihood_ratio.cpp:88-97)."""
    assert O.llr_quantize(8.0, 8.0) == 120
    assert O.llr_quantize(-100.0, 8.0) == -120
    assert O.llr_quantize(0.0, 8.0) == 0
    x = np.linspace(-10, 10, 1001).astype(np.float32)
    q = O.quantize_array(x, 8.0)
    assert all(q[i] == O.llr_quantize(float(x[i]), 8.0) for i in range(0, 1001, 7))


# ---- hard_decision_test.cpp:51-78 ---------------------------------------------------------------------------------
def test_hard_decision_packing():
    rng = np.random.default_rng(1234)
    for _ in range(100):
        n = int(rng.integers(1, 1000))
        llr = rng.integers(-127, 128, n).astype(np.int8)
        packed, ok = O.hard_decision(llr)
        bits = np.unpackbits(packed)[:n]
        np.testing.assert_array_equal(bits, (llr <= 0).astype(np.uint8))  # to_hard_bit: llr <= 0 -> 1
        assert ok == (not np.any(llr == 0))


# ---- crc_calculator_test.cpp:32-110 (bitwise golden) --------------------------------------------------------------
POLYS = {O.CRC24A: (24, 0x1864CFB), O.CRC24B: (24, 0x1800063), O.CRC24C: (24, 0x1B2B117), O.CRC16: (16, 0x11021),
         O.CRC11: (11, 0xE21), O.CRC6: (6, 0x61)}


def _crc_py(bits, order, poly):
    rem = 0
    for b in list(bits) + [0] * order:
        rem = (rem << 1) | int(b)
        if rem >> order & 1:
            rem ^= poly
    return rem


@pytest.mark.parametrize("poly", list(POLYS))
def test_crc_vs_bitwise_golden(poly):
    order, g = POLYS[poly]
    rng = np.random.default_rng(poly)
    for n in (1, 7, 8, 31, 100, 257):
        bits = rng.integers(0, 2, n).astype(np.uint8)
        ref = _crc_py(bits, order, g)
        assert O.crc_bits(poly, bits) == ref
        assert O.crc_packed(poly, np.packbits(bits), n) == ref


@pytest.mark.parametrize("poly", [O.CRC24A, O.CRC24B, O.CRC16])
def test_crc_appended_checks_to_zero(poly):
    """The decoder's early-stop test: a message with its CRC appended has remainder 0 (ldpc_decoder_impl.cpp:131)."""
    order, _ = POLYS[poly]
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2, 500).astype(np.uint8)
    c = O.crc_bits(poly, bits)
    full = np.concatenate([bits, [(c >> (order - 1 - i)) & 1 for i in range(order)]]).astype(np.uint8)
    assert O.crc_bits(poly, full) == 0


# ---- graph tables ---------------------------------------------------------------------------------------------------
def test_graph_shapes_and_lifting():
    n1 = sum(len(O.graph_row(1, 384, m)[0]) for m in range(46))
    n2 = sum(len(O.graph_row(2, 384, m)[0]) for m in range(42))
    assert (n1, n2) == (316, 197)  # ldpc_luts_impl.cpp:4383-4519 adjacency
    assert O.lifting_index(384) == 1 and O.lifting_index(208) == 6 and O.lifting_index(52) == 6
    assert O.lifting_index(36) == 4 and O.lifting_index(17) == -1
    # rows m >= 4 carry exactly one extension column K + m with shift 0 (ldpc_decoder_impl.cpp:204-218)
    for bg, M, K in ((1, 46, 22), (2, 42, 10)):
        for m in range(4, M):
            cols, sh = O.graph_row(bg, 384, m)
            assert cols[-1] == K + m and sh[-1] == 0 and all(c < K + 4 for c in cols[:-1])


# ---- encoder: parity checks (independent of the encoder's own algebra) ---------------------------------------------
@pytest.mark.parametrize("bg,Z", [(1, 2), (1, 384), (2, 52), (2, 3), (1, 105 // 7 * 7 if False else 112)])
def test_encoder_satisfies_parity_checks(bg, Z):
    rng = np.random.default_rng(Z)
    K, M = O.BG_K[bg], O.BG_M[bg]
    msg = rng.integers(0, 2, K * Z).astype(np.uint8)
    cw = O.ldpc_encode(bg, Z, msg)                     # shortened: full codeblock bits [2Z, 2Z + N_short Z)
    full = np.concatenate([msg[:2 * Z], cw])
    for m in range(M):
        cols, sh = O.graph_row(bg, Z, m)
        acc = np.zeros(Z, dtype=np.uint8)
        for c, s in zip(cols, sh):
            acc ^= np.roll(full[c * Z:(c + 1) * Z], -s)   # row (m, t) touches bit (c, (t + s) mod Z)
        assert not acc.any(), f"row {m}"


# ---- decoder known answers (ldpc_enc_dec_test.cpp:287-358) ---------------------------------------------------------
@pytest.mark.parametrize("bg,Z", [(2, 52), (1, 20), (2, 208)])
def test_decoder_round_trip_and_zero_rules(bg, Z):
    rng = np.random.default_rng(3)
    K, N = O.BG_K[bg], O.BG_N_SHORT[bg]
    msg = rng.integers(0, 2, K * Z).astype(np.uint8)
    msg[K * Z - 12:] = O.FILLER_BIT
    cw = O.ldpc_encode(bg, Z, msg)
    for L in ((K + 2) * Z, (K + 2) * Z + 5, N * Z):
        llr = np.where(cw[:L] == 1, -10, 10).astype(np.int8)
        out, it = O.ldpc_decode(bg, Z, llr, 1, nof_filler_bits=12)
        bits = np.unpackbits(out)[:K * Z]
        assert np.all((bits == msg) | ((msg == O.FILLER_BIT) & (bits == 0))) and it is None
    zero = np.zeros(N * Z, dtype=np.int8)
    out, it = O.ldpc_decode(bg, Z, zero, 6)
    assert it is None and np.all(np.unpackbits(out)[:K * Z] == 1)
    sentinel = np.full((K * Z + 7) // 8, 0x5A, dtype=np.uint8)
    out, it = O.ldpc_decode(bg, Z, zero, 6, crc_poly=O.CRC24B, out=sentinel.copy())
    assert it is None and np.all(out == 0x5A)
    almost = np.zeros(N * Z, dtype=np.int8)
    for i in range((K + 2) * Z + 2, N * Z, 3):
        almost[i] = 1 if i % 2 == 0 else -1
    out, _ = O.ldpc_decode(bg, Z, almost, 6)
    assert np.all(np.unpackbits(out)[:K * Z] == 1)


def test_decoder_contract_violations():
    with pytest.raises(ValueError):
        O.ldpc_decode(1, 384, np.zeros(100, np.int8), 8)             # too short
    with pytest.raises(ValueError):
        O.ldpc_decode(1, 384, np.ones(66 * 384 + 1, np.int8), 8)     # too long
    with pytest.raises(ValueError):
        O.ldpc_decode(1, 17, np.ones(66 * 17, np.int8), 8)           # invalid lifting size


def test_early_stop_with_crc():
    rng = np.random.default_rng(9)
    from tests.vectors import codeword_llrs
    llr, msg = codeword_llrs(rng, 2, 208, 2.0, 0.5, crc=O.CRC24B)
    out, it = O.ldpc_decode(2, 208, llr, 10, crc_poly=O.CRC24B)
    assert it is not None and 1 <= it <= 10
    assert np.array_equal(np.unpackbits(out)[:2080], msg)


# ---- rate matching round trip (ldpc_rm_test.cpp:124-212) -----------------------------------------------------------
@pytest.mark.parametrize("bg,Z,E,rv,Qm,F,Nref", [(1, 384, 9728, 0, 8, 0, 0), (2, 36, 1248, 0, 2, 88, 0),
                                                 (2, 52, 3000, 2, 4, 20, 0), (1, 52, 1500, 3, 6, 0, 2000),
                                                 (2, 208, 4000, 1, 1, 100, 0), (1, 20, 3000, 0, 2, 0, 0)])
def test_rate_match_dematch_round_trip(bg, Z, E, rv, Qm, F, Nref):
    """rate_match(rate_dematch(llr(bits))) == bits; filler bits <-> +inf (ldpc_rm_test.cpp:191-211)."""
    rng = np.random.default_rng(E + rv)
    K, N = O.BG_K[bg], O.BG_N_SHORT[bg] * Z
    msg = rng.integers(0, 2, K * Z).astype(np.uint8)
    if F:
        msg[K * Z - F:] = O.FILLER_BIT
    cw = O.ldpc_encode(bg, Z, msg)
    matched = O.rate_match(cw, E, rv, Qm, Nref, bg, Z)
    llr = np.where(matched == 1, -10, 10).astype(np.int8)
    buf = np.zeros(N, dtype=np.int8)
    O.rate_dematch(buf, llr, True, rv, Qm, Nref, F)
    nsys, ninfo = (K - 2) * Z, (K - 2) * Z - F
    assert np.all(buf[ninfo:nsys] == 127)                      # filler -> +inf
    # hard decisions of the dematched buffer re-match to the transmitted bits
    hard = np.where(buf < 0, 1, 0).astype(np.uint8)
    hard[ninfo:nsys] = O.FILLER_BIT
    assert np.array_equal(O.rate_match(hard, E, rv, Qm, Nref, bg, Z), matched)


def test_rate_dematch_combining_saturates():
    """Second transmission combines with saturated '+' (ldpc_rate_dematcher_impl.cpp:116-126)."""
    N = 50 * 52
    buf = np.zeros(N, dtype=np.int8)
    llr = np.full(1000, 100, dtype=np.int8)
    O.rate_dematch(buf, llr, True, 0, 2, 0, 0)
    O.rate_dematch(buf, llr, False, 0, 2, 0, 0)
    assert buf[0] == 120 and buf[999] == 120 and buf[1000] == 0


# ---- segmenter (ldpc_segmenter_impl.cpp:254-331) ------------------------------------------------------------------
def test_segmenter_c4_slot():
    """UE0 TBS 1,078,248, BG1, 4 layers 256QAM on 250 PRB x 156 RE."""
    metas = O.segment_rx(1078248, 1, 250 * 156 * 4, 8, 4)
    assert len(metas) == 128 and metas[0]["Z"] == 384 and metas[0]["nof_filler_bits"] == 0
    Es = sorted({m["rm_length"] for m in metas})
    assert Es == [9728, 9760] and sum(m["rm_length"] for m in metas) == 250 * 156 * 4 * 8
    assert sum(1 for m in metas if m["rm_length"] == 9728) == 40
    small = O.segment_rx(256, 2, 156 * 4, 2, 4)
    assert len(small) == 1 and small[0]["Z"] == 36 and small[0]["nof_filler_bits"] == 88
    assert small[0]["rm_length"] == 1248 and small[0]["nof_crc_bits"] == 16


def test_tb_join_matches_transport_block():
    """join_and_notify / concatenate_codeblocks (pusch_decoder_impl.cpp:384-497) on error-free CB messages: the TB
    comes back bit-exact with a passing TB CRC; a flipped data bit fails the TB CRC24A; a failed CB CRC leaves the
    TB untouched."""
    from tests.tb_chain import TransportBlock
    rng = np.random.default_rng(5)
    for tbs, bg, syms in ((20496, 1, 10000), (3000, 2, 3000), (256, 2, 624), (60000, 1, 30000)):
        tb = TransportBlock(rng, tbs, bg, syms, "QAM16", 2)
        KZ = tb.K * tb.Z
        msgs = np.zeros((tb.C, (KZ + 7) // 8), np.uint8)
        for r, m in enumerate(tb.msgs):
            bits = np.where(m == O.FILLER_BIT, 0, m).astype(np.uint8)
            msgs[r] = np.packbits(bits)[: msgs.shape[1]]
        cb_crc_bits = tb.cb_crc_len if tb.C > 1 else tb.tb_crc_len
        out, ok = O.tb_join(msgs, KZ, tb.F, cb_crc_bits, tbs, [1] * tb.C)
        assert ok
        assert np.array_equal(np.unpackbits(out)[:tbs], tb.data)
        if tb.C > 1:
            bad = msgs.copy()
            bad[0, 0] ^= 0x80
            _, ok = O.tb_join(bad, KZ, tb.F, cb_crc_bits, tbs, [1] * tb.C)
            assert not ok
        flags = [1] * tb.C
        flags[-1] = 0
        out2 = np.full_like(out, 0x5A)
        _, ok = O.tb_join(msgs, KZ, tb.F, cb_crc_bits, tbs, flags, out2)
        assert not ok and np.all(out2 == 0x5A)


def test_cpu_port_matches_oracle():
    """The vectorisable CPU port (bench.py's cpu_baseline) is bit-exact with the oracle: random and codeword LLRs,
    both base graphs, several lifting sizes, short lengths, CRC early stop."""
    from tests.vectors import codeword_llrs, random_llrs
    rng = np.random.default_rng(17)
    for bg, Z in ((1, 384), (2, 208), (1, 36), (2, 52), (1, 7), (2, 15), (1, 104), (2, 384)):
        N = O.BG_N_SHORT[bg] * Z
        for kind in ("pm10", "mixed"):
            llr = random_llrs(rng, N, kind)
            for it in (1, 3, 8):
                a, ra = O.ldpc_decode(bg, Z, llr, it)
                b, rb = O.ldpc_decode_port(bg, Z, llr, it)
                assert np.array_equal(a, b) and ra == rb, (bg, Z, kind, it)
        L = (O.BG_K[bg] + 2) * Z + Z // 2 + 1      # short, non-multiple of Z
        llr = random_llrs(rng, L, "mixed")
        assert np.array_equal(O.ldpc_decode(bg, Z, llr, 4)[0], O.ldpc_decode_port(bg, Z, llr, 4)[0])
        if O.BG_K[bg] * Z > 64:
            llr, _ = codeword_llrs(rng, bg, Z, 2.0, 1.2, crc=O.CRC24B)
            a, ra = O.ldpc_decode(bg, Z, llr, 10, O.CRC24B)
            b, rb = O.ldpc_decode_port(bg, Z, llr, 10, O.CRC24B)
            assert np.array_equal(a, b) and ra == rb


def test_port_crc_matches_oracle_crc():
    """The CPU port's table-driven CRC (orc_crc_port) gives the oracle's bit-serial remainder
    (crc_calculator_generic_impl.cpp:111-133) for CRC24A/24B/16 on every length from 1 to 2 bytes past a word, and on
    long messages; early stop with CRC16 and CRC24A matches the oracle's decoder too."""
    import ctypes

    from tests.vectors import codeword_llrs
    rng = np.random.default_rng(23)
    L = O.lib()
    for poly in (O.CRC24A, O.CRC24B, O.CRC16):
        for nbits in list(range(1, 80)) + [8447, 8448, 3824, 1000]:
            msg = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
            p = msg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
            assert L.orc_crc_port(poly, p, nbits) == L.orc_crc_packed(poly, p, nbits), (poly, nbits)
    for bg, Z, poly in ((2, 36, O.CRC16), (1, 384, O.CRC24A), (2, 52, O.CRC16)):
        llr, _ = codeword_llrs(rng, bg, Z, 2.0, 1.2, crc=poly)
        a, ra = O.ldpc_decode(bg, Z, llr, 10, poly)
        b, rb = O.ldpc_decode_port(bg, Z, llr, 10, poly)
        assert np.array_equal(a, b) and ra == rb, (bg, Z)
