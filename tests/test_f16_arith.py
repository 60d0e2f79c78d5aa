"""The binary16 check-node arithmetic of the specialised decoders (ldpc_spec.h SOFT_BYTES = 2; ldpc_decode_body.h
sp::pass1 / pass2 / row_consts under LDPC_SPEC_F16, soft_f16x4, block_hard_decision16) against the int8 arithmetic
it replaces, over every input the decoder can form -- exhaustively, on the CPU (numpy float16: IEEE binary16 with
round-to-nearest-even; a fused multiply-add is emulated as one rounding of the exact float64 result). The GPU tests
then check the decoders bit for bit against the oracle."""
import numpy as np

F16 = np.float16


def h(x):
    return np.asarray(x, dtype=np.float64).astype(F16)


def fma16(a, b, c):
    """one rounding of a * b + c (v_pk_fma_f16); all operands exact binary16 values"""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F16)


def bits16(x):
    return np.asarray(x, dtype=F16).view(np.uint16).astype(np.int64)


def as16(b):
    return np.asarray(b, dtype=np.uint16).view(F16)


def i16(b):
    """a binary16 bit pattern read as a signed 16-bit integer (v_pk_min/max_i16 on the patterns)"""
    b = np.asarray(b, dtype=np.int64) & 0xFFFF
    return np.where(b >= 0x8000, b - 0x10000, b)


# ---- int8 reference arithmetic (sp::pass1 / pass2 / row_consts, LDPC_SPEC_F16 = 0) ----------------------------------
def int_pass1(s, c):
    d = s - c
    g = np.where(d < 0, -1, 1)
    af = np.minimum(d * g, 120)
    iv = s * s - 14400
    a = np.maximum(af, iv)
    return g, a


def int_row(m1, m2, sx_neg):
    n1 = (52432 * m1 + 26216) >> 16
    n2 = (52432 * m2 + 26216) >> 16
    return n1, n2 + m1, np.where(sx_neg, -1, 1)


def int_pass2(g, a, n1, cc, pp):
    f = np.maximum(n1, cc - a)
    pf = f * pp
    u = np.minimum(a + pf, 121)
    return u * g, pf * g  # soft', c2v'


# ---- binary16 arithmetic, as the kernel computes it ------------------------------------------------------------------
def f16_pass1(s, c):
    d = bits16(h(s) - h(c))
    g = d & 0x8000
    af = np.minimum(d ^ g, 0x5780)  # v_pk_min_u16 on |d|
    iv = bits16(fma16(h(s), h(s), h(-14400.0)))
    a = np.where(i16(af) >= i16(iv), af, iv)  # v_pk_max_i16
    return g, a


def f16_row(m1b, m2b, sx_neg):
    nn = fma16(as16(np.array([m1b, m2b], dtype=np.uint16).T.reshape(-1)), h(0.7998046875), h(1024.0)) - h(1024.0)
    nn = nn.reshape(-1, 2)
    n1 = bits16(nn[:, 0])
    cc = bits16(nn[:, 1] + as16(np.asarray(m1b, dtype=np.uint16)))
    ps = np.where(sx_neg, 0x8000, 0)
    return n1, cc, ps


def f16_pass2(g, a, n1, cc, ps):
    t = bits16(as16(cc) - as16(a))
    f = np.where(i16(n1) >= i16(t), n1, t) & 0xFFFF  # v_pk_max_i16
    pf = f ^ ps
    x = bits16(as16(a) + as16(pf))
    u = np.where(i16(x) <= i16(0x5790), x, 0x5790)  # v_pk_min_i16
    snew = bits16(fma16(as16(u), as16(g | 0x3C00), h(0.0)))
    cnew = pf ^ g
    return snew, cnew


def test_llr_conversion_exact():
    """soft_f16x4: 0x6580 + (b ^ 0x80) is 1536 + b in binary16, minus 1536 is b exactly (+0 for 0)"""
    b = np.arange(-121, 122)
    pat = 0x6580 + ((b & 0xFF) ^ 0x80)
    v = as16(pat) - h(1536.0)
    assert np.array_equal(v.astype(np.int64), b)
    assert bits16(v[b == 0])[0] == 0  # +0, never -0


def test_round_0_8_exact():
    """row_consts: fma(m, 0.8h, 1024) - 1024 = round(0.8 m) (gen.cpp:70-79) for every m in [0, 120]"""
    m = np.arange(0, 121)
    n = (fma16(h(m), h(0.7998046875), h(1024.0)) - h(1024.0)).astype(np.int64)
    assert np.array_equal(n, (52432 * m + 26216) >> 16)
    assert np.array_equal(n, np.floor(m * 0.8 + 0.5).astype(np.int64))


def test_pass1_matches_int8():
    """every soft value (+-121 = infinity) against every c2v value a check node can hold (|c| <= 96)"""
    s, c = np.meshgrid(np.arange(-121, 122), np.arange(-96, 97), indexing="ij")
    s, c = s.ravel(), c.ravel()
    gi, ai = int_pass1(s, c)
    gf, af = f16_pass1(s, c)
    assert np.array_equal(np.where(gf != 0, -1, 1), gi)
    assert np.array_equal(as16(af).astype(np.int64), ai)  # 241 marks infinity in both


def test_pass2_matches_int8():
    """every magnitude a (0..120 and 241), every pair of minima m1 <= m2 <= 120, both parities and signs"""
    m1, m2 = np.meshgrid(np.arange(0, 121), np.arange(0, 121), indexing="ij")
    keep = m1 <= m2
    m1, m2 = m1[keep], m2[keep]
    for sx_neg in (False, True):
        n1i, cci, ppi = int_row(m1, m2, sx_neg)
        n1f, ccf, psf = f16_row(bits16(h(m1)), bits16(h(m2)), sx_neg)
        assert np.array_equal(as16(n1f).astype(np.int64), n1i)
        assert np.array_equal(as16(ccf).astype(np.int64), cci)
        for a in list(range(0, 121)) + [241]:
            # a check node whose edge has |v2c| = a: a >= m1 always (m1 is the minimum), a == m1 or a >= m2
            ok = (a == m1) | (a >= m2)
            for gneg in (False, True):
                gi = np.full(ok.sum(), -1 if gneg else 1)
                si, ci = int_pass2(gi, np.full(ok.sum(), a), n1i[ok], cci[ok], ppi)
                sf, cf = f16_pass2(np.full(ok.sum(), 0x8000 if gneg else 0), np.full(ok.sum(), bits16(h(a))),
                                   n1f[ok], ccf[ok], psf)
                assert np.array_equal(as16(sf).astype(np.int64), si), (a, gneg, sx_neg)
                assert np.array_equal(as16(cf).astype(np.int64), ci), (a, gneg, sx_neg)
                assert not np.any(sf == 0x8000)  # soft' is never -0


def test_hard_decision16_swar():
    """block_hard_decision16 on 16-bit halves: hard = s <= 0, zero = s == 0 (no -0 in the soft bits)"""
    rng = np.random.default_rng(7)
    vals = rng.integers(-121, 122, size=4096)
    vals[::17] = 0
    pat = bits16(h(vals))
    w = (pat[0::2] | (pat[1::2] << 16)).astype(np.uint64)
    t = ((w & 0x7FFF7FFF) + 0x7FFF7FFF) & 0xFFFFFFFF
    hard = (w | (~t & 0xFFFFFFFF)) & 0x80008000
    zero = (~t & 0xFFFFFFFF) & 0x80008000
    for k, sh in ((0, 15), (1, 31)):
        v = vals[k::2]
        assert np.array_equal(((hard >> sh) & 1).astype(bool), v <= 0)
        assert np.array_equal(((zero >> sh) & 1).astype(bool), v == 0)
