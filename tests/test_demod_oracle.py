"""CPU tests of the soft-demodulation restatement (oracle/ldpc_oracle.c orc_demodulate_soft).

The reference's demodulation_mapper_test.cpp compares against MATLAB .dat vectors that are absent from the snapshot,
so these LLRs are pinned by (i) the reference test's own special-case rules (noise variance 0 / inf / negative / NaN
-> LLR 0, symbol 0 -> LLR 0, infinite symbols stay in range: demodulation_mapper_test.cpp:128-346), (ii) the
TS 38.211 §5.1 constellation: noiseless symbols give the transmitted bits as hard decisions, and (iii) an independent
numpy float32 restatement of the same per-symbol functions (bit-exact)."""
import numpy as np
import pytest

import oracle as O
from tests.vectors import modulate, noisy_symbols

MODS = [0, 1, 2, 4, 6, 8]


def _qm(mod):
    return O.bits_per_symbol(mod)


def _np_quantize(v, r):
    return O.quantize_array(v, r)


def _np_interval(x, rn, width, nof, sl, ic):
    f32 = np.float32
    q = np.floor((x / f32(width)).astype(np.float32))
    idx = np.where(np.isfinite(q) & (np.abs(q) < 2.0 ** 31), q, -2.0 ** 31)
    idx = np.clip(np.maximum(idx, -nof) + nof // 2, 0, nof - 1).astype(np.int64)
    sl = np.asarray(sl, np.float32)
    ic = np.asarray(ic, np.float32)
    return ((sl[idx] * x).astype(np.float32) + ic[idx]).astype(np.float32) * f32(rn)


def _np_demod(mod, sym, nv):
    """Independent numpy float32 restatement (no FMA: numpy rounds every op)."""
    f32 = np.float32
    re, im = sym.real.astype(np.float32), sym.imag.astype(np.float32)
    n = sym.size
    qm = _qm(mod)
    out = np.zeros((n, qm), np.int8)
    gain = f32(2.0) * f32(1.41421356237309504880)
    with np.errstate(all="ignore"):
        if mod in (0, 1):
            r, i = re.copy(), im.copy()
            if mod == 0:
                r[1::2], i[1::2] = im[1::2], -re[1::2]
            l = (gain * (r + i)).astype(np.float32) / nv
            out[:, 0] = np.where(nv > 0, _np_quantize(l, 24), 0)
            return out.ravel()
        if mod == 2:
            for c, x in enumerate((re, im)):
                out[:, c] = np.where(nv > 0, _np_quantize((gain * x).astype(np.float32) / nv, 24), 0)
            return out.ravel()
        near0 = (re * re + im * im) < f32(1e-9)
        if mod == 4:
            s10 = f32(1.0) / np.sqrt(f32(10.0))
            for c, x in enumerate((re, im)):
                l01 = ((f32(4) * s10) * x).astype(np.float32)
                l01 = np.where(np.abs(x) > f32(2) * s10, f32(2) * l01 - np.copysign(f32(0.8), x), l01)
                l01 = (l01 / nv).astype(np.float32)
                l23 = ((f32(0.8) - (f32(4) * s10) * np.abs(x)) / nv).astype(np.float32)
                out[:, c] = np.where(nv > 0, _np_quantize(l01, 24), 0)
                out[:, 2 + c] = np.where(nv > 0, _np_quantize(l23, 24), 0)
        else:
            rn = np.where(nv > 0, f32(1) / nv, f32(0)).astype(np.float32)
            if mod == 6:
                s = f32(1.0) / np.sqrt(f32(42.0))
                tabs = [(2 * s, 8, [16, 12, 8, 4, 4, 8, 12, 16], [24, 12, 4, 0, 0, -4, -12, -24]),
                        (2 * s, 8, [8, 4, 4, 8, -8, -4, -4, -8], [20, 8, 8, 12, 12, 8, 8, 20]),
                        (4 * s, 4, [4, -4, 4, -4], [12, -4, -4, 12])]
                den = f32(21)
            else:
                s = f32(1.0) / np.sqrt(f32(170.0))
                tabs = [(2 * s, 16, [32, 28, 24, 20, 16, 12, 8, 4, 4, 8, 12, 16, 20, 24, 28, 32],
                         [112, 84, 60, 40, 24, 12, 4, 0, 0, -4, -12, -24, -40, -60, -84, -112]),
                        (2 * s, 16, [16, 12, 8, 4, 4, 8, 12, 16, -16, -12, -8, -4, -4, -8, -12, -16],
                         [88, 60, 36, 16, 16, 28, 36, 40, 40, 36, 28, 16, 16, 36, 60, 88]),
                        (2 * s, 16, [8, 4, 4, 8, -8, -4, -4, -8, 8, 4, 4, 8, -8, -4, -4, -8],
                         [52, 24, 24, 44, -20, -8, -8, -12, -12, -8, -8, -20, 44, 24, 24, 52]),
                        (4 * s, 8, [4, -4, 4, -4, 4, -4, 4, -4], [28, -20, 12, -4, -4, 12, -20, 28])]
                den = f32(85)
            for j, (w, nof, k, ic) in enumerate(tabs):
                sl = [f32(kk) * s for kk in k]
                icf = [f32(v) / den for v in ic]
                for c, x in enumerate((re, im)):
                    out[:, 2 * j + c] = _np_quantize(_np_interval(x, rn, np.float32(w), nof, sl, icf), 20)
        out[near0] = 0
    return out.ravel()


@pytest.mark.parametrize("mod", MODS)
def test_oracle_matches_numpy_restatement(mod):
    rng = np.random.default_rng(mod)
    _, sym, nv = noisy_symbols(rng, 4099, mod, noise_var=0.08)
    sym[::37] = 0  # near-zero symbols
    nv[5::101] = 0.0
    nv[7::103] = -2.0
    nv[9::107] = np.inf
    nv[11::109] = np.nan
    assert np.array_equal(O.demodulate_soft(mod, sym, nv), _np_demod(mod, sym, nv))


@pytest.mark.parametrize("mod", MODS)
def test_noiseless_constellation_hard_bits(mod):
    """TS 38.211 §5.1: the hard decision (LLR <= 0 -> 1, log_likelihood_ratio.h:86) of a clean symbol is its bit."""
    rng = np.random.default_rng(10 + mod)
    qm = _qm(mod)
    bits = rng.integers(0, 2, 2048 * qm).astype(np.uint8)
    sym = modulate(bits, mod)
    llr = O.demodulate_soft(mod, sym, np.full(sym.size, 0.01, np.float32))
    assert np.all(llr != 0)
    assert np.array_equal((llr <= 0).astype(np.uint8), bits)


@pytest.mark.parametrize("mod", MODS)
@pytest.mark.parametrize("bad", [0.0, np.inf, -2.0, np.nan])
def test_bad_noise_gives_zero_llrs(mod, bad):
    """demodulation_mapper_test.cpp DemodulatorNoiseZero/Infinity/Negative/NaN: even-indexed symbols with a bad
    noise variance give LLR 0, the others are unaffected."""
    rng = np.random.default_rng(3)
    _, sym, nv = noisy_symbols(rng, 18, mod)
    ref = O.demodulate_soft(mod, sym, nv).reshape(18, -1)
    nv2 = nv.copy()
    nv2[::2] = bad
    got = O.demodulate_soft(mod, sym, nv2).reshape(18, -1)
    assert np.all(got[::2] == 0)
    assert np.array_equal(got[1::2], ref[1::2])


@pytest.mark.parametrize("mod", MODS)
def test_infinite_symbols_stay_in_range(mod):
    """demodulation_mapper_test.cpp DemodulatorSymbolInfinity."""
    rng = np.random.default_rng(4)
    _, sym, nv = noisy_symbols(rng, 18, mod)
    ref = O.demodulate_soft(mod, sym, nv).reshape(18, -1)
    inf = np.float32(np.inf)
    bad = [complex(inf, 0), complex(-inf, 0), complex(0, inf), complex(0, -inf), complex(inf, -inf),
           complex(inf, inf), complex(-inf, 0), complex(0, inf), complex(0, -inf)]
    for k, b in enumerate(bad):
        sym[2 * k] = b
    got = O.demodulate_soft(mod, sym, nv).reshape(18, -1)
    assert np.all((got[::2] >= -120) & (got[::2] <= 120))
    assert np.array_equal(got[1::2], ref[1::2])


@pytest.mark.parametrize("mod", [4, 6, 8])
def test_zero_symbols_give_zero_llrs(mod):
    """demodulation_mapper_test.cpp DemodulatorSymbolZero (the QAM scalar paths' is_near_zero rule)."""
    rng = np.random.default_rng(5)
    _, sym, nv = noisy_symbols(rng, 600, mod)
    sym[::12] = 0
    got = O.demodulate_soft(mod, sym, nv).reshape(600, -1)
    assert np.all(got[::12] == 0)
