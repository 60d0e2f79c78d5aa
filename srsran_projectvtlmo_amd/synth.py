"""Device-side synthesis of PUSCH soft bits for benchmarks and examples (no oracle involved): CB messages are encoded
and rate-matched on the GPU (ldpc_hip_encode_launch / ldpc_hip_rate_match_launch), mapped to BPSK-like amplitudes
amp * (1 - 2 b), disturbed with Gaussian noise and quantised like log_likelihood_ratio::quantize (llr.cpp:88-97:
round(clip(x, +-R) / R * 120), R = 8). torch provides the device buffers, the noise and the element-wise maths."""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import _lib
from . import channel_coding as cc


def _quantize(x, rng: float = 8.0):
    import torch
    return torch.round(torch.clamp(x, -rng, rng) / rng * 120.0).to(torch.int8)


def _unpack(packed, nbits: int):
    import torch
    shifts = torch.arange(7, -1, -1, device=packed.device, dtype=torch.uint8)
    return ((packed.unsqueeze(-1) >> shifts) & 1).reshape(-1)[:nbits]


def encode_messages(ctx: _lib.Context, bg: int, Z: int, msgs_bits: np.ndarray, cw_length: Optional[int] = None,
                    stream: int = 0):
    """(C, K*Z) unpacked messages -> device tensor (C, cw_bytes) of packed shortened codewords and the stride."""
    import torch
    C, KZ = msgs_bits.shape
    L = cw_length if cw_length is not None else cc.BG_N_SHORT[bg] * Z
    mstride = ((KZ + 7) // 8 + 15) // 16 * 16
    cstride = ((L + 7) // 8 + 15) // 16 * 16
    h = np.zeros((C, mstride), np.uint8)
    h[:, : (KZ + 7) // 8] = np.packbits(msgs_bits.astype(np.uint8), axis=1)
    d_msg = torch.from_numpy(h).cuda()
    d_cw = torch.zeros((C, cstride), dtype=torch.uint8, device="cuda")
    specs = [cc.cb_encode_spec(bg, Z, L, i * mstride, i * cstride) for i in range(C)]
    cc.encode_launch(ctx, specs, d_msg.data_ptr(), d_cw.data_ptr(), stream)
    return d_cw, cstride, L


def codeword_llrs(ctx: _lib.Context, bg: int, Z: int, msgs_bits: np.ndarray, amp: float, noise: float, seed: int,
                  stream: int = 0):
    """Full shortened codewords (N_short * Z soft bits per CB), as the decoder's input without rate matching."""
    import torch
    d_cw, cstride, L = encode_messages(ctx, bg, Z, msgs_bits, None, stream)
    torch.cuda.synchronize()
    g = torch.Generator(device="cuda").manual_seed(seed)
    bits = torch.stack([_unpack(d_cw[i], L) for i in range(d_cw.shape[0])])
    x = (1.0 - 2.0 * bits.float()) * amp + noise * torch.randn(bits.shape, device="cuda", generator=g)
    return _quantize(x)


def rate_matched_llrs(ctx: _lib.Context, bg: int, Z: int, msgs_bits: np.ndarray, rm_lengths: Sequence[int],
                      Qm: int, rv: int, nof_filler_bits: int, amp: float, noise: float, seed: int, Nref: int = 0,
                      stream: int = 0):
    """Encode, rate-match every CB to its E_r, and return the list of per-CB device int8 soft-bit tensors."""
    import torch
    C = msgs_bits.shape[0]
    d_cw, cstride, N = encode_messages(ctx, bg, Z, msgs_bits, None, stream)
    offs, o = [], 0
    for E in rm_lengths:
        offs.append(o)
        o += ((E + 7) // 8 + 15) // 16 * 16
    d_e = torch.zeros(max(16, o), dtype=torch.uint8, device="cuda")
    specs = [cc.cb_rate_match_spec(N, E, Qm, rv, Nref, nof_filler_bits, i * cstride, offs[i])
             for i, E in enumerate(rm_lengths)]
    cc.rate_match_launch(ctx, specs, d_cw.data_ptr(), d_e.data_ptr(), stream)
    torch.cuda.synchronize()
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = []
    for i, E in enumerate(rm_lengths):
        bits = _unpack(d_e[offs[i]:offs[i] + (E + 7) // 8], E)
        x = (1.0 - 2.0 * bits.float()) * amp + noise * torch.randn((E,), device="cuda", generator=g)
        out.append(_quantize(x))
    return out


def modulate(bits, mod: int):
    """TS 38.211 §5.1 modulation of a device bit tensor (QPSK, 16/64/256-QAM; modulation_scheme values 2/4/6/8) into
    complex64 symbols (torch), for the symbol-fed slot (SlotPipeline.upload_symbols_device)."""
    import torch
    s = (1.0 - 2.0 * bits.float()).reshape(-1, mod)
    if mod == 2:
        re, im, norm = s[:, 0], s[:, 1], 2.0
    elif mod == 4:
        re, im, norm = s[:, 0] * (2 - s[:, 2]), s[:, 1] * (2 - s[:, 3]), 10.0
    elif mod == 6:
        re, im, norm = s[:, 0] * (4 - s[:, 2] * (2 - s[:, 4])), s[:, 1] * (4 - s[:, 3] * (2 - s[:, 5])), 42.0
    elif mod == 8:
        re = s[:, 0] * (8 - s[:, 2] * (4 - s[:, 4] * (2 - s[:, 6])))
        im = s[:, 1] * (8 - s[:, 3] * (4 - s[:, 5] * (2 - s[:, 7])))
        norm = 170.0
    else:
        raise ValueError("modulation")
    return torch.complex(re, im) / float(np.sqrt(norm))


def rate_matched_symbols(ctx: _lib.Context, bg: int, Z: int, msgs_bits: np.ndarray, rm_lengths: Sequence[int],
                         Qm: int, rv: int, nof_filler_bits: int, noise_var: float, seed: int, Nref: int = 0,
                         stream: int = 0):
    """Encode and rate-match every CB, concatenate the codeword, modulate (TS 38.211 §5.1) and add complex AWGN of
    variance noise_var: (device complex64 symbols, device float32 noise variances) of the TB's codeword."""
    import torch
    C = msgs_bits.shape[0]
    d_cw, cstride, N = encode_messages(ctx, bg, Z, msgs_bits, None, stream)
    offs, o = [], 0
    for E in rm_lengths:
        offs.append(o)
        o += ((E + 7) // 8 + 15) // 16 * 16
    d_e = torch.zeros(max(16, o), dtype=torch.uint8, device="cuda")
    specs = [cc.cb_rate_match_spec(N, E, Qm, rv, Nref, nof_filler_bits, i * cstride, offs[i])
             for i, E in enumerate(rm_lengths)]
    cc.rate_match_launch(ctx, specs, d_cw.data_ptr(), d_e.data_ptr(), stream)
    torch.cuda.synchronize()
    bits = torch.cat([_unpack(d_e[offs[i]:offs[i] + (E + 7) // 8], E) for i, E in enumerate(rm_lengths)])
    z = modulate(bits, Qm)
    g = torch.Generator(device="cuda").manual_seed(seed)
    w = torch.complex(torch.randn(z.shape, device="cuda", generator=g), torch.randn(z.shape, device="cuda",
                                                                                   generator=g))
    sym = (z + w * float(np.sqrt(noise_var / 2))).to(torch.complex64)
    return sym, torch.full((sym.numel(),), noise_var, dtype=torch.float32, device="cuda")
