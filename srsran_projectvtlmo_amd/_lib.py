"""ctypes binding of the C ABI in include/srsran_ldpc_hip.h (libsrsran_ldpc_hip.so, built in-tree for gfx950).

The product path is the HIP library: if it is missing or cannot be loaded this module raises; there is no CPU
fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "lib" / "libsrsran_ldpc_hip.so"

OK, NOT_READY, DROPPED = 0, 1, 2
EINVAL, EDEVICE, EFULL, ENOMEM, ESTATE = -1, -2, -3, -4, -5

CRC16, CRC24B, CRC24A = 0, 1, 2          # hal::hw_dec_cb_crc_type numbering
CRC_NONE = -1
CRC_MODE_NONE, CRC_MODE_EARLY_STOP, CRC_MODE_CHECK_AFTER = 0, 1, 2
CRC_MODE_FLAG_KEEP_PASSED = 0x80
STATUS_OUTPUT_WRITTEN, STATUS_DROPPED = 0x1, 0x2

EXPORTED_SYMBOLS = [
    "ldpc_hip_open", "ldpc_hip_close", "ldpc_hip_last_error", "ldpc_hip_stream",
    "ldpc_hip_decode_plan_create", "ldpc_hip_decode_plan_destroy", "ldpc_hip_decode_launch",
    "ldpc_hip_decode_sync", "ldpc_hip_rate_dematch_sync",
    "ldpc_hip_queue_reserve", "ldpc_hip_queue_free", "ldpc_hip_enqueue", "ldpc_hip_dequeue",
    "ldpc_hip_read_outputs", "ldpc_hip_harq_free", "ldpc_hip_external_harq_supported",
    "ldpc_hip_schedule_groups", "ldpc_hip_specialised", "ldpc_hip_version",
    "ldpc_hip_rate_dematch_launch", "ldpc_hip_encode_launch", "ldpc_hip_rate_match_launch", "ldpc_hip_tb_join_launch",
    "ldpc_hip_demodulate_launch", "ldpc_hip_demodulate_sync",
    "ldpc_hip_capture_begin", "ldpc_hip_capture_end", "ldpc_hip_graph_launch", "ldpc_hip_graph_destroy",
    "ldpc_hip_demod_dematch_launch", "ldpc_hip_dematch_decode_launch",
    "ldpc_hip_enc_queue_create", "ldpc_hip_enc_queue_destroy", "ldpc_hip_enc_reserve", "ldpc_hip_enc_free",
    "ldpc_hip_enc_configure", "ldpc_hip_enc_enqueue", "ldpc_hip_enc_dequeue", "ldpc_hip_enc_cb_mode",
    "ldpc_hip_enc_max_tb_size",
    "ldpc_hip_harq_repo_create", "ldpc_hip_harq_repo_release", "ldpc_hip_harq_repo_entry", "ldpc_hip_harq_repo_read",
    "ldpc_hip_open_harq", "ldpc_hip_harq_device_memory", "ldpc_hip_harq_capacity", "ldpc_hip_auto_device",
    "ldpc_hip_decode_work", "ldpc_hip_auto_min_work",
]
HARQ_STRIDE = 25344   # LDPC_HIP_HARQ_STRIDE


# ldpc_hip_params.launch_flags (tests / diagnostics; 0 = the default launch forms)
LAUNCH_NO_SPEC, LAUNCH_NO_MIXED, LAUNCH_NARROW_ALWAYS, LAUNCH_NARROW_NEVER = 0x1, 0x2, 0x4, 0x8
LAUNCH_HAL_COPY = 0x10
LAUNCH_SEPARATE_DEMATCH = 0x20
LAUNCH_HAL_EARLY_COPY = 0x100
LAUNCH_SHARED_QUEUE = 0x40
LAUNCH_NO_DWQ = 0x80


class Params(ctypes.Structure):
    _fields_ = [("max_queue_cbs", ctypes.c_uint32), ("max_cb_llrs", ctypes.c_uint32),
                ("nof_harq_slots", ctypes.c_uint32), ("launch_flags", ctypes.c_uint32)]


class DecDesc(ctypes.Structure):
    _fields_ = [("base_graph", ctypes.c_uint8), ("max_iterations", ctypes.c_uint8), ("crc_mode", ctypes.c_uint8),
                ("crc_poly", ctypes.c_int8), ("lifting_size", ctypes.c_uint16), ("nof_filler_bits", ctypes.c_uint16),
                ("llr_length", ctypes.c_uint32), ("scaling_factor", ctypes.c_float), ("llr_offset", ctypes.c_uint64),
                ("out_offset", ctypes.c_uint64)]


class DematchDesc(ctypes.Structure):
    _fields_ = [("modulation_order", ctypes.c_uint8), ("rv", ctypes.c_uint8), ("new_data", ctypes.c_uint8),
                ("reserved", ctypes.c_uint8), ("cb_length", ctypes.c_uint32), ("rm_length", ctypes.c_uint32),
                ("Nref", ctypes.c_uint32), ("nof_filler_bits", ctypes.c_uint32)]


class EncHwConfig(ctypes.Structure):
    """ldpc_hip_enc_hw_config = hal::hw_pdsch_encoder_configuration (hw_accelerator_pdsch_enc.h:37-76)."""
    _fields_ = [("nof_tb_bits", ctypes.c_uint32), ("nof_tb_crc_bits", ctypes.c_uint32),
                ("base_graph", ctypes.c_uint8), ("modulation", ctypes.c_uint8), ("rv", ctypes.c_uint8),
                ("cb_mode", ctypes.c_uint8), ("nof_segments", ctypes.c_uint32), ("nof_short_segments", ctypes.c_uint32),
                ("cw_length_a", ctypes.c_uint32), ("cw_length_b", ctypes.c_uint32), ("lifting_size", ctypes.c_uint32),
                ("Ncb", ctypes.c_uint32), ("Nref", ctypes.c_uint32), ("nof_segment_bits", ctypes.c_uint32),
                ("nof_filler_bits", ctypes.c_uint32), ("rm_length", ctypes.c_uint32), ("tb_crc", ctypes.c_uint8 * 3),
                ("reserved", ctypes.c_uint8)]


class HwConfig(ctypes.Structure):
    _fields_ = [("base_graph", ctypes.c_uint8), ("modulation_order", ctypes.c_uint8), ("rv", ctypes.c_uint8),
                ("new_data", ctypes.c_uint8), ("nof_segments", ctypes.c_uint32), ("cw_length", ctypes.c_uint32),
                ("lifting_size", ctypes.c_uint32), ("Ncb", ctypes.c_uint32), ("Nref", ctypes.c_uint32),
                ("nof_segment_bits", ctypes.c_uint32), ("nof_filler_bits", ctypes.c_uint32),
                ("max_nof_ldpc_iterations", ctypes.c_uint32), ("use_early_stop", ctypes.c_uint8),
                ("cb_crc_type", ctypes.c_uint8), ("cb_crc_len", ctypes.c_uint16),
                ("absolute_cb_id", ctypes.c_uint32)]


class CbResult(ctypes.Structure):
    _fields_ = [("crc_pass", ctypes.c_uint8), ("nof_iterations", ctypes.c_uint8), ("status", ctypes.c_uint16)]


assert ctypes.sizeof(DecDesc) == 32 and ctypes.sizeof(CbResult) == 4 and ctypes.sizeof(HwConfig) == 44

_lib = None


class TbDesc(ctypes.Structure):
    """ldpc_hip_tb_desc (include/srsran_ldpc_hip.h)."""
    _fields_ = [("msg_offset", ctypes.c_uint64), ("tb_offset", ctypes.c_uint64), ("msg_stride", ctypes.c_uint32),
                ("tbs", ctypes.c_uint32), ("result_index", ctypes.c_uint32), ("nof_cbs", ctypes.c_uint16),
                ("cb_msg_bits", ctypes.c_uint16), ("nof_filler_bits", ctypes.c_uint16), ("cb_crc_bits", ctypes.c_uint8),
                ("pad", ctypes.c_uint8)]


class EncDesc(ctypes.Structure):
    """ldpc_hip_enc_desc (include/srsran_ldpc_hip.h)."""
    _fields_ = [("msg_offset", ctypes.c_uint64), ("cw_offset", ctypes.c_uint64), ("cw_length", ctypes.c_uint32),
                ("lifting_size", ctypes.c_uint16), ("base_graph", ctypes.c_uint8), ("pad", ctypes.c_uint8)]


class RmDesc(ctypes.Structure):
    """ldpc_hip_rm_desc (include/srsran_ldpc_hip.h)."""
    _fields_ = [("cw_offset", ctypes.c_uint64), ("out_offset", ctypes.c_uint64), ("cb_length", ctypes.c_uint32),
                ("rm_length", ctypes.c_uint32), ("Nref", ctypes.c_uint32), ("nof_filler_bits", ctypes.c_uint16),
                ("modulation_order", ctypes.c_uint8), ("rv", ctypes.c_uint8)]


class DemodDesc(ctypes.Structure):
    """ldpc_hip_demod_desc (include/srsran_ldpc_hip.h)."""
    _fields_ = [("symbol_offset", ctypes.c_uint64), ("noise_offset", ctypes.c_uint64), ("llr_offset", ctypes.c_uint64),
                ("nof_symbols", ctypes.c_uint32), ("modulation", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 3)]


class TbResult(ctypes.Structure):
    _fields_ = [("tb_crc_ok", ctypes.c_uint8), ("written", ctypes.c_uint8), ("nof_cbs_ok", ctypes.c_uint16)]


class LdpcHipError(RuntimeError):
    pass


def load():
    """Load the HIP library. torch (when importable) is imported first so that the process uses ONE HIP runtime:
    torch's bundled libamdhip64.so.7 then satisfies the library's dependency by soname."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch is present in this image
        pass
    if not LIB_PATH.exists():
        raise LdpcHipError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(str(LIB_PATH))
    P = ctypes.c_void_p
    U32 = ctypes.c_uint32
    I = ctypes.c_int
    sig = {
        "ldpc_hip_open": (I, [I, ctypes.POINTER(Params), ctypes.POINTER(P)]),
        "ldpc_hip_open_harq": (I, [I, ctypes.POINTER(Params), P, ctypes.POINTER(P)]),
        "ldpc_hip_harq_repo_create": (I, [I, U32, I, ctypes.POINTER(P)]),
        "ldpc_hip_harq_repo_release": (I, [P]),
        "ldpc_hip_harq_repo_entry": (I, [P, U32, ctypes.POINTER(U32)]),
        "ldpc_hip_harq_repo_read": (I, [P, U32, P, U32]),
        "ldpc_hip_harq_device_memory": (I, [I, ctypes.POINTER(P)]),
        "ldpc_hip_harq_capacity": (U32, [P]),
        "ldpc_hip_auto_device": (I, []),
        "ldpc_hip_decode_work": (ctypes.c_uint64, [ctypes.POINTER(DecDesc), P]),
        "ldpc_hip_auto_min_work": (ctypes.c_uint64, []),
        "ldpc_hip_close": (I, [P]),
        "ldpc_hip_last_error": (ctypes.c_char_p, [P]),
        "ldpc_hip_stream": (P, [P]),
        "ldpc_hip_decode_plan_create": (I, [P, U32, ctypes.POINTER(DecDesc), ctypes.POINTER(P)]),
        "ldpc_hip_decode_plan_destroy": (I, [P]),
        "ldpc_hip_decode_launch": (I, [P, P, P, P, P]),
        "ldpc_hip_decode_sync": (I, [P, U32, ctypes.POINTER(DecDesc), ctypes.POINTER(P), ctypes.POINTER(P),
                                     ctypes.POINTER(CbResult)]),
        "ldpc_hip_rate_dematch_sync": (I, [P, U32, ctypes.POINTER(DematchDesc), ctypes.POINTER(P),
                                           ctypes.POINTER(P)]),
        "ldpc_hip_queue_reserve": (I, [P]),
        "ldpc_hip_queue_free": (I, [P]),
        "ldpc_hip_enqueue": (I, [P, U32, ctypes.POINTER(HwConfig), P, U32, P, U32]),
        "ldpc_hip_dequeue": (I, [P, U32, P, U32, P, U32]),
        "ldpc_hip_read_outputs": (I, [P, U32, U32, ctypes.POINTER(CbResult)]),
        "ldpc_hip_harq_free": (I, [P, U32]),
        "ldpc_hip_external_harq_supported": (I, [P]),
        "ldpc_hip_tb_join_launch": (I, [P, U32, ctypes.POINTER(TbDesc), P, P, P, P, P]),
        "ldpc_hip_encode_launch": (I, [P, U32, ctypes.POINTER(EncDesc), P, P, P]),
        "ldpc_hip_rate_match_launch": (I, [P, U32, ctypes.POINTER(RmDesc), P, P, P]),
        "ldpc_hip_rate_dematch_launch": (I, [P, U32, ctypes.POINTER(DematchDesc), P,
                                             ctypes.POINTER(ctypes.c_uint64), P, ctypes.POINTER(ctypes.c_uint64), P]),
        "ldpc_hip_demodulate_launch": (I, [P, U32, ctypes.POINTER(DemodDesc), P, P, P, P]),
        "ldpc_hip_demodulate_sync": (I, [P, U32, I, P, P, P]),
        "ldpc_hip_demod_dematch_launch": (I, [P, U32, ctypes.POINTER(DematchDesc), ctypes.POINTER(DemodDesc), P, P, P,
                                              ctypes.POINTER(ctypes.c_uint64), P]),
        "ldpc_hip_dematch_decode_launch": (I, [P, ctypes.POINTER(DematchDesc), P, ctypes.POINTER(ctypes.c_uint64),
                                               ctypes.POINTER(DemodDesc), P, P, P, P, P, P]),
        "ldpc_hip_capture_begin": (I, [P, P]),
        "ldpc_hip_capture_end": (I, [P, P, ctypes.POINTER(P)]),
        "ldpc_hip_graph_launch": (I, [P, P]),
        "ldpc_hip_graph_destroy": (I, [P]),
        "ldpc_hip_schedule_groups": (I, [I, U32]),
        "ldpc_hip_specialised": (I, [I, U32]),
        "ldpc_hip_version": (ctypes.c_char_p, []),
        "ldpc_hip_enc_queue_create": (I, [P, I, U32, U32, ctypes.POINTER(P)]),
        "ldpc_hip_enc_queue_destroy": (I, [P]),
        "ldpc_hip_enc_reserve": (I, [P]),
        "ldpc_hip_enc_free": (I, [P]),
        "ldpc_hip_enc_configure": (I, [P, U32, ctypes.POINTER(EncHwConfig)]),
        "ldpc_hip_enc_enqueue": (I, [P, U32, P, U32]),
        "ldpc_hip_enc_dequeue": (I, [P, U32, P, U32, P, U32]),
        "ldpc_hip_enc_cb_mode": (I, [P]),
        "ldpc_hip_enc_max_tb_size": (U32, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


STREAM_LEGACY = 1  # hipStreamLegacy: the C ABI launches on the legacy default (null) stream


def stream_arg(stream):
    """The hipStream_t a launch wrapper hands the C ABI. An explicit handle goes as given. For 0 / None the launch
    joins torch's current stream, so that torch's queued work on it (a torch.zeros output buffer's fill, an input copy)
    is ordered before the launch and later torch work after it, without a host synchronisation: that stream's handle,
    or hipStreamLegacy when it is the default stream (the ABI maps it to the null stream; round 4 synchronised torch's
    stream on the host instead, a hidden host sync per call, because the handle then crashed a multi-group plan's fork,
    DESIGN.md section 8). Without torch in use: None, the context's own stream."""
    if stream:
        return stream
    import sys
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        return torch.cuda.current_stream().cuda_stream or STREAM_LEGACY
    return None


def check(ctx, rc: int, what: str) -> int:
    if rc < 0:
        msg = load().ldpc_hip_last_error(ctx)
        raise LdpcHipError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


class HarqRepository:
    """One external HARQ buffer repository on a GPU (ldpc_hip_harq_repo): hal::ext_harq_buffer_context_repository
    (ext_harq_buffer_context_repository.h:44-96) with its HBM soft buffers, direct-indexed by absolute_cb_id and shared
    by every HAL context opened on it (hw_accelerator_factories.h:41)."""

    def __init__(self, device: int = 0, nof_codeblocks: int = 1024, debug_mode: bool = False):
        self.lib = load()
        self.device, self.nof_codeblocks, self.debug_mode = device, nof_codeblocks, debug_mode
        h = ctypes.c_void_p()
        rc = self.lib.ldpc_hip_harq_repo_create(device, nof_codeblocks, 1 if debug_mode else 0, ctypes.byref(h))
        if rc != OK:
            raise LdpcHipError(f"ldpc_hip_harq_repo_create(device={device}, {nof_codeblocks}) failed ({rc})")
        self.handle = h

    def entry(self, absolute_cb_id: int):
        """(empty, soft_data_len) of an entry."""
        n = ctypes.c_uint32()
        rc = self.lib.ldpc_hip_harq_repo_entry(self.handle, absolute_cb_id, ctypes.byref(n))
        if rc < 0:
            raise LdpcHipError(f"ldpc_hip_harq_repo_entry({absolute_cb_id}) failed ({rc})")
        return bool(rc), int(n.value)

    def read(self, absolute_cb_id: int, n: int):
        """The first n soft bits of an entry (int8, synchronous copy)."""
        import numpy as np
        out = np.zeros(n, np.int8)
        rc = self.lib.ldpc_hip_harq_repo_read(self.handle, absolute_cb_id, out.ctypes.data, n)
        if rc != OK:
            raise LdpcHipError(f"ldpc_hip_harq_repo_read({absolute_cb_id}) failed ({rc})")
        return out

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ldpc_hip_harq_repo_release(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class HarqDeviceMemory(HarqRepository):
    """The GPU's HARQ memory (ldpc_hip_harq_device_memory): one per device and process, soft bits per absolute_cb_id,
    the entry state kept by the caller's ext_harq_buffer_context_repository. This object holds one reference."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.device, self.debug_mode = device, False
        h = ctypes.c_void_p()
        rc = self.lib.ldpc_hip_harq_device_memory(device, ctypes.byref(h))
        if rc != OK:
            raise LdpcHipError(f"ldpc_hip_harq_device_memory(device={device}) failed ({rc})")
        self.handle = h

    @property
    def nof_codeblocks(self) -> int:
        return int(self.lib.ldpc_hip_harq_capacity(self.handle))


class Context:
    """Owns one ldpc_hip_ctx (one GPU, one HIP stream, graph schedules). Its HAL queue keeps soft buffers in
    `harq_repo` (shared) when given, else in a private repository of nof_harq_slots entries when that is non-zero."""

    def __init__(self, device: int = 0, max_queue_cbs: int = 0, max_cb_llrs: int = 0, nof_harq_slots: int = 0,
                 launch_flags: int = 0, harq_repo: "HarqRepository | None" = None):
        self.lib = load()
        self.device = device
        p = Params(max_queue_cbs, max_cb_llrs, nof_harq_slots, launch_flags)
        h = ctypes.c_void_p()
        rc = self.lib.ldpc_hip_open_harq(device, ctypes.byref(p), harq_repo.handle if harq_repo else None,
                                         ctypes.byref(h))
        if rc != OK:
            raise LdpcHipError(f"ldpc_hip_open(device={device}) failed ({rc})")
        self.handle = h
        self.harq_repo = harq_repo   # the context holds its own reference in the library; kept for introspection

    @property
    def stream(self) -> int:
        return self.lib.ldpc_hip_stream(self.handle) or 0

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ldpc_hip_close(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device: int = 0) -> Context:
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = Context(device, nof_harq_slots=0)
        _default_ctx[device] = ctx
    return ctx
