"""Python mirror of srsRAN's hardware-accelerated PUSCH decoder plugin surface, backed by the MI355X library.

Mirrors include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:36-115 and
include/srsran/hal/hw_accelerator.h:35-57 (same method names, argument meaning, return values):

  reserve_queue / free_queue / configure_operation / enqueue_operation / dequeue_operation /
  read_operation_outputs / free_harq_context_entry / is_external_harq_supported

and the factory selection of hw_accelerator_factories.cpp:63-66 with the new acc_type "mi355x". The caller flow it
serves is pusch_decoder_hw_impl::on_end_softbits (pusch_decoder_hw_impl.cpp:132-342): configure + enqueue every
codeblock (external HARQ) or one codeblock at a time (host HARQ), then dequeue (spinning on False) and read the
outputs. The first dequeue of a staged batch launches rate dematching + decoding of all its codeblocks on the device
(ldpc_hip_dequeue); once all are dequeued the next enqueue starts a new batch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import CbResult, DROPPED, EFULL, HwConfig, LdpcHipError, NOT_READY, OK

CRC16, CRC24B, CRC24A = 0, 1, 2  # hal::hw_dec_cb_crc_type
_MOD_BITS = {"BPSK": 1, "PI_2_BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


@dataclass
class hw_pusch_decoder_configuration:
    base_graph_index: int = 1
    modulation: str = "QPSK"
    nof_segments: int = 1
    rv: int = 0
    cw_length: int = 0
    lifting_size: int = 2
    Ncb: int = 0
    Nref: int = 0
    nof_segment_bits: int = 0
    nof_filler_bits: int = 0
    max_nof_ldpc_iterations: int = 6
    use_early_stop: bool = True
    new_data: bool = True
    cb_crc_len: int = 24
    cb_crc_type: int = CRC24B
    absolute_cb_id: int = 0


@dataclass
class hw_pusch_decoder_outputs:
    CRC_pass: bool = False
    nof_ldpc_iterations: int = 0


class hw_accelerator_pusch_dec:
    """Abstract interface (hw_accelerator_pusch_dec.h:83-115)."""


HARQ_INCR = 32768  # ext_harq_buffer_context_repository.h:37: bytes per accelerator HARQ slot


@dataclass
class ext_harq_buffer_context_entry:
    """ext_harq_buffer_context_repository.h:40-45."""
    soft_data_len: int = 0
    empty: bool = True


class ext_harq_buffer_context_repository:
    """hal::ext_harq_buffer_context_repository (ext_harq_buffer_context_repository.h:48-105): the HAL caller's per-CB
    HARQ metadata, direct-indexed by absolute_cb_id. The soft bits themselves live in the accelerator's memory (here
    the GPU's HARQ memory, one per device). Out-of-range ids raise, as the reference asserts."""

    def __init__(self, nof_codeblocks: int, ext_harq_buff_size: int, debug_mode: bool):
        if nof_codeblocks * HARQ_INCR > ext_harq_buff_size:
            raise LdpcHipError(f"Requested size ({nof_codeblocks * HARQ_INCR} bytes) for {nof_codeblocks} codeblocks "
                               f"exceeds external HARQ buffer capacity ({ext_harq_buff_size} bytes).")
        self.nof_codeblocks, self.debug_mode = nof_codeblocks, debug_mode
        self.repo = [ext_harq_buffer_context_entry() for _ in range(nof_codeblocks)]

    def _check(self, absolute_codeblock_id):
        if not 0 <= absolute_codeblock_id < self.nof_codeblocks:
            raise LdpcHipError(f"Absolute CB index {absolute_codeblock_id} out of bounds - HARQ buffer context has "
                               f"capacity for {self.nof_codeblocks} CBs.")

    def get(self, absolute_codeblock_id: int, new_data: bool) -> ext_harq_buffer_context_entry:
        self._check(absolute_codeblock_id)
        e = self.repo[absolute_codeblock_id]
        if e.empty or new_data:
            e.soft_data_len, e.empty = 0, False
        return e

    def free(self, absolute_codeblock_id: int) -> None:
        self._check(absolute_codeblock_id)
        if not self.debug_mode:
            self.repo[absolute_codeblock_id].empty = True


def create_ext_harq_buffer_context_repository(nof_codeblocks: int, ext_harq_buff_size: int,
                                              debug_mode: bool = False) -> ext_harq_buffer_context_repository:
    """ext_harq_buffer_context_repository_factory.cpp:28-34."""
    return ext_harq_buffer_context_repository(nof_codeblocks, ext_harq_buff_size, debug_mode)


def hip_device_of_acc_type(acc_type: str) -> int:
    """"mi355x" -> GPU 0, "mi355x:<n>" -> GPU n, anything else -> -1 (not this plugin)."""
    if acc_type == "mi355x":
        return 0
    if acc_type.startswith("mi355x:") and acc_type[7:].isdigit():
        return int(acc_type[7:])
    return -1


def read_harq_soft_bits(device: int, absolute_cb_id: int, n: int) -> np.ndarray:
    """The first n soft bits the GPU's HARQ memory holds for absolute_cb_id (diagnostics and tests)."""
    mem = _lib.HarqDeviceMemory(device)
    try:
        return mem.read(absolute_cb_id, n)
    finally:
        mem.close()


class hw_accelerator_pusch_dec_hip(hw_accelerator_pusch_dec):
    """hw_accelerator_pusch_dec on the GPU with acc100's HARQ split (hw_accelerator_pusch_dec_acc100_impl.cpp): the
    caller's repository keeps each CB's entry and decides drops; the soft bits stay in the GPU's HARQ memory
    (ext_softbuffer) or travel with the operation (host soft buffers)."""

    def __init__(self, ctx: _lib.Context, ext_softbuffer: bool, harq_buffer_context: ext_harq_buffer_context_repository):
        if harq_buffer_context is None:
            raise LdpcHipError("hw_accelerator_pusch_dec_configuration without harq_buffer_context")
        self.ctx = ctx
        self.ext_softbuffer = ext_softbuffer
        self.harq_buffer_context = harq_buffer_context
        self.cfg = {}
        self.harq_context_entries = {}
        self.drop_op = set()

    def _check(self, rc, what):
        return _lib.check(self.ctx.handle, rc, what)

    def reserve_queue(self) -> None:
        self._check(self.ctx.lib.ldpc_hip_queue_reserve(self.ctx.handle), "reserve_queue")

    def free_queue(self) -> None:
        self._check(self.ctx.lib.ldpc_hip_queue_free(self.ctx.handle), "free_queue")
        self.cfg.clear()

    def configure_operation(self, config: hw_pusch_decoder_configuration, cb_index: int = 0) -> None:
        if cb_index == 0:                                            # acc100_impl.cpp:106-110
            self.drop_op.clear()
            self.harq_context_entries.clear()
        # the CB's entry in the caller's repository (acc100_impl.cpp:113); raises for an out-of-range id
        self.harq_context_entries[cb_index] = self.harq_buffer_context.get(config.absolute_cb_id, config.new_data)
        c = HwConfig()
        c.base_graph = int(config.base_graph_index)
        c.modulation_order = _MOD_BITS[config.modulation] if isinstance(config.modulation, str) else int(
            config.modulation)
        c.rv = config.rv
        c.new_data = 1 if config.new_data else 0
        c.nof_segments = config.nof_segments
        c.cw_length = config.cw_length
        c.lifting_size = config.lifting_size
        c.Ncb = config.Ncb
        c.Nref = config.Nref
        c.nof_segment_bits = config.nof_segment_bits
        c.nof_filler_bits = config.nof_filler_bits
        c.max_nof_ldpc_iterations = config.max_nof_ldpc_iterations
        c.use_early_stop = 1 if config.use_early_stop else 0
        c.cb_crc_type = int(config.cb_crc_type)
        c.cb_crc_len = config.cb_crc_len
        c.absolute_cb_id = config.absolute_cb_id
        self.cfg[cb_index] = c

    def enqueue_operation(self, data: np.ndarray, aux_data: Optional[np.ndarray] = None, cb_index: int = 0) -> bool:
        """True when the operation was accepted -- also when it is accepted as dropped: a retransmission whose
        repository entry holds no soft data, which later reads as a CRC failure with the maximum number of iterations,
        as acc100 does (hw_accelerator_pusch_dec_acc100_impl.cpp:123-125, 184-186, 233-247). False when the batch
        cannot take it now (full, or still in flight): the caller dequeues and enqueues it again
        (pusch_decoder_hw_impl.cpp:237-241)."""
        if cb_index not in self.cfg:
            raise LdpcHipError("enqueue_operation without configure_operation")
        if not self.cfg[cb_index].new_data and self.harq_context_entries[cb_index].soft_data_len == 0:
            self.drop_op.add(cb_index)
            return True
        llr = np.ascontiguousarray(data, dtype=np.int8)
        soft = None if aux_data is None or len(aux_data) == 0 else np.ascontiguousarray(aux_data, dtype=np.int8)
        rc = self.ctx.lib.ldpc_hip_enqueue(self.ctx.handle, cb_index, ctypes.byref(self.cfg[cb_index]),
                                           llr.ctypes.data if llr.size else None, llr.size,
                                           soft.ctypes.data if soft is not None else None,
                                           0 if soft is None else soft.size)
        if rc == EFULL:
            return False
        self._check(rc, "enqueue_operation")
        self.drop_op.discard(cb_index)
        return True

    def dequeue_operation(self, data: np.ndarray, aux_data: Optional[np.ndarray] = None,
                          segment_index: int = 0) -> bool:
        """data: packed message buffer (uint8, modified); aux_data: soft buffer updated in place when the HARQ
        buffer is host-side. Returns False while the batch has not completed (the caller spins)."""
        if segment_index in self.drop_op:
            return True                                              # acc100_impl.cpp:217-219
        if not (isinstance(data, np.ndarray) and data.dtype == np.uint8 and data.flags.c_contiguous):
            raise LdpcHipError("data must be a contiguous uint8 array")
        soft = aux_data if (aux_data is not None and len(aux_data) != 0) else None
        rc = self.ctx.lib.ldpc_hip_dequeue(self.ctx.handle, segment_index, data.ctypes.data, data.size,
                                           soft.ctypes.data if soft is not None else None,
                                           0 if soft is None else soft.size)
        if rc == NOT_READY:
            return False
        self._check(rc, "dequeue_operation")
        c = self.cfg[segment_index]
        # the entry now holds the CB's soft data (acc100_impl.cpp:211-212)
        self.harq_context_entries[segment_index].soft_data_len = (66 if c.base_graph == 1 else 50) * c.lifting_size
        return True

    def read_operation_outputs(self, out: hw_pusch_decoder_outputs, cb_index: int = 0,
                               absolute_cb_id: int = 0) -> None:
        if cb_index in self.drop_op:                                 # acc100_impl.cpp:233-247
            out.CRC_pass = False
            out.nof_ldpc_iterations = int(self.cfg[cb_index].max_nof_ldpc_iterations)
            self.drop_op.discard(cb_index)
            return
        r = CbResult()
        self._check(self.ctx.lib.ldpc_hip_read_outputs(self.ctx.handle, cb_index, absolute_cb_id, ctypes.byref(r)),
                    "read_operation_outputs")
        out.CRC_pass = bool(r.crc_pass)
        out.nof_ldpc_iterations = int(r.nof_iterations)

    def free_harq_context_entry(self, absolute_cb_id: int) -> None:
        self.harq_buffer_context.free(absolute_cb_id)                # acc100_impl.cpp:268-271

    def is_external_harq_supported(self) -> bool:
        return bool(self.ext_softbuffer)


@dataclass
class hw_accelerator_pusch_dec_configuration:
    """hw_accelerator_pusch_dec_configuration (pusch/hw_accelerator_factories.h:33-44), field for field; acc_type
    "mi355x" or "mi355x:<n>" selects the GPU, bbdev_accelerator is unused. max_queue_cbs and launch_flags are this
    implementation's diagnostics (the CBs one batch holds; _lib.LAUNCH_* launch forms), not reference fields."""
    acc_type: str = "mi355x"
    bbdev_accelerator: object = None
    ext_softbuffer: bool = True
    harq_buffer_context: Optional[ext_harq_buffer_context_repository] = None
    dedicated_queue: bool = True
    max_queue_cbs: int = 162
    launch_flags: int = 0


class hw_accelerator_pusch_dec_factory:
    def __init__(self, cfg: hw_accelerator_pusch_dec_configuration):
        self.cfg = cfg
        self.device = hip_device_of_acc_type(cfg.acc_type)

    def create(self) -> hw_accelerator_pusch_dec_hip:
        flags = self.cfg.launch_flags | (0 if self.cfg.dedicated_queue else _lib.LAUNCH_SHARED_QUEUE)
        mem = _lib.HarqDeviceMemory(self.device) if self.cfg.ext_softbuffer else None
        try:
            ctx = _lib.Context(self.device, max_queue_cbs=self.cfg.max_queue_cbs, launch_flags=flags, harq_repo=mem)
        finally:
            if mem is not None:
                mem.close()       # the context holds its own reference
        return hw_accelerator_pusch_dec_hip(ctx, self.cfg.ext_softbuffer, self.cfg.harq_buffer_context)


def create_hw_accelerator_pusch_dec_factory(cfg: hw_accelerator_pusch_dec_configuration):
    """hw_accelerator_factories.cpp:61-69 with the "mi355x" branch: None for an accelerator type it does not know."""
    if hip_device_of_acc_type(cfg.acc_type) < 0:
        return None
    return hw_accelerator_pusch_dec_factory(cfg)


# ---- hw_accelerator_pdsch_enc (include/srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc.h) --------

_MOD_ID = {"PI_2_BPSK": 0, "BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}  # modulation_scheme numbering


@dataclass
class hw_pdsch_encoder_configuration:
    """hal::hw_pdsch_encoder_configuration (hw_accelerator_pdsch_enc.h:37-76): same fields and meaning."""
    nof_tb_bits: int = 0
    nof_tb_crc_bits: int = 24
    base_graph_index: int = 1
    modulation: str = "QPSK"
    nof_segments: int = 1
    nof_short_segments: int = 0
    rv: int = 0
    cw_length_a: int = 0
    cw_length_b: int = 0
    lifting_size: int = 2
    Ncb: int = 0
    Nref: int = 0
    nof_segment_bits: int = 0
    nof_filler_bits: int = 0
    rm_length: int = 0
    tb_crc: tuple = ()
    cb_mode: bool = False


class hw_accelerator_pdsch_enc:
    """Abstract interface (hw_accelerator_pdsch_enc.h:75-102)."""


class hw_accelerator_pdsch_enc_hip(hw_accelerator_pdsch_enc):
    """The PDSCH encoder plugin on the GPU (ldpc_hip_enc_* in include/srsran_ldpc_hip.h): configure_operation +
    enqueue_operation stage a codeblock (CB mode) or a transport block (TB mode); the first dequeue_operation of a
    staged batch encodes and rate-matches all of it on the device; dequeue_operation returns False until it is done
    (pdsch_encoder_hw_impl.cpp:125-140 spins on it)."""

    def __init__(self, ctx: _lib.Context, cb_mode: bool = False, max_queue_cbs: int = 0, max_tb_bytes: int = 0):
        self.ctx = ctx
        h = ctypes.c_void_p()
        rc = ctx.lib.ldpc_hip_enc_queue_create(ctx.handle, 1 if cb_mode else 0, max_queue_cbs, max_tb_bytes,
                                               ctypes.byref(h))
        self._check(rc, "hw_accelerator_pdsch_enc_hip")
        self.q = h

    def _check(self, rc, what):
        return _lib.check(self.ctx.handle, rc, what)

    def close(self):
        if getattr(self, "q", None):
            self.ctx.lib.ldpc_hip_enc_queue_destroy(self.q)
            self.q = None

    def reserve_queue(self) -> None:
        self._check(self.ctx.lib.ldpc_hip_enc_reserve(self.q), "reserve_queue")

    def free_queue(self) -> None:
        self._check(self.ctx.lib.ldpc_hip_enc_free(self.q), "free_queue")

    def configure_operation(self, config: hw_pdsch_encoder_configuration, cb_index: int = 0) -> None:
        c = _lib.EncHwConfig()
        c.nof_tb_bits = config.nof_tb_bits
        c.nof_tb_crc_bits = config.nof_tb_crc_bits
        c.base_graph = int(config.base_graph_index)
        c.modulation = _MOD_ID[config.modulation] if isinstance(config.modulation, str) else int(config.modulation)
        c.rv = config.rv
        c.cb_mode = 1 if config.cb_mode else 0
        c.nof_segments = config.nof_segments
        c.nof_short_segments = config.nof_short_segments
        c.cw_length_a = config.cw_length_a
        c.cw_length_b = config.cw_length_b
        c.lifting_size = config.lifting_size
        c.Ncb = config.Ncb
        c.Nref = config.Nref
        c.nof_segment_bits = config.nof_segment_bits
        c.nof_filler_bits = config.nof_filler_bits
        c.rm_length = config.rm_length
        for i, b in enumerate(config.tb_crc[:3]):
            c.tb_crc[i] = b
        self._check(self.ctx.lib.ldpc_hip_enc_configure(self.q, cb_index, ctypes.byref(c)), "configure_operation")

    def enqueue_operation(self, data: np.ndarray, aux_data: Optional[np.ndarray] = None, cb_index: int = 0) -> bool:
        """data: CB mode, the segment's packed bits (CB CRC included, filler bits excluded); TB mode, the TB bytes.
        False when the batch cannot take the operation now (full, or in flight): dequeue, then enqueue again."""
        d = np.ascontiguousarray(data, dtype=np.uint8)
        rc = self.ctx.lib.ldpc_hip_enc_enqueue(self.q, cb_index, d.ctypes.data if d.size else None, d.size)
        if rc == EFULL:
            return False
        self._check(rc, "enqueue_operation")
        return True

    def dequeue_operation(self, data: np.ndarray, packed_data: Optional[np.ndarray] = None,
                          segment_index: int = 0) -> bool:
        """data: the rate-matched bits, one per byte (uint8, written); packed_data: the same bits packed, each
        segment byte-aligned (written up to its size). False while the batch has not completed."""
        if not (isinstance(data, np.ndarray) and data.dtype == np.uint8 and data.flags.c_contiguous):
            raise LdpcHipError("data must be a contiguous uint8 array")
        pk = packed_data if (packed_data is not None and len(packed_data) != 0) else None
        rc = self.ctx.lib.ldpc_hip_enc_dequeue(self.q, segment_index, data.ctypes.data, data.size,
                                               pk.ctypes.data if pk is not None else None,
                                               0 if pk is None else pk.size)
        if rc == NOT_READY:
            return False
        self._check(rc, "dequeue_operation")
        return True

    def get_cb_mode(self) -> bool:
        return bool(self.ctx.lib.ldpc_hip_enc_cb_mode(self.q))

    def get_max_tb_size(self) -> int:
        return int(self.ctx.lib.ldpc_hip_enc_max_tb_size(self.q))


@dataclass
class hw_accelerator_pdsch_enc_configuration:
    """hw_accelerator_pdsch_enc_configuration (channel_processors/hw_accelerator_factories.h:31-43), field for field;
    acc_type "mi355x[:n]". max_queue_cbs is this implementation's (codeblocks one batch holds)."""
    acc_type: str = "mi355x"
    bbdev_accelerator: object = None
    cb_mode: bool = False
    max_tb_size: int = 0
    dedicated_queue: bool = True
    max_queue_cbs: int = 162


class hw_accelerator_pdsch_enc_factory:
    def __init__(self, cfg: hw_accelerator_pdsch_enc_configuration):
        self.cfg = cfg

    def create(self) -> hw_accelerator_pdsch_enc_hip:
        ctx = _lib.Context(hip_device_of_acc_type(self.cfg.acc_type),
                           launch_flags=0 if self.cfg.dedicated_queue else _lib.LAUNCH_SHARED_QUEUE)
        return hw_accelerator_pdsch_enc_hip(ctx, self.cfg.cb_mode, self.cfg.max_queue_cbs, self.cfg.max_tb_size)


def create_hw_accelerator_pdsch_enc_factory(cfg: hw_accelerator_pdsch_enc_configuration):
    """hw_accelerator_factories.cpp (create_hw_accelerator_pdsch_enc_factory): None for an unsupported acc_type."""
    if hip_device_of_acc_type(cfg.acc_type) < 0:
        return None
    return hw_accelerator_pdsch_enc_factory(cfg)
