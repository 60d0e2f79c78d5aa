"""CPU tests of the HAL mirror's host logic (no GPU call): the caller-side HARQ metadata repository with the
reference's semantics (ext_harq_buffer_context_repository.h:48-105), acc_type parsing and factory selection
(hw_accelerator_factories.cpp:61-69 with the "mi355x" branch)."""
import pytest


def test_repository_semantics():
    from srsran_projectvtlmo_amd import hal
    from srsran_projectvtlmo_amd._lib import LdpcHipError
    with pytest.raises(LdpcHipError):               # capacity check of the constructor (:58-63)
        hal.create_ext_harq_buffer_context_repository(4, 4 * hal.HARQ_INCR - 1, False)
    repo = hal.create_ext_harq_buffer_context_repository(4, 4 * hal.HARQ_INCR, False)
    e = repo.get(2, True)
    assert (e.empty, e.soft_data_len) == (False, 0)
    e.soft_data_len = 1800
    assert repo.get(2, False).soft_data_len == 1800     # retransmission: the entry keeps its soft-data length
    assert repo.get(2, True).soft_data_len == 0         # new data: a fresh entry
    repo.get(2, False).soft_data_len = 1800
    repo.free(2)
    assert repo.repo[2].empty
    assert repo.get(2, False).soft_data_len == 0        # an empty entry reopens with no soft data -> dropped op
    with pytest.raises(LdpcHipError):
        repo.get(4, True)                               # out of bounds asserts (:71-74)
    with pytest.raises(LdpcHipError):
        repo.free(4)


def test_repository_debug_mode_keeps_entries():
    from srsran_projectvtlmo_amd import hal
    repo = hal.create_ext_harq_buffer_context_repository(2, 2 * hal.HARQ_INCR, True)
    repo.get(1, True).soft_data_len = 2600
    repo.free(1)
    assert not repo.repo[1].empty and repo.get(1, False).soft_data_len == 2600


def test_acc_type_selection():
    from srsran_projectvtlmo_amd import hal
    assert hal.hip_device_of_acc_type("mi355x") == 0
    assert hal.hip_device_of_acc_type("mi355x:5") == 5
    for other in ("acc100", "mi355x:", "mi355x:a", "MI355X", ""):
        assert hal.hip_device_of_acc_type(other) == -1
    assert hal.create_hw_accelerator_pusch_dec_factory(hal.hw_accelerator_pusch_dec_configuration("acc100")) is None
    assert hal.create_hw_accelerator_pdsch_enc_factory(
        hal.hw_accelerator_pdsch_enc_configuration(acc_type="acc100")) is None
    cfg = hal.hw_accelerator_pusch_dec_configuration()
    # the reference's fields, in its order (pusch/hw_accelerator_factories.h:33-44)
    assert list(cfg.__dataclass_fields__)[:5] == ["acc_type", "bbdev_accelerator", "ext_softbuffer",
                                                  "harq_buffer_context", "dedicated_queue"]


def test_factory_type_strings():
    from srsran_projectvtlmo_amd import channel_coding as cc
    assert cc.hip_device_of("hip") == 0 and cc.hip_device_of("hip:7") == 7
    assert cc.hip_device_of("auto") is None and cc.hip_device_of("generic") is None
    assert cc.hip_device_of_dematcher_type("auto") is None  # the dematcher stays on the CPU for "auto"
