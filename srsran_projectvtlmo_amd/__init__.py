"""MI355X-native (gfx950) 5G-NR PUSCH LDPC decode path for srsRAN.

Product code only: HIP kernels + C ABI (csrc/, include/srsran_ldpc_hip.h) and the Python mirror of srsRAN's
plugin surfaces (channel_coding.py: ldpc_decoder / ldpc_rate_dematcher factories; hal.py:
hw_accelerator_pusch_dec). The CPU oracle in ../oracle is test infrastructure and is never imported from here.
"""
from ._lib import LIB_PATH, Context, LdpcHipError, load  # noqa: F401

__version__ = "0.1.0"
