/*
 * Specialised decoder kernels of the LDPC_SPEC_GRAPHS_MID_B graphs (ldpc_spec.h), in a translation unit of their own
 * so that the unrolled kernels compile in parallel. ldpc_hip_kernels.hip's launch_decode reaches them through
 * spec_kernel_<id>() (the host launch stub of ldpc_decode_kernel<true, id>), and its split-row address table
 * writer through spec_split_kernel_<id>().
 */
#define LDPC_SPEC_TU_GRAPHS LDPC_SPEC_GRAPHS_MID_B
#include "ldpc_decode_body.h"

namespace ldpc_hip {

#define LDPC_SPEC_KERNEL_DEF(id, bg, z, ils)                                                                           \
  const void* spec_kernel_##id() { return reinterpret_cast<const void*>(&ldpc_decode_kernel<true, id>); }           \
  const void* spec_split_kernel_##id() { return reinterpret_cast<const void*>(&ldpc_split_table_kernel<id>); }
LDPC_SPEC_GRAPHS_MID_B(LDPC_SPEC_KERNEL_DEF)
#undef LDPC_SPEC_KERNEL_DEF

/* the persistent work-queue kernels of this unit's graphs (ldpc_hip_dwq.cpp) */
LDPC_DWQ_KERNELS(dwq_kernel_b, LDPC_SPEC_GRAPHS_MID_B)
LDPC_DIAG_UNIT_READER(b)

} // namespace ldpc_hip
