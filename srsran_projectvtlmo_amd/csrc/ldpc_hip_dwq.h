/* Device work queue: single-codeblock operations (the software route's one-CB decode and dematch calls, the HAL
 * queue's small batches) handed to a resident grid through pinned memory instead of a kernel launch each.
 *
 * One queue per (device, unit): a unit is a translation unit of specialised decoder bodies (spec_unit), whose
 * persistent kernel (LDPC_DWQ_KERNEL) holds exactly those bodies. A queue's grid is launched on demand, exits by itself
 * after an idle period (LDPC_HIP_DWQ_IDLE_US, default 2000) or a bounded lifetime (50 ms), and is relaunched by the
 * next submitter or waiter that finds it gone. LDPC_HIP_DWQ=0 (environment) disables the queues: every operation then
 * takes the launch path. */
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ldpc_hip_device.h"

namespace ldpc_hip {

struct dwq;

/* The unit's queue on `device`, created on first use with the unit's workgroup size (threads) and dynamic LDS for its
 * bodies (bytes, before the queue's own words); nullptr when the queues are disabled or cannot be created. */
dwq* dwq_get(int device, int unit, int block, uint32_t body_lds);

/* Publishes one item (its ticket field is set here) and makes sure a grid is running. Thread-safe. */
hipError_t dwq_submit(dwq* q, dwq_item item, uint32_t& ticket);

/* True when the item of `ticket` has completed (its outputs are visible to the host). Relaunches the grid if it has
 * exited with the item unclaimed. */
bool dwq_done(dwq* q, uint32_t ticket);

/* Spins until the item of `ticket` has completed; hipErrorLaunchTimeOut after 10 s. */
hipError_t dwq_wait(dwq* q, uint32_t ticket);

/* Diagnostic build (LDPC_HIP_DIAG_DWQ) only: marks the calling thread's entry into a one-CB call; no-op otherwise. */
void dwq_diag_entry();

/* Whether the queues are enabled (LDPC_HIP_DWQ, default 1). */
bool dwq_enabled();

} // namespace ldpc_hip
