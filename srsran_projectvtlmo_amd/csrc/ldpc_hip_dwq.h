/* Device work queue: single-codeblock operations (the software route's one-CB decode and dematch calls, the HAL
 * queue's small batches) handed to a resident grid through pinned memory instead of a kernel launch each.
 *
 * One queue per (device, key): key 1 + id holds the items of specialised graph id, whose persistent kernel
 * (ldpc_dwq_decode_kernel<id>) holds that graph's fused dematch + decode body alone; key 0 holds dematch-only items
 * (ldpc_dwq_dematch_kernel); key DWQ_KEY_ENC the PDSCH encoder queue's small batches (ldpc_dwq_encode_kernel); key
 * DWQ_KEY_COPY the HAL decoder's early copy of a large batch's staged LLRs into HBM (ldpc_dwq_copy_kernel). A queue's grid is launched on demand, exits by itself
 * after an idle period (LDPC_HIP_DWQ_IDLE_US, default 2000) or a bounded lifetime (50 ms), and is relaunched by the
 * next submitter or waiter that finds it gone. LDPC_HIP_DWQ=0 (environment) disables the queues: every operation then
 * takes the launch path. */
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ldpc_hip_device.h"

namespace ldpc_hip {

struct dwq;

constexpr int DWQ_KEYS     = 105; /* dematch-only + one per specialised graph + the PDSCH encoder + copies */
constexpr int DWQ_KEY_ENC  = 103; /* ldpc_dwq_encode_kernel: one codeblock's encode + rate match per item */
constexpr int DWQ_KEY_COPY = 104; /* ldpc_dwq_copy_kernel: one host-to-HBM copy per item (the HAL's early copy) */

/* The queue of `key` on `device`, created on first use with its kernel's workgroup size (threads) and dynamic LDS for
 * its body (bytes, before the queue's own words); nullptr when the queues are disabled or cannot be created. */
dwq* dwq_get(int device, int key, int block, uint32_t body_lds);

/* Publishes one item (its ticket and checksum fields are set here) and makes sure a grid is running. Thread-safe.
 * may_refuse: when no grid of the queue runs and the device's residency budget has no stream free, nothing is
 * published and hipErrorLaunchOutOfResources is returned (the caller launches instead); otherwise the submit waits for
 * a stream (up to 1 s). ticket is set whenever the item was published, also when an error follows (the item is then a
 * no-op that a later grid completes without touching the caller's buffers). */
hipError_t dwq_submit(dwq* q, dwq_item item, uint32_t& ticket, bool may_refuse = true);

/* Whether items submitted to q now are served by a running grid, launching one if the budget allows (the HAL batch
 * checks every queue it is about to use before submitting any item). Thread-safe. On true the queue is pinned: its
 * pool stream is not handed to another queue until dwq_unpin, so the submits that follow (may_refuse = false) never
 * wait for a stream even if the grid idles out in between; the caller unpins once its items are submitted. */
bool dwq_admit(dwq* q);
void dwq_unpin(dwq* q);

/* True when the item of `ticket` has completed (its outputs are visible to the host). Relaunches the grid if it has
 * exited with the item unclaimed. */
bool dwq_done(dwq* q, uint32_t ticket);

/* Spins until the item of `ticket` has completed; hipErrorLaunchTimeOut after 10 s (LDPC_HIP_DWQ_WAIT_MS). After a
 * timeout the queue is marked failed: it takes no more items (dwq_get returns nullptr for it), its grid is stopped (a
 * stopped grid claims nothing) and the item, if unclaimed, is republished as a no-op; a line goes to stderr. The
 * caller's buffers of that call may be reused only once dwq_quiesced(q) is true (the grid has left; it waits up to
 * 200 ms for that before returning). */
hipError_t dwq_wait(dwq* q, uint32_t ticket);

/* Whether no grid of q is resident: nothing can claim, or still be running, one of its items. */
bool dwq_quiesced(dwq* q);

/* Diagnostic build (LDPC_HIP_DIAG_DWQ) only: marks the calling thread's entry into a one-CB call; no-op otherwise. */
void dwq_diag_entry();

/* Whether the queues are enabled (LDPC_HIP_DWQ, default 1). */
bool dwq_enabled();

} // namespace ldpc_hip
