/*
 * Device work queue (ldpc_hip_dwq.h): host side. Per (device, key): a ring of work items in pinned host memory the
 * persistent kernel reads, host control words (published count, stop, exit word), a device claim counter and exit
 * count, and done flags in pinned memory the kernel writes. Per device: a pool of CU-masked streams (one hardware queue
 * each) that bounds how many grids are resident at once (the residency budget).
 *
 * Protocol (device side: dwq_loop, ldpc_decode_body.h):
 *   submit  under the queue mutex: wait for the ring slot's previous item to be done, write the item into the slot
 *           (three lines, each line's sequence word = ticket + 1 written after its payload; word 44 a checksum of the
 *           item's words 0-43), make sure a grid is running (launching one on a free pool stream);
 *   claim   a workgroup claims ticket c only with slot c read, all three sequence words equal to c + 1 and the checksum
 *           matching the words it read (device-scope CAS of the claim counter), so a torn read of the slot is never
 *           decoded and an exiting grid leaves every published ticket either done or unclaimed;
 *   done    the workgroup stores ticket + 1 into the slot's done flag after a system-scope release;
 *   wait    the caller spins on its done flag; when the grid has left (its last workgroup wrote the exit word) with
 *           the ticket not done, the ticket is unclaimed and a new grid is launched.
 */
#include "ldpc_hip_dwq.h"
#include "ldpc_graph.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <immintrin.h>

namespace ldpc_hip {

const void* dwq_kernel_dematch();
const void* dwq_kernel_encode();
const void* dwq_kernel_copy();
#define LDPC_DWQ_UNIT_DECL(u) const void* dwq_kernel_##u(int id);
LDPC_DWQ_UNIT_DECL(core)
LDPC_DWQ_UNIT_DECL(a)
LDPC_DWQ_UNIT_DECL(b)
LDPC_DWQ_UNIT_DECL(c)
LDPC_DWQ_UNIT_DECL(d)
LDPC_DWQ_UNIT_DECL(e)
LDPC_DWQ_UNIT_DECL(f)
LDPC_DWQ_UNIT_DECL(g)
LDPC_DWQ_UNIT_DECL(h)
LDPC_DWQ_UNIT_DECL(i)
LDPC_DWQ_UNIT_DECL(j)
LDPC_DWQ_UNIT_DECL(k)
LDPC_DWQ_UNIT_DECL(l)
LDPC_DWQ_UNIT_DECL(m)
LDPC_DWQ_UNIT_DECL(n)
LDPC_DWQ_UNIT_DECL(o)
LDPC_DWQ_UNIT_DECL(p)
#undef LDPC_DWQ_UNIT_DECL

namespace {

/* the persistent kernel of a queue key: 0 dematch-only items, 1 + id the specialised graph id (found in its unit) */
const void* key_kernel(int key)
{
  static const void* (*const k[])(int) = {dwq_kernel_core, dwq_kernel_a, dwq_kernel_b, dwq_kernel_c, dwq_kernel_d,
                                          dwq_kernel_e,    dwq_kernel_f, dwq_kernel_g, dwq_kernel_h, dwq_kernel_i,
                                          dwq_kernel_j,    dwq_kernel_k, dwq_kernel_l, dwq_kernel_m, dwq_kernel_n,
                                          dwq_kernel_o,    dwq_kernel_p};
  if (key == 0) {
    return dwq_kernel_dematch();
  }
  if (key == DWQ_KEY_ENC) {
    return dwq_kernel_encode();
  }
  if (key == DWQ_KEY_COPY) {
    return dwq_kernel_copy();
  }
  const int unit = spec_unit(key - 1);
  return (unit >= 0 && unit < static_cast<int>(sizeof(k) / sizeof(k[0]))) ? k[unit](key - 1) : nullptr;
}

long env_long(const char* name, long dflt)
{
  const char* v = std::getenv(name);
  return v != nullptr ? std::atol(v) : dflt;
}

constexpr uint32_t RING = 1024; /* items in flight per queue at most (a power of two) */

#ifdef LDPC_HIP_DIAG_DWQ
/* diagnostic build: per completed item {host submit ns, host done-seen ns, device claim (100 MHz, low 32 bits), item
 * copied (ticks after the claim), body done (ticks after the claim), workgroup, graph + 1, caller entry ns} */
std::mutex            g_diag_mu;
std::vector<uint64_t> g_diag;
uint64_t              host_ns()
{
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count());
}
thread_local uint64_t g_entry_ns = 0;
#endif

} // namespace

struct dwq;

/* Per device: the streams resident grids run on. Each is CU-masked, so it has a hardware queue of its own and a
 * resident grid never holds up another stream's kernels queued behind it on a shared hardware queue. The pool's size
 * bounds the grids resident at once: budget / grid by the residency budget (LDPC_HIP_DWQ_BUDGET workgroups, default
 * 128, half of the MI355X's 256 CUs), and at most LDPC_HIP_DWQ_MAX_QUEUES (default 3) by the hardware-queue tax
 * (pool_of); with the defaults the queue cap is the one that binds. Every key, whatever its grid, takes one stream: a
 * decode graph's workgroups reserve more than half a CU's LDS and own their CUs, the PDSCH encoder's (about 13 KB of
 * static LDS) and the copy key's (none) do not, but each of their grids holds a hardware queue all the same. A key
 * that finds every stream held by a resident grid is refused and its call takes the launch path (bit-exact; what that
 * costs: profiles/r06/queue_cap_ab.json). A queue key takes a free stream when its grid launches and holds it until
 * that grid has left. Round 4 gave every key a stream and a grid of its own: 8 active graphs could hold every CU, a
 * ninth graph's grid waited for one to leave (2 ms idle, 50 ms lifetime), and up to 103 hardware queues per device
 * were created. */
struct dwq_pool {
  std::mutex               mu;
  std::vector<hipStream_t> streams;
  std::vector<dwq*>        owner; /* the queue whose grid runs (or last ran) on the stream, nullptr: never used */
};

struct dwq {
  int         device = 0;
  int         key    = 0;
  const void* kernel = nullptr;
  int         block  = 768;
  uint32_t    ctl_lds = 0, lds = 0;
  int         grid    = 32;
  uint32_t    idle_ticks = 200000, life_ticks = 5000000;
  uint32_t    slot_ticks = 25, poll_flags = 0;
  uint32_t*   ring = nullptr; /* pinned, DWQ_WIRE_WORDS per slot */
  void*       ring_dev = nullptr;
  uint32_t*   hctl = nullptr; /* pinned */
  void*       hctl_dev = nullptr;
  uint32_t*   done = nullptr; /* pinned */
  void*       done_dev = nullptr;
  uint32_t*   dctl = nullptr; /* device */
  dwq_pool*   pool = nullptr;
  int         pool_slot = -1; /* the pool stream this queue's grid runs on (-1: none held) */
  hipStream_t stream = nullptr;
  hipEvent_t  ended  = nullptr; /* recorded after every grid launch */
  bool        launched = false;
  std::atomic<bool>     failed{false};  /* a wait timed out: the queue takes no more items (ldpc_hip_dwq.h) */
  std::atomic<int>      pins{0};        /* dwq_admit .. dwq_unpin: the pool stream stays this queue's */
  std::atomic<uint32_t> exit_target{0}; /* workgroups launched so far (written under mu); hctl[DWQ_H_EXITED] ==
                                           exit_target: the grid has left */
  std::mutex  mu;
  uint64_t    next = 0; /* the next ticket; 64-bit on the host, so the ring-slot guard never wraps */
#ifdef LDPC_HIP_DIAG_DWQ
  uint64_t sub_ns[1024]   = {};
  uint32_t sub_spec[1024] = {};
#endif

  /* lock-free: whether every workgroup of the last grid has left (or none was launched), so that waiters take the
   * mutex only then and never hold up a submitter while the grid runs */
  bool maybe_gone() const
  {
    return __atomic_load_n(&hctl[DWQ_H_EXITED], __ATOMIC_ACQUIRE) == exit_target.load(std::memory_order_acquire);
  }

  /* Whether a grid is running (with mu held); with query_event the runtime is asked too (a faulted grid never writes
   * the exit word) and its error returned through e. */
  bool running(bool query_event, hipError_t& e)
  {
    e = hipSuccess;
    if (!launched) {
      return false;
    }
    if (!maybe_gone() && !query_event) {
      return true;
    }
    const hipError_t q = hipEventQuery(ended);
    if (q == hipErrorNotReady) {
      /* every workgroup may have left while the kernel is ending: the next grid queues behind it on the stream */
      return !maybe_gone();
    }
    if (q != hipSuccess) {
      e = q;
    }
    return false;
  }

  /* A pool stream for this queue's next grid (with mu held): the one it holds, else a stream never used or whose
   * owner's grid has left. false: every stream carries a resident grid (the budget is spent). */
  bool take_stream()
  {
    std::lock_guard<std::mutex> lock(pool->mu);
    if (pool_slot >= 0 && pool->owner[static_cast<size_t>(pool_slot)] == this) {
      return true;
    }
    for (size_t i = 0; i != pool->streams.size(); ++i) {
      dwq* o = pool->owner[i];
      /* a pinned queue (admitted, its batch's items not all submitted yet) keeps its stream even while its grid is
       * gone, so that the submits that follow its admission never wait for a stream (ldpc_hip_dwq.h dwq_admit) */
      if (o == nullptr || (o->maybe_gone() && o->pins.load(std::memory_order_acquire) == 0)) {
        if (o != nullptr) {
          o->pool_slot = -1; /* its grid has left; it takes a stream again when it next launches */
        }
        pool->owner[i] = this;
        pool_slot      = static_cast<int>(i);
        stream         = pool->streams[i];
        return true;
      }
    }
    return false;
  }

  /* A grid is running, or this launches one; called with mu held. The grid's last workgroup to leave stores
   * exit_target into the pinned word hctl[DWQ_H_EXITED], so the submit path reads one host word instead of querying
   * the runtime (hipEventQuery, plus hipSetDevice, on every submit serialised the T = 8 software route's threads on the
   * queue mutex); query_event (the waiters' periodic check) also asks the runtime, which reports a faulted grid.
   * no_stream is set (and hipSuccess returned) when no grid runs and the budget has no stream free. */
  hipError_t ensure_running(bool query_event, bool& no_stream)
  {
    no_stream    = false;
    hipError_t e = hipSuccess;
    if (failed.load(std::memory_order_acquire)) {
      return hipErrorLaunchTimeOut; /* never relaunched after a timed-out wait (dwq_wait) */
    }
    if (running(query_event, e) || e != hipSuccess) {
      return e;
    }
    if (!take_stream()) {
      no_stream = true;
      return hipSuccess;
    }
    (void)hipSetDevice(device);
    dwq_args a{};
    a.ring       = static_cast<const uint32_t*>(ring_dev);
    a.host_ctl   = static_cast<const uint32_t*>(hctl_dev);
    a.dev_ctl    = dctl;
    a.done       = static_cast<uint32_t*>(done_dev);
    a.ring_mask  = RING - 1;
    a.ctl_lds    = ctl_lds;
    a.idle_ticks = idle_ticks;
    a.life_ticks = life_ticks;
    a.slot_ticks = slot_ticks;
    a.poll_flags = poll_flags;
    a.host_exit  = static_cast<uint32_t*>(hctl_dev) + DWQ_H_EXITED;
    a.exit_target = exit_target.load() + static_cast<uint32_t>(grid);
    void* args[] = {&a};
    e            = hipLaunchKernel(kernel, dim3(grid), dim3(block), args, lds, stream);
    if (e == hipSuccess) {
      e = hipEventRecord(ended, stream);
    }
    launched = e == hipSuccess;
    if (launched) {
      exit_target.store(a.exit_target, std::memory_order_release);
    }
    return e;
  }
  hipError_t ensure_running(bool query_event = false)
  {
    bool no_stream = false;
    return ensure_running(query_event, no_stream);
  }
};

namespace {

std::mutex                                 g_mu;
std::map<std::pair<int, int>, dwq*>        g_queues; /* (device, key) -> queue, alive for the process */
std::map<int, dwq_pool*>                   g_pools;  /* device -> stream pool, alive for the process */
std::once_flag                             g_exit_once;

/* at process exit: ask every running grid to stop and give it a moment to drain (each exits within its idle period
 * anyway) */
void stop_all()
{
  std::lock_guard<std::mutex> lock(g_mu);
  for (auto& kv : g_queues) {
    dwq* q = kv.second;
    __atomic_store_n(&q->hctl[DWQ_H_STOP], 1U, __ATOMIC_RELEASE);
  }
  for (auto& kv : g_queues) {
    dwq* q = kv.second;
    if (!q->launched) {
      continue;
    }
    for (int i = 0; i != 200000 && hipEventQuery(q->ended) == hipErrorNotReady; ++i) {
      std::this_thread::yield();
    }
  }
}

/* the device's stream pool, created on first use (with g_mu held) */
dwq_pool* pool_of(int device, int grid)
{
  dwq_pool*& p = g_pools[device];
  if (p != nullptr) {
    return p;
  }
  auto      np     = std::make_unique<dwq_pool>();
  const long budget = std::max(1L, std::min(4096L, env_long("LDPC_HIP_DWQ_BUDGET", 128)));
  /* Resident grids at once: the residency budget in workgroups, and at most LDPC_HIP_DWQ_MAX_QUEUES (default 3, at
   * most 8) hardware queues. Every resident grid keeps a hardware queue active, and a batch kernel launched while
   * four other queues hold resident kernels runs 30-37% slower (eight: 94%), with one, two or three 2-5%, whatever
   * those kernels do and however few CUs they hold (profiles/r06/resident_tax_ab*.txt: sleeper kernels of 8-128
   * workgroups on 1-8 CU-masked streams beside C2; dwq_tax_ab_cap3.txt: four graphs' grids requested, three
   * resident, C2 +3.4%). */
  const long maxq = std::max(1L, std::min(8L, env_long("LDPC_HIP_DWQ_MAX_QUEUES", 3)));
  const long n    = std::max(1L, std::min(maxq, budget / std::max(1, grid)));
  (void)hipSetDevice(device);
  for (long i = 0; i != n; ++i) {
    hipStream_t st = nullptr;
    std::vector<uint32_t> mask(8, 0xffffffffU);
    /* CU-masked: a hardware queue of its own, so that a resident grid never holds up kernels queued behind it. A
     * plain stream would share a hardware queue with other streams: such a pool is not used (the launch path serves) */
    const hipError_t e = hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(mask.size()), mask.data());
    if (e != hipSuccess) {
      (void)hipGetLastError();
      std::fprintf(stderr, "ldpc_hip: device %d: hipExtStreamCreateWithCUMask failed (%s); the device work queue is "
                           "disabled there, the launch path serves\n", device, hipGetErrorString(e));
      for (hipStream_t s0 : np->streams) {
        (void)hipStreamDestroy(s0);
      }
      np->streams.clear();
      break;
    }
    np->streams.push_back(st);
    np->owner.push_back(nullptr);
  }
  if (np->streams.empty()) {
    return nullptr;
  }
  p = np.release();
  return p;
}

hipError_t create(dwq& q, int device, int key, int block, uint32_t body_lds)
{
  q.device  = device;
  q.key     = key;
  q.kernel  = key_kernel(key);
  q.block   = block;
  q.ctl_lds = (body_lds + 15U) & ~15U;
  q.lds     = q.ctl_lds + DWQ_LDS_EXTRA;
  /* One workgroup per CU: a small graph's workgroup (BG2 Z=36: 2 waves, 33 KB) would otherwise share a CU with up to
   * three others of its grid, and concurrent items then share its SIMDs. Reserving more than half of the CU's 160 KB
   * of LDS spreads the grid over as many CUs as it has workgroups (LDPC_HIP_DWQ_SPREAD=0: the body's LDS only). */
  if (env_long("LDPC_HIP_DWQ_SPREAD", 1) != 0) {
    q.lds = std::max<uint32_t>(q.lds, 84U * 1024U);
  }
  q.grid    = static_cast<int>(std::max(1L, std::min(1024L, env_long("LDPC_HIP_DWQ_WORKGROUPS", 32))));
  q.idle_ticks = static_cast<uint32_t>(std::max(10L, std::min(1000000L, env_long("LDPC_HIP_DWQ_IDLE_US", 2000))) * 100);
  q.life_ticks = 5000000; /* 50 ms */
  /* idle polling: the grid reads the next ring slot once per LDPC_HIP_DWQ_SLOT_TICKS (100 MHz ticks, default 25 =
   * 0.25 us), its workgroups in turns; LDPC_HIP_DWQ_POLL_FLAGS (DWQ_POLL_*) */
  q.slot_ticks = static_cast<uint32_t>(std::max(1L, std::min(100000L, env_long("LDPC_HIP_DWQ_SLOT_TICKS", 25))));
  q.poll_flags = static_cast<uint32_t>(env_long("LDPC_HIP_DWQ_POLL_FLAGS", 0));
  q.pool       = pool_of(device, q.grid);
  if (q.kernel == nullptr || q.pool == nullptr) {
    return hipErrorInvalidValue;
  }
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) {
    e = hipFuncSetAttribute(q.kernel, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(q.lds));
  }
  void* p = nullptr;
  if (e == hipSuccess && (e = hipHostMalloc(&p, RING * DWQ_WIRE_WORDS * 4, hipHostMallocMapped | hipHostMallocCoherent)) ==
                             hipSuccess) {
    q.ring = static_cast<uint32_t*>(p);
    std::memset(p, 0, RING * DWQ_WIRE_WORDS * 4);
    e = hipHostGetDevicePointer(&q.ring_dev, p, 0);
  }
  if (e == hipSuccess && (e = hipHostMalloc(&p, DWQ_H_WORDS * 4, hipHostMallocMapped | hipHostMallocCoherent)) ==
                             hipSuccess) {
    q.hctl = static_cast<uint32_t*>(p);
    std::memset(p, 0, DWQ_H_WORDS * 4);
    e = hipHostGetDevicePointer(&q.hctl_dev, p, 0);
  }
  if (e == hipSuccess && (e = hipHostMalloc(&p, RING * 4, hipHostMallocMapped | hipHostMallocCoherent)) == hipSuccess) {
    q.done = static_cast<uint32_t*>(p);
    std::memset(p, 0, RING * 4);
    e = hipHostGetDevicePointer(&q.done_dev, p, 0);
  }
  if (e == hipSuccess && (e = hipMalloc(&p, DWQ_D_WORDS * 4)) == hipSuccess) {
    q.dctl = static_cast<uint32_t*>(p);
    e      = hipMemset(p, 0, DWQ_D_WORDS * 4);
  }
  if (e == hipSuccess) {
    e = hipEventCreateWithFlags(&q.ended, hipEventDisableTiming);
  }
  return e;
}

/* An item's words on the wire, published: three 64-byte lines, each line's sequence word written after its payload;
 * a poller reading a line with the new sequence word reads its new payload too on x86 (stores become visible in
 * order), and the checksum in word 44 catches any read that is not a snapshot of one publication (dwq_item_checksum,
 * checked by dwq_loop before the claim). */
void publish(dwq* q, const dwq_item& item, uint32_t wire_ticket)
{
  const uint32_t  slot = wire_ticket & (RING - 1);
  const uint32_t* src  = reinterpret_cast<const uint32_t*>(&item);
  uint32_t*       dst  = q->ring + static_cast<size_t>(slot) * DWQ_WIRE_WORDS;
  for (uint32_t line = 0; line != 3; ++line) {
    std::memcpy(dst + 16U * line, src + 15U * line, 15U * 4U);
    __atomic_store_n(dst + 16U * line + 15U, wire_ticket + 1U, __ATOMIC_RELEASE);
  }
}


/* the item last published in `ticket`'s ring slot (publish() inverted) */
dwq_item read_back(const dwq* q, uint32_t ticket)
{
  dwq_item        it{};
  uint32_t        w[DWQ_ITEM_WORDS] = {};
  const uint32_t* src = q->ring + static_cast<size_t>(ticket & (RING - 1)) * DWQ_WIRE_WORDS;
  for (uint32_t line = 0; line != 3; ++line) {
    for (uint32_t k = 0; k != 15 && 15U * line + k < DWQ_ITEM_WORDS; ++k) {
      w[15U * line + k] = __atomic_load_n(src + 16U * line + k, __ATOMIC_RELAXED);
    }
  }
  std::memcpy(&it, w, sizeof(it));
  return it;
}

/* with q->mu held: no grid of the queue is resident (every launched workgroup has left, and the runtime has the last
 * grid ended), so nothing can claim or still be running one of its items */
bool quiesced_locked(dwq* q)
{
  hipError_t e = hipSuccess;
  return !q->running(true, e);
}

/* how long dwq_wait waits for an item (LDPC_HIP_DWQ_WAIT_MS, default 10 s; tests shorten it) */
std::chrono::milliseconds wait_limit()
{
  static const long ms = std::max(1L, env_long("LDPC_HIP_DWQ_WAIT_MS", 10000));
  return std::chrono::milliseconds(ms);
}
} // namespace

bool dwq_enabled()
{
  static const bool on = env_long("LDPC_HIP_DWQ", 1) != 0;
  return on;
}

dwq* dwq_get(int device, int key, int block, uint32_t body_lds)
{
  if (!dwq_enabled()) {
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  dwq*&                       q = g_queues[{device, key}];
  if (q == nullptr) {
    auto nq = std::make_unique<dwq>();
    if (create(*nq, device, key, block, body_lds) != hipSuccess) {
      (void)hipGetLastError();
      g_queues.erase({device, key}); /* leaks the partial buffers of a failed queue; the launch path serves */
      return nullptr;
    }
    q = nq.release();
    std::call_once(g_exit_once, [] { std::atexit(stop_all); });
  }
  if (q->failed.load(std::memory_order_acquire)) {
    return nullptr; /* a wait on this queue timed out: the launch path serves */
  }
  return (q->block >= block && q->ctl_lds >= body_lds) ? q : nullptr;
}

bool dwq_admit(dwq* q)
{
  std::lock_guard<std::mutex> lock(q->mu);
  bool             no_stream = false;
  const hipError_t e         = q->ensure_running(false, no_stream);
  const bool       ok        = e == hipSuccess && !no_stream && !q->failed.load(std::memory_order_acquire);
  if (ok) {
    q->pins.fetch_add(1, std::memory_order_acq_rel);
  }
  return ok;
}

void dwq_unpin(dwq* q)
{
  if (q != nullptr) {
    q->pins.fetch_sub(1, std::memory_order_acq_rel);
  }
}

hipError_t dwq_submit(dwq* q, dwq_item item, uint32_t& ticket, bool may_refuse)
{
  std::unique_lock<std::mutex> lock(q->mu);
  if (q->failed.load(std::memory_order_acquire)) {
    return hipErrorLaunchTimeOut;
  }
  if (may_refuse) {
    /* no grid running and none can start within the budget: nothing is published, the caller launches instead */
    bool             no_stream = false;
    const hipError_t e         = q->ensure_running(false, no_stream);
    if (e != hipSuccess) {
      return e;
    }
    if (no_stream) {
      return hipErrorLaunchOutOfResources;
    }
  }
  const uint64_t t    = q->next;
  const uint32_t wt   = static_cast<uint32_t>(t); /* the wire ticket (32 bits; the device compares modulo 2^32) */
  const uint32_t slot = wt & (RING - 1);
  /* the slot's previous item (ticket t - RING) must be done before its words are overwritten */
  for (long spins = 0; t >= RING; ++spins) {
    const uint32_t d = __atomic_load_n(&q->done[slot], __ATOMIC_ACQUIRE);
    if (static_cast<int32_t>(d - (wt - RING + 1U)) >= 0) {
      break;
    }
    if ((spins & 255) == 0) {
      const hipError_t e = q->ensure_running();
      if (e != hipSuccess) {
        return e;
      }
    }
    lock.unlock();
    std::this_thread::yield();
    lock.lock();
  }
  item.ticket = wt;
  item.pad[0] = dwq_item_checksum(item);
  publish(q, item, wt);
#ifdef LDPC_HIP_DIAG_DWQ
  q->sub_ns[slot]   = host_ns();
  q->sub_spec[slot] = item.spec;
#endif
  __atomic_store_n(&q->hctl[DWQ_H_PUBLISHED], wt + 1U, __ATOMIC_RELEASE); /* diagnostics only */
  q->next = t + 1U;
  ticket  = wt;
  /* a grid for the item: when none runs and the budget has no stream free, wait (bounded by the other grids' 2 ms
   * idle period and 50 ms lifetime) -- the item is published and its ticket must be served in order */
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    bool             no_stream = false;
    const hipError_t e         = q->ensure_running(false, no_stream);
    if (e != hipSuccess || !no_stream) {
      if (e != hipSuccess) {
        /* the grid could not be launched: the item becomes a no-op, so that a later grid that claims its ticket
         * touches none of the caller's buffers (which the caller frees or reuses after this error) */
        item.spec   = DWQ_SPEC_NOOP;
        item.pad[0] = dwq_item_checksum(item);
        publish(q, item, wt);
      }
      return e;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
      item.spec   = DWQ_SPEC_NOOP;
      item.pad[0] = dwq_item_checksum(item);
      publish(q, item, wt);
      return hipErrorLaunchOutOfResources;
    }
    lock.unlock();
    std::this_thread::yield();
    lock.lock();
  }
}

#ifdef LDPC_HIP_DIAG_DWQ
void diag_record(dwq* q, uint32_t ticket)
{
  const uint32_t  slot = ticket & (RING - 1);
  const uint64_t  now  = host_ns();
  const uint32_t* pw   = q->ring + static_cast<size_t>(slot) * DWQ_WIRE_WORDS;
  std::lock_guard<std::mutex> lock(g_diag_mu);
  g_diag.insert(g_diag.end(), {q->sub_ns[slot], now, pw[44], pw[45], pw[46], pw[14], q->sub_spec[slot], g_entry_ns});
}
#endif

void dwq_diag_entry()
{
#ifdef LDPC_HIP_DIAG_DWQ
  g_entry_ns = host_ns();
#endif
}

bool dwq_done(dwq* q, uint32_t ticket)
{
  const uint32_t d = __atomic_load_n(&q->done[ticket & (RING - 1)], __ATOMIC_ACQUIRE);
  if (static_cast<int32_t>(d - (ticket + 1U)) >= 0) {
#ifdef LDPC_HIP_DIAG_DWQ
    diag_record(q, ticket);
#endif
    return true;
  }
  if (q->maybe_gone()) {
    std::unique_lock<std::mutex> lock(q->mu, std::try_to_lock);
    if (lock.owns_lock()) {
      (void)q->ensure_running();
    }
  }
  return false;
}

hipError_t dwq_wait(dwq* q, uint32_t ticket)
{
  const uint32_t* flag = &q->done[ticket & (RING - 1)];
  const auto      t0   = std::chrono::steady_clock::now();
  auto            tq   = t0; /* the last runtime query (a faulted grid never reports its exit) */
  for (uint32_t spins = 1;; ++spins) {
    if (static_cast<int32_t>(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - (ticket + 1U)) >= 0) {
#ifdef LDPC_HIP_DIAG_DWQ
      diag_record(q, ticket);
#endif
      return hipSuccess;
    }
    _mm_pause();
    if ((spins & 1023) == 0) {
      const auto now   = std::chrono::steady_clock::now();
      const bool query = now - tq > std::chrono::milliseconds(1);
      if (query || q->maybe_gone()) {
        std::lock_guard<std::mutex> lock(q->mu);
        const hipError_t            e = q->ensure_running(query);
        if (e != hipSuccess) {
          return e;
        }
        tq = query ? now : tq;
      }
      if (now - t0 > wait_limit()) {
        /* The queue takes no more items (dwq_get returns nullptr for it, so callers launch instead) and no grid is
         * launched for it again. Its grid is stopped (a stopped grid claims nothing, dwq_loop) and the item, if still
         * unclaimed, is republished as a no-op; once the grid has left, no item of the queue can touch the caller's
         * buffers any more (dwq_quiesced). */
        std::lock_guard<std::mutex> lock(q->mu);
        q->failed.store(true, std::memory_order_release);
        __atomic_store_n(&q->hctl[DWQ_H_STOP], 1U, __ATOMIC_RELEASE);
        if (static_cast<int32_t>(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - (ticket + 1U)) < 0) {
          dwq_item it = read_back(q, ticket);
          it.spec     = DWQ_SPEC_NOOP;
          it.pad[0]   = dwq_item_checksum(it);
          publish(q, it, ticket);
        }
        bool left = false;
        for (int i = 0; i != 200 && !(left = quiesced_locked(q)); ++i) {
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        std::fprintf(stderr,
                     "ldpc_hip: work queue %d on device %d: item %u not done after %lld ms; queue disabled (later calls "
                     "take the launch path), grid %s\n",
                     q->key, q->device, ticket,
                     static_cast<long long>(std::chrono::duration_cast<std::chrono::milliseconds>(wait_limit()).count()),
                     left ? "stopped and gone" : "asked to stop but still resident");
        return hipErrorLaunchTimeOut;
      }
    }
  }
}

bool dwq_quiesced(dwq* q)
{
  std::lock_guard<std::mutex> lock(q->mu);
  return quiesced_locked(q);
}

} // namespace ldpc_hip

#ifdef LDPC_HIP_DIAG_DWQ
/* diagnostic build only: copies up to max_records completed-item records (8 uint64 each, diag_record) and clears them */
extern "C" __attribute__((visibility("default"))) uint32_t ldpc_hip_diag_dwq_read(uint64_t* out, uint32_t max_records)
{
  std::lock_guard<std::mutex> lock(ldpc_hip::g_diag_mu);
  const uint32_t n = static_cast<uint32_t>(std::min<size_t>(max_records, ldpc_hip::g_diag.size() / 8));
  std::memcpy(out, ldpc_hip::g_diag.data(), static_cast<size_t>(n) * 8 * sizeof(uint64_t));
  ldpc_hip::g_diag.clear();
  return n;
}
#endif
