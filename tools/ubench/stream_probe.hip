// Which HIP runtime calls accept the special stream handles hipStreamLegacy ((hipStream_t)1) and hipStreamPerThread
// ((hipStream_t)2)? Round 4's hipStreamLegacy launch segfaulted in a multi-group decode plan's fork
// (ldpc_hip_api.cpp launch_plan: hipEventRecord on the caller's stream, hipStreamWaitEvent of the auxiliary streams,
// launches, then hipEventRecord on the auxiliary streams and hipStreamWaitEvent of the caller's stream).
// This probe makes each of those calls once per handle, in that order, printing (unbuffered) the call it is about to
// make: the last "call" line before a crash names the faulting call; a SIGSEGV handler prints the runtime frames.
// Build: hipcc -O1 -g --offload-arch=gfx950 -o stream_probe stream_probe.hip   (diagnostic, not product code)
#include <hip/hip_runtime.h>

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <execinfo.h>
#include <unistd.h>

__global__ void touch(int* p) { p[threadIdx.x] += 1; }

static void on_segv(int sig)
{
  void*     frames[32];
  const int n = backtrace(frames, 32);
  dprintf(2, "signal %d, backtrace:\n", sig);
  backtrace_symbols_fd(frames, n, 2);
  _exit(128 + sig);
}

static int check(const char* what, hipError_t e)
{
  std::printf("  -> %s: %s\n", what, hipGetErrorString(e));
  std::fflush(stdout);
  return (e == hipSuccess || e == hipErrorNotReady) ? 0 : 1; /* hipStreamQuery: not ready is an answer */
}

#define CALL(expr)                                                                                                     \
  do {                                                                                                                 \
    std::printf("call %s\n", #expr);                                                                                   \
    std::fflush(stdout);                                                                                               \
    bad += check(#expr, (expr));                                                                                       \
  } while (0)

int main(int argc, char** argv)
{
  std::signal(SIGSEGV, on_segv);
  std::signal(SIGBUS, on_segv);
  const int which = argc > 1 ? std::atoi(argv[1]) : 1; /* 1 = hipStreamLegacy, 2 = hipStreamPerThread */
  const hipStream_t h = which == 2 ? hipStreamPerThread : hipStreamLegacy;
  std::printf("handle %s (%p)\n", which == 2 ? "hipStreamPerThread" : "hipStreamLegacy", static_cast<void*>(h));
  int*        d   = nullptr;
  hipStream_t aux = nullptr;
  hipEvent_t  fork = nullptr, join = nullptr;
  int         bad = 0;
  CALL(hipMalloc(&d, 256));
  CALL(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
  CALL(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CALL(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CALL(hipMemsetAsync(d, 0, 256, h));
  std::printf("call hipLaunchKernelGGL(touch, h)\n");
  std::fflush(stdout);
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, h, d);
  bad += check("hipLaunchKernelGGL(touch, h)", hipGetLastError());
  CALL(hipStreamQuery(h));
  CALL(hipEventRecord(fork, h));                 /* launch_plan: fork point on the caller's stream */
  CALL(hipStreamWaitEvent(aux, fork, 0));        /* auxiliary stream waits for it */
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, aux, d);
  CALL(hipEventRecord(join, aux));               /* auxiliary stream done */
  CALL(hipStreamWaitEvent(h, join, 0));          /* caller's stream waits for it (the join) */
  CALL(hipStreamSynchronize(h));
  int flags = -1;
  CALL(hipStreamGetFlags(h, reinterpret_cast<unsigned int*>(&flags)));
  CALL(hipDeviceSynchronize());
  int host[64] = {};
  CALL(hipMemcpy(host, d, sizeof(host), hipMemcpyDeviceToHost));
  std::printf("result %d %d (expect 2 2), failed calls %d\n", host[0], host[63], bad);
  return bad == 0 && host[0] == 2 ? 0 : 1;
}
