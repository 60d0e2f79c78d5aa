/*
 * TEST / BASELINE INFRASTRUCTURE ONLY -- never part of the product path.
 *
 * Timing loop of bench.py's cpu_baseline leg, in C so that the threads of the all-cores figure never wait on the
 * Python interpreter between decodes. It follows the reference's decoder benchmark
 * (tests/benchmarks/phy/upper/channel_coding/ldpc/ldpc_decoder_benchmark.cpp:87-189 with benchmark_utils.h:156-230):
 * one decoder per thread (the CPU port keeps one state per thread), `reps` timed single-codeblock decodes per thread,
 * every decode's latency recorded for the median / 99th percentile, and the wall time of the whole run.
 */
#define _GNU_SOURCE
#include "ldpc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <time.h>

typedef struct {
  int            bg;
  unsigned       Z, llr_len, iters, reps;
  const int8_t*  llr;
  uint32_t*      lat_ns; /* reps entries of this thread */
  int            status;
} bench_arg;

static uint64_t now_ns(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ULL + (uint64_t)ts.tv_nsec;
}

static void* bench_thread(void* p)
{
  bench_arg* a = (bench_arg*)p;
  uint8_t    out[(26 * 384 + 7) / 8];
  /* warm-up: the thread's decoder state and its first page faults (one decode, inside the wall time) */
  a->status = orc_ldpc_decode_port(a->bg, a->Z, 0, a->llr, a->llr_len, a->iters, -1, out) < 0 ? -1 : 0;
  for (unsigned r = 0; r != a->reps && a->status == 0; ++r) {
    const uint64_t t0 = now_ns();
    if (orc_ldpc_decode_port(a->bg, a->Z, 0, a->llr, a->llr_len, a->iters, -1, out) < 0) {
      a->status = -1;
    }
    const uint64_t dt = now_ns() - t0;
    a->lat_ns[r]      = dt > 0xffffffffULL ? 0xffffffffU : (uint32_t)dt;
  }
  return NULL;
}

int orc_bench_port(int bg, unsigned Z, const int8_t* llr, unsigned llr_len, unsigned iters, unsigned threads,
                   unsigned reps, uint32_t* lat_ns, double* wall_s)
{
  if (threads == 0 || threads > 1024 || reps == 0 || lat_ns == NULL || wall_s == NULL || Z > 384) {
    return -1;
  }
  bench_arg* args = (bench_arg*)calloc(threads, sizeof(bench_arg));
  pthread_t* tids = (pthread_t*)calloc(threads, sizeof(pthread_t));
  int        rc   = 0;
  if (args == NULL || tids == NULL) {
    free(args);
    free(tids);
    return -1;
  }
  const uint64_t t0      = now_ns();
  unsigned       started = 0;
  for (unsigned t = 0; t != threads; ++t) {
    args[t] = (bench_arg){bg, Z, llr_len, iters, reps, llr, lat_ns + (size_t)t * reps, 0};
    if (pthread_create(&tids[t], NULL, bench_thread, &args[t]) != 0) {
      rc = -1;
      break;
    }
    ++started;
  }
  for (unsigned t = 0; t != started; ++t) {
    pthread_join(tids[t], NULL);
    rc = (args[t].status != 0) ? -1 : rc;
  }
  *wall_s = (double)(now_ns() - t0) * 1e-9;
  free(args);
  free(tids);
  return rc;
}
