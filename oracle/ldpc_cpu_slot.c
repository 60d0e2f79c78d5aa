/*
 * TEST / BASELINE INFRASTRUCTURE ONLY -- never part of the product path.
 *
 * The CPU leg of bench.py's software-route figure (extra.sw_route.cpu): one PUSCH slot's codeblocks decoded on the host
 * CPU the way the reference's software PUSCH decoder schedules them (pusch_decoder_impl.cpp:309-382 forks one task
 * per codeblock onto its executor; each task runs pusch_codeblock_decoder::decode, pusch_codeblock_decoder.cpp:35-71:
 * rate_dematch into the codeblock's soft buffer, then decode with CRC early stop, on the decoder pair of its worker
 * thread, pusch_decoder_impl.h:48). Workers take codeblocks from a shared counter in slot order, exactly as
 * tests/cpp/bench_sw.cpp runs the GPU pairs, so the two legs time the same schedule:
 *   with_dematch 1: orc_rate_dematch (ldpc_rate_dematcher_impl.cpp:46-213 restated) + the CPU decoder port;
 *   with_dematch 0: decoder only, each soft buffer copied from a pre-dematched one first (bench_sw's decoder_only).
 * The decoder is the AVX2 port (ldpc_cpu_port.c, bit-exact with the oracle); the reference's own AVX2/AVX-512 decoders
 * cannot be built here.
 */
#define _GNU_SOURCE
#include "ldpc_oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
  int                  with_dematch;
  unsigned             n;
  const orc_slot_cb*   cbs;
  int8_t**             soft;  /* per CB: N LLRs (the rx_buffer codeblock) */
  int8_t**             soft0; /* per CB: the pre-dematched soft buffer (decoder only) */
  uint8_t**            msg;
  double*              dec_us; /* per CB, the last rep */
  double*              dm_us;
  atomic_int           gen;
  atomic_size_t        next, done;
  atomic_uint          ok;
  atomic_int           quit;
  atomic_int           fail;
} slot_run;

static uint64_t slot_now_ns(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ULL + (uint64_t)ts.tv_nsec;
}

static unsigned cb_len_of(const orc_slot_cb* c) { return (c->bg == 1 ? 66U : 50U) * c->Z; }

/* pusch_codeblock_decoder::decode for codeblock i on the calling worker */
static void slot_task(slot_run* r, size_t i)
{
  const orc_slot_cb* c  = &r->cbs[i];
  const unsigned     N  = cb_len_of(c);
  const uint64_t     t0 = slot_now_ns();
  if (r->with_dematch) {
    memset(r->soft[i], 0, N); /* a clean rx_buffer codeblock (new data) */
    if (orc_rate_dematch(r->soft[i], N, c->llr, c->E, 1, c->rv, c->Qm, 0, c->F) != 0) {
      atomic_store(&r->fail, 1);
    }
  } else {
    memcpy(r->soft[i], r->soft0[i], N);
  }
  const uint64_t t1 = slot_now_ns();
  const int      it = orc_ldpc_decode_port(c->bg, c->Z, c->F, r->soft[i], N, c->iters, c->crc_poly, r->msg[i]);
  const uint64_t t2 = slot_now_ns();
  if (it < 0) {
    atomic_store(&r->fail, 1);
  }
  r->dm_us[i]  = (double)(t1 - t0) * 1e-3;
  r->dec_us[i] = (double)(t2 - t1) * 1e-3;
  if (it > 0) {
    atomic_fetch_add(&r->ok, 1U);
  }
}

static void* slot_worker(void* p)
{
  slot_run* r    = (slot_run*)p;
  int       seen = 0;
  for (;;) {
    int g;
    while ((g = atomic_load(&r->gen)) == seen && !atomic_load(&r->quit)) {
    }
    if (atomic_load(&r->quit)) {
      return NULL;
    }
    seen = g;
    for (size_t i; (i = atomic_fetch_add(&r->next, 1)) < r->n;) {
      slot_task(r, i);
      atomic_fetch_add(&r->done, 1);
    }
  }
}

int orc_bench_slot(const orc_slot_cb* cbs, unsigned n, unsigned threads, unsigned reps, int with_dematch,
                   double* slot_us, double* dec_us, double* dm_us, unsigned* crc_ok)
{
  if (cbs == NULL || n == 0 || threads == 0 || threads > 256 || reps == 0 || slot_us == NULL || dec_us == NULL ||
      dm_us == NULL || crc_ok == NULL) {
    return -1;
  }
  slot_run   r;
  pthread_t* tids = (pthread_t*)calloc(threads, sizeof(pthread_t));
  memset(&r, 0, sizeof(r));
  r.with_dematch = with_dematch;
  r.n            = n;
  r.cbs          = cbs;
  r.soft         = (int8_t**)calloc(n, sizeof(int8_t*));
  r.soft0        = (int8_t**)calloc(n, sizeof(int8_t*));
  r.msg          = (uint8_t**)calloc(n, sizeof(uint8_t*));
  int rc         = (tids != NULL && r.soft != NULL && r.soft0 != NULL && r.msg != NULL) ? 0 : -1;
  for (unsigned i = 0; i != n && rc == 0; ++i) {
    const unsigned N = cb_len_of(&cbs[i]);
    r.soft[i]        = (int8_t*)calloc(N, 1);
    r.soft0[i]       = (int8_t*)calloc(N, 1);
    r.msg[i]         = (uint8_t*)calloc((N + 7) / 8, 1);
    if (r.soft[i] == NULL || r.soft0[i] == NULL || r.msg[i] == NULL ||
        orc_rate_dematch(r.soft0[i], N, cbs[i].llr, cbs[i].E, 1, cbs[i].rv, cbs[i].Qm, 0, cbs[i].F) != 0) {
      rc = -1;
    }
  }
  unsigned started = 0;
  for (unsigned t = 0; t != threads && rc == 0; ++t) {
    if (pthread_create(&tids[t], NULL, slot_worker, &r) != 0) {
      rc = -1;
      break;
    }
    ++started;
  }
  /* two untimed warm-up slots (thread states, page faults), then `reps` timed ones, as bench_sw */
  for (int rep = -2; rep < (int)reps && rc == 0; ++rep) {
    atomic_store(&r.next, 0);
    atomic_store(&r.done, 0);
    atomic_store(&r.ok, 0);
    r.dec_us = dec_us + (size_t)(rep < 0 ? 0 : rep) * n;
    r.dm_us  = dm_us + (size_t)(rep < 0 ? 0 : rep) * n;
    const uint64_t t0 = slot_now_ns();
    atomic_fetch_add(&r.gen, 1);
    while (atomic_load(&r.done) != n) {
    }
    const uint64_t t1 = slot_now_ns();
    if (rep >= 0) {
      slot_us[rep] = (double)(t1 - t0) * 1e-3;
    }
  }
  atomic_store(&r.quit, 1);
  for (unsigned t = 0; t != started; ++t) {
    pthread_join(tids[t], NULL);
  }
  *crc_ok = atomic_load(&r.ok);
  if (atomic_load(&r.fail)) {
    rc = -1;
  }
  for (unsigned i = 0; r.soft != NULL && i != n; ++i) {
    free(r.soft[i]);
    free(r.soft0[i]);
    free(r.msg[i]);
  }
  free(r.soft);
  free(r.soft0);
  free(r.msg);
  free(tids);
  return rc;
}
