/* A verifier (include/fd_verify_tile.h fdgpu_verifier_t) that accepts every
   transaction at once, with no GPU and no signature check: a host-path cost
   probe for the verify tile (tools/tile_host_probe.py), so ingest, parse,
   tcache and publish are timed without the engine.  Bench infrastructure
   only -- it verifies nothing.
   Build: gcc -O2 -shared -fPIC -I include tools/null_verifier.c -o tools/libnullver.so */
#include <stdlib.h>
#include <string.h>

#include "fd_verify_tile.h"

#define NV_RING 256

typedef struct { int64_t next; uint64_t cnt[NV_RING]; fdgpu_frag_io_t const *sz[NV_RING]; } nv_t;

static int64_t nv_submit(void *ctx, uint8_t const *arena, uint64_t arena_sz, fdgpu_txn_t const *txns, uint64_t n) {
  (void)arena; (void)arena_sz; (void)txns;
  nv_t *v = (nv_t *)ctx;
  v->cnt[v->next % NV_RING] = n;
  return v->next++;
}

static int nv_poll(void *ctx, int64_t ticket, int8_t *codes, int blocking) {
  (void)blocking;
  nv_t *v = (nv_t *)ctx;
  if (codes) memset(codes, 0, v->cnt[ticket % NV_RING]);
  return FDGPU_OK;
}

/* frag batches: every frag "parses" to the footprint the tile reserved */
static int64_t nv_submit_frags(void *ctx, uint8_t const *arena, uint64_t arena_sz, fdgpu_frag_ex_t const *frags,
                               uint64_t n, uint64_t trailer_sz) {
  (void)arena; (void)arena_sz; (void)frags; (void)trailer_sz;
  nv_t *v = (nv_t *)ctx;
  v->cnt[v->next % NV_RING] = n;
  return v->next++;
}

static int nv_poll_frags(void *ctx, int64_t ticket, int8_t *codes, uint8_t *trailers, int blocking) {
  (void)trailers;
  return nv_poll(ctx, ticket, codes, blocking);
}

/* gathered frag batches: every frag accepted with a distinct tag and an out
   size within its reservation; nothing is read or written */
static uint64_t nv_tag = 1;
static int64_t nv_submit_io(void *ctx, fdgpu_frag_io_t const *frags, uint64_t n, uint8_t *out, uint64_t out_sz,
                            uint64_t seed, fdgpu_link_t const *links, uint64_t link_cnt) {
  (void)out; (void)out_sz; (void)seed; (void)links; (void)link_cnt;
  nv_t *v = (nv_t *)ctx;
  v->cnt[v->next % NV_RING] = n;
  v->sz[v->next % NV_RING] = frags;
  return v->next++;
}

static int nv_poll_io(void *ctx, int64_t ticket, int8_t *codes, uint64_t *tags, uint16_t *out_szs, int blocking) {
  nv_t *v = (nv_t *)ctx;
  const uint64_t n = v->cnt[ticket % NV_RING];
  fdgpu_frag_io_t const *f = v->sz[ticket % NV_RING];
  for (uint64_t i = 0; i < n; i++) { tags[i] = __atomic_fetch_add(&nv_tag, 1, __ATOMIC_RELAXED); out_szs[i] = (uint16_t)(f[i].sz + 32u); }
  return nv_poll(ctx, ticket, codes, blocking);
}

void null_verifier_make(fdgpu_verifier_t *out) {
  memset(out, 0, sizeof(*out));
  out->ctx = calloc(1, sizeof(nv_t));
  out->submit = nv_submit;
  out->poll = nv_poll;
  out->submit_frags = nv_submit_frags;
  out->poll_frags = nv_poll_frags;
  out->submit_io = nv_submit_io;
  out->poll_io = nv_poll_io;
}
