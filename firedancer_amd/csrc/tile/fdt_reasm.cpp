/* fdt_reasm.cpp -- TPU stream reassembly, the producer side of the
   quic -> verify link (SURVEY.md §8(f) row 2, Appendix B "quic->verify
   input"), restated from the behaviour documented in
   src/disco/quic/fd_tpu.h:20-246 and fd_tpu_reasm.c.

   The verify tile's in link in the reference is not a compact dcache: frags
   point into a slot arena of depth + burst reassembly buffers of
   FD_TPU_REASM_MTU (1280) bytes each, and the tile's valid chunk range is
   [chunk0, chunk0 + (depth + burst - 1) * 20] (fd_verify.c:186-191).
   Ownership rules reproduced here:
     * exactly `depth` slots are published (owned by the mcache lines; the
       slot behind line seq & (depth-1) is recorded in pub[]) and exactly
       `burst` are owned by reassembly (FREE or BUSY) at any time;
     * publishing seq hands the slot that line held back to reassembly, so
       a consumer's payload stays intact until `depth` later publishes --
       the window the mcache overrun check protects;
     * prepare takes a FREE slot if there is one, else cancels the least
       recently prepared BUSY one (FIFO eviction: unfragmented txns are
       never dropped);
     * append accepts in-order stream data only (gap: cancel + ERR_SKIP,
       already-seen prefix skipped, > FD_TXN_MTU: cancel + ERR_SZ).
   Reassembly-owned slots live on one index-linked list: FREE ones at the
   back, BUSY ones in front of them, most recently prepared first. */
#include <string.h>

#include "../../../include/fd_verify_tile.h"

namespace {

constexpr uint64_t REASM_MAGIC = 0xFD7A9E5A5300C0DEull;
constexpr uint32_t NIL = 0xFFFFFFFFu;

struct slot_t {
  uint32_t prev, next;     /* reassembly list links (NIL at the ends) */
  uint32_t tsorig;
  uint16_t sz;
  uint8_t state;
  uint8_t _pad;
};

struct reasm_t {
  uint64_t magic;
  uint32_t depth, burst, slot_cnt, orig;
  uint32_t front, back;    /* reassembly list: front = newest BUSY, back = FREE end */
  uint64_t pub_off, slots_off, data_off;
};

uint64_t up(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

uint32_t *pub_of(reasm_t *r) { return (uint32_t *)((uint8_t *)r + r->pub_off); }
slot_t *slots_of(reasm_t *r) { return (slot_t *)((uint8_t *)r + r->slots_off); }
uint8_t *data_of(reasm_t *r, uint32_t i) { return (uint8_t *)r + r->data_off + (uint64_t)i * FDT_TPU_REASM_MTU; }

void unlink_slot(reasm_t *r, uint32_t i) {
  slot_t *s = slots_of(r);
  if (s[i].prev != NIL) s[s[i].prev].next = s[i].next; else r->front = s[i].next;
  if (s[i].next != NIL) s[s[i].next].prev = s[i].prev; else r->back = s[i].prev;
  s[i].prev = s[i].next = NIL;
}
void push_front(reasm_t *r, uint32_t i) {
  slot_t *s = slots_of(r);
  s[i].prev = NIL; s[i].next = r->front;
  if (r->front != NIL) s[r->front].prev = i; else r->back = i;
  r->front = i;
}
void push_back(reasm_t *r, uint32_t i) {
  slot_t *s = slots_of(r);
  s[i].next = NIL; s[i].prev = r->back;
  if (r->back != NIL) s[r->back].next = i; else r->front = i;
  r->back = i;
}

reasm_t *cast(void *p) {
  auto *r = (reasm_t *)p;
  return (r && r->magic == REASM_MAGIC) ? r : nullptr;
}

}  // namespace

extern "C" {

uint64_t fdt_tpu_reasm_footprint(uint64_t depth, uint64_t burst) {
  if (!depth || (depth & (depth - 1)) || depth > 0x7fffffffu || burst < 2 || burst > 0x7fffffffu) return 0;
  const uint64_t n = depth + burst;
  uint64_t off = up(sizeof(reasm_t), 64);
  off = up(off + depth * 4, 64);
  off = up(off + n * sizeof(slot_t), 64);
  return off + n * FDT_TPU_REASM_MTU;
}

void fdt_tpu_reasm_reset(void *mem) {
  reasm_t *r = cast(mem);
  if (!r) return;
  slot_t *s = slots_of(r);
  uint32_t *pub = pub_of(r);
  for (uint32_t j = 0; j < r->slot_cnt; j++) s[j] = slot_t{NIL, NIL, 0, 0, FDT_TPU_REASM_STATE_FREE, 0};
  for (uint32_t j = 0; j < r->depth; j++) { s[j].state = FDT_TPU_REASM_STATE_PUB; pub[j] = j; }
  r->front = r->back = NIL;
  for (uint32_t j = r->depth; j < r->slot_cnt; j++) push_back(r, j);
}

void *fdt_tpu_reasm_new(void *mem, uint64_t depth, uint64_t burst, uint64_t orig) {
  if (!mem || ((uintptr_t)mem & 63) || !fdt_tpu_reasm_footprint(depth, burst)) return nullptr;
  auto *r = (reasm_t *)mem;
  memset(r, 0, sizeof(*r));
  r->depth = (uint32_t)depth;
  r->burst = (uint32_t)burst;
  r->slot_cnt = (uint32_t)(depth + burst);
  r->orig = (uint32_t)orig;
  r->pub_off = up(sizeof(reasm_t), 64);
  r->slots_off = up(r->pub_off + depth * 4, 64);
  r->data_off = up(r->slots_off + (depth + burst) * sizeof(slot_t), 64);
  r->magic = REASM_MAGIC;
  fdt_tpu_reasm_reset(r);
  return r;
}

uint64_t fdt_tpu_reasm_chunk0(void *mem, void const *base) {
  reasm_t *r = cast(mem);
  return r ? (uint64_t)(data_of(r, 0) - (const uint8_t *)base) >> FDT_CHUNK_LG_SZ : 0;
}
uint64_t fdt_tpu_reasm_wmark(void *mem, void const *base) {
  reasm_t *r = cast(mem);
  return r ? fdt_tpu_reasm_chunk0(mem, base) + (uint64_t)(r->slot_cnt - 1) * FDT_TPU_REASM_CHUNK_MTU : 0;
}

uint32_t fdt_tpu_reasm_prepare(void *mem, uint64_t tsorig) {
  reasm_t *r = cast(mem);
  if (!r) return NIL;
  const uint32_t i = r->back;               /* FREE, or the oldest BUSY when none is free */
  slot_t *s = slots_of(r);
  unlink_slot(r, i);
  s[i].state = FDT_TPU_REASM_STATE_BUSY;
  s[i].sz = 0;
  s[i].tsorig = (uint32_t)tsorig;
  push_front(r, i);
  return i;
}

void fdt_tpu_reasm_cancel(void *mem, uint32_t slot) {
  reasm_t *r = cast(mem);
  if (!r || slot >= r->slot_cnt || slots_of(r)[slot].state != FDT_TPU_REASM_STATE_BUSY) return;
  unlink_slot(r, slot);
  slots_of(r)[slot].state = FDT_TPU_REASM_STATE_FREE;
  push_back(r, slot);
}

int fdt_tpu_reasm_append(void *mem, uint32_t slot, uint8_t const *data, uint64_t data_sz, uint64_t data_off) {
  reasm_t *r = cast(mem);
  if (!r || slot >= r->slot_cnt || slots_of(r)[slot].state != FDT_TPU_REASM_STATE_BUSY)
    return FDT_TPU_REASM_ERR_STATE;
  slot_t &s = slots_of(r)[slot];
  const uint64_t have = s.sz;
  if (data_off > have) { fdt_tpu_reasm_cancel(r, slot); return FDT_TPU_REASM_ERR_SKIP; }
  const uint64_t seen = have - data_off;     /* prefix already reassembled */
  if (seen > data_sz) return FDT_TPU_REASM_SUCCESS;
  data += seen;
  data_sz -= seen;
  if (have + data_sz > FDT_TXN_MTU) { fdt_tpu_reasm_cancel(r, slot); return FDT_TPU_REASM_ERR_SZ; }
  memcpy(data_of(r, slot) + have, data, data_sz);
  s.sz = (uint16_t)(have + data_sz);
  return FDT_TPU_REASM_SUCCESS;
}

int fdt_tpu_reasm_publish(void *mem, uint32_t slot, fdt_frag_meta_t *mcache, void const *base, uint64_t seq,
                          uint64_t tspub) {
  reasm_t *r = cast(mem);
  if (!r || slot >= r->slot_cnt || slots_of(r)[slot].state != FDT_TPU_REASM_STATE_BUSY)
    return FDT_TPU_REASM_ERR_STATE;
  slot_t *s = slots_of(r);
  const uint8_t *d = data_of(r, slot);
  if (d < (const uint8_t *)base || ((uint64_t)(d - (const uint8_t *)base) >> FDT_CHUNK_LG_SZ) > 0xffffffffull)
    return FDT_TPU_REASM_ERR_STATE;
  const uint64_t line = seq & (r->depth - 1);
  uint32_t *pub = pub_of(r);
  const uint32_t freed = pub[line];
  if (freed >= r->slot_cnt || s[freed].state != FDT_TPU_REASM_STATE_PUB) {
    fdt_tpu_reasm_reset(r);                  /* line/slot bookkeeping out of sync */
    return FDT_TPU_REASM_ERR_STATE;
  }
  unlink_slot(r, slot);
  s[slot].state = FDT_TPU_REASM_STATE_PUB;
  pub[line] = slot;
  s[freed].state = FDT_TPU_REASM_STATE_FREE;
  push_back(r, freed);
  fdt_mcache_publish(mcache, r->depth, seq, 0, (uint64_t)(d - (const uint8_t *)base) >> FDT_CHUNK_LG_SZ,
                     s[slot].sz, fdt_frag_meta_ctl(r->orig, 1, 1, 0), s[slot].tsorig, tspub);
  return FDT_TPU_REASM_SUCCESS;
}

int fdt_tpu_reasm_slot_state(void *mem, uint32_t slot) {
  reasm_t *r = cast(mem);
  return (r && slot < r->slot_cnt) ? slots_of(r)[slot].state : -1;
}

}  // extern "C"
