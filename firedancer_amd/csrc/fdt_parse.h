/* fdt_parse.h -- fd_txn_parse as one source for the host and the GPU.

   Restates src/ballet/txn/fd_txn_parse.c:7-243 (with the compact-u16 rules
   of fd_compact_u16.h:29-75): every read is preceded by a check that the
   bytes remain, compact-u16 values must be minimally encoded and fit 16
   bits, and the structural checks run in the reference's order.  Compiled
   by g++ into libfd_verify_tile.so (fdt_txn_parse, the host verify tile)
   and by hipcc into the GPU ingest kernel (fdgpu_frag_parse_kernel, one
   payload per lane), so the two parsers are the same code.

   fdt_parse_core() writes the fd_txn_t (if t != NULL; t needs
   FDT_TXN_MAX_SZ bytes) and returns its footprint, or 0 with *fail set to
   the reason (FDT_PF_*) when the payload is not a valid transaction. */
#pragma once

#include <stdint.h>

#include "../../include/fd_verify_tile.h"

#if defined(__HIPCC__)
#define FDT_HD __host__ __device__ __forceinline__
#define FDT_HDM __host__ __device__ __forceinline__
#else
#define FDT_HD static inline
#define FDT_HDM inline
#endif

/* Failure reasons (the reference records the source line of the failed
   check; any non-zero token serves). */
#define FDT_PF_MTU             1u
#define FDT_PF_SHORT           2u
#define FDT_PF_SIG_CNT         3u
#define FDT_PF_VERSION         4u
#define FDT_PF_HDR_SIG_CNT     5u
#define FDT_PF_RO_SIGNED       6u
#define FDT_PF_CU16            7u
#define FDT_PF_ACCT_CNT        8u
#define FDT_PF_ACCT_SIGNERS    9u
#define FDT_PF_INSTR_CNT      10u
#define FDT_PF_NO_PROGRAM_ACCT 11u
#define FDT_PF_PROGRAM_ID     12u
#define FDT_PF_LUT_CNT        13u
#define FDT_PF_LUT_WRITABLE   14u
#define FDT_PF_LUT_READONLY   15u
#define FDT_PF_LUT_EMPTY      16u
#define FDT_PF_TRAILING       17u
#define FDT_PF_TOTAL_ACCTS    18u
#define FDT_PF_ACCT_IDX       19u

/* A valid txn with s signatures is at least 96 s + 38 bytes (s signatures,
   s signer keys, the blockhash, the counts): an upper bound on the
   signatures a frag of sz bytes can send to the verifier. */
FDT_HD uint32_t fdt_frag_sig_bound(uint64_t sz) {
  return sz >= 134u ? (uint32_t)((sz - 38u) / 96u < 16u ? (sz - 38u) / 96u : 16u) : 0u;
}

FDT_HD uint64_t fdt_parse_footprint(uint64_t instr_cnt, uint64_t lut_cnt) {
  return sizeof(fdt_txn_t) + instr_cnt * sizeof(fdt_txn_instr_t) + lut_cnt * sizeof(fdt_txn_acct_addr_lut_t);
}

/* An upper bound on the footprint of any transaction parsed from sz bytes,
   from the size alone: past the 134 bytes every transaction holds (count,
   one signature, header, one account, blockhash, instruction count) each
   instruction takes at least 3 bytes and each lookup table 34, and the
   parser caps both counts and the footprint (FDT_TXN_MAX_SZ).  The verify
   tile reserves align2(sz) + this + 2 out-dcache bytes for a frag it never
   reads (fdgpu_submit_frags_io: the GPU writes the trailer). */
FDT_HD uint64_t fdt_frag_fp_bound(uint64_t sz) {
  const uint64_t room = sz > 134u ? sz - 134u : 0u;
  const uint64_t ni = room / 3u < FDT_TXN_INSTR_MAX ? room / 3u : FDT_TXN_INSTR_MAX;
  const uint64_t nl0 = (room - 3u * ni) / 34u;
  const uint64_t nl = nl0 < FDT_TXN_ADDR_TABLE_LOOKUP_MAX ? nl0 : FDT_TXN_ADDR_TABLE_LOOKUP_MAX;
  const uint64_t fp = fdt_parse_footprint(ni, nl);
  return fp < FDT_TXN_MAX_SZ ? fp : FDT_TXN_MAX_SZ;
}

/* Bounds-checked reader over an untrusted payload (fd_txn_parse.c:12-75).
   at(k) reads payload byte k (k < sz, checked by the callers).  On the host
   it is a plain load.  On the GPU each lane parses its own payload, so
   byte loads from 64 payloads hundreds of bytes apart would each touch a
   different line, and with every lane of the chip in flight the lines are
   evicted from L2 before the lane comes back for the next byte; there the
   reader keeps the aligned 16 B around the cursor in registers and reloads
   them only when the cursor leaves them (one dwordx4 per 16 bytes read;
   the batch arena has FDGPU_ARENA_SLACK readable bytes past its end). */
struct fdt_reader {
  const uint8_t *p;
  uint64_t sz, i, fail;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint8_t *wb = nullptr;           /* 16-B aligned address of the window */
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  __device__ __forceinline__ uint8_t at(uint64_t k) {
    const uint8_t *a = p + k;
    const uint32_t o = (uint32_t)((uintptr_t)a & 15u);
    const uint8_t *b = a - o;
    if (b != wb) {
      const uint4 v = *(const uint4 *)b;
      w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w; wb = b;
    }
    const uint32_t d = o < 8u ? (o < 4u ? w0 : w1) : (o < 12u ? w2 : w3);
    return (uint8_t)(d >> ((o & 3u) * 8u));
  }
#else
  FDT_HDM uint8_t at(uint64_t k) { return p[k]; }
#endif
  FDT_HDM bool need(uint64_t n, uint64_t why = FDT_PF_SHORT) {
    if (fail) return false;
    if (n > sz - i) { fail = why; return false; }
    return true;
  }
  FDT_HDM bool u8(uint8_t &v) { if (!need(1)) return false; v = at(i++); return true; }
  FDT_HDM bool skip(uint64_t n) { if (!need(n)) return false; i += n; return true; }
  /* fd_compact_u16.h:60-75 */
  FDT_HDM bool cu16(uint16_t &v) {
    if (fail) return false;
    const uint64_t avail = sz - i;
    const uint8_t b0 = avail >= 1 ? at(i) : 0, b1 = avail >= 2 ? at(i + 1) : 0, b2 = avail >= 3 ? at(i + 2) : 0;
    if (avail >= 1 && !(b0 & 0x80)) { v = b0; i += 1; return true; }
    if (avail >= 2 && !(b1 & 0x80)) {
      if (!b1) { fail = FDT_PF_CU16; return false; }
      v = (uint16_t)((b0 & 0x7f) | (b1 << 7)); i += 2; return true;
    }
    if (avail >= 3 && !(b2 & 0xfc)) {
      if (!b2) { fail = FDT_PF_CU16; return false; }
      v = (uint16_t)((b0 & 0x7f) | ((b1 & 0x7f) << 7) | (b2 << 14)); i += 3; return true;
    }
    fail = FDT_PF_CU16;
    return false;
  }
  FDT_HDM bool check(bool ok, uint64_t why) { if (!fail && !ok) fail = why; return !fail; }
};

FDT_HD uint64_t fdt_parse_core(const uint8_t *payload, uint64_t payload_sz, fdt_txn_t *t, uint64_t *fail) {
  fdt_reader r;
  r.p = payload; r.sz = payload_sz; r.i = 0; r.fail = 0;
  uint64_t fp = 0;
  do {
    if (!r.check(payload_sz <= FDT_TXN_MTU, FDT_PF_MTU)) break;

    /* signatures: count (u8 == compact-u16 below 128), at least one signer */
    uint8_t sig_cnt;
    if (!r.u8(sig_cnt) || !r.check(sig_cnt >= 1 && sig_cnt <= FDT_TXN_SIG_MAX, FDT_PF_SIG_CNT)) break;
    const uint64_t sig_off = r.i;
    if (!r.skip(64ULL * sig_cnt)) break;

    /* message header: optional version prefix, then the signer count again */
    const uint64_t msg_off = r.i;
    uint8_t b0;
    if (!r.u8(b0)) break;
    uint8_t version;
    if (b0 & 0x80) {
      version = b0 & 0x7f;
      uint8_t n;
      if (!r.check(version == FDT_TXN_V0, FDT_PF_VERSION) || !r.u8(n) || !r.check(n == sig_cnt, FDT_PF_HDR_SIG_CNT))
        break;
    } else {
      version = FDT_TXN_VLEGACY;
      if (!r.check(b0 == sig_cnt, FDT_PF_HDR_SIG_CNT)) break;
    }
    uint8_t ro_signed, ro_unsigned;
    if (!r.u8(ro_signed) || !r.check(ro_signed < sig_cnt, FDT_PF_RO_SIGNED) || !r.u8(ro_unsigned)) break;

    /* account addresses and the recent blockhash */
    uint16_t acct_cnt;
    if (!r.cu16(acct_cnt)) break;
    if (!r.check(sig_cnt <= acct_cnt && acct_cnt <= FDT_TXN_ACCT_ADDR_MAX, FDT_PF_ACCT_CNT) ||
        !r.check((uint64_t)sig_cnt + ro_unsigned <= acct_cnt, FDT_PF_ACCT_SIGNERS))
      break;
    const uint64_t acct_off = r.i;
    if (!r.skip(32ULL * acct_cnt)) break;
    const uint64_t blockhash_off = r.i;
    if (!r.skip(32)) break;

    /* instructions: each at least 3 bytes (program id, two empty lists) */
    uint16_t instr_cnt;
    if (!r.cu16(instr_cnt) || !r.check(instr_cnt <= FDT_TXN_INSTR_MAX, FDT_PF_INSTR_CNT) || !r.need(3ULL * instr_cnt) ||
        !r.check(acct_cnt > (instr_cnt ? 1 : 0), FDT_PF_NO_PROGRAM_ACCT))
      break;
    if (t) {
      t->transaction_version = version;
      t->signature_cnt = sig_cnt;
      t->signature_off = (uint16_t)sig_off;
      t->message_off = (uint16_t)msg_off;
      t->readonly_signed_cnt = ro_signed;
      t->readonly_unsigned_cnt = ro_unsigned;
      t->acct_addr_cnt = acct_cnt;
      t->acct_addr_off = (uint16_t)acct_off;
      t->recent_blockhash_off = (uint16_t)blockhash_off;
      t->instr_cnt = instr_cnt;
    }
    uint8_t max_acct = 0;
    bool ok = true;
    for (uint16_t j = 0; j < instr_cnt && ok; j++) {
      uint8_t program_id;
      uint16_t n_acct, data_sz;
      if (!r.need(3) || !r.u8(program_id) || !r.cu16(n_acct) || !r.need(n_acct)) { ok = false; break; }
      const uint64_t a_off = r.i;
      for (uint16_t k = 0; k < n_acct; k++) {
        const uint8_t x = r.at(a_off + k);
        max_acct = x > max_acct ? x : max_acct;
      }
      r.i += n_acct;
      if (!r.cu16(data_sz) || !r.need(data_sz)) { ok = false; break; }
      const uint64_t d_off = r.i;
      r.i += data_sz;
      /* the program is neither the fee payer nor outside the static keys */
      if (!r.check(program_id > 0 && program_id < acct_cnt, FDT_PF_PROGRAM_ID)) { ok = false; break; }
      if (t) {
        fdt_txn_instr_t &ins = t->instr[j];
        ins.program_id = program_id;
        ins._padding_reserved_1 = 0;
        ins.acct_cnt = n_acct;
        ins.data_sz = data_sz;
        ins.acct_off = (uint16_t)a_off;
        ins.data_off = (uint16_t)d_off;
      }
    }
    if (!ok) break;

    /* v0 address lookup tables: each >= 34 bytes (key + two lists) */
    uint16_t lut_cnt = 0;
    uint64_t adtl_w = 0, adtl = 0;
    fdt_txn_acct_addr_lut_t *luts = t ? (fdt_txn_acct_addr_lut_t *)(t->instr + instr_cnt) : nullptr;
    if (version == FDT_TXN_V0) {
      if (!r.cu16(lut_cnt) || !r.check(lut_cnt <= FDT_TXN_ADDR_TABLE_LOOKUP_MAX, FDT_PF_LUT_CNT) ||
          !r.need(34ULL * lut_cnt))
        break;
      for (uint16_t j = 0; j < lut_cnt && ok; j++) {
        uint16_t nw, nr;
        const uint64_t addr_off = r.i;
        if (!r.skip(32) || !r.cu16(nw) || !r.need(nw)) { ok = false; break; }
        const uint64_t w_off = r.i;
        r.i += nw;
        if (!r.cu16(nr) || !r.need(nr)) { ok = false; break; }
        const uint64_t ro_off = r.i;
        r.i += nr;
        if (!r.check(nw <= FDT_TXN_ACCT_ADDR_MAX - acct_cnt, FDT_PF_LUT_WRITABLE) ||
            !r.check(nr <= FDT_TXN_ACCT_ADDR_MAX - acct_cnt, FDT_PF_LUT_READONLY) ||
            !r.check(nw + nr >= 1, FDT_PF_LUT_EMPTY)) {
          ok = false;
          break;
        }
        if (luts) {
          luts[j].addr_off = (uint16_t)addr_off;
          luts[j].writable_cnt = (uint8_t)nw;
          luts[j].readonly_cnt = (uint8_t)nr;
          luts[j].writable_off = (uint16_t)w_off;
          luts[j].readonly_off = (uint16_t)ro_off;
        }
        adtl_w += nw;
        adtl += (uint64_t)nw + nr;
      }
      if (!ok) break;
    }
    if (!r.check(r.i == payload_sz, FDT_PF_TRAILING) ||
        !r.check(acct_cnt + adtl <= FDT_TXN_ACCT_ADDR_MAX, FDT_PF_TOTAL_ACCTS) ||
        !r.check(max_acct < acct_cnt + adtl, FDT_PF_ACCT_IDX))
      break;
    if (t) {
      t->addr_table_lookup_cnt = (uint8_t)lut_cnt;
      t->addr_table_adtl_writable_cnt = (uint8_t)adtl_w;
      t->addr_table_adtl_cnt = (uint8_t)adtl;
      t->_padding_reserved_1 = 0;
    }
    fp = fdt_parse_footprint(instr_cnt, lut_cnt);
  } while (0);
  if (fail) *fail = fp ? 0u : (r.fail ? r.fail : FDT_PF_SHORT);
  return fp;
}

/* The footprint fdt_parse_core would return for this payload if it parses,
   read from the counts alone (signature, account, instruction and lookup
   table counts; for v0 the instruction list is walked to reach the table
   count) with none of the structural checks: the same reads of the same
   bytes as the parser, so whenever the payload is a valid transaction the
   two agree.  0 when the walk runs past the payload or the footprint would
   exceed FDT_TXN_MAX_SZ (the parser then fails too).  *sig_cnt gets the leading signature count.  The verify tile uses it
   to reserve a frag's trailer before the GPU has parsed the frag. */
FDT_HD uint64_t fdt_peek_core(const uint8_t *payload, uint64_t payload_sz, uint64_t *sig_cnt_out) {
  fdt_reader r;
  r.p = payload; r.sz = payload_sz; r.i = 0; r.fail = 0;
  uint8_t sig_cnt = 0, b0, x;
  uint16_t acct_cnt, instr_cnt, lut_cnt = 0;
  uint64_t fp = 0;
  do {
    if (payload_sz > FDT_TXN_MTU || !r.u8(sig_cnt) || sig_cnt < 1 || sig_cnt > FDT_TXN_SIG_MAX) break;
    if (!r.skip(64ULL * sig_cnt) || !r.u8(b0)) break;
    const bool v0 = (b0 & 0x80) != 0;
    if (v0 && ((b0 & 0x7f) != FDT_TXN_V0 || !r.u8(x))) break;
    if (!r.skip(2) || !r.cu16(acct_cnt) || !r.skip(32ULL * acct_cnt + 32) || !r.cu16(instr_cnt) ||
        instr_cnt > FDT_TXN_INSTR_MAX || !r.need(3ULL * instr_cnt))
      break;
    if (v0) {
      bool ok = true;
      for (uint16_t j = 0; j < instr_cnt && ok; j++) {
        uint16_t n_acct, data_sz;
        ok = r.u8(x) && r.cu16(n_acct) && r.skip(n_acct) && r.cu16(data_sz) && r.skip(data_sz);
      }
      if (!ok || !r.cu16(lut_cnt) || lut_cnt > FDT_TXN_ADDR_TABLE_LOOKUP_MAX || !r.need(34ULL * lut_cnt)) break;
    }
    fp = fdt_parse_footprint(instr_cnt, lut_cnt);
    if (fp > FDT_TXN_MAX_SZ) fp = 0;               /* no transaction has one: the parse fails */
  } while (0);
  if (sig_cnt_out) *sig_cnt_out = sig_cnt;
  return fp;
}
