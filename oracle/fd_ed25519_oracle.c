/* fd_ed25519_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Ed25519 verify path, used as the
 * parity checker for the MI355X engine.  Nothing in firedancer_amd/
 * links, loads or calls this file: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it.
 *
 * It restates, in plain C (radix-2^51 field on unsigned __int128), the
 * observable semantics of the AVX-512 backend of the reference
 * (SURVEY.md §0, Appendix A), with a run-time switch for the portable
 * ("ref") backend's error-code mapping:
 *
 *   fd_ed25519_verify                   src/ballet/ed25519/fd_ed25519_user.c:135-230
 *   fd_ed25519_verify_batch_single_msg  src/ballet/ed25519/fd_ed25519_user.c:232-310
 *   fd_curve25519_scalar_validate       src/ballet/ed25519/fd_curve25519_scalar.h:57-73
 *   fd_curve25519_scalar_reduce         src/ballet/ed25519/fd_curve25519_scalar.c:4-110
 *   fd_r43x6_ge_decode2 (AVX-512)       src/ballet/ed25519/avx512/fd_r43x6_ge.c:163-254
 *   fd_ed25519_point_frombytes (ref)    src/ballet/ed25519/fd_curve25519.c:22-49,
 *                                       src/ballet/ed25519/ref/fd_curve25519.c:209-224
 *   fd_ed25519_affine_is_small_order    src/ballet/ed25519/fd_curve25519.h:84-114
 *   fd_ed25519_double_scalar_mul_base   src/ballet/ed25519/fd_curve25519.c:109-153
 *                                       (math only: any exact scalar mul gives the same point)
 *   fd_ed25519_point_eq_z1              src/ballet/ed25519/avx512/fd_curve25519.h:126-130
 *   fd_sha512_init/append/fini          src/ballet/sha512/fd_sha512.c:264-399
 *
 * Pinned by the reference's own golden vectors (tests/golden/, see
 * tests/test_oracle_golden.py): cctv (914), wycheproof (133),
 * malleability (196+200), txn fixtures, SHA-512 CAVP .rsp files and the
 * test_ed25519.c encodings/KATs.
 *
 * No code from the reference is copied here; constants are derived at
 * init time (d = -121665/121666, sqrt(-1) = 2^((p-1)/4), B decoded from
 * its RFC 8032 encoding, mu = floor(2^512/L) by long division).
 */
#define _GNU_SOURCE
#include "fd_ed25519_oracle.h"

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

/* ===================================================================
   SHA-512 (FIPS 180-4).  Follows fd_sha512.c:264-399: init, append of
   arbitrary byte strings, fini with 0x80 pad + 128-bit big-endian bit
   length.  Round constants generated from the prime cube roots.
   =================================================================== */

static const u64 SHA512_K[80] = {
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL,
};

static const u64 SHA512_H0[8] = {
  0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
  0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL,
};

typedef struct {
  u64     h[8];
  uint8_t buf[128];
  u64     buf_used;
  u64     bit_cnt_lo; /* total bytes hashed * 8 (low 64 bits; messages here are < 2^61 B) */
} sha512_t;

static inline u64 ror64( u64 x, int r ) { return (x>>r) | (x<<(64-r)); }

static u64 load_be64( uint8_t const * p ) {
  u64 x = 0; for( int i=0; i<8; i++ ) x = (x<<8) | p[i]; return x;
}
static void store_be64( uint8_t * p, u64 x ) {
  for( int i=7; i>=0; i-- ) { p[i] = (uint8_t)x; x >>= 8; }
}
static u64 load_le64( uint8_t const * p ) {
  u64 x = 0; for( int i=7; i>=0; i-- ) x = (x<<8) | p[i]; return x;
}
static void store_le64( uint8_t * p, u64 x ) {
  for( int i=0; i<8; i++ ) { p[i] = (uint8_t)x; x >>= 8; }
}

static void sha512_block( u64 h[8], uint8_t const * blk ) {
  u64 w[80];
  for( int t=0; t<16; t++ ) w[t] = load_be64( blk + 8*t );
  for( int t=16; t<80; t++ ) {
    u64 s0 = ror64( w[t-15], 1 ) ^ ror64( w[t-15], 8 ) ^ (w[t-15]>>7);
    u64 s1 = ror64( w[t-2], 19 ) ^ ror64( w[t-2], 61 ) ^ (w[t-2]>>6);
    w[t] = w[t-16] + s0 + w[t-7] + s1;
  }
  u64 a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
  for( int t=0; t<80; t++ ) {
    u64 S1  = ror64( e, 14 ) ^ ror64( e, 18 ) ^ ror64( e, 41 );
    u64 ch  = (e & f) ^ (~e & g);
    u64 t1  = hh + S1 + ch + SHA512_K[t] + w[t];
    u64 S0  = ror64( a, 28 ) ^ ror64( a, 34 ) ^ ror64( a, 39 );
    u64 maj = (a & b) ^ (a & c) ^ (b & c);
    u64 t2  = S0 + maj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

static void sha512_init( sha512_t * s ) {
  memcpy( s->h, SHA512_H0, sizeof(SHA512_H0) );
  s->buf_used = 0; s->bit_cnt_lo = 0;
}

static void sha512_append( sha512_t * s, uint8_t const * data, u64 sz ) {
  s->bit_cnt_lo += sz<<3;
  if( s->buf_used ) {
    u64 take = 128 - s->buf_used; if( take > sz ) take = sz;
    memcpy( s->buf + s->buf_used, data, take );
    s->buf_used += take; data += take; sz -= take;
    if( s->buf_used==128 ) { sha512_block( s->h, s->buf ); s->buf_used = 0; }
  }
  while( sz>=128 ) { sha512_block( s->h, data ); data += 128; sz -= 128; }
  if( sz ) { memcpy( s->buf, data, sz ); s->buf_used = sz; }
}

static void sha512_fini( sha512_t * s, uint8_t out[64] ) {
  u64 bits = s->bit_cnt_lo;
  uint8_t pad = 0x80;
  /* pad 0x80, zeros to 112 mod 128, then 128-bit length (high 64 bits 0) */
  s->buf[ s->buf_used++ ] = pad;
  if( s->buf_used > 112 ) {
    memset( s->buf + s->buf_used, 0, 128 - s->buf_used );
    sha512_block( s->h, s->buf ); s->buf_used = 0;
  }
  memset( s->buf + s->buf_used, 0, 112 - s->buf_used );
  store_be64( s->buf + 112, 0 );
  store_be64( s->buf + 120, bits );
  sha512_block( s->h, s->buf );
  for( int i=0; i<8; i++ ) store_be64( out + 8*i, s->h[i] );
}

void oracle_sha512( uint8_t const * data, uint64_t sz, uint8_t out[64] ) {
  sha512_t s; sha512_init( &s ); sha512_append( &s, data, sz ); sha512_fini( &s, out );
}

/* ===================================================================
   GF(2^255-19), radix 2^51, 5 limbs.  Invariant for every fe handed
   between functions: limbs < 2^52 ("weakly reduced").  Values may be
   >= p; canonical form is produced only by fe_tobytes.
   =================================================================== */

typedef struct { u64 v[5]; } fe;
#define M51 ((((u64)1)<<51)-1)

static void fe_0( fe * h ) { memset( h, 0, sizeof(*h) ); }
static void fe_1( fe * h ) { fe_0( h ); h->v[0] = 1; }

static void fe_carry( fe * h ) {
  u64 c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1]>>51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2]>>51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3]>>51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4]>>51; h->v[4] &= M51; h->v[0] += 19*c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
}

static void fe_add( fe * h, fe const * f, fe const * g ) {
  for( int i=0; i<5; i++ ) h->v[i] = f->v[i] + g->v[i];
  fe_carry( h );
}

/* h = f - g computed as f + 4p - g: g limbs < 2^52 < 4p limbs */
static void fe_sub( fe * h, fe const * f, fe const * g ) {
  static const u64 P4_0 = 4*(M51-18), P4_i = 4*M51;
  h->v[0] = f->v[0] + P4_0 - g->v[0];
  for( int i=1; i<5; i++ ) h->v[i] = f->v[i] + P4_i - g->v[i];
  fe_carry( h );
}

static void fe_neg( fe * h, fe const * f ) { fe z; fe_0( &z ); fe_sub( h, &z, f ); }

static void fe_mul( fe * h, fe const * f, fe const * g ) {
  u64 f0=f->v[0], f1=f->v[1], f2=f->v[2], f3=f->v[3], f4=f->v[4];
  u64 g0=g->v[0], g1=g->v[1], g2=g->v[2], g3=g->v[3], g4=g->v[4];
  u64 g1_19=19*g1, g2_19=19*g2, g3_19=19*g3, g4_19=19*g4;
  u128 r0 = (u128)f0*g0 + (u128)f1*g4_19 + (u128)f2*g3_19 + (u128)f3*g2_19 + (u128)f4*g1_19;
  u128 r1 = (u128)f0*g1 + (u128)f1*g0    + (u128)f2*g4_19 + (u128)f3*g3_19 + (u128)f4*g2_19;
  u128 r2 = (u128)f0*g2 + (u128)f1*g1    + (u128)f2*g0    + (u128)f3*g4_19 + (u128)f4*g3_19;
  u128 r3 = (u128)f0*g3 + (u128)f1*g2    + (u128)f2*g1    + (u128)f3*g0    + (u128)f4*g4_19;
  u128 r4 = (u128)f0*g4 + (u128)f1*g3    + (u128)f2*g2    + (u128)f3*g1    + (u128)f4*g0;
  r1 += (u64)(r0>>51); u64 h0 = (u64)r0 & M51;
  r2 += (u64)(r1>>51); u64 h1 = (u64)r1 & M51;
  r3 += (u64)(r2>>51); u64 h2 = (u64)r2 & M51;
  r4 += (u64)(r3>>51); u64 h3 = (u64)r3 & M51;
  u64 c = (u64)(r4>>51); u64 h4 = (u64)r4 & M51;
  h0 += 19*c; h1 += h0>>51; h0 &= M51;
  h->v[0]=h0; h->v[1]=h1; h->v[2]=h2; h->v[3]=h3; h->v[4]=h4;
}

static void fe_sq( fe * h, fe const * f ) { fe_mul( h, f, f ); }

static void fe_sqn( fe * h, fe const * f, int n ) {
  fe_sq( h, f ); for( int i=1; i<n; i++ ) fe_sq( h, h );
}

/* Load 255 bits (bit 255 dropped), NOT reduced mod p: matches
   fd_f25519_frombytes / decode2's mask of bit 63 of the top word
   (avx512/fd_f25519.h:100-109, avx512/fd_r43x6_ge.c:195-199). */
static void fe_frombytes( fe * h, uint8_t const s[32] ) {
  u64 w0 = load_le64( s ), w1 = load_le64( s+8 ), w2 = load_le64( s+16 ), w3 = load_le64( s+24 ) & 0x7fffffffffffffffULL;
  h->v[0] =  w0                  & M51;
  h->v[1] = ((w0>>51) | (w1<<13)) & M51;
  h->v[2] = ((w1>>38) | (w2<<26)) & M51;
  h->v[3] = ((w2>>25) | (w3<<39)) & M51;
  h->v[4] =  (w3>>12)             & M51;
}

/* Canonical little-endian encoding in [0,p): pack the exact integer
   value (< 2p after one carry pass) and subtract p if needed. */
static void fe_tobytes( uint8_t s[32], fe const * f ) {
  fe h = *f;
  fe_carry( &h );
  u64 w[5];
  u128 acc = h.v[0];
  acc += (u128)h.v[1] << 51;      w[0] = (u64)acc; acc >>= 64;
  acc += (u128)h.v[2] << 38;      w[1] = (u64)acc; acc >>= 64;
  acc += (u128)h.v[3] << 25;      w[2] = (u64)acc; acc >>= 64;
  acc += (u128)h.v[4] << 12;      w[3] = (u64)acc; acc >>= 64;
  w[4] = (u64)acc;
  static u64 const P64[5] = { 0xffffffffffffffedULL, 0xffffffffffffffffULL, 0xffffffffffffffffULL, 0x7fffffffffffffffULL, 0 };
  for( int it=0; it<2; it++ ) {
    int ge = 1;
    for( int i=4; i>=0; i-- ) { if( w[i] > P64[i] ) { ge = 1; break; } if( w[i] < P64[i] ) { ge = 0; break; } }
    if( !ge ) break;
    u64 bw = 0;
    for( int i=0; i<5; i++ ) { u128 t = (u128)w[i] - P64[i] - bw; w[i] = (u64)t; bw = (u64)(t>>64) & 1; }
  }
  for( int i=0; i<4; i++ ) store_le64( s + 8*i, w[i] );
}

static int fe_iszero( fe const * f ) {
  uint8_t s[32]; fe_tobytes( s, f );
  uint8_t acc = 0; for( int i=0; i<32; i++ ) acc |= s[i];
  return acc==0;
}
static int fe_isodd( fe const * f ) { uint8_t s[32]; fe_tobytes( s, f ); return s[0]&1; }
static int fe_eq( fe const * a, fe const * b ) { fe t; fe_sub( &t, a, b ); return fe_iszero( &t ); }

/* z^(2^252-3) and z^(p-2) by the usual 2^k-1 addition chain. */
static void fe_pow22523( fe * out, fe const * z ) {
  fe t0, t1, t2;
  fe_sq( &t0, z );              /* 2 */
  fe_sqn( &t1, &t0, 2 );        /* 8 */
  fe_mul( &t1, z, &t1 );        /* 9 */
  fe_mul( &t0, &t0, &t1 );      /* 11 */
  fe_sq( &t0, &t0 );            /* 22 */
  fe_mul( &t0, &t1, &t0 );      /* 31 = 2^5-1 */
  fe_sqn( &t1, &t0, 5 );  fe_mul( &t0, &t1, &t0 );   /* 2^10-1 */
  fe_sqn( &t1, &t0, 10 ); fe_mul( &t1, &t1, &t0 );   /* 2^20-1 */
  fe_sqn( &t2, &t1, 20 ); fe_mul( &t1, &t2, &t1 );   /* 2^40-1 */
  fe_sqn( &t1, &t1, 10 ); fe_mul( &t0, &t1, &t0 );   /* 2^50-1 */
  fe_sqn( &t1, &t0, 50 ); fe_mul( &t1, &t1, &t0 );   /* 2^100-1 */
  fe_sqn( &t2, &t1, 100 ); fe_mul( &t1, &t2, &t1 );  /* 2^200-1 */
  fe_sqn( &t1, &t1, 50 ); fe_mul( &t0, &t1, &t0 );   /* 2^250-1 */
  fe_sqn( &t0, &t0, 2 );                             /* 2^252-4 */
  fe_mul( out, &t0, z );                             /* 2^252-3 */
}

static void fe_invert( fe * out, fe const * z ) {
  fe t0, t1, t2, z11;
  fe_sq( &t0, z );
  fe_sqn( &t1, &t0, 2 );
  fe_mul( &t1, z, &t1 );        /* 9 */
  fe_mul( &z11, &t0, &t1 );     /* 11 */
  fe_sq( &t0, &z11 );           /* 22 */
  fe_mul( &t0, &t1, &t0 );      /* 31 */
  fe_sqn( &t1, &t0, 5 );  fe_mul( &t0, &t1, &t0 );
  fe_sqn( &t1, &t0, 10 ); fe_mul( &t1, &t1, &t0 );
  fe_sqn( &t2, &t1, 20 ); fe_mul( &t1, &t2, &t1 );
  fe_sqn( &t1, &t1, 10 ); fe_mul( &t0, &t1, &t0 );
  fe_sqn( &t1, &t0, 50 ); fe_mul( &t1, &t1, &t0 );
  fe_sqn( &t2, &t1, 100 ); fe_mul( &t1, &t2, &t1 );
  fe_sqn( &t1, &t1, 50 ); fe_mul( &t0, &t1, &t0 );   /* 2^250-1 */
  fe_sqn( &t0, &t0, 5 );                             /* 2^255-32 */
  fe_mul( out, &t0, &z11 );                          /* 2^255-21 = p-2 */
}

static void fe_small( fe * h, u64 x ) { fe_0( h ); h->v[0] = x; }

/* ===================================================================
   Curve constants (derived, not transcribed)
   =================================================================== */

typedef struct { fe X, Y, Z, T; } ge_p3;      /* extended: x=X/Z, y=Y/Z, xy=T/Z */
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe X, Y, Z, T; } ge_p1p1;    /* completed: x=X/Z, y=Y/T */
typedef struct { fe ypx, ymx, xy2d; } ge_niels;            /* affine, Z=1 */
typedef struct { fe YpX, YmX, Z, T2d; } ge_cached;

static fe       C_D, C_D2, C_SQRTM1;
static ge_p3    C_B;
static u64      C_MU[5];             /* floor(2^512 / L), 5 limbs */
#define BTAB_W 8
static ge_niels C_BTAB[1<<(BTAB_W-2)]; /* odd multiples B,3B,..,127B */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static u64 const L64[4] = { 0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL };

/* ===================================================================
   Group law on -x^2+y^2 = 1 + d x^2 y^2 (a = -1), extended coordinates
   (Hisil-Wong-Carter-Dawson 2008).  Complete for Ed25519.
   =================================================================== */

static void ge_p3_0( ge_p3 * h ) { fe_0( &h->X ); fe_1( &h->Y ); fe_1( &h->Z ); fe_0( &h->T ); }

static void p1p1_to_p2( ge_p2 * r, ge_p1p1 const * p ) {
  fe_mul( &r->X, &p->X, &p->T ); fe_mul( &r->Y, &p->Y, &p->Z ); fe_mul( &r->Z, &p->Z, &p->T );
}
static void p1p1_to_p3( ge_p3 * r, ge_p1p1 const * p ) {
  fe_mul( &r->X, &p->X, &p->T ); fe_mul( &r->Y, &p->Y, &p->Z );
  fe_mul( &r->Z, &p->Z, &p->T ); fe_mul( &r->T, &p->X, &p->Y );
}
static void p3_to_p2( ge_p2 * r, ge_p3 const * p ) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }

static void p2_dbl( ge_p1p1 * r, ge_p2 const * p ) {
  fe XX, YY, B, A, AA;
  fe_sq( &XX, &p->X ); fe_sq( &YY, &p->Y ); fe_sq( &B, &p->Z ); fe_add( &B, &B, &B );
  fe_add( &A, &p->X, &p->Y ); fe_sq( &AA, &A );
  fe_add( &r->Y, &YY, &XX );
  fe_sub( &r->Z, &YY, &XX );
  fe_sub( &r->X, &AA, &r->Y );
  fe_sub( &r->T, &B, &r->Z );
}
static void p3_dbl( ge_p1p1 * r, ge_p3 const * p ) { ge_p2 q; p3_to_p2( &q, p ); p2_dbl( r, &q ); }

static void p3_to_cached( ge_cached * r, ge_p3 const * p ) {
  fe_add( &r->YpX, &p->Y, &p->X ); fe_sub( &r->YmX, &p->Y, &p->X );
  r->Z = p->Z; fe_mul( &r->T2d, &p->T, &C_D2 );
}

static void ge_add_cached( ge_p1p1 * r, ge_p3 const * p, ge_cached const * q, int sub ) {
  fe A, B, C, D, t;
  fe_add( &t, &p->Y, &p->X ); fe_mul( &A, &t, sub ? &q->YmX : &q->YpX );
  fe_sub( &t, &p->Y, &p->X ); fe_mul( &B, &t, sub ? &q->YpX : &q->YmX );
  fe_mul( &C, &q->T2d, &p->T );
  fe_mul( &D, &p->Z, &q->Z ); fe_add( &D, &D, &D );
  fe_sub( &r->X, &A, &B ); fe_add( &r->Y, &A, &B );
  if( sub ) { fe_sub( &r->Z, &D, &C ); fe_add( &r->T, &D, &C ); }
  else      { fe_add( &r->Z, &D, &C ); fe_sub( &r->T, &D, &C ); }
}

static void ge_add_niels( ge_p1p1 * r, ge_p3 const * p, ge_niels const * q, int sub ) {
  fe A, B, C, D, t;
  fe_add( &t, &p->Y, &p->X ); fe_mul( &A, &t, sub ? &q->ymx : &q->ypx );
  fe_sub( &t, &p->Y, &p->X ); fe_mul( &B, &t, sub ? &q->ypx : &q->ymx );
  fe_mul( &C, &q->xy2d, &p->T );
  fe_add( &D, &p->Z, &p->Z );
  fe_sub( &r->X, &A, &B ); fe_add( &r->Y, &A, &B );
  if( sub ) { fe_sub( &r->Z, &D, &C ); fe_add( &r->T, &D, &C ); }
  else      { fe_add( &r->Z, &D, &C ); fe_sub( &r->T, &D, &C ); }
}

static void p3_add( ge_p3 * r, ge_p3 const * p, ge_p3 const * q ) {
  ge_cached c; ge_p1p1 t; p3_to_cached( &c, q ); ge_add_cached( &t, p, &c, 0 ); p1p1_to_p3( r, &t );
}

static void p3_to_niels( ge_niels * r, ge_p3 const * p ) {
  fe zi, x, y;
  fe_invert( &zi, &p->Z ); fe_mul( &x, &p->X, &zi ); fe_mul( &y, &p->Y, &zi );
  fe_add( &r->ypx, &y, &x ); fe_sub( &r->ymx, &y, &x );
  fe_mul( &r->xy2d, &x, &y ); fe_mul( &r->xy2d, &r->xy2d, &C_D2 );
}

static void p3_tobytes( uint8_t s[32], ge_p3 const * p ) {
  fe zi, x, y;
  fe_invert( &zi, &p->Z ); fe_mul( &x, &p->X, &zi ); fe_mul( &y, &p->Y, &zi );
  fe_tobytes( s, &y ); s[31] ^= (uint8_t)(fe_isodd( &x ) << 7);
}

/* Projective equality X1 Z2 == X2 Z1 and Y1 Z2 == Y2 Z1, with full
   reduction (fd_r43x6_ge_is_eq, avx512/fd_r43x6_ge.h:52-82). */
static int p3_eq( ge_p3 const * a, ge_p3 const * b ) {
  fe l, r;
  fe_mul( &l, &a->X, &b->Z ); fe_mul( &r, &b->X, &a->Z ); if( !fe_eq( &l, &r ) ) return 0;
  fe_mul( &l, &a->Y, &b->Z ); fe_mul( &r, &b->Y, &a->Z ); if( !fe_eq( &l, &r ) ) return 0;
  return 1;
}

/* ===================================================================
   Point decoding.
   mapping==ORACLE_MAP_AVX512: fd_r43x6_ge_decode (avx512/fd_r43x6_ge.c:
     163-254): y = enc & (2^255-1) used mod p (non-canonical accepted);
     u = y^2-1, v = d y^2+1, x = u v^3 (u v^7)^((p-5)/8); fail if
     v x^2 != +-u; x *= sqrt(-1) if v x^2 == -u; FAIL if x == 0 and
     sign == 1; negate x if parity != sign.
   mapping==ORACLE_MAP_REF: fd_ed25519_point_frombytes (fd_curve25519.c:
     22-49): same, but x == 0 with sign == 1 is accepted (x = -0 = 0).
   Returns 0 on success, -1 on failure.
   =================================================================== */

static int ge_decode( ge_p3 * P, uint8_t const s[32], int mapping ) {
  fe y, ysq, u, v, v2, v3, v4, uv3, uv7, t0, x, x2, vx2, t1, t2, one;
  int sign = s[31]>>7;
  fe_1( &one );
  fe_frombytes( &y, s );
  fe_sq( &ysq, &y );
  fe_sub( &u, &ysq, &one );
  fe_mul( &v, &C_D, &ysq ); fe_add( &v, &v, &one );
  fe_sq( &v2, &v ); fe_sq( &v4, &v2 ); fe_mul( &v3, &v, &v2 );
  fe_mul( &uv3, &u, &v3 ); fe_mul( &uv7, &uv3, &v4 );
  fe_pow22523( &t0, &uv7 );
  fe_mul( &x, &uv3, &t0 );
  fe_sq( &x2, &x ); fe_mul( &vx2, &v, &x2 );
  fe_sub( &t1, &vx2, &u ); fe_add( &t2, &vx2, &u );
  int t1nz = !fe_iszero( &t1 ), t2nz = !fe_iszero( &t2 );
  if( t1nz && t2nz ) return -1;
  if( t1nz ) fe_mul( &x, &x, &C_SQRTM1 );
  int xz = fe_iszero( &x );
  if( mapping==ORACLE_MAP_AVX512 && xz && sign ) return -1;
  if( fe_isodd( &x ) != sign ) fe_neg( &x, &x );
  P->X = x; P->Y = y; fe_1( &P->Z ); fe_mul( &P->T, &x, &y );
  return 0;
}

/* [8]P == O  <=>  x==0 or y==0 or y==y0 or y==y1 (fd_curve25519.h:
   84-114).  Evaluated exactly mod p on an affine (Z=1) decoded point.
   The order-8 y values are derived from C_SQRTM1 at init. */
static fe C_Y0, C_Y1;

static int ge_is_small_order_affine( ge_p3 const * P ) {
  return fe_iszero( &P->X ) | fe_iszero( &P->Y ) | fe_eq( &P->Y, &C_Y0 ) | fe_eq( &P->Y, &C_Y1 );
}

/* ===================================================================
   Scalars mod L
   =================================================================== */

static int sc_lt_L( u64 const s[4] ) {   /* s < L */
  for( int i=3; i>=0; i-- ) { if( s[i] < L64[i] ) return 1; if( s[i] > L64[i] ) return 0; }
  return 0;
}

/* fd_curve25519_scalar_validate: S <= L-1 (fd_curve25519_scalar.h:57-73) */
int oracle_scalar_validate( uint8_t const s[32] ) {
  u64 w[4] = { load_le64( s ), load_le64( s+8 ), load_le64( s+16 ), load_le64( s+24 ) };
  return sc_lt_L( w );
}

/* Barrett reduction, HAC 14.42 with b = 2^64, k = 4, mu = floor(b^8/L). */
static void sc_reduce512( u64 out[4], u64 const x[8] ) {
  /* q1 = x >> 192 (5 limbs); q2 = q1*mu (10 limbs); q3 = q2 >> 320 (5 limbs) */
  u64 q1[5] = { x[3], x[4], x[5], x[6], x[7] };
  u64 q2[10] = {0};
  for( int i=0; i<5; i++ ) {
    u64 c = 0;
    for( int j=0; j<5; j++ ) {
      u128 t = (u128)q1[i]*C_MU[j] + q2[i+j] + c;
      q2[i+j] = (u64)t; c = (u64)(t>>64);
    }
    q2[i+5] = c;
  }
  u64 q3[5] = { q2[5], q2[6], q2[7], q2[8], q2[9] };
  /* r2 = (q3*L) mod b^5 */
  u64 r2[5] = {0};
  for( int i=0; i<5; i++ ) {
    u64 c = 0;
    for( int j=0; j<4 && i+j<5; j++ ) {
      u128 t = (u128)q3[i]*L64[j] + r2[i+j] + c;
      r2[i+j] = (u64)t; c = (u64)(t>>64);
    }
    if( i+4<5 ) r2[i+4] += c;
  }
  /* r = (x mod b^5) - r2 mod b^5 */
  u64 r[5]; u64 bw = 0;
  for( int i=0; i<5; i++ ) {
    u128 t = (u128)x[i] - r2[i] - bw;
    r[i] = (u64)t; bw = (u64)(t>>64) & 1;
  }
  /* while r >= L: r -= L (at most twice) */
  for( int it=0; it<3; it++ ) {
    int ge = 0;
    if( r[4] ) ge = 1;
    else { ge = 1; for( int i=3; i>=0; i-- ) { if( r[i] > L64[i] ) { ge = 1; break; } if( r[i] < L64[i] ) { ge = 0; break; } } }
    if( !ge ) break;
    u64 b2 = 0;
    for( int i=0; i<5; i++ ) {
      u128 t = (u128)r[i] - (i<4 ? L64[i] : 0) - b2;
      r[i] = (u64)t; b2 = (u64)(t>>64) & 1;
    }
  }
  out[0]=r[0]; out[1]=r[1]; out[2]=r[2]; out[3]=r[3];
}

void oracle_scalar_reduce( uint8_t out[32], uint8_t const in[64] ) {
  oracle_init();
  u64 x[8]; for( int i=0; i<8; i++ ) x[i] = load_le64( in + 8*i );
  u64 r[4]; sc_reduce512( r, x );
  for( int i=0; i<4; i++ ) store_le64( out + 8*i, r[i] );
}

/* s = (a*b + c) mod L, for the test-only signer. */
static void sc_muladd( uint8_t s[32], uint8_t const a[32], uint8_t const b[32], uint8_t const c[32] ) {
  u64 A[4], B[4], x[8] = {0};
  for( int i=0; i<4; i++ ) { A[i] = load_le64( a+8*i ); B[i] = load_le64( b+8*i ); }
  for( int i=0; i<4; i++ ) {
    u64 cy = 0;
    for( int j=0; j<4; j++ ) { u128 t = (u128)A[i]*B[j] + x[i+j] + cy; x[i+j] = (u64)t; cy = (u64)(t>>64); }
    x[i+4] = cy;
  }
  u64 cy = 0;
  for( int i=0; i<8; i++ ) {
    u128 t = (u128)x[i] + (i<4 ? load_le64( c+8*i ) : 0) + cy; x[i] = (u64)t; cy = (u64)(t>>64);
  }
  u64 r[4]; sc_reduce512( r, x );
  for( int i=0; i<4; i++ ) store_le64( s+8*i, r[i] );
}

/* Signed sliding-window (wNAF) recoding, digits odd in (-2^(w-1),2^(w-1)). */
static void sc_wnaf( int8_t naf[257], uint8_t const s[32], int w ) {
  u64 k[5] = { load_le64( s ), load_le64( s+8 ), load_le64( s+16 ), load_le64( s+24 ), 0 };
  memset( naf, 0, 257 );
  int carry = 0, bit = 0;
  while( bit < 257 ) {
    int b = (int)((k[bit>>6] >> (bit&63)) & 1);
    if( b==carry ) { bit++; continue; }
    int now = w; if( now > 257-bit ) now = 257-bit;
    /* extract `now` bits at position bit */
    u64 lo = k[bit>>6] >> (bit&63);
    if( (bit&63) && (bit>>6)+1 < 5 ) lo |= k[(bit>>6)+1] << (64-(bit&63));
    int word = (int)(lo & ((1ULL<<now)-1)) + carry;
    carry = (word >> (w-1)) & 1;
    word -= carry << w;
    naf[bit] = (int8_t)word;
    bit += now;
  }
}

/* ===================================================================
   Init
   =================================================================== */

static void init_once( void ) {
  fe t, one; fe_1( &one );
  /* d = -121665/121666 */
  fe n, dd; fe_small( &n, 121665 ); fe_neg( &n, &n ); fe_small( &dd, 121666 ); fe_invert( &dd, &dd );
  fe_mul( &C_D, &n, &dd ); fe_add( &C_D2, &C_D, &C_D );
  /* sqrt(-1) = 2^((p-1)/4); (p-1)/4 = 2^253-5 = 2*(2^252-3)+1 -> (2^(2^252-3))^2 * 2 */
  fe two; fe_small( &two, 2 );
  fe_pow22523( &t, &two ); fe_sq( &t, &t ); fe_mul( &C_SQRTM1, &t, &two );
  /* B: y = 4/5, x even ("positive") */
  uint8_t benc[32]; memset( benc, 0x66, 32 ); benc[0] = 0x58;
  ge_decode( &C_B, benc, ORACLE_MAP_AVX512 );
  /* Order-8 points Q: 2Q = (+-sqrt(-1), 0), i.e. y(2Q) = (y^2+x^2)/(1-dx^2y^2) = 0
     => x^2 = -y^2; on -x^2+y^2 = 1+dx^2y^2 this gives d y^4 + 2 y^2 - 1 = 0,
     y^2 = (-1 +- sqrt(1+d))/d.  Exactly one root is a square (their
     product -1/d is not); y0 = sqrt(root), y1 = -y0. */
  {
    fe dp1, s, r, y, chk, nd;
    fe_add( &dp1, &C_D, &one );
    /* sqrt via candidate x = a^((p+3)/8) = a * a^((p-5)/8)... use
       sqrt(a) = a^((p+3)/8): candidate c = a * (a^((p-5)/8)) * ... */
    fe_pow22523( &t, &dp1 ); fe_mul( &s, &dp1, &t );           /* s^2 = +-(1+d) */
    fe_sq( &chk, &s ); if( !fe_eq( &chk, &dp1 ) ) fe_mul( &s, &s, &C_SQRTM1 );
    fe_invert( &nd, &C_D );
    for( int sg=0; sg<2; sg++ ) {
      fe num; fe m1; fe_neg( &m1, &one );
      if( sg ) { fe_neg( &num, &s ); fe_add( &num, &num, &m1 ); } else fe_add( &num, &m1, &s );
      fe_mul( &r, &num, &nd );                                   /* candidate y^2 */
      fe_pow22523( &t, &r ); fe_mul( &y, &r, &t );
      fe_sq( &chk, &y );
      if( !fe_eq( &chk, &r ) ) { fe_mul( &y, &y, &C_SQRTM1 ); fe_sq( &chk, &y ); }
      if( fe_eq( &chk, &r ) ) { C_Y0 = y; fe_neg( &C_Y1, &y ); break; }
    }
  }
  /* mu = floor(2^512 / L) by bit-serial long division */
  {
    u64 rem[5] = {0}, q[9] = {0};
    for( int bit=512; bit>=0; bit-- ) {
      /* rem = 2*rem + (bit==512) */
      for( int i=4; i>0; i-- ) rem[i] = (rem[i]<<1) | (rem[i-1]>>63);
      rem[0] = (rem[0]<<1) | (u64)(bit==512);
      int ge = rem[4] ? 1 : 0;
      if( !rem[4] ) { ge = 1; for( int i=3; i>=0; i-- ) { if( rem[i] > L64[i] ) { ge=1; break; } if( rem[i] < L64[i] ) { ge=0; break; } } }
      if( ge ) {
        u64 bw = 0;
        for( int i=0; i<5; i++ ) { u128 tt = (u128)rem[i] - (i<4?L64[i]:0) - bw; rem[i] = (u64)tt; bw = (u64)(tt>>64)&1; }
        q[bit>>6] |= 1ULL << (bit&63);
      }
    }
    for( int i=0; i<5; i++ ) C_MU[i] = q[i];
  }
  /* odd multiples of B for the w=8 wNAF */
  {
    ge_p3 Bi = C_B, B2; ge_p1p1 t2;
    p3_dbl( &t2, &C_B ); p1p1_to_p3( &B2, &t2 );
    for( int i=0; i<(1<<(BTAB_W-2)); i++ ) {
      p3_to_niels( &C_BTAB[i], &Bi );
      p3_add( &Bi, &Bi, &B2 );
    }
  }
}

void oracle_init( void ) { pthread_once( &g_once, init_once ); }

/* ===================================================================
   [k]A + [s]B with A in extended coords (any exact algorithm yields the
   same point; the reference uses wNAF-4 on k and wNAF-8 on s,
   fd_curve25519.c:109-153).
   =================================================================== */

static void ge_double_scalar_mul_base( ge_p3 * r, uint8_t const k[32], ge_p3 const * A, uint8_t const s[32] ) {
  int8_t kn[257], sn[257];
  sc_wnaf( kn, k, 5 );
  sc_wnaf( sn, s, BTAB_W );
  ge_cached Ai[8];                     /* A,3A,..,15A */
  ge_p3 A2, t3; ge_p1p1 t;
  p3_dbl( &t, A ); p1p1_to_p3( &A2, &t );
  p3_to_cached( &Ai[0], A );
  t3 = *A;
  for( int i=1; i<8; i++ ) { p3_add( &t3, &t3, &A2 ); p3_to_cached( &Ai[i], &t3 ); }

  int i;
  for( i=256; i>=0; i-- ) if( kn[i] || sn[i] ) break;
  ge_p3_0( r );
  if( i<0 ) return;                    /* k == s == 0: identity */
  ge_p2 r2; p3_to_p2( &r2, r );
  for( ; i>=0; i-- ) {
    p2_dbl( &t, &r2 );                 /* t = 2r */
    if( kn[i] ) { p1p1_to_p3( r, &t ); ge_add_cached( &t, r, &Ai[ (kn[i]>0 ? kn[i] : -kn[i])/2 ], kn[i]<0 ); }
    if( sn[i] ) { p1p1_to_p3( r, &t ); ge_add_niels ( &t, r, &C_BTAB[ (sn[i]>0 ? sn[i] : -sn[i])/2 ], sn[i]<0 ); }
    p1p1_to_p2( &r2, &t );
  }
  p1p1_to_p3( r, &t );
}

static void ge_scalarmult_base( ge_p3 * r, uint8_t const s[32] ) {
  uint8_t zero[32] = {0};
  ge_p3 O; ge_p3_0( &O );
  ge_double_scalar_mul_base( r, zero, &O, s );
}

/* ===================================================================
   Verify (fd_ed25519_user.c:135-310)
   =================================================================== */

/* Pass 1 for one signature: checks 1-5 of SURVEY Appendix A.
   Returns the error code (0 if all pass) and fills A' (negated), R, k. */
static int verify_pass1( uint8_t const * msg, u64 msg_sz, uint8_t const sig[64], uint8_t const pub[32],
                         int mapping, ge_p3 * Aneg, ge_p3 * R, uint8_t k[32] ) {
  uint8_t const * r = sig;
  uint8_t const * S = sig + 32;
  if( !oracle_scalar_validate( S ) ) return ORACLE_ERR_SIG;                 /* user.c:159-161 */
  ge_p3 A;
  if( ge_decode( &A, pub, mapping ) ) {                                      /* decode2 A first */
    return mapping==ORACLE_MAP_AVX512 ? ORACLE_ERR_SIG : ORACLE_ERR_PUBKEY;  /* user.c:191-193 */
  }
  if( ge_decode( R, r, mapping ) ) return ORACLE_ERR_SIG;
  if( ge_is_small_order_affine( &A ) ) return ORACLE_ERR_PUBKEY;            /* user.c:194-196 */
  if( ge_is_small_order_affine( R ) ) return ORACLE_ERR_SIG;                /* user.c:197-199 */
  uint8_t h[64];
  sha512_t sh; sha512_init( &sh );
  sha512_append( &sh, r, 32 ); sha512_append( &sh, pub, 32 );
  if( msg_sz ) sha512_append( &sh, msg, msg_sz );
  sha512_fini( &sh, h );
  oracle_scalar_reduce( k, h );
  /* A' := -A (fd_ed25519_point_neg) */
  fe_neg( &Aneg->X, &A.X ); Aneg->Y = A.Y; Aneg->Z = A.Z; fe_neg( &Aneg->T, &A.T );
  return 0;
}

static int verify_pass2( uint8_t const S[32], ge_p3 const * Aneg, ge_p3 const * R, uint8_t const k[32] ) {
  ge_p3 Rcmp;
  ge_double_scalar_mul_base( &Rcmp, k, Aneg, S );
  return p3_eq( &Rcmp, R ) ? ORACLE_SUCCESS : ORACLE_ERR_MSG;
}

int oracle_verify( uint8_t const * msg, uint64_t msg_sz, uint8_t const sig[64], uint8_t const pub[32], int mapping ) {
  oracle_init();
  ge_p3 Aneg, R; uint8_t k[32];
  int rc = verify_pass1( msg, msg_sz, sig, pub, mapping, &Aneg, &R, k );
  if( rc ) return rc;
  return verify_pass2( sig+32, &Aneg, &R, k );
}

int oracle_verify_batch_single_msg( uint8_t const * msg, uint64_t msg_sz, uint8_t const * sigs,
                                    uint8_t const * pubs, uint32_t batch_sz, int mapping ) {
  oracle_init();
  if( batch_sz==0 || batch_sz>16 ) return ORACLE_ERR_SIG;                   /* user.c:238-241 */
  ge_p3 Aneg[16], R[16]; uint8_t k[16][32];
  for( uint32_t j=0; j<batch_sz; j++ ) {
    int rc = verify_pass1( msg, msg_sz, sigs+64*j, pubs+32*j, mapping, &Aneg[j], &R[j], k[j] );
    if( rc ) return rc;
  }
  for( uint32_t j=0; j<batch_sz; j++ ) {
    if( verify_pass2( sigs+64*j+32, &Aneg[j], &R[j], k[j] ) ) return ORACLE_ERR_MSG;
  }
  return ORACLE_SUCCESS;
}

/* Per-signature detail for debugging parity mismatches: pass-1 code and
   the equation bit (eq is -1 when pass 1 failed and the equation was not
   evaluated). */
void oracle_verify_detail( uint8_t const * msg, uint64_t msg_sz, uint8_t const sig[64], uint8_t const pub[32],
                           int mapping, int * pass1_code, int * eq, uint8_t k_out[32] ) {
  oracle_init();
  ge_p3 Aneg, R; uint8_t k[32] = {0};
  *pass1_code = verify_pass1( msg, msg_sz, sig, pub, mapping, &Aneg, &R, k );
  *eq = -1;
  if( !*pass1_code ) *eq = verify_pass2( sig+32, &Aneg, &R, k )==ORACLE_SUCCESS;
  if( k_out ) memcpy( k_out, k, 32 );
}

/* Point decode + small-order probe for unit tests: returns decode code
   (0/-1) and sets *small_order. */
int oracle_point_decode( uint8_t const enc[32], int mapping, int * small_order, uint8_t xy_out[64] ) {
  oracle_init();
  ge_p3 P;
  int rc = ge_decode( &P, enc, mapping );
  *small_order = rc ? -1 : ge_is_small_order_affine( &P );
  if( xy_out && !rc ) { fe_tobytes( xy_out, &P.X ); fe_tobytes( xy_out+32, &P.Y ); }
  return rc;
}

/* ===================================================================
   Bulk verification of transactions (batch_single_msg semantics per
   txn) over a flat arena, multi-threaded.  Used by tests to produce the
   expected codes for large synthetic sets and by bench.py's
   cpu_baseline leg.
   =================================================================== */

typedef struct {
  uint8_t const *              arena;
  oracle_txn_t const *         txns;
  uint64_t                     n;
  int8_t *                     codes;
  int                          mapping;
  int                          nthreads;
  int                          tid;
  int                          cpu;      /* pin to this CPU (-1: no pinning) */
} bulk_arg_t;

static void * bulk_worker( void * _a ) {
  bulk_arg_t * a = (bulk_arg_t *)_a;
  if( a->cpu >= 0 ) {
    cpu_set_t set; CPU_ZERO( &set ); CPU_SET( a->cpu, &set );
    (void)pthread_setaffinity_np( pthread_self(), sizeof(set), &set );
  }
  uint64_t lo = a->n * (uint64_t)a->tid / (uint64_t)a->nthreads;
  uint64_t hi = a->n * (uint64_t)(a->tid+1) / (uint64_t)a->nthreads;
  for( uint64_t i=lo; i<hi; i++ ) {
    oracle_txn_t const * t = &a->txns[i];
    a->codes[i] = (int8_t)oracle_verify_batch_single_msg( a->arena + t->msg_off, t->msg_sz,
                                                          a->arena + t->sig_off, a->arena + t->pub_off,
                                                          t->sig_cnt, a->mapping );
  }
  return NULL;
}

/* cpus: NULL, or nthreads CPU ids -- worker t is pinned to cpus[t] (the
   CPU baseline: one pinned thread per physical core, static partition) */
void oracle_verify_txns_pinned( uint8_t const * arena, oracle_txn_t const * txns, uint64_t n,
                                int8_t * codes, int mapping, int nthreads, int const * cpus ) {
  oracle_init();
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 256 ) nthreads = 256;
  pthread_t th[256]; bulk_arg_t args[256];
  for( int t=0; t<nthreads; t++ ) {
    args[t] = (bulk_arg_t){ arena, txns, n, codes, mapping, nthreads, t, cpus ? cpus[t] : -1 };
    if( nthreads==1 && !cpus ) { bulk_worker( &args[t] ); return; }
    pthread_create( &th[t], NULL, bulk_worker, &args[t] );
  }
  for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
}

void oracle_verify_txns( uint8_t const * arena, oracle_txn_t const * txns, uint64_t n,
                         int8_t * codes, int mapping, int nthreads ) {
  oracle_verify_txns_pinned( arena, txns, n, codes, mapping, nthreads, NULL );
}

/* ===================================================================
   RFC 8032 keygen / sign -- test-only fixture generator (SURVEY §2.3:
   "the build needs an RFC 8032 signer CPU-side for fixtures only").
   =================================================================== */

void oracle_public_from_private( uint8_t pub[32], uint8_t const prv[32] ) {
  oracle_init();
  uint8_t h[64]; oracle_sha512( prv, 32, h );
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  /* a may exceed L; [a]B == [a mod L]B */
  uint8_t wide[64] = {0}, a[32]; memcpy( wide, h, 32 ); oracle_scalar_reduce( a, wide );
  ge_p3 A; ge_scalarmult_base( &A, a );
  p3_tobytes( pub, &A );
}

void oracle_sign( uint8_t sig[64], uint8_t const * msg, uint64_t sz, uint8_t const pub[32], uint8_t const prv[32] ) {
  oracle_init();
  uint8_t h[64]; oracle_sha512( prv, 32, h );
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  uint8_t rh[64], r[32];
  sha512_t s; sha512_init( &s ); sha512_append( &s, h+32, 32 ); if( sz ) sha512_append( &s, msg, sz ); sha512_fini( &s, rh );
  oracle_scalar_reduce( r, rh );
  ge_p3 R; ge_scalarmult_base( &R, r ); p3_tobytes( sig, &R );
  uint8_t kh[64], k[32];
  sha512_init( &s ); sha512_append( &s, sig, 32 ); sha512_append( &s, pub, 32 ); if( sz ) sha512_append( &s, msg, sz ); sha512_fini( &s, kh );
  oracle_scalar_reduce( k, kh );
  sc_muladd( sig+32, k, h, r );   /* S = k*a + r mod L */
}
