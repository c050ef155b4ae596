// ILP microbenchmark for the radix-2^25.5 field product on gfx950: does a
// wave with ONE feed-forward product chain (fdgpu_fe.h: every v_mad_u64_u32
// of a product depends on the previous one) leave the VALU idle at the
// verify kernel's occupancy (2 waves per SIMD), and do TWO independent
// products interleaved mad by mad (madc2 below) recover it?
//
//   V0 x = x*y            one chain (fe_mul)
//   V1 x = x^2            one chain (fe_sq)
//   V2 two chains x1*y, x2*y, sequential fe_mul calls (scheduling fence each)
//   V3 two chains, fe_mul_x2 (interleaved)
//   V4 two squaring chains, sequential
//   V5 two squaring chains, fe_sq_x2 (interleaved)
// at 1, 2 and 4 waves per SIMD (grid = CUs x waves blocks of 256 threads).
// Results are canonicalised and compared between the sequential and the
// interleaved forms.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_ilp.hip -o tools/ubench_ilp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../firedancer_amd/csrc/fdgpu_fe.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace fdgpu;

/* madc2<N>::run(sa, sb, a, b, c, d): two independent column chains in one
   asm block, interleaved mad by mad (sa += a.b, sb += c.d): a wave with
   two products in flight issues the second chain's mad while the first's
   is still in the pipeline. */
template <int N> struct madc2;
template <> struct madc2<1> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]));
    (void)cc;
  }
};
template <> struct madc2<2> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]));
    (void)cc;
  }
};
template <> struct madc2<3> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]));
    (void)cc;
  }
};
template <> struct madc2<4> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]));
    (void)cc;
  }
};
template <> struct madc2<5> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        "v_mad_u64_u32 %0, %2, %19, %20, %0\n"
        "v_mad_u64_u32 %1, %2, %21, %22, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]), "v"(a[4]), "v"(b[4]), "v"(c[4]), "v"(d[4]));
    (void)cc;
  }
};
template <> struct madc2<6> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        "v_mad_u64_u32 %0, %2, %19, %20, %0\n"
        "v_mad_u64_u32 %1, %2, %21, %22, %1\n"
        "v_mad_u64_u32 %0, %2, %23, %24, %0\n"
        "v_mad_u64_u32 %1, %2, %25, %26, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]), "v"(a[4]), "v"(b[4]), "v"(c[4]), "v"(d[4]), "v"(a[5]), "v"(b[5]), "v"(c[5]), "v"(d[5]));
    (void)cc;
  }
};
template <> struct madc2<7> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        "v_mad_u64_u32 %0, %2, %19, %20, %0\n"
        "v_mad_u64_u32 %1, %2, %21, %22, %1\n"
        "v_mad_u64_u32 %0, %2, %23, %24, %0\n"
        "v_mad_u64_u32 %1, %2, %25, %26, %1\n"
        "v_mad_u64_u32 %0, %2, %27, %28, %0\n"
        "v_mad_u64_u32 %1, %2, %29, %30, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]), "v"(a[4]), "v"(b[4]), "v"(c[4]), "v"(d[4]), "v"(a[5]), "v"(b[5]), "v"(c[5]), "v"(d[5]), "v"(a[6]), "v"(b[6]), "v"(c[6]), "v"(d[6]));
    (void)cc;
  }
};
template <> struct madc2<8> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        "v_mad_u64_u32 %0, %2, %19, %20, %0\n"
        "v_mad_u64_u32 %1, %2, %21, %22, %1\n"
        "v_mad_u64_u32 %0, %2, %23, %24, %0\n"
        "v_mad_u64_u32 %1, %2, %25, %26, %1\n"
        "v_mad_u64_u32 %0, %2, %27, %28, %0\n"
        "v_mad_u64_u32 %1, %2, %29, %30, %1\n"
        "v_mad_u64_u32 %0, %2, %31, %32, %0\n"
        "v_mad_u64_u32 %1, %2, %33, %34, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]), "v"(a[4]), "v"(b[4]), "v"(c[4]), "v"(d[4]), "v"(a[5]), "v"(b[5]), "v"(c[5]), "v"(d[5]), "v"(a[6]), "v"(b[6]), "v"(c[6]), "v"(d[6]), "v"(a[7]), "v"(b[7]), "v"(c[7]), "v"(d[7]));
    (void)cc;
  }
};
template <> struct madc2<9> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        "v_mad_u64_u32 %0, %2, %19, %20, %0\n"
        "v_mad_u64_u32 %1, %2, %21, %22, %1\n"
        "v_mad_u64_u32 %0, %2, %23, %24, %0\n"
        "v_mad_u64_u32 %1, %2, %25, %26, %1\n"
        "v_mad_u64_u32 %0, %2, %27, %28, %0\n"
        "v_mad_u64_u32 %1, %2, %29, %30, %1\n"
        "v_mad_u64_u32 %0, %2, %31, %32, %0\n"
        "v_mad_u64_u32 %1, %2, %33, %34, %1\n"
        "v_mad_u64_u32 %0, %2, %35, %36, %0\n"
        "v_mad_u64_u32 %1, %2, %37, %38, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]), "v"(a[4]), "v"(b[4]), "v"(c[4]), "v"(d[4]), "v"(a[5]), "v"(b[5]), "v"(c[5]), "v"(d[5]), "v"(a[6]), "v"(b[6]), "v"(c[6]), "v"(d[6]), "v"(a[7]), "v"(b[7]), "v"(c[7]), "v"(d[7]), "v"(a[8]), "v"(b[8]), "v"(c[8]), "v"(d[8]));
    (void)cc;
  }
};
template <> struct madc2<10> {
  static FDG_DEV void run(uint64_t &sa, uint64_t &sb, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n"
        "v_mad_u64_u32 %1, %2, %5, %6, %1\n"
        "v_mad_u64_u32 %0, %2, %7, %8, %0\n"
        "v_mad_u64_u32 %1, %2, %9, %10, %1\n"
        "v_mad_u64_u32 %0, %2, %11, %12, %0\n"
        "v_mad_u64_u32 %1, %2, %13, %14, %1\n"
        "v_mad_u64_u32 %0, %2, %15, %16, %0\n"
        "v_mad_u64_u32 %1, %2, %17, %18, %1\n"
        "v_mad_u64_u32 %0, %2, %19, %20, %0\n"
        "v_mad_u64_u32 %1, %2, %21, %22, %1\n"
        "v_mad_u64_u32 %0, %2, %23, %24, %0\n"
        "v_mad_u64_u32 %1, %2, %25, %26, %1\n"
        "v_mad_u64_u32 %0, %2, %27, %28, %0\n"
        "v_mad_u64_u32 %1, %2, %29, %30, %1\n"
        "v_mad_u64_u32 %0, %2, %31, %32, %0\n"
        "v_mad_u64_u32 %1, %2, %33, %34, %1\n"
        "v_mad_u64_u32 %0, %2, %35, %36, %0\n"
        "v_mad_u64_u32 %1, %2, %37, %38, %1\n"
        "v_mad_u64_u32 %0, %2, %39, %40, %0\n"
        "v_mad_u64_u32 %1, %2, %41, %42, %1\n"
        : "+v"(sa), "+v"(sb), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(c[0]), "v"(d[0]), "v"(a[1]), "v"(b[1]), "v"(c[1]), "v"(d[1]), "v"(a[2]), "v"(b[2]), "v"(c[2]), "v"(d[2]), "v"(a[3]), "v"(b[3]), "v"(c[3]), "v"(d[3]), "v"(a[4]), "v"(b[4]), "v"(c[4]), "v"(d[4]), "v"(a[5]), "v"(b[5]), "v"(c[5]), "v"(d[5]), "v"(a[6]), "v"(b[6]), "v"(c[6]), "v"(d[6]), "v"(a[7]), "v"(b[7]), "v"(c[7]), "v"(d[7]), "v"(a[8]), "v"(b[8]), "v"(c[8]), "v"(d[8]), "v"(a[9]), "v"(b[9]), "v"(c[9]), "v"(d[9]));
    (void)cc;
  }
};

/* Two independent products at once, their column chains interleaved mad by
   mad (madc2): h = f * g and h2 = f2 * g2 with fe_mul's bounds.  Outputs are
   written last, so they may alias any input. */
FDG_DEV void fe_mul_x2(fe &h, const fe &f, const fe &g, fe &h2, const fe &f_, const fe &g_) {
  uint32_t ga[10], fa[10], gb[10], fb[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    ga[i] = 19u * g.v[i]; fa[i] = f.v[i] << 1;
    gb[i] = 19u * g_.v[i]; fb[i] = f_.v[i] << 1;
  }
  uint32_t ra[10], rb[10];
  uint64_t ca = 0, cb = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t sa = ca, sb = cb;
    uint32_t xa[10], ya[10], xb[10], yb[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      const bool dbl = (i & 1) && (j & 1);
      xa[i] = dbl ? fa[i] : f.v[i];  ya[i] = wrap ? ga[j] : g.v[j];
      xb[i] = dbl ? fb[i] : f_.v[i]; yb[i] = wrap ? gb[j] : g_.v[j];
    }
    madc2<10>::run(sa, sb, xa, ya, xb, yb);
    const int bits = (k & 1) ? 25 : 26;
    ra[k] = (uint32_t)sa & ((1u << bits) - 1); ca = sa >> bits;
    rb[k] = (uint32_t)sb & ((1u << bits) - 1); cb = sb >> bits;
  }
  fe_ff_close(h, ra, ca);
  fe_ff_close(h2, rb, cb);
  FDG_SCHED_FENCE();
}

/* h = 2^SH f^2 and h2 = 2^SH f_^2 interleaved (fe_sq_sh's bounds). */
template <int SH>
FDG_DEV void fe_sq_sh_x2(fe &h, const fe &f, fe &h2, const fe &f_) {
  uint32_t a2[10], a4[10], a8[10], a19[10], b2[10], b4[10], b8[10], b19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    a2[i] = f.v[i] << 1; a4[i] = f.v[i] << 2; a8[i] = f.v[i] << 3; a19[i] = 19u * f.v[i];
    b2[i] = f_.v[i] << 1; b4[i] = f_.v[i] << 2; b8[i] = f_.v[i] << 3; b19[i] = 19u * f_.v[i];
  }
  auto pa = [&](int m, int i) { return m == 0 ? f.v[i] : m == 1 ? a2[i] : m == 2 ? a4[i] : a8[i]; };
  auto pb = [&](int m, int i) { return m == 0 ? f_.v[i] : m == 1 ? b2[i] : m == 2 ? b4[i] : b8[i]; };
  uint32_t ra[10], rb[10];
  uint64_t ca = 0, cb = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t sa = ca, sb = cb;
    uint32_t xa[6], ya[6], xb[6], yb[6];
    int n = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        const int mul2 = (i != j ? 1 : 0) + (((i & 1) && (j & 1)) ? 1 : 0) + SH;
        xa[n] = pa(mul2, i); ya[n] = (i + j) >= 10 ? a19[j] : f.v[j];
        xb[n] = pb(mul2, i); yb[n] = (i + j) >= 10 ? b19[j] : f_.v[j];
        n++;
      }
    }
    if (k & 1) madc2<5>::run(sa, sb, xa, ya, xb, yb);
    else madc2<6>::run(sa, sb, xa, ya, xb, yb);
    const int bits = (k & 1) ? 25 : 26;
    ra[k] = (uint32_t)sa & ((1u << bits) - 1); ca = sa >> bits;
    rb[k] = (uint32_t)sb & ((1u << bits) - 1); cb = sb >> bits;
  }
  fe_ff_close(h, ra, ca);
  fe_ff_close(h2, rb, cb);
  FDG_SCHED_FENCE();
}

FDG_DEV void fe_sq_x2(fe &h, const fe &f, fe &h2, const fe &f_) { fe_sq_sh_x2<0>(h, f, h2, f_); }

template <int V>
__global__ void __launch_bounds__(256) kbench(uint32_t *out, const uint32_t *in, int iters) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, x2, y;
#pragma unroll
  for (int w = 0; w < 10; w++) {
    x.v[w] = in[w * 64 + (gid & 63)]; y.v[w] = in[(10 + w) * 64 + (gid & 63)];
    x2.v[w] = in[(20 + w) * 64 + (gid & 63)];
  }
  for (int it = 0; it < iters; it++) {
    if constexpr (V == 0) fe_mul(x, x, y);
    else if constexpr (V == 1) fe_sq(x, x);
    else if constexpr (V == 2) { fe_mul(x, x, y); fe_mul(x2, x2, y); }
    else if constexpr (V == 3) fe_mul_x2(x, x, y, x2, x2, y);
    else if constexpr (V == 4) { fe_sq(x, x); fe_sq(x2, x2); }
    else fe_sq_x2(x, x, x2, x2);
  }
  fe_canon(x); fe_canon(x2);
#pragma unroll
  for (int w = 0; w < 10; w++) { out[(size_t)gid * 20 + w] = x.v[w]; out[(size_t)gid * 20 + 10 + w] = x2.v[w]; }
}

template <int V>
static double run(uint32_t *dout, const uint32_t *din, int ncu, int waves, int iters, uint32_t *canon) {
  const int blocks = ncu * waves, threads = 256;
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  kbench<V><<<blocks, threads>>>(dout, din, 2); CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0)); kbench<V><<<blocks, threads>>>(dout, din, iters); CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1)); float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  kbench<V><<<1, 64>>>(dout, din, 37); CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(canon, dout, 64 * 20 * 4, hipMemcpyDeviceToHost));
  const int chains = (V >= 2) ? 2 : 1;
  return (double)blocks * threads * iters * chains / (best * 1e-3);   /* products per second */
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  uint32_t hin[30 * 64];
  srand(7);
  for (int i = 0; i < 30 * 64; i++) hin[i] = ((uint32_t)rand() ^ ((uint32_t)rand() << 16)) & (((i / 64) & 1) ? 0x1ffffff : 0x3ffffff);
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, sizeof(hin)));
  CHECK(hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&dout, (size_t)ncu * 4 * 256 * 20 * 4));
  const int iters = 4096;
  static uint32_t c[6][1280];
  int ok = 1;
  for (int w : {1, 2, 4}) {
    const double r0 = run<0>(dout, din, ncu, w, iters, c[0]), r1 = run<1>(dout, din, ncu, w, iters, c[1]);
    const double r2 = run<2>(dout, din, ncu, w, iters, c[2]), r3 = run<3>(dout, din, ncu, w, iters, c[3]);
    const double r4 = run<4>(dout, din, ncu, w, iters, c[4]), r5 = run<5>(dout, din, ncu, w, iters, c[5]);
    const int eq_mul = !memcmp(c[2], c[3], sizeof(c[2])), eq_sq = !memcmp(c[4], c[5], sizeof(c[4]));
    ok &= eq_mul & eq_sq;
    printf("{\"waves_per_simd\": %d, \"mul1\": %.4e, \"sq1\": %.4e, \"mul2_seq\": %.4e, \"mul2_x2\": %.4e, "
           "\"sq2_seq\": %.4e, \"sq2_x2\": %.4e, \"mul_x2_gain\": %.4f, \"sq_x2_gain\": %.4f, \"eq_mul\": %d, \"eq_sq\": %d}\n",
           w, r0, r1, r2, r3, r4, r5, r3 / r2 - 1, r5 / r4 - 1, eq_mul, eq_sq);
  }
  return ok ? 0 : 1;
}
