// rti_perpixel.hip -- reference-faithful per-pixel PTM fit on gfx950.
//
// In the reference every pixel has its OWN light list: compute_intensities
// (analysis.py:221-232) gives pixel (x, y) and camera i the direction
// l = (cam_i − (x, y, 0)) / ‖cam_i − (x, y, 0)‖, kept as float32 lx/ly, and
// _interpolate_PTM (analysis.py:280-298) solves that pixel's N×6 system by SVD
// without rcond.  Here one lane owns one pixel: it forms the PTM row in fp32
// (as the reference's float32 monomials), accumulates the 6×6 normal
// equations AᵀA, Aᵀb in fp64 and solves them by Cholesky in fp64.  For a
// full-rank A that is the same least-squares solution the SVD returns (the
// fp64 normal equations lose cond(A)²·1e-16); a pixel whose Cholesky pivots
// show an ill-conditioned A (ne_solve) is marked and re-solved by a second,
// refine launch (refine_*) with a streaming fp64 Givens QR of A itself
// (qr_solve_wave), which loses cond(A)·1e-16 like the reference's SVD; a
// rank-deficient A gives NaN coefficients, as the reference's division by a
// zero singular value does.
//
//  * fit_perpixel_cam : directions generated in-kernel from cams[N][3]
//    (light-major, coalesced intensity planes; no lx/ly traffic at all).
//  * fit_perpixel_dirs: explicit pixel-major lx/ly/I [P][N], exactly the
//    arrays interpolate_intensities receives (analysis.py:341-354).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "rti_basis.h"
#include "rti_internal.h"

namespace rti {
namespace {

template <typename T>
__device__ __forceinline__ double ld_d(const T* p) {
  return (double)*p;
}

// Packed upper triangle of the symmetric 6×6 normal matrix.
constexpr int tri(int i, int j) {
  return i <= j ? i * 6 - i * (i - 1) / 2 + (j - i) : j * 6 - j * (j - 1) / 2 + (i - j);
}

struct Normal6 {
  double m[21];
  double b[6];
};

__device__ __forceinline__ void ne_zero(Normal6& ne) {
#pragma unroll
  for (int i = 0; i < 21; ++i) ne.m[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) ne.b[i] = 0.0;
}

// Row (lu², lv², lu·lv, lu, lv, 1.) with fp32 monomials (analysis.py:284-285).  The
// constant column costs adds, not FMAs, and its diagonal entry Σ 1·1 = N is set once
// before the solve (ne_finish).
__device__ __forceinline__ void ne_add(Normal6& ne, float lu, float lv, double L) {
  const double r[5] = {(double)(lu * lu), (double)(lv * lv), (double)(lu * lv), (double)lu, (double)lv};
#pragma unroll
  for (int i = 0; i < 5; ++i) {
#pragma unroll
    for (int j = i; j < 5; ++j) ne.m[tri(i, j)] = fma(r[i], r[j], ne.m[tri(i, j)]);
    ne.m[tri(i, 5)] += r[i];
    ne.b[i] = fma(r[i], L, ne.b[i]);
  }
  ne.b[5] += L;
}

__device__ __forceinline__ void ne_finish(Normal6& ne, int N) { ne.m[tri(5, 5)] = (double)N; }

// compute_intensities' direction l = d / ‖d‖ (analysis.py:228-229), components rounded to fp32
// (:230-231), BIT-EXACT with the reference's arrays at the cost of an rsq: the reference rounds
// s = (dx² + dy²) + dz² op by op, n = sqrt(s) and q = dx / n correctly (IEEE fp64), then q to fp32.
// Here s = fma(dx, dx, fma(dy, dy, dz²)) (within 2 ulps of the reference's s), 1/√s is the v_rsq_f64 seed
// refined by ONE Newton step, and q̃ = dx·(1/√s) lies within ~200 fp64 ulps of q.  fp32 rounding looks only
// at the low 29 bits of q's fp64 significand, so fp32(q̃) == fp32(q) unless q̃ lies within those ulps of an
// fp32 rounding midpoint (low 29 bits = 2^28), or the fp32 result is subnormal.  The fast form folds both
// tests into two running minima (mid_key < MID_KEY_MAX, or |l| < FLT_MIN, flags the light: ≈1 in 5·10⁵
// components, a few thousand pixels of a 4K image), and a flagged pixel is re-solved by the refine pass,
// whose light_dir_exact uses the IEEE sqrt and divide of rti_light_dirs.  Pinned by
// tests/golden/ptm_perpixel_32x32_N50.npz through rti_fit_perpixel_cam (test_gpu_perpixel_relight.py).
// Ulp budget of q̃ (tools/probe/rsq_probe.hip, profiles/r03_rsq_probe.log: v_rsq_f64 ≤ 2.46e8 ulps measured,
// 2^29 documented; one Newton step ≤ 19.8 ulps measured, ≤ 1.5·(2^-23)² relative = 192 ulps from the
// documented seed; two steps 0.99): s two fma roundings vs the reference's four (≤ 4 ulps of s -> 2 of
// 1/√s), the product 0.5, the reference's sqrt and divide 0.5 each: ≤ 196 ulps, so a margin of 512 leaves
// a factor 2.6.  One Newton step instead of two saves 3 of the ≈57 VALU ops per pixel·light; the extra
// flagged pixels cost the wave-cooperative refine a few µs.
// NW Newton steps on the rsq seed, and the midpoint margin that covers the resulting ulp budget: one step
// (≤ 196 ulps) with a margin of 512, or two steps (≤ 4.5 ulps: rsq + 2 Newton steps 0.99 ulp, the rest as
// above) with a margin of 16.  AUTO uses one step (profiles/r03_c6_variants_sweep.log).
template <int NW>
constexpr uint32_t mid_margin() { return NW >= 2 ? 16 : 512; }

// mid_key(q) < 16·margin iff the low 29 significand bits of q lie within `margin` of 2^28 (an fp32 rounding
// midpoint): with lo29 = those bits, (lo << 3) + 2^31 + 8·margin = 8·((lo29 − 2^28 + margin) mod 2^29)
// (mod 2^32; the shift drops bits 29..31 and adding 2^31 flips bit 28 of lo29), one v_lshl_add_u32 per
// component.
template <int NW>
__device__ __forceinline__ uint32_t mid_key(double q) {
  const uint32_t lo = (uint32_t)__double_as_longlong(q);
  return (lo << 3) + (0x80000000u + 8 * mid_margin<NW>());
}

template <int NW>
struct DirCheck {
  uint32_t key = 0xFFFFFFFFu;  // min of mid_key over the pixel's light components
  float lmin = 1.0f;           // min of |l| (an fp32 subnormal or 0 result rounds on more bits)
  __device__ __forceinline__ bool ambiguous() const {
    return key < 16 * mid_margin<NW>() || !(lmin >= 0x1p-126f);
  }
};

template <int NW>
__device__ __forceinline__ void light_dir_fast(double dx, double dy, double dz2, float& lu, float& lv,
                                               DirCheck<NW>& chk) {
  const double s = fma(dx, dx, fma(dy, dy, dz2));
  double y = __builtin_amdgcn_rsq(s);
  const double h = 0.5 * s;
#pragma unroll
  for (int i = 0; i < NW; ++i) y = fma(y, fma(-h * y, y, 0.5), y);
  const double qx = dx * y, qy = dy * y;
  lu = (float)qx;
  lv = (float)qy;
  chk.key = min(chk.key, min(mid_key<NW>(qx), mid_key<NW>(qy)));
  chk.lmin = fminf(chk.lmin, fminf(fabsf(lu), fabsf(lv)));
}

// the reference's arithmetic exactly (rti_light_dirs): separately rounded IEEE ops, no contraction
__device__ __forceinline__ void light_dir_exact(double dx, double dy, double dz, float& lu, float& lv) {
#pragma clang fp contract(off)
  const double n = sqrt(dx * dx + dy * dy + dz * dz);
  lu = (float)(dx / n);
  lv = (float)(dy / n);
}

// Cholesky solve of (AᵀA) a = Aᵀb.  rcond < 0: singular only at a non-positive
// pivot (reference semantics); rcond >= 0: pivots <= rcond²·max(diag) count
// as singular.  Singular -> all-NaN coefficients.  Returns true when the system is
// ill-conditioned for the normal equations: a pivot kept less than ILL_RATIO of its
// column's squared norm (the scaled cond(A)² ≳ 1/ILL_RATIO, where the normal equations
// lose cond(A)²·1e-16 against the reference's SVD) — the caller then re-solves the pixel by
// Givens QR of A itself (qr_solve_wave), which loses only cond(A)·1e-16 like the SVD.
constexpr double ILL_RATIO = 1e-6;

__device__ __forceinline__ bool ne_solve(const Normal6& ne, double rcond, double (&a)[6]) {
  double L[6][6];
  double dmax = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) dmax = fmax(dmax, ne.m[tri(i, i)]);
  const double thr = rcond < 0.0 ? 0.0 : rcond * rcond * dmax;
  bool ok = true, ill = false;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double d = ne.m[tri(j, j)];
#pragma unroll
    for (int p = 0; p < j; ++p) d -= L[j][p] * L[j][p];
    ok = ok && (d > thr);
    ill = ill || !(d > ILL_RATIO * ne.m[tri(j, j)]);
    const double ljj = sqrt(d > 0.0 ? d : 1.0);
    L[j][j] = ljj;
    const double inv = 1.0 / ljj;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double s = ne.m[tri(i, j)];
#pragma unroll
      for (int p = 0; p < j; ++p) s -= L[i][p] * L[j][p];
      L[i][j] = s * inv;
    }
  }
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = ne.b[i];
#pragma unroll
    for (int p = 0; p < i; ++p) s -= L[i][p] * y[p];
    y[i] = s / L[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
#pragma unroll
    for (int p = i + 1; p < 6; ++p) s -= L[p][i] * a[p];
    a[i] = s / L[i][i];
  }
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 6; ++i) a[i] = __builtin_nan("");
  }
  return ok && ill;  // an exactly singular system stays NaN (the reference's zero singular value)
}

// Least squares by Givens QR of [A | L] streamed row by row in fp64 (R upper 6×6 packed, z = QᵀL):
// backward stable in A itself, so the solution carries cond(A)·1e-16 relative error — the accuracy of
// the reference's SVD (analysis.py:295-298) for the ill-conditioned light sets the normal equations
// cannot take (tests/golden/ptm_edge.npz near-collinear lights, cond(A) = 1.1e8).  `row(n, r, L)`
// yields light n's PTM row and intensity.  Singular semantics as ne_solve: AᵀA = RᵀR, so a pivot
// R_jj² <= rcond²·max diag(AᵀA) (rcond >= 0) or R_jj = 0 gives NaN coefficients.
struct QR6 {
  double R[21];  // upper 6×6 R, packed (tri)
  double z[6];   // Qᵀ·L
  double cn[6];  // squared column norms of A (the rcond threshold)
};

__device__ __forceinline__ void qr_zero(QR6& s) {
#pragma unroll
  for (int i = 0; i < 21; ++i) s.R[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) s.z[i] = s.cn[i] = 0.0;
}

// rotate the row [x | l] into R (Givens, column by column; x is consumed)
__device__ __forceinline__ void qr_rot(QR6& s, double (&x)[6], double l) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double xj = x[j];
    if (xj == 0.0) continue;
    const double rjj = s.R[tri(j, j)];
    // h = hypot(rjj, xj) and 1/h from v_rsq_f64 + two Newton steps (≈1 ulp, tools/probe/rsq_probe.hip):
    // the rotation stays orthogonal to ~1e-16, so the QR keeps its backward stability, at a third of the
    // latency of IEEE sqrt + divides.  Intensities and PTM rows are O(1e3) at most: h² neither overflows
    // nor underflows.
    const double h2 = fma(rjj, rjj, xj * xj);
    double y = __builtin_amdgcn_rsq(h2);
    const double hh = 0.5 * h2;
    y = fma(y, fma(-hh * y, y, 0.5), y);
    y = fma(y, fma(-hh * y, y, 0.5), y);
    const double c = rjj * y, sn = xj * y;
    s.R[tri(j, j)] = h2 * y;
#pragma unroll
    for (int k = j + 1; k < 6; ++k) {
      const double t = s.R[tri(j, k)];
      s.R[tri(j, k)] = fma(c, t, sn * x[k]);
      x[k] = fma(-sn, t, c * x[k]);
    }
    const double t = s.z[j];
    s.z[j] = fma(c, t, sn * l);
    l = fma(-sn, t, c * l);
  }
}

__device__ __forceinline__ void qr_add(QR6& s, double (&x)[6], double l) {
#pragma unroll
  for (int i = 0; i < 6; ++i) s.cn[i] = fma(x[i], x[i], s.cn[i]);
  qr_rot(s, x, l);
}

// TSQR merge: the rows of o's [R | z] rotated into s (QR of the stacked pair)
__device__ __forceinline__ void qr_merge(QR6& s, const QR6& o) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double x[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) x[j] = j < i ? 0.0 : o.R[tri(i, j)];
    qr_rot(s, x, o.z[i]);
    s.cn[i] += o.cn[i];
  }
}

// Singular semantics as ne_solve: AᵀA = RᵀR, so a pivot R_jj² <= rcond²·max diag(AᵀA) (rcond >= 0) or
// R_jj = 0 gives NaN coefficients.
__device__ __forceinline__ void qr_finish(const QR6& s, double rcond, double (&a)[6]) {
  double cmax = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) cmax = fmax(cmax, s.cn[i]);
  const double thr = rcond < 0.0 ? 0.0 : rcond * sqrt(cmax);
  bool ok = true;
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    ok = ok && (s.R[tri(i, i)] > thr);
    double t = s.z[i];
#pragma unroll
    for (int p = i + 1; p < 6; ++p) t -= s.R[tri(i, p)] * a[p];
    a[i] = t / s.R[tri(i, i)];
  }
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 6; ++i) a[i] = __builtin_nan("");
  }
}

// Least squares by Givens QR of [A | L] in fp64 (R upper 6×6 packed, z = QᵀL): backward stable in A
// itself, so the solution carries cond(A)·1e-16 relative error — the accuracy of the reference's SVD
// (analysis.py:295-298) for the ill-conditioned light sets the normal equations cannot take
// (tests/golden/ptm_edge.npz near-collinear lights, cond(A) = 1.1e8).  Wave-cooperative (TSQR): lane l
// rotates in the rows n = l, l + 64, ..., then the 64 lanes' [R | z] are merged by an xor butterfly of
// pairwise QRs; lane 0's result is used.  `row(n, r, L)` yields light n's PTM row and intensity.
template <typename Row>
__device__ __forceinline__ void qr_solve_wave(int N, double rcond, Row row, double (&a)[6]) {
  QR6 s;
  qr_zero(s);
  for (int n = threadIdx.x & 63; n < N; n += 64) {
    double x[6], l;
    row(n, x, l);
    qr_add(s, x, l);
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    QR6 o;
#pragma unroll
    for (int i = 0; i < 21; ++i) o.R[i] = __shfl_xor(s.R[i], off);
#pragma unroll
    for (int i = 0; i < 6; ++i) o.z[i] = __shfl_xor(s.z[i], off), o.cn[i] = __shfl_xor(s.cn[i], off);
    qr_merge(s, o);
  }
  qr_finish(s, rcond, a);
}

__device__ __forceinline__ void ptm_row_d(float lu, float lv, double (&r)[6]) {
  r[0] = (double)(lu * lu);
  r[1] = (double)(lv * lv);
  r[2] = (double)(lu * lv);
  r[3] = (double)lu;
  r[4] = (double)lv;
  r[5] = 1.0;
}

template <typename TC, int LAYOUT>
__device__ __forceinline__ void store_coef(TC* __restrict__ coef, int64_t P, int64_t p, const double (&a)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if constexpr (LAYOUT == RTI_COEF_PLANAR)
      coef[(int64_t)i * P + p] = (TC)a[i];
    else
      coef[p * 6 + i] = (TC)a[i];
  }
}

// A pixel the fast kernel cannot finish leaves one of two signalling-NaN bit patterns in its first
// coefficient for the refine pass (refine_*): EXACT = a light vector the fast form could not round with
// certainty (redo the pixel with the IEEE light vectors), QR = an ill-conditioned system (redo it by Givens
// QR).  No arithmetic produces these patterns (results are quiet NaNs), and the refine pass overwrites them.
constexpr int MARK_NONE = 0, MARK_EXACT = 1, MARK_QR = 2;
template <typename TC>
struct Mark;
template <>
struct Mark<double> {
  using U = unsigned long long;
  static constexpr U exact = 0x7FF0515249514D45ull, qr = 0x7FF0515249514D4Bull;
};
template <>
struct Mark<float> {
  using U = unsigned int;
  static constexpr U exact = 0x7FA51A10u, qr = 0x7FA51A11u;
};

template <typename TC, int LAYOUT>
__device__ __forceinline__ TC* coef0(TC* coef, int64_t P, int64_t p) {
  (void)P;
  return LAYOUT == RTI_COEF_PLANAR ? coef + p : coef + p * 6;
}

template <typename TC, int LAYOUT>
__device__ __forceinline__ void put_mark(TC* coef, int64_t P, int64_t p, int mark) {
  *reinterpret_cast<typename Mark<TC>::U*>(coef0<TC, LAYOUT>(coef, P, p)) =
      mark == MARK_QR ? Mark<TC>::qr : Mark<TC>::exact;
}

// Solve and store one pixel; a pixel the fast path cannot finish is marked, and so is the first pixel of its
// wave (MARK_EXACT: "redo this pixel from the start"), so the refine pass reads one coefficient per wave
// (64 pixels) instead of one per pixel and looks at the wave's pixels only when that one is marked.
template <typename TC, int LAYOUT>
__device__ __forceinline__ void solve_store(const Normal6& ne, double rcond, TC* __restrict__ coef, int64_t P,
                                            int64_t p, bool inexact_dirs = false) {
  double a[6];
  const bool ill = ne_solve(ne, rcond, a);
  const bool marked = ill || inexact_dirs;
  // lane 0 = the wave's first pixel (launches of 256-thread blocks): it carries the wave's flag
  const bool any = __ballot(marked) != 0;  // every active lane takes part (not under a lane-dependent branch)
  const bool flag = (threadIdx.x & 63) == 0 && any;
  store_coef<TC, LAYOUT>(coef, P, p, a);
  if (__builtin_expect(marked || flag, 0)) put_mark<TC, LAYOUT>(coef, P, p, ill && !flag ? MARK_QR : MARK_EXACT);
}

template <typename TC, int LAYOUT>
__device__ __forceinline__ int mark_of(const TC* coef, int64_t P, int64_t p) {
  const auto u = *reinterpret_cast<const typename Mark<TC>::U*>(coef0<TC, LAYOUT>(const_cast<TC*>(coef), P, p));
  return u == Mark<TC>::exact ? MARK_EXACT : (u == Mark<TC>::qr ? MARK_QR : MARK_NONE);
}

// The fused fit: each light enters the normal equations as soon as its fast light vector is formed, and the
// DirCheck of each group of 4 lights is tested once.  A lane whose group holds an ambiguous component (≈1 in
// 5·10⁵ components, so a wave takes the branch about once in 40 groups of its 25) recomputes the group's fast
// vectors (deterministic: the same bits) and replaces every one that differs from the reference's IEEE vector
// (light_dir_exact) by subtracting its row and adding the exact one.  Every light vector in the final normal
// equations is the reference's, bit for bit (the sums carry one extra rounding per replaced row, ≈1e-16
// relative), and only ill-conditioned pixels (MARK_QR) are left to the refine pass.  The fix-up recomputes
// rather than keeps the group's vectors so the hot loop stays within its 80-VGPR budget (6 waves per SIMD);
// a whole-pixel redo in the same place measured 1.71 ms against 1.51 ms + a 96 µs refine pass.
__device__ __forceinline__ void ne_sub(Normal6& ne, float lu, float lv, double L) {
  const double r[5] = {(double)(lu * lu), (double)(lv * lv), (double)(lu * lv), (double)lu, (double)lv};
#pragma unroll
  for (int i = 0; i < 5; ++i) {
#pragma unroll
    for (int j = i; j < 5; ++j) ne.m[tri(i, j)] = fma(-r[i], r[j], ne.m[tri(i, j)]);
    ne.m[tri(i, 5)] -= r[i];
    ne.b[i] = fma(-r[i], L, ne.b[i]);
  }
  ne.b[5] -= L;
}

// VAR (measurement switch RTI_PERPIXEL_VARIANT, default 3): 0 = two Newton steps, an ambiguous pixel marked
// for the refine pass; 1 = one step, marked; 2 = one step, fixed up in place per group of 4 lights;
// 3 = 2 at 5 waves per SIMD (96 VGPRs: the fix-up's IEEE temporaries without spills); 4 = 2 at 4 waves;
// 5 = 3 with every group fixed up (test-only: exercises the replace path on any input).
template <typename T, typename TC, int LAYOUT, int VAR>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(VAR == 3 || VAR == 5 ? 5 : (VAR == 4 ? 4 : 6))))
fit_perpixel_cam(const double* __restrict__ cams, int N, const T* __restrict__ I, int H, int W, int64_t lstride,
                 double x0, double y0, double rcond, TC* __restrict__ coef) {
  constexpr int NW = VAR == 0 ? 2 : 1;
  const int64_t P = (int64_t)H * W;
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const double px = x0 + (double)(p % W);
  const double py = y0 + (double)(p / W);
  Normal6 ne;
  ne_zero(ne);
  const uint32_t po = (uint32_t)(p * (int64_t)sizeof(T));  // per-lane byte offset into each plane (< 2^32: launcher)
  auto plane = [&](int n) {  // cams and the plane base are wave-uniform: scalar loads
    return ld_d(reinterpret_cast<const T*>(reinterpret_cast<const char*>(I + (int64_t)n * lstride) + po));
  };
  auto light = [&](int n, DirCheck<NW>& chk) {
    float lu, lv;
    const double cz = cams[3 * n + 2];
    light_dir_fast<NW>(cams[3 * n + 0] - px, cams[3 * n + 1] - py, cz * cz, lu, lv, chk);
    ne_add(ne, lu, lv, plane(n));
  };
  if constexpr (VAR < 2) {
    DirCheck<NW> chk;
#pragma unroll 4
    for (int n = 0; n < N; ++n) light(n, chk);
    ne_finish(ne, N);
    solve_store<TC, LAYOUT>(ne, rcond, coef, P, p, chk.ambiguous());
  } else {
    auto fix = [&](int n0, int G) {
#pragma clang loop unroll(disable)
      for (int u = 0; u < G; ++u) {
        const int n = n0 + u;
        const double cz = cams[3 * n + 2];
        float fu, fv, eu, ev;
        DirCheck<NW> unused;
        light_dir_fast<NW>(cams[3 * n + 0] - px, cams[3 * n + 1] - py, cz * cz, fu, fv, unused);
        light_dir_exact(cams[3 * n + 0] - px, cams[3 * n + 1] - py, cz, eu, ev);
        if (__float_as_uint(fu) != __float_as_uint(eu) || __float_as_uint(fv) != __float_as_uint(ev)) {
          const double L = plane(n);
          ne_sub(ne, fu, fv, L);
          ne_add(ne, eu, ev, L);
        }
      }
    };
    int n = 0;
    for (; n + 4 <= N; n += 4) {
      DirCheck<NW> chk;
#pragma unroll
      for (int u = 0; u < 4; ++u) light(n + u, chk);
      if (__builtin_expect(VAR == 5 || chk.ambiguous(), 0)) fix(n, 4);
    }
    for (; n < N; ++n) {
      DirCheck<NW> chk;
      light(n, chk);
      if (__builtin_expect(VAR == 5 || chk.ambiguous(), 0)) fix(n, 1);
    }
    ne_finish(ne, N);
    solve_store<TC, LAYOUT>(ne, rcond, coef, P, p);
  }
}

// Refine launches (refine_grid): wave gw looks after the 64 fit waves (4096 pixels) [64·gw, 64·gw + 64): lane i
// reads the flag of fit wave 64·gw + i (its first pixel's first coefficient), so the pass reads one value
// per 64 pixels and dispatches one workgroup per 16 384 pixels.  A flagged fit wave's 64 marks are read
// by the 64 lanes and its marked pixels redone one after another, all 64 lanes on each (lights n = lane,
// lane + 64, ...; the normal equations summed by an xor butterfly, so every lane holds the same sums and
// takes the same branch).  A lane per marked pixel would run its N lights serially, each waiting for its
// own HBM load (≈70 µs for one marked wave on c6); the wave does the same pixel in a few µs.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

template <typename RowF>
__device__ __forceinline__ void ne_wave(int N, RowF row, Normal6& ne) {
  ne_zero(ne);
  for (int n = threadIdx.x & 63; n < N; n += 64) {
    float lu, lv;
    double L;
    row(n, lu, lv, L);
    ne_add(ne, lu, lv, L);
  }
#pragma unroll
  for (int i = 0; i < 21; ++i) ne.m[i] = wave_sum(ne.m[i]);
#pragma unroll
  for (int i = 0; i < 6; ++i) ne.b[i] = wave_sum(ne.b[i]);
  ne_finish(ne, N);
}

// Calls solve(q, mark) for every marked pixel q of the flagged fit waves this wave looks after (wave-uniform).
template <typename TC, int LAYOUT, typename F>
__device__ __forceinline__ void refine_scan(const TC* coef, int64_t P, F&& solve) {
  const int lane = threadIdx.x & 63;
  const int64_t fw0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64, nfw = (P + 63) / 64;
  const bool flagged = fw0 + lane < nfw && mark_of<TC, LAYOUT>(coef, P, (fw0 + lane) * 64) != MARK_NONE;
  uint64_t fm = __ballot(flagged);
  while (fm) {
    const int64_t w0 = (fw0 + __builtin_ctzll(fm)) * 64;
    fm &= fm - 1;
    const int64_t p = w0 + lane;
    const int mark = p < P ? mark_of<TC, LAYOUT>(coef, P, p) : MARK_NONE;
    uint64_t m = __ballot(mark != MARK_NONE);
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      solve(w0 + l, __shfl(mark, l));
    }
  }
}

// one refine wave per 64 fit waves
inline dim3 refine_grid(int64_t P) { return dim3((unsigned)(((P + 63) / 64 + 255) / 256)); }

// Refine pass of fit_perpixel_cam: QR pixels (ill-conditioned) are solved by the Givens QR of their exact
// rows; an EXACT mark is a wave's flag on its first pixel, which is re-accumulated with the IEEE light
// vectors (light_dir_exact, the vectors the fit used) and solved as in the fit (falling through to QR if
// ill-conditioned).
template <typename T, typename TC, int LAYOUT>
__global__ void __launch_bounds__(256)
refine_cam(const double* __restrict__ cams, int N, const T* __restrict__ I, int H, int W, int64_t lstride,
           double x0, double y0, double rcond, TC* __restrict__ coef) {
  const int64_t P = (int64_t)H * W;
  const int lane = threadIdx.x & 63;
  refine_scan<TC, LAYOUT>(coef, P, [&](int64_t q, int mk) {
    const double px = x0 + (double)(q % W);
    const double py = y0 + (double)(q / W);
    const T* __restrict__ src = I + q;
    auto row = [&](int n, float& lu, float& lv, double& L) {
      light_dir_exact(cams[3 * n + 0] - px, cams[3 * n + 1] - py, cams[3 * n + 2], lu, lv);
      L = ld_d(src + (int64_t)n * lstride);
    };
    double a[6];
    bool qr = mk == MARK_QR;
    if (!qr) {
      Normal6 ne;
      ne_wave(N, row, ne);
      qr = ne_solve(ne, rcond, a);
    }
    if (qr)
      qr_solve_wave(N, rcond, [&](int n, double (&r)[6], double& L) {
        float lu, lv;
        row(n, lu, lv, L);
        ptm_row_d(lu, lv, r);
      }, a);
    if (lane == 0) store_coef<TC, LAYOUT>(coef, P, q, a);
  });
}

template <typename T, typename TC, int LAYOUT>
__global__ void __launch_bounds__(256)
fit_perpixel_dirs(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N,
                  int64_t P, double rcond, TC* __restrict__ coef) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int64_t base = p * N;
  Normal6 ne;
  ne_zero(ne);
#pragma unroll 4
  for (int n = 0; n < N; ++n) ne_add(ne, lu[base + n], lv[base + n], ld_d(I + base + n));
  ne_finish(ne, N);
  solve_store<TC, LAYOUT>(ne, rcond, coef, P, p);
}

template <typename T, typename TC, int LAYOUT>
__global__ void __launch_bounds__(256)
refine_dirs(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N,
               int64_t P, double rcond, TC* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  refine_scan<TC, LAYOUT>(coef, P, [&](int64_t q, int mk) {
    const int64_t base = q * N;
    double a[6];
    bool qr = mk == MARK_QR;
    if (!qr) {  // the wave's first pixel (or a pixel redone from the start): the fit's own normal equations
      Normal6 ne;
      ne_wave(N, [&](int n, float& u, float& v, double& L) {
        u = lu[base + n];
        v = lv[base + n];
        L = ld_d(I + base + n);
      }, ne);
      qr = ne_solve(ne, rcond, a);
    }
    if (qr)
      qr_solve_wave(N, rcond, [&](int n, double (&r)[6], double& L) {
        ptm_row_d(lu[base + n], lv[base + n], r);
        L = ld_d(I + base + n);
      }, a);
    if (lane == 0) store_coef<TC, LAYOUT>(coef, P, q, a);
  });
}

// compute_intensities' light vectors (analysis.py:225-231); lane = (pixel, camera),
// camera fastest so the pixel-major [P][N] stores are contiguous.  Every operation is a
// separately rounded IEEE fp64 op in the order (dx² + dy²) + dz², sqrt, divide — no FMA
// contraction — so the fp32 results are bit-identical to the reference's arrays (pinned by
// tests/golden/ptm_perpixel_32x32_N50.npz).
__global__ void __launch_bounds__(256)
light_dirs(const double* __restrict__ cams, int N, int W, int64_t total, double x0, double y0,
           float* __restrict__ lu, float* __restrict__ lv) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int n = (int)(i % N);
  const int64_t p = i / N;
  const double dx = cams[3 * n + 0] - (x0 + (double)(p % W));
  const double dy = cams[3 * n + 1] - (y0 + (double)(p / W));
  const double dz = cams[3 * n + 2];
  const double nrm = sqrt(dx * dx + dy * dy + dz * dz);
  lu[i] = (float)(dx / nrm);
  lv[i] = (float)(dy / nrm);
}

template <typename T, typename TC, int LAYOUT>
void launch_cam(const double* cams, int N, const void* I, int H, int W, int64_t ls, double x0, double y0,
                double rcond, void* coef, hipStream_t s) {
  const int64_t P = (int64_t)H * W;
  const char* ev = getenv("RTI_PERPIXEL_VARIANT");  // measurement switch, read per call (A/B in one process)
  const int var = ev ? atoi(ev) : 3;
  auto kern = var == 0 ? fit_perpixel_cam<T, TC, LAYOUT, 0>
             : var == 1 ? fit_perpixel_cam<T, TC, LAYOUT, 1>
             : var == 2 ? fit_perpixel_cam<T, TC, LAYOUT, 2>
             : var == 4 ? fit_perpixel_cam<T, TC, LAYOUT, 4>
             : var == 5 ? fit_perpixel_cam<T, TC, LAYOUT, 5> : fit_perpixel_cam<T, TC, LAYOUT, 3>;
  hipLaunchKernelGGL(kern, dim3(grid_1d(P, 256)), dim3(256), 0, s, cams, N, static_cast<const T*>(I), H, W, ls, x0,
                     y0, rcond, static_cast<TC*>(coef));
  hipLaunchKernelGGL((refine_cam<T, TC, LAYOUT>), refine_grid(P), dim3(256), 0, s, cams, N,
                     static_cast<const T*>(I), H, W, ls, x0, y0, rcond, static_cast<TC*>(coef));
}

template <typename T, typename TC>
void launch_cam_l(int layout, const double* cams, int N, const void* I, int H, int W, int64_t ls, double x0,
                  double y0, double rcond, void* coef, hipStream_t s) {
  if (layout == RTI_COEF_PLANAR)
    launch_cam<T, TC, RTI_COEF_PLANAR>(cams, N, I, H, W, ls, x0, y0, rcond, coef, s);
  else
    launch_cam<T, TC, RTI_COEF_PIXEL_MAJOR>(cams, N, I, H, W, ls, x0, y0, rcond, coef, s);
}

template <typename T>
void launch_cam_c(int cdt, int layout, const double* cams, int N, const void* I, int H, int W, int64_t ls,
                  double x0, double y0, double rcond, void* coef, hipStream_t s) {
  if (cdt == RTI_F64)
    launch_cam_l<T, double>(layout, cams, N, I, H, W, ls, x0, y0, rcond, coef, s);
  else
    launch_cam_l<T, float>(layout, cams, N, I, H, W, ls, x0, y0, rcond, coef, s);
}

template <typename T, typename TC, int LAYOUT>
void launch_dirs(const float* lu, const float* lv, const void* I, int N, int64_t P, double rcond, void* coef,
                 hipStream_t s) {
  hipLaunchKernelGGL((fit_perpixel_dirs<T, TC, LAYOUT>), dim3(grid_1d(P, 256)), dim3(256), 0, s, lu, lv,
                     static_cast<const T*>(I), N, P, rcond, static_cast<TC*>(coef));
  hipLaunchKernelGGL((refine_dirs<T, TC, LAYOUT>), refine_grid(P), dim3(256), 0, s, lu, lv,
                     static_cast<const T*>(I), N, P, rcond, static_cast<TC*>(coef));
}

template <typename T>
void launch_dirs_c(int cdt, int layout, const float* lu, const float* lv, const void* I, int N, int64_t P,
                   double rcond, void* coef, hipStream_t s) {
  if (cdt == RTI_F64) {
    if (layout == RTI_COEF_PLANAR)
      launch_dirs<T, double, RTI_COEF_PLANAR>(lu, lv, I, N, P, rcond, coef, s);
    else
      launch_dirs<T, double, RTI_COEF_PIXEL_MAJOR>(lu, lv, I, N, P, rcond, coef, s);
  } else {
    if (layout == RTI_COEF_PLANAR)
      launch_dirs<T, float, RTI_COEF_PLANAR>(lu, lv, I, N, P, rcond, coef, s);
    else
      launch_dirs<T, float, RTI_COEF_PIXEL_MAJOR>(lu, lv, I, N, P, rcond, coef, s);
  }
}

int check_common(const char* fn, const void* I, int in_dtype, int N, int64_t P, void* coef, int coef_dtype,
                 int coef_layout) {
  if (!I || !coef) return fail(RTI_ERR_BAD_ARG, "%s: null pointer", fn);
  if (N <= 0 || P <= 0) return fail(RTI_ERR_BAD_ARG, "%s: N and P must be positive", fn);
  if (N < 6) return fail(RTI_ERR_BAD_ARG, "%s: %d lights < 6 PTM terms (analysis.py:298 raises ValueError)", fn, N);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "%s: input dtype %d", fn, in_dtype);
  if (coef_dtype != RTI_F32 && coef_dtype != RTI_F64)
    return fail(RTI_ERR_UNSUPPORTED, "%s: coef dtype %d", fn, coef_dtype);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "%s: coef layout %d", fn, coef_layout);
  return RTI_OK;
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_fit_perpixel_cam(const double* cams, int N, const void* I, int in_dtype, int H, int W,
                                    int64_t light_stride, double x0, double y0, double rcond, void* coef,
                                    int coef_dtype, int coef_layout, rti_stream_t stream) {
  if (!cams) return fail(RTI_ERR_BAD_ARG, "rti_fit_perpixel_cam: null cams");
  if (H <= 0 || W <= 0) return fail(RTI_ERR_BAD_ARG, "rti_fit_perpixel_cam: H and W must be positive");
  if ((int64_t)H * W * 4 >= ((int64_t)1 << 32))
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_perpixel_cam: H*W >= 2^30 pixels (32-bit plane byte offsets)");
  const int64_t P = (int64_t)H * W;
  int st = check_common("rti_fit_perpixel_cam", I, in_dtype, N, P, coef, coef_dtype, coef_layout);
  if (st != RTI_OK) return st;
  const int64_t ls = light_stride ? light_stride : P;
  if (ls < P) return fail(RTI_ERR_BAD_ARG, "rti_fit_perpixel_cam: light_stride < H*W");
  hipStream_t s = (hipStream_t)stream;
  switch (in_dtype) {
    case RTI_F32: launch_cam_c<float>(coef_dtype, coef_layout, cams, N, I, H, W, ls, x0, y0, rcond, coef, s); break;
    case RTI_I32: launch_cam_c<int32_t>(coef_dtype, coef_layout, cams, N, I, H, W, ls, x0, y0, rcond, coef, s); break;
    default: launch_cam_c<uint8_t>(coef_dtype, coef_layout, cams, N, I, H, W, ls, x0, y0, rcond, coef, s); break;
  }
  return check_launch("rti_fit_perpixel_cam");
}

extern "C" int rti_fit_perpixel_dirs(const float* lu, const float* lv, const void* I, int in_dtype, int N,
                                     int64_t P, double rcond, void* coef, int coef_dtype, int coef_layout,
                                     rti_stream_t stream) {
  if (!lu || !lv) return fail(RTI_ERR_BAD_ARG, "rti_fit_perpixel_dirs: null lu/lv");
  int st = check_common("rti_fit_perpixel_dirs", I, in_dtype, N, P, coef, coef_dtype, coef_layout);
  if (st != RTI_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  switch (in_dtype) {
    case RTI_F32: launch_dirs_c<float>(coef_dtype, coef_layout, lu, lv, I, N, P, rcond, coef, s); break;
    case RTI_I32: launch_dirs_c<int32_t>(coef_dtype, coef_layout, lu, lv, I, N, P, rcond, coef, s); break;
    default: launch_dirs_c<uint8_t>(coef_dtype, coef_layout, lu, lv, I, N, P, rcond, coef, s); break;
  }
  return check_launch("rti_fit_perpixel_dirs");
}

extern "C" int rti_light_dirs(const double* cams, int N, int H, int W, double x0, double y0, float* lu, float* lv,
                              rti_stream_t stream) {
  if (!cams || !lu || !lv) return fail(RTI_ERR_BAD_ARG, "rti_light_dirs: null pointer");
  if (N <= 0 || H <= 0 || W <= 0) return fail(RTI_ERR_BAD_ARG, "rti_light_dirs: N, H, W must be positive");
  const int64_t total = (int64_t)H * W * N;
  hipLaunchKernelGGL(light_dirs, dim3(grid_1d(total, 256)), dim3(256), 0, (hipStream_t)stream, cams, N, W, total, x0,
                     y0, lu, lv);
  return check_launch("rti_light_dirs");
}
