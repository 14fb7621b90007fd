// rti_rbf.hip -- per-pixel linear RBF on gfx950 (the reference's default method
// with its own geometry).
//
// interpolate_intensities (analysis.py:350-363) calls _interpolate_RBF
// (analysis.py:249-260) once per pixel: SciPy Rbf(lx, ly, I, function='linear')
// builds A_ij = ‖x_i − x_j‖ over that pixel's N light directions, solves A w = I
// (LAPACK gesv: LU with partial pivoting) and evaluates f(q) = Σ_j w_j ‖q − x_j‖
// on the 100×100 grid.  Every pixel has its own light list (compute_intensities,
// analysis.py:225-231), so there is no shared operator: one workgroup owns one
// pixel and solves its N×N system — fp64 Gauss-Jordan in registers up to N = 80, above that
// (to N = 256; the systems reach cond ≈ 1e4–1e5 at N = 100–200) an fp32 Gauss-Jordan inverse of
// the Householder-projected system held in registers as 8×8 blocks, plus fp64 iterative
// refinement, above N = 256 a blocked fp64 Cholesky of the same system in global memory
// (rbf_solve_chol) — and a second kernel streams the E evaluations in fp64.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "rti_convert.h"
#include "rti_internal.h"

namespace rti {
namespace {

constexpr int RBF_MAX_N = 256;  // largest N of rbf_solve_gji (an 8·32-row block grid)

template <typename T>
__device__ __forceinline__ double ldd(const T* p) {
  return (double)*p;
}

// fp64 Euclidean distance between nodes i and j (pdist / cdist 'euclidean').
__device__ __forceinline__ double dist64(double xi, double yi, double xj, double yj) {
  const double dx = xi - xj, dy = yi - yj;
  return sqrt(dx * dx + dy * dy);
}

// The correctly rounded fp64 sqrt for 0 <= s < 2^767 (squared distances of nodes in [-1, 1]²: never denormal): LLVM's
// own expansion of sqrt() (v_rsq_f64 seed, two Newton-Goldschmidt steps, the final residual correction) without its
// scaling for s < 2^-767 and its inf/NaN fixup, s = 0 selected directly — the same bits in 13 instead of 18 VALU ops.
// (r06: the left-looking Cholesky evaluates ≈ 1.5·N² distances per pixel.)
__device__ __forceinline__ double sqrt_pos(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  double g = s * y, h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, s);
  g = fma(d, h, g);
  d = fma(-g, g, s);
  g = fma(d, h, g);
  return s == 0.0 ? 0.0 : g;
}
__device__ __forceinline__ double dist64_pos(double xi, double yi, double xj, double yj) {
  const double dx = xi - xj, dy = yi - yj;
  return sqrt_pos(dx * dx + dy * dy);
}

// ‖·‖ for the evaluation sweep: the fp64 rsq approximation and one Newton step,
// d = s·r + (s − (s·r)²)·r/2 — 8 issue slots against ≈ 17 for the correctly rounded fp64 sqrt.
// (The fp32 rsq seed with conversions and a clamp ran at the same speed on MI355X, 229.6 vs 230.4 ms
// for N = 200, with 4× the error against SciPy: 1.8e-11 vs 4.3e-12 of max(|f|, 255).)  The solve
// itself (A and the refinement residuals) keeps the correctly rounded sqrt.
__device__ __forceinline__ double norm_eval_pos(double s) {  // s > 0
  const double r = __builtin_amdgcn_rsq(s);
  const double d0 = s * r;
  return fma(fma(-d0, d0, s), 0.5 * r, d0);
}
__device__ __forceinline__ double norm_eval(double s) { return norm_eval_pos(fmax(s, 1e-300)); }

__device__ __forceinline__ double dist_eval(double qu, double qv, double xj, double yj) {
  const double dx = qu - xj, dy = qv - yj;
  return norm_eval(fma(dy, dy, dx * dx));
}


typedef double dx4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double readlane64(double x, int l) {
  const uint64_t u = __double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// ---- Register-blocked Gauss-Jordan inverse + fp64 refinement (N ≤ 256) ---------------------------
// A of distinct nodes is symmetric and strictly conditionally negative definite (negative definite
// on 1^⊥).  With the Householder reflector H that maps e = 1/√N onto the last unit vector,
// HAH = [M m; mᵀ μ] has S = −M symmetric positive definite of order n = N − 1, and A w = b is solved
// by block elimination of the bordered system:
//   c = H b,  z1 = S⁻¹ c₁,  z2 = S⁻¹ m,  y_n = (c_n + mᵀz1)/(μ + mᵀz2),  y₁ = −z1 + z2·y_n,  w = H y.
// S is INVERTED in fp32 by in-place Gauss-Jordan without pivoting (stable on SPD matrices: every
// pivot is a positive Schur complement) and the inverse never leaves the registers: an NB×NB grid of
// threads (NB = 16 for N ≤ 128, 32 for N ≤ 256) each holds one 8×8 block of S in 64 VGPRs.  Step k:
// the threads owning row k and column k publish them to LDS (16 floats each, double-buffered, ONE
// barrier per step), every thread reads the 8 + 8 entries that meet its block and does a rank-1
// update of its 64 entries:
//     a_ij ← a_ij − a_ik·a_kj/a_kk,  a_ik ← −a_ik/a_kk,  a_kj ← a_kj/a_kk,  a_kk ← 1/a_kk
// (one FMA per entry: the pivot row and column are folded into the multipliers, see the step).
// LDS traffic is 64 B per thread and step, and no step is serial on one wave: the triangular
// substitutions of a factorization (N dependent steps, repeated every refinement sweep) become
// matrix-vector products with the explicit inverse, reduced across each block row in registers.
// The fp32 inverse is the approximate inverse of mixed-precision iterative refinement: residuals
// b − A·w in fp64 from the node coordinates (correctly rounded sqrt, so A is pdist's), corrections
// through the bordered system, until the fp64 floor — the weights are SciPy's fp64 LU solution to
// rounding.  It contracts the error by ≈1e-5 per sweep at cond(A) ≈ 1e4–1e5; at least 3 sweeps run
// (2 left 3e-10 of max(|f|, 255) against SciPy at N = 200, 3 give 2e-11, the fp64 floor).  Exactly
// repeated nodes (SciPy: LinAlgError) are detected up front, a non-positive pivot (cond beyond
// fp32) reports the same status.
constexpr int RBF_GJI_MAX_REFINE = 16;

// Lane reductions without address registers: DPP inside each row of 16 lanes (quad_perm 1032,
// quad_perm 2301, row_half_mirror, row_mirror leave the row's total in all 16 lanes) and
// ds_swizzle xor 16 across row pairs.  (__shfl_xor keeps a permute-address VGPR per offset alive
// across the whole kernel, which here pushed the 64-register S⁻¹ block into scratch.)
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double swz_xor16(double v) {  // bit mode: and 0x1F, or 0, xor 0x10
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_ds_swizzle((int)(uint32_t)u, 0x401F);
  const uint32_t hi = __builtin_amdgcn_ds_swizzle((int)(uint32_t)(u >> 32), 0x401F);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
template <bool MAX>
__device__ __forceinline__ double comb(double a, double b) { return MAX ? fmax(a, b) : a + b; }
template <bool MAX>
__device__ __forceinline__ double row16_reduce(double v) {
  v = comb<MAX>(v, dpp64<0xB1>(v));
  v = comb<MAX>(v, dpp64<0x4E>(v));
  v = comb<MAX>(v, dpp64<0x141>(v));
  return comb<MAX>(v, dpp64<0x140>(v));
}

template <int NB>
__device__ __forceinline__ double row_sum(double v) {  // over the NB lanes of one block row (its first lane)
  v = row16_reduce<false>(v);
  if constexpr (NB == 32) v += swz_xor16(v);
  return v;
}

template <int WAVES, bool MAX>
__device__ __forceinline__ double block_reduce(double v, double* red) {  // every thread gets the result
  v = row16_reduce<MAX>(v);
  v = comb<MAX>(v, swz_xor16(v));
  v = comb<MAX>(readlane64(v, 0), readlane64(v, 32));
  __syncthreads();  // the previous reduction's readers are done with red
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int i = 1; i < WAVES; ++i) r = comb<MAX>(r, red[i]);
  return r;
}

template <int NB, typename T>
__global__ void __launch_bounds__(NB * NB, NB <= 16 ? 2 : 4)
rbf_solve_gji(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
              double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status, int* __restrict__ redo,
              int max_refine) {
  constexpr int THREADS = NB * NB, WAVES = THREADS / 64, NV = 8 * NB;
  __shared__ double xs[NV], ys[NV], bv[NV], uv[NV], wv[NV], vv[NV], cv[NV], zv[NV], z2v[NV], mv[NV];
  __shared__ __attribute__((aligned(16))) float prow[2][NV], pcol[2][NV];
  __shared__ double red[WAVES];
  __shared__ int s_flag;
  const int t = threadIdx.x;
  const int bi = t / NB, bj = t % NB;
  const int i0 = 8 * bi, j0 = 8 * bj;
  const int n = N - 1;
  const int64_t p = blockIdx.x, base = p * N;
  const double e = 1.0 / sqrt((double)N), beta = 1.0 / (1.0 - e);  // H = I − β u uᵀ, u = e·1 − e_n
  auto u = [&](int j) __attribute__((always_inline)) { return j < n ? e : (j == n ? e - 1.0 : 0.0); };

  for (int j = t; j < NV; j += THREADS) {
    float x = 0.f, y = 0.f;
    double bb = 0.0;
    if (j < N) {
      x = lu[base + j], y = lv[base + j], bb = ldd(I + base + j);
      xyT[(int64_t)j * P + p] = make_float2(x, y);
    }
    xs[j] = (double)x, ys[j] = (double)y, bv[j] = bb, uv[j] = u(j);  // SciPy's float64 copies of the nodes
    wv[j] = vv[j] = cv[j] = zv[j] = z2v[j] = mv[j] = 0.0;  // entries past N take part in block products
    prow[0][j] = prow[1][j] = pcol[0][j] = pcol[1][j] = 0.f;
  }
  if (t == 0) s_flag = 0;
  __syncthreads();

  // out[r] = (A·x)[i0 + r] for x in LDS (zero past N): this thread's 8×8 block of A, reduced over the
  // block row (lanes bi·NB .. bi·NB + NB − 1).  Rows past N come out as garbage and are never used.
  // (two passes of 4 rows keep the live fp64 state small next to the 64-register S⁻¹ block)
  auto a_times = [&](const double* x, double (&out)[8], bool check) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 8; h += 4) {
      double o[4] = {0.0, 0.0, 0.0, 0.0};
      if (i0 < N && j0 < N) {
        float xi[4], yi[4];  // the nodes are fp32 values: exact in 32-bit registers
#pragma unroll
        for (int r = 0; r < 4; ++r)
          xi[r] = (float)xs[min(i0 + h + r, N - 1)], yi[r] = (float)ys[min(i0 + h + r, N - 1)];
#pragma unroll 1
        for (int c = 0; c < 8; ++c) {  // not unrolled: 32 fp64 sqrt chains in flight would evict S⁻¹
          const double xc = xs[j0 + c], yc = ys[j0 + c], xj = x[j0 + c];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o[r] = fma(dist64((double)xi[r], (double)yi[r], xc, yc), xj, o[r]);
            if (check && i0 + h + r < N && j0 + c < N && i0 + h + r != j0 + c && (double)xi[r] == xc &&
                (double)yi[r] == yc)
              s_flag = 1;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) out[h + r] = row_sum<NB>(o[r]);
    }
  };
  double part[8];
  a_times(uv, part, true);  // g = A u, and the repeated-node check
  if (bj == 0) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      if (i0 + r < N) vv[i0 + r] = part[r];
  }
  __syncthreads();
  const double sg = block_reduce<WAVES, false>(t < N ? u(t) * vv[t] : 0.0, red);  // uᵀAu
  const double b2 = beta * beta * sg;
  auto hah = [&](int i, int j) __attribute__((always_inline)) {
    return dist64(xs[i], ys[i], xs[j], ys[j]) - beta * (u(i) * vv[j] + vv[i] * u(j)) + b2 * u(i) * u(j);
  };
  float a[8][8];  // the thread's 8×8 block of S (rows i0.., columns j0..)
  const int nb = (n + 7) >> 3;
  const bool live = bi < nb && bj < nb;
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) a[r][c] = (live && i0 + r < n && j0 + c < n) ? (float)(-hah(i0 + r, j0 + c)) : 0.f;
  if (t <= n) mv[t] = hah(t, n);  // m, and μ at n
  bool singular = s_flag != 0;  // written before the reduction's barriers: block-uniform
  __syncthreads();

  // Step k = 8·kb + KR: KR is a compile-time constant (the step loop is unrolled by 8), so the pivot
  // row and column are fixed registers of the owning threads.
  bool lost = false;  // a non-positive pivot: cond(S) beyond fp32 (the pixel goes to rbf_solve_fp64)
  auto step = [&](auto KRc, int kb) __attribute__((always_inline)) {
    constexpr int KR = decltype(KRc)::value;
    const int k = 8 * kb + KR, buf = KR & 1;
    if (k >= n) return;  // uniform
    if (bi == kb) {  // publish row k (this thread's 8 columns of it)
      *reinterpret_cast<float4*>(&prow[buf][j0]) = make_float4(a[KR][0], a[KR][1], a[KR][2], a[KR][3]);
      *reinterpret_cast<float4*>(&prow[buf][j0 + 4]) = make_float4(a[KR][4], a[KR][5], a[KR][6], a[KR][7]);
    }
    if (bj == kb) {  // publish column k
      *reinterpret_cast<float4*>(&pcol[buf][i0]) = make_float4(a[0][KR], a[1][KR], a[2][KR], a[3][KR]);
      *reinterpret_cast<float4*>(&pcol[buf][i0 + 4]) = make_float4(a[4][KR], a[5][KR], a[6][KR], a[7][KR]);
    }
    __syncthreads();
    const float piv = pcol[buf][k];
    const bool bad = !(piv > 0.f);  // block-uniform (one LDS word after the barrier)
    lost |= bad;  // no early exit: a straight-line step keeps the block in registers
    const float inv = __builtin_amdgcn_rcpf(piv);  // an approximate inverse is all the refinement needs
    if (live && !bad) {
      const float4 r0 = *reinterpret_cast<const float4*>(&prow[buf][j0]);
      const float4 r1 = *reinterpret_cast<const float4*>(&prow[buf][j0 + 4]);
      const float4 c0 = *reinterpret_cast<const float4*>(&pcol[buf][i0]);
      const float4 c1 = *reinterpret_cast<const float4*>(&pcol[buf][i0 + 4]);
      const float pr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
      const float d[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      // One FMA pass does the whole step: with â_kk := 1 + 1/a_kk the pivot column comes out as
      // a_ik − a_ik(1 + 1/a_kk) = −a_ik/a_kk, and with the pivot row's multiplier a_kk − 1 the pivot
      // row comes out as a_kj − (a_kk − 1)·a_kj/a_kk = a_kj/a_kk (and 1/a_kk on the diagonal)
      float nrf[8], dm[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) nrf[c] = pr[c] * -inv;
      if (bj == kb) nrf[KR] = -(1.f + inv);
#pragma unroll
      for (int r = 0; r < 8; ++r) dm[r] = d[r];
      if (bi == kb) dm[KR] = d[KR] - 1.f;
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) a[r][c] = fmaf(dm[r], nrf[c], a[r][c]);
    }
  };
  using std::integral_constant;
  for (int kb = 0; kb < nb && !singular && !lost; ++kb) {
    // steps past n - 1 are skipped (uniform); the LDS buffers alternate with KR's parity, so two
    // consecutive steps never share one (the barrier of step k orders the reads of step k - 2)
    step(integral_constant<int, 0>(), kb);
    step(integral_constant<int, 1>(), kb);
    step(integral_constant<int, 2>(), kb);
    step(integral_constant<int, 3>(), kb);
    step(integral_constant<int, 4>(), kb);
    step(integral_constant<int, 5>(), kb);
    step(integral_constant<int, 6>(), kb);
    step(integral_constant<int, 7>(), kb);
  }

  double w_t = 0.0;
  bool conv = max_refine == 0;  // the refinement reached the fp64 floor (measurement runs without it)
  bool slow = false;
  if (!singular && !lost) {
    // dst[i0 + r] = (S⁻¹·x)[i0 + r] for x in LDS; entries of S⁻¹ past n are zero
    auto sinv_times = [&](const double* x, double* dst) __attribute__((always_inline)) {
      double out[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) out[r] = 0.0;
      if (live) {
        double xj[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) xj[c] = x[j0 + c];
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            // opaque to the optimizer: hoisting the 64 fp64 conversions out of the refinement loop
            // would need 128 live registers and spill S⁻¹ itself
            asm volatile("" : "+v"(a[r][c]));
            out[r] = fma((double)a[r][c], xj[c], out[r]);
          }
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) out[r] = row_sum<NB>(out[r]);
      if (bj == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (i0 + r < n) dst[i0 + r] = out[r];
      }
      __syncthreads();
    };
    sinv_times(mv, z2v);  // z2 = S⁻¹ m
    const double mu = mv[n];
    const double mz2 = block_reduce<WAVES, false>(t < n ? mv[t] * z2v[t] : 0.0, red);
    // A⁻¹ r for r in LDS, through the bordered Householder system; thread t returns entry t (< N)
    auto solve = [&](const double* rv) __attribute__((always_inline)) {
      const double ub = block_reduce<WAVES, false>(t < N ? u(t) * rv[t] : 0.0, red);
      if (t < N) cv[t] = fma(-beta * u(t), ub, rv[t]);  // c = H r
      __syncthreads();
      const double cn = cv[n];
      sinv_times(cv, zv);  // z1 = S⁻¹ c₁ (entries of S⁻¹ in column n are zero, so c_n drops out)
      const double mz1 = block_reduce<WAVES, false>(t < n ? mv[t] * zv[t] : 0.0, red);
      const double yn = (cn + mz1) / (mu + mz2);
      const double y = t < n ? fma(z2v[t], yn, -zv[t]) : (t == n ? yn : 0.0);
      const double uy = block_reduce<WAVES, false>(t < N ? u(t) * y : 0.0, red);
      return fma(-beta * u(t), uy, y);  // w = H y
    };
    w_t = solve(bv);
    if (t < N) wv[t] = w_t;
    double dprev = __builtin_inf();
    const int sweeps = max_refine < 0 ? -max_refine : max_refine;  // < 0: exactly that many (measurement)
    for (int it = 0; it < sweeps; ++it) {
      __syncthreads();
      a_times(wv, part, false);  // v = b − A w in fp64
      if (bj == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (i0 + r < N) vv[i0 + r] = bv[i0 + r] - part[r];
      }
      __syncthreads();
      const double dv = solve(vv);
      double dn = 0.0, wn = 0.0;
      if (t < N) {
        w_t += dv;
        wv[t] = w_t;
        dn = fabs(dv), wn = fabs(w_t);
      }
      dn = block_reduce<WAVES, true>(dn, red);
      wn = block_reduce<WAVES, true>(wn, red);
      // remaining error ≈ ρ·dn with ρ = dn / dprev the observed contraction (rbf_solve_lds's rule)
      const bool more =
          dn > 1e-16 * wn && dn < 0.5 * dprev && (dprev == __builtin_inf() || (dn / dprev) * dn > 4e-13 * wn);
      // converged: the last correction is at most 1e-10 of the weights (≈1e-16 at cond 1e4–1e5) and no
      // sweep above the fp64 floor contracted by less than 4× (error ≈ dn·ρ/(1 − ρ): at ρ → 1 small
      // corrections hide large errors).  An fp32 inverse of cond ≳ 1e7 contracts slowly, stalls or
      // diverges instead, and such pixels are solved again in fp64.
      if (dprev != __builtin_inf() && dn > 1e-14 * wn && dn > 0.25 * dprev) slow = true;
      dprev = dn;
      conv = dn <= 1e-10 * wn && !slow;
      if (!more && it >= 2 && max_refine >= 0) break;  // uniform: every thread computed the same reductions
    }
  }
  if (singular && t == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
  const bool again = !singular && (lost || !conv);  // block-uniform
  if (again && t == 0) redo[1 + atomicAdd(redo, 1)] = (int)p;  // the fp64 fallback's list
  if (t < N) wT[(int64_t)t * P + p] = (singular || again) ? __builtin_nan("") : w_t;
}

// Lower-triangle form (the kernel below): the in-place Gauss-Jordan sweep keeps the matrix symmetric up to
// sign — after steps 0..k−1, a_ij = a_ji when i and j are both swept or both not, a_ij = −a_ji when
// exactly one is — so only the blocks (bi, bj) with bj ≤ bi are held (diagonal blocks whole), one
// thread per block: nb(nb+1)/2 threads for nb = ⌈n/8⌉ (325 at N = 200 against 625 for the full grid).
// Step k needs only the column v = a_·k: rows ≥ 8⌊k/8⌋ come from the block column ⌊k/8⌋, rows above
// it from block row ⌊k/8⌋ as −a_kx (k unswept, x swept), and row k is a_kj = ±v_j (− for j < k).
// Products with the symmetric S⁻¹ and A use each off-diagonal block twice (its rows and, transposed,
// its columns); the partial sums land in an LDS table P[column block][row], every (block, row) slot
// written exactly once, and each row adds its slots in a fixed order (deterministic).
// 8 waves, 512 blocks: ⌈N/8⌉ ≤ 31 block rows of A, N ≤ 248, with the 256-VGPR budget of 2 waves per
// SIMD (no spills).  N ≤ 128 and N = 249..256 take rbf_solve_gji's full grid (for N ≤ 128 its
// 256-thread workgroups, four per CU, beat this kernel's: 20–24 vs 31 ms at N = 100).
template <int NB>
struct GjsShape {
  static constexpr int NV = 8 * NB;                              // vector capacity
  static constexpr int BLOCKS = NB * (NB + 1) / 2;
  static constexpr int THREADS = BLOCKS > 512 ? 512 : (BLOCKS + 63) / 64 * 64;
  static constexpr int WAVES = THREADS / 64;
  static constexpr int MIN_WAVES = 2;                            // VGPR cap 256 (no spills)
  static constexpr int MAX_N = NB <= 16 ? 128 : 248;
};

template <int NB, typename T>
__global__ void __launch_bounds__(GjsShape<NB>::THREADS, GjsShape<NB>::MIN_WAVES)
rbf_solve_gjs(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
              double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status, int* __restrict__ redo,
              int max_refine) {
  using SH = GjsShape<NB>;
  constexpr int THREADS = SH::THREADS, WAVES = SH::WAVES, NV = SH::NV;
  __shared__ double xs[NV], ys[NV], bv[NV], uv[NV], wv[NV], vv[NV], cv[NV], zv[NV], z2v[NV], mv[NV];
  __shared__ double Pt[NB][NV];  // partial products: Pt[column block][row]
  __shared__ __attribute__((aligned(16))) float vcol[2][NV];
  __shared__ double red[WAVES];
  __shared__ int s_flag;
  const int t = threadIdx.x;
  int bi = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);  // t = bi(bi+1)/2 + bj, bj <= bi
  if ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
  if (bi * (bi + 1) / 2 > t) --bi;
  const int bj = t - bi * (bi + 1) / 2;
  const int i0 = 8 * bi, j0 = 8 * bj;
  const bool diag = bi == bj;
  const int n = N - 1;
  const int nb = (n + 7) >> 3, nbA = (N + 7) >> 3;        // block rows of S and of A
  const bool liveS = t < nb * (nb + 1) / 2, liveA = t < nbA * (nbA + 1) / 2;
  const int64_t p = blockIdx.x, base = p * N;
  const double e = 1.0 / sqrt((double)N), beta = 1.0 / (1.0 - e);  // H = I − β u uᵀ, u = e·1 − e_n
  auto u = [&](int j) __attribute__((always_inline)) { return j < n ? e : (j == n ? e - 1.0 : 0.0); };

  for (int j = t; j < NV; j += THREADS) {
    float x = 0.f, y = 0.f;
    double bb = 0.0;
    if (j < N) {
      x = lu[base + j], y = lv[base + j], bb = ldd(I + base + j);
      xyT[(int64_t)j * P + p] = make_float2(x, y);
    }
    xs[j] = (double)x, ys[j] = (double)y, bv[j] = bb, uv[j] = u(j);  // SciPy's float64 copies of the nodes
    wv[j] = vv[j] = cv[j] = zv[j] = z2v[j] = mv[j] = 0.0;  // entries past N take part in block products
    vcol[0][j] = vcol[1][j] = 0.f;
  }
  if (t == 0) s_flag = 0;
  __syncthreads();

  // dst[x] = Σ_y M_xy src[y] for symmetric M given by this thread's lower block (element (r, c) =
  // elem(r, c), rows i0.., columns j0..), for x < len; src zero past its length.  Ends with a barrier.
  // REG: elem reads the register block (columns unrolled: compile-time indices); otherwise elem
  // computes A's entries (columns not unrolled: 32 fp64 sqrt chains in flight would evict S⁻¹).
  auto sym_times = [&](const double* src, double* dst, int len, bool live, auto elem, auto REG)
                       __attribute__((always_inline)) {
    if (live) {
#pragma unroll
      for (int h = 0; h < 8; h += 4) {  // two passes of 4 rows: little fp64 state next to the S⁻¹ block
        double xr[4], rp[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) xr[r] = src[i0 + h + r], rp[r] = 0.0;
        auto col = [&](int c) __attribute__((always_inline)) {
          const double xc = src[j0 + c];
          double cc = 0.0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double m = elem(h + r, c);
            rp[r] = fma(m, xc, rp[r]);
            cc = fma(m, xr[r], cc);
          }
          if (!diag) Pt[bi][j0 + c] = h ? Pt[bi][j0 + c] + cc : cc;  // this thread's slot
        };
        if constexpr (decltype(REG)::value) {
#pragma unroll
          for (int c = 0; c < 8; ++c) col(c);
        } else {
#pragma unroll 1
          for (int c = 0; c < 8; ++c) col(c);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Pt[bj][i0 + h + r] = rp[r];
      }
    }
    __syncthreads();
    const int nbl = (len + 7) >> 3;
    for (int x = t; x < len; x += THREADS) {
      double sacc = 0.0;
      for (int cb = 0; cb < nbl; ++cb) sacc += Pt[cb][x];
      dst[x] = sacc;
    }
    __syncthreads();
  };
  // A's entries from the node coordinates (correctly rounded fp64 sqrt: pdist's values)
  auto a_elem = [&](int r, int c) __attribute__((always_inline)) {
    return dist64(xs[i0 + r], ys[i0 + r], xs[j0 + c], ys[j0 + c]);
  };
  if (liveA) {  // repeated nodes: A singular (SciPy: LinAlgError)
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (i0 + r < N && j0 + c < N && i0 + r != j0 + c && xs[i0 + r] == xs[j0 + c] && ys[i0 + r] == ys[j0 + c])
          s_flag = 1;
  }
  sym_times(uv, vv, N, liveA, a_elem, std::false_type());  // g = A u
  const double sg = block_reduce<WAVES, false>(t < N ? u(t) * vv[t] : 0.0, red);  // uᵀAu
  const double b2 = beta * beta * sg;
  auto hah = [&](int i, int j) __attribute__((always_inline)) {
    return dist64(xs[i], ys[i], xs[j], ys[j]) - beta * (u(i) * vv[j] + vv[i] * u(j)) + b2 * u(i) * u(j);
  };
  float a[8][8];  // this thread's lower block of S
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) a[r][c] = (liveS && i0 + r < n && j0 + c < n) ? (float)(-hah(i0 + r, j0 + c)) : 0.f;
  if (t <= n) mv[t] = hah(t, n);  // m, and μ at n
  bool singular = s_flag != 0;  // set before the reduction's barriers: block-uniform
  __syncthreads();

  // Step k = 8·kb + KR (KR compile-time: the loop is unrolled by 8, so the pivot row/column is a fixed
  // register set of its owners).  vcol alternates with KR's parity; the barrier of step k orders the
  // reads of step k − 2.
  bool lost = false;  // a non-positive pivot: cond(S) beyond fp32 (the pixel goes to rbf_solve_fp64)
  auto step = [&](auto KRc, int kb) __attribute__((always_inline)) {
    constexpr int KR = decltype(KRc)::value;
    const int k = 8 * kb + KR;
    if (k >= n) return;  // uniform
    float* v = vcol[KR & 1];
    if (liveS && bi == kb && !diag) {  // rows x < 8kb of column k: −a_kx (row KR of block (kb, bj))
      *reinterpret_cast<float4*>(&v[j0]) = make_float4(-a[KR][0], -a[KR][1], -a[KR][2], -a[KR][3]);
      *reinterpret_cast<float4*>(&v[j0 + 4]) = make_float4(-a[KR][4], -a[KR][5], -a[KR][6], -a[KR][7]);
    }
    if (liveS && bj == kb) {  // rows x >= 8kb: column KR of block (bi, kb), the diagonal block whole
      *reinterpret_cast<float4*>(&v[i0]) = make_float4(a[0][KR], a[1][KR], a[2][KR], a[3][KR]);
      *reinterpret_cast<float4*>(&v[i0 + 4]) = make_float4(a[4][KR], a[5][KR], a[6][KR], a[7][KR]);
    }
    __syncthreads();
    const float piv = v[k];
    const bool bad = !(piv > 0.f);  // block-uniform (one LDS word after the barrier)
    lost |= bad;  // no early exit: a straight-line step keeps the block in registers
    // an approximate reciprocal is enough: the inverse only has to be a good approximate inverse
    const float inv = __builtin_amdgcn_rcpf(piv);
    if (liveS && !bad) {
      const float4 q0 = *reinterpret_cast<const float4*>(&v[j0]);
      const float4 q1 = *reinterpret_cast<const float4*>(&v[j0 + 4]);
      const float4 c0 = *reinterpret_cast<const float4*>(&v[i0]);
      const float4 c1 = *reinterpret_cast<const float4*>(&v[i0 + 4]);
      const float vj[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
      const float vi[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      // one FMA pass: row k is a_kj = ±v_j (− where j is swept: j < k), and with â_kk := 1 + 1/a_kk and
      // the pivot row's multiplier a_kk − 1 the pivot column and row come out as −a_ik/a_kk and
      // a_kj/a_kk.  j < k is bj ≤ kb for the columns c < KR of a block and bj < kb for c ≥ KR, so the
      // signs cost two selects per step; the FMA takes the negated row factor.
      const float nlo = bj <= kb ? inv : -inv, nhi = bj < kb ? inv : -inv;  // −(sign · 1/a_kk)
      float nrf[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) nrf[c] = vj[c] * (c < KR ? nlo : nhi);
      if (bj == kb) nrf[KR] = -(1.f + inv);
      float dm[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) dm[r] = vi[r];
      if (bi == kb) dm[KR] = vi[KR] - 1.f;
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) a[r][c] = fmaf(dm[r], nrf[c], a[r][c]);
    }
  };
  using std::integral_constant;
  for (int kb = 0; kb < nb && !singular && !lost; ++kb) {
    step(integral_constant<int, 0>(), kb);
    step(integral_constant<int, 1>(), kb);
    step(integral_constant<int, 2>(), kb);
    step(integral_constant<int, 3>(), kb);
    step(integral_constant<int, 4>(), kb);
    step(integral_constant<int, 5>(), kb);
    step(integral_constant<int, 6>(), kb);
    step(integral_constant<int, 7>(), kb);
  }

  double w_t = 0.0;
  bool conv = max_refine == 0;  // the refinement reached the fp64 floor (measurement runs without it)
  bool slow = false;
  if (!singular && !lost) {
    // S⁻¹ (all of 0..n−1 swept: symmetric again); the asm makes each entry opaque so the 64 fp64
    // conversions are not hoisted out of the refinement loop (128 live registers would spill S⁻¹)
    auto s_elem = [&](int r, int c) __attribute__((always_inline)) {
      float x = a[r][c];
      asm volatile("" : "+v"(x));
      return (double)x;
    };
    sym_times(mv, z2v, n, liveS, s_elem, std::true_type());  // z2 = S⁻¹ m (μ at n meets a zero column)
    const double mu = mv[n];
    const double mz2 = block_reduce<WAVES, false>(t < n ? mv[t] * z2v[t] : 0.0, red);
    // A⁻¹ r for r in LDS, through the bordered Householder system; thread t returns entry t (< N)
    auto solve = [&](const double* rv) __attribute__((always_inline)) {
      const double ub = block_reduce<WAVES, false>(t < N ? u(t) * rv[t] : 0.0, red);
      if (t < N) cv[t] = fma(-beta * u(t), ub, rv[t]);  // c = H r
      __syncthreads();
      const double cn = cv[n];
      sym_times(cv, zv, n, liveS, s_elem, std::true_type());  // z1 = S⁻¹ c₁ (c_n meets S⁻¹'s zero column n)
      const double mz1 = block_reduce<WAVES, false>(t < n ? mv[t] * zv[t] : 0.0, red);
      const double yn = (cn + mz1) / (mu + mz2);
      const double y = t < n ? fma(z2v[t], yn, -zv[t]) : (t == n ? yn : 0.0);
      const double uy = block_reduce<WAVES, false>(t < N ? u(t) * y : 0.0, red);
      return fma(-beta * u(t), uy, y);  // w = H y
    };
    w_t = solve(bv);
    if (t < N) wv[t] = w_t;
    __syncthreads();
    double dprev = __builtin_inf();
    const int sweeps = max_refine < 0 ? -max_refine : max_refine;  // < 0: exactly that many (measurement)
    for (int it = 0; it < sweeps; ++it) {
      sym_times(wv, vv, N, liveA, a_elem, std::false_type());  // A w in fp64
      if (t < N) vv[t] = bv[t] - vv[t];
      __syncthreads();
      const double dv = solve(vv);
      double dn = 0.0, wn = 0.0;
      if (t < N) {
        w_t += dv;
        wv[t] = w_t;
        dn = fabs(dv), wn = fabs(w_t);
      }
      dn = block_reduce<WAVES, true>(dn, red);
      wn = block_reduce<WAVES, true>(wn, red);
      // remaining error ≈ ρ·dn with ρ = dn / dprev the observed contraction; at least 3 sweeps
      const bool more =
          dn > 1e-16 * wn && dn < 0.5 * dprev && (dprev == __builtin_inf() || (dn / dprev) * dn > 4e-13 * wn);
      // converged: the last correction is at most 1e-10 of the weights (≈1e-16 at cond 1e4–1e5) and no
      // sweep above the fp64 floor contracted by less than 4× (error ≈ dn·ρ/(1 − ρ): at ρ → 1 small
      // corrections hide large errors).  An fp32 inverse of cond ≳ 1e7 contracts slowly, stalls or
      // diverges instead, and such pixels are solved again in fp64.
      if (dprev != __builtin_inf() && dn > 1e-14 * wn && dn > 0.25 * dprev) slow = true;
      dprev = dn;
      conv = dn <= 1e-10 * wn && !slow;
      if (!more && it >= 2 && max_refine >= 0) break;  // uniform: every thread computed the same reductions
    }
  }
  if (singular && t == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
  const bool again = !singular && (lost || !conv);  // block-uniform
  if (again && t == 0) redo[1 + atomicAdd(redo, 1)] = (int)p;  // the fp64 fallback's list
  if (t < N) wT[(int64_t)t * P + p] = (singular || again) ? __builtin_nan("") : w_t;
}

// Wave-wide max of a u32 key: DPP within each row of 16 lanes, then the four row maxima
// through readlane (scalar).  No LDS round trips on the pivot search's critical path.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const uint32_t r2 = __builtin_amdgcn_readlane(v, 47), r3 = __builtin_amdgcn_readlane(v, 63);
  return max(max(r0, r1), max(r2, r3));
}

// Per-pixel solve for N ≤ NMAX ≤ 80: Gauss-Jordan elimination with partial pivoting in
// fp64 registers (what SciPy's gesv computes, to rounding: cond·eps ≈ 1e-12 relative).
//
// One workgroup per pixel, one thread per row: thread t holds row t of [A | b] in
// registers, a[0..NMAX) fp64.  After step k every row shifts left by one, so the column
// being eliminated is always a[0] and every register index is a compile-time constant;
// the live width N − k shrinks, and the step body is instantiated for widths NMAX,
// NMAX − 8, …, 8 (phases) so the work follows the triangle.  Gauss-Jordan also
// eliminates above the pivot — free here, since every row is updated in lock-step anyway
// — which leaves the system diagonal: x at node k is b[p_k] / pivot_k, with no L or U
// storage and no substitution passes.
//
// Pivot search: key = (float bits of |a_t0| with the low 7 bits replaced by 127 − t),
// reduced across the wave with DPP; ties and near-ties (2⁻¹⁶ relative) go to the lower
// row.  Each wave stages its candidate row in LDS, one barrier, and every thread reads
// the winner's row with broadcast loads.
template <int NMAX, typename T>
struct GjSolve {
  static constexpr int WAVES = NMAX <= 64 ? 1 : 2;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int LDR = NMAX + 2;  // staged row: a[1..], b at [NMAX], 16-byte aligned pitch

  struct Smem {
    double xs[NMAX], ys[NMAX];
    __attribute__((aligned(16))) double stage[2][WAVES][LDR];
    uint32_t key[2][WAVES];
  };

  // One elimination step at static width WS (N − k ≤ WS).
  template <int WS>
  static __device__ __forceinline__ bool step(Smem& sm, double (&a)[NMAX], double& b, bool& used, int& my_step,
                                              double& my_d, int k, int t, int wave) {
    uint32_t key = 0;
    if (!used) key = (__float_as_uint((float)fabs(a[0])) & ~127u) | (uint32_t)(127 - t);
    key = wave_max_u32(key);
    const int buf = k & 1;
    if (t == 127 - (int)(key & 127u) && (key >> 7)) {  // this wave's candidate row → LDS
      double* r = sm.stage[buf][wave];
#pragma unroll
      for (int s = 1; s < WS; ++s) r[s - 1] = a[s];
      r[NMAX] = b;
      r[NMAX + 1] = a[0];
    }
    if ((t & 63) == 0) sm.key[buf][wave] = key;
    __syncthreads();
    uint32_t best = sm.key[buf][0];
    int win = 0;
    if constexpr (WAVES == 2) {
      const uint32_t k1 = sm.key[buf][1];
      if (k1 > best) best = k1, win = 1;
    }
    if (!(best >> 7)) return false;  // exactly zero pivot column: singular
    const int pr = 127 - (int)(best & 127u);
    const double* r = sm.stage[buf][win];
    const double piv = r[NMAX + 1];
    const bool me = t == pr;
    const double l = me ? 0.0 : a[0] * (1.0 / piv);
    if (me) used = true, my_step = k, my_d = piv;
#pragma unroll
    for (int s = 1; s < WS; ++s) a[s - 1] = fma(-l, r[s - 1], a[s]);
    b = fma(-l, r[NMAX], b);
    return true;
  }

  template <int WS>
  static __device__ __forceinline__ bool phases(Smem& sm, double (&a)[NMAX], double& b, bool& used, int& my_step,
                                                double& my_d, int& k, int N, int t, int wave) {
    for (; k < N && N - k > WS - 8; ++k)
      if (!step<WS>(sm, a, b, used, my_step, my_d, k, t, wave)) return false;
    if constexpr (WS > 8) return phases<WS - 8>(sm, a, b, used, my_step, my_d, k, N, t, wave);
    return true;
  }
};

template <int NMAX, typename T>
__global__ void __launch_bounds__(NMAX <= 64 ? 64 : 128)
rbf_solve_gj(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
             double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status) {
  using G = GjSolve<NMAX, T>;
  __shared__ typename G::Smem sm;
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t p = blockIdx.x;
  const int64_t base = p * N;
  if (t < N) {
    const float x = lu[base + t], y = lv[base + t];
    sm.xs[t] = (double)x;  // SciPy holds float64 copies of the float32 nodes
    sm.ys[t] = (double)y;
    xyT[(int64_t)t * P + p] = make_float2(x, y);
  }
  double b = t < N ? ldd(I + base + t) : 0.0;
  __syncthreads();
  double a[NMAX];
  {
    const int tc = min(t, N - 1);
    const double xi = sm.xs[tc], yi = sm.ys[tc];
#pragma unroll
    for (int j = 0; j < NMAX; ++j) a[j] = (j < N && t < N) ? dist64(xi, yi, sm.xs[min(j, N - 1)], sm.ys[min(j, N - 1)]) : 0.0;
  }
  bool used = t >= N;  // rows past N: zero, never pivots, never read
  int my_step = 0;
  double my_d = 1.0;
  int k = 0;
  const bool ok = G::template phases<NMAX>(sm, a, b, used, my_step, my_d, k, N, t, wave);
  if (!ok && t == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
  if (t < N) wT[(int64_t)(ok ? my_step : t) * P + p] = ok ? b / my_d : __builtin_nan("");
}

// f(q_e) = Σ_j w_j ‖q_e − x_j‖ for a 64-pixel tile × 4·TE queries per workgroup (TE = 20:
// a wave's queries then lie in one row of the reference's 100 × 100 grid and share (qv − y)²).  Lanes
// run over pixels (node tables are [N][P], so each load is one coalesced 512-byte row and
// eval-major stores are coalesced); each thread keeps TE accumulators, the queries are
// wave-uniform (scalar loads).  fp64 throughout; ‖·‖ via dist_eval.
template <int TE, typename TO, int OL>
__global__ void __launch_bounds__(256)
rbf_eval(const double* __restrict__ wT, const float2* __restrict__ xyT, int N, int64_t P,
         const double* __restrict__ luv, int E, TO* __restrict__ out, int64_t pbase) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int e0 = (blockIdx.x * 4 + wave) * TE;
  if (e0 >= E) return;  // wave-uniform
  const int64_t p = pbase + (int64_t)blockIdx.y * 64 + lane;
  const int64_t pc = p < P ? p : P - 1;
  double qu[TE], qv[TE], acc[TE];
#pragma unroll
  for (int i = 0; i < TE; ++i) {
    const int e = min(e0 + i, E - 1);
    qu[i] = luv[2 * e], qv[i] = luv[2 * e + 1], acc[i] = 0.0;
  }
  bool same_v = true;  // a grid row: every query of this wave shares qv, so (qv − y)² is shared
#pragma unroll
  for (int i = 1; i < TE; ++i) same_v = same_v && qv[i] == qv[0];
  if (same_v) {
    for (int j = 0; j < N; ++j) {
      const double w = wT[(int64_t)j * P + pc];
      const float2 xy = xyT[(int64_t)j * P + pc];
      // + 1e-300 keeps every s > 0 (rsq(0) = inf would make 0·inf = NaN at a query on a node) for one
      // add per node and row instead of a clamp per term: 8 issue slots per term instead of 9
      const double x = xy.x, dy = qv[0] - (double)xy.y, dy2 = fma(dy, dy, 1e-300);
#pragma unroll
      for (int i = 0; i < TE; ++i) {
        const double dx = qu[i] - x;
        acc[i] = fma(w, norm_eval_pos(fma(dx, dx, dy2)), acc[i]);
      }
    }
  } else {
    for (int j = 0; j < N; ++j) {
      const double w = wT[(int64_t)j * P + pc];
      const float2 xy = xyT[(int64_t)j * P + pc];
      const double x = xy.x, y = xy.y;
#pragma unroll
      for (int i = 0; i < TE; ++i) acc[i] = fma(w, dist_eval(qu[i], qv[i], x, y), acc[i]);
    }
  }
  if (p >= P) return;
#pragma unroll
  for (int i = 0; i < TE; ++i) {
    const int e = e0 + i;
    if (e < E) {
      if constexpr (OL == RTI_OUT_PIXEL_MAJOR)
        out[p * E + e] = cvt_out<TO>(acc[i]);
      else
        out[(int64_t)e * P + p] = cvt_out<TO>(acc[i]);
    }
  }
}

// ---- fp64 fallback for the pixels the fp32 inverse cannot take ------------------------------------
// rbf_solve_gji / rbf_solve_gjs list a pixel (redo[0] = count, redo[1 ..] = pixels) when a Gauss-Jordan
// pivot of S is not positive in fp32 or the refinement does not reach the fp64 floor — cond(A) ≳ 1e8:
// nearly repeated light directions.  With per-pixel directions that happens wherever the line through two
// light positions meets the ROI plane (the two directions coincide there), so a few pixels of a real
// capture need it (c8: 8 of 160 000) and SciPy's fp64 LU still returns a solution for them.  This kernel
// solves exactly those pixels the way SciPy does: fp64 Gauss-Jordan with partial pivoting on [A | b], rows
// never swapped (a used-row mask; the pivot of step k is the largest |a_ik| among unused rows, ties to the
// lower row), the system left diagonal, w at node k = b_p / a_pk of step k's pivot row p.  The listed pixels
// are spread over the grid (workgroup b takes list entries b, b + G, ...: one pixel per CU for a handful of
// them), and [A | b] lives in LDS up to N = RBF_FB_LDS_N (else in a per-workgroup global slot), eliminated
// by a 16 × 16 thread grid (rows × columns).  A launch with an empty list reads one int.
constexpr int RBF_FB_THREADS = 256;
constexpr size_t RBF_FB_LDS = 152 * 1024;  // dynamic LDS for [A | b] (the static part is ≈ 7.3 KiB)
__host__ __device__ constexpr bool fb_in_lds(int N) { return (size_t)N * (N + 1) * sizeof(double) <= RBF_FB_LDS; }
constexpr int RBF_FB_LDS_N = 138;
static_assert(fb_in_lds(RBF_FB_LDS_N) && !fb_in_lds(RBF_FB_LDS_N + 1), "RBF_FB_LDS_N");

template <typename T, bool LDSM>
__global__ void __launch_bounds__(RBF_FB_THREADS)
rbf_solve_fp64(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
               const int* __restrict__ list, double* __restrict__ ws, double* __restrict__ wT,
               int* __restrict__ status, int* __restrict__ fallback_px) {
  extern __shared__ double ldsM[];
  __shared__ double xs[RBF_MAX_N], ys[RBF_MAX_N], lf[RBF_MAX_N];
  __shared__ int used[RBF_MAX_N];
  __shared__ double s_val[RBF_FB_THREADS / 64];
  __shared__ int s_row[RBF_FB_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, tx = t & 15, ty = t >> 4;
  const int ld = N + 1;
  double* M = LDSM ? ldsM : ws + (int64_t)blockIdx.x * N * ld;  // [N][N + 1]: A | b
  const int count = list[0];
  if (blockIdx.x == 0 && t == 0 && count > 0 && fallback_px) atomicAdd(fallback_px, count);  // (rti_rbf_perpixel_ex)
  for (int li = blockIdx.x; li < count; li += gridDim.x) {
    const int64_t p = list[1 + li];
    const int64_t base = p * N;
    for (int j = t; j < N; j += RBF_FB_THREADS) xs[j] = (double)lu[base + j], ys[j] = (double)lv[base + j], used[j] = 0;
    __syncthreads();
    for (int idx = t; idx < N * ld; idx += RBF_FB_THREADS) {
      const int i = idx / ld, j = idx - i * ld;
      M[idx] = j < N ? dist64(xs[i], ys[i], xs[j], ys[j]) : ldd(I + base + i);
    }
    __syncthreads();
    bool singular = false;
    for (int k = 0; k < N; ++k) {
      // pivot: the largest |a_ik| over unused rows (lower row on ties)
      double best = -1.0;
      int row = N;
      for (int i = t; i < N; i += RBF_FB_THREADS)
        if (!used[i]) {
          const double v = fabs(M[(int64_t)i * ld + k]);
          if (v > best) best = v, row = i;
        }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int orow = __shfl_xor(row, off);
        if (ob > best || (ob == best && orow < row)) best = ob, row = orow;
      }
      if (lane == 0) s_val[wave] = best, s_row[wave] = row;
      __syncthreads();
      best = s_val[0], row = s_row[0];
#pragma unroll
      for (int w = 1; w < RBF_FB_THREADS / 64; ++w)
        if (s_val[w] > best || (s_val[w] == best && s_row[w] < row)) best = s_val[w], row = s_row[w];
      if (!(best > 0.0)) {  // an exactly zero pivot column: singular (block-uniform)
        singular = true;
        break;
      }
      const double piv = M[(int64_t)row * ld + k];
      for (int i = t; i < N; i += RBF_FB_THREADS) lf[i] = i == row ? 0.0 : M[(int64_t)i * ld + k] / piv;
      __syncthreads();
      // eliminate column k from every other row (Gauss-Jordan): rows over ty, columns k+1 .. N over tx
      const double* prow = M + (int64_t)row * ld;
      for (int i = ty; i < N; i += RBF_FB_THREADS / 16) {
        if (i == row) continue;
        const double f = lf[i];
        double* mi = M + (int64_t)i * ld;
        for (int j = k + 1 + tx; j <= N; j += 16) mi[j] = fma(-f, prow[j], mi[j]);
      }
      if (t == 0) used[row] = k + 1;  // step of this pivot row, + 1
      __syncthreads();
    }
    if (singular) {
      if (t == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
      for (int j = t; j < N; j += RBF_FB_THREADS) wT[(int64_t)j * P + p] = __builtin_nan("");
    } else {
      for (int i = t; i < N; i += RBF_FB_THREADS) {  // row i pivoted step k = used[i] − 1: w_k = b_i / a_ik
        const int k = used[i] - 1;
        wT[(int64_t)k * P + p] = M[(int64_t)i * ld + N] / M[(int64_t)i * ld + k];
      }
    }
    __syncthreads();  // xs / used / M are reused by the next listed pixel
  }
}

// ---- Blocked fp64 Cholesky of the bordered system (N > 256; no cap) ------------------------------
// The register-blocked inverses stop at N = 256 (an 8·32-row grid of 8×8 fp32 blocks is the whole
// register file); the reference takes N = frames/8 lights (analysis.py:120,152), beyond 256 for any
// capture over ≈ 68 s.  For those N the same bordered system (see rbf_solve_gji:
// S = −(HAH)[:n, :n] symmetric positive definite, n = N − 1) is factored S = L Lᵀ in fp64 — SciPy's fp64
// accuracy without refinement — by a right-looking blocked Cholesky whose matrix lives in a per-workgroup
// slot of global memory (the lower triangle in packed rows, 4·ld² bytes; r04: the packed slot and a
// left-looking form that writes each L panel once were measured and neither moved the solve — c8n400 478 ms
// full or packed, 1384–1584 ms left-looking, DESIGN §4.3 — the panel loop is latency-bound, not slot-bound):
//   setup: A's row sums from every distance of a row (g = A u needs no column pass over a stored A), then
//   S written in one pass from the distances evaluated again (write-only);
//   per panel of NB columns: the panel rows [k0, n) are staged in LDS (a short last panel padded with the
//   identity, so the diagonal-block code runs without per-column guards), the NB×NB diagonal block is
//   factored in place in LDS by wave 0 (pivot inverse square roots by the fp64 rsq and two Newton steps,
//   1 / L[c][c] kept in the panel's pitch column), the rows below are solved against it (one thread per
//   row, multiplies by the stored reciprocals), the panel is written back, and the trailing lower
//   triangle is updated S[i][j] −= Σ_q L[i][q]·L[j][q] in 8×4 register tiles per lane whose old values
//   are loaded before the products;
// then L y = [c₁ | m] and Lᵀ z = y by blocked substitutions (diagonal blocks on wave 0, the off-diagonal
// products over the threads, each thread's first backward row loaded with the diagonal block), the bordered
// elimination gives y_n and w = H y.  One workgroup per CU strides over the pixels (its slot is reused
// pixel after pixel; 2 or 4 smaller workgroups per CU measured slower, their slots outgrow the MALL).  A
// non-positive fp64 pivot (nodes closer than fp64 can separate, or repeated ones) reports RTI_ERR_SINGULAR
// with NaN weights, where SciPy raises LinAlgError for repeated nodes.  Cost ≈ n³/3 fp64 FMAs per pixel
// (SciPy's LU: 2n³/3).
constexpr int RBF_CH_THREADS = 512;
constexpr size_t RBF_CH_LDS = 160 * 1024 - 256;  // dynamic LDS per workgroup (the static part is < 256 B)

// LDS of one workgroup: the panel [N][NB + 1] doubles (a bank shift per row), the two right-hand sides /
// solutions [2][N] doubles and the nodes [2][N] floats
__host__ __device__ constexpr size_t chol_lds_bytes(int N, int NB) { return (size_t)N * (8 * NB + 8 + 16 + 8); }
// widest panel whose LDS fits: 32 to N = 568, 16 to 1022, 8 to 1704, 4 to 2556, 2 to 3408, 1 to 4089
// (0: too many lights).  The narrow panels are slow (the trailing triangle is rewritten every NB columns:
// ≈ 16·n³/(6·NB) bytes of slot traffic per pixel) but keep the reference's uncapped N = frames/8 − failures
// (analysis.py:120,152) solvable to a 17-minute capture at 30 fps.
__host__ __device__ constexpr int chol_nb(int N) {
  return chol_lds_bytes(N, 32) <= RBF_CH_LDS ? 32
         : chol_lds_bytes(N, 16) <= RBF_CH_LDS ? 16
         : chol_lds_bytes(N, 8) <= RBF_CH_LDS ? 8
         : chol_lds_bytes(N, 4) <= RBF_CH_LDS ? 4
         : chol_lds_bytes(N, 2) <= RBF_CH_LDS ? 2
         : chol_lds_bytes(N, 1) <= RBF_CH_LDS ? 1 : 0;
}
constexpr int RBF_CH_MAX_N = 4089;
static_assert(chol_nb(568) == 32 && chol_nb(569) == 16 && chol_nb(2556) == 4 && chol_nb(2557) == 2 &&
                  chol_nb(RBF_CH_MAX_N) == 1 && chol_nb(RBF_CH_MAX_N + 1) == 0, "RBF_CH_MAX_N");

__host__ __device__ constexpr int chol_ld(int N) { return (N + 31) / 32 * 32; }
// per-workgroup slot in global memory: the lower triangle of M in packed rows + the vectors g (= A u), c, m
// ([ld] each)
__host__ __device__ constexpr int64_t chol_matrix_doubles(int N) {
  return ((int64_t)chol_ld(N) * (chol_ld(N) + 1) / 2 + 31) / 32 * 32;
}
__host__ __device__ constexpr int64_t chol_slot_doubles(int N) { return chol_matrix_doubles(N) + 3 * chol_ld(N); }
// GP form (N > RBF_CH_MAX_N): + y1, y2 and the nodes (two float rows) in the slot
__host__ __device__ constexpr int64_t chol_slot_doubles_gp(int N) { return chol_slot_doubles(N) + 3 * chol_ld(N); }
constexpr int RBF_CH_GP_NB = 32;  // GP panel width (only its diagonal block is in LDS)
constexpr int RBF_GP_MAX_N = 32768;  // a 4.3 GB slot per workgroup (the grid shrinks to fit gp_ws_budget)
constexpr size_t RBF_GP_WS_BYTES = (size_t)48 << 30;

// GP slot budget: at most RBF_GP_WS_BYTES, and at most 90 % of the device's free memory less the node-major
// weights and nodes (`other` bytes) allocated with the slots; RTI_RBF_GP_WS_BYTES (environment, read per call)
// lowers it (tests force a one-slot grid).  The grid is at least one slot whatever the budget.
size_t gp_ws_budget(size_t other) {
  size_t budget = RBF_GP_WS_BYTES;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
    const size_t usable = free_b / 10 * 9;
    budget = usable > other ? (usable - other < budget ? usable - other : budget) : 0;
  } else {
    (void)hipGetLastError();
  }
  if (const char* e = getenv("RTI_RBF_GP_WS_BYTES")) {
    const long long v = atoll(e);
    if (v >= 0 && (size_t)v < budget) budget = (size_t)v;
  }
  return budget;
}
thread_local int64_t rbf_last_chol_grid_v = 0;  // slots (= Cholesky workgroups) of the last rti_rbf_perpixel call

// Phase timer for tools/probe/chol_probe.hip (compiled in only there): per workgroup, the steady-clock
// ticks spent in each phase, summed over its pixels (a barrier closes every phase).
#ifdef RTI_CHOL_PROFILE
__device__ unsigned long long rti_chol_prof[1024][16];
#define CH_MARK(k)                                   \
  do {                                               \
    __syncthreads();                                 \
    if (t == 0) {                                    \
      const long long now_ = wall_clock64();         \
      prof_[k] += now_ - last_;                      \
      last_ = now_;                                  \
    }                                                \
  } while (0)
#else
#define CH_MARK(k) \
  do {             \
  } while (0)
#endif

// GP (N > RBF_CH_MAX_N, whose one-column panel no longer fits the LDS): the same algorithm with only the NB×NB
// diagonal block in LDS; the panel rows below it are read and solved in place in the slot's packed L (they ARE
// the panel), and the right-hand sides and nodes live in the slot too (chol_slot_doubles_gp).
// TH: threads per workgroup, one workgroup per CU (r05 measured 256-thread workgroups two per CU, NB = 16:
// 527 vs 441 ms at N = 400, profiles/r05m_chol_shape_sweep.log)
template <int NB, typename T, bool GP = false, int TH = RBF_CH_THREADS>
__global__ void __launch_bounds__(TH)
rbf_solve_chol(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
               double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status,
               double* __restrict__ ws) {
  static_assert(NB <= 32, "a wave solves both right-hand sides of a diagonal block (2·NB lanes)");
  constexpr int LDP = NB + 1;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = N - 1, ld = chol_ld(N);
  double* M = ws + (int64_t)blockIdx.x * (GP ? chol_slot_doubles_gp(N) : chol_slot_doubles(N));
  double* pan = smem;                                                       // [N][LDP] (GP: [NB][LDP])
  double* y1 = GP ? M + chol_slot_doubles(N) : pan + (size_t)N * LDP;      // c₁ -> L⁻¹c₁ -> S⁻¹c₁
  double* y2 = y1 + (GP ? ld : N);                                          // m  -> L⁻¹m  -> S⁻¹m
  float* xs = reinterpret_cast<float*>(y2 + (GP ? ld : N));
  float* ys = xs + (GP ? ld : N);
  __shared__ double red[TH / 64];
  __shared__ int s_bad;
  // the lower triangle in packed rows (row i at i(i+1)/2): 4·ld² bytes per slot
  auto at = [&](int i, int j) -> int64_t { return (int64_t)i * (i + 1) / 2 + j; };
  // element (r, c) of the panel at column k0: LDS, or (GP, rows below the diagonal block) the slot's L in place
  auto pan_at = [&](int k0, int r, int c) -> double& {
    return GP && r >= NB ? M[at(k0 + r, k0 + c)] : pan[r * LDP + c];
  };
  double* gv = M + chol_matrix_doubles(N);  // g = A u
  double* cv = gv + ld;               // c = H b
  double* mv = cv + ld;               // m = (HAH)[:n, n], μ at n
  const double e = 1.0 / sqrt((double)N), beta = 1.0 / (1.0 - e);  // H = I − β u uᵀ, u = e·1 − e_n
  auto u = [&](int j) { return j < n ? e : (j == n ? e - 1.0 : 0.0); };
  auto sum_all = [&](double v) {  // block-wide sum, every thread gets it
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();  // the previous sum's readers are done with red
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < TH / 64; ++i) r += red[i];
    return r;
  };
  auto dist = [&](int i, int j) { return dist64((double)xs[i], (double)ys[i], (double)xs[j], (double)ys[j]); };
#ifdef RTI_CHOL_PROFILE
  long long prof_[16] = {}, last_ = wall_clock64();
#endif
  // one diagonal block's two triangular solves on wave 0: lanes r and 32 + r hold row r's entries of the
  // two right-hand sides; L[r][c] at Ld[r·LDP + c], 1 / L[c][c] at Ld[c·LDP + NB] (the pitch column).
  // Forward: L z = s; backward: Lᵀ z = s.  Unrolled over NB so the block's LDS reads issue ahead of the
  // dependent chain; z_c reaches every lane by readlane (no LDS round trip per step).
  const int r32 = lane & 31;
  // (the block is padded to NB with the identity and rows >= kb start at 0, so the steps run unguarded)
  auto diag_fwd = [&](const double* Ld, int kb, double* ya, double* yb) {
    double v = r32 < kb ? (lane < 32 ? ya[r32] : yb[r32]) : 0.0;
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      const double l = Ld[r32 * LDP + c], rd = Ld[c * LDP + NB];
      if (r32 == c) v *= rd;
      const double z0 = readlane64(v, c), z1 = readlane64(v, 32 + c);
      if (r32 > c) v = fma(-l, lane < 32 ? z0 : z1, v);
    }
    if (r32 < kb) (lane < 32 ? ya : yb)[r32] = v;
  };
  auto diag_bwd = [&](const double* Ld, int kb, double* ya, double* yb) {
    double v = r32 < kb ? (lane < 32 ? ya[r32] : yb[r32]) : 0.0;
#pragma unroll
    for (int c = NB - 1; c >= 0; --c) {
      const double l = Ld[c * LDP + r32], rd = Ld[c * LDP + NB];
      if (r32 == c) v *= rd;
      const double z0 = readlane64(v, c), z1 = readlane64(v, 32 + c);
      if (r32 < c) v = fma(-l, lane < 32 ? z0 : z1, v);
    }
    if (r32 < kb) (lane < 32 ? ya : yb)[r32] = v;
  };

  for (int64_t p = blockIdx.x; p < P; p += gridDim.x) {
    const int64_t base = p * N;
    if (t == 0) s_bad = 0;
    for (int j = t; j < N; j += TH) {
      const float x = lu[base + j], y = lv[base + j];
      xs[j] = x, ys[j] = y;
      xyT[(int64_t)j * P + p] = make_float2(x, y);
      y1[j] = ldd(I + base + j);  // b (y1 holds b until c is formed)
    }
    __syncthreads();
    CH_MARK(0);
    // A's row sums (one wave per row; every distance of the row, so no column pass over a stored A) and the
    // repeated-node check (SciPy: LinAlgError); g = A u = e·(row sums) − A[:, n]
    bool dup = false;
    // (r05) SYMMETRIC form where its partial sums fit in the (still unused) panel LDS: each distance of the
    // lower triangle once, in 64×64 tiles (lane = column, rows in chunks of 8): the column partials stay in
    // registers, the row partials are transposed through a per-wave LDS slice; per tile they go to LDS and
    // every row's sum is added up in a fixed order (deterministic).  Diagonal tiles are computed whole (their
    // row partials cover both halves); A's lower triangle is stored coalesced on the way.
    const int T64r = (N + 63) / 64, ntl = T64r * (T64r + 1) / 2;
    const bool sym = !GP && (size_t)ntl * 1024 + (size_t)(TH / 64) * 8 * 64 * 8 <= (size_t)N * LDP * 8;
    if (sym) {
      double* rowp = pan;                         // [ntl][64]
      double* colp = rowp + (size_t)ntl * 64;     // [ntl][64]
      double* rbuf = colp + (size_t)ntl * 64 + wave * (8 * 64);  // [8][64] per wave
      for (int st = wave; st < ntl; st += TH / 64) {
        int tI = 0;
        while ((tI + 1) * (tI + 2) / 2 <= st) ++tI;
        const int tJ = st - tI * (tI + 1) / 2;
        const int j = 64 * tJ + lane;
        const bool jv = j < N;
        const double xj = (double)xs[jv ? j : 0], yj = (double)ys[jv ? j : 0];
        double cacc = 0.0;
        const int rows_t = min(64, N - 64 * tI);
        for (int m0 = 0; m0 < rows_t; m0 += 8) {
          double v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int i = 64 * tI + m0 + q;
            const bool iv = i < N;
            const double d = dist64((double)xs[iv ? i : 0], (double)ys[iv ? i : 0], xj, yj);
            const double dd = iv && jv ? d : 0.0;
            v[q] = dd;
            if (tI > tJ) cacc += dd;
            dup = dup || (iv && jv && j != i && d == 0.0);
            if (iv && jv && j <= i && i < n) M[at(i, j)] = d;  // raw A, turned into S on its first read
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) rbuf[q * 64 + lane] = v[q];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const int q = lane & 7, sg = lane >> 3;  // row q of the chunk, columns 8·sg .. 8·sg + 7
          double rsum = 0.0;
#pragma unroll
          for (int c = 0; c < 8; ++c) rsum += rbuf[q * 64 + 8 * sg + c];
          rsum += __shfl_xor(rsum, 8, 64);
          rsum += __shfl_xor(rsum, 16, 64);
          rsum += __shfl_xor(rsum, 32, 64);
          if (lane < 8) rowp[(size_t)st * 64 + m0 + q] = rsum;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the reads before the next chunk's writes
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (tI > tJ) colp[(size_t)st * 64 + lane] = cacc;
      }
      __syncthreads();
      for (int i = t; i < N; i += TH) {  // row i: its row-block's row partials, then the column partials below
        const int tI = i >> 6, r = i & 63;
        double rs = 0.0;
        for (int tJ = 0; tJ <= tI; ++tJ) rs += rowp[(size_t)(tI * (tI + 1) / 2 + tJ) * 64 + r];
        for (int I2 = tI + 1; I2 < T64r; ++I2) rs += colp[(size_t)(I2 * (I2 + 1) / 2 + tI) * 64 + r];
        gv[i] = fma(e, rs, -(i < n ? dist(n, i) : 0.0));
      }
    } else {
      // (r05) RB rows per wave at a time: RB independent sqrt chains and butterflies in flight, each column's node
      // read once per RB rows (the same rows per wave and the same order of additions per row: bit-identical)
      constexpr int RB = 4, WV = TH / 64;
      for (int i0 = wave; i0 < N; i0 += RB * WV) {
        double rs[RB], xi[RB], yi[RB];
  #pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int i = min(i0 + r * WV, N - 1);
          xi[r] = (double)xs[i], yi[r] = (double)ys[i], rs[r] = 0.0;
        }
        for (int j = lane; j < N; j += 64) {
          const double xj = (double)xs[j], yj = (double)ys[j];
  #pragma unroll
          for (int r = 0; r < RB; ++r) {
            const int i = i0 + r * WV;
            const double d = dist64(xi[r], yi[r], xj, yj);
            rs[r] += d;
            dup = dup || (i < N && j != i && d == 0.0);
            if (!GP && j <= i && i < n) M[at(i, j)] = d;  // raw A, turned into S on its first read
          }
        }
  #pragma unroll
        for (int off = 32; off >= 1; off >>= 1)
  #pragma unroll
          for (int r = 0; r < RB; ++r) rs[r] += __shfl_xor(rs[r], off, 64);
  #pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int i = i0 + r * WV;
          if (lane == 0 && i < N) gv[i] = fma(e, rs[r], -(i < n ? dist(n, i) : 0.0));
        }
      }
    }
    if (dup) s_bad = 1;
    __syncthreads();
    CH_MARK(1);
    CH_MARK(2);
    double ub = 0.0, ug = 0.0;
    for (int i = t; i < N; i += TH) ub = fma(u(i), y1[i], ub), ug = fma(u(i), gv[i], ug);
    const double utb = sum_all(ub), b2 = beta * beta * sum_all(ug);
    // HAH from the distances (i >= j)
    auto hah = [&](int i, int j, double d) { return d - beta * (u(i) * gv[j] + gv[i] * u(j)) + b2 * u(i) * u(j); };
    for (int i = t; i < N; i += TH) {
      const double ci = y1[i] - beta * u(i) * utb, mi = hah(n, i, i < n ? dist(n, i) : 0.0);
      cv[i] = ci, mv[i] = mi, y1[i] = ci, y2[i] = mi;
    }
    // S = −(HAH)[:n, :n]: (r05) M holds A's lower triangle from the row-sum pass, and the first panel's staging
    // and trailing update (which between them read every element once) apply S = −hah(A) as they load it, with
    // g copied into the LDS of the dead node coordinates — no second pass over the distances or over M.
    // (GP, whose panel rows are read in place: the old write-only pass, the distances again.)
    double* gl = reinterpret_cast<double*>(xs);  // [N] (xs, ys: 2N floats, dead from here on)
    if constexpr (GP) {
      for (int i = wave; i < n; i += TH / 64)
        for (int j = lane; j <= i; j += 64) M[at(i, j)] = -hah(i, j, dist(i, j));
    } else {
      __syncthreads();  // every dist(n, i) above has read xs / ys
      for (int i = t; i < N; i += TH) gl[i] = gv[i];
    }
    auto s_of = [&](int i, int j, double d) {  // hah's operations with g from LDS (bit-identical)
      return -(d - beta * (u(i) * gl[j] + gl[i] * u(j)) + b2 * u(i) * u(j));
    };
    __syncthreads();
    CH_MARK(3);

    // ---- blocked Cholesky S = L Lᵀ, with the forward substitutions L y = [c₁ | m] panel by panel --------
    for (int k0 = 0; k0 < n && !s_bad; k0 += NB) {  // s_bad: block-uniform after each sync
      auto PAN = [&](int r, int c) -> double& { return pan_at(k0, r, c); };
      const int kb = min(NB, n - k0), rows = n - k0;
      // stage the panel rows [k0, n), columns [k0, k0 + kb); a short last panel (kb < NB, then rows = kb) is
      // padded to NB rows and columns with the identity, so the diagonal block's code below runs unguarded
      {  // (GP: the rest is in place); SU loads in flight per thread (r05: one at a time was latency-bound)
        constexpr int SU = 8;
        const int tot = (GP ? NB : max(rows, NB)) * NB;
        for (int i0 = t; i0 < tot; i0 += SU * TH) {
          double v[SU];
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int idx = i0 + u * TH, r = idx / NB, c = idx - r * NB;
            v[u] = r == c && r >= kb ? 1.0 : 0.0;
            if (idx < tot && c < kb && c <= r && r < rows) v[u] = M[at(k0 + r, k0 + c)];
          }
          if (!GP && k0 == 0) {  // first touch: A -> S
#pragma unroll
            for (int u = 0; u < SU; ++u) {
              const int idx = i0 + u * TH, r = idx / NB, c = idx - r * NB;
              if (idx < tot && c < kb && c <= r && r < rows) v[u] = s_of(r, c, v[u]);
            }
          }
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int idx = i0 + u * TH, r = idx / NB, c = idx - r * NB;
            if (idx < tot) pan[r * LDP + c] = v[u];
          }
        }
      }
      __syncthreads();
      CH_MARK(4);
      if (wave == 0 && lane < NB) {  // the diagonal block, lane r updating row r (right-looking), IN REGISTERS (r05):
        // lane r holds its row a[0..NB) for the whole factorization; step c's pivot is lane c's a[c] and column c
        // of L reaches every lane by readlane (no LDS round trip, fence or wave barrier per step: r04's form
        // spent ≈ 220 µs per pixel at N = 400 on those).  The pivot's inverse square root is the fp64 rsq with
        // two Newton steps; the arithmetic is r04's operation for operation (bit-identical L); the block and the
        // reciprocals 1 / L[c][c] (pitch column) go back to LDS once, for the solves
        double a[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) a[q] = pan[lane * LDP + q];
        double rinv = 0.0;
        bool bad = false;
#pragma unroll
        for (int c = 0; c < NB; ++c) {
          const double d = readlane64(a[c], c);
          bad = bad || !(d > 0.0);
          double inv = __builtin_amdgcn_rsq(d);
          inv = fma(0.5 * inv, fma(-d * inv, inv, 1.0), inv);
          inv = fma(0.5 * inv, fma(-d * inv, inv, 1.0), inv);
          if (lane == c) rinv = inv;
          const double lrc = lane == c ? d * inv : a[c] * inv;  // L[r][c] (rows r >= c are used)
          if (lane >= c) a[c] = lrc;
#pragma unroll
          for (int q = c + 1; q < NB; ++q) a[q] = fma(-lrc, readlane64(a[c], q), a[q]);  // −= L[r][c]·L[q][c]
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) pan[lane * LDP + q] = a[q];
        pan[lane * LDP + NB] = rinv;
        if (bad && lane == 0) s_bad = 1;
      }
      __syncthreads();
      CH_MARK(5);
      if (s_bad) break;  // a non-positive pivot
      // rows below the block: x·L_Dᵀ = panel row  ->  forward substitution against the diagonal block;
      // wave 0 meanwhile solves the block's part of L y = [c₁ | m]
      // (waves 1.. take the rows, so wave 0's serial block solve is not followed by a share of them)
      if (wave == 0) diag_fwd(pan, kb, y1 + k0, y2 + k0);
      for (int r = kb + t - 64; wave > 0 && r < rows; r += TH - 64) {
        double x[NB];
#pragma unroll
        for (int c = 0; c < NB; ++c) {  // (rows below the block exist only when kb = NB)
          double s = PAN(r, c);
#pragma unroll
          for (int q = 0; q < c; ++q) s = fma(-x[q], pan[c * LDP + q], s);
          x[c] = s * pan[c * LDP + NB];
        }
#pragma unroll
        for (int c = 0; c < NB; ++c) PAN(r, c) = x[c];
      }
      __syncthreads();
      CH_MARK(6);
      for (int idx = t; idx < (GP ? min(rows, NB) : rows) * NB; idx += TH) {  // L's panel back to the slot
        const int r = idx / NB, c = idx - r * NB;
        if (c < kb && c <= r) M[at(k0 + r, k0 + c)] = pan[r * LDP + c];
      }
      for (int r = kb + t; r < rows; r += TH) {  // y[i] −= L[i][k0:k0+kb]·y_block (LDS)
        double s1 = y1[k0 + r], s2 = y2[k0 + r];
#pragma unroll
        for (int q = 0; q < NB; ++q) {  // (kb = NB here, as above)
          const double l = PAN(r, q);
          s1 = fma(-l, y1[k0 + q], s1);
          s2 = fma(-l, y2[k0 + q], s2);
        }
        y1[k0 + r] = s1, y2[k0 + r] = s2;
      }
      CH_MARK(7);
      // trailing update of the lower triangle of rows/columns [k0 + kb, n): a wave per 64×32 tile, lane
      // (x, y) = (lane & 7, lane >> 3) owns rows y + 8a (a < 8) and columns x + 8b (b < 4) — each LDS read
      // touches 8 distinct panel rows (distinct banks with the NB + 1 pitch), broadcast over 8 lanes;
      // 12 reads per 32 fp64 FMAs
      const int m = rows - kb, T64 = (m + 63) / 64, nst = T64 * (T64 + 1);  // row tile I: 2I + 2 col tiles
      const int lx = lane & 7, ly = lane >> 3;
      if constexpr (NB % 4 == 0) {
        // (r05) on the fp64 matrix cores: the wave's 64×32 tile is 4×2 blocks of v_mfma_f64_16x16x4f64
        // (A = 16 panel rows × 4 columns, B = 4 columns × 16 panel rows, lane (l & 15, l >> 4) supplying
        // element (row l & 15, column q + (l >> 4)) of each; D: column l & 15, rows (l >> 4) + 4·reg).  6 LDS reads
        // per 8 MFMAs against the VALU form's 12 per 32 FMAs, which made that form LDS-bound; blocks wholly above
        // the diagonal or past the trailing rows are skipped (wave-uniform).  Not bit-identical to the VALU form
        // (the matrix core's product order), held to the oracle by the same tests.
        // (r05) 32×32 wave tiles (2×2 blocks): twice the 64×32 form's tiles to balance over the waves, and
        // half its accumulators (no spills at NB <= 16): 346.3 vs 352.8 ms at N = 400, bit-identical
        // (profiles/r05ak_chol_ab_32x32_tiles.log; the next tile's old values prefetched spilled: 587-593 ms)
        const int lr = lane & 15, lk = lane >> 4;
        const int T32 = (m + 31) / 32, nst32 = T32 * (T32 + 1) / 2;
        auto tile_at = [&](int st, int& ri0, int& rj0) {  // st -> (I, J), J <= I
          int tI = 0;
          while ((tI + 1) * (tI + 2) / 2 <= st) ++tI;
          ri0 = kb + 32 * tI, rj0 = kb + 32 * (st - tI * (tI + 1) / 2);
        };
        auto load_old = [&](int ri0, int rj0, double (&o)[2][2][4]) {
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const int rr = min(ri0 + 16 * bi + lk + 4 * g, rows - 1), cc = rj0 + 16 * bj + lr;
                o[bi][bj][g] = M[at(k0 + rr, k0 + min(cc, rr))];  // clamped into the stored lower triangle
              }
        };
        for (int st = wave; st < nst32; st += TH / 64) {
          int ri0 = 0, rj0 = 0;
          tile_at(st, ri0, rj0);
          double oa[2][2][4];
          load_old(ri0, rj0, oa);
          auto live = [&](int bi, int bj) {  // the block has a stored element (row >= column, both < rows)
            return ri0 + 16 * bi < rows && rj0 + 16 * bj < rows && rj0 + 16 * bj <= ri0 + 16 * bi + 15;
          };
          dx4 acc[2][2];
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = dx4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int q = 0; q < NB; q += 4) {  // (kb = NB whenever there are trailing rows)
            double a[2], b[2];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi) a[bi] = PAN(min(ri0 + 16 * bi + lr, rows - 1), q + lk);
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) b[bj] = PAN(min(rj0 + 16 * bj + lr, rows - 1), q + lk);
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
              for (int bj = 0; bj < 2; ++bj)
                if (live(bi, bj)) acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[bi], b[bj], acc[bi][bj], 0, 0, 0);
          }
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const int r = ri0 + 16 * bi + lk + 4 * g, c = rj0 + 16 * bj + lr;
                double o = oa[bi][bj][g];
                if (!GP && k0 == 0) {  // first touch: A -> S (the clamped elements are never stored)
                  const int rr = min(r, rows - 1);
                  o = s_of(rr, min(c, rr), o);
                }
                if (r < rows && c <= r) M[at(k0 + r, k0 + c)] = o - acc[bi][bj][g];
              }
        }
      } else {
        for (int st = wave; st < nst; st += TH / 64) {
          int I64 = 0;
          while ((I64 + 1) * (I64 + 2) <= st) ++I64;  // st -> (I64, J32), J32 <= 2·I64 + 1 (wave-uniform)
          const int J32 = st - I64 * (I64 + 1);
          const int ri = kb + 64 * I64 + ly, rj = kb + 32 * J32 + lx;
          if (32 * J32 >= m) continue;  // past the trailing block (the last row tile's right half)
          // the tile's old values are loaded ahead of the products (their latency hides behind the FMAs)
          double acc[8][4], old[8][4];
  #pragma unroll
          for (int a = 0; a < 8; ++a) {
            const int rr = min(ri + 8 * a, rows - 1);
            const double* row = M + at(k0 + rr, k0);
  #pragma unroll
            for (int b = 0; b < 4; ++b) {
              acc[a][b] = 0.0;
              old[a][b] = row[min(rj + 8 * b, rr)];  // clamped into the stored lower triangle
              if (!GP && k0 == 0) old[a][b] = s_of(rr, min(rj + 8 * b, rr), old[a][b]);  // first touch: A -> S
            }
          }
          for (int q = 0; q < kb; ++q) {
            double li[8], lj[4];
  #pragma unroll
            for (int a = 0; a < 8; ++a) li[a] = PAN(min(ri + 8 * a, rows - 1), q);  // rows past n: clamped
  #pragma unroll
            for (int b = 0; b < 4; ++b) lj[b] = PAN(min(rj + 8 * b, rows - 1), q);  // reads, masked below
  #pragma unroll
            for (int a = 0; a < 8; ++a)
  #pragma unroll
              for (int b = 0; b < 4; ++b) acc[a][b] = fma(li[a], lj[b], acc[a][b]);
          }
  #pragma unroll
          for (int a = 0; a < 8; ++a) {
            if (ri + 8 * a >= rows) continue;
            double* row = M + at(k0 + ri + 8 * a, k0);
  #pragma unroll
            for (int b = 0; b < 4; ++b)
              if (rj + 8 * b < rows && rj + 8 * b <= ri + 8 * a) row[rj + 8 * b] = old[a][b] - acc[a][b];
          }
        }
      }
      __syncthreads();
      CH_MARK(8);
    }

    if (s_bad) {
      if (t == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
      for (int j = t; j < N; j += TH) wT[(int64_t)j * P + p] = __builtin_nan("");
      __syncthreads();
      continue;
    }
    // ---- Lᵀ z = y (backward), blocked by NB: diagonal blocks staged in LDS (the panel is free) --------
    // Each thread's first row of the off-diagonal update (i = t) is loaded with the diagonal block, so one
    // global-memory latency per block sits on the serial path.
    for (int k0 = (n - 1) / NB * NB; k0 >= 0; k0 -= NB) {
      const int kb = min(NB, n - k0);
      double lp[NB];
#pragma unroll
      for (int q = 0; q < NB; ++q) lp[q] = t < k0 ? M[at(k0 + min(q, kb - 1), t)] : 0.0;
      for (int idx = t; idx < NB * NB; idx += TH) {  // (a short block padded with the identity)
        const int r = idx / NB, c = idx - r * NB;
        const double l = r < kb && c <= r ? M[at(k0 + r, k0 + c)] : (r == c ? 1.0 : 0.0);
        pan[r * LDP + c] = l;
        if (c == r) pan[r * LDP + NB] = 1.0 / l;
      }
      __syncthreads();
      CH_MARK(11);
      if (wave == 0) diag_bwd(pan, kb, y1 + k0, y2 + k0);
      __syncthreads();
      CH_MARK(12);
      // y[i] −= Σ_q L[k0+q][i]·z[k0+q]: rows of L, coalesced over i (z = 0 past a short block's end)
      auto upd = [&](int i, auto&& lval) {
        double s1 = y1[i], s2 = y2[i];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const double l = lval(q), z1 = q < kb ? y1[k0 + q] : 0.0, z2 = q < kb ? y2[k0 + q] : 0.0;
          s1 = fma(-l, z1, s1);
          s2 = fma(-l, z2, s2);
        }
        y1[i] = s1, y2[i] = s2;
      };
      if (t < k0) upd(t, [&](int q) { return lp[q]; });
      for (int i = t + TH; i < k0; i += TH) upd(i, [&](int q) { return M[at(k0 + min(q, kb - 1), i)]; });
      __syncthreads();
      CH_MARK(13);
    }
    CH_MARK(9);
    // bordered elimination: y_n = (c_n + mᵀz1)/(μ + mᵀz2), y₁ = −z1 + z2·y_n, w = H y
    double a1 = 0.0, a2 = 0.0;
    for (int i = t; i < n; i += TH) a1 = fma(mv[i], y1[i], a1), a2 = fma(mv[i], y2[i], a2);
    const double mz1 = sum_all(a1), mz2 = sum_all(a2);
    const double yn = (cv[n] + mz1) / (mv[n] + mz2);
    double uy = 0.0;
    for (int i = t; i < N; i += TH) uy = fma(u(i), i < n ? -y1[i] + y2[i] * yn : yn, uy);
    const double uty = sum_all(uy);
    for (int i = t; i < N; i += TH) {
      const double yi = i < n ? -y1[i] + y2[i] * yn : yn;
      wT[(int64_t)i * P + p] = yi - beta * u(i) * uty;
    }
    __syncthreads();  // the slot, the vectors, xs/ys and the panel are reused by the next pixel
    CH_MARK(10);
  }
#ifdef RTI_CHOL_PROFILE
  if (t == 0 && blockIdx.x < 1024)
    for (int k = 0; k < 16; ++k) rti_chol_prof[blockIdx.x][k] = prof_[k];
#endif
}

// ---- Left-looking tiled Cholesky on the fp64 matrix cores (r06; 256 < N <= RBF_LL_MAX_N) ------------------
// The same bordered system as rbf_solve_chol (S = −(HAH)[:n, :n] = L Lᵀ, n = N − 1), factored LEFT-looking in block
// columns of 64 with L kept in the slot in the matrix cores' own operand layout, so that every element of the
// trailing matrix is formed ONCE (in registers) instead of being read and rewritten by every panel:
//   * tile (rg, jg) = rows 16·rg .. +15, columns 4·jg .. +3 of L, 64 doubles in lane order l = row%16 + 16·(col%4):
//     exactly what lane l supplies as the A or B operand of v_mfma_f64_16x16x4f64 (A[m][k] / B[k][n], m or n = l&15,
//     k = l>>4), and what lane l holds in register g of a D tile whose rows are 4g + (l>>4) and columns l & 15 —
//     so loads, MFMAs and stores are all whole 512-B tiles, coalesced, with no shuffles;
//   * block column J (columns J0 .. J0 + 63): every wave owns up to 4 row groups (16 rows) per pass and holds
//     Cᵀ[c][i] = Σ_q L[J0+c][q]·L[i][q] for them in 16 accumulator tiles; per earlier block column K the 64 rows
//     J0 .. J0+63 of K (32 KB, the A operands, = the B operands of the diagonal row groups) are staged in LDS
//     (double-buffered, the next chunk's loads in flight during this chunk's MFMAs) and the other row groups'
//     B tiles stream from the slot.  Then C = S − Cᵀ with S formed from the node distances in registers (the
//     slot never holds S or A);
//   * the 64 columns are finished in 4 sub-panels of 16: sub-panel j is updated by the finished sub-panels k < j
//     (MFMA, L_D(j,k) from LDS), its 16×16 diagonal block is factored AND inverted by one wave in registers (lane
//     per row, readlane broadcasts, 16 steps), and every row group below multiplies by that inverse (4 MFMAs);
//   * the right-hand sides c₁ and m ride along as two extra ROWS (n64, n64 + 1) of the matrix: their rows of L are
//     L⁻¹c₁ and L⁻¹m, so the forward substitution is the factorization itself;
//   * rows/columns n .. n64 − 1 are padded with the identity (the last block column runs unguarded).
// The backward substitution Lᵀ z = y is a GEMV per block column over its tiles (coalesced) plus the 64×64
// diagonal part from the 16×16 inverses; then the bordered elimination and w = H y as rbf_solve_chol.
// Slot traffic per pixel at N = 400: ≈ 2.0 MB of B/A tiles read, 0.9 MB of L written, 0.9 MB read back by the
// backward pass — against ≈ 8 MB for the right-looking panels (each panel re-read and re-wrote the trailing
// triangle).  A non-positive pivot (repeated or nearly repeated nodes) reports RTI_ERR_SINGULAR like rbf_solve_chol.
// TWO pixels per CU: workgroups of 4 waves (one per SIMD) with 256 registers each (amdgpu_waves_per_eu(2)) and at
// most half the LDS, so one pixel's serial phases (the 16×16 leaves, the barriers, the distance evaluations on the
// VALU) run while the other pixel's waves keep the matrix cores busy.  (One 8-wave workgroup per CU: 333.7 ms at
// N = 400; 4 waves of 8 row groups with 512 registers each spilled 738 VGPRs.)
// Above N = 448 the LDS no longer fits twice per CU: one workgroup of 8 waves per CU instead (RBF_LL_TH1).
constexpr int RBF_LL_TH = 256, RBF_LL_TH1 = 512;
constexpr int RBF_LL_RGW = 4;  // row groups per wave per pass (16 accumulator tiles)
constexpr int RBF_LL_TWO_MAX_N = 641;
constexpr int RBF_LL_MAX_N = 1022;
__host__ __device__ constexpr int ll_n64(int N) { return (N - 1 + 63) / 64 * 64; }
__host__ __device__ constexpr int ll_groups(int N) { return ll_n64(N) / 16 + 1; }  // + the right-hand-side group
// (tiles / 16) of the block columns before K: block column K' holds row groups 4(K' + 1) .. G − 1
__host__ __device__ constexpr int64_t ll_col_tiles(int G, int K) { return (int64_t)K * (G - 4) - 2 * (int64_t)K * (K - 1); }
constexpr int LL_DIAG = 2560;  // per block column: 6 off-diagonal 16×16 blocks of L_D + 4 diagonal inverses
__host__ __device__ constexpr int64_t ll_slot_doubles(int N) {
  return ll_col_tiles(ll_groups(N), ll_n64(N) / 64) * 1024 + (int64_t)(ll_n64(N) / 64) * LL_DIAG;
}
// LDS: the A chunk [4096] (the backward pass's z [2][n64] in its place), the block column's L_D blocks / inverses
// [2560], the leaf's 16×17 matrix (backward: 2×64 right-hand sides) [576], g, c, m [np] each, the nodes [2][np]
// floats; np = n64 + 64 >= N, the entries past N zero, so every column index j < n64 reads in bounds and the (many)
// per-column loads share one base address.  Up to N = 641 that is <= 80 KiB: two workgroups per CU.
constexpr int LL_OFF_DG = 4096, LL_OFF_LF = LL_OFF_DG + 2560, LL_OFF_G = LL_OFF_LF + 576;
__host__ __device__ constexpr int ll_np(int N) { return ll_n64(N) + 64; }
__host__ __device__ constexpr size_t ll_lds_bytes(int N) { return (size_t)(LL_OFF_G + 4 * ll_np(N)) * 8; }
static_assert(ll_lds_bytes(RBF_LL_TWO_MAX_N) + 64 <= 80 * 1024 && 2 * ll_n64(RBF_LL_MAX_N) <= LL_OFF_DG,
              "two workgroups per CU; z fits in the chunk's place");
static_assert(ll_lds_bytes(RBF_LL_MAX_N) <= 160 * 1024 - 256, "RBF_LL_MAX_N");
__host__ __device__ constexpr int ll_ls(int jp, int j) { return jp * (jp - 1) / 2 + j; }  // L_D block (jp, j), jp > j

// The 16×16 leaf of rbf_solve_llt on one wave: T (symmetric, LDS [16][17] at smem + off_t) is FACTORED lane per row in
// registers (lane r holds row r; step c's pivot and column c of L reach every lane by readlane: the chain per step
// is one readlane, the pivot's inverse square root and one FMA), then INVERTED lane per column by substitution (lane
// k computes column k of L⁻¹, L's rows broadcast from LDS); L⁻¹ is written as the A operand of the sub-panel solves
// (slab k/4, lane r + 16·(k % 4)) at smem + off_w.  Returns true for a non-positive pivot.  Out of line: its 32
// registers are allocated apart from the kernel's 128 of accumulators (inlined, the same code spilled 840 VGPRs;
// r06's first quad form with ds_bpermute broadcasts took ≈ 7 µs per leaf).
__device__ __noinline__ bool rbf_ll_leaf(int off_t, int off_w) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Lm = smem + off_t;  // [16][17]: T, then L
  double* sv = Lm + 272;      // [16]: 1 / L[r][r]
  double* Wd = smem + off_w;  // [4][64]
  const int lane = threadIdx.x & 63, lr = lane & 15;
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  bool bad = false;
  {
    double a[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) a[q] = Lm[lr * 17 + q];
    double si = 0.0;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const double d = readlane64(a[c], c);
      bad = bad || !(d > 0.0);
      double inv = __builtin_amdgcn_rsq(d);
      inv = fma(0.5 * inv, fma(-d * inv, inv, 1.0), inv);
      inv = fma(0.5 * inv, fma(-d * inv, inv, 1.0), inv);
      const double lrc = lr == c ? d * inv : a[c] * inv;  // L[r][c] (rows r >= c are used)
      a[c] = lr >= c ? lrc : a[c];
      si = lr == c ? inv : si;
#pragma unroll
      for (int q = c + 1; q < 16; ++q) a[q] = fma(-lrc, readlane64(a[c], q), a[q]);  // −= L[r][c]·L[q][c]
    }
    wave_sync();  // every lane has read T before L overwrites it
    if (lane < 16) {
#pragma unroll
      for (int q = 0; q < 16; ++q) Lm[lr * 17 + q] = a[q];
      sv[lr] = si;
    }
  }
  wave_sync();
  double x[16];  // column k = lr of L⁻¹
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    double v = r == lr ? 1.0 : 0.0;
#pragma unroll
    for (int q = 0; q < r; ++q) v = fma(-Lm[r * 17 + q], x[q], v);
    x[r] = v * sv[r];
  }
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 16; ++r) Wd[(lr >> 2) * 64 + r + 16 * (lr & 3)] = x[r];
  }
  return bad;
}

template <typename T, int TH>
__global__ void __launch_bounds__(TH) __attribute__((amdgpu_waves_per_eu(2, 2)))
rbf_solve_llt(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
              double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status, double* __restrict__ ws) {
  constexpr int RGW = RBF_LL_RGW, NWV = TH / 64, PASS = NWV * RGW;  // row groups per pass
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // wave index through readfirstlane: the compiler then knows every wave-dependent condition (row groups, diagonal
  // sub-blocks) is uniform and branches on SCC instead of masking EXEC around the MFMAs
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lk = lane >> 4;
  const int n = N - 1, n64 = ll_n64(N), nbc = n64 / 64, G = n64 / 16 + 1;
  double* slot = ws + (int64_t)blockIdx.x * ll_slot_doubles(N);
  double* diagw = slot + ll_col_tiles(G, nbc) * 1024;  // [nbc][LL_DIAG]
  const __amdgpu_buffer_rsrc_t slot_rs =  // the slot's tiles, for the A chunks' LDS-DMA
      __builtin_amdgcn_make_buffer_rsrc(slot, (short)0, (int)(ll_col_tiles(G, nbc) * 1024 * 8), 0x00020000);
  double* Ab = smem;                                   // [4096]: the A chunk, tiles [c-group][jl][64]
  double* Dg = smem + LL_OFF_DG;                       // [10][4][64]: L_D(jp, j) (6), then the inverses (4)
  double* lf = smem + LL_OFF_LF;                       // [576] the leaf; backward: [2][64] right-hand sides + [2][16]
  double* zv = smem;                                   // [2][n64] (backward; the chunk's place)
  const int np = ll_np(N);
  double* gl = smem + LL_OFF_G;                        // g = A u
  double* cvl = gl + np;                               // c = H b
  double* mvl = cvl + np;                              // m = (HAH)[:, n]
  float* xs = reinterpret_cast<float*>(mvl + np);
  float* ys = xs + np;
  __shared__ double red[TH / 64];
  __shared__ int s_bad;
  const double e = 1.0 / sqrt((double)N), beta = 1.0 / (1.0 - e);  // H = I − β u uᵀ, u = e·1 − e_n
  auto u = [&](int j) { return j < n ? e : (j == n ? e - 1.0 : 0.0); };
  auto sum_all = [&](double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < TH / 64; ++i) r += red[i];
    return r;
  };
  auto dist = [&](int i, int j) { return dist64((double)xs[i], (double)ys[i], (double)xs[j], (double)ys[j]); };
  // the slot's tile (rg, jg), rg >= 4·(jg/16 + 1)
  auto tile = [&](int rg, int jg) -> double* {
    const int K = jg >> 4;
    return slot + ((ll_col_tiles(G, K) + (rg - 4 * (K + 1))) * 16 + (jg & 15)) * 64;
  };
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
#ifdef RTI_CHOL_PROFILE
  long long prof_[16] = {}, last_ = wall_clock64();
#endif
  // (r06) the row groups past n — the padding up to n64, all inside the last block column's diagonal block — are never
  // factored as rows below an earlier block: their L rows there are zero (S is the identity on the padding), so their
  // tiles are zeroed once per launch and afterwards only read (as the last block column's A chunk and B operands)
  const int nrr = (n + 15) / 16;  // row groups holding real rows
  for (int K = 0; K + 1 < nbc; ++K)
    for (int rg = nrr; rg < G - 1; ++rg) {
      double* tb = tile(rg, 16 * K);  // the row group's 16 tiles of block column K are consecutive
      for (int idx = t; idx < 1024; idx += TH) tb[idx] = 0.0;
    }
  __syncthreads();

  for (int64_t p = blockIdx.x; p < P; p += gridDim.x) {
    const int64_t base = p * N;
    if (t == 0) s_bad = 0;
    for (int j = t; j < np; j += TH) {
      if (j < N) {
        const float x = lu[base + j], y = lv[base + j];
        xs[j] = x, ys[j] = y;
        xyT[(int64_t)j * P + p] = make_float2(x, y);
        cvl[j] = ldd(I + base + j);  // b (c = H b is formed in place)
      } else {
        xs[j] = 0.f, ys[j] = 0.f, gl[j] = 0.0, cvl[j] = 0.0, mvl[j] = 0.0;
      }
    }
    __syncthreads();
    CH_MARK(0);
    // A's row sums and the repeated-node check (SciPy: LinAlgError).  Where its partials fit in the (still unused)
    // chunk / diagonal / leaf LDS, the SYMMETRIC form of rbf_solve_chol: each distance of the lower triangle once, in
    // 64×64 tiles (lane = column), column partials in registers, row partials through a per-wave LDS slice, every
    // row's sum added up in a fixed order; otherwise RB rows per wave, every distance of a row
    bool dup = false;
    const int T64r = (N + 63) / 64, ntl = T64r * (T64r + 1) / 2;
    if (ntl * 128 + (TH / 64) * 512 <= LL_OFF_G) {
      double* rowp = smem;                                  // [ntl][64]
      double* colp = rowp + ntl * 64;                       // [ntl][64]
      double* rbuf = colp + ntl * 64 + wave * 512;          // [8][64] per wave
      for (int st = wave; st < ntl; st += TH / 64) {
        int tI = 0;
        while ((tI + 1) * (tI + 2) / 2 <= st) ++tI;
        const int tJ = st - tI * (tI + 1) / 2;
        const int j = 64 * tJ + lane;  // < np: the nodes past N read as zeros, masked below
        const bool jv = j < N;
        const double xj = (double)xs[j], yj = (double)ys[j];
        double cacc = 0.0;
        const int rows_t = min(64, N - 64 * tI);
        for (int m0 = 0; m0 < rows_t; m0 += 8) {
          double v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int i = 64 * tI + m0 + q;
            const bool iv = i < N;
            const double d = dist64_pos((double)xs[i], (double)ys[i], xj, yj);
            const double dd = iv && jv ? d : 0.0;
            v[q] = dd;
            if (tI > tJ) cacc += dd;
            dup = dup || (iv && jv && j != i && d == 0.0);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) rbuf[q * 64 + lane] = v[q];
          wave_sync();
          const int q = lane & 7, sg = lane >> 3;  // row q of the chunk, columns 8·sg .. 8·sg + 7
          double rsum = 0.0;
#pragma unroll
          for (int c = 0; c < 8; ++c) rsum += rbuf[q * 64 + 8 * sg + c];
          rsum += __shfl_xor(rsum, 8, 64);
          rsum += __shfl_xor(rsum, 16, 64);
          rsum += __shfl_xor(rsum, 32, 64);
          if (lane < 8) rowp[st * 64 + m0 + q] = rsum;
          wave_sync();
        }
        if (tI > tJ) colp[st * 64 + lane] = cacc;
      }
      __syncthreads();
      for (int i = t; i < N; i += TH) {  // row i: its row block's row partials, then the column partials below
        const int tI = i >> 6, r = i & 63;
        double rs = 0.0;
        for (int tJ = 0; tJ <= tI; ++tJ) rs += rowp[(tI * (tI + 1) / 2 + tJ) * 64 + r];
        for (int I2 = tI + 1; I2 < T64r; ++I2) rs += colp[(I2 * (I2 + 1) / 2 + tI) * 64 + r];
        gl[i] = fma(e, rs, -(i < n ? dist(n, i) : 0.0));
      }
    } else {
      constexpr int RB = 4, WV = TH / 64;
      for (int i0 = wave; i0 < N; i0 += RB * WV) {
        double rs[RB], xi[RB], yi[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int i = min(i0 + r * WV, N - 1);
          xi[r] = (double)xs[i], yi[r] = (double)ys[i], rs[r] = 0.0;
        }
        for (int j = lane; j < N; j += 64) {
          const double xj = (double)xs[j], yj = (double)ys[j];
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const double d = dist64_pos(xi[r], yi[r], xj, yj);
            rs[r] += d;
            dup = dup || (i0 + r * WV < N && j != i0 + r * WV && d == 0.0);
          }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
          for (int r = 0; r < RB; ++r) rs[r] += __shfl_xor(rs[r], off, 64);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int i = i0 + r * WV;
          if (lane == 0 && i < N) gl[i] = fma(e, rs[r], -(i < n ? dist(n, i) : 0.0));
        }
      }
    }
    if (dup) s_bad = 1;
    __syncthreads();
    CH_MARK(1);
    double ub = 0.0, ug = 0.0;
    for (int i = t; i < N; i += TH) ub = fma(u(i), cvl[i], ub), ug = fma(u(i), gl[i], ug);
    const double utb = sum_all(ub), b2 = beta * beta * sum_all(ug);
    auto hah = [&](int i, int j, double d) { return d - beta * (u(i) * gl[j] + gl[i] * u(j)) + b2 * u(i) * u(j); };
    for (int i = t; i < N; i += TH) {
      cvl[i] = cvl[i] - beta * u(i) * utb;
      mvl[i] = hah(n, i, i < n ? dist(n, i) : 0.0);
    }
    __syncthreads();
    CH_MARK(2);
    // element (i, j) of the padded matrix [S | I_pad; c₁ᵀ; mᵀ] (row i, column j < n64), branch-free: for i, j < n,
    // −hah(i, j, d) = β·e·(g_i + g_j) − d − b2·e² (u = e on both); the right-hand-side rows are their own row group
    const double be = beta * e, b2e2 = b2 * e * e;
    // (the column index enters as o = 16·cg + 4·g, a compile-time offset from J0 + lk: the per-element tests are one
    // compare against that immediate and one against a lane value, and the loads share one base — r06: with the column
    // index itself per element the compiler kept 16 column indices per lane, spilled them, and waited on a scratch
    // reload for every element)
    // ---- the factorization, block column by block column -------------------------------------------
    for (int J = 0; J < nbc && !s_bad; ++J) {  // s_bad: block-uniform after each sync
      const int J0 = 64 * J, rgd = J0 / 16;
      // the block column's row groups, as logical indices q in [rgd, Ge): q < Ge − 1 is row group q, q = Ge − 1 the
      // right-hand-side group G − 1; before the last block column the padding groups [nrr, G − 1) are left out
      const int Ge = J + 1 < nbc ? nrr + 1 : G;
      // the 16-column sub-panels holding real columns (4 but in the last block column)
      const int nsp4 = J + 1 < nbc ? 4 : (n - J0 + 15) / 16;
      if (nsp4 < 4) {  // the padding sub-panels are skipped below: their L_D blocks are zero, their inverses I
        for (int idx = t; idx < 2560; idx += TH) {
          const int sl = idx >> 8, e = idx & 255, jp = sl < 6 ? (sl >= 3 ? 3 : sl >= 1 ? 2 : 1) : 0;
          const int jj = sl < 6 ? sl - jp * (jp - 1) / 2 : sl - 6;  // slot ll_ls(jp, jj) or the inverse of jj
          const int c = 4 * (e >> 6) + ((e & 63) >> 4), r = e & 15;
          if (jj >= nsp4) Dg[idx] = sl >= 6 && r == c ? 1.0 : 0.0;
        }
      }
      for (int rgp = rgd; rgp < Ge; rgp += PASS) {  // passes of up to PASS row groups
        const bool p0 = rgp == rgd;
        int rgt[RGW];
        bool vt[RGW];
#pragma unroll
        for (int tt = 0; tt < RGW; ++tt) {
          const int q = rgp + wave + NWV * tt;
          rgt[tt] = q < Ge - 1 ? q : G - 1, vt[tt] = q < Ge;
        }
        static_assert(NWV >= 4, "the 4 diagonal sub-blocks are the first row groups of waves 0..3");
        const bool dg = p0 && wave < 4;  // this wave's first row group is diagonal sub-block `wave`
        dx4 acc[RGW][4];
#pragma unroll
        for (int tt = 0; tt < RGW; ++tt)
#pragma unroll
          for (int cg = 0; cg < 4; ++cg) acc[tt][cg] = dx4{0.0, 0.0, 0.0, 0.0};
        // Cᵀ[c][i] = Σ_{q < J0} L[J0 + c][q]·L[i][q], one earlier block column K per LDS chunk
        // the row groups this wave holds in this pass are a prefix tt < ntt (wave-uniform): one branch-free K loop per
        // count, so the inner loop has no per-row-group conditions (every wave still takes every chunk's barrier)
        const int ntt = max(0, min(RGW, (Ge - rgp - wave + NWV - 1) / NWV));
        auto kloop = [&](auto ntc, auto ncgc) {
          constexpr int NT = decltype(ntc)::value, NCG = decltype(ncgc)::value;  // NCG: column groups with real columns
          // B operands from the slot (the diagonal row groups' too: the chunk just staged left them in L2) through a
          // 4-deep ring that runs across the chunks: column group jl + 4's loads issue behind jl's MFMAs, the next
          // chunk's first four during this chunk's last four (the tiles were written block columns ago: no barrier
          // orders them); the scheduling fences keep the compiler from hoisting all 16 column groups' loads (spills)
          [[maybe_unused]] double bq[4][NT > 0 ? NT : 1];
          auto ldb = [&](int K, int jl, int tt) { return tile(rgt[tt], 16 * K + jl)[lane]; };
          if constexpr (NT > 0) {
            if (J > 0)
#pragma unroll
              for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) bq[d][tt] = ldb(0, d, tt);
          }
          // (r06) the A chunk in two 16-KB halves (column tiles 0–7 / 8–15 of its row groups), each filled by LDS-DMA one
          // half-step ahead into the other buffer: half-step h = 2K + hf computes from Ab + 2048·(h & 1) while the DMA of
          // h + 1 is in flight.  Per half-step: this wave's DMA(h) retired by a counted vmcnt (the 8·NT B-ring loads issued
          // after it may stay in flight), one barrier (every wave's DMA(h) landed, every read of the other buffer done),
          // then DMA(h + 1) and the MFMAs.  (Measured: the synchronous register-staged chunk cost up to 18 % of the solve.)
          const int nh = 2 * J;
          auto dma_half = [&](int h) {
            const int K = h >> 1, hf = h & 1;
            double* dst = Ab + (h & 1) * 2048;
            for (int q = wave; q < 4 * nsp4; q += NWV) {  // 1 KB per instruction: row group q >> 2, part q & 3
              const int cg = q >> 2, part = q & 3;
              const double* src = tile(rgd + cg, 16 * K + 8 * hf) + part * 128;
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  slot_rs, (__attribute__((address_space(3))) void*)(dst + cg * 512 + part * 128), 16,
                  (int)((src - slot) * 8) + 16 * lane, 0, 0, 0);
            }
          };
          if (J > 0) {
            dma_half(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          for (int h = 0; h < nh; ++h) {
            const int K = h >> 1, hf = h & 1;
            if (h > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * NT) : "memory");  // this wave's DMA(h) retired
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every ds_read of the other buffer returned
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (h + 1 < nh) dma_half(h + 1);
            const double* Ak = Ab + (h & 1) * 2048;
            if constexpr (NT > 0) {
              __builtin_amdgcn_s_setprio(1);  // (the MFMA stream ahead of the other pixel's VALU phases on this SIMD)
              const double* bp[NT];
#pragma unroll
              for (int tt = 0; tt < NT; ++tt) bp[tt] = tile(rgt[tt], 16 * K) + lane;
              const int kn = K + 1 < J ? K + 1 : K;  // (the last chunk re-reads its own first tiles: harmless)
#pragma unroll
              for (int j8 = 0; j8 < 8; ++j8) {
                const int jl = 8 * hf + j8;
                double a[NCG];
#pragma unroll
                for (int cg = 0; cg < NCG; ++cg) a[cg] = Ak[(cg * 8 + j8) * 64 + lane];
#pragma unroll
                for (int tt = 0; tt < NT; ++tt)
#pragma unroll
                  for (int cg = 0; cg < NCG; ++cg)
                    acc[tt][cg] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cg], bq[j8 & 3][tt], acc[tt][cg], 0, 0, 0);
#pragma unroll
                for (int tt = 0; tt < NT; ++tt)
                  bq[j8 & 3][tt] = jl + 4 < 16 ? bp[tt][(jl + 4) * 64] : ldb(kn, jl - 12, tt);
                __builtin_amdgcn_sched_barrier(0);
              }
              __builtin_amdgcn_s_setprio(0);
            }
          }
          if (J > 0) {  // the chunk buffers are restaged by the next pass / block column: every read returned first
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
          }
        };
        static_assert(RGW == 4, "the K-loop dispatch below");
        using I4 = std::integral_constant<int, 4>;
        // (r06) the last block column's column groups past n are padding: their Cᵀ is zero (the A chunk's padding
        // rows are zero tiles), so the K loop runs only the first nsp of them — for the wave counts the last block
        // column has (its 4 diagonal row groups and the right-hand-side group: at most 2 per wave)
        switch (nsp4 < 4 ? ntt * 8 + nsp4 : 64 + ntt) {
          case 1 * 8 + 1: kloop(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}); break;
          case 1 * 8 + 2: kloop(std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{}); break;
          case 1 * 8 + 3: kloop(std::integral_constant<int, 1>{}, std::integral_constant<int, 3>{}); break;
          case 2 * 8 + 1: kloop(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{}); break;
          case 2 * 8 + 2: kloop(std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{}); break;
          case 2 * 8 + 3: kloop(std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{}); break;
          case 64 + 4: case 4 * 8 + 1: case 4 * 8 + 2: case 4 * 8 + 3:
            kloop(std::integral_constant<int, 4>{}, I4{}); break;
          case 64 + 3: case 3 * 8 + 1: case 3 * 8 + 2: case 3 * 8 + 3:
            kloop(std::integral_constant<int, 3>{}, I4{}); break;
          case 64 + 2: kloop(std::integral_constant<int, 2>{}, I4{}); break;
          case 64 + 1: kloop(std::integral_constant<int, 1>{}, I4{}); break;
          default: kloop(std::integral_constant<int, 0>{}, I4{}); break;
        }
        CH_MARK(3);
        // C = S − Cᵀ (S from the distances, in registers).  (r06) Column-group outer: a column group's 4 node columns
        // (x, y, g of node J0 + lk + 16·cg + 4·g) are read from LDS once and serve every row group of the wave, whose
        // rows' x, y, g were read once before the loop
        {
          double xi[RGW], yi[RGW], gi[RGW];
          int di[RGW];  // i − J0 − lk: the padding rows' identity entry sits at o = di
          bool iv[RGW];
#pragma unroll
          for (int tt = 0; tt < RGW; ++tt) {
            const int i = 16 * rgt[tt] + lr, ic = vt[tt] && i < np ? i : 0;
            xi[tt] = (double)xs[ic], yi[tt] = (double)ys[ic], gi[tt] = gl[ic];
            iv[tt] = i < n, di[tt] = i - J0 - lk;
          }
          const int jrem = n - J0 - lk;
          const float* xj = xs + J0 + lk;
          const float* yj = ys + J0 + lk;
          const double* gj = gl + J0 + lk;
          const double* cj = cvl + J0 + lk;
          const double* mj = mvl + J0 + lk;
#pragma unroll
          for (int cg = 0; cg < 4; ++cg) {
            if (cg >= nsp4) break;  // padding column groups: S and Cᵀ are zero, acc stays 0
            double xc[4], yc[4], gc[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int o = 16 * cg + 4 * g;
              xc[g] = (double)xj[o], yc[g] = (double)yj[o], gc[g] = gj[o];
            }
#pragma unroll
            for (int tt = 0; tt < RGW; ++tt) {
              if (!vt[tt]) continue;
              const bool rhs = rgt[tt] == G - 1;  // wave-uniform: the right-hand-side rows n64 + lr (c₁ for lr = 0, m for 1)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const int o = 16 * cg + 4 * g;
                double v;
                if (rhs) {
                  v = lr < 2 && o < jrem ? (lr == 0 ? cj[o] : mj[o]) : 0.0;
                } else {
                  const double sv = fma(be, gi[tt] + gc[g], -dist64_pos(xi[tt], yi[tt], xc[g], yc[g]) - b2e2);
                  v = iv[tt] ? (o < jrem ? sv : 0.0) : (di[tt] == o ? 1.0 : 0.0);
                }
                acc[tt][cg][g] = v - acc[tt][cg][g];
              }
            }
            __builtin_amdgcn_sched_barrier(0);  // (else every distance's operands are hoisted: spills)
          }
        }
        CH_MARK(4);
        // the four 16-column sub-panels (a barrier-bound chain: at wave priority 1, the leaves at 2)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j >= nsp4) break;  // padding sub-panels (block-uniform): acc stays S − Cᵀ = 0 for every row but the
                                 // padding rows' own diagonal, which the diagonal area already holds as L_D = I
          // (1) update by the finished sub-panels k < j: acc[j] −= L_D(j, k) · X_k  (rows of the diagonal
          // sub-block `wave` need sub-panels j <= wave only)
#pragma unroll
          for (int tt = 0; tt < RGW; ++tt) {
            if (!vt[tt] || (tt == 0 && dg && j > wave) || j == 0) continue;
            dx4 s = dx4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < j; ++k)
#pragma unroll
              for (int sl = 0; sl < 4; ++sl)
                s = __builtin_amdgcn_mfma_f64_16x16x4f64(Dg[(ll_ls(j, k) * 4 + sl) * 64 + lane], acc[tt][k][sl], s, 0, 0, 0);
            acc[tt][j] -= s;
          }
          // (2) the diagonal 16×16 block T, on wave j: factored and inverted by rbf_ll_leaf (out of line, so its 32
          // registers are allocated apart from the kernel's accumulators)
          if (p0 && wave == j) {
            __builtin_amdgcn_s_setprio(2);  // the serial leaf is every wave's critical path: ahead of the other pixel
#pragma unroll
            for (int g = 0; g < 4; ++g) lf[lr * 17 + 4 * g + lk] = acc[0][j][g];  // lf[i][c] = T[c][i] (symmetric)
            wave_sync();
            const bool bad = rbf_ll_leaf(LL_OFF_LF, LL_OFF_DG + (6 + j) * 256);
            __builtin_amdgcn_s_setprio(1);
#ifndef RTI_LLT_NOSTAGE
            if (bad && lane == 0) s_bad = 1;
#else
            (void)bad;
#endif
          }
          __syncthreads();
          CH_MARK(5);
          // (3) rows below the diagonal block: X_j = L_jj⁻¹ · acc[j]; the diagonal sub-blocks below publish theirs
          // as the L_D(wave, j) operand of the later sub-panels
#pragma unroll
          for (int tt = 0; tt < RGW; ++tt) {
            if (!vt[tt] || (tt == 0 && dg && j >= wave)) continue;
            dx4 s = dx4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int sl = 0; sl < 4; ++sl)
              s = __builtin_amdgcn_mfma_f64_16x16x4f64(Dg[((6 + j) * 4 + sl) * 64 + lane], acc[tt][j][sl], s, 0, 0, 0);
            acc[tt][j] = s;
            if (tt == 0 && dg)
#pragma unroll
              for (int g = 0; g < 4; ++g) Dg[(ll_ls(wave, j) * 4 + g) * 64 + lane] = s[g];
          }
          __syncthreads();
          CH_MARK(6);
        }
        __builtin_amdgcn_s_setprio(0);
        // L's tiles of this block column (the diagonal sub-blocks go to the slot's diagonal area below)
#pragma unroll
        for (int tt = 0; tt < RGW; ++tt) {
          if (!vt[tt] || rgt[tt] < rgd + 4) continue;
          double* tb = tile(rgt[tt], 16 * J) + lane;  // the block column's 16 tiles of this row group are consecutive
#pragma unroll
          for (int cg = 0; cg < 4; ++cg)
#pragma unroll
            for (int g = 0; g < 4; ++g) tb[(4 * cg + g) * 64] = acc[tt][cg][g];
        }
        CH_MARK(7);
        if (s_bad) break;
      }
      for (int idx = t; idx < LL_DIAG; idx += TH) diagw[(int64_t)J * LL_DIAG + idx] = Dg[idx];
      __syncthreads();  // Dg and the A chunks are reused by the next block column
      CH_MARK(8);
    }

    if (s_bad) {
      if (t == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
      for (int j = t; j < N; j += TH) wT[(int64_t)j * P + p] = __builtin_nan("");
      __syncthreads();
      continue;
    }
    // ---- Lᵀ z = y: y = the right-hand-side rows of L (row group G − 1, lanes 0 and 1 of each tile) ------------
    for (int idx = t; idx < n64; idx += TH) {
      const double* tl = tile(G - 1, idx >> 2);
      zv[idx] = tl[16 * (idx & 3)], zv[n64 + idx] = tl[1 + 16 * (idx & 3)];
    }
    __syncthreads();
    // Per block column J (last to first): rhs = y_J − Σ_{i >= J0 + 64} L[i][J-block]ᵀ z_i (a GEMV over its tiles, wave w
    // taking column groups CW·w .. CW·w + CW − 1, RU row groups' loads in flight), then L_Dᵀ z_J = rhs on wave 0.  The
    // GEMV is software-pipelined across J: the rows beyond block J + 1 have their z before block J + 1's diagonal solve,
    // so that part of J's GEMV runs DURING it (wave 0 first takes its own share); after the barrier only block J + 1's
    // four row groups are left.  The partial sums stay in registers across the barrier.
    constexpr int CW = 16 / NWV, RU = 4;
    double s1[CW], s2[CW];
#pragma unroll
    for (int h = 0; h < CW; ++h) s1[h] = 0.0, s2[h] = 0.0;
    auto gemv = [&](int J, int rg0, int rg1) {  // rows of row groups [rg0, rg1) of block column J into s1, s2
      const int nrg = rg1 - rg0;
      if (nrg <= 0) return;
      const double* gb = tile(rg0, 16 * J + CW * wave) + lane;  // + (rg − rg0)·1024 + h·64
      for (int r0 = 0; r0 < nrg; r0 += RU) {
        double lv[RU][CW], z1[RU], z2[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int rr = min(r0 + u, nrg - 1);
#pragma unroll
          for (int h = 0; h < CW; ++h) lv[u][h] = gb[(int64_t)rr * 1024 + h * 64];
          const bool ok = r0 + u < nrg;
          z1[u] = ok ? zv[16 * (rg0 + rr) + lr] : 0.0, z2[u] = ok ? zv[n64 + 16 * (rg0 + rr) + lr] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < RU; ++u)
#pragma unroll
          for (int h = 0; h < CW; ++h) s1[h] = fma(lv[u][h], z1[u], s1[h]), s2[h] = fma(lv[u][h], z2[u], s2[h]);
      }
    };
    for (int J = nbc - 1; J >= 0; --J) {
      const int J0 = 64 * J, rgd = J0 / 16;
      // (rows of the padding groups are zero in L and in z: the ranges end at nrr)
      if (J + 1 < nbc) gemv(J, rgd + 4, min(rgd + 8, nrr));  // block J + 1's rows (its z_{J+1} was solved last iteration)
#pragma unroll
      for (int h = 0; h < CW; ++h)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) s1[h] += __shfl_xor(s1[h], off, 64), s2[h] += __shfl_xor(s2[h], off, 64);
      if (lr == 0) {
#pragma unroll
        for (int h = 0; h < CW; ++h) {
          const int c = 4 * (CW * wave + h) + lk;
          lf[c] = zv[J0 + c] - s1[h], lf[64 + c] = zv[n64 + J0 + c] - s2[h];
        }
      }
#pragma unroll
      for (int h = 0; h < CW; ++h) s1[h] = 0.0, s2[h] = 0.0;
      for (int idx = t; idx < LL_DIAG; idx += TH) Dg[idx] = diagw[(int64_t)J * LL_DIAG + idx];
      __syncthreads();
      CH_MARK(9);
      if (J > 0) gemv(J - 1, rgd + 4, nrr);  // block column J − 1's rows beyond block J: their z are final
      if (wave == 0) {  // L_Dᵀ z = rhs by 16×16 blocks: lanes 0–15 the first right-hand side, 16–31 the second
        __builtin_amdgcn_s_setprio(2);  // (the serial solve ahead of the GEMV loads and the other pixel)
        const int c = lr, rh = lk & 1;
        double* zl = zv + rh * n64 + J0;
        // (loops kept rolled: unrolled, the compiler hoisted all 96 LDS operands and spilled the whole kernel)
#pragma unroll 1
        for (int j = 3; j >= 0; --j) {
          double v = lf[rh * 64 + 16 * j + c];
#pragma unroll 1
          for (int jp = j + 1; jp < 4; ++jp) {
            double v2 = 0.0;
#pragma unroll
            for (int m = 0; m < 16; m += 2) {
              v = fma(-Dg[ll_ls(jp, j) * 256 + (c >> 2) * 64 + m + 16 * (c & 3)], zl[16 * jp + m], v);
              v2 = fma(-Dg[ll_ls(jp, j) * 256 + (c >> 2) * 64 + m + 1 + 16 * (c & 3)], zl[16 * jp + m + 1], v2);
            }
            v += v2;
          }
          double* tmp = lf + 128 + rh * 16;
          if (lane < 32) tmp[c] = v;
          wave_sync();
          double z = 0.0, z2 = 0.0;
#pragma unroll
          for (int cc = 0; cc < 16; cc += 2) {
            z = fma(Dg[(6 + j) * 256 + (c >> 2) * 64 + cc + 16 * (c & 3)], tmp[cc], z);
            z2 = fma(Dg[(6 + j) * 256 + (c >> 2) * 64 + cc + 1 + 16 * (c & 3)], tmp[cc + 1], z2);
          }
          z += z2;
          if (lane < 32) zl[16 * j + c] = z;
          wave_sync();
        }
        __builtin_amdgcn_s_setprio(0);
      }
      __syncthreads();
      CH_MARK(10);
    }
    // bordered elimination: y_n = (c_n + mᵀz1)/(μ + mᵀz2), y₁ = −z1 + z2·y_n, w = H y
    double a1 = 0.0, a2 = 0.0;
    for (int i = t; i < n; i += TH) a1 = fma(mvl[i], zv[i], a1), a2 = fma(mvl[i], zv[n64 + i], a2);
    const double mz1 = sum_all(a1), mz2 = sum_all(a2);
    const double yn = (cvl[n] + mz1) / (mvl[n] + mz2);
    double uy = 0.0;
    for (int i = t; i < N; i += TH) uy = fma(u(i), i < n ? -zv[i] + zv[n64 + i] * yn : yn, uy);
    const double uty = sum_all(uy);
    for (int i = t; i < N; i += TH) {
      const double yi = i < n ? -zv[i] + zv[n64 + i] * yn : yn;
      wT[(int64_t)i * P + p] = yi - beta * u(i) * uty;
    }
    __syncthreads();  // the slot and the LDS are reused by the next pixel
    CH_MARK(11);
  }
#ifdef RTI_CHOL_PROFILE
  if (t == 0 && blockIdx.x < 1024)
    for (int k = 0; k < 16; ++k) rti_chol_prof[blockIdx.x][k] = prof_[k];
#endif
}

// fp64 register Gauss-Jordan up to here, rbf_solve_gji above (solve of a 400×400 ROI, MI355X:
// N = 64: 6.3 vs 13.2 ms, N = 96: 27.9 vs 18.1 ms; tools/time_rbf_solve.py)
constexpr int RBF_GJ_MAX_N = 80;
constexpr int RBF_TE = 20;  // divides the reference's 100-wide grid rows (shared qv)

// Measurement overrides (environment, read once): RTI_RBF_GJI_MIN_N lowers the smallest N solved by
// rbf_solve_gji, RTI_RBF_GJI_REFINE = its refinement sweep cap (< 0: exactly that many sweeps).
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
int gji_min_n() {
  static const int v = env_int("RTI_RBF_GJI_MIN_N", RBF_GJ_MAX_N + 1);
  return v;
}
int gji_refine() {
  static const int v = env_int("RTI_RBF_GJI_REFINE", RBF_GJI_MAX_REFINE);
  return v;
}

bool uses_gji(int N) { return N > RBF_GJ_MAX_N || (N >= 2 && N >= gji_min_n()); }
// (r06) the left-looking matrix-core Cholesky for RBF_LL_MIN_N <= N <= RBF_LL_MAX_N: in fp64 throughout it also
// replaces the fp32 Gauss-Jordan inverses + refinement (and their fp64 fallback) above 128 lights — solve of a
// 400² ROI 32.8 vs 64.4 ms at N = 129, 85.8 vs 104.1 at 200, 88.9 vs 413.3 at 256, while at N <= 128 the
// register-blocked inverse stays faster (27.9 vs 32.2 ms at 128; profiles/r06k_rbf_llt_small_n_ab.log).
// Measurement switches (environment, read per call): RTI_RBF_LLT_MIN_N moves the lower bound, RTI_RBF_CHOL_OLD=1
// turns the left-looking form off (r05's solvers: rbf_solve_gjs / gji above 128, rbf_solve_chol above 256)
constexpr int RBF_LL_MIN_N = 129;
bool uses_llt(int N) {
  const char* lo = getenv("RTI_RBF_LLT_MIN_N");
  if (N < (lo ? atoi(lo) : RBF_LL_MIN_N) || N < 2 || N > RBF_LL_MAX_N) return false;
  const char* e = getenv("RTI_RBF_CHOL_OLD");
  return !(e && atoi(e));
}

// redo / fb_ws: the fallback's pixel list (redo[0] = count, zeroed) and its workspace, when uses_gji(N)
template <typename T>
void launch_solve(const float* lu, const float* lv, const void* I, int N, int64_t P, double* wT, float2* xyT,
                  int* status, int* redo, double* fb_ws, int64_t chol_grid, int64_t fb_grid, int* fallback_px,
                  hipStream_t s) {
  const T* In = static_cast<const T*>(I);
  const dim3 g((unsigned)P);
  if (N > RBF_MAX_N || uses_llt(N)) {  // blocked fp64 Cholesky, one workgroup per CU striding over the pixels
    const unsigned cg = (unsigned)(P < chol_grid ? P : chol_grid);
    if (uses_llt(N)) {  // (r06) left-looking on the matrix cores: two 4-wave pixels per CU, or one 8-wave
      const size_t lds = ll_lds_bytes(N);
      auto kern = N <= RBF_LL_TWO_MAX_N ? rbf_solve_llt<T, RBF_LL_TH> : rbf_solve_llt<T, RBF_LL_TH1>;
      (void)reserve_lds(reinterpret_cast<const void*>(kern), lds);
      hipLaunchKernelGGL(kern, dim3(cg), dim3(N <= RBF_LL_TWO_MAX_N ? RBF_LL_TH : RBF_LL_TH1), lds, s, lu, lv, In, N, P,
                         wT, xyT, status, fb_ws);
      return;
    }
    auto go = [&](auto kern, int nb) {
      const size_t lds = chol_lds_bytes(N, nb);
      (void)reserve_lds(reinterpret_cast<const void*>(kern), lds);
      hipLaunchKernelGGL(kern, dim3(cg), dim3(RBF_CH_THREADS), lds, s, lu, lv, In, N, P, wT, xyT, status, fb_ws);
    };
    if (N > RBF_CH_MAX_N) {  // the panel below the diagonal block solved in place in the slot
      constexpr int NB = RBF_CH_GP_NB;
      auto kern = rbf_solve_chol<NB, T, true>;
      const size_t lds = (size_t)NB * (NB + 1) * sizeof(double);
      hipLaunchKernelGGL(kern, dim3(cg), dim3(RBF_CH_THREADS), lds, s, lu, lv, In, N, P, wT, xyT, status, fb_ws);
      return;
    }
    const int nb = chol_nb(N);
    switch (nb) {
      case 32: go(rbf_solve_chol<32, T>, 32); break;
      case 16: go(rbf_solve_chol<16, T>, 16); break;
      case 8: go(rbf_solve_chol<8, T>, 8); break;
      case 4: go(rbf_solve_chol<4, T>, 4); break;
      case 2: go(rbf_solve_chol<2, T>, 2); break;
      default: go(rbf_solve_chol<1, T>, 1); break;
    }
    return;
  }
  if (uses_gji(N)) {
    if (N <= 128)
      hipLaunchKernelGGL((rbf_solve_gji<16, T>), g, dim3(256), 0, s, lu, lv, In, N, P, wT, xyT, status, redo,
                         gji_refine());
    else if (N <= GjsShape<32>::MAX_N)
      hipLaunchKernelGGL((rbf_solve_gjs<32, T>), g, dim3(GjsShape<32>::THREADS), 0, s, lu, lv, In, N, P, wT, xyT,
                         status, redo, gji_refine());
    else
      hipLaunchKernelGGL((rbf_solve_gji<32, T>), g, dim3(1024), 0, s, lu, lv, In, N, P, wT, xyT, status, redo,
                         gji_refine());
    const unsigned fg = (unsigned)(P < fb_grid ? P : fb_grid);
    if (fb_in_lds(N)) {
      const size_t mb = (size_t)N * (N + 1) * sizeof(double);
      (void)reserve_lds(reinterpret_cast<const void*>(rbf_solve_fp64<T, true>), mb);
      hipLaunchKernelGGL((rbf_solve_fp64<T, true>), dim3(fg), dim3(RBF_FB_THREADS), mb, s, lu, lv, In, N, P, redo,
                         fb_ws, wT, status, fallback_px);
    } else {
      hipLaunchKernelGGL((rbf_solve_fp64<T, false>), dim3(fg), dim3(RBF_FB_THREADS), 0, s, lu, lv, In, N, P, redo,
                         fb_ws, wT, status, fallback_px);
    }
    return;
  }
#define RBF_GJ(NM)                                                                                       \
  hipLaunchKernelGGL((rbf_solve_gj<NM, T>), g, dim3(GjSolve<NM, T>::THREADS), 0, s, lu, lv, In, N, P, wT, \
                     xyT, status)
  if (N <= 16) RBF_GJ(16);
  else if (N <= 32) RBF_GJ(32);
  else if (N <= 48) RBF_GJ(48);
  else if (N <= 64) RBF_GJ(64);
  else RBF_GJ(80);
#undef RBF_GJ
}

// grid x = eval groups, y = 64-pixel tiles (consecutive blocks share a tile's nodes and weights in
// L2); more than 65535 tiles (P > 4.19 M) go out as several launches over pixel ranges
template <typename TO>
void launch_eval(int ol, const double* wT, const float2* xyT, int N, int64_t P, const double* luv, int E, void* out,
                 hipStream_t s) {
  constexpr int64_t TILES = 65535;
  const unsigned gx = (unsigned)((E + 4 * RBF_TE - 1) / (4 * RBF_TE));
  for (int64_t pb = 0; pb < P; pb += TILES * 64) {
    const int64_t tiles = (P - pb + 63) / 64 < TILES ? (P - pb + 63) / 64 : TILES;
    const dim3 g(gx, (unsigned)tiles);
    if (ol == RTI_OUT_PIXEL_MAJOR)
      hipLaunchKernelGGL((rbf_eval<RBF_TE, TO, RTI_OUT_PIXEL_MAJOR>), g, dim3(256), 0, s, wT, xyT, N, P, luv, E,
                         static_cast<TO*>(out), pb);
    else
      hipLaunchKernelGGL((rbf_eval<RBF_TE, TO, RTI_OUT_EVAL_MAJOR>), g, dim3(256), 0, s, wT, xyT, N, P, luv, E,
                         static_cast<TO*>(out), pb);
  }
}

}  // namespace
}  // namespace rti

using namespace rti;


extern "C" int64_t rti_rbf_last_chol_grid(void) { return rbf_last_chol_grid_v; }

extern "C" int rti_rbf_perpixel(const float* lu, const float* lv, const void* I, int in_dtype, int N, int64_t P,
                                const double* luv, int E, void* out, int out_dtype, int out_layout, int* status,
                                rti_stream_t stream) {
  return rti_rbf_perpixel_ex(lu, lv, I, in_dtype, N, P, luv, E, out, out_dtype, out_layout, status, nullptr, stream);
}

extern "C" int rti_rbf_perpixel_ex(const float* lu, const float* lv, const void* I, int in_dtype, int N, int64_t P,
                                   const double* luv, int E, void* out, int out_dtype, int out_layout, int* status,
                                   int* fallback_px, rti_stream_t stream) {
  if (!lu || !lv || !I || !luv || !out || !status) return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: null pointer");
  if (N <= 0 || P <= 0 || E <= 0) return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: N, P, E must be positive");
  if (N > RBF_GP_MAX_N)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: N=%d > %d lights", N, RBF_GP_MAX_N);
  if (P > 0x7fffffff) return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: P too large for one launch");
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: input dtype %d", in_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: out dtype %d", out_dtype);
  if (out_layout != RTI_OUT_PIXEL_MAJOR && out_layout != RTI_OUT_EVAL_MAJOR)
    return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: out layout %d", out_layout);
  if ((int64_t)((E + 4 * RBF_TE - 1) / (4 * RBF_TE)) > 0x7fffffff)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: grid too large (E=%d)", E);
  hipStream_t s = (hipStream_t)stream;
  // workspace: per-pixel weights and nodes, node-major ([N][P]) for the coalesced evaluation
  void* ws = nullptr;
  // + for the block solvers: the fp64 fallback's pixel list and (N > RBF_FB_LDS_N) per-workgroup matrices
  const bool chol = N > RBF_MAX_N || uses_llt(N), fb = !chol && uses_gji(N);
  // the Cholesky path: one workgroup (and one [ld][ld] fp64 slot) per CU, striding over the pixels
  int64_t chol_grid = chol ? (uses_llt(N) && N <= RBF_LL_TWO_MAX_N ? 2 * (int64_t)device_cus() : device_cus()) : 0;
  if (chol_grid > P) chol_grid = P;
  const int64_t slot_doubles = N > RBF_CH_MAX_N ? chol_slot_doubles_gp(N) : uses_llt(N) ? ll_slot_doubles(N)
                                                                                 : chol_slot_doubles(N);
  const size_t node_bytes = (size_t)N * P * (sizeof(double) + sizeof(float2));
  if (chol && N > RBF_CH_MAX_N) {  // GP slots (≈ 4·N² bytes each): as many workgroups as the budget holds
    const int64_t fit = (int64_t)(gp_ws_budget(node_bytes) / ((size_t)slot_doubles * sizeof(double)));
    chol_grid = fit < 1 ? 1 : (fit < chol_grid ? fit : chol_grid);
  }
  const int64_t fb_grid = fb ? (P < device_cus() ? P : device_cus()) : 0;
  const size_t fb_ws_bytes = fb ? (fb_in_lds(N) ? 0 : (size_t)fb_grid * N * (N + 1) * sizeof(double))
                                : (chol ? (size_t)chol_grid * slot_doubles * sizeof(double) : 0);
  const size_t flag_bytes = fb ? ((size_t)(P + 1) * sizeof(int) + 255) / 256 * 256 : 0;  // count + pixel list
  size_t fb_ws_bytes_v = fb_ws_bytes;
  size_t bytes = node_bytes + fb_ws_bytes_v + flag_bytes;
  while (hipMallocAsync(&ws, bytes, s) != hipSuccess) {
    // the GP path strides over the pixels from any number of slots: retry with half as many before failing
    if (!(chol && N > RBF_CH_MAX_N && chol_grid > 1))
      return fail(RTI_ERR_HIP, "rti_rbf_perpixel: workspace allocation of %zu bytes failed", bytes);
    (void)hipGetLastError();
    chol_grid = (chol_grid + 1) / 2;
    fb_ws_bytes_v = (size_t)chol_grid * slot_doubles * sizeof(double);
    bytes = node_bytes + fb_ws_bytes_v + flag_bytes;
  }
  rbf_last_chol_grid_v = chol ? chol_grid : 0;
  double* wT = static_cast<double*>(ws);
  float2* xyT = reinterpret_cast<float2*>(wT + (size_t)N * P);
  double* fb_ws = reinterpret_cast<double*>(xyT + (size_t)N * P);
  int* redo = reinterpret_cast<int*>(reinterpret_cast<char*>(fb_ws) + fb_ws_bytes_v);
  if (fb && hipMemsetAsync(redo, 0, sizeof(int), s) != hipSuccess) {
    (void)hipFreeAsync(ws, s);
    return fail(RTI_ERR_HIP, "rti_rbf_perpixel: clearing the fallback count failed");
  }
  switch (in_dtype) {
    case RTI_F32: launch_solve<float>(lu, lv, I, N, P, wT, xyT, status, redo, fb_ws, chol_grid, fb_grid, fallback_px, s); break;
    case RTI_I32: launch_solve<int32_t>(lu, lv, I, N, P, wT, xyT, status, redo, fb_ws, chol_grid, fb_grid, fallback_px, s); break;
    default: launch_solve<uint8_t>(lu, lv, I, N, P, wT, xyT, status, redo, fb_ws, chol_grid, fb_grid, fallback_px, s); break;
  }
  switch (out_dtype) {
    case RTI_F64: launch_eval<double>(out_layout, wT, xyT, N, P, luv, E, out, s); break;
    case RTI_F32: launch_eval<float>(out_layout, wT, xyT, N, P, luv, E, out, s); break;
    case RTI_I32: launch_eval<int32_t>(out_layout, wT, xyT, N, P, luv, E, out, s); break;
    default: launch_eval<uint8_t>(out_layout, wT, xyT, N, P, luv, E, out, s); break;
  }
  const int rc = check_launch("rti_rbf_perpixel");
  (void)hipFreeAsync(ws, s);
  return rc;
}
