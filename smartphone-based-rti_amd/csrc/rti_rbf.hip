// rti_rbf.hip -- per-pixel linear RBF on gfx950 (the reference's default method
// with its own geometry).
//
// interpolate_intensities (analysis.py:350-363) calls _interpolate_RBF
// (analysis.py:249-260) once per pixel: SciPy Rbf(lx, ly, I, function='linear')
// builds A_ij = ‖x_i − x_j‖ over that pixel's N light directions, solves A w = I
// (LAPACK gesv: LU with partial pivoting) and evaluates f(q) = Σ_j w_j ‖q − x_j‖
// on the 100×100 grid.  Every pixel has its own light list (compute_intensities,
// analysis.py:225-231), so there is no shared operator: one workgroup owns one
// pixel and solves its N×N system — fp64 Gauss-Jordan in registers up to N = 112, fp32 LU in LDS
// + fp64 iterative refinement up to 128, Householder-projected fp32 Cholesky (packed triangle in
// LDS) + fp64 refinement up to 256 (the systems reach cond ≈ 1e4–1e5 at N = 100–200) — and a
// second kernel streams the E evaluations in fp64.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "rti_convert.h"
#include "rti_internal.h"

namespace rti {
namespace {

constexpr int RBF_MAX_N = 128;      // rbf_solve_lds (fp32 LU in LDS) up to here; Householder-Cholesky above
constexpr int RBF_MAX_REFINE = 10;  // refinement sweeps of the fp32-LU fallback

template <typename T>
__device__ __forceinline__ double ldd(const T* p) {
  return (double)*p;
}

// fp64 Euclidean distance between nodes i and j (pdist / cdist 'euclidean').
__device__ __forceinline__ double dist64(double xi, double yi, double xj, double yj) {
  const double dx = xi - xj, dy = yi - yj;
  return sqrt(dx * dx + dy * dy);
}

// ‖·‖ for the evaluation sweep: fp32 rsqrt seed (≤ 2 ulp, 2⁻²² relative) and one fp64
// Newton step, d = s·r + (s − (s·r)²)·r/2, relative error ≲ 2⁻⁴⁴ (≈ 6e-14) — 9 issue slots
// against ≈ 17 for the correctly rounded fp64 sqrt.  With |Σ w_j d_j| terms ≲ 1e5 the
// interpolated value moves by ≲ 1e-8 absolute.  The solve itself (A and the refinement
// residuals) keeps the correctly rounded sqrt.
__device__ __forceinline__ double norm_eval(double s) {
  const double r = (double)__builtin_amdgcn_rsqf(fmaxf((float)s, 1e-30f));
  const double d0 = s * r;
  return fma(fma(-d0, d0, s), 0.5 * r, d0);
}

__device__ __forceinline__ double dist_eval(double qu, double qv, double xj, double yj) {
  const double dx = qu - xj, dy = qv - yj;
  return norm_eval(fma(dy, dy, dx * dx));
}


__device__ __forceinline__ double readlane64(double x, int l) {
  const uint64_t u = __double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// Per-lane view of the fp32 factors for wave 0's triangular solves.  The factorization
// never moves rows: physical row i became the pivot of step so[i]; A[i][k] holds the
// multiplier l_ik for k < so[i] and the U entry u_{so[i],k} for k ≥ so[i].  Lane l owns
// physical rows l and l + 64 (N ≤ 128); the pivot list and the reciprocal diagonal are
// lane-distributed by step and broadcast with readlane.
struct LuLane {
  int r0, r1;    // physical rows (clamped to N − 1 for the address when absent)
  int s0, s1;    // their pivot steps (N when the row does not exist)
  int pk0, pk1;  // piv[lane], piv[lane + 64]
  double rd0, rd1;  // 1 / u_kk for k = lane, lane + 64
};

// z = U⁻¹ L⁻¹ P v on (v0, v1) = v at physical rows (lane, lane + 64); on return the
// value held for physical row i is z at node so[i].  Column-oriented, one wave, the
// chain runs through registers (readlane) and only the factor columns come from LDS.
__device__ __forceinline__ void lu_solve_regs(const float* A, int lda, int N, const LuLane& q, double& v0,
                                              double& v1, int lane) {
  float c0 = A[q.r0 * lda], c1 = A[q.r1 * lda];
  for (int k = 0; k < N; ++k) {  // forward: rows not yet pivoted at step k lose l_ik · y_k
    const float n0 = A[q.r0 * lda + min(k + 1, N - 1)], n1 = A[q.r1 * lda + min(k + 1, N - 1)];
    const int p = __builtin_amdgcn_readlane(k < 64 ? q.pk0 : q.pk1, k & 63);
    const double y = readlane64(p < 64 ? v0 : v1, p & 63);
    if (q.s0 > k) v0 = fma(-(double)c0, y, v0);
    if (q.s1 > k) v1 = fma(-(double)c1, y, v1);
    c0 = n0, c1 = n1;
  }
  c0 = A[q.r0 * lda + N - 1], c1 = A[q.r1 * lda + N - 1];
  for (int k = N - 1; k >= 0; --k) {  // backward: z_k = y_k / u_kk; earlier pivots lose u_ik · z_k
    const float n0 = A[q.r0 * lda + max(k - 1, 0)], n1 = A[q.r1 * lda + max(k - 1, 0)];
    const int p = __builtin_amdgcn_readlane(k < 64 ? q.pk0 : q.pk1, k & 63);
    const double z = readlane64(p < 64 ? v0 : v1, p & 63) * readlane64(k < 64 ? q.rd0 : q.rd1, k & 63);
    if (q.s0 == k) v0 = z;
    if (q.s1 == k) v1 = z;
    if (q.s0 < k) v0 = fma(-(double)c0, z, v0);
    if (q.s1 < k) v1 = fma(-(double)c1, z, v1);
    c0 = n0, c1 = n1;
  }
}

// Fallback for 112 < N ≤ 128 (register budget of rbf_solve_gj).
// One workgroup (4 waves) per pixel.  The distance matrix is factored in fp32 in LDS
// (LU with partial pivoting; 40 KB at N = 100, so several pixels share a CU) and the
// solution is brought to fp64 accuracy by mixed-precision iterative refinement: the
// residual b − A·w is formed in fp64 from the node coordinates (A is never stored in
// fp64) and the correction solved with the fp32 factors.  Each sweep shrinks the error
// by ≈cond(A)·2⁻²⁴ (≤ 6e-3 up to cond 1e5); sweeps stop when the correction stops
// shrinking or falls below 1e-16 of the solution.
//
// Elimination: rows are never swapped.  Wave w owns physical rows i ≡ w (mod 4) and
// keeps the not-yet-pivoted ones in a bit mask; lanes own columns.  Step k updates the
// wave's remaining rows against pivot row p and, in the same pass, lane 0 (column k+1)
// tracks the largest |a_i,k+1| — the next pivot candidate — so a step costs one barrier.
template <typename T>
__global__ void __launch_bounds__(256)
rbf_solve_lds(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
              double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lda = (N + 2) & ~1;  // even row pitch (floats) with ≥ 1 zero pad column: 8-byte pairs
  double* xs = smem;      // [N] node coordinates (fp64 copies of the fp32 light vectors)
  double* ys = xs + N;    // [N]
  double* b = ys + N;     // [N] intensities (the right-hand side)
  double* w = b + N;      // [N] solution, by node
  double* v = w + N;      // [N] residual, by physical row
  int* piv = reinterpret_cast<int*>(v + N);  // [N] pivot row of each step
  int* so = piv + N;                         // [N] pivot step of each row
  float* A = reinterpret_cast<float*>(so + N);  // [N][lda] fp32 LU factors
  __shared__ float s_pmax[2][4];
  __shared__ int s_pidx[2][4];
  __shared__ int s_more;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: row ownership, masks, branches
  const int64_t p = blockIdx.x;
  const int64_t base = p * N;

  for (int j = tid; j < N; j += 256) {
    xs[j] = (double)lu[base + j];  // SciPy holds float64 copies of the float32 nodes
    ys[j] = (double)lv[base + j];
    b[j] = ldd(I + base + j);
  }
  __syncthreads();
  for (int idx = tid; idx < N * lda; idx += 256) {
    const int i = idx / lda, j = idx - i * lda;
    A[idx] = j < N ? (float)dist64(xs[i], ys[i], xs[j], ys[j]) : 0.f;
  }
  __syncthreads();

  uint32_t mask = 0;  // this wave's rows that are not pivots yet (bit s ↔ row wave + 4s)
  {
    const int i = wave + 4 * lane;
    float best = -1.f;
    int bi = N;
    if (lane < 32 && i < N) best = fabsf(A[i * lda]), bi = i;
    mask = __builtin_amdgcn_readfirstlane((uint32_t)__ballot(lane < 32 && i < N));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ob = __shfl_xor(best, off);
      const int oi = __shfl_xor(bi, off);
      if (ob > best || (ob == best && oi < bi)) best = ob, bi = oi;
    }
    if (lane == 0) s_pmax[0][wave] = best, s_pidx[0][wave] = bi;
  }

  bool singular = false;
  for (int k = 0; k < N; ++k) {
    __syncthreads();
    float best = s_pmax[k & 1][0];
    int pr = s_pidx[k & 1][0];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float ob = s_pmax[k & 1][q];
      const int oi = s_pidx[k & 1][q];
      if (ob > best || (ob == best && oi < pr)) best = ob, pr = oi;
    }
    pr = __builtin_amdgcn_readfirstlane(pr);  // identical on every lane
    if (!(best > 0.f)) {  // block-uniform: an exactly zero pivot column
      singular = true;
      break;
    }
    if (tid == 0) piv[k] = pr, so[pr] = k;
    if ((pr & 3) == wave) mask &= ~(1u << (pr >> 2));
    const float inv = 1.f / A[pr * lda + k];
    // lane l owns the column pair (kb + 2l, kb + 2l + 1), kb = k rounded down to even:
    // one 8-byte LDS access per row.  Pivot entries at columns ≤ k are zeroed so those
    // columns pass through unchanged, and column k receives the multiplier l_ik.
    const int kb = k & ~1, c0 = kb + 2 * lane;
    const bool kodd = k & 1;
    float bm = -1.f;
    int bidx = N;
    if (c0 < N) {
      float2 pp = *reinterpret_cast<const float2*>(A + pr * lda + c0);
      if (c0 <= k) pp.x = 0.f;
      if (c0 + 1 <= k) pp.y = 0.f;
      const bool put0 = lane == 0 && !kodd, put1 = lane == 0 && kodd;
      // rows in batches of RB: all LDS reads of a batch are issued before its first use
      constexpr int RB = 8;
      for (uint32_t m = mask; m;) {
        int ri[RB];
        float lk[RB];
        float2 av[RB];
#pragma unroll
        for (int t = 0; t < RB; ++t) {
          ri[t] = m ? wave + 4 * __builtin_ctz(m) : -1;
          m &= m - 1;
        }
#pragma unroll
        for (int t = 0; t < RB; ++t)
          if (ri[t] >= 0) {
            const float* row = A + ri[t] * lda;
            lk[t] = row[k];
            av[t] = *reinterpret_cast<const float2*>(row + c0);
          }
#pragma unroll
        for (int t = 0; t < RB; ++t)
          if (ri[t] >= 0) {
            const float l = lk[t] * inv;
            float2 n;
            n.x = put0 ? l : fmaf(-l, pp.x, av[t].x);
            n.y = put1 ? l : fmaf(-l, pp.y, av[t].y);
            *reinterpret_cast<float2*>(A + ri[t] * lda + c0) = n;
            const float tv = fabsf(kodd ? n.x : n.y);  // column k + 1 on lane (k & 1)
            if (tv > bm) bm = tv, bidx = ri[t];
          }
      }
    }
    if (lane == (k & 1)) s_pmax[(k + 1) & 1][wave] = bm, s_pidx[(k + 1) & 1][wave] = bidx;
  }
  if (singular && tid == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
  __syncthreads();

  if (!singular) {
    LuLane q;
    double v0 = 0.0, v1 = 0.0;
    if (wave == 0) {
      q.r0 = min(lane, N - 1), q.r1 = min(lane + 64, N - 1);
      q.s0 = lane < N ? so[lane] : N, q.s1 = lane + 64 < N ? so[lane + 64] : N;
      q.pk0 = piv[min(lane, N - 1)], q.pk1 = piv[min(lane + 64, N - 1)];
      q.rd0 = 1.0 / (double)A[q.pk0 * lda + min(lane, N - 1)];
      q.rd1 = 1.0 / (double)A[q.pk1 * lda + min(lane + 64, N - 1)];
      v0 = lane < N ? b[lane] : 0.0, v1 = lane + 64 < N ? b[lane + 64] : 0.0;
      lu_solve_regs(A, lda, N, q, v0, v1, lane);
      if (lane < N) w[q.s0] = v0;
      if (lane + 64 < N) w[q.s1] = v1;
    }
    double dprev = __builtin_inf();
    for (int it = 0; it < RBF_MAX_REFINE; ++it) {
      __syncthreads();
      // v = b − A w in fp64, two threads per row (A recomputed from the coordinates)
      {
        const int i = tid >> 1, h = tid & 1;
        double r = 0.0;
        if (i < N) {
          const double xi = xs[i], yi = ys[i];
          for (int j = h; j < N; j += 2) r = fma(-dist64(xi, yi, xs[j], ys[j]), w[j], r);
        }
        r += __shfl_xor(r, 1);
        if (i < N && h == 0) v[i] = b[i] + r;
      }
      __syncthreads();
      if (wave == 0) {
        v0 = lane < N ? v[lane] : 0.0, v1 = lane + 64 < N ? v[lane + 64] : 0.0;
        lu_solve_regs(A, lda, N, q, v0, v1, lane);
        double dn = 0.0, wn = 0.0;
        if (lane < N) {
          const double t = w[q.s0] + v0;
          w[q.s0] = t;
          dn = fabs(v0), wn = fabs(t);
        }
        if (lane + 64 < N) {
          const double t = w[q.s1] + v1;
          w[q.s1] = t;
          dn = fmax(dn, fabs(v1)), wn = fmax(wn, fabs(t));
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          dn = fmax(dn, __shfl_xor(dn, off));
          wn = fmax(wn, __shfl_xor(wn, off));
        }
        // remaining error ≈ ρ·dn with ρ = dn / dprev the observed contraction; stop at the
        // fp64 floor (≈ cond·eps) or when a sweep no longer halves the correction
        if (lane == 0)
          s_more = dn > 1e-16 * wn && dn < 0.5 * dprev && (dprev == __builtin_inf() || (dn / dprev) * dn > 4e-13 * wn);
        dprev = dn;
      }
      __syncthreads();
      if (!s_more) break;  // uniform
    }
  }
  __syncthreads();

  for (int j = tid; j < N; j += 256) {
    wT[(int64_t)j * P + p] = singular ? __builtin_nan("") : w[j];
    xyT[(int64_t)j * P + p] = make_float2(lu[base + j], lv[base + j]);
  }
}

// ---- 128 < N <= 256: Householder-projected Cholesky in LDS + fp64 refinement --------------
// An fp32 LU of a 200×200 system no longer fits 160 KiB of LDS (and a 256×256 one is 256 KiB), but
// the linear-RBF matrix A_ij = ‖x_i − x_j‖ of distinct nodes is symmetric and strictly
// conditionally negative definite (negative definite on 1^⊥).  With the Householder reflector H
// that maps e = 1/√N to the last unit vector, HAH = [M m; mᵀ μ] where M (order n = N − 1) is
// Q̃ᵀAQ̃ on 1^⊥, so S = −M is symmetric positive definite: its fp32 Cholesky factor needs only the
// packed lower triangle (n(n+1)/2 floats, 127.5 KiB at N = 256).  A w = b is then
//   c = H b,  z1 = S⁻¹ c₁,  z2 = S⁻¹ m,  y_n = (c_n + mᵀz1)/(μ + mᵀz2),  y₁ = −z1 + z2·y_n,  w = H y
// (block elimination of the bordered system), used as the approximate inverse of mixed-precision
// iterative refinement exactly as rbf_solve_lds does: residuals b − A·w in fp64 from the node
// coordinates, corrections through the fp32 factor, until the fp64 floor (cond·eps), so the result
// is what SciPy's fp64 LU returns to rounding.  Exactly repeated nodes make A singular (SciPy's
// LinAlgError): they are detected up front; a Cholesky pivot <= 0 (cond far beyond fp32) reports
// the same status.
constexpr int RBF_CH_MAX_N = 256;
constexpr int RBF_CH_THREADS = 512;
constexpr int RBF_CH_MAX_REFINE = 16;

__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }  // packed lower, j <= i

__device__ __forceinline__ double pick4(const double (&v)[4], int q) {
  return q == 0 ? v[0] : (q == 1 ? v[1] : (q == 2 ? v[2] : v[3]));
}

__device__ __forceinline__ double wave_sum64(double t) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  return t;
}

// v ← S⁻¹ v for S = L Lᵀ (packed fp32 L of order n <= 256) on one wave: lane owns entries
// lane + 64s; rd[s] = 1 / L_ii for the same entries.  Column-oriented forward then backward
// substitution; the chain runs through registers (readlane), the next step's factor entries are
// loaded before the current step's update.  Entries >= n are left unchanged.
__device__ __forceinline__ void chol_solve(const float* __restrict__ L, int n, const double (&rd)[4], double (&v)[4],
                                           int lane) {
  float cur[4], nxt[4];
  auto fwd_load = [&](int k, float (&dst)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) dst[s] = L[tri(max(min(lane + 64 * s, n - 1), k), k)];
  };
  fwd_load(0, cur);
  for (int k = 0; k < n; ++k) {
    if (k + 1 < n) fwd_load(k + 1, nxt);
    const int q = k >> 6;
    const double yk = readlane64(pick4(v, q), k & 63) * readlane64(pick4(rd, q), k & 63);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int i = lane + 64 * s;
      if (i == k) v[s] = yk;
      else if (i > k && i < n) v[s] = fma(-(double)cur[s], yk, v[s]);
      cur[s] = nxt[s];
    }
  }
  auto bwd_load = [&](int k, float (&dst)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) dst[s] = L[tri(k, min(lane + 64 * s, k))];
  };
  bwd_load(n - 1, cur);
  for (int k = n - 1; k >= 0; --k) {
    if (k > 0) bwd_load(k - 1, nxt);
    const int q = k >> 6;
    const double xk = readlane64(pick4(v, q), k & 63) * readlane64(pick4(rd, q), k & 63);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int i = lane + 64 * s;
      if (i == k) v[s] = xk;
      else if (i < k) v[s] = fma(-(double)cur[s], xk, v[s]);
      cur[s] = nxt[s];
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(RBF_CH_THREADS)
rbf_solve_chol(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
               double* __restrict__ wT, float2* __restrict__ xyT, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int n = N - 1;
  double* xs = smem;     // [N] nodes (fp64 copies of the fp32 light vectors)
  double* ys = xs + N;   // [N]
  double* b = ys + N;    // [N] right-hand side
  double* w = b + N;     // [N] solution
  double* v = w + N;     // [N] residual
  double* g = v + N;     // [N] A·u
  double* m = g + N;     // [N] (HAH)[·][n]; m[n] = μ
  float* col = reinterpret_cast<float*>(m + N);  // [N] current Cholesky column
  float* S = col + ((N + 3) & ~3);                // packed lower triangle of order n
  __shared__ double s_red;
  __shared__ int s_flag, s_more;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t p = blockIdx.x;
  const int64_t base = p * N;

  for (int j = tid; j < N; j += RBF_CH_THREADS) {
    const float x = lu[base + j], y = lv[base + j];
    xs[j] = (double)x;
    ys[j] = (double)y;
    b[j] = ldd(I + base + j);
    xyT[(int64_t)j * P + p] = make_float2(x, y);
  }
  if (tid == 0) s_flag = 0;
  __syncthreads();
  // exactly repeated nodes: A has two equal rows (SciPy: LinAlgError)
  for (int i = wave; i < N; i += RBF_CH_THREADS / 64)
    for (int j = i + 1 + lane; j < N; j += 64)
      if (xs[i] == xs[j] && ys[i] == ys[j]) s_flag = 1;
  // Householder vector u = e − e_n (e = 1/√N), H = I − β u uᵀ, β = 2/uᵀu = 1/(1 − 1/√N)
  const double e = 1.0 / sqrt((double)N), beta = 1.0 / (1.0 - e);
  auto u = [&](int i) { return i < n ? e : e - 1.0; };
  {  // g = A u, two threads per row
    const int i = tid >> 1, h = tid & 1;
    double r = 0.0;
    if (i < N) {
      const double xi = xs[i], yi = ys[i];
      for (int j = h; j < N; j += 2) r = fma(dist64(xi, yi, xs[j], ys[j]), u(j), r);
    }
    r += __shfl_xor(r, 1);
    if (i < N && h == 0) g[i] = r;
  }
  __syncthreads();
  if (wave == 0) {
    double t = 0.0;
    for (int j = lane; j < N; j += 64) t = fma(u(j), g[j], t);
    t = wave_sum64(t);
    if (lane == 0) s_red = t;
  }
  __syncthreads();
  bool singular = s_flag != 0;  // block-uniform
  if (!singular) {
    const double sg = s_red, b2 = beta * beta * sg;
    auto hah = [&](int i, int j) {
      return dist64(xs[i], ys[i], xs[j], ys[j]) - beta * (u(i) * g[j] + g[i] * u(j)) + b2 * u(i) * u(j);
    };
    for (int i = wave; i < n; i += RBF_CH_THREADS / 64)
      for (int j = lane; j <= i; j += 64) S[tri(i, j)] = (float)(-hah(i, j));
    for (int i = tid; i < N; i += RBF_CH_THREADS) m[i] = hah(i, n);
    __syncthreads();
    // right-looking Cholesky of S: column k scaled, then the trailing triangle updated
    for (int k = 0; k < n; ++k) {
      const float dkk = S[tri(k, k)];
      if (!(dkk > 0.f)) {  // uniform (one LDS word after a barrier)
        singular = true;
        break;
      }
      const float d = sqrtf(dkk), inv = 1.f / d;
      for (int i = k + 1 + tid; i < n; i += RBF_CH_THREADS) {
        const float l = S[tri(i, k)] * inv;
        S[tri(i, k)] = l;
        col[i] = l;
      }
      __syncthreads();
      if (tid == 0) S[tri(k, k)] = d;
      for (int i = k + 1 + wave; i < n; i += RBF_CH_THREADS / 64) {
        const float li = col[i];
        float* row = S + tri(i, 0);
        for (int j = k + 1 + lane; j <= i; j += 64) row[j] = fmaf(-li, col[j], row[j]);
      }
      __syncthreads();
    }
  }
  if (!singular) {
    double rd[4], z2[4], mr[4], wr[4];
    double mz2 = 0.0, mu = 0.0;
    if (wave == 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int i = lane + 64 * s;
        rd[s] = i < n ? 1.0 / (double)S[tri(i, i)] : 0.0;
        mr[s] = i < n ? m[i] : 0.0;
        z2[s] = mr[s];
      }
      mu = m[n];
      chol_solve(S, n, rd, z2, lane);
      double t = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) t = fma(mr[s], z2[s], t);
      mz2 = wave_sum64(t);
    }
    // A⁻¹ r through the bordered Householder system; r: entries lane + 64s (wave 0)
    auto solve = [&](double (&r)[4]) {
      double t = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) t = fma(lane + 64 * s < N ? u(lane + 64 * s) : 0.0, r[s], t);
      const double ub = wave_sum64(t);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int i = lane + 64 * s;
        r[s] = i < N ? fma(-beta * u(i), ub, r[s]) : 0.0;  // c = H r
      }
      const double cn = readlane64(pick4(r, n >> 6), n & 63);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (lane + 64 * s >= n) r[s] = 0.0;
      chol_solve(S, n, rd, r, lane);  // z1
      t = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) t = fma(mr[s], r[s], t);
      const double yn = (cn + wave_sum64(t)) / (mu + mz2);
      t = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int i = lane + 64 * s;
        r[s] = i < n ? fma(z2[s], yn, -r[s]) : (i == n ? yn : 0.0);
        t = fma(i < N ? u(i) : 0.0, r[s], t);
      }
      const double uy = wave_sum64(t);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int i = lane + 64 * s;
        if (i < N) r[s] = fma(-beta * u(i), uy, r[s]);  // w = H y
      }
    };
    if (wave == 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s) wr[s] = lane + 64 * s < N ? b[lane + 64 * s] : 0.0;
      solve(wr);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (lane + 64 * s < N) w[lane + 64 * s] = wr[s];
    }
    double dprev = __builtin_inf();
    for (int it = 0; it < RBF_CH_MAX_REFINE; ++it) {
      __syncthreads();
      {  // v = b − A w in fp64, two threads per row
        const int i = tid >> 1, h = tid & 1;
        double r = 0.0;
        if (i < N) {
          const double xi = xs[i], yi = ys[i];
          for (int j = h; j < N; j += 2) r = fma(-dist64(xi, yi, xs[j], ys[j]), w[j], r);
        }
        r += __shfl_xor(r, 1);
        if (i < N && h == 0) v[i] = b[i] + r;
      }
      __syncthreads();
      if (wave == 0) {
        double dv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) dv[s] = lane + 64 * s < N ? v[lane + 64 * s] : 0.0;
        solve(dv);
        double dn = 0.0, wn = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int i = lane + 64 * s;
          if (i < N) {
            wr[s] += dv[s];
            w[i] = wr[s];
            dn = fmax(dn, fabs(dv[s]));
            wn = fmax(wn, fabs(wr[s]));
          }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          dn = fmax(dn, __shfl_xor(dn, off));
          wn = fmax(wn, __shfl_xor(wn, off));
        }
        if (lane == 0)
          s_more = dn > 1e-16 * wn && dn < 0.5 * dprev && (dprev == __builtin_inf() || (dn / dprev) * dn > 4e-13 * wn);
        dprev = dn;
      }
      __syncthreads();
      if (!s_more) break;  // uniform
    }
  }
  if (singular && tid == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);
  __syncthreads();
  for (int j = tid; j < N; j += RBF_CH_THREADS) wT[(int64_t)j * P + p] = singular ? __builtin_nan("") : w[j];
}

size_t rbf_chol_lds(int N) {
  const int n = N - 1;
  return 7 * (size_t)N * sizeof(double) + (size_t)((N + 3) & ~3) * sizeof(float) +
         (size_t)n * (n + 1) / 2 * sizeof(float);
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

// Per-pixel solve for N ≤ NMAX ≤ 112: Gauss-Jordan elimination with partial pivoting in
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
         const double* __restrict__ luv, int E, TO* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int e0 = (blockIdx.x * 4 + wave) * TE;
  if (e0 >= E) return;  // wave-uniform
  const int64_t p = (int64_t)blockIdx.y * 64 + lane;
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
      const double x = xy.x, dy = qv[0] - (double)xy.y, dy2 = dy * dy;
#pragma unroll
      for (int i = 0; i < TE; ++i) {
        const double dx = qu[i] - x;
        acc[i] = fma(w, norm_eval(fma(dx, dx, dy2)), acc[i]);
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

constexpr int RBF_GJ_MAX_N = 112;
constexpr int RBF_TE = 20;  // divides the reference's 100-wide grid rows (shared qv)

template <typename T>
void launch_solve(const float* lu, const float* lv, const void* I, int N, int64_t P, double* wT, float2* xyT,
                  int* status, hipStream_t s) {
  const T* In = static_cast<const T*>(I);
  const dim3 g((unsigned)P);
#define RBF_GJ(NM)                                                                                       \
  hipLaunchKernelGGL((rbf_solve_gj<NM, T>), g, dim3(GjSolve<NM, T>::THREADS), 0, s, lu, lv, In, N, P, wT, \
                     xyT, status)
  if (N <= 16) RBF_GJ(16);
  else if (N <= 32) RBF_GJ(32);
  else if (N <= 48) RBF_GJ(48);
  else if (N <= 64) RBF_GJ(64);
  else if (N <= 80) RBF_GJ(80);
  else if (N <= 96) RBF_GJ(96);
  else if (N <= RBF_GJ_MAX_N) RBF_GJ(112);
  else if (N > RBF_MAX_N) {
    const size_t lds = rbf_chol_lds(N);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rbf_solve_chol<T>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((rbf_solve_chol<T>), g, dim3(RBF_CH_THREADS), lds, s, lu, lv, In, N, P, wT, xyT, status);
  } else {
    const size_t lds = 5 * (size_t)N * sizeof(double) + 2 * (size_t)N * sizeof(int) + (size_t)N * ((N + 2) & ~1) * sizeof(float);
    if (lds > 65536)  // opt in to more than 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rbf_solve_lds<T>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((rbf_solve_lds<T>), g, dim3(256), lds, s, lu, lv, In, N, P, wT, xyT, status);
  }
#undef RBF_GJ
}

template <typename TO>
void launch_eval(int ol, const double* wT, const float2* xyT, int N, int64_t P, const double* luv, int E, void* out,
                 hipStream_t s) {
  const dim3 g((unsigned)((E + 4 * RBF_TE - 1) / (4 * RBF_TE)), (unsigned)((P + 63) / 64));
  if (ol == RTI_OUT_PIXEL_MAJOR)
    hipLaunchKernelGGL((rbf_eval<RBF_TE, TO, RTI_OUT_PIXEL_MAJOR>), g, dim3(256), 0, s, wT, xyT, N, P, luv, E,
                       static_cast<TO*>(out));
  else
    hipLaunchKernelGGL((rbf_eval<RBF_TE, TO, RTI_OUT_EVAL_MAJOR>), g, dim3(256), 0, s, wT, xyT, N, P, luv, E,
                       static_cast<TO*>(out));
}

}  // namespace
}  // namespace rti

using namespace rti;


extern "C" int rti_rbf_perpixel(const float* lu, const float* lv, const void* I, int in_dtype, int N, int64_t P,
                                const double* luv, int E, void* out, int out_dtype, int out_layout, int* status,
                                rti_stream_t stream) {
  if (!lu || !lv || !I || !luv || !out || !status) return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: null pointer");
  if (N <= 0 || P <= 0 || E <= 0) return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: N, P, E must be positive");
  if (N > RBF_CH_MAX_N) return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: N=%d > %d lights", N, RBF_CH_MAX_N);
  if (P > 0x7fffffff) return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: P too large for one launch");
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: input dtype %d", in_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: out dtype %d", out_dtype);
  if (out_layout != RTI_OUT_PIXEL_MAJOR && out_layout != RTI_OUT_EVAL_MAJOR)
    return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: out layout %d", out_layout);
  if ((int64_t)((E + 4 * RBF_TE - 1) / (4 * RBF_TE)) > 0x7fffffff || (P + 63) / 64 > 65535)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: grid too large (P=%lld, E=%d)", (long long)P, E);
  hipStream_t s = (hipStream_t)stream;
  // workspace: per-pixel weights and nodes, node-major ([N][P]) for the coalesced evaluation
  void* ws = nullptr;
  if (hipMallocAsync(&ws, (size_t)N * P * (sizeof(double) + sizeof(float2)), s) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_rbf_perpixel: workspace allocation of %zu bytes failed",
                (size_t)N * P * (sizeof(double) + sizeof(float2)));
  double* wT = static_cast<double*>(ws);
  float2* xyT = reinterpret_cast<float2*>(wT + (size_t)N * P);
  switch (in_dtype) {
    case RTI_F32: launch_solve<float>(lu, lv, I, N, P, wT, xyT, status, s); break;
    case RTI_I32: launch_solve<int32_t>(lu, lv, I, N, P, wT, xyT, status, s); break;
    default: launch_solve<uint8_t>(lu, lv, I, N, P, wT, xyT, status, s); break;
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
