// rti_rbf.hip -- per-pixel linear RBF on gfx950 (the reference's default method
// with its own geometry).
//
// interpolate_intensities (analysis.py:350-363) calls _interpolate_RBF
// (analysis.py:249-260) once per pixel: SciPy Rbf(lx, ly, I, function='linear')
// builds A_ij = ‖x_i − x_j‖ over that pixel's N light directions, solves A w = I
// (LAPACK gesv: LU with partial pivoting) and evaluates f(q) = Σ_j w_j ‖q − x_j‖
// on the 100×100 grid.  Every pixel has its own light list (compute_intensities,
// analysis.py:225-231), so there is no shared operator: one workgroup owns one
// pixel, factors its N×N system in LDS in fp64 (the systems reach cond ≈ 1e4–1e5
// at N = 100–200) and streams the E evaluations, one query per lane.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "rti_convert.h"
#include "rti_internal.h"

namespace rti {
namespace {

constexpr int RBF_MAX_N = 128;

template <typename T>
__device__ __forceinline__ double ldd(const T* p) {
  return (double)*p;
}

template <typename T, typename TO, int OL>
__global__ void __launch_bounds__(256)
rbf_perpixel(const float* __restrict__ lu, const float* __restrict__ lv, const T* __restrict__ I, int N, int64_t P,
             const double* __restrict__ luv, int E, TO* __restrict__ out, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lda = N + 1;  // odd row pitch: column walks do not hit one bank
  double* A = smem;                       // [N][lda]
  double* xs = A + (size_t)N * lda;       // [N]
  double* ys = xs + N;                    // [N]
  double* d = ys + N;                     // [N] right-hand side, then the solution w
  __shared__ int s_piv;
  __shared__ int s_sing;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t p = blockIdx.x;
  const int64_t base = p * N;

  for (int j = tid; j < N; j += 256) {
    xs[j] = (double)lu[base + j];  // SciPy holds float64 copies of the float32 nodes
    ys[j] = (double)lv[base + j];
    d[j] = ldd(I + base + j);
  }
  if (tid == 0) s_sing = 0;
  __syncthreads();
  for (int idx = tid; idx < N * N; idx += 256) {
    const int i = idx / N, j = idx - i * N;
    const double dx = xs[i] - xs[j], dy = ys[i] - ys[j];
    A[i * lda + j] = sqrt(dx * dx + dy * dy);
  }
  __syncthreads();

  // ---- LU with partial pivoting; the row operations are applied to d on the fly ----
  for (int k = 0; k < N; ++k) {
    if (wave == 0) {  // pivot: first row with the largest |A[i][k]|, i >= k (idamax)
      double best = -1.0;
      int bi = N;
      for (int i = k + lane; i < N; i += 64) {
        const double v = fabs(A[i * lda + k]);
        if (v > best) best = v, bi = i;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        if (ob > best || (ob == best && oi < bi)) best = ob, bi = oi;
      }
      if (lane == 0) {
        s_piv = bi;
        if (!(best > 0.0)) s_sing = 1;
      }
    }
    __syncthreads();
    const int pv = s_piv;
    if (s_sing) break;  // uniform across the workgroup
    if (pv != k) {
      for (int j = k + tid; j < N; j += 256) {
        const double t = A[k * lda + j];
        A[k * lda + j] = A[pv * lda + j];
        A[pv * lda + j] = t;
      }
      if (tid == 0) {
        const double t = d[k];
        d[k] = d[pv];
        d[pv] = t;
      }
      __syncthreads();
    }
    const double inv = 1.0 / A[k * lda + k];
    for (int i = k + 1 + tid; i < N; i += 256) A[i * lda + k] *= inv;  // multipliers l_i
    __syncthreads();
    const int m = N - k - 1;
    const double dk = d[k];
    for (int idx = tid; idx < m * (m + 1); idx += 256) {  // trailing update, plus column N = rhs
      const int ii = idx / (m + 1), jj = idx - ii * (m + 1);
      const int i = k + 1 + ii;
      const double l = A[i * lda + k];
      if (jj < m) {
        const int j = k + 1 + jj;
        A[i * lda + j] = fma(-l, A[k * lda + j], A[i * lda + j]);
      } else {
        d[i] = fma(-l, dk, d[i]);
      }
    }
    __syncthreads();
  }
  const bool singular = s_sing != 0;
  if (singular && tid == 0) atomicExch(status, (int)RTI_ERR_SINGULAR);

  // ---- back substitution U w = d, one wave (lock-step; LDS ordered within the wave) ----
  if (!singular && wave == 0) {
    for (int i = N - 1; i >= 0; --i) {
      const double wi = d[i] / A[i * lda + i];
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) d[i] = wi;
      for (int j = lane; j < i; j += 64) d[j] = fma(-A[j * lda + i], wi, d[j]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();

  // ---- evaluate f(q_e) = Σ_j w_j ‖q_e − x_j‖ (cdist · nodes, analysis.py:260) ----
  for (int e = tid; e < E; e += 256) {
    double f;
    if (singular) {
      f = __builtin_nan("");
    } else {
      const double qu = luv[2 * e], qv = luv[2 * e + 1];
      f = 0.0;
      for (int j = 0; j < N; ++j) {
        const double dx = qu - xs[j], dy = qv - ys[j];
        f = fma(d[j], sqrt(dx * dx + dy * dy), f);
      }
    }
    if constexpr (OL == RTI_OUT_PIXEL_MAJOR)
      out[p * E + e] = cvt_out<TO>(f);
    else
      out[(int64_t)e * P + p] = cvt_out<TO>(f);
  }
}

template <typename T, typename TO>
void launch_ol(int ol, const float* lu, const float* lv, const void* I, int N, int64_t P, const double* luv, int E,
               void* out, int* status, hipStream_t s) {
  const size_t lds = ((size_t)N * (N + 1) + 3 * (size_t)N) * sizeof(double);
  if (lds > 65536) {  // opt in to more than 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rbf_perpixel<T, TO, RTI_OUT_PIXEL_MAJOR>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rbf_perpixel<T, TO, RTI_OUT_EVAL_MAJOR>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  if (ol == RTI_OUT_PIXEL_MAJOR)
    hipLaunchKernelGGL((rbf_perpixel<T, TO, RTI_OUT_PIXEL_MAJOR>), dim3((unsigned)P), dim3(256), lds, s, lu, lv,
                       static_cast<const T*>(I), N, P, luv, E, static_cast<TO*>(out), status);
  else
    hipLaunchKernelGGL((rbf_perpixel<T, TO, RTI_OUT_EVAL_MAJOR>), dim3((unsigned)P), dim3(256), lds, s, lu, lv,
                       static_cast<const T*>(I), N, P, luv, E, static_cast<TO*>(out), status);
}

template <typename T>
void launch_out(int odt, int ol, const float* lu, const float* lv, const void* I, int N, int64_t P, const double* luv,
                int E, void* out, int* status, hipStream_t s) {
  switch (odt) {
    case RTI_F64: launch_ol<T, double>(ol, lu, lv, I, N, P, luv, E, out, status, s); break;
    case RTI_F32: launch_ol<T, float>(ol, lu, lv, I, N, P, luv, E, out, status, s); break;
    case RTI_I32: launch_ol<T, int32_t>(ol, lu, lv, I, N, P, luv, E, out, status, s); break;
    default: launch_ol<T, uint8_t>(ol, lu, lv, I, N, P, luv, E, out, status, s); break;
  }
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_rbf_perpixel(const float* lu, const float* lv, const void* I, int in_dtype, int N, int64_t P,
                                const double* luv, int E, void* out, int out_dtype, int out_layout, int* status,
                                rti_stream_t stream) {
  if (!lu || !lv || !I || !luv || !out || !status) return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: null pointer");
  if (N <= 0 || P <= 0 || E <= 0) return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: N, P, E must be positive");
  if (N > RBF_MAX_N) return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: N=%d > %d lights", N, RBF_MAX_N);
  if (P > 0x7fffffff) return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: P too large for one launch");
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: input dtype %d", in_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_rbf_perpixel: out dtype %d", out_dtype);
  if (out_layout != RTI_OUT_PIXEL_MAJOR && out_layout != RTI_OUT_EVAL_MAJOR)
    return fail(RTI_ERR_BAD_ARG, "rti_rbf_perpixel: out layout %d", out_layout);
  hipStream_t s = (hipStream_t)stream;
  switch (in_dtype) {
    case RTI_F32: launch_out<float>(out_dtype, out_layout, lu, lv, I, N, P, luv, E, out, status, s); break;
    case RTI_I32: launch_out<int32_t>(out_dtype, out_layout, lu, lv, I, N, P, luv, E, out, status, s); break;
    default: launch_out<uint8_t>(out_dtype, out_layout, lu, lv, I, N, P, luv, E, out, status, s); break;
  }
  return check_launch("rti_rbf_perpixel");
}
