// rti_residual.hip -- per-pixel fit residuals of the shared-direction fit on gfx950.
//
// The reference never reports how well _interpolate_PTM's least-squares solution
// (analysis.py:280-298) explains a pixel's N samples; the north_star asks for the
// per-pixel residual next to the coefficients.  For a shared light set the design
// matrix A[N][k] is the same for every pixel, so
//     ss[c][p]  = Σ_n (I[c][n][p] − Σ_i A[n][i] · coef[c][p][i])²
//     res[c][p] = sqrt(ss / N)                       (RMS residual, intensity units)
//     partial[c][b] = Σ_{p in workgroup b} ss[c][p]  (fp64, one per workgroup)
// The single-pass identity ‖I‖² − cᵀAᵀA c cancels catastrophically in fp32 (‖I‖² ≈ 4e6
// against residual energies of a few hundred at N=100), so this is a second stream
// over the intensity stack, HBM-bound like the fit: 4 + 4(k+1)/N bytes per pixel·light.
//
// One lane owns VEC adjacent pixels: their k coefficients are loaded once, then every
// light plane is one 16-B load; A's row n is wave-uniform (scalar loads into SGPRs).
// The per-workgroup sum is a wavefront reduction (DPP/shuffle, fp64) plus one LDS
// exchange between the 4 waves, written by lane 0 with a plain vector store: no atomics,
// so the partial sums are deterministic.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "rti_internal.h"

namespace rti {
namespace {

constexpr int RES_THREADS = 256;

template <typename T, int VEC>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&x)[VEC]) {
  if constexpr (VEC == 1) {
    x[0] = (float)__builtin_nontemporal_load(p);
  } else {
    typedef T vec_t __attribute__((ext_vector_type(VEC)));
    const vec_t v = __builtin_nontemporal_load(reinterpret_cast<const vec_t*>(p));
#pragma unroll
    for (int i = 0; i < VEC; ++i) x[i] = (float)v[i];
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Wide lanes (as the fit): a wave owns NC·64·VEC consecutive pixels and
// lane l's chunk j is the VEC pixels at wave_base + j·64·VEC + VEC·l, so the wave's NC loads
// of one light plane cover NC KiB contiguous (VEC = 4, fp32).
template <int K, int VEC, int NC, typename T>
__global__ __launch_bounds__(RES_THREADS) void fit_residual_k(const float* __restrict__ A, int N,
                                                             const T* __restrict__ I, int64_t P,
                                                             int64_t lstride, int64_t cstride,
                                                             const float* __restrict__ coef, int layout,
                                                             int64_t ocstride, float* __restrict__ res,
                                                             double* __restrict__ partial, int64_t pstride) {
  const int c = blockIdx.y;
  const int64_t wave = ((int64_t)blockIdx.x * RES_THREADS + threadIdx.x) >> 6;
  const int64_t base = wave * (NC * 64 * VEC) + (threadIdx.x & 63) * VEC;
  const T* Ic = I + c * cstride;
  const float* cc = coef + c * ocstride;
  double mine = 0.0;
  bool live[NC];
  float a[NC][VEC][K];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int64_t p0 = base + j * 64 * VEC;
    live[j] = p0 < P;
    if (!live[j]) continue;
    if (layout == RTI_COEF_PIXEL_MAJOR) {
#pragma unroll
      for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int i = 0; i < K; ++i) a[j][v][i] = cc[(p0 + v) * K + i];
    } else {
#pragma unroll
      for (int i = 0; i < K; ++i) {
        float x[VEC];
        load_vec<float, VEC>(cc + i * P + p0, x);
#pragma unroll
        for (int v = 0; v < VEC; ++v) a[j][v][i] = x[v];
      }
    }
  }
  float ss[NC][VEC] = {};
  for (int n = 0; n < N; ++n) {
    float x[NC][VEC];
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (live[j]) load_vec<T, VEC>(Ic + n * lstride + base + j * 64 * VEC, x[j]);
    const float* An = A + (int64_t)n * K;  // wave-uniform row
#pragma unroll
    for (int j = 0; j < NC; ++j) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float pred = 0.f;
#pragma unroll
        for (int i = 0; i < K; ++i) pred = fmaf(An[i], a[j][v][i], pred);
        const float r = x[j][v] - pred;
        ss[j][v] = fmaf(r, r, ss[j][v]);
      }
    }
  }
  const float invN = 1.0f / (float)N;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (!live[j]) continue;
    float out[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      out[v] = sqrtf(ss[j][v] * invN);
      mine += (double)ss[j][v];
    }
    float* rc = res + c * P + base + j * 64 * VEC;
    if constexpr (VEC == 4) {
      *reinterpret_cast<float4*>(rc) = make_float4(out[0], out[1], out[2], out[3]);
    } else {
#pragma unroll
      for (int v = 0; v < VEC; ++v) rc[v] = out[v];
    }
  }
  if (partial) {
    __shared__ double wsum[RES_THREADS / 64];
    const double w = wave_sum(mine);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < RES_THREADS / 64; ++i) t += wsum[i];
      partial[(int64_t)c * pstride + blockIdx.x] = t;
    }
  }
}

struct ResArgs {
  const float* A;
  int k, N;
  const void* I;
  int64_t P, lstride, cstride;
  const float* coef;
  int layout;
  int64_t ocstride;
  float* res;
  double* partial;
  int C;
  hipStream_t s;
};

template <int K, int VEC, int NC, typename T>
int launch_res(const ResArgs& a) {
  const dim3 grid(grid_1d(a.P, RES_THREADS * VEC * NC), a.C);
  hipLaunchKernelGGL((fit_residual_k<K, VEC, NC, T>), grid, dim3(RES_THREADS), 0, a.s, a.A, a.N,
                     static_cast<const T*>(a.I), a.P, a.lstride, a.cstride, a.coef, a.layout, a.ocstride, a.res,
                     a.partial, (int64_t)grid_1d(a.P, RES_THREADS));
  return check_launch("rti_fit_residual");
}

// Chunks per lane, measured at 4K x 100 (profiles/r01_residual_c3_nc_sweep.log): PTM-6
// NC = 1 / 2 / 4 / 8 -> 0.522 / 0.520 / 0.505 / 0.578 ms (8 chunks = 256 VGPRs, 1 wave/SIMD,
// cannot hide the coefficient loads).  HSH-9/16 keep one chunk (wide lanes not measured).
// The wide form needs enough waves to cover the chip (1024 SIMDs, 2 waves each at 4 chunks);
// the cutoff is the fit's heuristic (rti_fit.hip AUTO: >= 2000 waves), not a residual sweep.
constexpr int64_t kResWideMinWaves = 2000;

template <int K, typename T>
int launch_res_v(const ResArgs& a, bool vec4) {
  if (!vec4) return launch_res<K, 1, 1, T>(a);
  if constexpr (K == 6) {
    constexpr int NC = 4;
    if (a.P * a.C / (64 * 4 * NC) >= kResWideMinWaves) return launch_res<K, 4, NC, T>(a);
  }
  return launch_res<K, 4, 1, T>(a);
}

template <typename T>
int launch_res_k(const ResArgs& a, bool vec4) {
  switch (a.k) {
    case 6: return launch_res_v<6, T>(a, vec4);
    case 9: return launch_res_v<9, T>(a, vec4);
    case 16: return launch_res_v<16, T>(a, vec4);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_residual: k=%d (supported: 6, 9, 16)", a.k);
  }
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int64_t rti_fit_residual_blocks(int64_t P) {
  if (P <= 0) return 0;
  // per-channel stride of `partial`: the VEC = 1 grid, so it bounds either launch; entries
  // past the launched grid are not written (the caller zeroes the buffer)
  return (int64_t)grid_1d(P, RES_THREADS);
}

extern "C" int rti_fit_residual(const float* A, int k, int N, const void* I, int in_dtype, int64_t P, int C,
                                int64_t light_stride, int64_t channel_stride, const float* coef, int coef_layout,
                                int64_t coef_channel_stride, float* res, double* partial, rti_stream_t stream) {
  if (!A || !I || !coef || !res) return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: null pointer");
  if (N <= 0 || P <= 0 || C <= 0 || C > 65535) return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: bad N/P/C");
  if (N < k) return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: N=%d < k=%d", N, k);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_residual: input dtype %d", in_dtype);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: coef layout %d", coef_layout);
  ResArgs a;
  a.A = A;
  a.k = k;
  a.N = N;
  a.I = I;
  a.P = P;
  a.lstride = light_stride ? light_stride : P;
  a.cstride = channel_stride ? channel_stride : (int64_t)N * a.lstride;
  a.coef = coef;
  a.layout = coef_layout;
  a.ocstride = coef_channel_stride ? coef_channel_stride : P * k;
  a.res = res;
  a.partial = partial;
  a.C = C;
  a.s = (hipStream_t)stream;
  if (a.lstride < P) return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: light_stride < P");
  if (C > 1 && a.cstride < (int64_t)N * a.lstride) return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: channel_stride");
  if (C > 1 && a.ocstride < P * k) return fail(RTI_ERR_BAD_ARG, "rti_fit_residual: coef_channel_stride");
  const size_t es = in_dtype == RTI_U8 ? 1 : 4;
  const bool vec4 = P % 4 == 0 && a.lstride % 4 == 0 && a.cstride % 4 == 0 && aligned_to(I, 4 * es) &&
                    aligned_to(res, 16) && aligned_to(coef, 16) && a.ocstride % 4 == 0;
  switch (in_dtype) {
    case RTI_F32: return launch_res_k<float>(a, vec4);
    case RTI_U8: return launch_res_k<uint8_t>(a, vec4);
    default: return launch_res_k<int32_t>(a, vec4);
  }
}
