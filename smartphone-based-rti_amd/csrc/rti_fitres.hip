// rti_fitres.hip -- shared-direction fit AND per-pixel residuals in one HBM pass (gfx950).
//
// The reference solves each pixel's least squares (analysis.py:280-298) and never reports how
// well the solution explains the N samples; the north_star asks for per-pixel residuals from
// wavefront reductions next to the coefficients.  rti_fit_residual does that as a second stream
// over the stack; this kernel reads the stack ONCE:
//
//     b[c][p]   = Aᵀ I[c][·][p]            (k fp64 accumulators per pixel, A = design [N][k])
//     q[c][p]   = ‖I[c][·][p]‖²            (fp64)
//     coef      = G⁺ b                     (G⁺ = (AᵀA)⁺ = V Σ⁻² Vᵀ from the host SVD, so G⁺Aᵀ = pinv)
//     ss        = q − coefᵀ b = ‖I − A·coef‖²  (the least-squares residual energy)
//     res[c][p] = sqrt(ss / N),  partial[c][blk] = Σ ss over the workgroup (fp64)
//
// or, with the thin SVD factors A = U Σ Vᵀ instead of (A, G⁺) (rti_fit_shared_residual_svd, the
// reference's own solve, analysis.py:295-298: c = uᵀL, w = c/s, a = vᵀw):
//
//     y         = Uᵀ I                     (k fp64 accumulators per pixel, U orthonormal [N][k])
//     coef      = (V Σ⁻¹) y
//     ss        = q − yᵀ y                 (‖I‖² minus the energy of its projection on range(A))
//
// The SVD form never forms AᵀA: its coefficients carry cond(A)·1e-16 relative error like the
// reference's SVD, where the Gram form's carry cond(A)²·1e-16 (near-collinear lights,
// tests/golden/ptm_edge.npz: 2.7e-7 vs 1e-15 of max|c| at cond(A) = 1.1e8).
//
// fp32 × fp32 products are exact in fp64, so b and q carry ~1e-16 relative error and the
// subtraction q − coefᵀb (≈4e6 − 4e6 → ≈400 at N = 100, 8-bit data) keeps ~1e-9 absolute:
// the one-pass identity that cancels catastrophically in fp32 (rti_residual.hip) is exact enough
// in fp64.  Coefficients come out of fp64 accumulation (rounded once to fp32), tighter than the
// fp32 stream of rti_fit_shared.
//
// Layout and lane map as fit_shared_valu (rti_fit.hip): a wave owns NC·64·VEC consecutive pixels,
// lane l's chunk c is the VEC pixels at wave_base + c·64·VEC + VEC·l, one 16-B non-temporal load
// per chunk and light plane; A's row and G⁺ are wave-uniform (scalar loads).  The fp64 state is
// 2k + 2 VGPRs per pixel, which caps the wide-lane run length.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "rti_internal.h"

namespace rti {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr int FR_THREADS = 256;

template <typename T, int VEC>
__device__ __forceinline__ void load_nt(const T* __restrict__ p, float (&x)[VEC]) {
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

// pixel-major coefficient rows leave through LDS as whole 1 KiB rows per store instruction
template <int K, int VEC>
constexpr bool fr_stage() { return VEC == 4 && (VEC * K) % 4 == 0 && K <= 9; }

template <int K, int VEC, int NC, int U, typename T, int LAYOUT, bool TAIL>
__device__ __forceinline__ double fitres_body(const double* __restrict__ A, const double* __restrict__ G, int N, bool orth,
                                              const T* __restrict__ src, int64_t P, int64_t pe, int64_t lstride,
                                              float* __restrict__ dst, float* __restrict__ res,
                                              int64_t wave_base, int lane, float* lds_wave) {
  constexpr int CH = 64 * VEC;
  bool ok[NC];
  int64_t off[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int64_t p0 = wave_base + (int64_t)c * CH + (int64_t)lane * VEC;
    ok[c] = !TAIL || p0 < pe;
    off[c] = ok[c] ? p0 : 0;  // a chunk past the image re-reads pixel 0 and is neither stored nor summed
  }
  double b[K][NC * VEC], q[NC * VEC];
#pragma unroll
  for (int v = 0; v < NC * VEC; ++v) {
    q[v] = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) b[i][v] = 0.0;
  }
  constexpr int UP = U / NC > 0 ? U / NC : 1;  // light planes per step: U loads in flight per lane
  int n = 0;
  for (; n + UP <= N; n += UP) {
    float x[UP][NC][VEC];
#pragma unroll
    for (int u = 0; u < UP; ++u)
#pragma unroll
      for (int c = 0; c < NC; ++c) load_nt<T, VEC>(src + (int64_t)(n + u) * lstride + off[c], x[u][c]);
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const double* An = A + (int64_t)(n + u) * K;  // wave-uniform row -> SGPR pairs
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const double xd = (double)x[u][c][v];
          const int j = c * VEC + v;
          q[j] = fma(xd, xd, q[j]);
#pragma unroll
          for (int i = 0; i < K; ++i) b[i][j] = fma(An[i], xd, b[i][j]);
        }
    }
  }
  for (; n < N; ++n) {
    float x[NC][VEC];
#pragma unroll
    for (int c = 0; c < NC; ++c) load_nt<T, VEC>(src + (int64_t)n * lstride + off[c], x[c]);
    const double* An = A + (int64_t)n * K;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const double xd = (double)x[c][v];
        const int j = c * VEC + v;
        q[j] = fma(xd, xd, q[j]);
#pragma unroll
        for (int i = 0; i < K; ++i) b[i][j] = fma(An[i], xd, b[i][j]);
      }
  }

  const double invN = 1.0 / (double)N;
  double ss_sum = 0.0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float o[VEC * K], r[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const int j = c * VEC + v;
      double s = q[j];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        double ci = 0.0;
#pragma unroll
        for (int l = 0; l < K; ++l) ci = fma(G[i * K + l], b[l][j], ci);
        s = fma(orth ? -b[i][j] : -ci, b[i][j], s);
        o[v * K + i] = (float)ci;
      }
      s = s < 0.0 ? 0.0 : s;  // rounding can leave an exact fit a few ulps below zero; NaN passes
      r[v] = (float)sqrt(s * invN);
      if (ok[c]) ss_sum += s;
    }
    const int64_t p0 = wave_base + (int64_t)c * CH + (int64_t)lane * VEC;
    if (res && ok[c]) {
      if constexpr (VEC == 4)
        *reinterpret_cast<floatx4*>(res + p0) = floatx4{r[0], r[1], r[2], r[3]};
      else
        res[p0] = r[0];
    }
    if constexpr (LAYOUT == RTI_COEF_PLANAR) {
      if (ok[c]) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
          if constexpr (VEC == 4)
            *reinterpret_cast<floatx4*>(dst + (int64_t)i * P + p0) = floatx4{o[i], o[K + i], o[2 * K + i], o[3 * K + i]};
          else
            dst[(int64_t)i * P + p0] = o[i];
        }
      }
    } else {
      if constexpr (fr_stage<K, VEC>()) {
        constexpr int F = VEC * K;
        const int64_t cbase = wave_base + (int64_t)c * CH;
        if (cbase + CH <= pe) {  // wave-uniform: the whole chunk is in the image
#pragma unroll
          for (int i = 0; i < F; i += 4)
            *reinterpret_cast<floatx4*>(lds_wave + lane * F + i) = floatx4{o[i], o[i + 1], o[i + 2], o[i + 3]};
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          float* wdst = dst + cbase * K;
#pragma unroll
          for (int j = 0; j < F / 4; ++j)
            *reinterpret_cast<floatx4*>(wdst + j * 256 + lane * 4) =
                *reinterpret_cast<const floatx4*>(lds_wave + j * 256 + lane * 4);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // slab reused by the next chunk
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          continue;
        }
      }
      if (ok[c]) {
#pragma unroll
        for (int i = 0; i < VEC * K; ++i) dst[p0 * K + i] = o[i];
      }
    }
  }
  return ss_sum;
}

template <int K, int VEC, int NC, int U, typename T, int LAYOUT>
__global__ void __launch_bounds__(FR_THREADS)
fit_shared_residual_k(const double* __restrict__ A, const double* __restrict__ G, int N, int orth, const T* __restrict__ I,
                      int64_t P, int64_t pb, int64_t pe, int64_t lstride, int64_t cstride, float* __restrict__ coef,
                      int64_t ocstride, float* __restrict__ res, double* __restrict__ partial, int64_t pstride) {
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  __shared__ double wsum[FR_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // pixels [pb, pe) of P; pb is a multiple of the workgroup's pixel span, so the workgroup's partial slot is
  // its block index in a one-launch grid
  const int64_t blk = blockIdx.x + pb / (FR_THREADS * VEC * NC);
  const int64_t wave_base = (blk * (FR_THREADS / 64) + wave) * (64 * VEC * NC);
  const T* __restrict__ src = I + (int64_t)blockIdx.y * cstride;
  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
  float* __restrict__ rc = res ? res + (int64_t)blockIdx.y * P : nullptr;
  float* lds_wave = lds_dyn + wave * 64 * VEC * K;
  double mine = 0.0;
  if (wave_base < pe) {  // wave-uniform; idle waves of the last workgroup still join the reduction
    if (wave_base + (int64_t)(64 * VEC * NC) <= pe)
      mine = fitres_body<K, VEC, NC, U, T, LAYOUT, false>(A, G, N, orth != 0, src, P, pe, lstride, dst, rc, wave_base, lane,
                                                          lds_wave);
    else
      mine = fitres_body<K, VEC, NC, U, T, LAYOUT, true>(A, G, N, orth != 0, src, P, pe, lstride, dst, rc, wave_base, lane,
                                                         lds_wave);
  }
  if (partial) {
    const double w = wave_sum(mine);
    if (lane == 0) wsum[wave] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < FR_THREADS / 64; ++i) t += wsum[i];
      partial[(int64_t)blockIdx.y * pstride + blk] = t;
    }
  }
}

struct FrArgs {
  const double *A, *G;
  int k, N;
  const void* I;
  int64_t P, lstride, cstride;
  int C;
  float* coef;
  int layout;
  int64_t ocstride;
  float* res;
  double* partial;
  int nc;
  int orth = 0;  // (A, G) = (U, V Σ⁻¹): ss = q − yᵀy
  hipStream_t s;
  int64_t pb = 0, pe = 0;  // this launch's pixel range [pb, pe) (pe 0 = P); pb a multiple of the workgroup span
};

template <int K, int VEC, int NC, typename T, int LAYOUT>
int launch_fr_t(const FrArgs& a) {
  constexpr int U = 4;  // loads in flight per lane: the fp64 work per load hides more latency than fp32
  const int64_t pe = a.pe ? a.pe : a.P;
  const dim3 grid(grid_1d(pe - a.pb, FR_THREADS * VEC * NC), a.C);
  const size_t lds =
      (LAYOUT == RTI_COEF_PIXEL_MAJOR && fr_stage<K, VEC>()) ? (size_t)FR_THREADS * VEC * K * sizeof(float) : 0;
  hipLaunchKernelGGL((fit_shared_residual_k<K, VEC, NC, U, T, LAYOUT>), grid, dim3(FR_THREADS), lds, a.s, a.A, a.G,
                     a.N, a.orth, static_cast<const T*>(a.I), a.P, a.pb, pe, a.lstride, a.cstride, a.coef, a.ocstride, a.res, a.partial,
                     (int64_t)grid_1d(a.P, FR_THREADS));
  return check_launch("rti_fit_shared_residual");
}

template <int K, int VEC, typename T, int LAYOUT>
int launch_fr_nc(const FrArgs& a) {
  // fp64 state 2k + 2 VGPRs per pixel: PTM-6 fits 4 chunks (256 VGPRs, 1 wave/SIMD), HSH-9 2 (3 or
  // more spill into AGPRs), HSH-16 one
  if constexpr (VEC == 4 && K <= 6) {
    if (a.nc >= 4) return launch_fr_t<K, VEC, 4, T, LAYOUT>(a);
    if (a.nc == 3) return launch_fr_t<K, VEC, 3, T, LAYOUT>(a);
  }
  if constexpr (VEC == 4 && K <= 9)
    if (a.nc >= 2) return launch_fr_t<K, VEC, 2, T, LAYOUT>(a);
  return launch_fr_t<K, VEC, 1, T, LAYOUT>(a);
}

template <int K, int VEC, typename T>
int launch_fr_l(const FrArgs& a) {
  return a.layout == RTI_COEF_PLANAR ? launch_fr_nc<K, VEC, T, RTI_COEF_PLANAR>(a)
                                     : launch_fr_nc<K, VEC, T, RTI_COEF_PIXEL_MAJOR>(a);
}

template <int K, typename T>
int launch_fr_v(const FrArgs& a, bool vec4) {
  return vec4 ? launch_fr_l<K, 4, T>(a) : launch_fr_l<K, 1, T>(a);
}

template <typename T>
int launch_fr_k(const FrArgs& a, bool vec4) {
  switch (a.k) {
    case 6: return launch_fr_v<6, T>(a, vec4);
    case 9: return launch_fr_v<9, T>(a, vec4);
    case 16: return launch_fr_v<16, T>(a, vec4);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_residual: k=%d (supported: 6, 9, 16)", a.k);
  }
}

// AUTO chunks per lane (profiles/r02_fitres_c3_sweep.log, c3 4K x 100 PTM-6: 1 / 2 / 3 / 4 chunks
// -> 0.618 / 0.603 / 0.598 / 0.718 ms; 4 chunks need 256 VGPRs = 1 wave per SIMD): 3 for PTM-6 while
// the launch keeps >= 2000 waves, else 2 or 1; HSH-9/16 one (their fp64 state fills the registers).
constexpr int64_t FR_MIN_WAVES = 2000;

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int64_t rti_fit_shared_residual_blocks(int64_t P) {
  if (P <= 0) return 0;
  return (int64_t)grid_1d(P, FR_THREADS);  // bounds every (VEC, NC) grid of the launch
}

namespace {
int fit_shared_residual_impl(bool orth, const double* A, const double* ginv, int k, int N, const void* I, int in_dtype,
                             int64_t P, int C, int64_t light_stride, int64_t channel_stride, float* coef,
                             int coef_layout, int64_t coef_channel_stride, float* res, double* partial, int kernel,
                             rti_stream_t stream) {
  if (!kernel_bits_ok(kernel, RTI_KERNEL_AUTO, RTI_KERNEL_ONE_LAUNCH | RTI_FIELD_CHUNKS))
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: unknown kernel bits 0x%x", kernel);
  if (!A || !ginv || !I || !coef) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: null pointer");
  if (N <= 0 || P <= 0 || C <= 0 || C > 65535) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: bad N/P/C");
  if (N < k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: N=%d < k=%d", N, k);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_residual: input dtype %d", in_dtype);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: coef layout %d", coef_layout);
  note_launches(1);
  FrArgs a;
  a.A = A;
  a.G = ginv;
  a.k = k;
  a.N = N;
  a.I = I;
  a.P = P;
  a.C = C;
  a.lstride = light_stride ? light_stride : P;
  a.cstride = channel_stride ? channel_stride : (int64_t)N * a.lstride;
  a.coef = coef;
  a.layout = coef_layout;
  a.ocstride = coef_channel_stride ? coef_channel_stride : P * k;
  a.res = res;
  a.partial = partial;
  a.orth = orth ? 1 : 0;
  a.s = (hipStream_t)stream;
  if (a.lstride < P) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: light_stride < P");
  if (C > 1 && a.cstride < (int64_t)N * a.lstride)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: channel_stride");
  if (C > 1 && a.ocstride < P * k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_residual: coef_channel_stride");
  const size_t es = in_dtype == RTI_U8 ? 1 : 4;
  const bool vec4 = P % 4 == 0 && a.lstride % 4 == 0 && a.cstride % 4 == 0 && aligned_to(I, 4 * es) &&
                    (!res || aligned_to(res, 16)) && aligned_to(coef, 16) && a.ocstride % 4 == 0;
  a.nc = (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF;
  // launch generations (rti_fit.hip): PTM-6 on 16-B lanes as consecutive launches over pixel ranges of
  // whole workgroups, each giving the SIMDs one or two waves (3 or 2 chunks per lane: 205 / <= 160
  // VGPRs, two waves resident per SIMD); profiles/r02_generations_sweep.log
  int parts = 1;
  const bool gens = k == 6 && vec4 && a.nc <= 3 && !(kernel & RTI_KERNEL_ONE_LAUNCH);
  if (gens) {
    // efficiency of a launch = its waves / (SIMDs x the waves of the busiest SIMD); AUTO takes the
    // better-balanced of 3 and 2 chunks (3 unless 2 is > 3 points better): c3 as 6 launches of 1800
    // waves at 3 chunks 0.5835 ms, 8 launches of 2025 at 2 chunks 0.5775, one launch 0.6155
    const int64_t simds = 4 * (int64_t)device_cus();
    double best = 0.0;
    const int want = a.nc;  // explicit chunks (0 = AUTO)
    for (int nc : {3, 2}) {
      if (want && nc != want) continue;
      const int64_t span = (int64_t)FR_THREADS * 4 * nc, bpc = (P + span - 1) / span;  // workgroups per channel
      int p = 1;
      int64_t per = bpc * C * 4;  // waves in one launch
      if (per > 2 * simds) {
        p = (int)((4 * bpc + 2 * simds - 1) / (2 * simds));
        per = 4 * ((bpc + p - 1) / p);
      }
      const double eff = (double)per / (double)(((per + simds - 1) / simds) * simds);
      if (eff < 0.85 || (p > 1 && (double)per * 256 * nc * N * es < 256.0 * (1 << 20))) continue;
      if (eff > best + 0.03) {
        best = eff;
        a.nc = nc;
        parts = p;
      }
    }
  }
  if (a.nc == 0) {
    a.nc = 1;
    if (k == 6)
      for (int nc = 3; nc > 1; --nc)
        if (P * C / (64 * 4 * nc) >= FR_MIN_WAVES) {
          a.nc = nc;
          break;
        }
  }
  auto launch = [&](const FrArgs& b) {
    switch (in_dtype) {
      case RTI_F32: return launch_fr_k<float>(b, vec4);
      case RTI_U8: return launch_fr_k<uint8_t>(b, vec4);
      default: return launch_fr_k<int32_t>(b, vec4);
    }
  };
  if (parts == 1) return launch(a);
  const int64_t span = (int64_t)FR_THREADS * 4 * a.nc, units = (P + span - 1) / span;
  const int64_t per = (units + parts - 1) / parts, pstride = rti_fit_shared_residual_blocks(P);
  for (int c = 0; c < C; ++c) {
    FrArgs b = a;
    b.C = 1;
    b.I = static_cast<const char*>(I) + (size_t)c * a.cstride * es;
    b.coef = coef + (size_t)c * a.ocstride;
    b.res = res ? res + (size_t)c * P : nullptr;
    b.partial = partial ? partial + (size_t)c * pstride : nullptr;
    for (int i = 0; i < parts; ++i) {
      b.pb = i * per * span;
      b.pe = (i + 1) * per * span < P ? (i + 1) * per * span : P;
      if (b.pb >= b.pe) break;
      const int st = launch(b);
      if (st != RTI_OK) return st;
      note_launches(c * parts + i + 1);
    }
  }
  return RTI_OK;
}
}  // namespace

extern "C" int rti_fit_shared_residual(const double* A, const double* ginv, int k, int N, const void* I, int in_dtype,
                                       int64_t P, int C, int64_t light_stride, int64_t channel_stride, float* coef,
                                       int coef_layout, int64_t coef_channel_stride, float* res, double* partial,
                                       int kernel, rti_stream_t stream) {
  return fit_shared_residual_impl(false, A, ginv, k, N, I, in_dtype, P, C, light_stride, channel_stride, coef,
                                  coef_layout, coef_channel_stride, res, partial, kernel, stream);
}

extern "C" int rti_fit_shared_residual_svd(const double* U, const double* W, int k, int N, const void* I,
                                           int in_dtype, int64_t P, int C, int64_t light_stride,
                                           int64_t channel_stride, float* coef, int coef_layout,
                                           int64_t coef_channel_stride, float* res, double* partial, int kernel,
                                           rti_stream_t stream) {
  return fit_shared_residual_impl(true, U, W, k, N, I, in_dtype, P, C, light_stride, channel_stride, coef,
                                  coef_layout, coef_channel_stride, res, partial, kernel, stream);
}
