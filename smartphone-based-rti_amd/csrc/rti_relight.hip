// rti_relight.hip -- per-pixel relight evaluator on gfx950.
//
// out(e, p) = Σ_i coef[p][i] · b_i(lu_e, lv_e) for E light directions.
// Replaces:
//  * the grid evaluation of _interpolate_PTM (analysis.py:300-315), which the
//    reference runs as a 10⁴-iteration Python loop per pixel;
//  * prepare_images_data's [y][x][ly][lx] -> [ly][lx][y][x] transpose and the
//    float64 -> int32 truncation (analysis.py:401-409): eval-major output with
//    out_dtype = I32 is that table directly;
//  * relighting_event's clip to [0, 255] (interactive_relighting.py:35-36):
//    out_dtype = U8.
// Arithmetic is done in the coefficient type.  In the fp64 path the terms are
// multiplied and summed left to right with no contraction
// (a0·lu² + a1·lv² + a2·(lu·lv) + a3·lu + a4·lv + a5, analysis.py:307-312), so
// fp64 coefficients equal to the reference's reproduce its grid bit for bit.
//
// Traffic per (pixel, eval): eval-major reads the pixel's k coefficients once
// per block of up to 64 evals and writes one output element per eval, so a
// single-eval launch moves 4k + 4 B per pixel (28 B for PTM-6 fp32).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "rti_basis.h"
#include "rti_convert.h"
#include "rti_internal.h"

namespace rti {
namespace {

constexpr int ECH = 64;  // evals per eval-major block (basis table in LDS)

// fp64: the reference's order, every product and sum rounded (analysis.py:307-312).
template <int K>
__device__ __forceinline__ double dot_k(const double (&c)[K], const double* b) {
#pragma clang fp contract(off)
  double acc = c[0] * b[0];
#pragma unroll
  for (int k = 1; k < K; ++k) acc = acc + c[k] * b[k];
  return acc;
}

// fp32: fused multiply-adds in the same order.
template <int K>
__device__ __forceinline__ float dot_k(const float (&c)[K], const float* b) {
  float acc = c[0] * b[0];
#pragma unroll
  for (int k = 1; k < K; ++k) acc = fmaf(c[k], b[k], acc);
  return acc;
}

// Eval-major: block = 256 lanes × VEC pixels, up to ECH evals (blockIdx.y).
template <int K, int VEC, typename TC, typename TO, int CL>
__global__ void __launch_bounds__(256)
relight_eval_major(const TC* __restrict__ coef, int basis, int64_t P, const double* __restrict__ luv, int E,
                   TO* __restrict__ out) {
  __shared__ TC btab[ECH * K];
  const int e0 = blockIdx.y * ECH;
  const int ne = min(ECH, E - e0);
  for (int i = threadIdx.x; i < ne; i += 256) {
    TC b[K];
    basis_eval<TC>(basis, (TC)luv[2 * (e0 + i)], (TC)luv[2 * (e0 + i) + 1], b);
#pragma unroll
    for (int k = 0; k < K; ++k) btab[i * K + k] = b[k];
  }
  __syncthreads();
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
  if (p0 >= P) return;

  TC c[VEC][K];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int k = 0; k < K; ++k)
      c[v][k] = (CL == RTI_COEF_PLANAR) ? coef[(int64_t)k * P + p0 + v] : coef[(p0 + v) * K + k];

  for (int e = 0; e < ne; ++e) {
    const TC* b = btab + e * K;
    TO* dst = out + (int64_t)(e0 + e) * P + p0;
    if constexpr (VEC == 1) {
      dst[0] = cvt_out<TO>(dot_k<K>(c[0], b));
    } else {
      typedef TO vec_t __attribute__((ext_vector_type(VEC)));
      vec_t o;
#pragma unroll
      for (int v = 0; v < VEC; ++v) o[v] = cvt_out<TO>(dot_k<K>(c[v], b));
      *reinterpret_cast<vec_t*>(dst) = o;
    }
  }
}

// Pixel-major ([p][e], interpolate_intensities' [y][x][ly][lx]): lane = eval,
// a block covers 256 evals × 8 pixels; grid flattened over (pixel, eval) blocks.
constexpr int PPB = 8;
template <int K, typename TC, typename TO, int CL>
__global__ void __launch_bounds__(256)
relight_pixel_major(const TC* __restrict__ coef, int basis, int64_t P, const double* __restrict__ luv, int E,
                    TO* __restrict__ out, int64_t e_blocks) {
  const int64_t eb = blockIdx.x % e_blocks;
  const int64_t pb = blockIdx.x / e_blocks;
  const int e = (int)(eb * 256) + threadIdx.x;
  TC b[K];
  const int ee = e < E ? e : E - 1;
  basis_eval<TC>(basis, (TC)luv[2 * ee], (TC)luv[2 * ee + 1], b);
  for (int j = 0; j < PPB; ++j) {
    const int64_t p = pb * PPB + j;
    if (p >= P) break;
    TC c[K];
#pragma unroll
    for (int k = 0; k < K; ++k) c[k] = (CL == RTI_COEF_PLANAR) ? coef[(int64_t)k * P + p] : coef[p * K + k];
    if (e < E) out[p * E + e] = cvt_out<TO>(dot_k<K>(c, b));
  }
}

struct RelightArgs {
  const void* coef;
  int basis;
  int64_t P;
  int cl;
  const double* luv;
  int E;
  void* out;
  int out_layout;
  hipStream_t s;
};

template <int K, typename TC, typename TO, int CL>
void launch_t(const RelightArgs& a) {
  const TC* coef = static_cast<const TC*>(a.coef);
  TO* out = static_cast<TO*>(a.out);
  if (a.out_layout == RTI_OUT_PIXEL_MAJOR) {
    const int64_t eblocks = (a.E + 255) / 256;
    const int64_t pblocks = (a.P + PPB - 1) / PPB;
    hipLaunchKernelGGL((relight_pixel_major<K, TC, TO, CL>), dim3((unsigned)(eblocks * pblocks)), dim3(256), 0, a.s,
                       coef, a.basis, a.P, a.luv, a.E, out, eblocks);
    return;
  }
  const unsigned ey = (unsigned)((a.E + ECH - 1) / ECH);
  const bool vec = a.P % 4 == 0 && aligned_to(a.out, 4 * sizeof(TO)) && aligned_to(a.coef, sizeof(TC));
  if (vec)
    hipLaunchKernelGGL((relight_eval_major<K, 4, TC, TO, CL>), dim3(grid_1d(a.P / 4, 256), ey), dim3(256), 0, a.s,
                       coef, a.basis, a.P, a.luv, a.E, out);
  else
    hipLaunchKernelGGL((relight_eval_major<K, 1, TC, TO, CL>), dim3(grid_1d(a.P, 256), ey), dim3(256), 0, a.s,
                       coef, a.basis, a.P, a.luv, a.E, out);
}

template <int K, typename TC, typename TO>
void launch_cl(const RelightArgs& a) {
  if (a.cl == RTI_COEF_PLANAR)
    launch_t<K, TC, TO, RTI_COEF_PLANAR>(a);
  else
    launch_t<K, TC, TO, RTI_COEF_PIXEL_MAJOR>(a);
}

template <int K, typename TC>
void launch_out(const RelightArgs& a, int odt) {
  switch (odt) {
    case RTI_F32: launch_cl<K, TC, float>(a); break;
    case RTI_F64: launch_cl<K, TC, double>(a); break;
    case RTI_I32: launch_cl<K, TC, int32_t>(a); break;
    default: launch_cl<K, TC, uint8_t>(a); break;
  }
}

template <typename TC>
void launch_k(const RelightArgs& a, int odt) {
  switch (basis_terms(a.basis)) {
    case 6: launch_out<6, TC>(a, odt); break;
    case 9: launch_out<9, TC>(a, odt); break;
    default: launch_out<16, TC>(a, odt); break;
  }
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_relight(const void* coef, int coef_dtype, int basis, int64_t P, int coef_layout,
                           const double* luv, int E, void* out, int out_dtype, int out_layout,
                           rti_stream_t stream) {
  if (!coef || !luv || !out) return fail(RTI_ERR_BAD_ARG, "rti_relight: null pointer");
  if (P <= 0 || E <= 0) return fail(RTI_ERR_BAD_ARG, "rti_relight: P and E must be positive");
  if (basis_terms(basis) < 0) return fail(RTI_ERR_BAD_ARG, "rti_relight: unknown basis %d", basis);
  if (coef_dtype != RTI_F32 && coef_dtype != RTI_F64)
    return fail(RTI_ERR_UNSUPPORTED, "rti_relight: coef dtype %d", coef_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_relight: out dtype %d", out_dtype);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_relight: coef layout %d", coef_layout);
  if (out_layout != RTI_OUT_EVAL_MAJOR && out_layout != RTI_OUT_PIXEL_MAJOR)
    return fail(RTI_ERR_BAD_ARG, "rti_relight: out layout %d", out_layout);
  if (out_layout == RTI_OUT_EVAL_MAJOR && (E + ECH - 1) / ECH > 65535)
    return fail(RTI_ERR_UNSUPPORTED, "rti_relight: E too large for one eval-major launch");
  RelightArgs a{coef, basis, P, coef_layout, luv, E, out, out_layout, (hipStream_t)stream};
  if (coef_dtype == RTI_F64)
    launch_k<double>(a, out_dtype);
  else
    launch_k<float>(a, out_dtype);
  return check_launch("rti_relight");
}
