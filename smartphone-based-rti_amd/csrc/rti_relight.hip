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

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Pixel-major coefficient rows through LDS.  A lane's own 4 pixels are K·sizeof(TC)·4 contiguous
// bytes, so per-lane loads stride that far across the wave (96 B for PTM-6 fp32) and every
// 128-B line is requested by several load instructions.  Instead the wave reads its 256 pixels'
// rows as PIECES coalesced 1-KiB loads (lane l, piece j: bytes 16·(64·j + l) of the chunk),
// parks them in its LDS slab and reads back its own 4 pixels' rows (cold c5: DESIGN.md §4.4).
template <int K, typename TC>
constexpr bool coef_staged() {
  return (K * sizeof(TC)) % 4 == 0 && 4 * 256 * K * sizeof(TC) <= 48 * 1024;
}

template <int K, typename TC>
__device__ __forceinline__ void load_coef_staged(const TC* __restrict__ coef, int64_t wave_px, int lane,
                                                 floatx4* __restrict__ slab, TC (&c)[4][K]) {
  constexpr int PIECES = K * (int)sizeof(TC) / 4;  // 16-B pieces per lane (6 for PTM-6 fp32)
  const floatx4* g = reinterpret_cast<const floatx4*>(coef + wave_px * K);
  floatx4 t[PIECES];
#pragma unroll
  for (int j = 0; j < PIECES; ++j) t[j] = __builtin_nontemporal_load(g + j * 64 + lane);
#pragma unroll
  for (int j = 0; j < PIECES; ++j) slab[j * 64 + lane] = t[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  union {
    floatx4 v[PIECES];
    TC c[4][K];
  } u;
#pragma unroll
  for (int j = 0; j < PIECES; ++j) u.v[j] = slab[lane * PIECES + j];
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int k = 0; k < K; ++k) c[v][k] = u.c[v][k];
}

// Eval-major: block = 256 lanes × VEC pixels, up to ECH evals (blockIdx.y).
template <int K, int VEC, typename TC, typename TO, int CL>
__global__ void __launch_bounds__(256)
relight_eval_major(const TC* __restrict__ coef, int basis, int64_t P, const double* __restrict__ luv, int E,
                   TO* __restrict__ out) {
  constexpr bool STAGED = VEC == 4 && CL == RTI_COEF_PIXEL_MAJOR && coef_staged<K, TC>();
  __shared__ floatx4 slab[STAGED ? 4 * 64 * K * sizeof(TC) / 4 : 1];  // 4 waves × 256 px rows
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
  const int lane = threadIdx.x & 63;
  const int64_t wave_px = p0 - 4 * lane;
  if constexpr (STAGED) {
    if (wave_px + 256 <= P) {  // wave-uniform: the whole 256-pixel chunk is in the image
      load_coef_staged<K, TC>(coef, wave_px, lane, slab + (threadIdx.x >> 6) * (64 * K * (int)sizeof(TC) / 4), c);
      goto evaluate;
    }
  }
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int k = 0; k < K; ++k)
      c[v][k] = (CL == RTI_COEF_PLANAR) ? coef[(int64_t)k * P + p0 + v] : coef[(p0 + v) * K + k];
evaluate:

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
  const bool vec = a.P % 4 == 0 && aligned_to(a.out, 4 * sizeof(TO)) && aligned_to(a.coef, 16);
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

// ---- interactive relight frame (interactive_relighting.py:22-38) ---------------------
// OpenCV 4.x COLOR_HSV2BGR for 8-bit images, hue range 180 (HSV2RGB_b + HSV2RGB_native,
// scalar form): s and v scaled by 1/255 in fp32, h·(6/180), sector = floor, the four
// tab[] products, saturate_cast<uchar>(x·255) = round-half-even then clamp.  No FP
// contraction, so the oracle's NumPy restatement is matched bit for bit.
__device__ __forceinline__ uint8_t sat_u8(float x) {
  const float r = rintf(x);
  return (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
}

__device__ __forceinline__ void hsv2bgr_u8(uint32_t H, uint32_t S, uint32_t V, uint8_t (&bgr)[3]) {
#pragma clang fp contract(off)
  const float hscale = 6.0f / 180.0f;
  const float s = (float)S * (1.0f / 255.0f);
  const float v = (float)V * (1.0f / 255.0f);
  float b, g, r;
  if (s == 0.f) {
    b = g = r = v;
  } else {
    float h = (float)H * hscale;
    if (h >= 6.f) h -= 6.f;  // H <= 255 -> h < 8.5: one subtraction (OpenCV's loop / fmod)
    int sector = (int)floorf(h);
    h -= (float)sector;
    if ((unsigned)sector >= 6u) {
      sector = 0;
      h = 0.f;
    }
    const float t0 = v, t1 = v * (1.f - s), t2 = v * (1.f - s * h), t3 = v * (1.f - s * (1.f - h));
    // sector_data = {{1,3,0}, {1,0,2}, {3,0,1}, {0,2,1}, {0,1,3}, {2,1,0}} -> (b, g, r)
    switch (sector) {
      case 0: b = t1; g = t3; r = t0; break;
      case 1: b = t1; g = t0; r = t2; break;
      case 2: b = t3; g = t0; r = t1; break;
      case 3: b = t0; g = t2; r = t1; break;
      case 4: b = t0; g = t1; r = t3; break;
      default: b = t2; g = t1; r = t0; break;
    }
  }
  bgr[0] = sat_u8(b * 255.f);
  bgr[1] = sat_u8(g * 255.f);
  bgr[2] = sat_u8(r * 255.f);
}

// One lane = 4 pixels: 12 B of HSV in, 12 B of BGR out (dword loads/stores), V from the
// int32 table image or from the pixel's coefficients at (lu, lv).
template <int K, typename TC, int CL>
__global__ void __launch_bounds__(256)
relight_frame_k(const void* __restrict__ src, int basis, int64_t P, double lu, double lv,
                const uint8_t* __restrict__ hsv, uint8_t* __restrict__ bgr) {
  constexpr bool STAGED = K > 0 && CL == RTI_COEF_PIXEL_MAJOR && coef_staged<K, TC>();
  __shared__ floatx4 slab[STAGED ? 4 * 64 * K * sizeof(TC) / 4 : 1];  // 4 waves × 256 px rows
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= P) return;
  const int np = P - p0 < 4 ? (int)(P - p0) : 4;
  uint8_t Vv[4];
  const int lane = threadIdx.x & 63;
  const int64_t wave_px = p0 - 4 * lane;
  if constexpr (STAGED) {
    if (wave_px + 256 <= P && aligned_to(src, 16)) {  // wave-uniform
      TC b[K], c[4][K];
      basis_eval<TC>(basis, (TC)lu, (TC)lv, b);
      load_coef_staged<K, TC>(static_cast<const TC*>(src), wave_px, lane,
                              slab + (threadIdx.x >> 6) * (64 * K * (int)sizeof(TC) / 4), c);
#pragma unroll
      for (int j = 0; j < 4; ++j) Vv[j] = cvt_out<uint8_t>(dot_k<K>(c[j], b));
      goto convert;
    }
  }
  if constexpr (K == 0) {
    const int32_t* t = static_cast<const int32_t*>(src);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t x = j < np ? t[p0 + j] : 0;
      Vv[j] = (uint8_t)(x > 255 ? 255 : (x <= 0 ? 0 : x));  // interactive_relighting.py:35-37
    }
  } else {
    const TC* coef = static_cast<const TC*>(src);
    TC b[K];
    basis_eval<TC>(basis, (TC)lu, (TC)lv, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      TC c[K];
      const int64_t p = j < np ? p0 + j : p0;
#pragma unroll
      for (int k = 0; k < K; ++k) c[k] = (CL == RTI_COEF_PLANAR) ? coef[(int64_t)k * P + p] : coef[p * K + k];
      Vv[j] = cvt_out<uint8_t>(dot_k<K>(c, b));
    }
  }
convert:
  uint8_t in[12], o[12];
  const uint8_t* hp = hsv + p0 * 3;
  uint8_t* op = bgr + p0 * 3;
  const bool full = np == 4 && aligned_to(hp, 4) && aligned_to(op, 4);
  if (full) {
    const uint32_t* h4 = reinterpret_cast<const uint32_t*>(hp);
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const uint32_t d = h4[w];
#pragma unroll
      for (int i = 0; i < 4; ++i) in[4 * w + i] = (uint8_t)(d >> (8 * i));
    }
  } else {
    for (int i = 0; i < 3 * np; ++i) in[i] = hp[i];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint8_t px[3];
    hsv2bgr_u8(in[3 * j], in[3 * j + 1], Vv[j], px);  // img[:, :, 2] = values (:37)
    o[3 * j] = px[0];
    o[3 * j + 1] = px[1];
    o[3 * j + 2] = px[2];
  }
  if (full) {
    uint32_t* o4 = reinterpret_cast<uint32_t*>(op);
#pragma unroll
    for (int w = 0; w < 3; ++w)
      o4[w] = (uint32_t)o[4 * w] | ((uint32_t)o[4 * w + 1] << 8) | ((uint32_t)o[4 * w + 2] << 16) |
              ((uint32_t)o[4 * w + 3] << 24);
  } else {
    for (int i = 0; i < 3 * np; ++i) op[i] = o[i];
  }
}

template <int K, typename TC>
void launch_frame_cl(const void* src, int basis, int cl, int64_t P, double lu, double lv, const uint8_t* hsv,
                     uint8_t* bgr, hipStream_t s) {
  const dim3 grid(grid_1d((P + 3) / 4, 256));
  if (cl == RTI_COEF_PLANAR)
    hipLaunchKernelGGL((relight_frame_k<K, TC, RTI_COEF_PLANAR>), grid, dim3(256), 0, s, src, basis, P, lu, lv, hsv,
                       bgr);
  else
    hipLaunchKernelGGL((relight_frame_k<K, TC, RTI_COEF_PIXEL_MAJOR>), grid, dim3(256), 0, s, src, basis, P, lu, lv,
                       hsv, bgr);
}

template <typename TC>
void launch_frame(const void* src, int basis, int cl, int64_t P, double lu, double lv, const uint8_t* hsv,
                  uint8_t* bgr, hipStream_t s) {
  switch (basis_terms(basis)) {
    case 6: launch_frame_cl<6, TC>(src, basis, cl, P, lu, lv, hsv, bgr, s); break;
    case 9: launch_frame_cl<9, TC>(src, basis, cl, P, lu, lv, hsv, bgr, s); break;
    default: launch_frame_cl<16, TC>(src, basis, cl, P, lu, lv, hsv, bgr, s); break;
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

extern "C" int rti_relight_frame(const void* src, int src_dtype, int basis, int coef_layout, int64_t P, double lu,
                                 double lv, const uint8_t* hsv, uint8_t* bgr, rti_stream_t stream) {
  if (!src || !hsv || !bgr) return fail(RTI_ERR_BAD_ARG, "rti_relight_frame: null pointer");
  if (P <= 0) return fail(RTI_ERR_BAD_ARG, "rti_relight_frame: P must be positive");
  hipStream_t s = (hipStream_t)stream;
  if (src_dtype == RTI_I32) {
    hipLaunchKernelGGL((relight_frame_k<0, float, RTI_COEF_PIXEL_MAJOR>), dim3(grid_1d((P + 3) / 4, 256)), dim3(256),
                       0, s, src, basis, P, lu, lv, hsv, bgr);
    return check_launch("rti_relight_frame");
  }
  if (src_dtype != RTI_F32 && src_dtype != RTI_F64)
    return fail(RTI_ERR_UNSUPPORTED, "rti_relight_frame: src dtype %d", src_dtype);
  if (basis_terms(basis) < 0) return fail(RTI_ERR_BAD_ARG, "rti_relight_frame: unknown basis %d", basis);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_relight_frame: coef layout %d", coef_layout);
  if (src_dtype == RTI_F64)
    launch_frame<double>(src, basis, coef_layout, P, lu, lv, hsv, bgr, s);
  else
    launch_frame<float>(src, basis, coef_layout, P, lu, lv, hsv, bgr, s);
  return check_launch("rti_relight_frame");
}
