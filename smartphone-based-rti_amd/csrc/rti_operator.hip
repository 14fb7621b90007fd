// rti_operator.hip -- apply a light operator to the intensity stack on gfx950 (MFMA).
//
//     out[c][e][p] = Σ_n opT[n][e] · I[c][n][p]
//
// The operator maps a pixel's N intensities to E outputs.  With the linear-RBF
// operator M = Φ(q) A⁻¹ (rti_rbf_operator) evaluated on the reference's 100×100
// grid, one launch is the reference's default interpolation (SciPy Rbf
// 'linear', analysis.py:249-260 via interpolate_intensities :361-363) plus the
// prepare_images_data layout (analysis.py:375-411): out[e][p] with e = ly·G + lx.
// With M = B(q)·pinv it is the PTM/HSH fit fused with its grid evaluation.
//
// Shape: a GEMM with a short reduction (K = N ≤ 256 lights) and a huge output
// (E·P), so it is MFMA- or store-bound, never load-bound.  A workgroup owns a
// 64-pixel tile: it stages the tile's N×64 intensities in LDS once (read from
// HBM exactly once over the whole launch) and sweeps every operator row over
// them.  Each wave computes 64 rows × 64 pixels per sweep step with
// v_mfma_f32_16x16x4_f32: the A operand is a 16-byte load of 4 consecutive
// operator rows (rows 4q+rb of the wave's 64, rb = MFMA row block), the B
// operand one ds_read_b128 of 4 adjacent pixels (pixel 4q+c for accumulator c),
// i.e. 16 MFMAs per pair of 16-byte loads.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "rti_convert.h"
#include "rti_internal.h"

namespace rti {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int TILE_P = 64;    // pixels per workgroup tile
constexpr int ROWS_WG = 256;  // operator rows per workgroup sweep step (4 waves × 64)

template <typename T, typename TO, bool VEC>
__global__ void __launch_bounds__(256)
apply_op_mfma(const float* __restrict__ opT, int E, int N, int64_t ostride, const T* __restrict__ I, int64_t P,
              int64_t lstride, int64_t cstride, TO* __restrict__ out, int64_t orow, int64_t ocs) {
  extern __shared__ __attribute__((aligned(16))) float sB[];  // [Npad][TILE_P]
  const int Npad = (N + 3) & ~3;
  const int64_t p0 = (int64_t)blockIdx.x * TILE_P;
  const T* __restrict__ src = I + (int64_t)blockIdx.z * cstride;

  // stage the tile's intensities (zero beyond N and beyond P)
  for (int idx = threadIdx.x; idx < Npad * (TILE_P / 4); idx += 256) {
    const int n = idx / (TILE_P / 4), q4 = idx % (TILE_P / 4);
    const int64_t px = p0 + 4 * q4;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (n < N) {
      const T* s = src + (int64_t)n * lstride + px;
      if (VEC && px + 3 < P) {
        typedef T vec_t __attribute__((ext_vector_type(4)));
        const vec_t t = __builtin_nontemporal_load(reinterpret_cast<const vec_t*>(s));
        v = floatx4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (px + c < P) v[c] = (float)s[c];
      }
    }
    *reinterpret_cast<floatx4*>(sB + n * TILE_P + 4 * q4) = v;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane & 15, r = lane >> 4;
  const int ntiles = (E + ROWS_WG - 1) / ROWS_WG;
  TO* __restrict__ dst = out + (int64_t)blockIdx.z * ocs;
  for (int rt = blockIdx.y; rt < ntiles; rt += gridDim.y) {
    const int row0 = rt * ROWS_WG + wave * 64;
    if (row0 >= E) continue;  // wave-uniform
    const int rowq = row0 + 4 * q;
    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int n0 = 0; n0 < Npad; n0 += 4) {
      const int n = n0 + r;
      floatx4 a = {0.f, 0.f, 0.f, 0.f};
      if (n < N) {
        const float* op = opT + (int64_t)n * ostride + rowq;
        if (VEC && rowq + 3 < E) {
          a = *reinterpret_cast<const floatx4*>(op);
        } else {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
            if (rowq + rb < E) a[rb] = op[rb];
        }
      }
      const floatx4 b = *reinterpret_cast<const floatx4*>(sB + n * TILE_P + 4 * q);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb], b[c], acc[rb][c], 0, 0, 0);
    }
    // acc[rb][c][rr] = out row (row0 + 16r + 4rr + rb), pixel (p0 + 4q + c)
    const int64_t px = p0 + 4 * q;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = row0 + 16 * r + 4 * rr + rb;
        if (row >= E) continue;
        TO* o = dst + (int64_t)row * orow + px;
        if (VEC && px + 3 < P) {
          typedef TO ovec_t __attribute__((ext_vector_type(4)));
          ovec_t v;
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = cvt_out<TO>(acc[rb][c][rr]);
          *reinterpret_cast<ovec_t*>(o) = v;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (px + c < P) o[c] = cvt_out<TO>(acc[rb][c][rr]);
        }
      }
  }
}

template <typename T, typename TO>
int launch(const float* opT, int E, int N, int64_t os, const void* I, int64_t P, int C, int64_t ls, int64_t cs,
           void* out, int64_t orow, int64_t ocs, bool vec, hipStream_t s) {
  const int Npad = (N + 3) & ~3;
  const size_t lds = (size_t)Npad * TILE_P * sizeof(float);
  const unsigned gx = (unsigned)((P + TILE_P - 1) / TILE_P);
  const int ntiles = (E + ROWS_WG - 1) / ROWS_WG;
  // enough workgroups to fill 256 CUs; with many pixel tiles each workgroup sweeps every row
  const unsigned gy = (unsigned)std::max(1, std::min(ntiles, (int)((2048 + gx - 1) / gx)));
  dim3 grid(gx, gy, C);
  if (vec)
    hipLaunchKernelGGL((apply_op_mfma<T, TO, true>), grid, dim3(256), lds, s, opT, E, N, os, static_cast<const T*>(I),
                       P, ls, cs, static_cast<TO*>(out), orow, ocs);
  else
    hipLaunchKernelGGL((apply_op_mfma<T, TO, false>), grid, dim3(256), lds, s, opT, E, N, os, static_cast<const T*>(I),
                       P, ls, cs, static_cast<TO*>(out), orow, ocs);
  return check_launch("rti_apply_operator");
}

template <typename T>
int launch_out(int odt, const float* opT, int E, int N, int64_t os, const void* I, int64_t P, int C, int64_t ls,
               int64_t cs, void* out, int64_t orow, int64_t ocs, bool vec, hipStream_t s) {
  switch (odt) {
    case RTI_F32: return launch<T, float>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_F64: return launch<T, double>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_I32: return launch<T, int32_t>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    default: return launch<T, uint8_t>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
  }
}

size_t esize(int dt) { return dt == RTI_U8 ? 1 : dt == RTI_F64 ? 8 : 4; }

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_apply_operator(const float* opT, int E, int N, int64_t op_stride, const void* I, int in_dtype,
                                  int64_t P, int C, int64_t light_stride, int64_t channel_stride, void* out,
                                  int out_dtype, int64_t out_row_stride, int64_t out_channel_stride,
                                  rti_stream_t stream) {
  if (!opT || !I || !out) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator: null pointer");
  if (E <= 0 || N <= 0 || P <= 0 || C <= 0 || C > 65535)
    return fail(RTI_ERR_BAD_ARG, "rti_apply_operator: bad E/N/P/C");
  if (N > 256) return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator: N=%d > 256 lights", N);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator: input dtype %d", in_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator: out dtype %d", out_dtype);
  const int64_t os = op_stride ? op_stride : E;
  const int64_t ls = light_stride ? light_stride : P;
  const int64_t cs = channel_stride ? channel_stride : (int64_t)N * ls;
  const int64_t orow = out_row_stride ? out_row_stride : P;
  const int64_t ocs = out_channel_stride ? out_channel_stride : (int64_t)E * orow;
  if (os < E || ls < P || orow < P) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator: stride smaller than extent");
  const size_t ie = esize(in_dtype), oe = esize(out_dtype);
  const bool vec = os % 4 == 0 && aligned_to(opT, 16) && P % 4 == 0 && ls % 4 == 0 && cs % 4 == 0 &&
                   aligned_to(I, 4 * ie) && orow % 4 == 0 && ocs % 4 == 0 && aligned_to(out, 4 * oe);
  hipStream_t s = (hipStream_t)stream;
  switch (in_dtype) {
    case RTI_F32: return launch_out<float>(out_dtype, opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_I32: return launch_out<int32_t>(out_dtype, opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    default: return launch_out<uint8_t>(out_dtype, opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
  }
}
