// rti_fit_q8.hip -- shared-direction fit of 8-bit stacks on the int8 matrix cores (gfx950).
//
// The reference's intensities are the uint8 V channel (FeatureMatcher.py:183-184, widened to int32 at
// analysis.py:219,232).  At one byte per pixel·light an HBM-rate fit needs k multiply-adds per byte:
// 8e12 pixel·lights/s × 16 (HSH-16) is 1.6× the whole fp32 VALU/MFMA rate of the chip, so the fp32 stream
// tops out near 0.6 of the HBM roofline on u8.  Here the contraction runs on
// v_mfma_i32_16x16x64_i8 with the pseudo-inverse as four int8 digits of a 27-bit fixed-point operator
// (rti_q8.h: exact int32 accumulation, one fp64 rounding at the end; more accurate than the fp32 stream):
//
//   * a 512-thread workgroup owns a tile of R = 1024 pixels of one channel and sweeps the lights in steps
//     of 64; per step wave w loads planes 8w..8w+7 of the tile (one 16-byte non-temporal load per lane and
//     plane: 1 KiB per wave-instruction), flips the sign bit (x − 128) and parks them in a double-buffered
//     LDS tile [2][64 planes][R + 16 bytes]; one barrier per step, the loads of the next two steps in flight
//     in registers (128 KiB per CU) while the current step's MFMAs run;
//   * each wave then reads its 128 pixels back as MFMA B operands with ds_read_b64_tr_b8 (the hardware
//     transpose: a lane receives 8 planes of one pixel), two reads per 16-pixel column group, and issues
//     one MFMA per digit against the digit's A fragment (the operator, staged in LDS once per workgroup);
//   * epilogue: per pixel and coefficient the four int32 digit sums are combined exactly in fp64, scaled,
//     rounded to fp32 and stored (pixel-major rows of 16 pixels × k floats are contiguous per wave).
//
// Traffic = the algorithmic bytes: every stack byte once + 4k bytes of coefficients per pixel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "rti_internal.h"
#include "rti_q8.h"

namespace rti {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int Q8_R = 1024;            // tile pixels
constexpr int Q8_W = 8;               // waves per workgroup
constexpr int Q8_RS = Q8_R + 16;      // LDS row stride: 16 consecutive rows span all 64 banks
constexpr int Q8_WPX = Q8_R / Q8_W;   // pixels per wave (8 column groups of 16)
constexpr int Q8_G = Q8_WPX / 16;

__device__ __forceinline__ v2i tr8(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(p));
}

template <int K, int LAYOUT>
__device__ __forceinline__ void q8_store(float* __restrict__ dst, int64_t P, int64_t p, int g, const float (&v)[4]) {
  // v[r] = coefficient 4g + r of pixel p
  if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < K) dst[(int64_t)(4 * g + r) * P + p] = v[r];
  } else if constexpr (K == 16) {
    *reinterpret_cast<floatx4*>(dst + p * 16 + 4 * g) = floatx4{v[0], v[1], v[2], v[3]};
  } else if constexpr (K % 2 == 0) {  // rows of K floats are 8-byte aligned
#pragma unroll
    for (int r = 0; r < 4; r += 2)
      if (4 * g + r < K) *reinterpret_cast<floatx2*>(dst + p * K + 4 * g + r) = floatx2{v[r], v[r + 1]};
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < K) dst[p * K + 4 * g + r] = v[r];
  }
}

template <int K, int LAYOUT, bool STAGE>
__global__ void __launch_bounds__(64 * Q8_W)
fit_q8(const unsigned char* __restrict__ op, int N, const unsigned char* __restrict__ I, int64_t pb, int64_t pe,
       int tpw, int64_t P, int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int T = q8_steps(N);
  // the whole operator (A fragments [T][4][64][16], scales, corrections) is staged in LDS once: the stream
  // loop then issues no global loads but the stack's, so its counted vmcnt waits only ever wait for stack bytes
  unsigned char* __restrict__ lfrag = lds;                          // [T][4][64][16] + scale[16] + corr[16][4]
  unsigned char* __restrict__ tile = lds + q8_operator_bytes(N);    // [2][64][RS]
  for (int i = threadIdx.x; i < (int)(q8_operator_bytes(N) / 16); i += 64 * Q8_W)
    *reinterpret_cast<v4i*>(lfrag + 16 * i) = *reinterpret_cast<const v4i*>(op + 16 * i);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // this workgroup's tiles: tiles blockIdx.x, blockIdx.x + G, blockIdx.x + 2G, ... (G = gridDim.x) of the
  // [pb, pe) range, at most tpw of them, streamed as S = ntiles·T steps of 64 lights through one pipeline (only
  // the first step waits for HBM cold).  Interleaved, not consecutive, tiles: the workgroups sweep the planes
  // in step, so at any moment the chip reads one contiguous G-tile slab of each plane (c4 u8
  // 1.91 ms with each workgroup on its own consecutive run of tiles)
  const int64_t ntot = (pe - pb + Q8_R - 1) / Q8_R;
  const int G = gridDim.x;
  const int ntiles = (int)min((int64_t)tpw, (ntot - blockIdx.x + G - 1) / G);
  const int S = ntiles * T;
  auto tile_px = [&](int ti) { return pb + ((int64_t)ti * G + blockIdx.x) * Q8_R; };
  const unsigned char* __restrict__ src = I + (int64_t)blockIdx.y * cstride;

  auto load = [&](int s, v4i (&st)[8]) {
    const int ti = s / T, t = s - ti * T;
    int64_t px = tile_px(ti) + 16 * lane;
    px = px < pe ? px : pe - 16;  // lanes past the image re-read its last 16 pixels (never stored)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int n = t * Q8_STEP + 8 * wave + j;
      n = n < N ? n : N - 1;  // lights past N carry zero weights
      st[j] = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(src + (int64_t)n * lstride + px));
    }
  };
  auto park = [&](int b, const v4i (&st)[8]) {
    unsigned char* tb = tile + b * (Q8_STEP * Q8_RS) + (8 * wave) * Q8_RS + 16 * lane;
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<v4i*>(tb + j * Q8_RS) = st[j] ^ (int)0x80808080;
  };

  v4i acc[Q8_G][Q8_DIGITS];
  auto zero = [&]() {
#pragma unroll
    for (int c = 0; c < Q8_G; ++c)
#pragma unroll
      for (int d = 0; d < Q8_DIGITS; ++d) acc[c][d] = v4i{0, 0, 0, 0};
  };
  zero();

  // transposed-read address of this lane: group g reads rows 8g + q (and 32 + 8g + q), q = (lane & 15) >> 1,
  // bytes 8·(lane & 1) of each 16-pixel column group
  const int g = lane >> 4;
  const int roff = (8 * g + ((lane & 15) >> 1)) * Q8_RS + 8 * (lane & 1) + Q8_WPX * wave;
  auto compute = [&](int b, int t) {
    v4i a[Q8_DIGITS];
#pragma unroll
    for (int d = 0; d < Q8_DIGITS; ++d)
      a[d] = *reinterpret_cast<const v4i*>(lfrag + (((t * Q8_DIGITS + d) * 64) + lane) * 16);
    const unsigned char* tb = tile + b * (Q8_STEP * Q8_RS) + roff;
#pragma unroll
    for (int c = 0; c < Q8_G; ++c) {
      const v2i lo = tr8(tb + 16 * c), hi = tr8(tb + 32 * Q8_RS + 16 * c);
      const v4i x = {lo[0], lo[1], hi[0], hi[1]};
#pragma unroll
      for (int d = 0; d < Q8_DIGITS; ++d) acc[c][d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[d], x, acc[c][d], 0, 0, 0);
    }
  };

  // per-row scale and sign-flip corrections of the coefficients (rows 4g .. 4g+3 for this lane), read per
  // tile from the LDS copy of the operator rather than held in registers across the stream
  const double* scale = reinterpret_cast<const double*>(lfrag + q8_frag_bytes(N));
  const int* corr = reinterpret_cast<const int*>(scale + 16);
  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
  // acc[c][d][r] = digit d's sum for coefficient 4g + r of pixel t0 + 128·wave + 16c + (lane & 15); the stores
  // of tile i are issued while the loads of tile i + 1 are in flight
  // Pixel-major rows leave through LDS: the wave parks its 128 pixels' rows (128·K floats, contiguous in
  // coef) in ITS OWN rows 8·wave .. 8·wave + 7 of the tile buffer that is free at that point (no other wave
  // writes them; every wave finished reading that buffer before the last barrier), reads them back 16 B per
  // lane at a 1 KiB stride and stores whole 1 KiB runs per instruction (the direct form writes 8-B pieces of
  // 24-B rows from half the lanes).  `fb` = the free tile buffer.  STAGE = RTI_KERNEL_STAGE (measurement).
  auto finish = [&](int ti, int fb) {
    const int64_t t0 = tile_px(ti);
    double sc[4];
    int cr[4][Q8_DIGITS];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = 4 * g + r < K ? scale[4 * g + r] : 0.0;
#pragma unroll
      for (int d = 0; d < Q8_DIGITS; ++d) cr[r][d] = 4 * g + r < K ? corr[(4 * g + r) * Q8_DIGITS + d] : 0;
    }
    auto value = [&](int c, int r) {
      double sm = (double)(acc[c][0][r] + cr[r][0]);  // exact: |Σ| < 2^53 for N < 2^18
#pragma unroll
      for (int d = 1; d < Q8_DIGITS; ++d) sm = fma(sm, 128.0, (double)(acc[c][d][r] + cr[r][d]));
      return (float)(sm * sc[r]);
    };
    if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR && STAGE) {
      float* __restrict__ st = reinterpret_cast<float*>(tile + fb * (Q8_STEP * Q8_RS) + (8 * wave) * Q8_RS);
      if (4 * g < K) {
#pragma unroll
        for (int c = 0; c < Q8_G; ++c) {
          float* row = st + (16 * c + (lane & 15)) * K + 4 * g;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (4 * g + r < K) row[r] = value(c, r);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int CH = Q8_WPX * K / 4;  // 16-B chunks of the wave's rows: 192 (K = 6) .. 512 (K = 16)
      const int64_t pw = t0 + Q8_WPX * wave;
      float* __restrict__ wdst = dst + pw * K;
#pragma unroll
      for (int i = lane; i < CH; i += 64) {
        // a chunk never straddles a 16-pixel block (16·K floats = 4K chunks), and pe is 16-pixel aligned
        if (pw + (4 * i) / K < pe)
          *reinterpret_cast<floatx4*>(wdst + 4 * i) = *reinterpret_cast<const floatx4*>(st + 4 * i);
      }
    } else if (4 * g < K) {
#pragma unroll
      for (int c = 0; c < Q8_G; ++c) {
        const int64_t p = t0 + Q8_WPX * wave + 16 * c + (lane & 15);
        if (p >= pe) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = value(c, r);
        q8_store<K, LAYOUT>(dst, P, p, g, v);
      }
    }
    zero();
  };
  // The stream loop keeps every vector-memory operation unconditional or in a fixed place, so the compiler's
  // counted vmcnt waits stay exact (a load or store on one branch of a loop makes it wait conservatively,
  // which here drained the prefetch every step): loads of steps past the end re-read step S − 1, an odd
  // stream gets one dummy step that is parked but not computed, and a finished tile's stores are issued at
  // the start of the next step, before that step's loads, so waiting for the older step never waits for
  // the newer one.  Two steps of loads in flight (128 KiB per CU): sb holds step s + 1 (loaded during step
  // s − 1), sa receives step s + 2; the roles swap every step.
  v4i sa[8], sb[8];
  load(0, sa);
  load(S > 1 ? 1 : 0, sb);
  park(0, sa);
  __syncthreads();
  const int S2 = S + (S & 1);
  for (int s = 0; s < S2; s += 2) {
    if (s > 0 && s % T == 0) finish(s / T - 1, 1);
    load(min(s + 2, S - 1), sa);
    compute(0, s % T);
    park(1, sb);
    __syncthreads();
    if (s + 1 < S && (s + 1) % T == 0) finish((s + 1) / T - 1, 0);
    load(min(s + 3, S - 1), sb);
    if (s + 1 < S) compute(1, (s + 1) % T);
    park(0, sa);
    __syncthreads();
  }
  finish(ntiles - 1, 0);
}

struct Q8Args {
  const unsigned char* op;
  int k, N;
  const unsigned char* I;
  int64_t P, lstride, cstride;
  int C;
  float* coef;
  int layout;
  int64_t ocstride;
  hipStream_t s;
  int64_t pb = 0, pe = 0;
  int tpw = 1;  // consecutive tiles streamed by one workgroup
  bool stage = false;  // pixel-major rows staged through LDS (RTI_KERNEL_STAGE)
};

size_t q8_lds_bytes(int N) { return (size_t)q8_operator_bytes(N) + (size_t)2 * Q8_STEP * Q8_RS; }

template <int K, int LAYOUT>
int launch_q8_t(const Q8Args& a) {
  const size_t lds = q8_lds_bytes(a.N);
  auto kern = a.stage ? fit_q8<K, LAYOUT, true> : fit_q8<K, LAYOUT, false>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared_q8: cannot reserve %zu B of LDS", lds);
  const int64_t pe = a.pe ? a.pe : a.P;
  const int64_t tiles = (pe - a.pb + Q8_R - 1) / Q8_R;
  const int tpw = a.tpw > 0 ? a.tpw : 1;
  const dim3 grid((unsigned)((tiles + tpw - 1) / tpw), a.C);  // workgroup w streams tiles w, w + G, ...
  hipLaunchKernelGGL(kern, grid, dim3(64 * Q8_W), lds, a.s, a.op, a.N, a.I, a.pb, pe, tpw, a.P, a.lstride, a.cstride,
                     a.coef, a.ocstride);
  return check_launch("rti_fit_shared_q8");
}

template <int K>
int launch_q8_l(const Q8Args& a) {
  return a.layout == RTI_COEF_PLANAR ? launch_q8_t<K, RTI_COEF_PLANAR>(a) : launch_q8_t<K, RTI_COEF_PIXEL_MAJOR>(a);
}

int launch_q8(const Q8Args& a) {
  switch (a.k) {
    case 6: return launch_q8_l<6>(a);
    case 9: return launch_q8_l<9>(a);
    case 16: return launch_q8_l<16>(a);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_q8: k=%d (supported: 6, 9, 16)", a.k);
  }
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_fit_shared_q8_max_lights(void) {
  int n = Q8_STEP;
  while (q8_lds_bytes(n + Q8_STEP) <= 160 * 1024) n += Q8_STEP;
  return n;
}

extern "C" int rti_fit_shared_q8(const void* op, int k, int N, const uint8_t* I, int64_t P, int C,
                                 int64_t light_stride, int64_t channel_stride, float* coef, int coef_layout,
                                 int64_t coef_channel_stride, int kernel, rti_stream_t stream) {
  if (!kernel_bits_ok(kernel, RTI_KERNEL_AUTO, RTI_KERNEL_STAGE | RTI_FIELD_CHUNKS | RTI_FIELD_TILE_DEPTH))
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: unknown kernel bits 0x%x", kernel);
  if (!op || !I || !coef) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: null pointer");
  if (N <= 0 || P <= 0 || C <= 0 || C > 65535) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: bad N/P/C");
  if (N < k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: N=%d < k=%d", N, k);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: coef layout %d", coef_layout);
  if (N > rti_fit_shared_q8_max_lights())
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_q8: N=%d > %d (LDS)", N, rti_fit_shared_q8_max_lights());
  Q8Args a;
  a.op = static_cast<const unsigned char*>(op);
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
  a.s = (hipStream_t)stream;
  if (a.lstride < P) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: light_stride < P");
  if (C > 1 && a.cstride < (int64_t)N * a.lstride) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: channel_stride");
  if (C > 1 && a.ocstride < P * k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_q8: coef_channel_stride");
  // 16-byte lane loads of 16 pixels; coefficient rows stored as float2/float4 where k allows
  if (P % 16 || a.lstride % 16 || a.cstride % 16 || !aligned_to(I, 16) || !aligned_to(op, 16) ||
      !aligned_to(coef, 16) || a.ocstride % 4)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_q8: needs P, strides and pointers 16-byte aligned");
  note_launches(1);
  // One workgroup per CU (146 KiB of LDS), every workgroup streaming tpw tiles (interleaved with the other
  // workgroups') through its load pipeline: a tile of 1024 pixels x N <= 448 lights is only 2-7 steps, and
  // started cold each tile would wait for HBM once.  AUTO: one launch over the channels, tpw = ceil(tiles per channel / workgroups per
  // channel) with about one workgroup per CU; RTI_KERNEL_CHUNKS(n) sets tpw = n (measurement).
  // RTI_KERNEL_TILE_DEPTH(n) (measurement): n launch generations over consecutive pixel ranges of every
  // channel, each streamed by the same workgroups (the fp32 stream's launch generations, rti_fit.hip)
  const int64_t tpc = (P + Q8_R - 1) / Q8_R, cus = device_cus();
  const int want = (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF;
  a.stage = (kernel & RTI_KERNEL_STAGE) != 0;
  const int parts = std::max(1, (kernel >> RTI_KERNEL_TILE_DEPTH_SHIFT) & 0xF);
  const int64_t wpc = cus >= C ? cus / C : 1;  // workgroups per channel: at most one per CU over all channels
  const int64_t tpp = (tpc + parts - 1) / parts;  // tiles per part
  a.tpw = want ? want : (int)((tpp + wpc - 1) / wpc);
  if (parts == 1) return launch_q8(a);
  int launches = 0;
  for (int i = 0; i < parts; ++i) {
    a.pb = i * tpp * Q8_R;
    a.pe = std::min(P, (i + 1) * tpp * Q8_R);
    if (a.pb >= a.pe) break;
    const int st = launch_q8(a);
    if (st != RTI_OK) return st;
    note_launches(++launches);
  }
  return RTI_OK;
}
