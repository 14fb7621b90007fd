// rti_fit_h16.hip -- shared-direction fit of 8-bit stacks on the fp16 matrix cores (gfx950).
//
// The int8 form (rti_fit_q8.hip) keeps 4 digits × 16 MFMA rows of int32 sums per pixel, so a wave holds
// 128 pixels and reads one 1-KiB row per plane: the short per-wave runs that cost the fp32 stream 15 %
// (DESIGN.md §4.1, §4.1d).  Here the operator is split as w·s = hi + lo in fp16 (s a power of two per row:
// 22 significant bits, as the split-fp16 table operator, rti_operator.hip) and both halves accumulate into
// ONE fp32 sum per coefficient row: 16 sums per pixel, a quarter of the int8 form's, so a wave holds 256
// pixels and the 2048-pixel tile gives 2-KiB runs per wave and plane with 32-light steps
// (v_mfma_f32_16x16x32_f16):
//
//   * a 512-thread workgroup streams tiles of R pixels × 32-light steps (R = 2048, one workgroup per CU, or
//     since r04 R = 1024 with two per CU — AUTO for k <= 9); per step wave w loads planes 4w..4w+3 of the tile
//     (R/1024 16-byte non-temporal loads per lane and plane) into a double-buffered LDS tile [2][32][R + 16];
//     two steps of loads in flight (128 KiB per CU);
//   * B operands come back with ds_read_b64_tr_b8 (8 lights of one pixel per lane) and are widened to fp16
//     exactly: a byte permute makes 1024 + x (0x64xx), a packed fp16 add of −1024 leaves x;
//   * epilogue: the fp32 sums scaled by 1/s, stored like the q8 form's.
// Accuracy: the fp32 stream's (22-bit operator, fp32 accumulation).  Traffic = the algorithmic bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "rti_internal.h"

namespace rti {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

constexpr int H16_W = 8;     // waves per workgroup
constexpr int H16_PAD = 32;  // operator rows padded to whole 32-light steps

// operator: fp16 hi[16][Npad], lo[16][Npad] (row i = coefficient, Npad = N rounded up to 32, zero padded) +
// float inv_s[16]; A fragments are read straight from its LDS copy (8 or 16 contiguous bytes per lane)
__host__ __device__ constexpr int h16_npad(int N) { return (N + H16_PAD - 1) / H16_PAD * H16_PAD; }
__host__ __device__ constexpr int64_t h16_half_bytes(int N) { return (int64_t)16 * h16_npad(N) * 2; }
__host__ __device__ constexpr int64_t h16_operator_bytes(int N) { return 2 * h16_half_bytes(N) + 16 * 4; }

// Tile geometry: R pixels × STEP lights per step (v_mfma_f32_16x16x32_f16: 8 lights per lane), double-buffered
// in LDS with a 16-byte row pad.  (A 4096-pixel × 16-light form on v_mfma_f32_16x16x16_f16 — 4-KiB runs, the
// LDS the same — measured slower: c3 u8 0.228 vs 0.193 ms, it needs 128 accumulator VGPRs and spills.)
template <int R, int STEP, int W = H16_W>
struct H16Tile {
  static constexpr int RS = R + 16;           // LDS row stride: 16 consecutive rows span all 64 banks
  static constexpr int WPX = R / W;           // pixels per wave
  static constexpr int G = WPX / 16;          // 16-pixel column groups per wave
  static constexpr int PPW = STEP / W;        // planes per wave and step
  static constexpr int LPP = R / 1024;        // 16-byte lane loads per plane
  static constexpr int NL = PPW * LPP;        // lane loads per step
  static constexpr size_t tile_bytes = (size_t)2 * STEP * RS;
};
template <int R, int STEP>
size_t h16_lds_bytes(int N) { return (size_t)h16_operator_bytes(N) + H16Tile<R, STEP>::tile_bytes; }

__device__ __forceinline__ v2i tr8(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(p));
}

// bytes -> exact fp16: v_perm_b32 interleaves each byte with 0x64 (fp16 0x64xx = 1024 + x), a packed add of
// −1024 leaves x
__device__ __forceinline__ unsigned lo2(unsigned d) { return __builtin_amdgcn_perm(d, 0x64646464u, 0x00050004u); }
__device__ __forceinline__ unsigned hi2(unsigned d) { return __builtin_amdgcn_perm(d, 0x64646464u, 0x00070006u); }
__device__ __forceinline__ half8 widen8(v2i r) {
  const v4i w = {(int)lo2((unsigned)r[0]), (int)hi2((unsigned)r[0]), (int)lo2((unsigned)r[1]), (int)hi2((unsigned)r[1])};
  return __builtin_bit_cast(half8, w) - (half8)(_Float16)1024.0f;
}
// NT: non-temporal stores (the probe build's measurement variant)
template <int K, int LAYOUT, bool NT = false>
__device__ __forceinline__ void h16_store(float* __restrict__ dst, int64_t P, int64_t p, int g, const float (&v)[4]) {
  // v[r] = coefficient 4g + r of pixel p
  auto st = [](auto* q, auto x) {
    if constexpr (NT)
      __builtin_nontemporal_store(x, q);
    else
      *q = x;
  };
  if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < K) st(dst + (int64_t)(4 * g + r) * P + p, v[r]);
  } else if constexpr (K == 16) {
    st(reinterpret_cast<floatx4*>(dst + p * 16 + 4 * g), floatx4{v[0], v[1], v[2], v[3]});
  } else if constexpr (K % 2 == 0) {
#pragma unroll
    for (int r = 0; r < 4; r += 2)
      if (4 * g + r < K) st(reinterpret_cast<floatx2*>(dst + p * K + 4 * g + r), floatx2{v[r], v[r + 1]});
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < K) st(dst + p * K + 4 * g + r, v[r]);
  }
}

// CB: 16-pixel groups whose reads and MFMAs are batched per step (AUTO 4; 1 one group at a time)
// PROBE (not reachable from the C ABI; tools/probe/h16_probe.hip): 1 = the coefficient stores dropped, 2 = the
// per-lane stores non-temporal, 5 / 6 = as 1 with the transposed reads and MFMAs dropped / with those and the
// LDS parking dropped (the load pipeline alone)
// W: waves per workgroup (8; 16 with the 2048-pixel tile = 2-KiB runs per plane and wave)
// SM (PTM-6, pixel-major, 1024-pixel tiles on 8 waves): 0 per-lane coefficient stores, 1 / 2 each wave's 128
// finished rows staged in the free half of the LDS tile and written back as three whole 1-KiB lines, plain /
// non-temporal (2: AUTO since r05)
template <int K, int LAYOUT, int R, int STEP, int CB = 1, int PROBE = 0, int W = H16_W, int SM = 0>
__global__ void __launch_bounds__(64 * W)
fit_h16(const unsigned char* __restrict__ op, int N, const unsigned char* __restrict__ I, int64_t pb, int64_t pe,
        int tpw, int64_t P, int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  using TL = H16Tile<R, STEP, W>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int T = (N + STEP - 1) / STEP, Np = h16_npad(N);
  unsigned char* __restrict__ lop = lds;                           // hi[16][Np], lo[16][Np] fp16, inv_s[16]
  unsigned char* __restrict__ tile = lds + h16_operator_bytes(N);   // [2][STEP][RS]
  for (int i = threadIdx.x; i < (int)(h16_operator_bytes(N) / 16); i += 64 * W)
    *reinterpret_cast<v4i*>(lop + 16 * i) = *reinterpret_cast<const v4i*>(op + 16 * i);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // this workgroup's tiles: blockIdx.x, blockIdx.x + G, ... of the [pb, pe) range (at most tpw), streamed as
  // S = ntiles·T steps through one pipeline (the q8 form's interleaved tile streams)
  const int64_t ntot = (pe - pb + R - 1) / R;
  const int G = gridDim.x;
  const int ntiles = (int)min((int64_t)tpw, (ntot - blockIdx.x + G - 1) / G);
  const int S = ntiles * T;
  auto tile_px = [&](int ti) { return pb + ((int64_t)ti * G + blockIdx.x) * R; };
  const unsigned char* __restrict__ src = I + (int64_t)blockIdx.y * cstride;

  auto load = [&](int s, v4i (&st)[TL::NL]) {
    const int ti = s / T, t = s - ti * T;
    const int64_t px0 = tile_px(ti) + 16 * lane;
#pragma unroll
    for (int j = 0; j < TL::PPW; ++j) {
      int n = t * STEP + TL::PPW * wave + j;
      n = n < N ? n : N - 1;  // lights past N carry zero weights (re-reads of plane N − 1: L2 hits; zero-record
                              // buffer loads in their place measured flat, profiles/r05v_h16_ab_*, r05f_*)
#pragma unroll
      for (int h = 0; h < TL::LPP; ++h) {
        int64_t px = px0 + 1024 * h;
        px = px < pe ? px : pe - 16;  // lanes past the image re-read its last 16 pixels (never stored)
        st[j * TL::LPP + h] = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(src + (int64_t)n * lstride + px));
      }
    }
  };
  int sink = 0;  // PROBE 6: the loads' use when nothing is parked
  auto park = [&](int b, const v4i (&st)[TL::NL]) {
    if constexpr (PROBE == 6) {
#pragma unroll
      for (int j = 0; j < TL::NL; ++j) sink ^= st[j][0] ^ st[j][3];
      return;
    }
    unsigned char* tb = tile + b * (STEP * TL::RS) + (TL::PPW * wave) * TL::RS + 16 * lane;
#pragma unroll
    for (int j = 0; j < TL::PPW; ++j)
#pragma unroll
      for (int h = 0; h < TL::LPP; ++h) *reinterpret_cast<v4i*>(tb + j * TL::RS + 1024 * h) = st[j * TL::LPP + h];
  };

  floatx4 acc[TL::G];
  auto zero = [&]() {
#pragma unroll
    for (int c = 0; c < TL::G; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  };
  zero();

  // B operand: lane group g = lane >> 4 needs lights 8g .. 8g + 7 of its column (lane & 15): the transposed
  // read gives a lane those 8 rows of one column, rows 8g + q addressed by lane (q, h) = ((lane & 15) >> 1,
  // lane & 1) of the group (bytes 8h of each 16-pixel column group).  A: row lane & 15, the same 8 lights.
  static_assert(STEP == 32, "v_mfma_f32_16x16x32_f16 steps");
  const int g = lane >> 4;
  const int roff = (8 * g + ((lane & 15) >> 1)) * TL::RS + 8 * (lane & 1) + TL::WPX * wave;
  const int arow = (lane & 15) * Np + 8 * g;
  auto compute = [&](int b, int t) {
    if constexpr (PROBE == 5 || PROBE == 6) return;  // (probe: no transposed reads, no MFMAs)
    const unsigned char* tb = tile + b * (STEP * TL::RS) + roff;
    const half8 ah = *reinterpret_cast<const half8*>(lop + 2 * (arow + t * STEP));
    const half8 al = *reinterpret_cast<const half8*>(lop + h16_half_bytes(N) + 2 * (arow + t * STEP));
    if constexpr (CB == 1) {
#pragma unroll
      for (int c = 0; c < TL::G; ++c) {
        const half8 x = widen8(tr8(tb + 16 * c));
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, x, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, x, acc[c], 0, 0, 0);
      }
    } else {
      // batches of CB groups: their transposed reads issued together, then the hi MFMAs of the batch, then the
      // lo ones (each accumulator's two MFMAs CB apart instead of back to back)
#pragma unroll
      for (int c0 = 0; c0 < TL::G; c0 += CB) {
        v2i raw[CB];
#pragma unroll
        for (int c = 0; c < CB; ++c) raw[c] = tr8(tb + 16 * (c0 + c));
        half8 x[CB];
#pragma unroll
        for (int c = 0; c < CB; ++c) x[c] = widen8(raw[c]);
#pragma unroll
        for (int c = 0; c < CB; ++c)
          acc[c0 + c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, x[c], acc[c0 + c], 0, 0, 0);
#pragma unroll
        for (int c = 0; c < CB; ++c)
          acc[c0 + c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, x[c], acc[c0 + c], 0, 0, 0);
      }
    }
  };

  const float* inv_s = reinterpret_cast<const float*>(lop + 2 * h16_half_bytes(N));
  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
  // acc[c][r] = coefficient 4g + r of pixel t0 + WPX·wave + 16c + (lane & 15) (scaled by s)
  auto finish = [&](int ti) {
    const int64_t t0 = tile_px(ti);
    if (4 * g < K) {
      float sc[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[r] = inv_s[4 * g + r];
#pragma unroll
      for (int c = 0; c < TL::G; ++c) {
        const int64_t p = t0 + TL::WPX * wave + 16 * c + (lane & 15);
        if (p >= pe) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[c][r] * sc[r];
        if constexpr (PROBE == 1 || PROBE == 5 || PROBE == 6) {
          if (v[0] + v[1] + v[2] + v[3] == -1.2345f || sink == 0x7a5a5a5b) dst[0] = v[0];  // keeps the work alive
        } else {
          h16_store<K, LAYOUT, PROBE == 2>(dst, P, p, g, v);
        }
      }
    }
    zero();
  };
  // staged form (PROBE 3 / 4): the wave's 128 rows of 6 coefficients (3 KiB) parked in its slice of the free tile
  // buffer fb, read back as 16-B chunks 16·lane + 1 KiB·j and written as whole lines; the caller's barrier keeps
  // the other waves from parking into fb before every wave has read its slice back
  constexpr bool STG = SM != 0 && K == 6 && R == 1024 && W == 8 && LAYOUT == RTI_COEF_PIXEL_MAJOR && PROBE == 0;
  auto finish_staged = [&](int ti, int fb) {
    const int64_t w0 = tile_px(ti) + TL::WPX * wave;  // the wave's first pixel (1-KiB aligned rows)
    float* slice = reinterpret_cast<float*>(tile + fb * (STEP * TL::RS)) + wave * (TL::WPX * 6);
    if (g < 2) {
      float sc[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[r] = inv_s[(4 * g + r) & 7];
#pragma unroll
      for (int c = 0; c < TL::G; ++c) {
        float* row = slice + (16 * c + (lane & 15)) * 6 + 4 * g;
        *reinterpret_cast<floatx2*>(row) = floatx2{acc[c][0] * sc[0], acc[c][1] * sc[1]};
        if (g == 0) *reinterpret_cast<floatx2*>(row + 2) = floatx2{acc[c][2] * sc[2], acc[c][3] * sc[3]};
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int f = 256 * j + 4 * lane;  // the lane's first float of the wave's 768
      const floatx4 v = *reinterpret_cast<const floatx4*>(slice + f);
      float* d = dst + w0 * 6 + f;
      if (w0 + (f + 3) / 6 < pe) {
        if constexpr (SM == 2)
          __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(d));
        else
          *reinterpret_cast<floatx4*>(d) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (w0 + (f + e) / 6 < pe) d[e] = v[e];
      }
    }
    zero();
  };
  // The stream loop of the q8 form: every vector-memory operation unconditional or in a fixed place (exact
  // counted vmcnt waits), loads of steps past the end re-read step S − 1, an odd stream gets one dummy step,
  // a finished tile's stores are issued at the start of the next step, before that step's loads; sb holds
  // step s + 1, sa receives step s + 2.
  v4i sa[TL::NL], sb[TL::NL];
  load(0, sa);
  load(S > 1 ? 1 : 0, sb);
  park(0, sa);
  __syncthreads();
  const int S2 = S + (S & 1);
  for (int s = 0; s < S2; s += 2) {
    if (s > 0 && s % T == 0) {
      if constexpr (STG) {  // buffer 1 is free here (its step was computed before the last barrier)
        finish_staged(s / T - 1, 1);
        __syncthreads();
      } else {
        finish(s / T - 1);
      }
    }
    load(min(s + 2, S - 1), sa);
    compute(0, s % T);
    park(1, sb);
    __syncthreads();
    if (s + 1 < S && (s + 1) % T == 0) {
      if constexpr (STG) {  // buffer 0 is free here
        finish_staged((s + 1) / T - 1, 0);
        __syncthreads();
      } else {
        finish((s + 1) / T - 1);
      }
    }
    load(min(s + 3, S - 1), sb);
    if (s + 1 < S) compute(1, (s + 1) % T);
    park(0, sa);
    __syncthreads();
  }
  if constexpr (STG)
    finish_staged(ntiles - 1, 0);
  else
    finish(ntiles - 1);
}

template <int K, int LAYOUT, int R, int STEP, int W = H16_W>
int launch_h16_t(const unsigned char* op, int N, const unsigned char* I, int64_t P, int C, int64_t ls, int64_t cs,
                 float* coef, int64_t ocs, int tpw, int cb, hipStream_t s) {
  const size_t lds = h16_lds_bytes<R, STEP>(N);
  if (lds > 160 * 1024)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_h16: LDS of %zu B (N=%d) exceeds 160 KiB", lds, N);
  // AUTO batches 4 groups per read/MFMA round (c2 u8 0.0379 against 0.0443 ms one group at a time, c3 / c4 u8
  // within 1 %: profiles/r04z_h16_batch_sweep_c*.log); RTI_KERNEL_TILE_DEPTH(1|8) for measurement
  // PTM-6 pixel-major on 1024-pixel tiles: staged whole-line non-temporal coefficient stores (r05; c3 u8
  // 0.1833 vs 0.2148 ms, 0.1871 vs 0.1894 and 0.1909 vs 0.1899 on three boxes, bit-identical:
  // profiles/r05am_*, r05af_*, r05j_*)
  constexpr int SM = (K == 6 && R == 1024 && W == 8 && LAYOUT == RTI_COEF_PIXEL_MAJOR) ? 2 : 0;
  auto kern = cb == 8   ? fit_h16<K, LAYOUT, R, STEP, 8, 0, W, SM>
              : cb == 1 ? fit_h16<K, LAYOUT, R, STEP, 1, 0, W, SM>
                        : fit_h16<K, LAYOUT, R, STEP, 4, 0, W, SM>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared_h16: cannot reserve %zu B of LDS", lds);
  const int64_t tiles = (P + R - 1) / R;
  const dim3 grid((unsigned)((tiles + tpw - 1) / tpw), C);
  hipLaunchKernelGGL(kern, grid, dim3(64 * W), lds, s, op, N, I, (int64_t)0, P, tpw, P, ls, cs, coef, ocs);
  return check_launch("rti_fit_shared_h16");
}

struct H16Args {
  const unsigned char* op;
  int N;
  const unsigned char* I;
  int64_t P;
  int C;
  int64_t ls, cs;
  float* coef;
  int64_t ocs;
  int want;  // RTI_KERNEL_CHUNKS: tiles per workgroup (0 = AUTO)
  int cb;    // RTI_KERNEL_TILE_DEPTH: batched groups (measurement)
  hipStream_t s;
  int geom = 0;  // RTI_KERNEL_TILE_WAVES: 0 AUTO, 1 the 2048-pixel tile on 8 waves, 2 the 1024-pixel tile, 3 2048 on 16
};

template <int K, int LAYOUT, int R, int STEP, int W = H16_W>
int launch_h16_g(const H16Args& a) {
  // one workgroup per CU over all channels, each streaming tpw interleaved tiles
  const int64_t tpc = (a.P + R - 1) / R, cus = device_cus();
  const int64_t wpc = (cus >= a.C ? cus / a.C : 1) * (2048 / R);  // workgroups per channel: 2048/R per CU
  const int tpw = a.want ? a.want : (int)((tpc + wpc - 1) / wpc);
  return launch_h16_t<K, LAYOUT, R, STEP, W>(a.op, a.N, a.I, a.P, a.C, a.ls, a.cs, a.coef, a.ocs, tpw, a.cb, a.s);
}

// AUTO geometry: 1024-pixel tiles (1-KiB runs per wave and plane, two workgroups per CU) for k <= 9 where two
// fit in the LDS, else the 2048-pixel tile (one per CU).  Two independent workgroups per CU overlap each other's
// per-step barrier: c2 u8 0.036 vs 0.0395 ms, c3 u8 0.187 vs 0.193; HSH-16 c4 u8 1.29 either way
// (profiles/r04h_h16_geometry_sweep_c*.log, bit-identical).
bool h16_half_tiles(int k, int N, int geom) {
  if (geom) return geom == 2;
  return k <= 9 && h16_lds_bytes<1024, 32>(N) <= 80 * 1024;
}

template <int K>
int launch_h16_l(int layout, const H16Args& a) {
  // the 2048-pixel tile on 16 waves (2-KiB runs per plane and wave; AUTO where the 1024-pixel tile is not):
  // c4 u8 1.282 vs 1.308 ms on 8 waves, c3 u8 0.1866 vs 0.1866 on 1024-pixel tiles (profiles/r05w_h16_geometry_*)
  if (a.geom == 3 || (a.geom == 0 && !h16_half_tiles(K, a.N, 0)))
    return layout == RTI_COEF_PLANAR ? launch_h16_g<K, RTI_COEF_PLANAR, 2048, 32, 16>(a)
                                     : launch_h16_g<K, RTI_COEF_PIXEL_MAJOR, 2048, 32, 16>(a);
  if (h16_half_tiles(K, a.N, a.geom))
    return layout == RTI_COEF_PLANAR ? launch_h16_g<K, RTI_COEF_PLANAR, 1024, 32>(a)
                                     : launch_h16_g<K, RTI_COEF_PIXEL_MAJOR, 1024, 32>(a);
  return layout == RTI_COEF_PLANAR ? launch_h16_g<K, RTI_COEF_PLANAR, 2048, 32>(a)
                                   : launch_h16_g<K, RTI_COEF_PIXEL_MAJOR, 2048, 32>(a);
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int64_t rti_h16_operator_bytes(int k, int N) {
  if (k < 1 || k > 16 || N <= 0) return -1;
  return h16_operator_bytes(N);
}

// Host: pinv [k][N] fp64 -> hi, lo [16][Npad] fp16 with w·s_i = hi + lo (s_i = 2^(14 − ⌊log2 max_n|w_in|⌋):
// max|w·s| in [2^14, 2^15)) and inv_s[i] = 1/s_i; rows >= k and lights >= N zero.
extern "C" int rti_h16_operator(const double* pinv, int k, int N, void* op) {
  if (!pinv || !op) return fail(RTI_ERR_BAD_ARG, "rti_h16_operator: null pointer");
  if (k < 1 || k > 16 || N <= 0) return fail(RTI_ERR_BAD_ARG, "rti_h16_operator: k=%d N=%d", k, N);
  const int Np = h16_npad(N);
  _Float16* hi = static_cast<_Float16*>(op);
  _Float16* lo = hi + (size_t)16 * Np;
  float* inv_s = reinterpret_cast<float*>(lo + (size_t)16 * Np);
  for (int i = 0; i < 16; ++i) {
    double sc = 1.0;
    inv_s[i] = 0.f;
    if (i < k) {
      double m = 0.0;
      for (int n = 0; n < N; ++n) {
        const double w = pinv[(size_t)i * N + n];
        if (!std::isfinite(w))
          return fail(RTI_ERR_BAD_ARG, "rti_h16_operator: non-finite pseudo-inverse entry (row %d, light %d)", i, n);
        m = std::fmax(m, std::fabs(w));
      }
      sc = m > 0.0 ? std::ldexp(1.0, 14 - std::ilogb(m)) : 1.0;
      inv_s[i] = (float)(1.0 / sc);
    }
    for (int n = 0; n < Np; ++n) {
      const double v = (i < k && n < N) ? pinv[(size_t)i * N + n] * sc : 0.0;
      const _Float16 h = (_Float16)v;
      hi[(size_t)i * Np + n] = h;
      lo[(size_t)i * Np + n] = (_Float16)(v - (double)h);
    }
  }
  return RTI_OK;
}

extern "C" int rti_fit_shared_h16_max_lights(void) {
  int n = H16_PAD;
  while (h16_lds_bytes<2048, 32>(n + H16_PAD) <= 160 * 1024) n += H16_PAD;
  return n;
}

extern "C" int rti_fit_shared_h16(const void* op, int k, int N, const uint8_t* I, int64_t P, int C,
                                  int64_t light_stride, int64_t channel_stride, float* coef, int coef_layout,
                                  int64_t coef_channel_stride, int kernel, rti_stream_t stream) {
  if (!kernel_bits_ok(kernel, RTI_KERNEL_AUTO, RTI_FIELD_CHUNKS | RTI_FIELD_TILE_DEPTH | RTI_FIELD_TILE_WAVES))
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: unknown kernel bits 0x%x", kernel);
  if (!op || !I || !coef) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: null pointer");
  if (N <= 0 || P <= 0 || C <= 0 || C > 65535) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: bad N/P/C");
  if (N < k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: N=%d < k=%d", N, k);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: coef layout %d", coef_layout);
  if (N > rti_fit_shared_h16_max_lights())
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_h16: N=%d > %d (LDS)", N, rti_fit_shared_h16_max_lights());
  const int64_t ls = light_stride ? light_stride : P;
  const int64_t cs = channel_stride ? channel_stride : (int64_t)N * ls;
  const int64_t ocs = coef_channel_stride ? coef_channel_stride : P * k;
  if (ls < P) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: light_stride < P");
  if (C > 1 && cs < (int64_t)N * ls) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: channel_stride");
  if (C > 1 && ocs < P * k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_h16: coef_channel_stride");
  if (P > 0x7fffff00)  // plane offsets are 32-bit buffer offsets
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_h16: P=%lld pixels per plane", (long long)P);
  if (P % 16 || ls % 16 || cs % 16 || !aligned_to(I, 16) || !aligned_to(op, 16) || !aligned_to(coef, 16) || ocs % 4)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_h16: needs P, strides and pointers 16-byte aligned");
  note_launches(1);
  // RTI_KERNEL_CHUNKS(n): tiles per workgroup = n; RTI_KERNEL_TILE_DEPTH(1|4|8): groups batched per round;
  // RTI_KERNEL_TILE_WAVES(1|2|3): the 2048- or 1024-pixel tile, or 2048 pixels on 16 waves (measurement)
  const H16Args a{static_cast<const unsigned char*>(op), N, I, P, C, ls, cs, coef, ocs,
                  (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF, (kernel >> RTI_KERNEL_TILE_DEPTH_SHIFT) & 0xF,
                  (hipStream_t)stream, (kernel >> RTI_KERNEL_TILE_WAVES_SHIFT) & 0xF};
  switch (k) {
    case 6: return launch_h16_l<6>(coef_layout, a);
    case 9: return launch_h16_l<9>(coef_layout, a);
    case 16: return launch_h16_l<16>(coef_layout, a);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_h16: k=%d (supported: 6, 9, 16)", k);
  }
}
