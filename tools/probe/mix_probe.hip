// mix_probe.hip -- measurement-only kernels (not part of librti): the mixed read/write HBM
// ceiling of the shared fits' data flow with the arithmetic taken out.
//
// Each kernel reads the light-major stack in exactly the fit's shape and writes exactly the
// fit's coefficient bytes, in whole 1-KiB store instructions, with one add per loaded element
// (to keep the loads alive) instead of the contraction.  PLACE selects where the stores go:
//   0  no stores (the read ceiling of this shape)
//   1  all stores after the wave's last plane (the fits' shape: outputs exist only then)
//   2  the stores spread evenly over the sweep (an ideal pipeline that writes earlier outputs
//      while it reads: the best any store placement inside the read stream can do)
//   3  stores only, no loads (the write ceiling of this pattern)
//   4  as 1, non-temporal stores
//
//  mix_px   : the PTM-6 VALU stream (fit_shared_valu, c3): a wave owns NC·256 pixels, lane l's
//             chunk c is the 4 pixels at wave_base + c·256 + 4l, 8/NC planes per step.
//  mix_tile : the HSH-16 8-wave tile (fit_shared_tile_w<16,8,0>, c4): a W-wave workgroup owns
//             256·RC pixels, wave w reads plane s·W + w of the whole tile per step (RC·1 KiB runs).
// Launch generations as in the library (rti_fit.hip launch_generations): consecutive launches
// over pixel ranges of every plane.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ floatx4 ld_nt(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
}

template <bool NTS>
__device__ __forceinline__ void st4(float* p, floatx4 v) {
  if constexpr (NTS)
    __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p));
  else
    *reinterpret_cast<floatx4*>(p) = v;
}

template <int NC, int OUTF, int PLACE>
__global__ void __launch_bounds__(256) mix_px(const float* __restrict__ I, int N, int64_t P, int64_t pb, int64_t pe,
                                              float* __restrict__ out) {
  constexpr int UP = 8 / NC > 0 ? 8 / NC : 1;
  constexpr int NST = NC * OUTF;  // 1-KiB store instructions per wave (256 pixels x OUTF floats / 1 KiB)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t wb = pb + ((int64_t)blockIdx.x * 4 + wave) * (256 * NC);
  if (wb + 256 * NC > pe) return;  // whole waves only (the host checks P)
  float* o = out + wb * OUTF + 4 * lane;
  floatx4 acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = floatx4{(float)lane, 0.f, 0.f, 0.f};
  const int steps = N / UP;
  int j = 0;
  if constexpr (PLACE != 3) {
    const float* src = I + wb + 4 * lane;
    for (int s = 0; s < steps; ++s) {
      floatx4 x[UP][NC];
#pragma unroll
      for (int u = 0; u < UP; ++u)
#pragma unroll
        for (int c = 0; c < NC; ++c) x[u][c] = ld_nt(src + (int64_t)(s * UP + u) * P + c * 256);
#pragma unroll
      for (int u = 0; u < UP; ++u)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] += x[u][c];
      if constexpr (PLACE == 2) {
        for (; j < NST && j * steps < (s + 1) * NST; ++j) st4<false>(o + j * 256, acc[0] + (float)j);
      }
    }
  }
  if constexpr (PLACE == 0) {
    float t = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    if (t == -1.2345f) o[0] = t;
  } else {
#pragma unroll
    for (int jj = 0; jj < NST; ++jj)
      if (jj >= j) st4<PLACE == 4>(o + jj * 256, acc[jj % NC] + (float)jj);
  }
}

template <int RC, int W, int OUTF, int PLACE>
__global__ void __launch_bounds__(64 * W) mix_tile(const float* __restrict__ I, int N, int64_t P, int64_t tb,
                                                   float* __restrict__ out) {
  constexpr int R = 256 * RC;
  constexpr int NST = RC * OUTF / W;  // 1-KiB store instructions per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t px0 = (tb + blockIdx.x) * (int64_t)R;
  if (px0 + R > P) return;
  float* o = out + px0 * OUTF + (int64_t)wave * NST * 256 + 4 * lane;
  floatx4 acc[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) acc[r] = floatx4{(float)lane, 0.f, 0.f, 0.f};
  const int steps = N / W;
  int j = 0;
  if constexpr (PLACE != 3) {
    const float* src = I + px0 + 4 * lane;
    for (int s = 0; s < steps; ++s) {
      floatx4 x[RC];
      const float* pl = src + (int64_t)(s * W + wave) * P;
#pragma unroll
      for (int r = 0; r < RC; ++r) x[r] = ld_nt(pl + r * 256);
#pragma unroll
      for (int r = 0; r < RC; ++r) acc[r] += x[r];
      if constexpr (PLACE == 2) {
        for (; j < NST && j * steps < (s + 1) * NST; ++j) st4<false>(o + j * 256, acc[0] + (float)j);
      }
    }
  }
  if constexpr (PLACE == 0) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < RC; ++r) t += acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
    if (t == -1.2345f) o[0] = t;
  } else {
#pragma unroll
    for (int jj = 0; jj < NST; ++jj)
      if (jj >= j) st4<PLACE == 4>(o + jj * 256, acc[jj % RC] + (float)jj);
  }
}

template <int NC, int OUTF>
int launch_px(const float* I, int N, int64_t P, float* out, int place, int launches, hipStream_t s) {
  const int64_t wpx = 256 * NC;
  const int64_t waves = P / wpx;
  const int64_t per = (waves + launches - 1) / launches;
  for (int g = 0; g < launches; ++g) {
    const int64_t w0 = g * per, w1 = w0 + per < waves ? w0 + per : waves;
    if (w1 <= w0) break;
    const dim3 grid((unsigned)((w1 - w0 + 3) / 4));
    const int64_t pb = w0 * wpx, pe = w1 * wpx;
    switch (place) {
      case 0: hipLaunchKernelGGL((mix_px<NC, OUTF, 0>), grid, dim3(256), 0, s, I, N, P, pb, pe, out); break;
      case 1: hipLaunchKernelGGL((mix_px<NC, OUTF, 1>), grid, dim3(256), 0, s, I, N, P, pb, pe, out); break;
      case 2: hipLaunchKernelGGL((mix_px<NC, OUTF, 2>), grid, dim3(256), 0, s, I, N, P, pb, pe, out); break;
      case 3: hipLaunchKernelGGL((mix_px<NC, OUTF, 3>), grid, dim3(256), 0, s, I, N, P, pb, pe, out); break;
      default: hipLaunchKernelGGL((mix_px<NC, OUTF, 4>), grid, dim3(256), 0, s, I, N, P, pb, pe, out); break;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

template <int RC, int W, int OUTF>
int launch_tile(const float* I, int N, int64_t P, int C, float* out, int place, int parts, hipStream_t s) {
  const int64_t R = 256 * RC, tiles = P / R, per = (tiles + parts - 1) / parts;
  for (int c = 0; c < C; ++c) {
    const float* Ic = I + (int64_t)c * N * P;
    float* oc = out + (int64_t)c * P * OUTF;
    for (int g = 0; g < parts; ++g) {
      const int64_t t0 = g * per, t1 = t0 + per < tiles ? t0 + per : tiles;
      if (t1 <= t0) break;
      const dim3 grid((unsigned)(t1 - t0)), block(64 * W);
      switch (place) {
        case 0: hipLaunchKernelGGL((mix_tile<RC, W, OUTF, 0>), grid, block, 0, s, Ic, N, P, t0, oc); break;
        case 1: hipLaunchKernelGGL((mix_tile<RC, W, OUTF, 1>), grid, block, 0, s, Ic, N, P, t0, oc); break;
        case 2: hipLaunchKernelGGL((mix_tile<RC, W, OUTF, 2>), grid, block, 0, s, Ic, N, P, t0, oc); break;
        case 3: hipLaunchKernelGGL((mix_tile<RC, W, OUTF, 3>), grid, block, 0, s, Ic, N, P, t0, oc); break;
        default: hipLaunchKernelGGL((mix_tile<RC, W, OUTF, 4>), grid, block, 0, s, Ic, N, P, t0, oc); break;
      }
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

// c3 shape: nc 4 or 8 chunks per lane, outf coefficient floats per pixel (6), `launches` generations.
// Requires P % (256·nc) == 0 and N % (8 / nc) == 0; returns 2 otherwise.
extern "C" int probe_mix_px(const float* I, int N, int64_t P, float* out, int nc, int outf, int place, int launches,
                            void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (P % (256 * nc) != 0 || N % (8 / nc) != 0 || launches < 1) return 2;
  if (nc == 4 && outf == 6) return launch_px<4, 6>(I, N, P, out, place, launches, s);
  if (nc == 8 && outf == 6) return launch_px<8, 6>(I, N, P, out, place, launches, s);
  if (nc == 2 && outf == 6) return launch_px<2, 6>(I, N, P, out, place, launches, s);
  // 8-bit stacks viewed as 4-byte words (16 pixels per lane chunk, 24 output floats per word = PTM-6 fp32)
  if (nc == 1 && outf == 24) return launch_px<1, 24>(I, N, P, out, place, launches, s);
  if (nc == 2 && outf == 24) return launch_px<2, 24>(I, N, P, out, place, launches, s);
  if (nc == 4 && outf == 24) return launch_px<4, 24>(I, N, P, out, place, launches, s);
  if (nc == 8 && outf == 24) return launch_px<8, 24>(I, N, P, out, place, launches, s);
  return 2;
}

// c4 shape: 16 KiB runs (rc 16), 8 waves, outf 16, `parts` launches per channel.
// Requires P % 4096 == 0 and N % 8 == 0; returns 2 otherwise.
extern "C" int probe_mix_tile(const float* I, int N, int64_t P, int C, float* out, int outf, int place, int parts,
                              void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (P % 4096 != 0 || N % 8 != 0 || parts < 1 || outf != 16) return 2;
  return launch_tile<16, 8, 16>(I, N, P, C, out, place, parts, s);
}

// ---- pixel-major stream probes (r04): what the HBM gives a pure 1-KiB-per-instruction stream ------------
// Every wave reads `per` KiB as 1-KiB wave instructions, D instructions in flight, either as LDS-DMA
// (global_load_lds_dwordx4 into a D-KiB ring, counted vmcnt) or as plain global_load_dwordx4 into registers.
// ORDER 0: wave w reads KiB w·per .. (its own contiguous run); 1: KiB w, w + GW, w + 2·GW … (a chip-wide slab).
namespace {
// (a __device__ helper: a builtin called straight from the kernel body drops the host-side launch stub)
__device__ __forceinline__ void glds16(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 2);
}

template <int D, bool DMA, int ORDER, int BURST = 1>
__global__ void __launch_bounds__(512) pm_read(const float* __restrict__ I, int64_t kib, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave, GW = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t per = kib / GW;
  auto kaddr = [&](int64_t i) -> const float* {
    const int64_t k = ORDER == 0 ? gw * per + i : i * GW + gw;
    return I + k * 256 + 4 * lane;
  };
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (DMA) {
    float* rb = ring + wave * D * 256;
#pragma unroll
    for (int i = 0; i < D; ++i)
      glds16(kaddr(i), rb + i * 256);
    if constexpr (BURST == 1) {
      for (int64_t i = D; i < per; ++i) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
        const int s = (int)(i % D);
        acc += *reinterpret_cast<const floatx4*>(rb + s * 256 + 4 * lane);
        glds16(kaddr(i), rb + s * 256);
      }
    } else if constexpr (D > BURST) {  // the fits' shape: wait for BURST KiB, consume them, refill BURST KiB
      for (int64_t i = D; i + BURST <= per; i += BURST) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - BURST) : "memory");
#pragma unroll
        for (int b = 0; b < BURST; ++b) acc += *reinterpret_cast<const floatx4*>(rb + ((i + b) % D) * 256 + 4 * lane);
#pragma unroll
        for (int b = 0; b < BURST; ++b) glds16(kaddr(i + b), rb + ((i + b) % D) * 256);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    int64_t i = 0;
    for (; i + D <= per; i += D) {
      floatx4 x[D];
#pragma unroll
      for (int u = 0; u < D; ++u) x[u] = ld_nt(kaddr(i + u));
#pragma unroll
      for (int u = 0; u < D; ++u) acc += x[u];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == -1.2345f) out[0] = acc[0];
}

template <int D>
int launch_pm_read(const float* I, int64_t bytes, float* out, int dma, int order, int waves, hipStream_t s) {
  const int64_t kib = bytes >> 10;
  const int cus = 256;
  const size_t lds = dma ? (size_t)waves * D * 1024 : 0;
  const dim3 grid(cus), block(64 * waves);
#define PMRB(OR)                                                                                             \
  {                                                                                                          \
    if (lds > 65536)                                                                                         \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pm_read<D, true, OR, 6>),                      \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                       \
    hipLaunchKernelGGL((pm_read<D, true, OR, 6>), grid, block, lds, s, I, kib, out);                          \
  }
#define PMR(DM, OR)                                                                                          \
  {                                                                                                          \
    if (lds > 65536)                                                                                         \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pm_read<D, DM, OR>),                           \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                       \
    hipLaunchKernelGGL((pm_read<D, DM, OR>), grid, block, lds, s, I, kib, out);                               \
  }
  if (dma == 2) {  // bursts of 6 KiB (a 16-pixel group of 100 lights)
    if (order) PMRB(1) else PMRB(0)
  } else if (dma && order) PMR(true, 1) else if (dma) PMR(true, 0) else if (order) PMR(false, 1) else PMR(false, 0)
#undef PMR
#undef PMRB
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

// bytes: the stream (a multiple of 1 KiB × 256 CUs × waves); dma 0/1; order 0/1; waves per CU (<= 8); depth 4/8/16
extern "C" int probe_pm_read(const float* I, int64_t bytes, float* out, int dma, int order, int waves, int depth,
                             void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (waves < 1 || waves > 8 || (bytes >> 10) % (256 * waves) || (bytes >> 10) / (256 * waves) < depth) return 2;
  if (dma && (size_t)waves * depth * 1024 > 160 * 1024) return 2;
  switch (depth) {
    case 4: return dma == 2 ? 2 : launch_pm_read<4>(I, bytes, out, dma, order, waves, s);
    case 8: return launch_pm_read<8>(I, bytes, out, dma, order, waves, s);
    case 16: return launch_pm_read<16>(I, bytes, out, dma, order, waves, s);
    default: return 2;
  }
}
