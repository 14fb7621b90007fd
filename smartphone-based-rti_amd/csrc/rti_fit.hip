// rti_fit.hip -- shared-direction PTM/HSH fit on gfx950 (MI355X).
//
// Replaces the per-pixel loop of interpolate_intensities + the SVD solve of
// _interpolate_PTM (analysis.py:321-363, :293-298) for a shared light set:
//     coef[c][p][i] = Σ_n pinv[i][n] · I[c][n][p]
// i.e. the k×N pseudo-inverse applied to the light-major intensity stack.
//
// The contraction is HBM-bound (arithmetic intensity 1.5 flop/B for PTM-6,
// 4 flop/B for HSH-16, ridge ≈20 flop/B), so both kernels are built around
// the intensity stream: every byte of I is read exactly once, with 16-byte
// coalesced loads, and the k×N operator never touches HBM after the first
// wave reads it.
//
//  * fit_shared_valu<K>: one lane owns VEC adjacent pixels (16 B of one light
//    plane per load), the k×N pseudo-inverse is wave-uniform and is read with
//    scalar loads into SGPRs, the contraction is K·VEC fp32 FMAs per load.
//  * fit_shared_mfma: the pseudo-inverse is staged once per workgroup in LDS
//    as [N][16] and fed as the A operand of v_mfma_f32_16x16x4_f32; the
//    intensity stream is the B operand.  A lane's 16-B load (4 pixels of one
//    light) supplies B for four 16-pixel MFMA tiles (pixel j of tile c is
//    p0 + 4j + c), so the four accumulators are independent and the load is
//    still 256 contiguous bytes per 16 lanes.
#include <hip/hip_runtime.h>

#include <mutex>
#include <utility>
#include <vector>

#include <atomic>
#include <cstdint>
#include <type_traits>

#include "rti_basis.h"
#include "rti_internal.h"

namespace rti {

// compute units of the current device (cached; 256 on MI355X)
int device_cus() {
  static std::atomic<int> cache[64];  // 0 = not queried yet (concurrent first queries store the same value)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

hipError_t reserve_lds(const void* kern, size_t bytes) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, size_t>> done;  // (kernel, device) -> bytes reserved
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  const std::pair<const void*, int> key(kern, dev);
  {
    std::lock_guard<std::mutex> g(mu);
    for (const auto& e : done)
      if (e.first == key && e.second >= bytes) return hipSuccess;
  }
  const hipError_t st = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (st == hipSuccess) {
    std::lock_guard<std::mutex> g(mu);
    bool found = false;
    for (auto& e : done)
      if (e.first == key) e.second = std::max(e.second, bytes), found = true;
    if (!found) done.emplace_back(key, bytes);
  }
  return st;
}

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---- VEC adjacent pixels of one light plane -> fp32 registers ------------------------
template <typename T, int VEC, bool NT>
__device__ __forceinline__ void load_px(const T* __restrict__ p, float (&x)[VEC]) {
  if constexpr (VEC == 1) {
    x[0] = (float)(NT ? __builtin_nontemporal_load(p) : *p);
  } else {
    typedef T vec_t __attribute__((ext_vector_type(VEC)));
    const vec_t* vp = reinterpret_cast<const vec_t*>(p);
    vec_t v = NT ? __builtin_nontemporal_load(vp) : *vp;
#pragma unroll
    for (int i = 0; i < VEC; ++i) x[i] = (float)v[i];
  }
}

template <int N>
__device__ __forceinline__ void store_f32(float* __restrict__ dst, const float (&v)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      floatx4 t = {v[i], v[i + 1], v[i + 2], v[i + 3]};
      *reinterpret_cast<floatx4*>(dst + i) = t;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) dst[i] = v[i];
  }
}

// ---- VALU stream kernel ---------------------------------------------------------------
// MODE bits (tuning variants, picked by measurement):
//   VM_NT    : non-temporal loads of the intensity stream (read once)
//   VM_LDS   : pinv staged in LDS as [N][KP] (KP = K rounded up to 4), read back with
//              broadcast LDS loads instead of per-light scalar loads
//   VM_NTS   : non-temporal coefficient stores
//   VM_STAGE : pixel-major output transposed through LDS so every store instruction
//              writes 1 KiB contiguous (a lane's own VEC*K floats sit at a 4*VEC*K-byte
//              lane stride otherwise)
//   VM_ROT   : each wave sweeps the lights from its own start plane (measurement variant)
constexpr int VM_NT = 1, VM_LDS = 2, VM_NTS = 4, VM_STAGE = 8, VM_ROT = 16;

template <int N, bool NT>
__device__ __forceinline__ void store_f32_nt(float* __restrict__ dst, const float (&v)[N]) {
  if constexpr (!NT) {
    store_f32<N>(dst, v);
  } else if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      floatx4 t = {v[i], v[i + 1], v[i + 2], v[i + 3]};
      __builtin_nontemporal_store(t, reinterpret_cast<floatx4*>(dst + i));
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) __builtin_nontemporal_store(v[i], dst + i);
  }
}

// pixel-major stores staged through a per-wave LDS slab of 64 lanes x 4 pixels x K floats: 4-pixel
// lanes in one step, 16-pixel (u8) lanes in four steps of 16 lanes each
template <int K, int VEC>
constexpr bool stage_ok() { return (VEC == 4 || VEC == 16) && K <= 9; }

// Lane → pixel map.  A wave owns NC·64·VEC consecutive pixels; lane l's chunk c is the VEC
// pixels at wave_base + c·64·VEC + l·VEC, so each load instruction of the wave reads 64·VEC
// contiguous elements of one light plane and the wave's NC loads of a plane cover
// NC·64·VEC·sizeof(T) contiguous bytes (8 KiB for PTM-6 fp32 at NC = 8).  Long per-wave runs
// inside each plane are what moves this kernel toward the HBM peak: on MI355X the c3 read
// stream goes 0.50 → 0.46 ms and the whole fit 0.64 → 0.56 ms from NC = 1 to NC = 8, although
// NC = 8 needs 256 VGPRs (one wave per SIMD); occupancy does not matter, run length does
// (profiles/r01_c3_chunk_sweep.log).
//
// dynamic LDS: [pinv weights N*KP floats, 16-B aligned][staging 4 waves * 64 lanes * VEC*K floats]
template <int K, int VEC, int NC, typename T, int LAYOUT, int MODE, bool TAIL>
__device__ __forceinline__ void fit_valu_body(const float* __restrict__ pinv, int N, const T* __restrict__ I,
                                              int64_t P, int64_t pe, int64_t lstride, float* __restrict__ dst, int64_t pbase,
                                              int64_t wave_base, const float* lds_w, float* lds_dyn) {
  constexpr bool NT = (MODE & VM_NT) != 0;
  constexpr bool LDSW = (MODE & VM_LDS) != 0;
  constexpr bool NTS = (MODE & VM_NTS) != 0;
  constexpr bool STAGE =
      (MODE & VM_STAGE) != 0 && LAYOUT == RTI_COEF_PIXEL_MAJOR && stage_ok<K, VEC>();
  constexpr int KP = (K + 3) & ~3;
  constexpr int CH = 64 * VEC;  // elements between a lane's chunks
  const T* __restrict__ src = I + pbase;
  // chunk offsets; in the (single) partial wave a chunk past P re-reads chunk 0 and is not stored
  bool ok[NC];
  int coff[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    ok[c] = !TAIL || pbase + (int64_t)c * CH < pe;
    coff[c] = ok[c] ? c * CH : 0;
  }

  float acc[K][NC * VEC];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int v = 0; v < NC * VEC; ++v) acc[k][v] = 0.f;

  auto weight = [&](int k, int n) -> float {
    if constexpr (LDSW)
      return lds_w[n * KP + k];  // same address in every lane: broadcast
    else
      return pinv[k * N + n];  // wave-uniform -> s_load
  };

  constexpr int U = (VEC >= 16) ? 4 : 8;            // loads in flight per lane
  constexpr int UP = U / NC > 0 ? U / NC : 1;        // light planes per step
  // lights [nb, ne) of the sweep; VM_ROT (measurement variant) starts each wave at its own light
  // r0 and wraps, so the waves in flight read different planes at any moment
  auto sweep = [&](int nb, int ne) {
    int n = nb;
    for (; n + UP <= ne; n += UP) {
      float x[UP][NC][VEC];
#pragma unroll
      for (int u = 0; u < UP; ++u)
#pragma unroll
        for (int c = 0; c < NC; ++c) load_px<T, VEC, NT>(src + (int64_t)(n + u) * lstride + coff[c], x[u][c]);
#pragma unroll
      for (int u = 0; u < UP; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float w = weight(k, n + u);
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[k][c * VEC + v] = fmaf(w, x[u][c][v], acc[k][c * VEC + v]);
        }
    }
    for (; n < ne; ++n) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        float x[VEC];
        load_px<T, VEC, NT>(src + (int64_t)n * lstride + coff[c], x);
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float w = weight(k, n);
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[k][c * VEC + v] = fmaf(w, x[v], acc[k][c * VEC + v]);
        }
      }
    }
  };
  if constexpr ((MODE & VM_ROT) != 0) {
    const int r0 = (int)(((wave_base / (64 * VEC * NC)) * 13) % N);
    sweep(r0, N);
    sweep(0, r0);
  } else {
    sweep(0, N);
  }

#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (!ok[c]) continue;
    const int64_t p0 = pbase + (int64_t)c * CH;
    if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float o[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) o[v] = acc[k][c * VEC + v];
        store_f32_nt<VEC, NTS>(dst + (int64_t)k * P + p0, o);
      }
    } else {
      float o[VEC * K];
#pragma unroll
      for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int k = 0; k < K; ++k) o[v * K + k] = acc[k][c * VEC + v];
      if constexpr (STAGE) {
        constexpr int F4 = 4 * K;      // floats of a 4-pixel group (24 for PTM-6)
        constexpr int SUB = VEC / 4;   // steps: 1, or 4 for 16-pixel u8 lanes (16 lanes = 256 pixels each)
        constexpr int LPS = 64 / SUB;  // lanes per step
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int64_t cbase = wave_base + (int64_t)c * CH;  // the wave's first pixel of chunk c
        if (cbase + CH <= pe) {  // wave-uniform: the whole chunk's CH*K floats are in range
          const int woff = LDSW ? ((N * KP + 3) & ~3) : 0;
          float* st = lds_dyn + woff + wave * 64 * F4;
#pragma unroll
          for (int q = 0; q < SUB; ++q) {
            if (SUB == 1 || lane / LPS == q) {  // this step's lanes park their VEC pixels' rows
              float* ls = st + (lane % LPS) * (VEC * K);
#pragma unroll
              for (int i = 0; i < VEC * K; i += 4)
                *reinterpret_cast<floatx4*>(ls + i) = floatx4{o[i], o[i + 1], o[i + 2], o[i + 3]};
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float* wdst = dst + (cbase + (int64_t)q * 256) * K;  // 256 pixels' rows, 1 KiB per instruction
#pragma unroll
            for (int j = 0; j < F4 / 4; ++j) {
              const floatx4 t = *reinterpret_cast<const floatx4*>(st + j * 256 + lane * 4);
              if constexpr (NTS)
                __builtin_nontemporal_store(t, reinterpret_cast<floatx4*>(wdst + j * 256 + lane * 4));
              else
                *reinterpret_cast<floatx4*>(wdst + j * 256 + lane * 4) = t;
            }
            if constexpr (SUB > 1) {  // the slab is rewritten by the next step
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
          }
          continue;
        }
      }
      store_f32_nt<VEC * K, NTS>(dst + p0 * K, o);
    }
  }
}

template <int K, int VEC, int NC, typename T, int LAYOUT, int MODE>
__global__ void __launch_bounds__(256)
fit_shared_valu(const float* __restrict__ pinv, int N, const T* __restrict__ I, int64_t P, int64_t pb, int64_t pe,
                int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  constexpr bool LDSW = (MODE & VM_LDS) != 0;
  constexpr int KP = (K + 3) & ~3;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  float* lds_w = lds_dyn;
  if constexpr (LDSW) {
    for (int idx = threadIdx.x; idx < N * KP; idx += 256) {
      const int n = idx / KP, k = idx - n * KP;
      lds_w[idx] = k < K ? pinv[k * N + n] : 0.f;
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t wave_base = pb + ((int64_t)blockIdx.x * 4 + wave) * (64 * VEC * NC);  // pixels [pb, pe) of P
  const int64_t pbase = wave_base + (int64_t)lane * VEC;
  if (pbase >= pe) return;
  const T* __restrict__ Ic = I + (int64_t)blockIdx.y * cstride;
  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
  if (NC == 1 || wave_base + (int64_t)(64 * VEC * NC) <= pe)  // wave-uniform
    fit_valu_body<K, VEC, NC, T, LAYOUT, MODE, false>(pinv, N, Ic, P, pe, lstride, dst, pbase, wave_base, lds_w, lds_dyn);
  else
    fit_valu_body<K, VEC, NC, T, LAYOUT, MODE, true>(pinv, N, Ic, P, pe, lstride, dst, pbase, wave_base, lds_w, lds_dyn);
}

// Launch generations as rounds of ONE launch (RTI_KERNEL_ROUNDS): the grid is one generation's waves
// (`per` waves of NC·64·VEC pixels), and wave gw handles, in round r = (channel, part), the pixels
// [pb + part·span + gw·W, …) of that channel.  Every wave starts every round together with the others
// (equal work per round), as the separate launches of launch_generations do, but a round's coefficient
// stores drain while the next round's loads are already in flight, and no launch boundary (tail, ramp)
// separates the rounds.
template <int K, int VEC, int NC, typename T, int LAYOUT, int MODE>
__global__ void __launch_bounds__(256)
fit_shared_valu_rounds(const float* __restrict__ pinv, int N, const T* __restrict__ I, int64_t P, int64_t span,
                       int parts, int rounds, int64_t lstride, int64_t cstride, float* __restrict__ coef,
                       int64_t ocstride) {
  constexpr bool LDSW = (MODE & VM_LDS) != 0;
  static_assert(!LDSW, "rounds: SGPR weights only");
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  constexpr int64_t WPX = 64 * VEC * NC;  // pixels per wave and round
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  for (int r = 0; r < rounds; ++r) {
    const int c = r / parts, part = r - c * parts;
    const int64_t rb = (int64_t)part * span, re = rb + span < P ? rb + span : P;
    const int64_t wave_base = rb + gw * WPX;
    if (wave_base >= re) continue;  // wave-uniform
    const int64_t pbase = wave_base + (int64_t)lane * VEC;
    const T* __restrict__ Ic = I + (int64_t)c * cstride;
    float* __restrict__ dst = coef + (int64_t)c * ocstride;
    if (wave_base + WPX <= re) {  // wave-uniform
      fit_valu_body<K, VEC, NC, T, LAYOUT, MODE, false>(pinv, N, Ic, P, re, lstride, dst, pbase, wave_base, lds_dyn,
                                                         lds_dyn);
    } else if (pbase < re) {
      fit_valu_body<K, VEC, NC, T, LAYOUT, MODE, true>(pinv, N, Ic, P, re, lstride, dst, pbase, wave_base, lds_dyn,
                                                        lds_dyn);
    }
  }
}

// ---- MFMA kernel (k <= 16) ------------------------------------------------------------
// Block = 4 waves; wave w owns the 64 pixels [p0, p0+64) with
// p0 = (4·blockIdx.x + w)·64.  Lane l: q = l & 15 (MFMA column), r = l >> 4
// (MFMA k-row = light n0 + r).  D[i][j] of accumulator c is coefficient i of
// pixel p0 + 4j + c; lane l holds rows 4r..4r+3 of column q.
template <typename T, int LAYOUT, bool NT>
__global__ void __launch_bounds__(256)
fit_shared_mfma(const float* __restrict__ pinv, int k, int N, const T* __restrict__ I, int64_t P,
                int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  extern __shared__ __attribute__((aligned(16))) float lds_pinv[];  // [Npad][16]
  const int Npad = (N + 3) & ~3;
  for (int idx = threadIdx.x; idx < Npad * 16; idx += 256) {
    const int n = idx >> 4, i = idx & 15;
    lds_pinv[idx] = (i < k && n < N) ? pinv[i * N + n] : 0.f;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t p0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (p0 >= P) return;
  const int q = lane & 15, r = lane >> 4;
  const int64_t px = p0 + 4 * q;
  const bool lane_ok = px < P;                 // P % 4 == 0 is guaranteed by the launcher
  const T* __restrict__ src = I + (int64_t)blockIdx.y * cstride + (lane_ok ? px : P - 4);

  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  const float* a_col = lds_pinv + r * 16 + q;
  constexpr int S = 8;  // k-steps (4 lights each) whose loads are in flight together
  int n0 = 0;
  for (; n0 + 4 * S <= Npad; n0 += 4 * S) {
    float x[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      int n = n0 + 4 * s + r;
      n = n < N ? n : N - 1;  // the padded rows of A are zero
      load_px<T, 4, NT>(src + (int64_t)n * lstride, x[s]);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float a = a_col[(n0 + 4 * s) * 16];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[s][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[s][1], acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[s][2], acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[s][3], acc3, 0, 0, 0);
    }
  }
  for (; n0 < Npad; n0 += 4) {
    int n = n0 + r;
    n = n < N ? n : N - 1;
    float x[4];
    load_px<T, 4, NT>(src + (int64_t)n * lstride, x);
    const float a = a_col[n0 * 16];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[0], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[1], acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[2], acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[3], acc3, 0, 0, 0);
  }
  if (!lane_ok) return;

  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
  if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int i = 4 * r + rr;
      if (i < k) {
        floatx4 t = {acc0[rr], acc1[rr], acc2[rr], acc3[rr]};
        *reinterpret_cast<floatx4*>(dst + (int64_t)i * P + px) = t;
      }
    }
  } else {
    if (k == 16) {
      *reinterpret_cast<floatx4*>(dst + (px + 0) * 16 + 4 * r) = acc0;
      *reinterpret_cast<floatx4*>(dst + (px + 1) * 16 + 4 * r) = acc1;
      *reinterpret_cast<floatx4*>(dst + (px + 2) * 16 + 4 * r) = acc2;
      *reinterpret_cast<floatx4*>(dst + (px + 3) * 16 + 4 * r) = acc3;
    } else {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = 4 * r + rr;
        if (i < k) {
          dst[(px + 0) * k + i] = acc0[rr];
          dst[(px + 1) * k + i] = acc1[rr];
          dst[(px + 2) * k + i] = acc2[rr];
          dst[(px + 3) * k + i] = acc3[rr];
        }
      }
    }
  }
}

// ---- LDS-tiled MFMA stream (BASELINE configs[3]: HSH-16 "MFMA 16×N LDS tile") --------------
// A workgroup owns R = 256·RC consecutive pixels of one channel and sweeps the N lights in
// steps of S = 4·SP planes.  Per step wave w loads planes w·SP .. w·SP+SP-1 of the tile whole
// (RC 16-byte loads per lane and plane, so each wave reads R·4 contiguous bytes of every plane
// it touches: the per-wave run length that moved the PTM stream from 0.64 to 0.55 ms,
// DESIGN.md §4.1) and parks them in a double-buffered LDS tile [2][S][R].  After one barrier
// each wave reads its quarter of the pixels back as B operands of v_mfma_f32_16x16x4_f32; A is
// the pseudo-inverse, staged once per workgroup in LDS as [Npad][16] with rows >= k and padded
// lights zero.  The next step's loads are issued before the current step's MFMAs (split
// staging), so their HBM latency hides under the compute, and every byte of I is read once.
// B element j of accumulator c in group g is pixel pw + 64g + 4j + c (pw = the wave's first
// pixel): one ds_read_b128 feeds four MFMAs.
template <int RC, int LAYOUT>
__device__ __forceinline__ void tile_store(const floatx4 (&acc)[RC][4], float* __restrict__ dst, int64_t P, int k,
                                           int64_t p0, int q, int r);

template <int RC, int SP, typename T, int LAYOUT, bool NT>
__global__ void __launch_bounds__(256)
fit_shared_tile(const float* __restrict__ pinv, int k, int N, const T* __restrict__ I, int64_t P, int64_t lstride,
                int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  constexpr int R = 256 * RC, S = 4 * SP;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int Npad = (N + S - 1) / S * S;         // whole steps
  float* __restrict__ lds_pinv = lds_dyn;       // [Npad][16]
  float* __restrict__ tile = lds_dyn + Npad * 16;  // [2][S][R]
  for (int idx = threadIdx.x; idx < Npad * 16; idx += 256) {
    const int n = idx >> 4, i = idx & 15;
    lds_pinv[idx] = (i < k && n < N) ? pinv[i * N + n] : 0.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * R;
  const T* __restrict__ src = I + (int64_t)blockIdx.y * cstride + t0 + 4 * lane;
  bool pin[RC];  // this lane's chunk c lies inside the image (P % 4 == 0)
#pragma unroll
  for (int c = 0; c < RC; ++c) pin[c] = t0 + 256 * c + 4 * lane < P;

  floatx4 st[SP][RC];
  auto load_step = [&](int n0) {
#pragma unroll
    for (int j = 0; j < SP; ++j) {
      const int n = n0 + wave * SP + j;
#pragma unroll
      for (int c = 0; c < RC; ++c) {
        float x[4] = {0.f, 0.f, 0.f, 0.f};
        if (n < N && pin[c]) load_px<T, 4, NT>(src + (int64_t)n * lstride + 256 * c, x);
        st[j][c] = floatx4{x[0], x[1], x[2], x[3]};
      }
    }
  };
  auto write_step = [&](int b) {
    float* __restrict__ tb = tile + b * (S * R);
#pragma unroll
    for (int j = 0; j < SP; ++j)
#pragma unroll
      for (int c = 0; c < RC; ++c)
        *reinterpret_cast<floatx4*>(tb + (wave * SP + j) * R + 256 * c + 4 * lane) = st[j][c];
  };
  const int q = lane & 15, r = lane >> 4;
  const int pw = wave * 64 * RC;
  floatx4 acc[RC][4];
#pragma unroll
  for (int g = 0; g < RC; ++g)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[g][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int b, int n0) {
    const float* __restrict__ tb = tile + b * (S * R);
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      const float a = lds_pinv[(n0 + 4 * s + r) * 16 + q];
#pragma unroll
      for (int g = 0; g < RC; ++g) {
        const floatx4 x = *reinterpret_cast<const floatx4*>(tb + (4 * s + r) * R + pw + 64 * g + 4 * q);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[g][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[c], acc[g][c], 0, 0, 0);
      }
    }
  };

  load_step(0);
  write_step(0);
  __syncthreads();
  int b = 0;
  for (int n0 = 0; n0 < Npad; n0 += S) {
    const bool more = n0 + S < Npad;  // workgroup-uniform
    if (more) load_step(n0 + S);
    compute(b, n0);
    if (more) write_step(b ^ 1);  // tile b^1 was last read before the previous barrier
    __syncthreads();
    b ^= 1;
  }

  tile_store<RC, LAYOUT>(acc, coef + (int64_t)blockIdx.y * ocstride, P, k, t0 + pw, q, r);
}

// Wide-workgroup form: W waves (512 threads at W = 8), ONE light plane per wave and step (S = W
// planes), the same [2][S][R] double-buffered LDS tile, and the plane loads issued AHEAD steps
// before they are parked in LDS (AHEAD = 2 keeps two steps of loads in flight in registers: the
// register-staged kernel above has one, 64 KiB per CU).  Each wave computes R/W pixels of every
// step (acc = 4·R/(64·W) floatx4: 64 VGPRs at R = 2048, W = 8), so the MFMA accumulators shrink
// as the waves grow and the registers go to loads in flight instead.
// AHEAD = 0: ONE LDS tile (half the LDS, so twice the tile width fits: 16 KiB runs per wave and
// plane at RC = 16), the next step's loads in registers during the compute, two barriers per step.
// STORE: 1 plain coefficient stores, 2 non-temporal, 3 non-temporal through an LDS stage (whole 128-B lines,
// pixel-major k = 16), 0 none (probe)
template <int RC, int W, int AHEAD, typename T, int LAYOUT, bool NT, int STORE = 1>
__global__ void __launch_bounds__(64 * W)
fit_shared_tile_w(const float* __restrict__ pinv, int k, int N, const T* __restrict__ I, int64_t P, int64_t pb,
                  int64_t pe, int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  constexpr int R = 256 * RC, S = W, G = R / (64 * W);  // G = 64-pixel groups per wave
  static_assert(G >= 1 && R % (64 * W) == 0, "tile must split into 64-pixel groups per wave");
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int T_ = (N + S - 1) / S;  // steps
  float* __restrict__ lds_pinv = lds_dyn;             // [T_·S][16]
  float* __restrict__ tile = lds_dyn + T_ * S * 16;  // [2][S][R] ([1][S][R] at AHEAD = 0)
  for (int idx = threadIdx.x; idx < T_ * S * 16; idx += 64 * W) {
    const int n = idx >> 4, i = idx & 15;
    lds_pinv[idx] = (i < k && n < N) ? pinv[i * N + n] : 0.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t0 = pb + (int64_t)blockIdx.x * R;  // pixels [pb, pe) of P
  const T* __restrict__ src = I + (int64_t)blockIdx.y * cstride + t0 + 4 * lane;
  bool pin[RC];
#pragma unroll
  for (int c = 0; c < RC; ++c) pin[c] = t0 + 256 * c + 4 * lane < pe;
  auto load = [&](int t, floatx4 (&st)[RC]) {
    const int n = t * S + wave;
#pragma unroll
    for (int c = 0; c < RC; ++c) {
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      if (n < N && pin[c]) load_px<T, 4, NT>(src + (int64_t)n * lstride + 256 * c, x);
      st[c] = floatx4{x[0], x[1], x[2], x[3]};
    }
  };
  auto park = [&](int b, const floatx4 (&st)[RC]) {
    float* __restrict__ tb = tile + b * (S * R) + wave * R;
#pragma unroll
    for (int c = 0; c < RC; ++c) *reinterpret_cast<floatx4*>(tb + 256 * c + 4 * lane) = st[c];
  };
  const int q = lane & 15, r = lane >> 4;
  const int pw = wave * 64 * G;
  floatx4 acc[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[g][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int b, int t) {
    const float* __restrict__ tb = tile + b * (S * R);
#pragma unroll
    for (int s = 0; s < S / 4; ++s) {
      const float a = lds_pinv[(t * S + 4 * s + r) * 16 + q];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const floatx4 x = *reinterpret_cast<const floatx4*>(tb + (4 * s + r) * R + pw + 64 * g + 4 * q);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[g][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[c], acc[g][c], 0, 0, 0);
      }
    }
  };
  floatx4 sa[RC], sb[RC];
  load(0, sa);
  if constexpr (AHEAD >= 2) {
    if (T_ > 1) load(1, sb);
  }
  park(0, sa);
  __syncthreads();
  if constexpr (AHEAD == 0) {
    for (int t = 0; t < T_; ++t) {
      const bool more = t + 1 < T_;  // workgroup-uniform
      if (more) load(t + 1, sa);
      compute(0, t);
      __syncthreads();
      if (more) {
        park(0, sa);
        __syncthreads();
      }
    }
  } else if constexpr (AHEAD == 1) {
    for (int t = 0; t < T_; ++t) {
      const bool more = t + 1 < T_;  // workgroup-uniform
      if (more) load(t + 1, sa);
      compute(t & 1, t);
      if (more) park((t + 1) & 1, sa);
      __syncthreads();
    }
  } else {
    // sb holds step t + 1 (loaded during step t − 1), sa receives step t + 2; the roles swap every
    // step, so the loop body is written for an even and an odd step
    int t = 0;
    for (; t + 1 < T_; t += 2) {
      if (t + 2 < T_) load(t + 2, sa);
      compute(0, t);
      park(1, sb);
      __syncthreads();
      if (t + 3 < T_) load(t + 3, sb);
      compute(1, t + 1);
      if (t + 2 < T_) park(0, sa);
      __syncthreads();
    }
    if (t < T_) compute(t & 1, t);  // odd step count: the last step, parked by the previous one
  }
  // acc[g][c][rr] = coefficient 4r + rr of pixel t0 + pw + 64g + 4q + c
  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
  if constexpr (STORE == 0) {  // measurement probe (tools/probe/tile_probe.hip): the read stream alone
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int c = 0; c < 4; ++c) t += acc[g][c][0] + acc[g][c][1] + acc[g][c][2] + acc[g][c][3];
    if (t == -1.2345f) dst[0] = t;  // keeps the loads and MFMAs alive
    return;
  }
  auto st16 = [&](float* p, floatx4 v) {
    if constexpr (STORE >= 2)
      __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p));
    else
      *reinterpret_cast<floatx4*>(p) = v;
  };
  if constexpr (STORE == 3 && LAYOUT == RTI_COEF_PIXEL_MAJOR) {
    // k = 16, non-temporal and STAGED: a lane's registers hold 16-B quarters of 64-B pixel rows four pixels
    // apart, so direct stores write every 128-B line in two halves, and non-temporal halves reach HBM
    // separately (WRITE_SIZE 1.32x the coefficient bytes, r04).  Each wave instead parks a 64-pixel group
    // (4 KiB) in its own slice of the now free LDS tile (the last step ended on a barrier) and writes it back
    // as four 1-KiB contiguous non-temporal stores: whole lines.  16-B chunk ch of the group (pixel ch / 4,
    // coefficients 4(ch % 4) ..) sits at chunk ch ^ ((ch >> 4) & 15) of the slice: the 16 lanes of a pass
    // touch 16 distinct bank groups on both the writes and the reads.
    float* __restrict__ slice = tile + wave * 1024;
    auto sw = [](int ch) { return ch ^ ((ch >> 4) & 15); };
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t g0 = t0 + pw + 64 * g;  // first pixel of the group
#pragma unroll
      for (int c = 0; c < 4; ++c)
        *reinterpret_cast<floatx4*>(slice + 4 * sw((4 * q + c) * 4 + r)) = acc[g][c];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = 64 * j + lane;
        const floatx4 v = *reinterpret_cast<const floatx4*>(slice + 4 * sw(ch));
        if (g0 + (ch >> 2) < pe) st16(dst + g0 * 16 + 4 * ch, v);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the slice is rewritten by the next group
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    return;
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t px = t0 + pw + 64 * g + 4 * q;
    if (px >= pe) continue;
    if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = 4 * r + rr;
        if (i < k) st16(dst + (int64_t)i * P + px, floatx4{acc[g][0][rr], acc[g][1][rr], acc[g][2][rr], acc[g][3][rr]});
      }
    } else if (k == 16) {
#pragma unroll
      for (int c = 0; c < 4; ++c) st16(dst + (px + c) * 16 + 4 * r, acc[g][c]);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          if (4 * r + rr < k) dst[(px + c) * k + 4 * r + rr] = acc[g][c][rr];
    }
  }
}

// Tile STREAM form of the AHEAD = 0 kernel (RTI_KERNEL_ROUNDS): one workgroup per CU that streams
// the tiles u = blockIdx.x, blockIdx.x + G, ... of the flattened (channel, tile) space (G = gridDim.x)
// as ONE pipeline of ntiles·T steps, so only its first step waits for HBM cold, every workgroup sweeps
// the planes in step with the others (the chip reads one contiguous G-tile slab of a plane at a time),
// and a finished tile's coefficient stores drain while the next tile's loads are in flight, with no
// launch boundary in between (the separate launches of the launch generations end in a write burst
// and start with a cold ramp).  Every vector-memory operation of the loop is unconditional (lights
// past N and pixels past P re-read valid addresses: the values are zeroed by selects, or never
// stored), so the compiler's counted vmcnt waits stay exact; a finished tile's stores are issued at
// the start of the next tile's first step, before that step's loads.
template <int RC, int W, typename T, int LAYOUT, bool NT>
__global__ void __launch_bounds__(64 * W)
fit_shared_tile_s(const float* __restrict__ pinv, int k, int N, const T* __restrict__ I, int64_t P, int64_t tpc,
                  int64_t ntot, int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  constexpr int R = 256 * RC, S = W, G = R / (64 * W);
  static_assert(G >= 1 && R % (64 * W) == 0, "tile must split into 64-pixel groups per wave");
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int T_ = (N + S - 1) / S;
  float* __restrict__ lds_pinv = lds_dyn;            // [T_·S][16]
  float* __restrict__ tile = lds_dyn + T_ * S * 16;  // [S][R]
  for (int idx = threadIdx.x; idx < T_ * S * 16; idx += 64 * W) {
    const int n = idx >> 4, i = idx & 15;
    lds_pinv[idx] = (i < k && n < N) ? pinv[i * N + n] : 0.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t Gw = gridDim.x;
  const int ntiles = (int)((ntot - blockIdx.x + Gw - 1) / Gw);
  const int steps = ntiles * T_;
  auto tile_of = [&](int j, int& c, int64_t& t0) {
    const int64_t u = blockIdx.x + (int64_t)j * Gw;
    c = (int)(u / tpc);
    t0 = (u - (int64_t)c * tpc) * R;
  };
  auto load = [&](int s, floatx4 (&st)[RC]) {
    const int j = s / T_, t = s - j * T_;
    int c;
    int64_t t0;
    tile_of(j, c, t0);
    const int n = t * S + wave;
    const bool nok = n < N;
    const T* __restrict__ src = I + (int64_t)c * cstride + (int64_t)(nok ? n : N - 1) * lstride;
#pragma unroll
    for (int cc = 0; cc < RC; ++cc) {
      int64_t px = t0 + 256 * cc + 4 * lane;
      px = px < P ? px : P - 4;  // never stored
      float x[4];
      load_px<T, 4, NT>(src + px, x);
      st[cc] = nok ? floatx4{x[0], x[1], x[2], x[3]} : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto park = [&](const floatx4 (&st)[RC]) {
    float* __restrict__ tb = tile + wave * R;
#pragma unroll
    for (int cc = 0; cc < RC; ++cc) *reinterpret_cast<floatx4*>(tb + 256 * cc + 4 * lane) = st[cc];
  };
  const int q = lane & 15, r = lane >> 4;
  const int pw = wave * 64 * G;
  floatx4 acc[G][4];
  auto zero = [&]() {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[g][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  };
  auto compute = [&](int t) {
#pragma unroll
    for (int s = 0; s < S / 4; ++s) {
      const float a = lds_pinv[(t * S + 4 * s + r) * 16 + q];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const floatx4 x = *reinterpret_cast<const floatx4*>(tile + (4 * s + r) * R + pw + 64 * g + 4 * q);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[g][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[c], acc[g][c], 0, 0, 0);
      }
    }
  };
  // acc[g][c][rr] = coefficient 4r + rr of pixel t0 + pw + 64g + 4q + c
  auto finish = [&](int j) {
    int c;
    int64_t t0;
    tile_of(j, c, t0);
    float* __restrict__ dst = coef + (int64_t)c * ocstride;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t px = t0 + pw + 64 * g + 4 * q;
      if (px >= P) continue;
      if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int i = 4 * r + rr;
          if (i < k)
            *reinterpret_cast<floatx4*>(dst + (int64_t)i * P + px) =
                floatx4{acc[g][0][rr], acc[g][1][rr], acc[g][2][rr], acc[g][3][rr]};
        }
      } else if (k == 16) {
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) *reinterpret_cast<floatx4*>(dst + (px + c4) * 16 + 4 * r) = acc[g][c4];
      } else {
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            if (4 * r + rr < k) dst[(px + c4) * k + 4 * r + rr] = acc[g][c4][rr];
      }
    }
    zero();
  };
  if (ntiles <= 0) return;  // workgroup-uniform
  zero();
  floatx4 sa[RC];
  load(0, sa);
  park(sa);
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    const int j = s / T_, t = s - j * T_;
    if (t == 0 && j > 0) finish(j - 1);  // the previous tile's stores, before this step's loads
    load(s + 1 < steps ? s + 1 : s, sa);
    compute(t);
    __syncthreads();
    park(sa);
    __syncthreads();
  }
  finish(ntiles - 1);
}

// DMA form (fp32 stacks): the tile planes go HBM -> LDS by global_load_lds_dwordx4 (no VGPR
// hop, 1 KiB per wave instruction) into a ring of NB tiles, NB - 1 steps in flight.  A step
// waits for its own wave's DMAs with a counted vmcnt and one raw s_barrier publishes it to the
// workgroup (a __syncthreads() would drain every DMA in flight).  Lights past N re-read plane
// N - 1 (their weights are zero) and lanes past the image re-read its last 4 pixels (never
// stored), so every DMA is unconditional.
// one global_load_lds_dwordx4: lane i's 16 bytes land at lds + 16·i (lds wave-uniform)
template <bool NT>
__device__ __forceinline__ void glds16(const float* g, float* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, NT ? 2 : 0);
}

template <int L, int NB>
__device__ __forceinline__ void wait_dma(int after) {  // `after` steps of L DMAs issued since
  if constexpr (NB >= 4) {
    if (after >= 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
      return;
    }
  }
  if (after >= 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int RC, int SP, int NB, int LAYOUT, bool NT>
__global__ void __launch_bounds__(256)
fit_shared_tile_dma(const float* __restrict__ pinv, int k, int N, const float* __restrict__ I, int64_t P,
                    int64_t lstride, int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  constexpr int R = 256 * RC, S = 4 * SP, L = SP * RC;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int T = (N + S - 1) / S;  // steps
  float* __restrict__ lds_pinv = lds_dyn;            // [T·S][16]
  float* __restrict__ ring = lds_dyn + T * S * 16;  // [NB][S][R]
  for (int idx = threadIdx.x; idx < T * S * 16; idx += 256) {
    const int n = idx >> 4, i = idx & 15;
    lds_pinv[idx] = (i < k && n < N) ? pinv[i * N + n] : 0.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * R;
  const float* __restrict__ src = I + (int64_t)blockIdx.y * cstride;
  int64_t off[RC];
#pragma unroll
  for (int c = 0; c < RC; ++c) {
    const int64_t px = t0 + 256 * c + 4 * lane;
    off[c] = px < P ? px : P - 4;
  }
  auto issue = [&](int t, int b) {
    float* rb = ring + b * (S * R);
#pragma unroll
    for (int j = 0; j < SP; ++j) {
      int n = t * S + wave * SP + j;
      n = n < N ? n : N - 1;
#pragma unroll
      for (int c = 0; c < RC; ++c)
        glds16<NT>(src + (int64_t)n * lstride + off[c], rb + (wave * SP + j) * R + 256 * c);
    }
  };
  const int q = lane & 15, r = lane >> 4;
  const int pw = wave * 64 * RC;
  floatx4 acc[RC][4];
#pragma unroll
  for (int g = 0; g < RC; ++g)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[g][c] = floatx4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // pinv staged; no DMA in flight yet
#pragma unroll
  for (int t = 0; t < NB - 1; ++t)
    if (t < T) issue(t, t);
  int b = 0;  // ring slot of step t
  for (int t = 0; t < T; ++t) {
    wait_dma<L, NB>(min(NB - 2, T - 1 - t));
    __builtin_amdgcn_s_barrier();
    const float* __restrict__ tb = ring + b * (S * R);
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      const float a = lds_pinv[(t * S + 4 * s + r) * 16 + q];
#pragma unroll
      for (int g = 0; g < RC; ++g) {
        const floatx4 x = *reinterpret_cast<const floatx4*>(tb + (4 * s + r) * R + pw + 64 * g + 4 * q);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[g][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[c], acc[g][c], 0, 0, 0);
      }
    }
    // slot of step t - 1: every wave has passed this step's barrier, so it is done reading it
    const int bn = b == 0 ? NB - 1 : b - 1;
    if (t + NB - 1 < T) issue(t + NB - 1, bn);
    b = b == NB - 1 ? 0 : b + 1;
  }
  tile_store<RC, LAYOUT>(acc, coef + (int64_t)blockIdx.y * ocstride, P, k, t0 + pw, q, r);
}

// acc[g][c][rr] = coefficient 4r + rr of pixel p0 + 64g + 4q + c (p0 = the wave's first pixel)
template <int RC, int LAYOUT>
__device__ __forceinline__ void tile_store(const floatx4 (&acc)[RC][4], float* __restrict__ dst, int64_t P, int k,
                                           int64_t p0, int q, int r) {
#pragma unroll
  for (int g = 0; g < RC; ++g) {
    const int64_t px = p0 + 64 * g + 4 * q;
    if (px >= P) continue;
    if constexpr (LAYOUT == RTI_COEF_PLANAR) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = 4 * r + rr;
        if (i < k)
          *reinterpret_cast<floatx4*>(dst + (int64_t)i * P + px) =
              floatx4{acc[g][0][rr], acc[g][1][rr], acc[g][2][rr], acc[g][3][rr]};
      }
    } else if (k == 16) {
#pragma unroll
      for (int c = 0; c < 4; ++c) *reinterpret_cast<floatx4*>(dst + (px + c) * 16 + 4 * r) = acc[g][c];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          if (4 * r + rr < k) dst[(px + c) * k + 4 * r + rr] = acc[g][c][rr];
    }
  }
}

struct FitArgs {
  const float* pinv;
  int k, N;
  const void* I;
  int64_t P;
  int C;
  int64_t lstride, cstride;
  float* coef;
  int layout;
  int64_t ocstride;
  bool nt;
  int mode;  // VALU variant bits (VM_*)
  int nc;    // VALU chunks per lane (1 = one VEC-pixel group per lane)
  hipStream_t stream;
  int64_t pb = 0, pe = 0;  // this launch's pixel range [pb, pe) (pe 0 = P): VALU and 8-wave tile kernels
  // VALU generations as rounds of one launch (fit_shared_valu_rounds): parts per channel (0 = off), the
  // pixels per part and the waves of one round
  int rparts = 0;
  int64_t rspan = 0, rwaves = 0;
};

template <int K, int VEC, int NC, typename T, int LAYOUT, int MODE>
void launch_valu_t(const FitArgs& a) {
  const int64_t pe = a.pe ? a.pe : a.P;
  const int64_t groups = (pe - a.pb + VEC * NC - 1) / (VEC * NC);
  dim3 grid(grid_1d(groups, 256), a.C);
  constexpr int KP = (K + 3) & ~3;
  size_t lds = (MODE & VM_LDS) ? (((size_t)a.N * KP + 3) & ~(size_t)3) * sizeof(float) : 0;
  if constexpr ((MODE & VM_STAGE) && LAYOUT == RTI_COEF_PIXEL_MAJOR && stage_ok<K, VEC>())
    lds += (size_t)4 * 64 * 4 * K * sizeof(float);  // 4 waves x 64 lanes x 4 pixels x K
  // the forms AUTO's generations use (valu_generations: non-temporal loads, 4-pixel lanes, nc > 1)
  if constexpr ((MODE & VM_NT) && !(MODE & (VM_LDS | VM_ROT | VM_NTS)) && NC > 1 && VEC == 4 && K == 6 &&
                !std::is_same<T, uint8_t>::value) {
    if (a.rparts > 0) {
      const dim3 rgrid((unsigned)((a.rwaves + 3) / 4));
      hipLaunchKernelGGL((fit_shared_valu_rounds<K, VEC, NC, T, LAYOUT, MODE>), rgrid, dim3(256), lds, a.stream,
                         a.pinv, a.N, static_cast<const T*>(a.I), a.P, a.rspan, a.rparts, a.rparts * a.C, a.lstride,
                         a.cstride, a.coef, a.ocstride);
      return;
    }
  }
  hipLaunchKernelGGL((fit_shared_valu<K, VEC, NC, T, LAYOUT, MODE>), grid, dim3(256), lds, a.stream, a.pinv, a.N,
                     static_cast<const T*>(a.I), a.P, a.pb, pe, a.lstride, a.cstride, a.coef, a.ocstride);
}

// chunks per lane instantiated per k (accumulators K*NC*VEC must fit the 256 VGPRs of a wave)
template <int K>
constexpr int nc_max() { return K <= 6 ? 8 : (K <= 9 ? 4 : 3); }

template <int K, int VEC, int NC, typename T, int LAYOUT>
void launch_valu_ncm(const FitArgs& a) {
  const int m = a.mode & (VM_NT | VM_NTS | VM_STAGE);
  if constexpr (K == 6 && VEC == 4 && NC >= 4 && std::is_same<T, float>::value && LAYOUT == RTI_COEF_PIXEL_MAJOR) {
    if (a.mode & VM_ROT) return launch_valu_t<K, VEC, NC, T, LAYOUT, VM_NT | VM_STAGE | VM_ROT>(a);
  }
  if (m == (VM_NT | VM_NTS)) launch_valu_t<K, VEC, NC, T, LAYOUT, VM_NT | VM_NTS>(a);
  else if (m == (VM_NT | VM_STAGE)) launch_valu_t<K, VEC, NC, T, LAYOUT, VM_NT | VM_STAGE>(a);
  else if (m & VM_NT) launch_valu_t<K, VEC, NC, T, LAYOUT, VM_NT>(a);
  else if (m == VM_NTS) launch_valu_t<K, VEC, NC, T, LAYOUT, VM_NTS>(a);
  else launch_valu_t<K, VEC, NC, T, LAYOUT, 0>(a);
}

template <int K, int VEC, typename T, int LAYOUT>
void launch_valu_nc(const FitArgs& a) {
  // u8 lanes already hold 16 pixels (VEC = 16): at most 2 chunks
  constexpr int MAXC = VEC >= 16 ? (K <= 6 ? 2 : 1) : nc_max<K>();
  const int nc = a.nc < MAXC ? a.nc : MAXC;
  if constexpr (MAXC >= 8) if (nc >= 8) return launch_valu_ncm<K, VEC, 8, T, LAYOUT>(a);
  if constexpr (MAXC >= 4) if (nc >= 4) return launch_valu_ncm<K, VEC, 4, T, LAYOUT>(a);
  if constexpr (MAXC >= 3) if (nc == 3) return launch_valu_ncm<K, VEC, 3, T, LAYOUT>(a);
  if constexpr (MAXC >= 2) if (nc >= 2) return launch_valu_ncm<K, VEC, 2, T, LAYOUT>(a);
  launch_valu_ncm<K, VEC, 1, T, LAYOUT>(a);
}

template <int K, int VEC, typename T, int LAYOUT>
void launch_valu_m(const FitArgs& a) {
  // wide lanes (NC > 1 chunks per lane): non-temporal or plain loads, plain or NT stores
  if constexpr (VEC > 1) {
    if (a.nc > 1) {
      launch_valu_nc<K, VEC, T, LAYOUT>(a);
      return;
    }
  }
  // every mode for the fp32 16-byte path; the default mode for the others
  if constexpr (VEC > 1 && std::is_same<T, float>::value) {
    switch (a.mode & 15) {
#define RTI_MODE_CASE(m) \
  case m: launch_valu_t<K, VEC, 1, T, LAYOUT, m>(a); break;
      RTI_MODE_CASE(0) RTI_MODE_CASE(1) RTI_MODE_CASE(2) RTI_MODE_CASE(3) RTI_MODE_CASE(4) RTI_MODE_CASE(5)
      RTI_MODE_CASE(6) RTI_MODE_CASE(7) RTI_MODE_CASE(8) RTI_MODE_CASE(9) RTI_MODE_CASE(10) RTI_MODE_CASE(11)
      RTI_MODE_CASE(12) RTI_MODE_CASE(13) RTI_MODE_CASE(14) RTI_MODE_CASE(15)
#undef RTI_MODE_CASE
    }
  } else {
    // 16-pixel u8 lanes: PTM-6 pixel-major stores staged through LDS (AUTO's VM_STAGE) as for fp32
    if constexpr (VEC == 16 && K == 6 && LAYOUT == RTI_COEF_PIXEL_MAJOR) {
      if ((a.mode & (VM_NT | VM_STAGE)) == (VM_NT | VM_STAGE))
        return launch_valu_t<K, VEC, 1, T, LAYOUT, VM_NT | VM_STAGE>(a);
    }
    if (a.mode & VM_NT)
      launch_valu_t<K, VEC, 1, T, LAYOUT, VM_NT>(a);
    else
      launch_valu_t<K, VEC, 1, T, LAYOUT, 0>(a);
  }
}

template <int K, int VEC, typename T>
void launch_valu_l(const FitArgs& a) {
  if (a.layout == RTI_COEF_PLANAR)
    launch_valu_m<K, VEC, T, RTI_COEF_PLANAR>(a);
  else
    launch_valu_m<K, VEC, T, RTI_COEF_PIXEL_MAJOR>(a);
}

template <int K, typename T>
void launch_valu_v(const FitArgs& a, bool vec_ok) {
  constexpr int VEC = std::is_same<T, uint8_t>::value ? (K <= 6 ? 16 : 4) : 4;
  if (vec_ok)
    launch_valu_l<K, VEC, T>(a);
  else
    launch_valu_l<K, 1, T>(a);
}

template <typename T>
void launch_valu(const FitArgs& a, bool vec_ok) {
  switch (a.k) {
    case 6: launch_valu_v<6, T>(a, vec_ok); break;
    case 9: launch_valu_v<9, T>(a, vec_ok); break;
    default: launch_valu_v<16, T>(a, vec_ok); break;
  }
}

template <typename T>
void launch_mfma(const FitArgs& a) {
  const int Npad = (a.N + 3) & ~3;
  const size_t lds = (size_t)Npad * 16 * sizeof(float);
  dim3 grid(grid_1d(a.P, 256), a.C);
  if (a.layout == RTI_COEF_PLANAR) {
    if (a.nt)
      hipLaunchKernelGGL((fit_shared_mfma<T, RTI_COEF_PLANAR, true>), grid, dim3(256), lds, a.stream, a.pinv, a.k,
                         a.N, static_cast<const T*>(a.I), a.P, a.lstride, a.cstride, a.coef, a.ocstride);
    else
      hipLaunchKernelGGL((fit_shared_mfma<T, RTI_COEF_PLANAR, false>), grid, dim3(256), lds, a.stream, a.pinv, a.k,
                         a.N, static_cast<const T*>(a.I), a.P, a.lstride, a.cstride, a.coef, a.ocstride);
  } else {
    if (a.nt)
      hipLaunchKernelGGL((fit_shared_mfma<T, RTI_COEF_PIXEL_MAJOR, true>), grid, dim3(256), lds, a.stream, a.pinv,
                         a.k, a.N, static_cast<const T*>(a.I), a.P, a.lstride, a.cstride, a.coef, a.ocstride);
    else
      hipLaunchKernelGGL((fit_shared_mfma<T, RTI_COEF_PIXEL_MAJOR, false>), grid, dim3(256), lds, a.stream, a.pinv,
                         a.k, a.N, static_cast<const T*>(a.I), a.P, a.lstride, a.cstride, a.coef, a.ocstride);
  }
}

template <int RC, int SP, typename T, int LAYOUT, bool NT>
int launch_tile_t(const FitArgs& a) {
  constexpr int R = 256 * RC, S = 4 * SP;
  const int Npad = (a.N + S - 1) / S * S;
  const size_t lds = ((size_t)Npad * 16 + (size_t)2 * S * R) * sizeof(float);
  if (lds > 160 * 1024)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: LDS tile of %zu B (N=%d) exceeds 160 KiB", lds, a.N);
  auto kern = fit_shared_tile<RC, SP, T, LAYOUT, NT>;
  if (lds > 65536 && reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared: cannot reserve %zu B of LDS", lds);
  dim3 grid(grid_1d(a.P, R), a.C);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, a.stream, a.pinv, a.k, a.N, static_cast<const T*>(a.I), a.P,
                     a.lstride, a.cstride, a.coef, a.ocstride);
  return RTI_OK;
}

template <int RC, int SP, typename T>
int launch_tile_l(const FitArgs& a) {
  if (a.layout == RTI_COEF_PLANAR)
    return a.nt ? launch_tile_t<RC, SP, T, RTI_COEF_PLANAR, true>(a) : launch_tile_t<RC, SP, T, RTI_COEF_PLANAR, false>(a);
  return a.nt ? launch_tile_t<RC, SP, T, RTI_COEF_PIXEL_MAJOR, true>(a)
              : launch_tile_t<RC, SP, T, RTI_COEF_PIXEL_MAJOR, false>(a);
}

template <int RC, int W, int AHEAD, typename T, int LAYOUT, bool NT, int STORE = 1>
int launch_tile_w_t(const FitArgs& a) {
  constexpr int R = 256 * RC, S = W;
  const int T_ = (a.N + S - 1) / S;
  const size_t lds = ((size_t)T_ * S * 16 + (size_t)(AHEAD == 0 ? 1 : 2) * S * R) * sizeof(float);
  if (lds > 160 * 1024)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: LDS tile of %zu B (N=%d) exceeds 160 KiB", lds, a.N);
  auto kern = fit_shared_tile_w<RC, W, AHEAD, T, LAYOUT, NT, STORE>;
  if (lds > 65536 && reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared: cannot reserve %zu B of LDS", lds);
  const int64_t pe = a.pe ? a.pe : a.P;
  dim3 grid(grid_1d(pe - a.pb, R), a.C);
  hipLaunchKernelGGL(kern, grid, dim3(64 * W), lds, a.stream, a.pinv, a.k, a.N, static_cast<const T*>(a.I), a.P,
                     a.pb, pe, a.lstride, a.cstride, a.coef, a.ocstride);
  return RTI_OK;
}

// wide-workgroup tile (fp32): rc 4 or 8, 8 waves, loads 1 or 2 steps ahead
template <int RC, int AHEAD, int W = 8>
int launch_tile_w_l(const FitArgs& a) {
  if constexpr (RC == 16 && AHEAD == 0) {  // AUTO's kernel: non-temporal coefficient stores
    // pixel-major HSH-16 rows leave through the LDS stage as whole lines (c4 3.21 against 3.40 ms for the
    // per-lane quarter rows, profiles/r05d_c4_nts_staged_sweep.log; WRITE_SIZE back to the coefficient bytes)
    if ((a.mode & VM_NTS) && a.nt) {
      if (a.layout == RTI_COEF_PLANAR) return launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PLANAR, true, 2>(a);
      return a.k == 16 ? launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PIXEL_MAJOR, true, 3>(a)
                       : launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PIXEL_MAJOR, true, 2>(a);
    }
  }
  if (a.layout == RTI_COEF_PLANAR)
    return a.nt ? launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PLANAR, true>(a)
                : launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PLANAR, false>(a);
  return a.nt ? launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PIXEL_MAJOR, true>(a)
              : launch_tile_w_t<RC, W, AHEAD, float, RTI_COEF_PIXEL_MAJOR, false>(a);
}

// depth 1: one LDS tile (AHEAD 0, rc up to 16), 2: double tile, loads 1 step ahead, 3: loads 2 ahead
int launch_tile_w(const FitArgs& a, int rc, int depth) {
  if (depth == 1) return rc >= 12 ? launch_tile_w_l<16, 0>(a) : launch_tile_w_l<8, 0>(a);  // CHUNKS(15) = 16
  if (rc >= 8) return depth >= 3 ? launch_tile_w_l<8, 2>(a) : launch_tile_w_l<8, 1>(a);
  return depth >= 3 ? launch_tile_w_l<4, 2>(a) : launch_tile_w_l<4, 1>(a);
}

// tile stream (fit_shared_tile_s): one workgroup per CU over the flattened (channel, tile) space
template <int RC, int W, int LAYOUT, bool NT>
int launch_tile_s_t(const FitArgs& a) {
  constexpr int R = 256 * RC, S = W;
  const int T_ = (a.N + S - 1) / S;
  const size_t lds = ((size_t)T_ * S * 16 + (size_t)S * R) * sizeof(float);
  if (lds > 160 * 1024)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: LDS tile of %zu B (N=%d) exceeds 160 KiB", lds, a.N);
  auto kern = fit_shared_tile_s<RC, W, float, LAYOUT, NT>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared: cannot reserve %zu B of LDS", lds);
  const int64_t tpc = (a.P + R - 1) / R, ntot = tpc * a.C, cus = device_cus();
  const dim3 grid((unsigned)(ntot < cus ? ntot : cus));
  hipLaunchKernelGGL(kern, grid, dim3(64 * W), lds, a.stream, a.pinv, a.k, a.N, static_cast<const float*>(a.I), a.P,
                     tpc, ntot, a.lstride, a.cstride, a.coef, a.ocstride);
  return check_launch("rti_fit_shared");
}

int launch_tile_s(const FitArgs& a) {
  if (a.layout == RTI_COEF_PLANAR)
    return a.nt ? launch_tile_s_t<16, 8, RTI_COEF_PLANAR, true>(a) : launch_tile_s_t<16, 8, RTI_COEF_PLANAR, false>(a);
  return a.nt ? launch_tile_s_t<16, 8, RTI_COEF_PIXEL_MAJOR, true>(a)
              : launch_tile_s_t<16, 8, RTI_COEF_PIXEL_MAJOR, false>(a);
}

// 4-wave form of the same kernel at one wave per SIMD: a 4096-pixel tile (16 KiB per wave and
// plane), 4 planes per step, the tile double-buffered (2 x 64 KiB) so one barrier per step, and
// the 256 accumulator registers per lane (16 pixel groups x 4 floatx4) in the AGPR half of the
// unified 512-register file, which leaves the VGPRs to loads 1 (depth 2) or 2 (depth 3) steps ahead.
int launch_tile_w4(const FitArgs& a, int depth) {
  return depth >= 3 ? launch_tile_w_l<16, 2, 4>(a) : launch_tile_w_l<16, 1, 4>(a);
}

template <int RC, int SP, int NB, int LAYOUT, bool NT>
int launch_tile_dma_t(const FitArgs& a) {
  constexpr int R = 256 * RC, S = 4 * SP;
  const int Npad = (a.N + S - 1) / S * S;
  const size_t lds = ((size_t)Npad * 16 + (size_t)NB * S * R) * sizeof(float);
  if (lds > 160 * 1024)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: LDS tile ring of %zu B (N=%d) exceeds 160 KiB", lds, a.N);
  auto kern = fit_shared_tile_dma<RC, SP, NB, LAYOUT, NT>;
  if (lds > 65536 && reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared: cannot reserve %zu B of LDS", lds);
  dim3 grid(grid_1d(a.P, R), a.C);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, a.stream, a.pinv, a.k, a.N, static_cast<const float*>(a.I), a.P,
                     a.lstride, a.cstride, a.coef, a.ocstride);
  return RTI_OK;
}

template <int RC, int SP, int NB>
int launch_tile_dma_l(const FitArgs& a) {
  if (a.layout == RTI_COEF_PLANAR)
    return a.nt ? launch_tile_dma_t<RC, SP, NB, RTI_COEF_PLANAR, true>(a)
                : launch_tile_dma_t<RC, SP, NB, RTI_COEF_PLANAR, false>(a);
  return a.nt ? launch_tile_dma_t<RC, SP, NB, RTI_COEF_PIXEL_MAJOR, true>(a)
              : launch_tile_dma_t<RC, SP, NB, RTI_COEF_PIXEL_MAJOR, false>(a);
}

template <int NB>
int launch_tile_dma(const FitArgs& a, int rc, int sp) {
  if (sp >= 2) return rc >= 4 ? launch_tile_dma_l<4, 2, NB>(a) : launch_tile_dma_l<2, 2, NB>(a);
  return rc >= 8 ? launch_tile_dma_l<8, 1, NB>(a) : launch_tile_dma_l<4, 1, NB>(a);
}

// rc: 1 KiB chunks per wave and plane (tile = 256·rc pixels), sp: planes per wave and step,
// depth: tiles in the LDS ring (2 = register-staged double buffer; 3, 4 = DMA ring, fp32 only).
// Every (rc, sp) for fp32 stacks; 8-bit and int32 stacks use the register-staged (4, 1).
template <typename T>
int launch_tile(const FitArgs& a, int rc, int sp, int depth, int waves) {
  if constexpr (std::is_same<T, float>::value) {
    if (waves == 8) return launch_tile_w(a, rc, depth);
    if (waves == 4 && rc >= 12) return launch_tile_w4(a, depth);
    if (depth >= 4) return launch_tile_dma<4>(a, rc, sp);
    if (depth == 3) return launch_tile_dma<3>(a, rc, sp);
  }
  if (!std::is_same<T, float>::value || (rc == 4 && sp <= 1)) return launch_tile_l<4, 1, T>(a);
  if constexpr (std::is_same<T, float>::value) {
    if (sp >= 2) {
      if (rc >= 8) return launch_tile_l<8, 2, T>(a);
      if (rc >= 4) return launch_tile_l<4, 2, T>(a);
      if (rc >= 2) return launch_tile_l<2, 2, T>(a);
      return launch_tile_l<1, 2, T>(a);
    }
    if (rc >= 8) return launch_tile_l<8, 1, T>(a);
    if (rc >= 2) return launch_tile_l<2, 1, T>(a);
    return launch_tile_l<1, 1, T>(a);
  }
  return RTI_OK;
}

size_t dtype_size(int dt) {
  switch (dt) {
    case RTI_F32: return 4;
    case RTI_I32: return 4;
    case RTI_U8: return 1;
    case RTI_F64: return 8;
    default: return 0;
  }
}

// ---- launch generations (r02) ---------------------------------------------------------------
// The stack streams fastest when every wave on the chip sweeps the light planes in step with the
// others, so that at any moment they all read one contiguous slab of the same plane.  The waves of
// ONE launch start together and, with equal work, stay in step; the waves that start as earlier
// ones retire (a second "generation" inside the same launch) do not.  Measured on c3 (4K x 100,
// PTM-6, interleaved, profiles/r02_generations_sweep.log): one launch of 4050 waves 0.562 ms, the
// same pixels as 2 launches of 2025 waves 0.540, as 4 launches of 1013 waves (one per SIMD)
// 0.510 ms; launches of 1350 waves (a partial second wave on a third of the SIMDs) 0.637, and each
// wave starting its sweep at its own plane 0.69 ms.  So a large fit is issued as consecutive
// launches that give every SIMD one or two waves (VALU stream) or four workgroup rounds (8-wave tile), each
// over a pixel range [pb, pe) of every plane (same kernels, same per-pixel arithmetic: the
// coefficients are bit-identical to one launch).
struct Generations {
  bool split = false;  // false: one launch over all channels
  int parts = 1;       // launches per channel when split
  int64_t unit = 1;    // pixels per wave (VALU) or per workgroup tile; part bounds are multiples of it
};

// VALU stream (PTM-6 fp32 / int32, AUTO): chunks per lane nc and launches such that every launch gives
// every SIMD the same number of waves, one or two (all resident at once: one generation), trying
// nc = 4, 8, 2 in that order.  Two boxes agreed on nc = 4 (c3 as 4 launches of 2025 waves: 0.533 and
// 0.534 ms, against 0.562 / 0.597 for one launch at nc = 8); 8 chunks at one wave per SIMD ran
// 0.510 ms on one box and 0.575 on the other (profiles/r02_generations_sweep.log).  Parts that would
// move < 256 MiB stay one launch (a launch boundary costs a few microseconds).  Returns nc (0: no
// balanced split; the >= 1000-wave rule applies).
int valu_generations(const FitArgs& a, size_t es, Generations& g) {
  const int64_t simds = 4 * (int64_t)device_cus();
  auto balanced = [&](int64_t w) {  // every SIMD one wave (>= 85 % of them busy) or two (>= 85 % with two)
    return (w * 100 >= simds * 85 && w <= simds) || (w * 100 >= simds * 170 && w <= 2 * simds);
  };
  for (int nc : {4, 8, 2}) {
    const int64_t ppw = 256 * nc, wpc = (a.P + ppw - 1) / ppw, total = wpc * a.C;
    Generations t;
    t.unit = ppw;
    int64_t per = total;
    if (total > 2 * simds) {
      t.split = true;
      t.parts = (int)((wpc + 2 * simds - 1) / (2 * simds));
      per = (wpc + t.parts - 1) / t.parts;
    }
    if (!balanced(per)) continue;
    if (t.split && (double)per * ppw * a.N * es < 256.0 * (1 << 20)) return 0;
    g = t;
    return nc;
  }
  return 0;
}

// 8-wave tile kernel (one 4096-pixel workgroup per CU): launches of <= 4 rounds of workgroups per
// channel, the parts count chosen so the last round is >= 85 % full (c4 4K RGB x 200: 3.74 ms one
// launch, 3.61 one per channel, 3.57 two per channel = 1013 tiles; 1350-tile launches 3.82 ms).
Generations tile_generations(const FitArgs& a, int64_t tile_px) {
  const int64_t cus = device_cus(), cap = 4 * cus;
  const int64_t tpc = (a.P + tile_px - 1) / tile_px;
  Generations g;
  g.unit = tile_px;
  if (tpc * a.C <= cap) return g;
  g.split = true;
  const int p0 = (int)((tpc + cap - 1) / cap);
  g.parts = p0;
  for (int p = p0; p < p0 + 4; ++p) {
    const int64_t per = (tpc + p - 1) / p, last = per % cus;
    if (last == 0 || last * 100 >= cus * 85) {
      g.parts = p;
      break;
    }
  }
  return g;
}

// run `launch` over the generations: per channel (C = 1 views of I and coef), pixel ranges of
// whole units
template <typename F>
int launch_generations(const FitArgs& a, size_t es, const Generations& g, F&& launch) {
  if (!g.split) return launch(a);
  int launches = 0;
  const int64_t units = (a.P + g.unit - 1) / g.unit, per = (units + g.parts - 1) / g.parts;
  for (int c = 0; c < a.C; ++c) {
    FitArgs b = a;
    b.C = 1;
    b.I = static_cast<const char*>(a.I) + (size_t)c * a.cstride * es;
    b.coef = a.coef + (size_t)c * a.ocstride;
    for (int i = 0; i < g.parts; ++i) {
      b.pb = i * per * g.unit;
      b.pe = (i + 1) * per * g.unit < a.P ? (i + 1) * per * g.unit : a.P;
      if (b.pb >= b.pe) break;
      const int st = launch(b);
      if (st != RTI_OK) return st;
      note_launches(++launches);
    }
  }
  return RTI_OK;
}

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_fit_shared(const float* pinv, int k, int N, const void* I, int in_dtype, int64_t P, int C,
                              int64_t light_stride, int64_t channel_stride, float* coef, int coef_layout,
                              int64_t coef_channel_stride, int kernel, rti_stream_t stream) {
  constexpr int flags = RTI_KERNEL_NONTEMPORAL | RTI_KERNEL_PINV_LDS | RTI_KERNEL_NT_STORE | RTI_KERNEL_STAGE |
                        RTI_KERNEL_ROTATE | RTI_KERNEL_ROUNDS | RTI_KERNEL_ONE_LAUNCH | RTI_FIELD_CHUNKS |
                        RTI_FIELD_TILE_PLANES | RTI_FIELD_TILE_DEPTH | RTI_FIELD_TILE_WAVES;
  if (!kernel_bits_ok(kernel, RTI_KERNEL_TILE, flags))
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: unknown kernel bits 0x%x", kernel);
  if (!pinv || !I || !coef) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: null pointer");
  if (N <= 0 || P <= 0 || C <= 0 || C > 65535) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: bad N/P/C");
  if (k < 1 || k > 16) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: k=%d outside 1..16", k);
  if (N < k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: N=%d < k=%d", N, k);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: input dtype %d", in_dtype);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: coef layout %d", coef_layout);
  note_launches(1);
  FitArgs a;
  a.pinv = pinv;
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
  a.nt = (kernel & RTI_KERNEL_NONTEMPORAL) != 0;
  a.mode = (a.nt ? VM_NT : 0) | ((kernel & RTI_KERNEL_PINV_LDS) ? VM_LDS : 0) |
           ((kernel & RTI_KERNEL_NT_STORE) ? VM_NTS : 0) | ((kernel & RTI_KERNEL_STAGE) ? VM_STAGE : 0);
  if ((a.mode & VM_LDS) && (size_t)N * 16 * sizeof(float) > 24576) a.mode &= ~VM_LDS;  // keep LDS <= 64 KiB
  a.nc = (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF;  // 0 = AUTO below
  a.stream = (hipStream_t)stream;
  if (a.lstride < P) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: light_stride < P");
  if (C > 1 && a.cstride < (int64_t)N * a.lstride) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: channel_stride");
  if (C > 1 && a.ocstride < P * k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared: coef_channel_stride");

  const size_t es = dtype_size(in_dtype);
  auto vec_ok_for = [&](int vec) {
    const bool in_ok = P % vec == 0 && a.lstride % vec == 0 && a.cstride % vec == 0 && aligned_to(I, vec * es);
    const bool out_ok = aligned_to(coef, 16) && (a.ocstride % 4 == 0) &&
                        (coef_layout == RTI_COEF_PLANAR ? P % 4 == 0 : (vec * k) % 4 == 0);
    return in_ok && out_ok;
  };
  const int sel = kernel & 0xff;
  const bool valu_k = (k == 6 || k == 9 || k == 16);
  bool use_mfma;
  if (sel == RTI_KERNEL_MFMA) {
    use_mfma = true;
  } else if (sel == RTI_KERNEL_VALU || sel == RTI_KERNEL_TILE) {
    use_mfma = false;
  } else {
    // AUTO: measured best on MI355X (profiles/): the VALU stream with
    // non-temporal intensity loads and SGPR weights.
    use_mfma = !valu_k;
    a.nt = true;
    // PTM-6 pixel-major coefficients leave through LDS as whole 1 KiB rows per store
    // instruction: with wide lanes the direct 96-B-strided stores raised WRITE_SIZE to 1.46x
    // the coefficient bytes (c3 0.573 -> 0.549 ms, c2 0.082 -> 0.072 ms staged)
    // HSH-16 (tile_w<16,8,0>): non-temporal coefficient stores, the one store placement that beat the mixed
    // read/write probe's (c4 3.39 against 3.57 ms, profiles/r04r_c4_nts_sweep.log)
    a.mode = VM_NT | (k == 6 ? VM_STAGE : 0) | ((kernel & RTI_KERNEL_ROTATE) ? VM_ROT : 0) | (k == 16 ? VM_NTS : 0);
  }
  Generations gens;  // one launch unless AUTO splits it (launch generations, above)
  if (a.nc == 0) {
    // AUTO chunks per lane (PTM-6, 4-byte intensities): the longest per-wave run in each
    // plane whose accumulators fit, as long as the launch keeps >= 1000 waves (≈1 per SIMD).
    // r02 sweeps (profiles/r02_chunks_c2_shards_sweep.log, interleaved): c2 8 chunks (1012
    // waves) 0.0712 vs 4 chunks 0.0734 ms; 540-row shard 8: 0.1294 vs 4: 0.1335 ms; 270-row
    // shard 4 (1012 waves) 0.0675 vs 2 0.0679 vs 8 (506 waves) 0.0950 ms.  HSH-16 measured no
    // gain (c4: 3.88 ms at 1 and 2 chunks, 4.57 at 3) and keeps one chunk, as do the
    // LDS-weight tuning variants.
    // r02: AUTO picks nc and the launch generations together for 4-byte stacks (valu_generations
    // above; c3 fp32 0.593 -> 0.532 ms, int32 0.651 -> 0.532 ms).  8-bit stacks keep one launch of
    // one-chunk 16-pixel lanes: their 2-chunk generations ran 0.366 against 0.244 ms
    // (profiles/r02_generations_sweep.log).
    const bool plain = (a.mode & ~(VM_NT | VM_NTS | VM_STAGE | VM_ROT)) == 0;
    a.nc = 1;
    int gnc = 0;
    if (plain && k == 6 && in_dtype != RTI_U8 && sel == RTI_KERNEL_AUTO && !(kernel & RTI_KERNEL_ONE_LAUNCH) &&
        vec_ok_for(4))
      gnc = valu_generations(a, es, gens);
    if (gnc) {
      a.nc = gnc;
      if ((kernel & RTI_KERNEL_ROUNDS) && gens.split) {  // the generations as rounds of one launch
        const int64_t units = (P + gens.unit - 1) / gens.unit, per = (units + gens.parts - 1) / gens.parts;
        a.rparts = gens.parts;
        a.rspan = per * gens.unit;
        a.rwaves = per;  // one wave per unit (256·nc pixels)
        gens = Generations();
      }
    } else if (plain && in_dtype != RTI_U8 && k == 6) {
      const int64_t groups = P * C / 4;  // 4-pixel lane groups
      for (int nc = 8; nc > 1; nc >>= 1)
        if (groups / (64 * nc) >= 1000) {
          a.nc = nc;
          break;
        }
    }
  }
  const bool mfma_ok = N <= 1024 && P % 4 == 0 && a.lstride % 4 == 0 && a.cstride % 4 == 0 &&
                       aligned_to(I, 4 * es) && aligned_to(coef, 16) && a.ocstride % 4 == 0;
  // AUTO for HSH-16 on fp32 stacks: the LDS-tiled MFMA kernel (c4 4K RGB x 200: 3.54 vs 3.73 ms
  // and 3.94 vs 4.20 ms on two boxes, profiles/r01_c4_tile_sweep.log), when the image gives at
  // least 1024 tiles of 2048 pixels; PTM-6 stays on the VALU stream (c3: 0.54 vs 0.62 ms).
  const bool auto_tile = sel == RTI_KERNEL_AUTO && k == 16 && in_dtype == RTI_F32 && P * C >= (int64_t)1024 * 2048;
  if (sel == RTI_KERNEL_TILE || (auto_tile && mfma_ok)) {
    if (mfma_ok) {
      // explicit tile bits: the 4-wave kernels (2048 pixels x 8 planes per step, register-staged, or
      // the DMA ring) or the 8-wave kernels; 1024-pixel tiles above N = 512
      const int rc = (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF, sp = (kernel >> RTI_KERNEL_TILE_PLANES_SHIFT) & 0xF;
      const int depth = (kernel >> RTI_KERNEL_TILE_DEPTH_SHIFT) & 0xF;
      const int waves = (kernel >> RTI_KERNEL_TILE_WAVES_SHIFT) & 0xF;
      // AUTO (no tile bits set) for fp32 at N <= 512: the 8-wave kernel on ONE 4096-pixel LDS tile
      // (16 KiB per wave and plane; c4 3.74 vs 3.93 ms for the 2048-pixel double-buffered tile,
      // profiles/r02_c4_tile_rc16_sweep.log); above N = 512 its [N][16] pinv no longer fits.
      const bool tile_auto =
      (kernel & ~0xff & ~(RTI_KERNEL_NONTEMPORAL | RTI_KERNEL_ONE_LAUNCH | RTI_KERNEL_ROUNDS | RTI_KERNEL_NT_STORE)) == 0 &&
      N <= 512;
      const int rc0 = rc ? rc : (N <= 512 ? 8 : 4);
      int st;
      switch (in_dtype) {
        case RTI_F32: {
          // launch generations for the 4096-pixel tile_w kernels (AUTO, or explicit 8 waves at depth 1 /
          // 4 waves, rc >= 12: one workgroup per CU; launch_tile_w runs a 2048-pixel tile at depth 2+);
          // the other tile forms stay one launch
          if (tile_auto && (kernel & RTI_KERNEL_ROUNDS)) {  // the tile stream: one launch, no generations
            st = launch_tile_s(a);
            break;
          }
          const bool w4096 = tile_auto || (rc >= 12 && (waves == 4 || (waves == 8 && depth == 1)));
          if (w4096 && !(kernel & RTI_KERNEL_ONE_LAUNCH)) gens = tile_generations(a, 4096);
          st = launch_generations(a, es, gens, [&](const FitArgs& b) {
            return tile_auto ? launch_tile<float>(b, 15, 1, 1, 8)
                             : launch_tile<float>(b, rc0, sp ? sp : 2, depth ? depth : 2, waves);
          });
          break;
        }
        case RTI_I32: st = launch_tile<int32_t>(a, 4, 1, 2, 4); break;
        default: st = launch_tile<uint8_t>(a, 4, 1, 2, 4); break;
      }
      return st != RTI_OK ? st : check_launch("rti_fit_shared");
    }
    if (!valu_k) return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: tile path needs N<=1024 and 4-pixel alignment");
    a.nc = 1;  // ragged shapes: the one-chunk VALU stream
  }
  if (use_mfma && !mfma_ok) {
    if (sel == RTI_KERNEL_MFMA && !valu_k)
      return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: MFMA path needs N<=1024 and 4-pixel alignment");
    use_mfma = false;
  }
  if (!use_mfma && !valu_k) return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared: VALU path supports k in {6,9,16}");

  if (use_mfma) {
    switch (in_dtype) {
      case RTI_F32: launch_mfma<float>(a); break;
      case RTI_I32: launch_mfma<int32_t>(a); break;
      default: launch_mfma<uint8_t>(a); break;
    }
  } else {
    const int vec = in_dtype == RTI_U8 ? (k <= 6 ? 16 : 4) : 4;
    const bool vok = vec_ok_for(vec);
    switch (in_dtype) {
      case RTI_F32:
        launch_generations(a, es, gens, [vok](const FitArgs& b) {
          launch_valu<float>(b, vok);
          return RTI_OK;
        });
        break;
      case RTI_I32:
        launch_generations(a, es, gens, [vok](const FitArgs& b) {
          launch_valu<int32_t>(b, vok);
          return RTI_OK;
        });
        break;
      default: launch_valu<uint8_t>(a, vok); break;
    }
  }
  return check_launch("rti_fit_shared");
}
