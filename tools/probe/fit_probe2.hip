// fit_probe2.hip -- measurement-only variants of the shared PTM-6 fit (not part of librti).
// What they vary, with the fp32 light-major stream and pixel-major [P][6] stores fixed:
//   PXL  pixels per lane: 4 (one 16-B load per plane), 8 or 16 (2 or 4 loads per plane at
//        1 KiB spacing: a wave reads PXL/4 KiB contiguous from each plane)
//   U    16-B loads in flight per lane
//   MODE 0 one tile per workgroup (grid covers P), 1 grid-stride persistent (tile t =
//        blockIdx.x + i*gridDim.x: concurrently running tiles stay adjacent), 2 = 1 with the
//        next tile's first loads issued before the current tile's coefficient stores
//   STORE false: coefficients folded into a never-taken branch (read + FMA only)
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ floatx4 ldnt(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
}

template <int PXL, int U, int MODE, bool STORE, int WG = 256, bool BAR = false>
__global__ void __launch_bounds__(WG) fit6_v(const float* __restrict__ pinv, const float* __restrict__ I, int N,
                                              int64_t P, int64_t ls, float* __restrict__ coef) {
  constexpr int NC = PXL / 4;                  // 16-B chunks per plane per lane
  constexpr int UP = U / NC > 0 ? U / NC : 1;  // planes per step
  constexpr int64_t TILE = WG * PXL;           // pixels per workgroup tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ntiles = (P + TILE - 1) / TILE;
  int64_t t = blockIdx.x;
  const int64_t tstep = MODE == 0 ? ntiles : gridDim.x;
  if (t >= ntiles) return;
  // pixel of chunk j of this lane inside tile t
  auto base = [&](int64_t tt) { return tt * TILE + (int64_t)wave * 64 * PXL + lane * 4; };

  floatx4 pre[UP][NC];
  bool have_pre = false;
  for (; t < ntiles; t += tstep) {
    const float* src = I + base(t);
    bool ok[NC];
    int coff[NC];  // chunk offsets (a chunk past P re-reads the last 4 pixels and is not stored)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      ok[c] = base(t) + c * 256 < P;
      coff[c] = ok[c] ? c * 256 : (int)(P - 4 - base(t));
    }
    float acc[6][PXL];
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int v = 0; v < PXL; ++v) acc[k][v] = 0.f;
    int n = 0;
    for (; n + UP <= N; n += UP) {
      floatx4 x[UP][NC];
      if constexpr (BAR) __syncthreads();  // keep the workgroup's waves on the same planes
      if (MODE == 2 && have_pre && n == 0) {
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) x[u][c] = pre[u][c];
      } else {
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) x[u][c] = ldnt(src + (int64_t)(n + u) * ls + coff[c]);
      }
#pragma unroll
      for (int u = 0; u < UP; ++u)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const float w = pinv[k * N + n + u];
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[k][c * 4 + v] = fmaf(w, x[u][c][v], acc[k][c * 4 + v]);
        }
    }
    for (; n < N; ++n) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const floatx4 x = ldnt(src + (int64_t)n * ls + coff[c]);
#pragma unroll
        for (int k = 0; k < 6; ++k)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[k][c * 4 + v] = fmaf(pinv[k * N + n], x[v], acc[k][c * 4 + v]);
      }
    }
    if constexpr (MODE == 2) {
      have_pre = false;
      if (t + tstep < ntiles && N >= UP) {
        const float* nsrc = I + base(t + tstep);
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) pre[u][c] = ldnt(nsrc + (int64_t)u * ls + c * 256);
        have_pre = true;
      }
    }
    if constexpr (STORE) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (!ok[c]) continue;
        float* d = coef + (base(t) + c * 256) * 6;
        float o[24];
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
          for (int k = 0; k < 6; ++k) o[v * 6 + k] = acc[k][c * 4 + v];
#pragma unroll
        for (int i = 0; i < 24; i += 4) *reinterpret_cast<floatx4*>(d + i) = floatx4{o[i], o[i + 1], o[i + 2], o[i + 3]};
      }
    } else {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int v = 0; v < PXL; ++v) s += acc[k][v];
      if (s == -1.2345f) coef[0] = s;
    }
  }
}


// Phase-separated rounds: a persistent grid of G co-resident workgroups; round r fits tiles
// r*G + blockIdx.x (one contiguous slab of the image per round), holds the coefficients in
// registers, arrives at a device-wide counter and waits (bounded spin: a scheduling hint, never
// needed for correctness -- every lane stores only its own pixels) until every workgroup of the
// round has finished its reads, then stores.  `base` = arrivals counted before this launch.
template <int PXL, int U>
__global__ void __launch_bounds__(256) fit6_gb(const float* __restrict__ pinv, const float* __restrict__ I, int N,
                                               int64_t P, int64_t ls, float* __restrict__ coef,
                                               unsigned long long* __restrict__ ctr, unsigned long long base,
                                               int spin_max) {
  constexpr int NC = PXL / 4;
  constexpr int UP = U / NC > 0 ? U / NC : 1;
  constexpr int64_t TILE = 256 * PXL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ntiles = (P + TILE - 1) / TILE;
  const int64_t G = gridDim.x;
  const int64_t rounds = (ntiles + G - 1) / G;
  for (int64_t r = 0; r < rounds; ++r) {
    const int64_t t = r * G + blockIdx.x;
    const bool have = t < ntiles;
    const int64_t b0 = t * TILE + (int64_t)wave * 64 * PXL + lane * 4;
    float acc[6][PXL];
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int v = 0; v < PXL; ++v) acc[k][v] = 0.f;
    bool ok[NC];
    int coff[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      ok[c] = have && b0 + c * 256 < P;
      coff[c] = ok[c] ? c * 256 : 0;
    }
    if (have) {
      const float* src = I + (b0 + (int64_t)NC * 256 <= P ? b0 : P - 4 - 0 * b0);
      if (b0 + (int64_t)NC * 256 > P) {
#pragma unroll
        for (int c = 0; c < NC; ++c) coff[c] = ok[c] ? (int)(b0 + c * 256 - (P - 4)) : 0;
      }
      int n = 0;
      for (; n + UP <= N; n += UP) {
        floatx4 x[UP][NC];
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) x[u][c] = ldnt(src + (int64_t)(n + u) * ls + coff[c]);
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            const float w = pinv[k * N + n + u];
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
              for (int v = 0; v < 4; ++v) acc[k][c * 4 + v] = fmaf(w, x[u][c][v], acc[k][c * 4 + v]);
          }
      }
      for (; n < N; ++n) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const floatx4 x = ldnt(src + (int64_t)n * ls + coff[c]);
#pragma unroll
          for (int k = 0; k < 6; ++k)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[k][c * 4 + v] = fmaf(pinv[k * N + n], x[v], acc[k][c * 4 + v]);
        }
      }
    }
    // round barrier
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long target = base + (unsigned long long)(r + 1) * G;
      __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int i = 0; i < spin_max; ++i) {
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!ok[c]) continue;
      float* d = coef + (b0 + c * 256) * 6;
      float o[24];
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int k = 0; k < 6; ++k) o[v * 6 + k] = acc[k][c * 4 + v];
#pragma unroll
      for (int i = 0; i < 24; i += 4) *reinterpret_cast<floatx4*>(d + i) = floatx4{o[i], o[i + 1], o[i + 2], o[i + 3]};
    }
  }
}

template <int PXL, int U, int MODE, bool STORE, int WG = 256, bool BAR = false>
void go(const float* pinv, const float* I, int N, int64_t P, int64_t ls, float* coef, int grid, hipStream_t s) {
  const int64_t ntiles = (P + WG * PXL - 1) / (WG * PXL);
  const unsigned g = MODE == 0 ? (unsigned)ntiles : (unsigned)(grid < ntiles ? grid : ntiles);
  hipLaunchKernelGGL((fit6_v<PXL, U, MODE, STORE, WG, BAR>), dim3(g), dim3(WG), 0, s, pinv, I, N, P, ls, coef);
}

}  // namespace

// variant = PXL*10000 + U*100 + MODE*10 + STORE  (e.g. 40801 = PXL 4, U 8, mode 0, stores)
extern "C" int probe2_fit(const float* pinv, const float* I, int N, int64_t P, int64_t ls, float* coef, int variant, int grid,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int pxl = (variant % 1000000) / 10000, u = (variant / 100) % 100, mode = (variant / 10) % 10, st = variant % 10;
  if (P % 4 != 0 || ls % 4 != 0) return 1;
#define V(A, B, C, D) \
  if (pxl == A && u == B && mode == C && st == D) { go<A, B, C, D>(pinv, I, N, P, ls, coef, grid, s); return hipGetLastError() == hipSuccess ? 0 : 3; }
  V(4, 8, 0, 1) V(4, 8, 0, 0)
  V(8, 8, 0, 1) V(8, 8, 0, 0)
  V(16, 4, 0, 1) V(16, 4, 0, 0) V(16, 8, 0, 1) V(16, 8, 0, 0) V(16, 16, 0, 1) V(16, 16, 0, 0) V(16, 8, 1, 1)
  V(32, 8, 0, 1) V(32, 8, 0, 0) V(32, 4, 0, 1) V(32, 4, 1, 1) V(32, 4, 0, 0)
#undef V
  // barrier variants: variant = 1000000*WGsel + PXL*10000 + U*100 + STORE, WGsel 1: 256+bar, 2: 512+bar,
  // 4: 1024+bar, 5: 512 no bar, 6: 1024 no bar
  const int wsel = variant / 1000000;
  if (wsel) {
    const int v2 = variant % 1000000;
#define W(SEL, WGT, B, A, U2) \
  if (wsel == SEL && v2 == A * 10000 + U2 * 100 + 1) { go<A, U2, 0, true, WGT, B>(pinv, I, N, P, ls, coef, grid, s); return hipGetLastError() == hipSuccess ? 0 : 3; }
    W(1, 256, true, 16, 8) W(1, 256, true, 32, 8) W(2, 512, true, 16, 8) W(2, 512, true, 8, 8)
    W(4, 1024, true, 4, 8) W(4, 1024, true, 8, 8) W(5, 512, false, 16, 8) W(6, 1024, false, 4, 8) W(6, 1024, false, 8, 8)
#undef W
  }
  return 2;
}

// grid-barrier rounds (fit6_gb): returns the arrivals this launch adds to *ctr
extern "C" long long probe2_gb(const float* pinv, const float* I, int N, int64_t P, int64_t ls, float* coef, int pxl,
                               int u, int grid, unsigned long long* ctr, unsigned long long base, int spin_max,
                               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t ntiles = (P + 256 * pxl - 1) / (256 * pxl);
  const int64_t rounds = (ntiles + grid - 1) / grid;
#define GB(A, B) \
  if (pxl == A && u == B) { hipLaunchKernelGGL((fit6_gb<A, B>), dim3(grid), dim3(256), 0, s, pinv, I, N, P, ls, coef, ctr, base, spin_max); \
    return hipGetLastError() == hipSuccess ? rounds * grid : -3; }
  GB(32, 4) GB(32, 8) GB(16, 8) GB(16, 4)
#undef GB
  return -2;
}
