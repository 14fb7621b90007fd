// hbm_probe.hip -- measurement-only kernels (not part of librti): the achievable
// HBM read ceiling for a light-major stream, and fit-shaped variants that isolate
// what the PTM fit adds on top of the pure read (stores, weights, loop shape).
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ floatx4 ld4(const float* p) {
  const floatx4* q = reinterpret_cast<const floatx4*>(p);
  return NT ? __builtin_nontemporal_load(q) : *q;
}

// Pure read: each lane reads 16 B per light plane, UNROLL planes in flight.
template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) read_stream(const float* __restrict__ I, int N, int64_t P, float* __restrict__ out) {
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= P) return;
  floatx4 acc = {0, 0, 0, 0};
  int n = 0;
  for (; n + UNROLL <= N; n += UNROLL) {
    floatx4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) x[u] = ld4<NT>(I + (int64_t)(n + u) * P + p0);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += x[u];
  }
  for (; n < N; ++n) acc += ld4<NT>(I + (int64_t)n * P + p0);
  if (acc[0] + acc[1] + acc[2] + acc[3] == -1.2345f) out[0] = acc[0];  // keep the loads alive
}

// Fit-shaped: 6 coefficients, weights from global (scalar loads), optional stores,
// optional software pipelining (next 8 planes issued before this block's FMAs).
template <bool STORE, bool PIPE>
__global__ void __launch_bounds__(256) fit6(const float* __restrict__ pinv, const float* __restrict__ I, int N, int64_t P,
                                            float* __restrict__ coef) {
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= P) return;
  float acc[6][4] = {};
  constexpr int U = 8;
  const float* src = I + p0;
  auto fma_block = [&](const floatx4 (&x)[U], int n) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float w = pinv[k * N + n + u];
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[k][v] = fmaf(w, x[u][v], acc[k][v]);
      }
  };
  int n = 0;
  if constexpr (PIPE) {
    floatx4 x[U], y[U];
    if (N >= U) {
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ld4<true>(src + (int64_t)u * P);
      for (n = U; n + U <= N; n += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = ld4<true>(src + (int64_t)(n + u) * P);
        fma_block(x, n - U);
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = y[u];
      }
      fma_block(x, n - U);
    }
  } else {
    for (; n + U <= N; n += U) {
      floatx4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ld4<true>(src + (int64_t)(n + u) * P);
      fma_block(x, n);
    }
  }
  for (; n < N; ++n) {
    floatx4 x = ld4<true>(src + (int64_t)n * P);
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[k][v] = fmaf(pinv[k * N + n], x[v], acc[k][v]);
  }
  if constexpr (STORE) {
    float o[24];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int k = 0; k < 6; ++k) o[v * 6 + k] = acc[k][v];
    float* d = coef + p0 * 6;
#pragma unroll
    for (int i = 0; i < 24; i += 4) *reinterpret_cast<floatx4*>(d + i) = floatx4{o[i], o[i + 1], o[i + 2], o[i + 3]};
  } else {
    float s = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    if (s == -1.2345f) coef[0] = s;
  }
}

// Store-path diagnosis: fit6 body (NT loads, no pipelining) with different coefficient stores.
//   0 plain float4 pixel-major   1 sc1 (write-through, drop from L2) buffer stores   2 sc0|sc1
//   3 nt buffer stores           4 all waves store into one 64 KiB window (L2-resident)
//   5 planar float4 (1 KiB contiguous per wave instruction)   6 dword stores pixel-major
template <int SM, bool XCD = false>
__global__ void __launch_bounds__(256) fit6_store(const float* __restrict__ pinv, const float* __restrict__ I, int N,
                                                  int64_t P, float* __restrict__ coef, int64_t wmask = 16383) {
  int64_t bid = blockIdx.x;
  if constexpr (XCD) {  // blocks b, b+8, ... share an XCD: give each XCD one contiguous eighth of the image
    const int64_t nb = gridDim.x, per = nb / 8;
    if (bid < per * 8) bid = (bid % 8) * per + bid / 8;
  }
  const int64_t p0 = (bid * 256 + threadIdx.x) * 4;
  if (p0 >= P) return;
  float acc[6][4] = {};
  const float* src = I + p0;
  int n = 0;
  for (; n + 8 <= N; n += 8) {
    floatx4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = ld4<true>(src + (int64_t)(n + u) * P);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float w = pinv[k * N + n + u];
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[k][v] = fmaf(w, x[u][v], acc[k][v]);
      }
  }
  for (; n < N; ++n) {
    floatx4 x = ld4<true>(src + (int64_t)n * P);
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[k][v] = fmaf(pinv[k * N + n], x[v], acc[k][v]);
  }
  float o[24];
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int k = 0; k < 6; ++k) o[v * 6 + k] = acc[k][v];
  if constexpr (SM == 5) {
#pragma unroll
    for (int k = 0; k < 6; ++k)
      *reinterpret_cast<floatx4*>(coef + (int64_t)k * P + p0) = floatx4{acc[k][0], acc[k][1], acc[k][2], acc[k][3]};
  } else if constexpr (SM == 6) {
#pragma unroll
    for (int i = 0; i < 24; ++i) coef[p0 * 6 + i] = o[i];
  } else if constexpr (SM == 0 || SM == 4) {
    float* d = SM == 0 ? coef + p0 * 6 : coef + ((p0 * 6) & wmask);
#pragma unroll
    for (int i = 0; i < 24; i += 4) *reinterpret_cast<floatx4*>(d + i) = floatx4{o[i], o[i + 1], o[i + 2], o[i + 3]};
  } else {
    constexpr int aux = SM == 1 ? 16 : (SM == 2 ? 17 : 2);
    const int64_t base_f = (int64_t)blockIdx.x * 256 * 24;  // block base (floats), 32-bit voffset inside
    auto rsrc = __builtin_amdgcn_make_buffer_rsrc(coef + base_f, (short)0, 256 * 24 * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < 24; i += 4) {
      typedef int intx4 __attribute__((ext_vector_type(4)));
      floatx4 f = {o[i], o[i + 1], o[i + 2], o[i + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(intx4, f), rsrc, (int)(threadIdx.x * 96 + i * 4), 0, aux);
    }
  }
}

extern "C" int probe_store(const float* pinv, const float* I, int N, int64_t P, float* coef, int variant, void* stream) {
  dim3 grid((unsigned)((P / 4 + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL((fit6_store<0>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 1: hipLaunchKernelGGL((fit6_store<1>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 2: hipLaunchKernelGGL((fit6_store<2>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 3: hipLaunchKernelGGL((fit6_store<3>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 4: hipLaunchKernelGGL((fit6_store<4>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 5: hipLaunchKernelGGL((fit6_store<5>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 6: hipLaunchKernelGGL((fit6_store<6>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 7: hipLaunchKernelGGL((fit6_store<0, true>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 8: hipLaunchKernelGGL((fit6_store<5, true>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    default: {  // variant >= 100: stores wrap inside a window of (variant - 100) MiB
      const int64_t floats = (int64_t)(variant - 100) * 262144;
      hipLaunchKernelGGL((fit6_store<4>), grid, dim3(256), 0, s, pinv, I, N, P, coef, floats - 1);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

extern "C" int probe_read(const float* I, int N, int64_t P, float* out, int variant, void* stream) {
  dim3 grid((unsigned)((P / 4 + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL((read_stream<8, false>), grid, dim3(256), 0, s, I, N, P, out); break;
    case 1: hipLaunchKernelGGL((read_stream<8, true>), grid, dim3(256), 0, s, I, N, P, out); break;
    case 2: hipLaunchKernelGGL((read_stream<16, false>), grid, dim3(256), 0, s, I, N, P, out); break;
    case 3: hipLaunchKernelGGL((read_stream<16, true>), grid, dim3(256), 0, s, I, N, P, out); break;
    default: hipLaunchKernelGGL((read_stream<4, true>), grid, dim3(256), 0, s, I, N, P, out); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// variant: 0 = stores + no pipelining, 1 = no stores, 2 = stores + pipelined, 3 = no stores + pipelined
extern "C" int probe_fit6(const float* pinv, const float* I, int N, int64_t P, float* coef, int variant, void* stream) {
  dim3 grid((unsigned)((P / 4 + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL((fit6<true, false>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 1: hipLaunchKernelGGL((fit6<false, false>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    case 2: hipLaunchKernelGGL((fit6<true, true>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
    default: hipLaunchKernelGGL((fit6<false, true>), grid, dim3(256), 0, s, pinv, I, N, P, coef); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// Pure write of `bytes` (16 B per lane, contiguous), for the phase-separated lower bound.
__global__ void __launch_bounds__(256) write_stream(float* __restrict__ out, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) reinterpret_cast<floatx4*>(out)[i] = floatx4{1.f, 2.f, 3.f, (float)i};
}
extern "C" int probe_write(float* out, int64_t bytes, void* stream) {
  const int64_t n4 = bytes / 16;
  hipLaunchKernelGGL(write_stream, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out, n4);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// Soft phase separation: persistent workgroups (contiguous tile ranges) buffer F tiles of
// coefficients in LDS and flush them as 1 KiB-per-wave-instruction bursts.
template <int F>
__global__ void __launch_bounds__(256) fit6_persist(const float* __restrict__ pinv, const float* __restrict__ I, int N,
                                                    int64_t P, float* __restrict__ coef, int tiles_per_wg) {
  extern __shared__ __attribute__((aligned(16))) float buf[];  // [F][1024 px][6]
  const int64_t ntiles = P / 1024;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t t1 = t0 + tiles_per_wg < ntiles ? t0 + tiles_per_wg : ntiles;
  int pending = 0;
  int64_t first = t0;
  for (int64_t t = t0; t < t1; ++t) {
    const int64_t p0 = t * 1024 + threadIdx.x * 4;
    float acc[6][4] = {};
    const float* src = I + p0;
    int n = 0;
    for (; n + 8 <= N; n += 8) {
      floatx4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = ld4<true>(src + (int64_t)(n + u) * P);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const float w = pinv[k * N + n + u];
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[k][v] = fmaf(w, x[u][v], acc[k][v]);
        }
    }
    for (; n < N; ++n) {
      floatx4 x = ld4<true>(src + (int64_t)n * P);
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[k][v] = fmaf(pinv[k * N + n], x[v], acc[k][v]);
    }
    float* slot = buf + pending * 1024 * 6 + threadIdx.x * 24;
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int k = 0; k < 6; k += 2) *reinterpret_cast<float2*>(slot + v * 6 + k) = float2{acc[k][v], acc[k + 1][v]};
    ++pending;
    if (pending == F || t + 1 == t1) {
      __syncthreads();
      const int nf = pending * 1024 * 6 / 4;  // float4s to flush (contiguous in global)
      float* dst = coef + first * 1024 * 6;
      for (int i = threadIdx.x; i < nf; i += 256)
        reinterpret_cast<floatx4*>(dst)[i] = reinterpret_cast<const floatx4*>(buf)[i];
      __syncthreads();
      pending = 0;
      first = t + 1;
    }
  }
}

extern "C" int probe_persist(const float* pinv, const float* I, int N, int64_t P, float* coef, int variant,
                             void* stream) {
  // variant = F * 1000 + workgroups (e.g. 3512 = flush every 3 tiles, 512 workgroups)
  const int F = variant / 1000, wgs = variant % 1000;
  const int64_t ntiles = P / 1024;
  const int per = (int)((ntiles + wgs - 1) / wgs);
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)F * 1024 * 6 * 4;
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fit6_persist<3>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  switch (F) {
    case 1: hipLaunchKernelGGL(fit6_persist<1>, dim3(wgs), dim3(256), lds, s, pinv, I, N, P, coef, per); break;
    case 2: hipLaunchKernelGGL(fit6_persist<2>, dim3(wgs), dim3(256), lds, s, pinv, I, N, P, coef, per); break;
    default: hipLaunchKernelGGL(fit6_persist<3>, dim3(wgs), dim3(256), lds, s, pinv, I, N, P, coef, per); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
