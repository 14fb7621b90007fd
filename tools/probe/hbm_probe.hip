// hbm_probe.hip -- measurement-only kernels (not part of librti): the achievable
// HBM read ceiling for a light-major stream, to price the fit kernels against.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Each lane reads 16 B per "light" plane, UNROLL planes in flight, like the fit kernel,
// but does one add per element instead of the contraction.
template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) read_stream(const float* __restrict__ I, int N, int64_t P, float* __restrict__ out) {
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= P) return;
  floatx4 acc = {0, 0, 0, 0};
  int n = 0;
  for (; n + UNROLL <= N; n += UNROLL) {
    floatx4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const floatx4* p = reinterpret_cast<const floatx4*>(I + (int64_t)(n + u) * P + p0);
      x[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += x[u];
  }
  for (; n < N; ++n) acc += *reinterpret_cast<const floatx4*>(I + (int64_t)n * P + p0);
  if (acc[0] + acc[1] + acc[2] + acc[3] == -1.2345f) out[0] = acc[0];  // keep the loads alive
}

extern "C" int probe_read(const float* I, int N, int64_t P, float* out, int variant, void* stream) {
  dim3 grid((unsigned)((P / 4 + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL((read_stream<8, false>), grid, dim3(256), 0, s, I, N, P, out); break;
    case 1: hipLaunchKernelGGL((read_stream<8, true>), grid, dim3(256), 0, s, I, N, P, out); break;
    case 2: hipLaunchKernelGGL((read_stream<16, false>), grid, dim3(256), 0, s, I, N, P, out); break;
    default: hipLaunchKernelGGL((read_stream<4, false>), grid, dim3(256), 0, s, I, N, P, out); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
