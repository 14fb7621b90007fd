// Probe (measurement shim, not product): accuracy of v_rsq_f64 and of one / two Newton steps on it,
// in fp64 ulps of the correctly rounded 1/sqrt(s), over log-uniform s in [2^-20, 2^60].
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

__global__ void k(const double* s, double* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double x = s[i];
  double y0 = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double y1 = fma(y0, fma(-h * y0, y0, 0.5), y0);
  double y2 = fma(y1, fma(-h * y1, y1, 0.5), y1);
  out[3 * i] = y0;
  out[3 * i + 1] = y1;
  out[3 * i + 2] = y2;
}

int main() {
  const int n = 1 << 22;
  double *hs = (double*)malloc(n * 8), *ho = (double*)malloc(3 * n * 8), *ds, *dout;
  srand(1);
  for (int i = 0; i < n; ++i) hs[i] = std::ldexp(1.0 + (double)rand() / RAND_MAX, -20 + rand() % 80);
  (void)hipMalloc(&ds, n * 8);
  (void)hipMalloc(&dout, 3 * n * 8);
  (void)hipMemcpy(ds, hs, n * 8, hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(ds, dout, n);
  (void)hipMemcpy(ho, dout, 3 * n * 8, hipMemcpyDeviceToHost);
  double worst[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const long double ref = 1.0L / sqrtl((long double)hs[i]);
    const double ulp = std::ldexp(1.0, std::ilogb((double)ref) - 52);
    for (int j = 0; j < 3; ++j) {
      const double e = (double)fabsl((long double)ho[3 * i + j] - ref) / ulp;
      if (e > worst[j]) worst[j] = e;
    }
  }
  printf("max error in fp64 ulps: rsq %.4g  one Newton %.4g  two Newton %.4g\n", worst[0], worst[1], worst[2]);
  return 0;
}
