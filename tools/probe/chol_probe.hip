// chol_probe.hip -- measurement-only (not part of librti): rti_rbf_perpixel's blocked Cholesky solver
// (rbf_solve_chol, N > 256) compiled with its phase timer (RTI_CHOL_PROFILE), run on a bench-like ROI;
// prints the mean time per pixel of each phase.
//   tools/probe/chol_probe [N] [pixels]
#define RTI_CHOL_PROFILE 1
#include "../../smartphone-based-rti_amd/csrc/rti_rbf.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I smartphone-based-rti_amd/csrc
//        tools/probe/chol_probe.hip smartphone-based-rti_amd/csrc/rti_host.cpp -o tools/probe/chol_probe
namespace rti {
hipError_t reserve_lds(const void* kern, size_t bytes) {  // librti's (cached) lives in rti_fit.hip
  return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
int device_cus() {  // librti's lives in rti_fit.hip
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  return cus;
}
}  // namespace rti

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 400;
  const int64_t P = argc > 2 ? atoll(argv[2]) : 2560;
  std::mt19937 rng(7);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::vector<float> lu(P * N), lv(P * N), I(P * N);
  std::vector<double> cx(N), cy(N), cz(N);  // camera positions as in bench.py's synth_cams (one light list per pixel)
  for (int j = 0; j < N; ++j) cx[j] = 400 * U(rng), cy[j] = 400 * U(rng), cz[j] = 300 + 100 * U(rng);
  for (int64_t p = 0; p < P; ++p)
    for (int j = 0; j < N; ++j) {
      const double dx = cx[j] - (double)(p % 400), dy = cy[j] - (double)(p / 400), r = sqrt(dx * dx + dy * dy + cz[j] * cz[j]);
      lu[p * N + j] = (float)(dx / r), lv[p * N + j] = (float)(dy / r), I[p * N + j] = (float)(rng() % 256);
    }
  const int E = 10000;
  std::vector<double> luv(2 * E);
  for (int e = 0; e < E; ++e) luv[2 * e] = -1 + 0.02 * (e % 100), luv[2 * e + 1] = -1 + 0.02 * (e / 100);
  float *dlu, *dlv, *dI;
  double* dluv;
  int *dout, *dst;
  (void)hipMalloc(&dlu, 4 * P * N), (void)hipMalloc(&dlv, 4 * P * N), (void)hipMalloc(&dI, 4 * P * N);
  (void)hipMalloc(&dluv, 16 * E), (void)hipMalloc(&dout, 4 * (size_t)E * P), (void)hipMalloc(&dst, 4);
  (void)hipMemcpy(dlu, lu.data(), 4 * P * N, hipMemcpyHostToDevice);
  (void)hipMemcpy(dlv, lv.data(), 4 * P * N, hipMemcpyHostToDevice);
  (void)hipMemcpy(dI, I.data(), 4 * P * N, hipMemcpyHostToDevice);
  (void)hipMemcpy(dluv, luv.data(), 16 * E, hipMemcpyHostToDevice);
  (void)hipMemset(dst, 0, 4);
  int rc = rti_rbf_perpixel(dlu, dlv, dI, RTI_F32, N, P, dluv, E, dout, RTI_I32, RTI_OUT_EVAL_MAJOR, dst, nullptr);
  if (rc || hipDeviceSynchronize() != hipSuccess) return printf("rti_rbf_perpixel failed: %d\n", rc), 1;
  static unsigned long long prof[1024][16];
  (void)hipMemcpyFromSymbol(prof, HIP_SYMBOL(rti_chol_prof), sizeof(prof));
  int rate_khz = 0, cus = 0;
  (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int wg = uses_llt(N) && N <= RBF_LL_TWO_MAX_N ? 2 * cus : cus;  // (r06: up to 448 lights two pixels per CU)
  const int G = (int)(P < wg ? P : wg);
  const char* names_rl[14] = {"load", "A+rowsum", "g colsum", "c,m,S", "stage", "diag factor", "trsm+fwd diag",
                              "writeback+fwd upd", "trailing", "backward (rest)", "final", "  bwd: loads+stage",
                              "  bwd: diag solve", "  bwd: update"};
  // (r06) the left-looking matrix-core form (rbf_solve_llt) marks its own phases
  const char* names_ll[14] = {"load", "rowsum", "c,m", "update (K chunks)", "S init", "sub-panel upd + leaf",
                              "sub-panel solve", "L tile stores", "diag area copy", "bwd: GEMV", "bwd: diag solve",
                              "final", "-", "-"};
  const char** names = uses_llt(N) ? names_ll : names_rl;
  double tot = 0;
  for (int k = 0; k < 14; ++k) {
    double s = 0;
    for (int b = 0; b < G; ++b) s += (double)prof[b][k];
    const double us = s / G / ((double)P / G) / (rate_khz * 1e-3);  // µs per pixel (per workgroup)
    tot += us;
    printf("%-20s %9.2f us/px\n", names[k], us);
  }
  printf("%-20s %9.2f us/px  (N=%d, P=%lld, %d workgroups)\n", "total", tot, N, (long long)P, G);
  return 0;
}
