// Measurement-only build of the pixel-major VALU generations fit (not part of librti): the library's own
// kernel source is compiled here with its PROBE template argument, which the C ABI cannot reach.
//   pm_probe_vgen(mode = 0): exactly rti_fit_shared_pm's AUTO form (k = 6, fp32, pixel-major coefficients);
//   mode = 1: the same launches with the coefficient stores dropped (reads + arithmetic only);
//   mode | 2: each wave one contiguous run of blocks instead of interleaved units.
#include "../../smartphone-based-rti_amd/csrc/rti_fit_pm.hip"

#include <cstdio>

namespace rti {
int fail(int status, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
  return status;
}
int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? RTI_OK : fail(RTI_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}
hipError_t reserve_lds(const void* kern, size_t bytes) {  // librti's (cached) lives in rti_fit.hip
  return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
int device_cus() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus;
}
void note_launches(int) {}
}  // namespace rti

template <int PROBE, int IL>
static int probe_t(const float* pinv, int N, const float* I, int64_t P, float* coef, int w, int gens,
                   hipStream_t s) {
  using namespace rti;
  const VPlan pl = vgen_plan(6, N, 4, w);
  if (!pl.W || N % 4) return RTI_ERR_UNSUPPORTED;
  auto kern = fit_pm_vgen<6, float, RTI_COEF_PIXEL_MAJOR, 4, vgen_mb(6), IL, PROBE>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)pl.lds) != hipSuccess)
    return RTI_ERR_HIP;
  const int64_t cus = device_cus();
  const VGens g = vgen_split(P, 6, cus * pl.W, gens, 0);  // N % 4 == 0: one-block units
  for (int64_t b = 0; b < g.nbc; b += g.per) {
    const int64_t n = g.nbc - b < g.per ? g.nbc - b : g.per;
    const int64_t wgs = (n + pl.W - 1) / pl.W;
    hipLaunchKernelGGL(kern, dim3((unsigned)(wgs < cus ? wgs : cus)), dim3(64 * pl.W), pl.lds, s, pinv, N, I, P,
                       coef, 64 * b, n, pl.ring, 0);
  }
  return check_launch("pm_probe_vgen");
}

extern "C" int pm_probe_vgen(const float* pinv, int N, const float* I, int64_t P, float* coef, int w, int gens,
                             int mode, void* stream) {
  // mode bit 0: no stores; bit 1: each wave one contiguous run (else interleaved units, the library's AUTO)
  hipStream_t s = (hipStream_t)stream;
  switch (mode & 3) {
    case 0: return probe_t<0, 1>(pinv, N, I, P, coef, w, gens, s);
    case 1: return probe_t<1, 1>(pinv, N, I, P, coef, w, gens, s);
    case 2: return probe_t<0, 0>(pinv, N, I, P, coef, w, gens, s);
    default: return probe_t<1, 0>(pinv, N, I, P, coef, w, gens, s);
  }
}

// (r06) the DIRECT form at HSH-16 (k = 16, fp32 stack, pixel-major coefficients; the library's AUTO for
// c4 pixel-major): mode 0 = exactly the library's launch; bit 0: the bursts' global stores dropped; bit 2:
// non-temporal burst stores; bit 1: "phase" launches — runs of 20 groups (the whole 160-KiB LDS at 8 waves per CU)
// and one run per wave per launch, so every wave of a launch reads its run and then all of them store (the mix
// probe's "stores after the sweep" placement); bit 3: the same with runs of 10 groups, two per wave
// per launch.  C channels of P pixels, channel stride P·N.
template <int PROBE, int NS, int RUNX, bool NTS>
static int probe_direct_t(const float* pinv, int N, const float* I, int64_t P, int C, float* coef, int per_wave,
                          hipStream_t s) {
  using namespace rti;
  constexpr int K = 16, D = pm_direct_depth(NS), RUN = RUNX ? RUNX : pm_direct_run<K, NS>(), RPX = 16 * RUN;
  const int64_t ngrp = (P + 15) / 16, nrun = (P + RPX - 1) / RPX, tr = nrun * C;
  auto kern = fit_pm_direct<K, float, RTI_COEF_PIXEL_MAJOR, NS, D, NTS, PROBE, RUNX>;
  const size_t lds = (size_t)4 * RPX * K * sizeof(float);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return RTI_ERR_HIP;
  const int64_t cap = device_cus() * (int64_t)PM_DIRECT_WPC / 4;
  const int64_t per = per_wave ? cap * 4 * per_wave : tr;  // runs per launch
  for (int64_t r0 = 0; r0 < tr; r0 += per) {
    const int64_t n = tr - r0 < per ? tr - r0 : per, wgs = (n + 3) / 4;
    const unsigned grid = (unsigned)(wgs < cap ? wgs : cap);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, pinv, N, I, P, P * N, coef, P * K, (int)ngrp, (int)nrun,
                       (int)r0, (int)n);
  }
  return check_launch("pm_probe_direct");
}

template <int PROBE>
static int probe_direct_m(const float* pinv, int N, const float* I, int64_t P, int C, float* coef, int mode,
                          hipStream_t s) {
  const bool nts = mode & 4;
  if (mode & 2)
    return nts ? probe_direct_t<PROBE, 13, 20, true>(pinv, N, I, P, C, coef, 1, s)
               : probe_direct_t<PROBE, 13, 20, false>(pinv, N, I, P, C, coef, 1, s);
  if (mode & 8)
    return nts ? probe_direct_t<PROBE, 13, 10, true>(pinv, N, I, P, C, coef, 2, s)
               : probe_direct_t<PROBE, 13, 10, false>(pinv, N, I, P, C, coef, 2, s);
  return nts ? probe_direct_t<PROBE, 13, 0, true>(pinv, N, I, P, C, coef, 0, s)
             : probe_direct_t<PROBE, 13, 0, false>(pinv, N, I, P, C, coef, 0, s);
}

extern "C" int pm_probe_direct(const float* pinv, int N, const float* I, int64_t P, int C, float* coef, int mode,
                               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (rti::pm_direct_ns(N) != 13) return RTI_ERR_UNSUPPORTED;  // the c4 shape (N = 193 .. 208)
  return mode & 1 ? probe_direct_m<1>(pinv, N, I, P, C, coef, mode, s) : probe_direct_m<0>(pinv, N, I, P, C, coef, mode, s);
}
