// Measurement-only build of the 8-bit split-fp16 fit (not part of librti): rti_fit_h16.hip's own kernel and
// launcher compiled with the PROBE template argument, which the C ABI cannot reach.
//   h16_probe(mode = 0): exactly rti_fit_shared_h16's AUTO launch (1024-pixel tiles for k <= 9);
//   mode = 1: the same launch with the coefficient stores dropped (reads + arithmetic only);
//   mode = 2: the stores non-temporal;  mode = 3 / 4 (k = 6): the rows staged through LDS, whole-line plain / NT stores.
#include "../../smartphone-based-rti_amd/csrc/rti_fit_h16.hip"

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
int device_cus() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus;
}
void note_launches(int) {}
hipError_t reserve_lds(const void* kern, size_t bytes) {
  return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
}  // namespace rti

template <int K, int PROBE, int SM = 0>
static int probe_t(const unsigned char* op, int N, const unsigned char* I, int64_t P, float* coef, hipStream_t s) {
  using namespace rti;
  constexpr int R = K <= 9 ? 1024 : 2048, STEP = 32;
  const size_t lds = h16_lds_bytes<R, STEP>(N);
  auto kern = fit_h16<K, RTI_COEF_PIXEL_MAJOR, R, STEP, 4, PROBE, H16_W, SM>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess) return RTI_ERR_HIP;
  const int64_t tiles = (P + R - 1) / R, wpc = (int64_t)device_cus() * (2048 / R);
  const int tpw = (int)((tiles + wpc - 1) / wpc);
  hipLaunchKernelGGL(kern, dim3((unsigned)((tiles + tpw - 1) / tpw), 1), dim3(64 * H16_W), lds, s, op, N, I,
                     (int64_t)0, P, tpw, P, P, (int64_t)N * P, coef, P * K);
  return check_launch("h16_probe");
}

extern "C" int h16_probe(const void* op, int k, int N, const void* I, int64_t P, float* coef, int mode, void* stream) {
  const auto* o = static_cast<const unsigned char*>(op);
  const auto* x = static_cast<const unsigned char*>(I);
  hipStream_t s = (hipStream_t)stream;
  if (k == 6) switch (mode) {
      case 1: return probe_t<6, 1>(o, N, x, P, coef, s);
      case 2: return probe_t<6, 2>(o, N, x, P, coef, s);
      case 3: return probe_t<6, 0, 1>(o, N, x, P, coef, s);
      case 4: return probe_t<6, 0, 2>(o, N, x, P, coef, s);
      case 5: return probe_t<6, 5>(o, N, x, P, coef, s);
      case 6: return probe_t<6, 6>(o, N, x, P, coef, s);
      default: return probe_t<6, 0>(o, N, x, P, coef, s);
    }
  if (k == 16)
    return mode == 1 ? probe_t<16, 1>(o, N, x, P, coef, s) : mode == 2 ? probe_t<16, 2>(o, N, x, P, coef, s)
                                                           : probe_t<16, 0>(o, N, x, P, coef, s);
  return RTI_ERR_UNSUPPORTED;
}
