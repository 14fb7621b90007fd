// tile_probe.hip -- measurement-only (not part of librti): the HSH-16 AUTO tile kernel of
// rti_fit.hip (fit_shared_tile_w<16, 8, 0>) with its coefficient stores compiled out, so a sweep
// can split the c4 kernel time into the read stream + MFMA and what the 1.59 GB of stores add.
#include "../../smartphone-based-rti_amd/csrc/rti_fit.hip"

extern "C" int probe_tile_nostore(const float* pinv, int k, int N, const float* I, int64_t P, int C, float* coef,
                                  void* stream) {
  constexpr int RC = 16, W = 8, R = 256 * RC, S = W;
  const int T_ = (N + S - 1) / S;
  const size_t lds = ((size_t)T_ * S * 16 + (size_t)S * R) * sizeof(float);
  auto kern = rti::fit_shared_tile_w<RC, W, 0, float, RTI_COEF_PIXEL_MAJOR, true, 0>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return 3;
  dim3 grid((unsigned)((P + R - 1) / R), C);
  hipLaunchKernelGGL(kern, grid, dim3(64 * W), lds, (hipStream_t)stream, pinv, k, N, I, P, (int64_t)0, P, P, (int64_t)N * P, coef,
                     P * k);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
