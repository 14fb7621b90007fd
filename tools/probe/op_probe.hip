// op_probe.hip -- measurement-only (not part of librti): rti_operator.hip's split-fp16 table kernel
// (apply_op_f16s, fp32 stack -> int32 tables) launched over a pixel range with an explicit row split
// gy, so a sweep can ask whether keeping the resident workgroups in step (one generation per launch)
// helps the c7 table writes.
#include "../../smartphone-based-rti_amd/csrc/rti_operator.hip"

namespace rti {
hipError_t reserve_lds(const void* kern, size_t bytes) {  // librti's (cached) lives in rti_fit.hip
  return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
}  // namespace rti

extern "C" int probe_op(const void* hi, const void* lo, int Kp, float inv_s, int E, int N, const float* I, int64_t P,
                        int64_t p0, int64_t np, int gy, int* out, void* stream) {
  const size_t lds = (size_t)2 * rti::TP16 * (Kp + 8) * sizeof(_Float16);
  auto k = rti::apply_op_f16s<float, int32_t, true>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return 3;
  const unsigned gx = (unsigned)((np + rti::TP16 - 1) / rti::TP16);
  hipLaunchKernelGGL(k, dim3(gx, gy, 1), dim3(256), lds, (hipStream_t)stream, static_cast<const _Float16*>(hi),
                     static_cast<const _Float16*>(lo), Kp, inv_s, E, N, I + p0, np, P, (int64_t)N * P, out + p0, P,
                     (int64_t)E * P);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
