// rti_convert.h -- output conversions shared by the relight and operator kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

namespace rti {

template <typename TC>
__device__ __forceinline__ int32_t trunc_i32(TC v) {
  // C truncation toward zero; NaN / out of range -> INT32_MIN (x86 cvttsd2si,
  // which is what NumPy's float64 -> int32 element assignment produces).
  // (|v| < 2^31 is the same test: v = -2^31 converts to INT32_MIN either way; one compare)
  return (v < TC(2147483648.0) && -v < TC(2147483648.0)) ? (int32_t)v : INT32_MIN;
}

template <typename TO, typename TC>
__device__ __forceinline__ TO cvt_out(TC v) {
  if constexpr (std::is_same<TO, float>::value) return (float)v;
  else if constexpr (std::is_same<TO, double>::value) return (double)v;
  else if constexpr (std::is_same<TO, int32_t>::value) return trunc_i32(v);
  else {
    const int32_t i = trunc_i32(v);
    return (uint8_t)(i > 255 ? 255 : (i <= 0 ? 0 : i));
  }
}

}  // namespace rti
