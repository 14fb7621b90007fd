// rti_internal.h -- helpers shared by the C-ABI translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>

#include "../../include/rti.h"

namespace rti {

// Records a thread-local message (rti_last_error) and returns `status`.
int fail(int status, const char* fmt, ...);
// hipGetLastError after a launch -> RTI_OK or RTI_ERR_HIP.
int check_launch(const char* what);
// compute units of the current HIP device (cached per device; rti_fit.hip)
int device_cus();
// hipFuncSetAttribute(kern, MaxDynamicSharedMemorySize, bytes) once per (kernel, device) and size: the call costs
// microseconds of host time, which every launch of a stream-ordered entry point would otherwise pay
// (rti_fit.hip)
hipError_t reserve_lds(const void* kern, size_t bytes);
// records the kernel launches of the current C-ABI call (rti_last_launch_count)
void note_launches(int n);

// A kernel-selection word: selector (low byte) <= max_sel and no bit outside `flags`.  Every entry point that
// takes one refuses anything else with RTI_ERR_BAD_ARG, so no bit a caller passes can select a behaviour the
// entry does not document (tests/test_abi.py::test_entry_points_refuse_unknown_kernel_bits).
inline bool kernel_bits_ok(int kernel, int max_sel, int flags) {
  return (kernel & 0xff) <= max_sel && (kernel & ~0xff & ~flags) == 0;
}
constexpr int RTI_FIELD_CHUNKS = 0xF << RTI_KERNEL_CHUNKS_SHIFT;
constexpr int RTI_FIELD_TILE_PLANES = 0xF << RTI_KERNEL_TILE_PLANES_SHIFT;
constexpr int RTI_FIELD_TILE_DEPTH = 0xF << RTI_KERNEL_TILE_DEPTH_SHIFT;
constexpr int RTI_FIELD_TILE_WAVES = 0xF << RTI_KERNEL_TILE_WAVES_SHIFT;

__host__ __device__ inline bool aligned_to(const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; }

inline unsigned grid_1d(int64_t items, int per_block) { return (unsigned)((items + per_block - 1) / per_block); }

}  // namespace rti
