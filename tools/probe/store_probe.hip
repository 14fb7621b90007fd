// store_probe.hip -- measurement-only (not part of librti): the int32 table write pattern of
// rti_apply_operator_f16 (out[e][p], E rows of P pixels) without any compute, to separate the
// store ceiling from the MFMA/store interplay.  Grid and row sweep as launch_f16: gx = P/TP
// pixel tiles, each workgroup sweeps every 32-row block with its 4 waves.
//   variant 0: the kernel's pattern -- dword NT stores, per instruction 2 rows x 128 B (TP 128)
//   variant 1: same with plain (non-NT) stores
//   variant 2: dwordx4 NT stores, per instruction 2 rows x 512 B (TP 128)
//   variant 3: dwordx4 NT stores, per instruction 1 row x 1 KiB (TP 256)
//   variant 4: dwordx4 plain stores, 1 row x 1 KiB (TP 256)
//   variant 5: ROW SWEEP -- a workgroup owns 128 rows (4 waves x 32) and a segment of the pixels and
//              sweeps it in 128-pixel chunks: per chunk each wave stores its 32 rows x 512 B (dwordx4
//              NT, 2 rows per instruction), so consecutive chunks continue the same rows
//   variant 6: row sweep with 256-pixel chunks (1 row x 1 KiB per instruction)
//   variant 7: variant 5 with plain stores
#include <hip/hip_runtime.h>
#include <cstdint>

typedef int intx4 __attribute__((ext_vector_type(4)));

template <int V>
__global__ void __launch_bounds__(256) store_rows(int* __restrict__ out, int E, int64_t P, int TP) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t p0 = (int64_t)blockIdx.x * TP;
  const int nrb = (E + 31) / 32;
  for (int rb = blockIdx.y * 4 + wave; rb < nrb; rb += gridDim.y * 4) {
    const int val = rb * 7 + lane;
    if constexpr (V == 0 || V == 1) {
      const int r = lane & 31, h = lane >> 5;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = rb * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t px = p0 + 32 * b + r;
          if (row < E && px < P) {
            if constexpr (V == 0) __builtin_nontemporal_store(val + reg, out + (int64_t)row * P + px);
            else out[(int64_t)row * P + px] = val + reg;
          }
        }
      }
    } else if constexpr (V == 2) {
      const int q = lane & 31, h = lane >> 5;  // lanes 0-31 row 2i, 32-63 row 2i+1; 32 lanes x 16 B = 512 B
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = rb * 32 + 2 * i + h;
        const int64_t px = p0 + 4 * q;
        if (row < E && px + 3 < P)
          __builtin_nontemporal_store(intx4{val, i, 0, 1}, reinterpret_cast<intx4*>(out + (int64_t)row * P + px));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int row = rb * 32 + i;
        const int64_t px = p0 + 4 * lane;
        if (row < E && px + 3 < P) {
          intx4* d = reinterpret_cast<intx4*>(out + (int64_t)row * P + px);
          if constexpr (V == 3) __builtin_nontemporal_store(intx4{val, i, 0, 1}, d);
          else *d = intx4{val, i, 0, 1};
        }
      }
    }
  }
}

// row sweep: blockIdx.x = pixel segment, blockIdx.y = 128-row group
template <int CHUNK, bool NT>
__global__ void __launch_bounds__(256) store_sweep(int* __restrict__ out, int E, int64_t P, int64_t seg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = blockIdx.y * 128 + wave * 32;
  const int64_t s0 = (int64_t)blockIdx.x * seg, s1 = s0 + seg < P ? s0 + seg : P;
  for (int64_t c0 = s0; c0 < s1; c0 += CHUNK) {
    constexpr int RPI = CHUNK == 128 ? 2 : 1;  // rows per store instruction
    const int q = CHUNK == 128 ? (lane & 31) : lane, h = CHUNK == 128 ? (lane >> 5) : 0;
#pragma unroll
    for (int i = 0; i < 32 / RPI; ++i) {
      const int row = row0 + RPI * i + h;
      const int64_t px = c0 + 4 * q;
      if (row < E && px + 3 < s1) {
        intx4* d = reinterpret_cast<intx4*>(out + (int64_t)row * P + px);
        if constexpr (NT) __builtin_nontemporal_store(intx4{row, i, 0, 1}, d);
        else *d = intx4{row, i, 0, 1};
      }
    }
  }
}

extern "C" int probe_store_rows(int* out, int E, int64_t P, int variant, int gy, void* stream) {
  const int TP = variant >= 3 ? 256 : 128;
  dim3 grid((unsigned)((P + TP - 1) / TP), (unsigned)gy);
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL(store_rows<0>, grid, dim3(256), 0, s, out, E, P, TP); break;
    case 1: hipLaunchKernelGGL(store_rows<1>, grid, dim3(256), 0, s, out, E, P, TP); break;
    case 2: hipLaunchKernelGGL(store_rows<2>, grid, dim3(256), 0, s, out, E, P, TP); break;
    case 3: hipLaunchKernelGGL(store_rows<3>, grid, dim3(256), 0, s, out, E, P, TP); break;
    case 4: hipLaunchKernelGGL(store_rows<4>, grid, dim3(256), 0, s, out, E, P, TP); break;
    default: {  // row sweeps: gy = pixel segments
      const int64_t seg = ((P + gy - 1) / gy + 255) / 256 * 256;
      const dim3 g2((unsigned)((P + seg - 1) / seg), (unsigned)((E + 127) / 128));
      if (variant == 5) hipLaunchKernelGGL((store_sweep<128, true>), g2, dim3(256), 0, s, out, E, P, seg);
      else if (variant == 6) hipLaunchKernelGGL((store_sweep<256, true>), g2, dim3(256), 0, s, out, E, P, seg);
      else hipLaunchKernelGGL((store_sweep<128, false>), g2, dim3(256), 0, s, out, E, P, seg);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
