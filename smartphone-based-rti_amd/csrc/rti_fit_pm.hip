// rti_fit_pm.hip -- the shared-direction fit on PIXEL-major stacks, the reference's own layout.
//
// compute_intensities stacks the ROI as (R, R, N) (analysis.py:217-219): the N intensities of a
// pixel are contiguous.  For a shared light set the solve of analysis.py:293-298 is the same
// contraction as rti_fit.hip's,
//     coef[c][p][i] = Σ_n pinv[i][n] · I[c][p][n],
// but the operand arrives transposed.  A block of B consecutive pixels is then ONE contiguous run
// of B·N values, which is the best shape the HBM stream can ask for: the kernel copies whole
// blocks into LDS with LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, no VGPR hop)
// and contracts them on the matrix cores.
//
//  * fit_pm_dma: every wave owns a private double-buffered LDS ring of two blocks of B pixels
//    (B = 16, 32 or 64).  A wave waits for its block, issues the DMA of its next block (grid-
//    strided over the flattened (channel, block) space), then runs v_mfma_f32_16x16x4_f32 with
//    A = pinv (row i of the [16][N16] zero-padded operator in LDS: lane (q, r) reads
//    pinv[q][16m + 4r .. +3] with one ds_read_b128) and B = the block (lane (q, r) reads
//    I[p0 + q][16m + 4r .. +3]), four MFMAs per 16 lights: D[i][j] is coefficient i of pixel j.
//    The waves never synchronise with each other: each DMA is waited for by a counted vmcnt that
//    leaves the previous block's coefficient stores in flight (CDNA retires loads and stores on
//    one counter in issue order), so those stores are issued unconditionally as buffer stores
//    whose out-of-range lanes the buffer bounds drop.
//  * fit_pm_lane: one lane per pixel, the k×N operator in SGPRs, per-lane loads of the pixel's
//    row.  For what the DMA kernel does not take (uint8 stacks, a pixel stride other than N,
//    unaligned shapes, N past the LDS budget).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "rti_internal.h"

namespace rti {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef int intx4 __attribute__((ext_vector_type(4)));
typedef int intx2 __attribute__((ext_vector_type(2)));

constexpr int PM_LDS = 160 * 1024;
constexpr uint32_t PM_OOB = 0x80000000u;  // buffer offset past every num_records: the store is dropped

// One 1-KiB LDS-DMA (buffer_load_dwordx4 … lds): lane l's 16 bytes at src + voff + soff go to lds + 16·l.
// The descriptor bounds every read (a lane past num_records gets zeros), so no DMA can leave its run.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t src, int voff, int soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0,
                                           2 /* nt */);
}

// a descriptor over `bytes` bytes at p (bytes < 2^32)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(uint32_t)bytes, 0x00020000);
}

template <typename T>
__device__ __forceinline__ float to_f(T v) {
  return (float)v;
}

// 4 consecutive values of the LDS block at float offset `o` (aligned to ALIGN floats)
// a 4-byte value of type T from its bits (passed as a scalar: a bit_cast of a vector element reads element 0,
// clang / ROCm 7.2)
template <typename T>
__device__ __forceinline__ float bits_f(unsigned u) {
  if constexpr (std::is_same<T, float>::value) return __uint_as_float(u);
  else return (float)(int)u;
}

template <int ALIGN, typename T>
__device__ __forceinline__ floatx4 lds4(const float* blk, int o) {
  const T* b = reinterpret_cast<const T*>(blk);
  if constexpr (ALIGN == 4) {
    typedef T tx4 __attribute__((ext_vector_type(4)));
    const tx4 v = *reinterpret_cast<const tx4*>(b + o);
    return floatx4{to_f(v[0]), to_f(v[1]), to_f(v[2]), to_f(v[3])};
  } else if constexpr (ALIGN == 2) {
    typedef T tx2 __attribute__((ext_vector_type(2)));
    const tx2 u = *reinterpret_cast<const tx2*>(b + o), v = *reinterpret_cast<const tx2*>(b + o + 2);
    return floatx4{to_f(u[0]), to_f(u[1]), to_f(v[0]), to_f(v[1])};
  } else {
    return floatx4{to_f(b[o]), to_f(b[o + 1]), to_f(b[o + 2]), to_f(b[o + 3])};
  }
}

// Coefficient stores of one 16-pixel group: lane (q, r) holds coefficients 4r .. 4r+3 of pixel px.
// Every lane issues the same S_GROUP instructions; those of absent coefficients or pixels get an
// out-of-range offset.  Offsets are bytes inside the channel's coefficient buffer (< 2^31).
template <int K, int LAYOUT>
constexpr int stores_per_group() {
  if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR) return K % 4 == 0 ? 1 : (K % 2 == 0 ? 2 : 4);
  return 4;
}

// AUX: the stores' cache policy (0 plain, 2 non-temporal)
template <int K, int LAYOUT, int AUX = 0>
__device__ __forceinline__ void store_group(__amdgpu_buffer_rsrc_t rs, floatx4 d, int64_t px, int64_t P, int r) {
  const bool pin = px < P;
  if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR && K % 4 == 0) {
    const uint32_t off = (pin && 4 * r < K) ? (uint32_t)((px * K + 4 * r) * 4) : PM_OOB;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(intx4, d), rs, off, 0, AUX);
  } else if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR && K % 2 == 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 4 * r + 2 * h;
      const uint32_t off = (pin && i < K) ? (uint32_t)((px * K + i) * 4) : PM_OOB;
      const floatx2 v = h == 0 ? floatx2{d[0], d[1]} : floatx2{d[2], d[3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(intx2, v), rs, off, 0, 0);
    }
  } else {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int i = 4 * r + rr;
      const int64_t e = LAYOUT == RTI_COEF_PIXEL_MAJOR ? px * K + i : (int64_t)i * P + px;
      const uint32_t off = (pin && i < K) ? (uint32_t)(e * 4) : PM_OOB;
      const float v = d[rr];  // (a bit_cast of the vector element itself reads element 0: clang, ROCm 7.2)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), rs, off, 0, 0);
    }
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// BP pixels per block (16·G), K coefficients (<= 16), T = float / int32_t, ALIGN = the alignment of a
// pixel row in floats (4: N % 4 == 0 -> ds_read_b128; 2; 1).  Dynamic LDS: [16][N16] operator, then
// per wave two blocks of `slot` floats.
template <int G, int K, typename T, int LAYOUT, int ALIGN>
__global__ void __launch_bounds__(512)
fit_pm_dma(const float* __restrict__ pinv, int N, const T* __restrict__ I, int64_t P, int64_t cstride,
           float* __restrict__ coef, int64_t ocstride, int64_t nblk, int64_t units, int slot) {
  constexpr int BP = 16 * G;
  constexpr int S = G * stores_per_group<K, LAYOUT>();  // store instructions per block (compile-time)
  static_assert(S <= 63, "vmcnt immediate");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int N16 = (N + 15) & ~15;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar block walk
  float* __restrict__ lp = lds;  // [16][N16]
  for (int idx = threadIdx.x; idx < 16 * N16; idx += blockDim.x) {
    const int i = idx / N16, n = idx - i * N16;
    lp[idx] = (i < K && n < N) ? pinv[i * N + n] : 0.f;
  }
  __syncthreads();
  float* __restrict__ ring = lds + 16 * N16 + wave * 2 * slot;
  const int64_t gw = (int64_t)blockIdx.x * W + wave, GW = (int64_t)gridDim.x * W;
  if (gw >= units) return;
  const int64_t bbytes = (int64_t)BP * N * sizeof(T), cbytes = P * N * (int64_t)sizeof(T);
  const int L = (int)((bbytes + 1023) >> 10);  // DMA instructions per block
  auto issue = [&](int64_t u, int s) {
    const int64_t c = u / nblk, b = u - c * nblk;
    const int64_t rest = cbytes - b * bbytes;  // the block, or the channel's partial last block
    const __amdgpu_buffer_rsrc_t src =
        rsrc_at(reinterpret_cast<const char*>(I + c * cstride) + b * bbytes, rest < bbytes ? rest : bbytes);
    float* dst = ring + s * slot;
    for (int i = 0; i < L; ++i) dma16(src, 16 * lane, i << 10, dst + i * 256);  // lanes past the block read zeros
  };
  const int q = lane & 15, r = lane >> 4;
  const int nfull = N >> 4;  // whole 16-light chunks; a partial last chunk is masked
  issue(gw, 0);
  int s = 0;
  bool first = true;
  for (int64_t u = gw; u < units; u += GW) {
    // this block's DMAs were issued before the previous block's S stores
    if (first) wait_vm<0>(); else wait_vm<S>();
    first = false;
    if (u + GW < units) issue(u + GW, s ^ 1);
    const float* __restrict__ blk = ring + s * slot;
    floatx4 acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = floatx4{0.f, 0.f, 0.f, 0.f};
    int o = q * N + 4 * r;  // pixel q of group 0, lights 4r.. of chunk 0 (T elements)
    for (int m = 0; m < nfull; ++m, o += 16) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(lp + q * N16 + 16 * m + 4 * r);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const floatx4 x = lds4<ALIGN, T>(blk, o + 16 * g * N);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], x[c], acc[g], 0, 0, 0);
      }
    }
    if (N & 15) {  // lights 16·nfull .. N-1; the rest of the chunk reads the next pixel's values: zeroed
      const int n0 = 16 * nfull + 4 * r;
      const floatx4 a = *reinterpret_cast<const floatx4*>(lp + q * N16 + 16 * nfull + 4 * r);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        floatx4 x = lds4<1, T>(blk, o + 16 * g * N);
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = n0 + c < N ? x[c] : 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], x[c], acc[g], 0, 0, 0);
      }
    }
    const int64_t c = u / nblk, p0 = (u - c * nblk) * BP;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(coef + c * ocstride, (short)0,
                                                                        (int)(P * K * 4), 0x00020000);
#pragma unroll
    for (int g = 0; g < G; ++g) store_group<K, LAYOUT>(rs, acc[g], p0 + 16 * g + q, P, r);
    s ^= 1;
  }
}

// s_waitcnt vmcnt(m) for the largest m of {0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48} <= n (waiting for more
// than needed is safe; n is wave-uniform)
__device__ __forceinline__ void wait_vm_dyn(int n) {
  if (n >= 16) {
    if (n >= 32) {
      if (n >= 48) wait_vm<48>(); else wait_vm<32>();
    } else {
      if (n >= 24) wait_vm<24>(); else wait_vm<16>();
    }
  } else if (n >= 4) {
    if (n >= 8) {
      if (n >= 12) wait_vm<12>(); else wait_vm<8>();
    } else {
      if (n >= 6) wait_vm<6>(); else wait_vm<4>();
    }
  } else if (n >= 2) {
    if (n >= 3) wait_vm<3>(); else wait_vm<2>();
  } else if (n == 1) {
    wait_vm<1>();
  } else {
    wait_vm<0>();
  }
}

// Streaming form (AUTO).  The pixels are cut into UNITS of U 16-pixel groups, U = 16 / gcd(N, 16) (or a
// multiple), the fewest whose bytes (16·U·N values) are a whole number of KiB, so no 1-KiB LDS-DMA
// straddles two units and a lane's source pointer just advances by 1 KiB per DMA inside a unit.
// Wave w of the grid owns the units w, w + GW, w + 2·GW, … of the flattened (channel, unit) space
// (interleaved: at any moment the chip reads one contiguous slab of the stack, as the light-major fits do;
// `contig` = 1 gives each wave one contiguous run of units instead, for A/B) and streams them, as one
// virtual byte stream, HBM -> a private LDS ring of `ring` bytes, keeping the ring full: after each group
// it refills every KiB the consumed groups freed, so ≈ ring − 64N bytes per wave stay in flight (the
// double-buffered block form above keeps half its LDS in flight).  Group j of the stream occupies stream
// bytes [64N·j, 64N·(j+1)) (fp32/int32); element (q, n) sits at ring byte (64N·j + 4(qN + n)) mod ring.
// Before group j, the wave waits for the DMA holding its last byte, d = ⌈64N(j+1)/1024⌉ − 1, with an
// exact count of the vector-memory ops issued after it: the DMAs issued after d, plus the S stores of
// every group finished after d was issued (d was issued by the refill after group g(d), or by the prologue).
// NCH > 0: at most NCH 16-light chunks (N <= 16·NCH), fully unrolled with wave-uniform guards: the
// operator's A fragments live in VGPRs (read once from LDS) and every chunk's B reads of a group are issued
// before its first MFMA; NCH = 0: any N, one chunk per loop step with A from LDS.
// NTS: non-temporal coefficient stores (pixel-major k = 16: each group's 16 pixel rows are one 1-KiB line-aligned
// store, AUTO for HSH-16)
template <int K, typename T, int LAYOUT, int ALIGN, int NCH, bool NTS = false>
__global__ void __launch_bounds__(512)
fit_pm_stream(const float* __restrict__ pinv, int N, const T* __restrict__ I, int64_t P, int64_t cstride,
              float* __restrict__ coef, int64_t ocstride, int C, int U, int nu, int64_t tu, int ring, int contig) {
  constexpr int S = stores_per_group<K, LAYOUT>();
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int N16 = (N + 15) & ~15;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* __restrict__ lp = lds;  // [16][N16]
  for (int idx = threadIdx.x; idx < 16 * N16; idx += blockDim.x) {
    const int i = idx / N16, n = idx - i * N16;
    lp[idx] = (i < K && n < N) ? pinv[i * N + n] : 0.f;
  }
  __syncthreads();
  char* __restrict__ rp = reinterpret_cast<char*>(lds + 16 * N16) + wave * ring;
  const int64_t gw = (int64_t)blockIdx.x * W + wave, GW = (int64_t)gridDim.x * W;
  const int GBY = 16 * N * (int)sizeof(T);  // bytes of one 16-pixel group
  const int64_t cbytes = P * N * (int64_t)sizeof(T);
  const int q = lane & 15, r = lane >> 4;
  const int nch = N16 >> 4;                        // 16-light chunks, the last one partial if N % 16
  const int slots = ring >> 10;
  // lane's validity of the 4 lights it reads in the last chunk (the rest belongs to the next pixel)
  const int nlast = N - 16 * (nch - 1) - 4 * r;    // valid lights of the lane's 4 in the last chunk
  const float* __restrict__ lpq = lp + q * N16 + 4 * r;
  floatx4 areg[NCH > 0 ? NCH : 1];
  if constexpr (NCH > 0) {
#pragma unroll
    for (int m = 0; m < NCH; ++m)
      if (m < nch) areg[m] = *reinterpret_cast<const floatx4*>(lpq + 16 * m);
  }
  // this wave's units: k = 0 .. nk-1 -> global unit gu(k)
  int64_t u0, ustep, nk;
  if (contig) {
    const int64_t per = (tu + GW - 1) / GW;
    u0 = gw * per;
    ustep = 1;
    nk = u0 >= tu ? 0 : (tu - u0 < per ? tu - u0 : per);
  } else {
    u0 = gw;
    ustep = GW;
    nk = gw >= tu ? 0 : (tu - 1 - gw) / GW + 1;
  }
  if (nk == 0) return;
  // 32-bit stream counters (SALU has no 64-bit ordered compare): a wave streams < 2 GiB, far below the
  // 288 GB / (one wave per SIMD) of the largest stack; unit indices < nu < 2^31
  const int ng = (int)(nk * U);                 // groups of the stream
  const int dt = (int)(nk * ((U * GBY) >> 10));  // DMAs of the stream
  const int ust = (int)ustep;
  // DMA cursor: unit ud of channel cd, `left` DMAs of it still to issue, the unit's descriptor src (bounded by
  // the unit, or by the channel's end for its partial last unit) and the byte inb inside the unit; ring byte wslot
  int cd = (int)(u0 / nu), ud = (int)(u0 - (int64_t)cd * nu);
  int cg = cd, ug = ud;  // group cursor (below): unit ug of channel cg, group gi within the unit
  const int UB = U * GBY, UKB = UB >> 10;
  __amdgpu_buffer_rsrc_t src;
  int inb = 0;
  auto seek = [&]() {
    const int64_t ub = (int64_t)ud * UB, rest = cbytes - ub;
    src = rsrc_at(reinterpret_cast<const char*>(I + cd * cstride) + ub, rest < UB ? rest : UB);
    inb = 0;
  };
  seek();
  int left = UKB, wslot = 0;
  auto issue = [&]() {
    dma16(src, 16 * lane, inb, rp + wslot);
    inb += 1024;
    wslot += 1024;
    wslot = wslot == ring ? 0 : wslot;
    if (--left == 0) {  // next unit (no division: ustep = GW or 1 is far below nu in practice)
      left = UKB;
      ud += ust;
      while (ud >= nu) {
        ud -= nu;
        ++cd;
      }
      if (cd < C) seek();
    }
  };
  int issued = dt < slots ? dt : slots;
  for (int d = 0; d < issued; ++d) issue();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(coef + (int64_t)cg * ocstride, (short)0,
                                                                (int)(P * K * 4), 0x00020000);
  int gi = 0;
  int px0 = ug * U * 16;  // first pixel of group j (< P·... < 2^31)
  int base = 0;           // ring byte of group j's first byte
  int gd = -1;            // the refill (group index; -1 = prologue) that issued the DMA group j waits for
  int end = 0;            // stream bytes of groups 0..j
  const int e0b = (q * N + 4 * r) * (int)sizeof(T);  // the lane's first byte in a group
  for (int j = 0; j < ng; ++j) {
    end += GBY;
    const int dn = ((end + 1023) >> 10) - 1;
    // the refill after group g issues DMAs up to ((g+1)·GBY + ring)/1 KiB (prologue: ring/1 KiB)
    while (((GBY * (gd + 1) + ring) >> 10) < dn + 1) ++gd;
    const int nwait = (issued - 1 - dn) + S * (j - 1 - gd);
    wait_vm_dyn(nwait > 63 ? 63 : nwait);
    int a0 = base + e0b;  // ring byte of the lane's first value, chunks 64·sizeof(T)/4 bytes apart
    a0 -= a0 >= ring ? ring : 0;
    auto rdx = [&](int m) -> floatx4 {  // the lane's 4 values of chunk m (ring wrap per 16 B, or per value)
      if constexpr (ALIGN == 4) {
        int a = a0 + 16 * (int)sizeof(T) * m;
        a -= a >= ring ? ring : 0;
        return lds4<4, T>(reinterpret_cast<const float*>(rp + a), 0);
      } else {
        floatx4 v;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          int a = a0 + (16 * m + t) * (int)sizeof(T);
          a -= a >= ring ? ring : 0;
          v[t] = to_f(*reinterpret_cast<const T*>(rp + a));
        }
        return v;
      }
    };
    auto mask_last = [&](floatx4& x) {  // lights past N in the last chunk: the next pixel's values
#pragma unroll
      for (int t = 0; t < 4; ++t) x[t] = t < nlast ? x[t] : 0.f;
    };
    floatx4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto mma = [&](floatx4 a, floatx4 x) {
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], x[t], acc[t], 0, 0, 0);
    };
    if constexpr (NCH > 0) {
      floatx4 x[NCH];
#pragma unroll
      for (int m = 0; m < NCH; ++m)
        if (m < nch) x[m] = rdx(m);
#pragma unroll
      for (int m = 0; m < NCH; ++m)  // (compile-time index: no dynamic indexing of the register array)
        if (m == nch - 1 && (N & 15)) mask_last(x[m]);
#pragma unroll
      for (int m = 0; m < NCH; ++m)
        if (m < nch) mma(areg[m], x[m]);
    } else {
      for (int m = 0; m < nch; ++m) {
        floatx4 x = rdx(m);
        if (m == nch - 1 && (N & 15)) mask_last(x);
        mma(*reinterpret_cast<const floatx4*>(lpq + 16 * m), x);
      }
    }
    const floatx4 d = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    store_group<K, LAYOUT, NTS ? 2 : 0>(rs, d, px0 + q, P, r);  // groups past P: every store dropped
    // refill every KiB the groups 0..j freed
    const int lim0 = (end + ring) >> 10;
    const int lim = lim0 < dt ? lim0 : dt;
    for (; issued < lim; ++issued) issue();
    base += GBY;
    base -= base >= ring ? ring : 0;
    px0 += 16;
    if (++gi == U) {
      gi = 0;
      ug += ust;
      const int cg0 = cg;
      while (ug >= nu) {
        ug -= nu;
        ++cg;
      }
      px0 = ug * U * 16;
      if (cg != cg0 && cg < C)
        rs = __builtin_amdgcn_make_buffer_rsrc(coef + (int64_t)cg * ocstride, (short)0, (int)(P * K * 4), 0x00020000);
    }
  }
}

// VALU form (AUTO for k <= 9), r05: LAUNCH GENERATIONS with the coefficients parked in registers.
// A launch covers a range of one channel's 64-pixel blocks; wave w of its GW waves owns ONE contiguous run
// of nb <= MB blocks (nb·64·N values) and streams it HBM -> a private LDS ring of `ring` bytes with 1-KiB
// LDS-DMAs (buffer_load_dwordx4 … lds: the descriptor covers exactly the run, so a lane past it reads
// zeros and no DMA can leave the stack), keeping the ring full.  Lane l computes pixel l of each block
// (its row read from the ring by ds_read_b128, k coefficients by packed FMAs over light pairs, the
// weights broadcast from an LDS copy) and PARKS the k coefficients of block j in registers
// park[j][0..k-1] (j is a compile-time index: the block loop is unrolled MB times around the rolled
// light loop).  Only after its last block does the wave store, so every wave of the chip reads during
// the launch and writes at its end: the read/write phase separation the light-major fit gets from its
// own launch generations (the r04 form stored every block as it finished, "spread"
// through the read stream, and lost 0.13 ms of 0.63 on c3 to that placement).
// Waits: before block j the wave needs the DMA holding the block's last byte; only DMAs are in flight
// (no stores until the end), so vmcnt = the DMAs issued after it, exactly.
// IL = 1: the launch's UNITS (U blocks, U = 4 / gcd(N, 4): whole KiB of 4-byte values) are dealt to the waves
// round-robin (wave w: units w, w + GW, …), so at any moment the chip reads one contiguous slab of the stack,
// as the light-major fit's waves do; IL = 0: each wave one contiguous run of blocks.  The two are
// bit-identical; the wave's run is then a list of unit segments, each with its own bounded descriptor.
// PROBE (not reachable from the C ABI; tools/probe/pm_probe.hip): 1 = no coefficient stores.
template <int K, typename T, int LAYOUT, int ALIGN, int MB, int IL = 1, int PROBE = 0>
__global__ void __launch_bounds__(384)
fit_pm_vgen(const float* __restrict__ pinv, int N, const T* __restrict__ I, int64_t P, float* __restrict__ coef,
            int64_t pb, int64_t nblk, int ring, int ulog) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the operator in LDS as [N4/4][K][4] (zero padded): one broadcast ds_read_b128 gives pinv[i][n .. n+3]
  const int N4 = (N + 3) & ~3;
  float* __restrict__ lw = lds;
  for (int idx = threadIdx.x; idx < N4 * K; idx += blockDim.x) {
    const int nq = idx / (4 * K), rem = idx - nq * 4 * K, i = rem >> 2, n = 4 * nq + (rem & 3);
    lw[idx] = n < N ? pinv[i * N + n] : 0.f;
  }
  __syncthreads();
  char* __restrict__ rp = reinterpret_cast<char*>(lds + N4 * K) + wave * ring;
  const int64_t gw = (int64_t)blockIdx.x * W + wave, GW = (int64_t)gridDim.x * W;
  const int RB = N * (int)sizeof(T);  // bytes of one pixel row
  const int BB = 64 * RB;             // bytes of one block
  // this wave's blocks of the launch (IL: units of U = 2^ulog blocks; the launch covers nblk blocks = whole
  // units from block pb/64 on, except at the channel's end)
  int64_t px0, pxe;  // IL = 0: pixels [px0, pxe)
  int nb, bytes, cnt = 1;
  const int U = 1 << ulog, UB = BB << ulog;
  const int64_t u0 = pb / (64 * U) + gw;  // IL: this wave's first unit (units u0, u0 + GW, …)
  if constexpr (IL) {
    const int64_t nun = (nblk + U - 1) >> ulog;
    if (gw >= nun) return;
    cnt = (int)((nun - 1 - gw) / GW + 1);
    const int64_t last = (u0 + (int64_t)(cnt - 1) * GW) * U * 64;  // first pixel of the last unit
    const int lastpx = (int)(P - last < 64 * U ? P - last : 64 * U);
    nb = ((cnt - 1) << ulog) + (lastpx + 63) / 64;
    bytes = (cnt - 1) * UB + lastpx * RB;
    px0 = pxe = 0;
  } else {
    const int64_t b0 = nblk * gw / GW, b1 = nblk * (gw + 1) / GW;
    nb = (int)(b1 - b0);
    if (nb <= 0) return;
    px0 = pb + 64 * b0;
    pxe = pb + 64 * b1 < P ? pb + 64 * b1 : P;
    bytes = (int)(pxe - px0) * RB;
  }
  // descriptors: IL = unit s of the wave (UB bytes, or the channel's partial last unit), else the whole run;
  // num_records rounded up to 16 B so a segment's last 16-B DMA piece is in range (a segment starts 256-B
  // aligned; one that ends before P is followed by the channel's next pixels, one that ends at P by the
  // channel's 16-B aligned end: pm_dma_shape, P·N % 4 == 0, I 16-byte aligned)
  auto seg_src = [&](int sg) {
    if constexpr (IL) {
      const int64_t p0 = (u0 + sg * GW) * U * 64;
      const int64_t rest = (P - p0) * RB;
      return rsrc_at(I + p0 * N, ((rest < UB ? rest : UB) + 15) & ~15);
    } else {
      return rsrc_at(I + px0 * N, (bytes + 15) & ~15);
    }
  };
  const int seg_kb = IL ? UB >> 10 : 0x7fffffff;  // DMAs per segment
  const int dt = (bytes + 1023) >> 10;            // DMAs of the run
  const int slots = ring >> 10;
  int issued = 0, wslot = 0, seg = 0, dseg = 0;
  __amdgpu_buffer_rsrc_t src = seg_src(0);
  auto issue = [&]() {
    dma16(src, 16 * lane, dseg << 10, rp + wslot);
    wslot += 1024;
    wslot = wslot == ring ? 0 : wslot;
    if (++dseg == seg_kb) {
      dseg = 0;
      if (++seg < cnt) src = seg_src(seg);
    }
  };
  for (const int pro = dt < slots ? dt : slots; issued < pro; ++issued) issue();
  float park[MB][K];
  int base = 0;  // ring byte of block j's first byte
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    if (j < nb) {
      const int end = BB * (j + 1) < bytes ? BB * (j + 1) : bytes;  // (bytes: the run's last byte + 1)
      wait_vm_dyn(issued - ((end + 1023) >> 10));  // the DMAs issued after the one holding the block's last byte
      int a0 = base + RB * lane;
      a0 -= a0 >= ring ? ring : 0;
      f2 acc[K];
#pragma unroll
      for (int i = 0; i < K; ++i) acc[i] = f2{0.f, 0.f};
      float acc1[K];
#pragma unroll
      for (int i = 0; i < K; ++i) acc1[i] = 0.f;
      int n = 0;
      if constexpr (ALIGN == 4) {
        // one step of 4 lights ahead: step n + 4's row values and weights are read while step n's 2·K
        // packed FMAs issue (ping-pong register sets, no loop-carried copies)
        auto rdx = [&](int nn) {
          int a = a0 + nn * (int)sizeof(T);
          a -= a >= ring ? ring : 0;
          return lds4<4, T>(reinterpret_cast<const float*>(rp + a), 0);
        };
        auto wts = [&](int nn, int i) { return *reinterpret_cast<const floatx4*>(lw + nn * K + 4 * i); };
        auto step = [&](const floatx4& x, const floatx4 (&w)[K]) {
          const f2 x01 = {x[0], x[1]}, x23 = {x[2], x[3]};
#pragma unroll
          for (int i = 0; i < K; ++i) {
            acc[i] = x01 * f2{w[i][0], w[i][1]} + acc[i];
            acc[i] = x23 * f2{w[i][2], w[i][3]} + acc[i];
          }
        };
        const int n4 = N & ~3;
        if (n4 > 0) {
          floatx4 xa = rdx(0), xb, wa[K], wb[K];
#pragma unroll
          for (int i = 0; i < K; ++i) wa[i] = wts(0, i);
          for (n = 0; n < n4; n += 8) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this half's operands
            if (n + 4 < n4) {
              xb = rdx(n + 4);
#pragma unroll
              for (int i = 0; i < K; ++i) wb[i] = wts(n + 4, i);
            }
            __builtin_amdgcn_sched_barrier(0);
            step(xa, wa);
            if (n + 4 >= n4) break;
            __builtin_amdgcn_s_waitcnt(0xC07F);
            if (n + 8 < n4) {
              xa = rdx(n + 8);
#pragma unroll
              for (int i = 0; i < K; ++i) wa[i] = wts(n + 8, i);
            }
            __builtin_amdgcn_sched_barrier(0);
            step(xb, wb);
          }
          n = n4;
        }
      }
      if constexpr (ALIGN == 2) {  // N % 4 == 2: 8-byte aligned rows, light pairs by ds_read_b64
        typedef T tx2 __attribute__((ext_vector_type(2)));
        const int n2 = N & ~1;
#pragma unroll 2
        for (; n < n2; n += 2) {
          int a = a0 + n * (int)sizeof(T);
          a -= a >= ring ? ring : 0;
          const tx2 v = *reinterpret_cast<const tx2*>(rp + a);
          const f2 x = {to_f(v[0]), to_f(v[1])};
#pragma unroll
          for (int i = 0; i < K; ++i)
            acc[i] = x * *reinterpret_cast<const f2*>(lw + (n >> 2) * 4 * K + 4 * i + (n & 3)) + acc[i];
        }
      }
      for (; n < N; ++n) {  // N % 4 (or every light when the rows are not 8-byte aligned)
        int a = a0 + n * (int)sizeof(T);
        a -= a >= ring ? ring : 0;
        const float x = to_f(*reinterpret_cast<const T*>(rp + a));
#pragma unroll
        for (int i = 0; i < K; ++i) acc1[i] = fmaf(x, lw[(n >> 2) * 4 * K + 4 * i + (n & 3)], acc1[i]);
      }
#pragma unroll
      for (int i = 0; i < K; ++i) park[j][i] = (acc[i][0] + acc[i][1]) + acc1[i];
      // refill every KiB the blocks 0..j freed
      const int lim0 = (BB * (j + 1) + ring) >> 10;
      for (const int lim = lim0 < dt ? lim0 : dt; issued < lim; ++issued) issue();
      base += BB;  // (BB < ring)
      base -= base >= ring ? ring : 0;
    }
  }
  if constexpr (PROBE == 1) {  // measurement (tools/probe): keep the arithmetic, drop the stores
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < MB; ++j)
#pragma unroll
      for (int i = 0; i < K; ++i) t += park[j][i];
    if (t == -1.2345f) coef[0] = t;
    return;
  }
  // the burst: every parked coefficient, block by block (lanes past the run store nothing)
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    const int64_t px = IL ? ((u0 + (int64_t)(j >> ulog) * GW) * U + (j & (U - 1))) * 64 + lane : px0 + 64 * j + lane;
    if (j < nb && px < (IL ? P : pxe)) {
      if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR && K % 2 == 0) {
#pragma unroll
        for (int i = 0; i < K; i += 2)
          *reinterpret_cast<f2*>(coef + px * K + i) = f2{park[j][i], park[j][i + 1]};
      } else {
#pragma unroll
        for (int i = 0; i < K; ++i) coef[LAYOUT == RTI_COEF_PIXEL_MAJOR ? px * K + i : (int64_t)i * P + px] = park[j][i];
      }
    }
  }
}

// DIRECT form (AUTO for N % 4 == 0, N <= 256): the stack goes straight into VGPRs, LDS only stages the
// coefficients.  A wave streams 16-pixel groups (16·N contiguous values): for 16-light step s, lane (q, r)
// loads I[p0 + q][16s + 4r .. +3] with one 16-byte buffer load, which is the B operand of four
// v_mfma_f32_16x16x4_f32 (MFMA j takes element j: light 16s + 4r + j at k-index r, 16 pixels × 64 contiguous
// bytes per load instruction); the A operand, pinv[q][16s + 4r + j], stays in VGPRs for the whole launch
// (4·NS values per lane).  D groups of loads are in flight per wave.  Lights past N and pixels past P are
// out-of-range buffer offsets (they read zero and move no bytes), so no lane reads a neighbour pixel's values
// (a NaN stays in its pixel).  Loads are plain, not non-temporal: a load instruction touches each 128-byte
// line of its 16 rows by halves, and non-temporal halves went to HBM twice (c3 0.93 against 0.69 ms).
// Runs: a wave takes RUN consecutive groups (runs interleaved over the waves of the grid), parks each group's
// coefficients in its LDS run buffer and writes the run out as one burst of 1-KiB stores (pixel-major: the
// run's coefficients are one contiguous range).  Stores spread thinly through the read stream cost the most
// (the mixed read/write probes, DESIGN §4.1e: 0.61 against 0.52 ms for the same bytes written in bursts);
// the loads of the next D groups stay in flight across a burst.  The loads and MFMAs are straight-line code
// per group, so the compiler's own vmcnt waits are exact.
template <int K, int NS>
constexpr int pm_direct_run() { return K > 9 ? 12 : 24; }  // groups per run (a multiple of the depth)

// NTS: the bursts' stores non-temporal (RTI_KERNEL_NT_STORE; pixel-major).  PROBE (measurement builds only,
// tools/probe/pm_probe.hip; the C ABI cannot reach it): 1 = the bursts' global stores dropped.  RUNX: groups per
// run when non-zero (measurement builds)
template <int K, typename T, int LAYOUT, int NS, int D, bool NTS = false, int PROBE = 0, int RUNX = 0>
__global__ void __launch_bounds__(256)
fit_pm_direct(const float* __restrict__ pinv, int N, const T* __restrict__ I, int64_t P, int64_t cstride,
              float* __restrict__ coef, int64_t ocstride, int ngrp, int nrun, int r0, int tr) {
  constexpr int RUN = RUNX ? RUNX : pm_direct_run<K, NS>(), RPX = 16 * RUN;  // groups and pixels per run
  static_assert(RUN % D == 0, "runs of whole pipeline steps");
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) float runbuf[];  // per wave: RPX·K floats
  const int lane = threadIdx.x & 63, q = lane & 15, r = lane >> 4;
  const int W = blockDim.x >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gw = (int)blockIdx.x * W + wave, GW = (int)gridDim.x * W;
  // this wave's runs of [r0, r0 + tr): gw, gw + GW, ...; run index = channel·nrun + run in channel
  const int nr = gw < tr ? (tr - 1 - gw) / GW + 1 : 0;
  if (nr == 0) return;
  float* __restrict__ buf = runbuf + wave * RPX * K;
  float w[NS][4];
  int off[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int n = 16 * s + 4 * r;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[s][j] = (q < K && n + j < N) ? pinv[q * N + n + j] : 0.f;
    off[s] = n < N ? (q * N + n) * (int)sizeof(T) : (int)PM_OOB;
  }
  const int gq = GW / nrun, gr = GW - gq * nrun;  // advance of a run cursor by GW runs
  const int first = r0 + gw;
  // load cursor (D groups ahead of the compute): run (lc, lj), group lw inside it, runs left lrl
  int lc = first / nrun, lj = first - lc * nrun, lw = 0, lrl = nr;
  int sc = lc, sj = lj;  // the run being computed
  auto load = [&](u4 (&x)[NS]) {
    const int g = lj * RUN + lw;  // group in the channel
    const int64_t p0 = (int64_t)g * 16;
    const int rows = (lrl > 0 && g < ngrp) ? (int)(P - p0 < 16 ? P - p0 : 16) : 0;  // 0: zero-traffic loads
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(I + (int64_t)lc * cstride + p0 * N), (short)0, rows * N * (int)sizeof(T), 0x00020000);
#pragma unroll
    for (int s = 0; s < NS; ++s) x[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[s], 0, 0);
    if (++lw == RUN) {
      lw = 0;
      --lrl;
      lj += gr;
      lc += gq;
      if (lj >= nrun) {
        lj -= nrun;
        ++lc;
      }
    }
  };
  u4 x[D][NS];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    load(x[d]);
    __builtin_amdgcn_sched_barrier(0);  // the prologue's groups in stream order
  }
  for (int run = 0; run < nr; ++run) {
    for (int i = 0; i < RUN; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        __builtin_amdgcn_sched_barrier(0);  // each group's loads in their own place
        floatx4 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[s][j], bits_f<T>(x[d][s][j]), acc[j], 0, 0, 0);
        load(x[d]);
        const floatx4 c = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        // lane (q, r): coefficients 4r .. 4r+3 of pixel (i + d)·16 + q of the run
        const int px = (i + d) * 16 + q;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * r + e < K) {
            const float v = c[e];
            buf[LAYOUT == RTI_COEF_PIXEL_MAJOR ? px * K + 4 * r + e : (4 * r + e) * RPX + px] = v;
          }
      }
    }
    // the run's burst: its coefficients from the LDS buffer, 1 KiB per store instruction (pixel-major)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t px0 = (int64_t)sj * RPX;  // first pixel of the run in its channel
    if constexpr (PROBE == 1) {  // measurement: keep the LDS parking, drop the global stores
      if (buf[lane] == -1.2345f) coef[0] = buf[lane];
    } else {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(coef + (int64_t)sc * ocstride, (short)0,
                                                                        (int)(P * K * 4), 0x00020000);
    if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR) {
      constexpr int BYTES = RPX * K * 4, NI = (BYTES + 1023) / 1024;
#pragma unroll
      for (int n = 0; n < NI; ++n) {
        const int b = 1024 * n + 16 * lane;  // byte in the run (past P: beyond num_records, dropped)
        const floatx4 v = b < BYTES ? *reinterpret_cast<const floatx4*>(reinterpret_cast<const char*>(buf) + b)
                                    : floatx4{0.f, 0.f, 0.f, 0.f};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(intx4, v), rs,
                                               b < BYTES ? (int)(px0 * K * 4) + b : (int)PM_OOB, 0, NTS ? 2 : 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int n = 0; n < RPX / 64; ++n) {
          const int px = 64 * n + lane;
          const float v = buf[i * RPX + px];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), rs,
                                                px0 + px < P ? (int)(((int64_t)i * P + px0 + px) * 4) : (int)PM_OOB,
                                                0, 0);
        }
    }
    }  // (PROBE)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the buffer is rewritten by the next run
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    sj += gr;
    sc += gq;
    if (sj >= nrun) {
      sj -= nrun;
      ++sc;
    }
  }
}

// one lane per pixel: the fallback for every shape the DMA kernel does not take
template <int K, typename T, int LAYOUT>
__global__ void __launch_bounds__(256)
fit_pm_lane(const float* __restrict__ pinv, int k, int N, const T* __restrict__ I, int64_t P, int64_t pstride,
            int64_t cstride, float* __restrict__ coef, int64_t ocstride) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const T* __restrict__ row = I + (int64_t)blockIdx.y * cstride + p * pstride;
  float acc[K];
#pragma unroll
  for (int i = 0; i < K; ++i) acc[i] = 0.f;
  for (int n = 0; n < N; ++n) {
    const float x = (float)row[n];
#pragma unroll
    for (int i = 0; i < K; ++i)
      if (i < k) acc[i] = fmaf(pinv[i * N + n], x, acc[i]);  // wave-uniform: s_load
  }
  float* __restrict__ dst = coef + (int64_t)blockIdx.y * ocstride;
#pragma unroll
  for (int i = 0; i < K; ++i)
    if (i < k) dst[LAYOUT == RTI_COEF_PIXEL_MAJOR ? p * k + i : (int64_t)i * P + p] = acc[i];
}

struct PmArgs {
  const float* pinv;
  int k, N;
  const void* I;
  int64_t P;
  int C;
  int64_t ps, cs;
  float* coef;
  int layout;
  int64_t ocs;
  hipStream_t stream;
};

// LDS plan of the DMA kernel: G groups of 16 pixels per block, W waves per workgroup
struct PmPlan {
  int G = 0, W = 0, slot = 0;
  size_t lds = 0;
};

PmPlan pm_plan(int N, size_t es, int g_req, int w_req) {
  const size_t op = (size_t)16 * ((N + 15) & ~15) * sizeof(float);
  for (int G : {4, 2, 1}) {
    if (g_req && G != g_req) continue;
    // floats: whole KiB for the DMAs + 16 floats the masked tail chunk may read past the block
    const int slot = (int)((((int64_t)16 * G * N * es + 1023) >> 10) << 8) + 16;
    const size_t per_wave = (size_t)2 * slot * sizeof(float);
    if (op + per_wave > (size_t)PM_LDS) continue;
    int W = (int)((PM_LDS - op) / per_wave);
    W = W > 8 ? 8 : W;
    if (w_req) {
      if (w_req > W) continue;
      W = w_req;
    }
    // AUTO: the widest block that still leaves >= 4 waves per CU, else the most waves
    if (!g_req && !w_req && W < 4 && G > 1) continue;
    PmPlan pl;
    pl.G = G;
    pl.W = W;
    pl.slot = slot;
    pl.lds = op + (size_t)W * per_wave;
    return pl;
  }
  return PmPlan();
}

template <int G, int K, typename T, int LAYOUT, int ALIGN>
int launch_dma_t(const PmArgs& a, const PmPlan& pl) {
  auto kern = fit_pm_dma<G, K, T, LAYOUT, ALIGN>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), pl.lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared_pm: LDS attribute");
  const int64_t nblk = (a.P + 16 * G - 1) / (16 * G), units = nblk * a.C;
  const int64_t wgs_needed = (units + pl.W - 1) / pl.W;
  const int64_t cus = device_cus();
  const unsigned grid = (unsigned)(wgs_needed < cus ? wgs_needed : cus);  // one workgroup per CU (LDS-bound)
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * pl.W), pl.lds, a.stream, a.pinv, a.N, static_cast<const T*>(a.I),
                     a.P, a.cs, a.coef, a.ocs, nblk, units, pl.slot);
  return RTI_OK;
}

template <int G, int K, typename T, int LAYOUT>
int launch_dma_a(const PmArgs& a, const PmPlan& pl) {
  if (a.N % 4 == 0) return launch_dma_t<G, K, T, LAYOUT, 4>(a, pl);
  if (a.N % 2 == 0) return launch_dma_t<G, K, T, LAYOUT, 2>(a, pl);
  return launch_dma_t<G, K, T, LAYOUT, 1>(a, pl);
}

template <int K, typename T, int LAYOUT>
int launch_dma_g(const PmArgs& a, const PmPlan& pl) {
  switch (pl.G) {
    case 4: return launch_dma_a<4, K, T, LAYOUT>(a, pl);
    case 2: return launch_dma_a<2, K, T, LAYOUT>(a, pl);
    default: return launch_dma_a<1, K, T, LAYOUT>(a, pl);
  }
}

template <int K, typename T>
int launch_dma_l(const PmArgs& a, const PmPlan& pl) {
  return a.layout == RTI_COEF_PLANAR ? launch_dma_g<K, T, RTI_COEF_PLANAR>(a, pl)
                                     : launch_dma_g<K, T, RTI_COEF_PIXEL_MAJOR>(a, pl);
}

template <typename T>
int launch_dma(const PmArgs& a, const PmPlan& pl) {
  switch (a.k) {
    case 6: return launch_dma_l<6, T>(a, pl);
    case 9: return launch_dma_l<9, T>(a, pl);
    case 16: return launch_dma_l<16, T>(a, pl);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: k=%d", a.k);
  }
}

// streaming plan: W waves per workgroup (one workgroup per CU), a ring of whole KiB per wave that holds at
// least one group + 1 KiB.  AUTO takes the most waves that fit: the wave's issue rate, not the bytes in
// flight, bounds the stream (c3 4K×100: 8 waves 0.665 ms with 19-KiB rings, 4 waves 0.82, 2 waves 1.57
// with 76-KiB rings; c4 4K RGB×200: 8 waves 3.80 ms, 4 waves 4.15-4.63; profiles/r04_pm_sweep.log)
struct StreamPlan {
  int W = 0, ring = 0, contig = 0, unit = 1;
  bool nts = false;  // non-temporal coefficient stores (k = 16, pixel-major)
  size_t lds = 0;
};

StreamPlan stream_plan(int N, size_t es, int w_req, int u_req) {
  const size_t op = (size_t)16 * ((N + 15) & ~15) * sizeof(float);
  const int64_t gby = (int64_t)16 * N * es;
  for (int W : {8, 6, 4, 3, 2, 1}) {
    if (w_req && W != w_req) continue;
    if (op >= (size_t)PM_LDS) break;
    const int ring = (int)(((PM_LDS - op) / W) >> 10 << 10);
    if (ring < gby + 1024) continue;
    StreamPlan pl;
    pl.W = W;
    pl.ring = ring;
    pl.lds = op + (size_t)W * ring;
    pl.unit = u_req > 0 ? u_req : 1;
    return pl;
  }
  return StreamPlan();
}

template <int K, typename T, int LAYOUT, int ALIGN, int NCH>
int launch_stream_t(const PmArgs& a, const StreamPlan& pl) {
  auto kern = fit_pm_stream<K, T, LAYOUT, ALIGN, NCH>;
  if constexpr (K == 16 && LAYOUT == RTI_COEF_PIXEL_MAJOR)
    if (pl.nts) kern = fit_pm_stream<K, T, LAYOUT, ALIGN, NCH, true>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), pl.lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared_pm: LDS attribute");
  const int64_t cus = device_cus();
  int g = 16, nn = a.N;  // U = (16 / gcd(N, 16)) · unit: a whole number of KiB (4-byte values)
  while (g > 1 && nn % g) g >>= 1;
  const int U = 16 / g * pl.unit;
  const int64_t nu = (a.P + 16 * U - 1) / (16 * U), tu = nu * a.C;
  if (nu >= ((int64_t)1 << 31) / (16 * U)) return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: P too large");
  const int64_t wgs = (tu + pl.W - 1) / pl.W;
  const unsigned grid = (unsigned)(wgs < cus ? wgs : cus);  // one workgroup per CU (LDS-bound)
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * pl.W), pl.lds, a.stream, a.pinv, a.N, static_cast<const T*>(a.I),
                     a.P, a.cs, a.coef, a.ocs, a.C, U, (int)nu, tu, pl.ring, pl.contig);
  return RTI_OK;
}

template <int K, typename T, int LAYOUT, int ALIGN>
int launch_stream_n(const PmArgs& a, const StreamPlan& pl) {
  const int nch = (a.N + 15) >> 4;
  if (nch <= 4) return launch_stream_t<K, T, LAYOUT, ALIGN, 4>(a, pl);
  if (nch <= 8) return launch_stream_t<K, T, LAYOUT, ALIGN, 8>(a, pl);
  if (nch <= 16) return launch_stream_t<K, T, LAYOUT, ALIGN, 16>(a, pl);
  return launch_stream_t<K, T, LAYOUT, ALIGN, 0>(a, pl);
}

template <int K, typename T, int LAYOUT>
int launch_stream_a(const PmArgs& a, const StreamPlan& pl) {
  if (a.N % 4 == 0) return launch_stream_n<K, T, LAYOUT, 4>(a, pl);
  return launch_stream_n<K, T, LAYOUT, 1>(a, pl);
}

template <typename T>
int launch_stream(const PmArgs& a, const StreamPlan& pl) {
  const bool planar = a.layout == RTI_COEF_PLANAR;
  switch (a.k) {
    case 6: return planar ? launch_stream_a<6, T, RTI_COEF_PLANAR>(a, pl) : launch_stream_a<6, T, RTI_COEF_PIXEL_MAJOR>(a, pl);
    case 9: return planar ? launch_stream_a<9, T, RTI_COEF_PLANAR>(a, pl) : launch_stream_a<9, T, RTI_COEF_PIXEL_MAJOR>(a, pl);
    case 16: return planar ? launch_stream_a<16, T, RTI_COEF_PLANAR>(a, pl) : launch_stream_a<16, T, RTI_COEF_PIXEL_MAJOR>(a, pl);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: k=%d", a.k);
  }
}

// VALU generations (k <= 9): one workgroup of W waves per CU (W <= 6), a ring per wave that holds a block
// (64 pixel rows) + 1 KiB; AUTO takes the most waves that fit (6 up to N = 100 for 4-byte values, 4 up to
// 150).  MB (blocks a wave parks per launch: MB·k VGPRs) = 24 for k = 6, 12 for k = 9; a channel's blocks
// are cut into the fewest launches whose waves park at most MB blocks each, split evenly (c3 4K×100: 4
// launches of 32 400 blocks, 21–22 per wave).
struct VPlan {
  int W = 0, ring = 0;
  size_t lds = 0;
};

VPlan vgen_plan(int k, int N, size_t es, int w_req) {
  if (k != 6 && k != 9) return VPlan();
  const int64_t need = (int64_t)64 * N * es + 1024;
  const size_t op = (size_t)((N + 3) & ~3) * k * sizeof(float);
  for (int W : {6, 5, 4, 3, 2, 1}) {
    if (w_req && W != w_req) continue;
    const int ring = (int)(((PM_LDS - op) / W) >> 10 << 10);
    if (ring < need) continue;
    VPlan pl;
    pl.W = W;
    pl.ring = ring;
    pl.lds = op + (size_t)W * ring;
    return pl;
  }
  return VPlan();
}

constexpr int vgen_mb(int k) { return k <= 6 ? 24 : 12; }

// launches of one channel, in units of U = 2^ulog blocks: every wave parks at most MB blocks (MB / U units)
struct VGens {
  int64_t nbc = 0, per = 0;  // blocks of the channel, blocks per launch (a multiple of U; the last takes the rest)
  int launches = 0;
};

VGens vgen_split(int64_t P, int k, int64_t GW, int g_req, int ulog) {
  VGens g;
  g.nbc = (P + 63) / 64;
  const int64_t nun = (g.nbc + (1 << ulog) - 1) >> ulog, cap = GW * (vgen_mb(k) >> ulog);
  int64_t L = (nun + cap - 1) / cap;
  if (g_req > L) L = g_req;  // more (smaller) generations: measurement
  g.per = ((nun + L - 1) / L) << ulog;
  g.launches = (int)((g.nbc + g.per - 1) / g.per);
  return g;
}

// units of whole KiB: U = 4 / gcd(N, 4) 64-pixel blocks of 4-byte values
inline int vgen_ulog(int N) { return N % 4 == 0 ? 0 : N % 2 == 0 ? 1 : 2; }

template <int K, typename T, int LAYOUT, int ALIGN>
int launch_vgen_t(const PmArgs& a, const VPlan& pl, int g_req, bool contig) {
  constexpr int MB = vgen_mb(K);
  auto kern = contig ? fit_pm_vgen<K, T, LAYOUT, ALIGN, MB, 0> : fit_pm_vgen<K, T, LAYOUT, ALIGN, MB, 1>;
  if (reserve_lds(reinterpret_cast<const void*>(kern), pl.lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared_pm: LDS attribute");
  const int64_t cus = device_cus();
  const int ulog = contig ? 0 : vgen_ulog(a.N);
  const VGens g = vgen_split(a.P, K, cus * pl.W, g_req, ulog);
  int launches = 0;
  for (int c = 0; c < a.C; ++c) {
    const T* Ic = static_cast<const T*>(a.I) + c * a.cs;
    float* oc = a.coef + c * a.ocs;
    for (int64_t b = 0; b < g.nbc; b += g.per) {
      const int64_t n = g.nbc - b < g.per ? g.nbc - b : g.per;
      const int64_t waves = contig ? n : (n + (1 << ulog) - 1) >> ulog;  // waves with work
      const int64_t wgs = (waves + pl.W - 1) / pl.W;
      const unsigned grid = (unsigned)(wgs < cus ? wgs : cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * pl.W), pl.lds, a.stream, a.pinv, a.N, Ic, a.P, oc, 64 * b, n,
                         pl.ring, ulog);
      ++launches;
    }
  }
  note_launches(launches);
  return RTI_OK;
}

template <int K, typename T>
int launch_vgen_k(const PmArgs& a, const VPlan& pl, int g_req, bool contig) {
  const bool planar = a.layout == RTI_COEF_PLANAR;
  if (a.N % 4 == 0)
    return planar ? launch_vgen_t<K, T, RTI_COEF_PLANAR, 4>(a, pl, g_req, contig)
                  : launch_vgen_t<K, T, RTI_COEF_PIXEL_MAJOR, 4>(a, pl, g_req, contig);
  if (a.N % 2 == 0)
    return planar ? launch_vgen_t<K, T, RTI_COEF_PLANAR, 2>(a, pl, g_req, contig)
                  : launch_vgen_t<K, T, RTI_COEF_PIXEL_MAJOR, 2>(a, pl, g_req, contig);
  return planar ? launch_vgen_t<K, T, RTI_COEF_PLANAR, 1>(a, pl, g_req, contig)
                : launch_vgen_t<K, T, RTI_COEF_PIXEL_MAJOR, 1>(a, pl, g_req, contig);
}

template <typename T>
int launch_vgen(const PmArgs& a, const VPlan& pl, int g_req, bool contig) {
  return a.k == 6 ? launch_vgen_k<6, T>(a, pl, g_req, contig) : launch_vgen_k<9, T>(a, pl, g_req, contig);
}

// DIRECT plan: NS 16-light steps (a bucket >= ceil(N / 16): the extra steps' loads are out of range, no bytes),
// D groups of loads in flight per wave
constexpr int pm_direct_ns(int N) {
  return N <= 32 ? 2 : N <= 64 ? 4 : N <= 112 ? 7 : N <= 128 ? 8 : N <= 208 ? 13 : N <= 256 ? 16 : 0;
}
constexpr int pm_direct_depth(int ns) { return ns <= 4 ? 4 : ns <= 8 ? 3 : 2; }
constexpr int PM_DIRECT_WPC = 8;  // waves per CU (AUTO)

struct DirectOpts {
  int wpc = PM_DIRECT_WPC;  // waves per CU
  int gens = 1;             // launch generations (consecutive launches over equal run ranges)
  bool nts = false;         // non-temporal burst stores (pixel-major)
};

template <int K, typename T, int LAYOUT, int NS>
int launch_direct_t(const PmArgs& a, const DirectOpts& o) {
  constexpr int D = pm_direct_depth(NS), RPX = 16 * pm_direct_run<K, NS>();
  const int64_t ngrp = (a.P + 15) / 16, nrun = (a.P + RPX - 1) / RPX, tr = nrun * a.C;
  // the kernel's run and group cursors are 32-bit (first = r0 + gw, runs < tr + GW)
  if (ngrp >= ((int64_t)1 << 31) - 4096 || tr >= ((int64_t)1 << 31) - 65536 || a.P * K * 4 >= ((int64_t)1 << 31))
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: P too large");
  auto kern = fit_pm_direct<K, T, LAYOUT, NS, D>;
  if constexpr (LAYOUT == RTI_COEF_PIXEL_MAJOR)
    if (o.nts) kern = fit_pm_direct<K, T, LAYOUT, NS, D, true>;
  const size_t lds = (size_t)4 * RPX * K * sizeof(float);  // 4 waves per workgroup
  if (reserve_lds(reinterpret_cast<const void*>(kern), lds) != hipSuccess)
    return fail(RTI_ERR_HIP, "rti_fit_shared_pm: LDS attribute");
  const int64_t per = (tr + o.gens - 1) / o.gens;
  int launches = 0;
  for (int64_t r0 = 0; r0 < tr; r0 += per) {
    const int64_t n = tr - r0 < per ? tr - r0 : per;
    const int64_t wgs = (n + 3) / 4, cap = device_cus() * (int64_t)o.wpc / 4;
    const unsigned grid = (unsigned)(wgs < cap ? wgs : (cap > 0 ? cap : 1));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, a.stream, a.pinv, a.N, static_cast<const T*>(a.I), a.P,
                       a.cs, a.coef, a.ocs, (int)ngrp, (int)nrun, (int)r0, (int)n);
    note_launches(++launches);
  }
  return RTI_OK;
}

template <int K, typename T, int LAYOUT>
int launch_direct_n(const PmArgs& a, const DirectOpts& o) {
  switch (pm_direct_ns(a.N)) {
    case 2: return launch_direct_t<K, T, LAYOUT, 2>(a, o);
    case 4: return launch_direct_t<K, T, LAYOUT, 4>(a, o);
    case 7: return launch_direct_t<K, T, LAYOUT, 7>(a, o);
    case 8: return launch_direct_t<K, T, LAYOUT, 8>(a, o);
    case 13: return launch_direct_t<K, T, LAYOUT, 13>(a, o);
    default: return launch_direct_t<K, T, LAYOUT, 16>(a, o);
  }
}

template <typename T>
int launch_direct(const PmArgs& a, const DirectOpts& o) {
  const bool planar = a.layout == RTI_COEF_PLANAR;
  switch (a.k) {
    case 6: return planar ? launch_direct_n<6, T, RTI_COEF_PLANAR>(a, o) : launch_direct_n<6, T, RTI_COEF_PIXEL_MAJOR>(a, o);
    case 9: return planar ? launch_direct_n<9, T, RTI_COEF_PLANAR>(a, o) : launch_direct_n<9, T, RTI_COEF_PIXEL_MAJOR>(a, o);
    case 16: return planar ? launch_direct_n<16, T, RTI_COEF_PLANAR>(a, o) : launch_direct_n<16, T, RTI_COEF_PIXEL_MAJOR>(a, o);
    default: return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: k=%d", a.k);
  }
}

template <int K, typename T>
void launch_lane_t(const PmArgs& a) {
  const dim3 grid(grid_1d(a.P, 256), a.C);
  if (a.layout == RTI_COEF_PLANAR)
    hipLaunchKernelGGL((fit_pm_lane<K, T, RTI_COEF_PLANAR>), grid, dim3(256), 0, a.stream, a.pinv, a.k, a.N,
                       static_cast<const T*>(a.I), a.P, a.ps, a.cs, a.coef, a.ocs);
  else
    hipLaunchKernelGGL((fit_pm_lane<K, T, RTI_COEF_PIXEL_MAJOR>), grid, dim3(256), 0, a.stream, a.pinv, a.k, a.N,
                       static_cast<const T*>(a.I), a.P, a.ps, a.cs, a.coef, a.ocs);
}

template <typename T>
void launch_lane(const PmArgs& a) {
  if (a.k <= 6)
    launch_lane_t<6, T>(a);
  else if (a.k <= 9)
    launch_lane_t<9, T>(a);
  else
    launch_lane_t<16, T>(a);
}

}  // namespace
}  // namespace rti

using namespace rti;

// the shapes the DMA / MFMA kernels take: F32 / I32, pixel stride N, 16-byte aligned pixel runs and channels
// (P·N and the channel stride multiples of 4); `lim32`: the forms whose coefficient offsets are 32-bit
// (every form but the VALU generations) also need P·k·4 < 2^31
static bool pm_dma_shape(int k, int N, int in_dtype, int64_t P, int C, int64_t ps, int64_t cs, bool lim32) {
  if (k != 6 && k != 9 && k != 16) return false;
  if (in_dtype != RTI_F32 && in_dtype != RTI_I32) return false;
  return ps == N && (P * N) % 4 == 0 && (C <= 1 || cs % 4 == 0) && (!lim32 || P * (int64_t)k * 4 < ((int64_t)1 << 31));
}

// the kernel-selection bits rti_fit_shared_pm accepts: the selector (AUTO / VALU / MFMA / TILE) and the tuning
// fields of include/rti.h that it documents; anything else is RTI_ERR_BAD_ARG
static constexpr int PM_FLAGS = RTI_KERNEL_STAGE | RTI_KERNEL_NT_STORE | RTI_KERNEL_ROTATE |
                                (0xF << RTI_KERNEL_CHUNKS_SHIFT) | (0xF << RTI_KERNEL_TILE_WAVES_SHIFT);

static bool pm_flags_ok(int kernel) {
  const int sel = kernel & 0xff;
  return sel <= RTI_KERNEL_TILE && (kernel & ~0xff & ~PM_FLAGS) == 0;
}

// the form AUTO / the selector picks (0: one lane per pixel); `size` and `w` as rti_fit_shared_pm_plan reports them
static int pm_choose(int k, int N, int in_dtype, int64_t P, int C, int64_t ps, int64_t cs, int kernel, int* size,
                     int* w) {
  const int sel = kernel & 0xff;
  const int w_req = (kernel >> RTI_KERNEL_TILE_WAVES_SHIFT) & 0xF, c_req = (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF;
  const bool stage = (kernel & RTI_KERNEL_STAGE) != 0;
  const size_t es = 4;
  if (sel == RTI_KERNEL_VALU || !pm_dma_shape(k, N, in_dtype, P, C, ps, cs, false)) return 0;
  if (sel == RTI_KERNEL_AUTO && !stage) {
    const VPlan vp = vgen_plan(k, N, es, w_req);
    if (vp.W) {
      *size = vp.ring >> 10;
      *w = vp.W;
      return RTI_PM_VALU_STREAM;
    }
  }
  if (!pm_dma_shape(k, N, in_dtype, P, C, ps, cs, true)) return 0;
  if (sel == RTI_KERNEL_AUTO && N % 4 == 0 && pm_direct_ns(N)) {
    *size = pm_direct_ns(N);
    *w = w_req ? w_req : PM_DIRECT_WPC;
    return RTI_PM_DIRECT;
  }
  if (sel != RTI_KERNEL_TILE) {
    const StreamPlan sp = stream_plan(N, es, w_req, c_req);
    if (sp.W) {
      *size = sp.ring >> 10;
      *w = sp.W;
      return RTI_PM_MFMA_STREAM;
    }
  }
  const PmPlan pl = pm_plan(N, es, sel == RTI_KERNEL_TILE ? c_req : 0, w_req);
  if (!pl.G) return 0;
  *size = 16 * pl.G;
  *w = pl.W;
  return RTI_PM_BLOCK;
}

extern "C" int rti_fit_shared_pm_plan(int k, int N, int in_dtype, int64_t P, int C, int64_t pixel_stride,
                                      int64_t channel_stride, int kernel) {
  if (!pm_flags_ok(kernel) || N <= 0 || P <= 0 || C <= 0) return 0;
  const int64_t ps = pixel_stride ? pixel_stride : N;
  const int64_t cs = channel_stride ? channel_stride : P * ps;
  int size = 0, w = 0;
  const int form = pm_choose(k, N, in_dtype, P, C, ps, cs, kernel, &size, &w);
  return form ? form * 100000000 + size * 1000 + w : 0;
}

extern "C" int rti_fit_shared_pm(const float* pinv, int k, int N, const void* I, int in_dtype, int64_t P, int C,
                                 int64_t pixel_stride, int64_t channel_stride, float* coef, int coef_layout,
                                 int64_t coef_channel_stride, int kernel, rti_stream_t stream) {
  if (!pm_flags_ok(kernel)) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: unknown kernel bits 0x%x", kernel);
  if (!pinv || !I || !coef) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: null pointer");
  if (N <= 0 || P <= 0 || C <= 0 || C > 65535) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: bad N/P/C");
  if (k < 1 || k > 16) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: k=%d outside 1..16", k);
  if (N < k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: N=%d < k=%d", N, k);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: input dtype %d", in_dtype);
  if (coef_layout != RTI_COEF_PIXEL_MAJOR && coef_layout != RTI_COEF_PLANAR)
    return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: coef layout %d", coef_layout);
  PmArgs a;
  a.pinv = pinv;
  a.k = k;
  a.N = N;
  a.I = I;
  a.P = P;
  a.C = C;
  a.ps = pixel_stride ? pixel_stride : N;
  a.cs = channel_stride ? channel_stride : P * a.ps;
  a.coef = coef;
  a.layout = coef_layout;
  a.ocs = coef_channel_stride ? coef_channel_stride : P * k;
  a.stream = (hipStream_t)stream;
  if (a.ps < N) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: pixel_stride < N");
  if (C > 1 && a.cs < P * a.ps) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: channel_stride");
  if (C > 1 && a.ocs < P * k) return fail(RTI_ERR_BAD_ARG, "rti_fit_shared_pm: coef_channel_stride");
  note_launches(1);
  const int sel = kernel & 0xff;
  const int w_req = (kernel >> RTI_KERNEL_TILE_WAVES_SHIFT) & 0xF, c_req = (kernel >> RTI_KERNEL_CHUNKS_SHIFT) & 0xF;
  int size = 0, w = 0;
  int form = pm_choose(k, N, in_dtype, P, C, a.ps, a.cs, kernel, &size, &w);
  // the VALU generations store per lane (float2 pairs for even k, pixel-major): 8-byte aligned channels; the
  // other forms' buffer stores and LDS bursts want 16-byte aligned coefficient rows
  const bool coef_ok = form == RTI_PM_VALU_STREAM ? aligned_to(coef, 8) && a.ocs % 2 == 0
                                                  : aligned_to(coef, 16) && a.ocs % 4 == 0;
  if (!(aligned_to(I, 16) && coef_ok)) form = 0;
  const bool i32 = in_dtype == RTI_I32;
  int st = RTI_OK;
  switch (form) {
    case RTI_PM_VALU_STREAM: {  // AUTO, k <= 9 (c3: 0.55 ms, §4.1f)
      const VPlan vp = vgen_plan(k, N, 4, w_req);
      const bool contig = (kernel & RTI_KERNEL_ROTATE) != 0;  // each wave one contiguous run (A/B)
      st = i32 ? launch_vgen<int32_t>(a, vp, c_req, contig) : launch_vgen<float>(a, vp, c_req, contig);
      break;
    }
    case RTI_PM_DIRECT: {  // AUTO k = 16, AUTO | STAGE: straight to registers.  Tuning flags:
      DirectOpts o;        // TILE_WAVES(w) waves per CU, CHUNKS(n) launch generations, NT_STORE non-temporal bursts
      if (w_req) o.wpc = w_req;
      if (c_req) o.gens = c_req;
      // AUTO k = 16: the bursts non-temporal (whole 1-KiB lines; c4 3.677–3.696 against 3.731–3.745 ms plain,
      // profiles/r05h_pm_sweep_c4.log, r05g); the MFMA stream ran 3.49–3.71 ms interleaved with other kernels
      // but 4.13 ms back to back in bench.py (profiles/r05i_*), so it stays RTI_KERNEL_MFMA
      o.nts = (kernel & RTI_KERNEL_NT_STORE) != 0 || (k == 16 && sel == RTI_KERNEL_AUTO && !(kernel & RTI_KERNEL_STAGE));
      st = i32 ? launch_direct<int32_t>(a, o) : launch_direct<float>(a, o);
      break;
    }
    case RTI_PM_MFMA_STREAM: {  // RTI_KERNEL_MFMA: the MFMA stream through the LDS ring
      StreamPlan sp = stream_plan(N, 4, w_req, c_req);
      sp.contig = (kernel & RTI_KERNEL_ROTATE) != 0;  // each wave one contiguous run of units
      sp.nts = (kernel & RTI_KERNEL_NT_STORE) != 0;
      st = i32 ? launch_stream<int32_t>(a, sp) : launch_stream<float>(a, sp);
      break;
    }
    case RTI_PM_BLOCK: {  // RTI_KERNEL_TILE (or N too small for a ring): the double-buffered block form
      const PmPlan pl = pm_plan(N, 4, sel == RTI_KERNEL_TILE ? c_req : 0, w_req);
      st = i32 ? launch_dma<int32_t>(a, pl) : launch_dma<float>(a, pl);
      break;
    }
    default:
      if (sel == RTI_KERNEL_MFMA || sel == RTI_KERNEL_TILE)
        return fail(RTI_ERR_UNSUPPORTED, "rti_fit_shared_pm: the DMA/MFMA kernels do not take this shape");
      switch (in_dtype) {
        case RTI_F32: launch_lane<float>(a); break;
        case RTI_I32: launch_lane<int32_t>(a); break;
        default: launch_lane<uint8_t>(a); break;
      }
  }
  return st != RTI_OK ? st : check_launch("rti_fit_shared_pm");
}
