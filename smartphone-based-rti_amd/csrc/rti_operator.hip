// rti_operator.hip -- apply a light operator to the intensity stack on gfx950 (MFMA).
//
//     out[c][e][p] = Σ_n opT[n][e] · I[c][n][p]
//
// The operator maps a pixel's N intensities to E outputs.  With the linear-RBF
// operator M = Φ(q) A⁻¹ (rti_rbf_operator) evaluated on the reference's 100×100
// grid, one launch is the reference's default interpolation (SciPy Rbf
// 'linear', analysis.py:249-260 via interpolate_intensities :361-363) plus the
// prepare_images_data layout (analysis.py:375-411): out[e][p] with e = ly·G + lx.
// With M = B(q)·pinv it is the PTM/HSH fit fused with its grid evaluation.
//
// Shape: a GEMM with a short reduction (K = N lights, ≤ 256 in every BASELINE config) and a huge output
// (E·P), so it is MFMA- or store-bound, never load-bound.  A workgroup owns a
// 64-pixel tile: it stages the tile's N×64 intensities in LDS once (read from
// HBM exactly once over the whole launch) and sweeps every operator row over
// them.  Each wave computes 64 rows × 64 pixels per sweep step with
// v_mfma_f32_16x16x4_f32: the A operand is a 16-byte load of 4 consecutive
// operator rows (rows 4q+rb of the wave's 64, rb = MFMA row block), the B
// operand one ds_read_b128 of 4 adjacent pixels (pixel 4q+c for accumulator c),
// i.e. 16 MFMAs per pair of 16-byte loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "rti_convert.h"
#include "rti_internal.h"

namespace rti {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int TILE_P = 64;    // pixels per workgroup tile
constexpr int ROWS_WG = 256;  // operator rows per workgroup sweep step (4 waves × 64)
constexpr int KCHUNK = 512;   // lights staged at once (128 KiB of LDS); N above is swept in chunks

template <typename T, typename TO, bool VEC>
__global__ void __launch_bounds__(256)
apply_op_mfma(const float* __restrict__ opT, int E, int N, int64_t ostride, const T* __restrict__ I, int64_t P,
              int64_t lstride, int64_t cstride, TO* __restrict__ out, int64_t orow, int64_t ocs) {
  extern __shared__ __attribute__((aligned(16))) float sB[];  // [min(Npad, KCHUNK)][TILE_P]
  const int Npad = (N + 3) & ~3;
  const int64_t p0 = (int64_t)blockIdx.x * TILE_P;
  const T* __restrict__ src = I + (int64_t)blockIdx.z * cstride;

  // stage lights [c0, c0 + KCHUNK) of the tile's intensities (zero beyond N and beyond P)
  auto stage = [&](int c0) {
    const int cn = min(Npad - c0, KCHUNK);
    for (int idx = threadIdx.x; idx < cn * (TILE_P / 4); idx += 256) {
      const int nl = idx / (TILE_P / 4), q4 = idx % (TILE_P / 4), n = c0 + nl;
      const int64_t px = p0 + 4 * q4;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (n < N) {
        const T* s = src + (int64_t)n * lstride + px;
        if (VEC && px + 3 < P) {
          typedef T vec_t __attribute__((ext_vector_type(4)));
          const vec_t t = __builtin_nontemporal_load(reinterpret_cast<const vec_t*>(s));
          v = floatx4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (px + c < P) v[c] = (float)s[c];
        }
      }
      *reinterpret_cast<floatx4*>(sB + nl * TILE_P + 4 * q4) = v;
    }
  };
  // N <= KCHUNK (every BASELINE config): the tile is staged once and read from HBM exactly once.
  // Above, each row tile restages the light chunks (the intensities are re-read E/256 times, from L2).
  const bool once = Npad <= KCHUNK;
  if (once) stage(0);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane & 15, r = lane >> 4;
  const int ntiles = (E + ROWS_WG - 1) / ROWS_WG;
  TO* __restrict__ dst = out + (int64_t)blockIdx.z * ocs;
  for (int rt = blockIdx.y; rt < ntiles; rt += gridDim.y) {
    const int row0 = rt * ROWS_WG + wave * 64;
    if (once && row0 >= E) continue;  // wave-uniform (the chunked sweep keeps every wave for its barriers)
    const int rowq = row0 + 4 * q;
    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < Npad; c0 += KCHUNK) {
      if (!once) {
        __syncthreads();  // the previous chunk's readers are done
        stage(c0);
        __syncthreads();
      }
      if (row0 >= E) continue;
      const int cend = min(Npad, c0 + KCHUNK);
      for (int n0 = c0; n0 < cend; n0 += 4) {
        const int n = n0 + r;
        floatx4 a = {0.f, 0.f, 0.f, 0.f};
        if (n < N) {
          const float* op = opT + (int64_t)n * ostride + rowq;
          if (VEC && rowq + 3 < E) {
            a = *reinterpret_cast<const floatx4*>(op);
          } else {
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
              if (rowq + rb < E) a[rb] = op[rb];
          }
        }
        const floatx4 b = *reinterpret_cast<const floatx4*>(sB + (n - c0) * TILE_P + 4 * q);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb], b[c], acc[rb][c], 0, 0, 0);
      }
    }
    if (row0 >= E) continue;
    // acc[rb][c][rr] = out row (row0 + 16r + 4rr + rb), pixel (p0 + 4q + c)
    const int64_t px = p0 + 4 * q;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = row0 + 16 * r + 4 * rr + rb;
        if (row >= E) continue;
        TO* o = dst + (int64_t)row * orow + px;
        if (VEC && px + 3 < P) {
          typedef TO ovec_t __attribute__((ext_vector_type(4)));
          ovec_t v;
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = cvt_out<TO>(acc[rb][c][rr]);
          *reinterpret_cast<ovec_t*>(o) = v;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (px + c < P) o[c] = cvt_out<TO>(acc[rb][c][rr]);
        }
      }
  }
}

// ---- split-fp16 MFMA variant (v_mfma_f32_32x32x16_f16) ----------------------------------
// The fp32 operator is applied as two fp16 GEMMs: M·s = M_hi + M_lo (host split in fp64,
// s a power of two putting max|M·s| near 2^15), so M_hi + M_lo carries 22 significant bits.
// A workgroup stages its 128-pixel tile as fp16 x·t (t a per-tile power of two keeping
// |x·t| < 2^15; t = 1 for 8-bit data) in LDS, pixel-major with lights contiguous (the B
// operand's k-run); if any staged value is not exact in fp16 (x·t − hi ≠ 0, e.g. fractional
// fp32 input) the tile also stages the remainders and adds M_hi·I_lo.  Accumulation is fp32
// in the MFMA; the result is scaled back by 1/(s·t) (exact).  Integer 8-bit intensities —
// the reference's V channel — are exact, so it costs two f16 MFMAs (16× the fp32 MFMA rate
// each) per 32×32×16 block instead of sixteen v_mfma_f32_16x16x4_f32.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int TP16 = 128;  // pixels per workgroup tile (4 blocks of 32)
constexpr int KSMAX = 8;   // k-steps (16 lights each) the pipelined sweep holds in registers: N <= 128

// NTS: non-temporal table stores (AUTO; false = plain stores, a measurement variant: RTI_OP_PLAIN_STORES=1);
// NBLK: 32-pixel blocks per workgroup tile (4: 128 pixels; r04 measured 8 = 256 pixels at one wave per SIMD,
// 1.47 against 1.31 ms on c7, profiles/r04v_c7_tile_sweep.log)
template <typename T, typename TO, bool VEC, bool NTS = true, int NBLK = 4>
__global__ void __launch_bounds__(256)
apply_op_f16s(const _Float16* ohi, const _Float16* olo, int Kp, float inv_s, int E, int N,
              const T* __restrict__ I, int64_t P, int64_t lstride, int64_t cstride, TO* __restrict__ out,
              int64_t orow, int64_t ocs, int xcd_order) {
  constexpr bool EXACT = std::is_same<T, uint8_t>::value;  // 0..255: exact in fp16, t = 1
  constexpr int TP = 32 * NBLK;  // pixels per workgroup tile
  extern __shared__ __attribute__((aligned(16))) _Float16 sI[];  // [2][TP][KPITCH]
  __shared__ float s_red[4];
  const int KPITCH = Kp + 8;  // 16-B pad between pixel rows
  _Float16* sIlo = sI + TP * KPITCH;
  // xcd_order (measurement, RTI_OP_XCD=1): workgroups are dispatched round-robin over the 8 XCDs, so workgroup b
  // runs on XCD b % 8; this order gives each XCD one contiguous run of pixel tiles (its table writes stay in one
  // run of every output row) instead of every eighth tile
  int64_t tile = blockIdx.x;
  if (xcd_order) {
    const int64_t g = gridDim.x, per = (g + 7) / 8, x = blockIdx.x % 8, i = blockIdx.x / 8;
    const int64_t full = g - 8 * (per - 1);  // XCDs holding `per` tiles (the others per - 1)
    tile = x < full ? x * per + i : full * per + (x - full) * (per - 1) + i;
  }
  const int64_t p0 = tile * TP;
  const T* __restrict__ src = I + (int64_t)blockIdx.z * cstride;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  auto load4 = [&](int n, int q4, float (&v)[4]) {
    const int64_t px = p0 + 4 * q4;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = 0.f;
    if (n >= N) return;
    const T* sp = src + (int64_t)n * lstride + px;
    if (VEC && px + 3 < P) {
      typedef T vec_t __attribute__((ext_vector_type(4)));
      const vec_t t = __builtin_nontemporal_load(reinterpret_cast<const vec_t*>(sp));
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = (float)t[c];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (px + c < P) v[c] = (float)sp[c];
    }
  };

  // tile scale t = 2^-e with max|x|·t < 2^15 (non-finite values pass through as inf/NaN)
  float t = 1.f;
  if constexpr (!EXACT) {
    float m = 0.f;
    for (int idx = threadIdx.x; idx < N * (TP / 4); idx += 256) {
      float v[4];
      load4(idx / (TP / 4), idx % (TP / 4), v);
#pragma unroll
      for (int c = 0; c < 4; ++c) m = fmaxf(m, fabsf(v[c]) < INFINITY ? fabsf(v[c]) : 0.f);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) s_red[wave] = m;
    __syncthreads();
    m = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
    int e = 0;
    if (m >= 32768.f) {
      frexpf(m, &e);  // m < 2^e
      e -= 15;
    }
    t = ldexpf(1.f, -e);
  }
  int need_lo = 0;
  for (int idx = threadIdx.x; idx < Kp * (TP / 4); idx += 256) {
    const int n = idx / (TP / 4), q4 = idx % (TP / 4);
    float v[4];
    load4(n, q4, v);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float x = v[c] * t;
      const _Float16 hi = (_Float16)x;
      sI[(4 * q4 + c) * KPITCH + n] = hi;
      if constexpr (!EXACT) {
        const _Float16 lo = (_Float16)(x - (float)hi);
        sIlo[(4 * q4 + c) * KPITCH + n] = lo;
        need_lo |= (float)lo != 0.f;
      }
    }
  }
  if constexpr (!EXACT) need_lo = __syncthreads_or(need_lo);
  else __syncthreads();
  const float oscale = inv_s / t;

  const int r = lane & 31, h = lane >> 5;
  const int nrb = (E + 31) / 32;
  TO* __restrict__ dst = out + (int64_t)blockIdx.z * ocs;
  const int ksteps = Kp / 16;
  const int rb0 = blockIdx.y * 4 + wave, rbstep = gridDim.y * 4;

  // A operand of one 32-row block: lane (r, h) holds operator row rb*32 + r, k-offset 8h of
  // every 16-wide k-step, hi and lo halves.  Branch-free: k-steps past Kp re-read the last one
  // (their MFMAs are skipped) and rows past E read row 0 (never stored).
  auto load_a = [&](int rb, half8 (&ah)[KSMAX], half8 (&al)[KSMAX]) {
    const int arow = rb * 32 + r;
    const int64_t rowoff = (int64_t)(arow < E ? arow : 0) * Kp + 8 * h;
#pragma unroll
    for (int s = 0; s < KSMAX; ++s) {
      const int ss = s < ksteps ? s : ksteps - 1;
      ah[s] = *reinterpret_cast<const half8*>(ohi + rowoff + 16 * ss);
      al[s] = *reinterpret_cast<const half8*>(olo + rowoff + 16 * ss);
    }
  };
  auto mfma_block = [&](floatx16 (&acc)[NBLK], const half8& a_hi, const half8& a_lo, int k0) {
#pragma unroll
    for (int b = 0; b < NBLK; ++b) {
      const half8 bh = *reinterpret_cast<const half8*>(sI + (32 * b + r) * KPITCH + k0 + 8 * h);
      acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_hi, bh, acc[b], 0, 0, 0);
      acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_lo, bh, acc[b], 0, 0, 0);
    }
    if (!EXACT && need_lo) {
#pragma unroll
      for (int b = 0; b < NBLK; ++b) {
        const half8 bl = *reinterpret_cast<const half8*>(sIlo + (32 * b + r) * KPITCH + k0 + 8 * h);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_hi, bl, acc[b], 0, 0, 0);
      }
    }
  };
  // D: column (pixel) = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h
  // reg outer, pixel block inner: consecutive stores continue the same output row
  // (4 × 128 B = 512 B contiguous per row), which keeps HBM write pages open.
  // Non-temporal: the E×P output streams past the operator, which stays in L2.
  auto store_block = [&](const floatx16 (&acc)[NBLK], int rb, bool guard) {
    // lane base: row rb*32 + 4h, pixel p0 + r; the 16 row offsets are wave-uniform multiples of orow
    TO* __restrict__ lb = dst + (int64_t)(rb * 32 + 4 * h) * orow + p0 + r;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int dr = (reg & 3) + 8 * (reg >> 2);
      const int row = rb * 32 + dr + 4 * h;
      TO* __restrict__ rp = lb + (int64_t)dr * orow;
#pragma unroll
      for (int b = 0; b < NBLK; ++b) {
        if (!guard || (row < E && p0 + 32 * b + r < P)) {
          if constexpr (NTS)
            __builtin_nontemporal_store(cvt_out<TO>(acc[b][reg] * oscale), rp + 32 * b);
          else
            rp[32 * b] = cvt_out<TO>(acc[b][reg] * oscale);
        }
      }
    }
  };
  auto zero = [](floatx16 (&acc)[NBLK]) {
#pragma unroll
    for (int b = 0; b < NBLK; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[b][i] = 0.f;
  };

  int rb = rb0;
  const int nfull = E / 32;  // row blocks with all 32 rows in range
  if (ksteps <= KSMAX && p0 + TP <= P && rb < nfull) {
    // Software-pipelined sweep over whole row blocks of a whole pixel tile.  The next block's
    // operator rows are loaded BEFORE this block's 64 stores are issued: CDNA's single vmcnt
    // counter retires loads and stores in order, so a load issued after the stores cannot be
    // waited for without also waiting for every one of them -- which serialised the MFMAs
    // behind the table writes (c7 1.63 ms against a 0.99 ms store-only floor,
    // tools/sweep_store.py).  Loads and stores here are branch-free straight-line code, and the
    // first block is peeled, so the loop header sees the same outstanding-op pattern (16 loads
    // then 64 stores) from both edges and the compiler's waits stop at the loads.
    half8 ah[KSMAX], al[KSMAX];
    floatx16 acc[NBLK];
    load_a(rb, ah, al);
    zero(acc);
#pragma unroll
    for (int s = 0; s < KSMAX; ++s)
      if (s < ksteps) mfma_block(acc, ah[s], al[s], 16 * s);
    int nxt = rb + rbstep < nfull ? rb + rbstep : rb;
    load_a(nxt, ah, al);
    __asm__ volatile("" ::: "memory");  // keep every load ahead of the stores (IR and
    __builtin_amdgcn_sched_barrier(0);  // machine scheduler)
    store_block(acc, rb, false);
    for (rb += rbstep; rb < nfull; rb += rbstep) {
      zero(acc);
#pragma unroll
      for (int s = 0; s < KSMAX; ++s)
        if (s < ksteps) mfma_block(acc, ah[s], al[s], 16 * s);
      nxt = rb + rbstep < nfull ? rb + rbstep : rb;
      load_a(nxt, ah, al);
      __asm__ volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      store_block(acc, rb, false);
    }
  }
  // the rest (partial tile or row block, or N > 16·KSMAX): one block at a time, guarded stores
  for (; rb < nrb; rb += rbstep) {
    const int arow = rb * 32 + r;
    const bool aok = arow < E;
    const _Float16* ah = ohi + (int64_t)(aok ? arow : 0) * Kp + 8 * h;
    const _Float16* al = olo + (int64_t)(aok ? arow : 0) * Kp + 8 * h;
    floatx16 acc[NBLK];
    zero(acc);
    for (int k0 = 0; k0 < Kp; k0 += 16) {
      half8 a_hi = *reinterpret_cast<const half8*>(ah + k0);
      half8 a_lo = *reinterpret_cast<const half8*>(al + k0);
      if (!aok) {
        a_hi = half8{};
        a_lo = half8{};
      }
      mfma_block(acc, a_hi, a_lo, k0);
    }
    store_block(acc, rb, true);
  }
}

template <typename T, typename TO>
int launch_f16(const _Float16* hi, const _Float16* lo, int Kp, float inv_s, int E, int N, const void* I, int64_t P,
               int C, int64_t ls, int64_t cs, void* out, int64_t orow, int64_t ocs, bool vec, hipStream_t s) {
  constexpr bool EXACT = std::is_same<T, uint8_t>::value;
  const int tp = TP16;
  const size_t lds = (size_t)(EXACT ? 1 : 2) * tp * (Kp + 8) * sizeof(_Float16);
  const unsigned gx = (unsigned)((P + tp - 1) / tp);
  const int nwb = (E + 127) / 128;  // 4 waves × 32-row blocks per sweep step
  // E-split: one sweep over all row blocks per pixel tile once the tiles alone give two workgroups per CU
  // (c7 400²×100 → 10⁴ tables, 1250 tiles: 1.302 ms against 1.424 ms split in 2 and 1.549 in 3,
  // profiles/r03_c7_gy_sweep.log — each split re-stages the tile and halves the rows its prologue pays for);
  // smaller images split the rows until the grid reaches that
  const int want = 2 * device_cus();
  unsigned gy = (unsigned)std::max(1, std::min(nwb, (int)((want + gx - 1) / gx)));
  if (const char* e = getenv("RTI_OP_GY")) gy = (unsigned)std::max(1, std::min(nwb, atoi(e)));  // measurement
  dim3 grid(gx, gy, C);
  const char* ps = getenv("RTI_OP_PLAIN_STORES");  // measurement
  auto k = vec ? apply_op_f16s<T, TO, true> : apply_op_f16s<T, TO, false>;
  if (vec && ps && atoi(ps)) k = apply_op_f16s<T, TO, true, false>;
  if (lds > 65536 &&
      reserve_lds(reinterpret_cast<const void*>(k), lds) !=
          hipSuccess)
    return fail(RTI_ERR_HIP, "rti_apply_operator_f16: cannot reserve %zu B of LDS", lds);
  const char* xo = getenv("RTI_OP_XCD");  // measurement
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, hi, lo, Kp, inv_s, E, N, static_cast<const T*>(I), P, ls, cs,
                     static_cast<TO*>(out), orow, ocs, xo ? atoi(xo) : 0);
  return check_launch("rti_apply_operator_f16");
}

template <typename T>
int launch_f16_out(int odt, const _Float16* hi, const _Float16* lo, int Kp, float inv_s, int E, int N, const void* I,
                   int64_t P, int C, int64_t ls, int64_t cs, void* out, int64_t orow, int64_t ocs, bool vec,
                   hipStream_t s) {
  switch (odt) {
    case RTI_F32: return launch_f16<T, float>(hi, lo, Kp, inv_s, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_F64: return launch_f16<T, double>(hi, lo, Kp, inv_s, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_I32: return launch_f16<T, int32_t>(hi, lo, Kp, inv_s, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
    default: return launch_f16<T, uint8_t>(hi, lo, Kp, inv_s, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
  }
}

template <typename T, typename TO>
int launch(const float* opT, int E, int N, int64_t os, const void* I, int64_t P, int C, int64_t ls, int64_t cs,
           void* out, int64_t orow, int64_t ocs, bool vec, hipStream_t s) {
  const int Npad = (N + 3) & ~3;
  const size_t lds = (size_t)std::min(Npad, KCHUNK) * TILE_P * sizeof(float);
  const unsigned gx = (unsigned)((P + TILE_P - 1) / TILE_P);
  const int ntiles = (E + ROWS_WG - 1) / ROWS_WG;
  // enough workgroups to fill 256 CUs; with many pixel tiles each workgroup sweeps every row
  const unsigned gy = (unsigned)std::max(1, std::min(ntiles, (int)((2048 + gx - 1) / gx)));
  dim3 grid(gx, gy, C);
  if (lds > 65536) {
    (void)reserve_lds(reinterpret_cast<const void*>(apply_op_mfma<T, TO, true>), lds);
    (void)reserve_lds(reinterpret_cast<const void*>(apply_op_mfma<T, TO, false>), lds);
  }
  if (vec)
    hipLaunchKernelGGL((apply_op_mfma<T, TO, true>), grid, dim3(256), lds, s, opT, E, N, os, static_cast<const T*>(I),
                       P, ls, cs, static_cast<TO*>(out), orow, ocs);
  else
    hipLaunchKernelGGL((apply_op_mfma<T, TO, false>), grid, dim3(256), lds, s, opT, E, N, os, static_cast<const T*>(I),
                       P, ls, cs, static_cast<TO*>(out), orow, ocs);
  return check_launch("rti_apply_operator");
}

template <typename T>
int launch_out(int odt, const float* opT, int E, int N, int64_t os, const void* I, int64_t P, int C, int64_t ls,
               int64_t cs, void* out, int64_t orow, int64_t ocs, bool vec, hipStream_t s) {
  switch (odt) {
    case RTI_F32: return launch<T, float>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_F64: return launch<T, double>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_I32: return launch<T, int32_t>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    default: return launch<T, uint8_t>(opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
  }
}

size_t esize(int dt) { return dt == RTI_U8 ? 1 : dt == RTI_F64 ? 8 : 4; }

}  // namespace
}  // namespace rti

using namespace rti;

extern "C" int rti_apply_operator(const float* opT, int E, int N, int64_t op_stride, const void* I, int in_dtype,
                                  int64_t P, int C, int64_t light_stride, int64_t channel_stride, void* out,
                                  int out_dtype, int64_t out_row_stride, int64_t out_channel_stride,
                                  rti_stream_t stream) {
  if (!opT || !I || !out) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator: null pointer");
  if (E <= 0 || N <= 0 || P <= 0 || C <= 0 || C > 65535)
    return fail(RTI_ERR_BAD_ARG, "rti_apply_operator: bad E/N/P/C");
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator: input dtype %d", in_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator: out dtype %d", out_dtype);
  const int64_t os = op_stride ? op_stride : E;
  const int64_t ls = light_stride ? light_stride : P;
  const int64_t cs = channel_stride ? channel_stride : (int64_t)N * ls;
  const int64_t orow = out_row_stride ? out_row_stride : P;
  const int64_t ocs = out_channel_stride ? out_channel_stride : (int64_t)E * orow;
  if (os < E || ls < P || orow < P) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator: stride smaller than extent");
  const size_t ie = esize(in_dtype), oe = esize(out_dtype);
  const bool vec = os % 4 == 0 && aligned_to(opT, 16) && P % 4 == 0 && ls % 4 == 0 && cs % 4 == 0 &&
                   aligned_to(I, 4 * ie) && orow % 4 == 0 && ocs % 4 == 0 && aligned_to(out, 4 * oe);
  hipStream_t s = (hipStream_t)stream;
  switch (in_dtype) {
    case RTI_F32: return launch_out<float>(out_dtype, opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_I32: return launch_out<int32_t>(out_dtype, opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
    default: return launch_out<uint8_t>(out_dtype, opT, E, N, os, I, P, C, ls, cs, out, orow, ocs, vec, s);
  }
}

extern "C" int rti_operator_split_f16(const double* opT, int N, int E, int64_t op_stride, int Kp, uint16_t* hi,
                                      uint16_t* lo, float* inv_scale) {
  if (!opT || !hi || !lo || !inv_scale) return fail(RTI_ERR_BAD_ARG, "rti_operator_split_f16: null pointer");
  if (N <= 0 || E <= 0) return fail(RTI_ERR_BAD_ARG, "rti_operator_split_f16: N and E must be positive");
  if (Kp < N || Kp % 16 != 0) return fail(RTI_ERR_BAD_ARG, "rti_operator_split_f16: Kp must be a multiple of 16 >= N");
  const int64_t os = op_stride ? op_stride : E;
  if (os < E) return fail(RTI_ERR_BAD_ARG, "rti_operator_split_f16: op_stride < E");
  double m = 0.0;
  for (int n = 0; n < N; ++n)
    for (int e = 0; e < E; ++e) {
      const double v = opT[(int64_t)n * os + e];
      if (!std::isfinite(v)) return fail(RTI_ERR_BAD_ARG, "rti_operator_split_f16: non-finite operator entry");
      m = std::max(m, std::fabs(v));
    }
  int ex = 0;
  if (m > 0.0) std::frexp(m, &ex);  // m < 2^ex
  const double sc = std::ldexp(1.0, 15 - ex);  // max|M·s| < 2^15
  _Float16* H = reinterpret_cast<_Float16*>(hi);
  _Float16* L = reinterpret_cast<_Float16*>(lo);
  for (int e = 0; e < E; ++e)
    for (int n = 0; n < Kp; ++n) {
      const double v = n < N ? opT[(int64_t)n * os + e] * sc : 0.0;
      const _Float16 h = (_Float16)v;
      H[(int64_t)e * Kp + n] = h;
      L[(int64_t)e * Kp + n] = (_Float16)(v - (double)h);
    }
  *inv_scale = (float)(1.0 / sc);
  return RTI_OK;
}

extern "C" int rti_apply_operator_f16(const uint16_t* op_hi, const uint16_t* op_lo, int Kp, float inv_scale, int E,
                                      int N, const void* I, int in_dtype, int64_t P, int C, int64_t light_stride,
                                      int64_t channel_stride, void* out, int out_dtype, int64_t out_row_stride,
                                      int64_t out_channel_stride, rti_stream_t stream) {
  if (!op_hi || !op_lo || !I || !out) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator_f16: null pointer");
  if (E <= 0 || N <= 0 || P <= 0 || C <= 0 || C > 65535)
    return fail(RTI_ERR_BAD_ARG, "rti_apply_operator_f16: bad E/N/P/C");
  if (Kp < N || Kp % 16 != 0) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator_f16: Kp must be a multiple of 16 >= N");
  if (Kp > 256) return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator_f16: N=%d > 256 lights", N);
  if (in_dtype != RTI_F32 && in_dtype != RTI_U8 && in_dtype != RTI_I32)
    return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator_f16: input dtype %d", in_dtype);
  if (out_dtype != RTI_F32 && out_dtype != RTI_F64 && out_dtype != RTI_I32 && out_dtype != RTI_U8)
    return fail(RTI_ERR_UNSUPPORTED, "rti_apply_operator_f16: out dtype %d", out_dtype);
  if (!aligned_to(op_hi, 16) || !aligned_to(op_lo, 16))
    return fail(RTI_ERR_BAD_ARG, "rti_apply_operator_f16: operator halves must be 16-byte aligned");
  const int64_t ls = light_stride ? light_stride : P;
  const int64_t cs = channel_stride ? channel_stride : (int64_t)N * ls;
  const int64_t orow = out_row_stride ? out_row_stride : P;
  const int64_t ocs = out_channel_stride ? out_channel_stride : (int64_t)E * orow;
  if (ls < P || orow < P) return fail(RTI_ERR_BAD_ARG, "rti_apply_operator_f16: stride smaller than extent");
  const size_t ie = esize(in_dtype);
  const bool vec = P % 4 == 0 && ls % 4 == 0 && cs % 4 == 0 && aligned_to(I, 4 * ie);
  const _Float16* hi = reinterpret_cast<const _Float16*>(op_hi);
  const _Float16* lo = reinterpret_cast<const _Float16*>(op_lo);
  hipStream_t s = (hipStream_t)stream;
  switch (in_dtype) {
    case RTI_F32:
      return launch_f16_out<float>(out_dtype, hi, lo, Kp, inv_scale, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
    case RTI_I32:
      return launch_f16_out<int32_t>(out_dtype, hi, lo, Kp, inv_scale, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
    default:
      return launch_f16_out<uint8_t>(out_dtype, hi, lo, Kp, inv_scale, E, N, I, P, C, ls, cs, out, orow, ocs, vec, s);
  }
}
