// rti_q8.h -- the fixed-point light operator of the 8-bit fit (rti_fit_shared_q8), shared by the host
// builder (rti_host.cpp: rti_q8_operator) and the kernel (rti_fit_q8.hip).
//
// An 8-bit stack (the reference's V channel is uint8, analysis.py:219 / FeatureMatcher.py:183-184) is
// contracted on the int8 matrix cores: coefficient i of a pixel is
//     c_i = Σ_n w_in · x_n,   x_n ∈ [0, 255]
// with each row of the fp64 pseudo-inverse scaled to 27-bit fixed point, W_in = round(w_in / m_i · 2^27)
// (m_i = max_n |w_in|), split into four balanced base-128 int8 digits
//     W_in = d0·2^21 + d1·2^14 + d2·2^7 + d3        (d1..d3 ∈ [-64, 63], d0 ∈ [-64, 64])
// and the intensities made signed by x' = x ⊕ 0x80 = x − 128.  Then, exactly in int32 per digit j,
//     acc_ij = Σ_n d_jin · x'_n,        corr_ij = 128 · Σ_n d_jin
// and c_i = (m_i · 2^-27) · Σ_j 128^(3−j) · (acc_ij + corr_ij), the sum formed exactly in fp64 and rounded
// once.  The only approximation is the 2^-28 · m_i rounding of each weight: |Δc_i| ≤ 2^-28 · m_i · Σ_n x_n
// (3.7e-9 · m_i per unit of intensity sum; fp32 rounding of the result dominates: ≈6e-8 of max_k |c_k| on
// the BASELINE stacks, against ≈1e-6 for the fp32 stream).
//
// Operator buffer (rti_q8_operator_bytes(k, N) bytes, 16-byte aligned on the device):
//   int8    frag[T][4][64][16]   T = ⌈N/64⌉ steps of 64 lights; digit j's A fragment of
//                                v_mfma_i32_16x16x64_i8 for step t: lane l (row i = l & 15,
//                                group g = l >> 4) element e holds d_j[i][64t + q8_light(g, e)]
//                                (0 for i ≥ k or a light ≥ N)
//   double  scale[16]            m_i · 2^-27 (0 for i ≥ k)
//   int32   corr[16][4]          corr_ij
#pragma once

#include <cstdint>

namespace rti {

constexpr int Q8_STEP = 64;  // lights per MFMA K-step
constexpr int Q8_DIGITS = 4;

// Light (within a 64-light step) of fragment element e (0..15) held by lane group g (0..3): the kernel's
// two ds_read_b64_tr_b8 reads give elements 0..7 from rows 8g..8g+7 and 8..15 from rows 32+8g..32+8g+7
// of the LDS tile (a 32-lane half reads 16 consecutive rows: conflict-free with 16-B row padding).  A and
// B use the same map, so the MFMA's sum over k runs over all 64 lights exactly once.
__host__ __device__ constexpr int q8_light(int g, int e) { return e < 8 ? 8 * g + e : 32 + 8 * g + (e - 8); }

__host__ __device__ constexpr int q8_steps(int N) { return (N + Q8_STEP - 1) / Q8_STEP; }

__host__ __device__ constexpr int64_t q8_frag_bytes(int N) { return (int64_t)q8_steps(N) * Q8_DIGITS * 64 * 16; }

__host__ __device__ constexpr int64_t q8_operator_bytes(int N) { return q8_frag_bytes(N) + 16 * 8 + 16 * 4 * 4; }

}  // namespace rti
