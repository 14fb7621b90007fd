// rti_basis.h -- light-direction bases shared by host (pinv) and device (relight).
//
// PTM-6 follows the reference's row (lu², lv², lu·lv, lu, lv, 1.)
// (analysis.py:285) and its evaluation order (analysis.py:307-312).
// HSH is build-defined (the reference has none):
// hemispherical harmonics (Gautron et al. 2004) on the upper hemisphere with
// lw = sqrt(max(0, 1 - lu² - lv²)), t = 2·lw − 1, φ = atan2(lv, lu):
//   H_l^0 = K_l^0 P_l^0(t),  H_l^{±m} = √2 K_l^m {cos,sin}(mφ) P_l^m(t),
//   K_l^m = sqrt((2l+1)/(2π) · (l−m)!/(l+m)!),  column l² + l + m.
// P_l^m carries no Condon–Shortley phase.  cos(mφ)/sin(mφ) are formed
// algebraically from (lu, lv) / |(lu, lv)| (φ = 0 at the pole, like atan2(0,0)).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/rti.h"

namespace rti {

__host__ __device__ inline int basis_terms(int basis) {
  return basis == RTI_BASIS_PTM6 ? 6 : basis == RTI_BASIS_HSH16 ? 16 : basis == RTI_BASIS_HSH9 ? 9 : -1;
}

// Normalisation constants K_l^m (l = 0..3), precomputed in long double precision.
#define RTI_SQRT2 1.41421356237309504880
#define RTI_K00 0.39894228040143267794   // sqrt(1/(2π))
#define RTI_K10 0.69098829894267095853   // sqrt(3/(2π))
#define RTI_K11 0.48860251190291992159   // sqrt(3/(2π)/2)
#define RTI_K20 0.89206205807638555727   // sqrt(5/(2π))
#define RTI_K21 0.36418281019735969018   // sqrt(5/(2π)/6)
#define RTI_K22 0.18209140509867984509   // sqrt(5/(2π)/24)
#define RTI_K30 1.05550206141118803141   // sqrt(7/(2π))
#define RTI_K31 0.30469719964297715744   // sqrt(7/(2π)/12)
#define RTI_K32 0.09635371475468513518   // sqrt(7/(2π)/120)
#define RTI_K33 0.03933623932844290069   // sqrt(7/(2π)/720)

// Hemispherical harmonics, first k terms (k = 9 or 16), type T arithmetic.
template <typename T>
__host__ __device__ inline void hsh_eval(T lu, T lv, int k, T* out) {
#pragma clang fp contract(off)  // identical values in every kernel and on the host
  T r2 = lu * lu + lv * lv;
  T lw2 = T(1) - r2;
  T lw = lw2 > T(0) ? sqrt(lw2) : T(0);
  T t = T(2) * lw - T(1);
  T st2 = (T(1) - t) * (T(1) + t);
  T st = st2 > T(0) ? sqrt(st2) : T(0);
  T s = sqrt(r2);
  T c1 = s > T(0) ? lu / s : T(1);
  T s1 = s > T(0) ? lv / s : T(0);
  T c2 = c1 * c1 - s1 * s1, s2 = T(2) * s1 * c1;
  T c3 = c1 * c2 - s1 * s2, s3 = s1 * c2 + c1 * s2;
  const T r = T(RTI_SQRT2);
  // l = 0
  out[0] = T(RTI_K00);
  // l = 1 : m = -1, 0, 1
  T p11 = st;
  out[1] = r * T(RTI_K11) * s1 * p11;
  out[2] = T(RTI_K10) * t;
  out[3] = r * T(RTI_K11) * c1 * p11;
  // l = 2
  T p20 = (T(3) * t * t - T(1)) * T(0.5);
  T p21 = T(3) * t * st;
  T p22 = T(3) * st2;
  out[4] = r * T(RTI_K22) * s2 * p22;
  out[5] = r * T(RTI_K21) * s1 * p21;
  out[6] = T(RTI_K20) * p20;
  out[7] = r * T(RTI_K21) * c1 * p21;
  out[8] = r * T(RTI_K22) * c2 * p22;
  if (k <= 9) return;
  // l = 3
  T p30 = (T(5) * t * t * t - T(3) * t) * T(0.5);
  T p31 = T(1.5) * (T(5) * t * t - T(1)) * st;
  T p32 = T(15) * t * st2;
  T p33 = T(15) * st2 * st;
  out[9] = r * T(RTI_K33) * s3 * p33;
  out[10] = r * T(RTI_K32) * s2 * p32;
  out[11] = r * T(RTI_K31) * s1 * p31;
  out[12] = T(RTI_K30) * p30;
  out[13] = r * T(RTI_K31) * c1 * p31;
  out[14] = r * T(RTI_K32) * c2 * p32;
  out[15] = r * T(RTI_K33) * c3 * p33;
}

// PTM row in type T (used by the relight evaluator; analysis.py:307-311 forms
// lu**2, lv**2, lu*lv in the coefficient precision).
template <typename T>
__host__ __device__ inline void ptm_eval(T lu, T lv, T* out) {
#pragma clang fp contract(off)
  out[0] = lu * lu;
  out[1] = lv * lv;
  out[2] = lu * lv;
  out[3] = lu;
  out[4] = lv;
  out[5] = T(1);
}

template <typename T>
__host__ __device__ inline void basis_eval(int basis, T lu, T lv, T* out) {
  if (basis == RTI_BASIS_PTM6)
    ptm_eval(lu, lv, out);
  else
    hsh_eval(lu, lv, basis_terms(basis), out);
}

}  // namespace rti
