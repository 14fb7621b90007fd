// rti_host.cpp -- host half of the C ABI: status strings, design matrices and
// the shared pseudo-inverse (fp64 one-sided Jacobi SVD).
//
// rti_design_matrix restates the design-row loop of _interpolate_PTM
// (analysis.py:280-291); rti_pinv restates its SVD solve (analysis.py:293-298)
// as an explicit k×N operator so a single device contraction can apply it to
// every pixel.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>

#include "rti_basis.h"
#include "rti_internal.h"
#include "rti_q8.h"

namespace rti {

thread_local char g_last_error[512] = "";
thread_local int g_launches = 0;

void note_launches(int n) { g_launches = n; }

int fail(int status, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return status;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(RTI_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return RTI_OK;
}

// PTM row exactly as analysis.py:284-285: monomials of float32 lu/lv formed in
// float32, then widened (np.array of the tuple is float64).  The reference's
// `lu ** 2` is C powf on a NumPy float32 scalar; x*x is its correctly rounded
// value (they can differ by 1 ulp, far inside the fp32 parity tolerance).
static void ptm_row(float lu, float lv, double* row) {
  row[0] = (double)(lu * lu);
  row[1] = (double)(lv * lv);
  row[2] = (double)(lu * lv);
  row[3] = (double)lu;
  row[4] = (double)lv;
  row[5] = 1.0;
}

static void design_row(int basis, float lu, float lv, double* row) {
  if (basis == RTI_BASIS_PTM6)
    ptm_row(lu, lv, row);
  else
    hsh_eval<double>((double)lu, (double)lv, basis_terms(basis), row);
}

// One-sided (Hestenes) Jacobi SVD of A[n][k] (row-major, n >= k) and
// pinv[k][n] = V Σ⁻¹ Uᵀ = Σ_m v_m (A v_m)ᵀ / σ_m²; optionally the Gram (pseudo-)inverse
// ginv[k][k] = (AᵀA)⁺ = V Σ⁻² Vᵀ, so that pinv = ginv · Aᵀ, and the thin SVD factors themselves
// (Uo[n][k] = A v_m / σ_m, the orthonormal left singular vectors; Wo[k][k] = V Σ⁻¹), the two halves of
// analysis.py:295-298 (c = uᵀL, w = c/s, a = vᵀw).  A truncated σ (rcond) zeroes its column of Uo and Wo;
// σ = 0 without rcond gives 0·inf = NaN entries, the reference's division by a zero singular value.
static void jacobi_pinv(const double* A, int n, int k, double rcond, double* pinv, double* ginv = nullptr,
                        double* Uo = nullptr, double* Wo = nullptr) {
  std::vector<double> U(A, A + (size_t)n * k);  // column j = U[i*k + j]; becomes U·Σ
  std::vector<double> V((size_t)k * k, 0.0);
  for (int j = 0; j < k; ++j) V[(size_t)j * k + j] = 1.0;
  const double tol = 1e-15;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < k - 1; ++p) {
      for (int q = p + 1; q < k; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int i = 0; i < n; ++i) {
          const double up = U[(size_t)i * k + p], uq = U[(size_t)i * k + q];
          alpha += up * up;
          beta += uq * uq;
          gamma += up * uq;
        }
        if (gamma == 0.0 || alpha == 0.0 || beta == 0.0) continue;
        const double rel = std::fabs(gamma) / std::sqrt(alpha * beta);
        if (rel <= tol) continue;
        off = std::fmax(off, rel);
        const double zeta = (beta - alpha) / (2.0 * gamma);
        const double t = std::copysign(1.0, zeta) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
        for (int i = 0; i < n; ++i) {
          double& up = U[(size_t)i * k + p];
          double& uq = U[(size_t)i * k + q];
          const double a = up, b = uq;
          up = c * a - s * b;
          uq = s * a + c * b;
        }
        for (int i = 0; i < k; ++i) {
          double& vp = V[(size_t)i * k + p];
          double& vq = V[(size_t)i * k + q];
          const double a = vp, b = vq;
          vp = c * a - s * b;
          vq = s * a + c * b;
        }
      }
    }
    if (off <= tol) break;
  }
  std::vector<double> sig2(k);
  double smax = 0.0;
  for (int m = 0; m < k; ++m) {
    double s2 = 0;
    for (int i = 0; i < n; ++i) s2 += U[(size_t)i * k + m] * U[(size_t)i * k + m];
    sig2[m] = s2;
    smax = std::fmax(smax, std::sqrt(s2));
  }
  std::vector<double> inv2(k);
  for (int m = 0; m < k; ++m) {
    const double sm = std::sqrt(sig2[m]);
    if (rcond >= 0.0 && !(sm > rcond * smax))
      inv2[m] = 0.0;  // truncated
    else
      inv2[m] = 1.0 / sig2[m];  // reference semantics: σ = 0 -> inf -> NaN entries
  }
  if (pinv)
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < n; ++i) {
        double acc = 0.0;
        for (int m = 0; m < k; ++m) {
          if (inv2[m] == 0.0) continue;
          acc += V[(size_t)j * k + m] * (U[(size_t)i * k + m] * inv2[m]);
        }
        pinv[(size_t)j * n + i] = acc;
      }
  if (ginv)
    for (int j = 0; j < k; ++j)
      for (int l = 0; l < k; ++l) {
        double acc = 0.0;
        for (int m = 0; m < k; ++m) {
          if (inv2[m] == 0.0) continue;
          acc += V[(size_t)j * k + m] * (V[(size_t)l * k + m] * inv2[m]);
        }
        ginv[(size_t)j * k + l] = acc;
      }
  if (Uo && Wo)
    for (int m = 0; m < k; ++m) {
      const double is = inv2[m] == 0.0 ? 0.0 : 1.0 / std::sqrt(sig2[m]);
      for (int i = 0; i < n; ++i) Uo[(size_t)i * k + m] = U[(size_t)i * k + m] * is;
      for (int j = 0; j < k; ++j) Wo[(size_t)j * k + m] = V[(size_t)j * k + m] * is;
    }
}

// LU factorisation with partial pivoting (LAPACK getrf semantics), in place, row-major n×n.
// Returns false for an exactly singular matrix (a zero pivot), as dgesv reports info > 0.
static bool lu_factor(std::vector<double>& a, int n, std::vector<int>& piv) {
  piv.resize(n);
  for (int k = 0; k < n; ++k) {
    int p = k;
    double best = std::fabs(a[(size_t)k * n + k]);
    for (int i = k + 1; i < n; ++i) {
      const double v = std::fabs(a[(size_t)i * n + k]);
      if (v > best) best = v, p = i;
    }
    piv[k] = p;
    if (best == 0.0) return false;
    if (p != k)
      for (int j = 0; j < n; ++j) std::swap(a[(size_t)k * n + j], a[(size_t)p * n + j]);
    const double inv = 1.0 / a[(size_t)k * n + k];
    for (int i = k + 1; i < n; ++i) {
      double& l = a[(size_t)i * n + k];
      l *= inv;
      if (l == 0.0) continue;
      for (int j = k + 1; j < n; ++j) a[(size_t)i * n + j] -= l * a[(size_t)k * n + j];
    }
  }
  return true;
}

// Solve A X = B for X, B row-major n×m (overwritten), with the factors of lu_factor.
static void lu_solve(const std::vector<double>& a, const std::vector<int>& piv, int n, double* B, int m) {
  for (int k = 0; k < n; ++k)
    if (piv[k] != k)
      for (int j = 0; j < m; ++j) std::swap(B[(size_t)k * m + j], B[(size_t)piv[k] * m + j]);
  for (int i = 1; i < n; ++i)
    for (int k = 0; k < i; ++k) {
      const double l = a[(size_t)i * n + k];
      if (l == 0.0) continue;
      for (int j = 0; j < m; ++j) B[(size_t)i * m + j] -= l * B[(size_t)k * m + j];
    }
  for (int i = n - 1; i >= 0; --i) {
    for (int k = i + 1; k < n; ++k) {
      const double u = a[(size_t)i * n + k];
      if (u == 0.0) continue;
      for (int j = 0; j < m; ++j) B[(size_t)i * m + j] -= u * B[(size_t)k * m + j];
    }
    const double inv = 1.0 / a[(size_t)i * n + i];
    for (int j = 0; j < m; ++j) B[(size_t)i * m + j] *= inv;
  }
}

}  // namespace rti

using namespace rti;

extern "C" {

int rti_version(void) { return 100; /* 0.1.0 */ }

const char* rti_status_string(int status) {
  switch (status) {
    case RTI_OK: return "ok";
    case RTI_ERR_BAD_ARG: return "bad argument";
    case RTI_ERR_UNSUPPORTED: return "unsupported";
    case RTI_ERR_HIP: return "hip error";
    case RTI_ERR_SINGULAR: return "singular matrix";
    default: return "unknown status";
  }
}

const char* rti_last_error(void) { return g_last_error; }

int rti_last_launch_count(void) { return g_launches; }

int rti_basis_terms(int basis) { return basis_terms(basis); }

int rti_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int rti_design_matrix(int basis, const float* lu, const float* lv, int n, double* A) {
  const int k = basis_terms(basis);
  if (k < 0) return fail(RTI_ERR_BAD_ARG, "rti_design_matrix: unknown basis %d", basis);
  if (!lu || !lv || !A || n <= 0) return fail(RTI_ERR_BAD_ARG, "rti_design_matrix: null pointer or n <= 0");
  for (int i = 0; i < n; ++i) design_row(basis, lu[i], lv[i], A + (size_t)i * k);
  return RTI_OK;
}

int rti_pinv(int basis, const float* lu, const float* lv, int n, double rcond, double* pinv) {
  const int k = basis_terms(basis);
  if (k < 0) return fail(RTI_ERR_BAD_ARG, "rti_pinv: unknown basis %d", basis);
  if (!lu || !lv || !pinv || n <= 0) return fail(RTI_ERR_BAD_ARG, "rti_pinv: null pointer or n <= 0");
  if (n < k)
    return fail(RTI_ERR_BAD_ARG, "rti_pinv: %d lights < %d basis terms (shapes not aligned, analysis.py:298)", n, k);
  std::vector<double> A((size_t)n * k);
  for (int i = 0; i < n; ++i) design_row(basis, lu[i], lv[i], A.data() + (size_t)i * k);
  jacobi_pinv(A.data(), n, k, rcond, pinv);
  return RTI_OK;
}

int rti_gram_inverse(int basis, const float* lu, const float* lv, int n, double rcond, double* ginv) {
  const int k = basis_terms(basis);
  if (k < 0) return fail(RTI_ERR_BAD_ARG, "rti_gram_inverse: unknown basis %d", basis);
  if (!lu || !lv || !ginv || n <= 0) return fail(RTI_ERR_BAD_ARG, "rti_gram_inverse: null pointer or n <= 0");
  if (n < k)
    return fail(RTI_ERR_BAD_ARG, "rti_gram_inverse: %d lights < %d basis terms (shapes not aligned, analysis.py:298)",
                n, k);
  std::vector<double> A((size_t)n * k);
  for (int i = 0; i < n; ++i) design_row(basis, lu[i], lv[i], &A[(size_t)i * k]);
  jacobi_pinv(A.data(), n, k, rcond, nullptr, ginv);
  return RTI_OK;
}

int rti_lsq_factors(int basis, const float* lu, const float* lv, int n, double rcond, double* U, double* W) {
  const int k = basis_terms(basis);
  if (k < 0) return fail(RTI_ERR_BAD_ARG, "rti_lsq_factors: unknown basis %d", basis);
  if (!lu || !lv || !U || !W || n <= 0) return fail(RTI_ERR_BAD_ARG, "rti_lsq_factors: null pointer or n <= 0");
  if (n < k)
    return fail(RTI_ERR_BAD_ARG, "rti_lsq_factors: %d lights < %d basis terms (shapes not aligned, analysis.py:298)", n,
                k);
  std::vector<double> A((size_t)n * k);
  for (int i = 0; i < n; ++i) design_row(basis, lu[i], lv[i], &A[(size_t)i * k]);
  jacobi_pinv(A.data(), n, k, rcond, nullptr, nullptr, U, W);
  return RTI_OK;
}

int64_t rti_q8_operator_bytes(int k, int N) {
  if (k < 1 || k > 16 || N <= 0) return -1;
  return q8_operator_bytes(N);
}

int rti_q8_operator(const double* pinv, int k, int N, void* op) {
  if (!pinv || !op) return fail(RTI_ERR_BAD_ARG, "rti_q8_operator: null pointer");
  if (k < 1 || k > 16 || N <= 0) return fail(RTI_ERR_BAD_ARG, "rti_q8_operator: k=%d N=%d", k, N);
  const int T = q8_steps(N);
  int8_t* frag = static_cast<int8_t*>(op);
  double* scale = reinterpret_cast<double*>(static_cast<char*>(op) + q8_frag_bytes(N));
  int32_t* corr = reinterpret_cast<int32_t*>(scale + 16);
  std::vector<int8_t> dig((size_t)Q8_DIGITS * k * N);  // dig[j][i][n]
  for (int i = 0; i < 16; ++i) {
    scale[i] = 0.0;
    for (int j = 0; j < Q8_DIGITS; ++j) corr[i * Q8_DIGITS + j] = 0;
  }
  for (int i = 0; i < k; ++i) {
    double m = 0.0;
    for (int n = 0; n < N; ++n) {
      const double w = pinv[(size_t)i * N + n];
      if (!std::isfinite(w))
        return fail(RTI_ERR_BAD_ARG, "rti_q8_operator: non-finite pseudo-inverse entry (row %d, light %d)", i, n);
      m = std::fmax(m, std::fabs(w));
    }
    scale[i] = m * 0x1p-27;
    for (int n = 0; n < N; ++n) {
      int64_t W = m > 0.0 ? (int64_t)std::llround(pinv[(size_t)i * N + n] / m * 0x1p27) : 0;  // |W| <= 2^27
      int8_t d[Q8_DIGITS];
      for (int j = Q8_DIGITS - 1; j > 0; --j) {  // balanced base-128 digits, least significant first
        const int64_t r = ((W + 64) % 128 + 128) % 128 - 64;
        d[j] = (int8_t)r;
        W = (W - r) / 128;
      }
      d[0] = (int8_t)W;  // in [-64, 64]
      for (int j = 0; j < Q8_DIGITS; ++j) {
        dig[((size_t)j * k + i) * N + n] = d[j];
        corr[i * Q8_DIGITS + j] += 128 * d[j];
      }
    }
  }
  for (int t = 0; t < T; ++t)
    for (int j = 0; j < Q8_DIGITS; ++j)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 16; ++e) {
          const int i = l & 15, n = t * Q8_STEP + q8_light(l >> 4, e);
          frag[(((size_t)t * Q8_DIGITS + j) * 64 + l) * 16 + e] =
              (i < k && n < N) ? dig[((size_t)j * k + i) * N + n] : (int8_t)0;
        }
  return RTI_OK;
}

int rti_rbf_operator(const float* lu, const float* lv, int n, const double* qu, const double* qv, int E,
                     double* opT) {
  if (!lu || !lv || !qu || !qv || !opT || n <= 0 || E <= 0)
    return fail(RTI_ERR_BAD_ARG, "rti_rbf_operator: null pointer or non-positive size");
  // nodes as SciPy holds them: float64 copies of the float32 light vectors
  std::vector<double> x(n), y(n);
  for (int i = 0; i < n; ++i) x[i] = (double)lu[i], y[i] = (double)lv[i];
  std::vector<double> A((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      const double dx = x[i] - x[j], dy = y[i] - y[j];
      A[(size_t)i * n + j] = std::sqrt(dx * dx + dy * dy);  // pdist 'euclidean', linear kernel r
    }
  std::vector<int> piv;
  if (!lu_factor(A, n, piv)) return fail(RTI_ERR_SINGULAR, "rti_rbf_operator: Matrix is singular.");
  // X = A^-1 Φᵀ (n×E): A is symmetric, so row n of X is column n of M = Φ A^-1, i.e. opT[n][e]
  for (int j = 0; j < n; ++j)
    for (int e = 0; e < E; ++e) {
      const double dx = qu[e] - x[j], dy = qv[e] - y[j];
      opT[(size_t)j * E + e] = std::sqrt(dx * dx + dy * dy);
    }
  lu_solve(A, piv, n, opT, E);
  return RTI_OK;
}

int rti_basis_operator(int basis, const float* lu, const float* lv, int n, const double* qu, const double* qv,
                       int E, double rcond, double* opT) {
  const int k = basis_terms(basis);
  if (k < 0) return fail(RTI_ERR_BAD_ARG, "rti_basis_operator: unknown basis %d", basis);
  if (!lu || !lv || !qu || !qv || !opT || n <= 0 || E <= 0)
    return fail(RTI_ERR_BAD_ARG, "rti_basis_operator: null pointer or non-positive size");
  if (n < k) return fail(RTI_ERR_BAD_ARG, "rti_basis_operator: %d lights < %d basis terms", n, k);
  std::vector<double> A((size_t)n * k), pinv((size_t)k * n), b(k);
  for (int i = 0; i < n; ++i) design_row(basis, lu[i], lv[i], A.data() + (size_t)i * k);
  jacobi_pinv(A.data(), n, k, rcond, pinv.data());
  for (int e = 0; e < E; ++e) {
    basis_eval<double>(basis, qu[e], qv[e], b.data());
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int i = 0; i < k; ++i) s += b[i] * pinv[(size_t)i * n + j];
      opT[(size_t)j * E + e] = s;
    }
  }
  return RTI_OK;
}

int rti_basis_eval(int basis, const double* lu, const double* lv, int E, double* out) {
  const int k = basis_terms(basis);
  if (k < 0) return fail(RTI_ERR_BAD_ARG, "rti_basis_eval: unknown basis %d", basis);
  if (!lu || !lv || !out || E <= 0) return fail(RTI_ERR_BAD_ARG, "rti_basis_eval: null pointer or E <= 0");
  for (int e = 0; e < E; ++e) basis_eval<double>(basis, lu[e], lv[e], out + (size_t)e * k);
  return RTI_OK;
}

}  // extern "C"
