/*
 * rti.h -- C ABI of the MI355X-native RTI reflectance fitter (PTM / HSH).
 *
 * Drop-in boundary for the per-pixel reflectance-fit hot path of
 * bara96/Smartphone-based-RTI (reference @ v0).  The reference has no FFI of
 * its own: the path sits behind plain Python calls in analysis.py.  Each entry
 * point below names the reference code it replaces.  The Python package
 * (smartphone-based-rti_amd/rti) binds these symbols with ctypes; INTEGRATION.md
 * shows the binding a maintainer of the reference would add.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Functions named rti_fit_* / rti_relight*
 *     take DEVICE pointers (hipMalloc'd or torch CUDA tensors) and enqueue
 *     asynchronously on `stream` (a hipStream_t; NULL = default stream).  They
 *     never allocate, free or synchronise, so they can be captured in a
 *     hipGraph.  Functions named rti_design_* / rti_pinv / rti_basis_* are
 *     host-only and take HOST pointers.
 *   - Return value: RTI_OK (0) or an RTI_ERR_* status; rti_last_error()
 *     returns a thread-local message for the most recent failure.
 *   - Reentrant: no global mutable state besides the thread-local message.
 *   - Intensity stacks are LIGHT-MAJOR: I[c][n][p] with pixel p = y*W + x
 *     contiguous inside one light plane (strides in elements; 0 = dense).
 *     The reference stacks pixel-major [y][x][n] (analysis.py:217-219);
 *     rti_fit_shared_pm and the per-pixel "dirs" entry point take that layout.
 */
#ifndef RTI_H
#define RTI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define RTI_OK              0
#define RTI_ERR_BAD_ARG     1   /* null pointer, non-positive size, k/N mismatch, N < k */
#define RTI_ERR_UNSUPPORTED 2   /* valid but unsupported combination (dtype/basis/layout) */
#define RTI_ERR_HIP         3   /* HIP runtime error at launch */
#define RTI_ERR_SINGULAR    4   /* singular system (the reference's SciPy Rbf raises LinAlgError) */

/* ---- bases ---- */
#define RTI_BASIS_PTM6  0   /* (lu², lv², lu·lv, lu, lv, 1), analysis.py:285 */
#define RTI_BASIS_HSH16 1   /* hemispherical harmonics l=0..3 (build-defined) */
#define RTI_BASIS_HSH9  2   /* hemispherical harmonics l=0..2 */

/* ---- element types ---- */
#define RTI_F32 0
#define RTI_U8  1
#define RTI_I32 2
#define RTI_F64 3

/* ---- coefficient layouts ---- */
#define RTI_COEF_PIXEL_MAJOR 0  /* coef[c][p][k] */
#define RTI_COEF_PLANAR      1  /* coef[c][k][p] */

/* ---- relight output layouts ---- */
#define RTI_OUT_EVAL_MAJOR  0   /* out[e][p]: one image per light (prepare_images_data order) */
#define RTI_OUT_PIXEL_MAJOR 1   /* out[p][e]: interpolate_intensities order [y][x][ly][lx] */

/* ---- shared-fit kernel selection ---- */
#define RTI_KERNEL_AUTO 0
#define RTI_KERNEL_VALU 1   /* pinv in SGPRs, fp32 FMA stream */
#define RTI_KERNEL_MFMA 2   /* v_mfma_f32_16x16x4_f32, pinv staged in LDS */
#define RTI_KERNEL_TILE 3   /* the same MFMA fed from a double-buffered LDS tile [4·sp lights][256·rc pixels] */
/* OR-able tuning flags (VALU kernel; only NONTEMPORAL applies to the MFMA kernel) */
#define RTI_KERNEL_NONTEMPORAL 0x100  /* non-temporal intensity loads (the stack is read once) */
#define RTI_KERNEL_PINV_LDS    0x200  /* stage pinv in LDS instead of scalar loads */
#define RTI_KERNEL_NT_STORE    0x400  /* non-temporal coefficient stores */
#define RTI_KERNEL_STAGE       0x800  /* pixel-major output transposed through LDS (1 KiB stores) */
#define RTI_KERNEL_ROTATE      0x10000000  /* AUTO PTM-6 fp32: each wave starts its light sweep at its own plane; rti_fit_shared_pm: each wave streams one contiguous run of units (measurement variants) */
#define RTI_KERNEL_ROUNDS      0x40000000  /* AUTO PTM-6 fp32/int32: launch generations as rounds of one launch (rti_fit.hip) */
#define RTI_KERNEL_ONE_LAUNCH  0x20000000  /* AUTO: one launch, no launch generations (measurement variant; rti_fit.hip) */
/* VALU chunks per lane (bits 12-15; 0 = AUTO): a wave reads chunks*1 KiB contiguous per plane */
#define RTI_KERNEL_CHUNKS_SHIFT 12
#define RTI_KERNEL_CHUNKS(n)   ((n) << RTI_KERNEL_CHUNKS_SHIFT)
/* TILE kernel: CHUNKS(rc) sets the tile width (256·rc pixels; 0 = 8, or 4 above N = 512),
 * TILE_PLANES(sp) the light planes each wave loads per step (bits 16-19, 0 = 2) */
#define RTI_KERNEL_TILE_PLANES_SHIFT 16
#define RTI_KERNEL_TILE_PLANES(n)    ((n) << RTI_KERNEL_TILE_PLANES_SHIFT)
/* TILE kernel: tiles in the LDS ring (bits 20-23; 0 = 2): 2 = register-staged double buffer,
 * 3 or 4 = global_load_lds ring with depth-1 steps in flight (fp32 stacks) */
#define RTI_KERNEL_TILE_DEPTH_SHIFT 20
#define RTI_KERNEL_TILE_DEPTH(n)    ((n) << RTI_KERNEL_TILE_DEPTH_SHIFT)
/* TILE kernel, fp32 stacks: waves per workgroup (bits 24-27; 0 = 4).  8 = one light plane per wave
 * and step with the plane loads issued DEPTH − 1 steps ahead in registers (DEPTH 2 or 3) */
#define RTI_KERNEL_TILE_WAVES_SHIFT 24
#define RTI_KERNEL_TILE_WAVES(n)    ((n) << RTI_KERNEL_TILE_WAVES_SHIFT)

typedef void* rti_stream_t; /* hipStream_t */

/* ---- library info ---- */
int         rti_version(void);                 /* 10000*major + 100*minor + patch */
const char* rti_status_string(int status);
const char* rti_last_error(void);
/* Kernel launches issued by this thread's most recent rti_fit_shared / rti_fit_shared_residual call:
 * 1, or more when AUTO issues a large fit as consecutive "launch generations" over pixel ranges
 * (rti_fit.hip).  For timing tools (per-launch figures); the results do not depend on it. */
int rti_last_launch_count(void);
int         rti_basis_terms(int basis);        /* k for a basis, or -1 */
int         rti_device_count(void);            /* hipGetDeviceCount, 0 on failure */

/* ---- host: basis / design matrix / pseudo-inverse ----------------------------------
 * rti_design_matrix replaces the design-row loop of _interpolate_PTM
 * (analysis.py:280-291): A[n][k] in fp64 with PTM monomials formed in fp32 from
 * fp32 (lu, lv), as the reference does.
 * rti_pinv replaces the SVD solve (analysis.py:293-298) for a SHARED light set:
 * pinv[k][n] = V Σ⁻¹ Uᵀ by one-sided Jacobi SVD in fp64.  rcond < 0 keeps the
 * reference's semantics (no threshold: a zero singular value gives inf/NaN);
 * rcond >= 0 zeroes σ <= rcond·σ_max.  Returns RTI_ERR_BAD_ARG when n < k
 * (the reference raises ValueError at analysis.py:298).
 * rti_basis_eval evaluates the basis at E host (lu, lv) pairs (fp64 inputs). */
int rti_design_matrix(int basis, const float* lu, const float* lv, int n, double* A);
int rti_pinv(int basis, const float* lu, const float* lv, int n, double rcond, double* pinv);
int rti_basis_eval(int basis, const double* lu, const double* lv, int E, double* out);
/* rti_gram_inverse: the Gram (pseudo-)inverse ginv[k][k] = (AᵀA)⁺ = V Σ⁻² Vᵀ of the same shared
 * design and SVD as rti_pinv (so pinv = ginv·Aᵀ; rcond as there), the operator with which
 * rti_fit_shared_residual turns Aᵀ I into coefficients (analysis.py:293-298). */
int rti_gram_inverse(int basis, const float* lu, const float* lv, int n, double rcond, double* ginv);
/* rti_lsq_factors: the thin SVD A = U Σ Vᵀ of the same shared design (same Jacobi SVD, rcond as in
 * rti_pinv) split as the reference's solve splits it (analysis.py:295-298: c = uᵀL, w = c/s, a = vᵀw):
 * U[n][k] = the orthonormal left singular vectors, W[k][k] = V Σ⁻¹ (W[i][m] = v_im / σ_m), so that
 * pinv = W·Uᵀ.  A truncated σ_m zeroes column m of both; σ_m = 0 without rcond leaves NaN in
 * column m (0·inf), the reference's division by a zero singular value.  Host fp64. */
int rti_lsq_factors(int basis, const float* lu, const float* lv, int n, double rcond, double* U, double* W);

/* ---- device: shared-direction fit (the north_star hot path) ------------------------
 * Replaces interpolate_intensities' per-pixel loop + _interpolate_PTM's solve
 * (analysis.py:321-363, :293-298) when every pixel sees the same light set:
 *   coef[c][p][i] = Σ_n pinv[i][n] · I[c][n][p]
 * pinv: device fp32 [k][N].  I: device, dtype in_dtype (F32, U8 or I32),
 * element (c,n,p) at c*channel_stride + n*light_stride + p
 * (light_stride 0 = P, channel_stride 0 = N*light_stride).
 * coef: device fp32, layout coef_layout, channel stride coef_channel_stride
 * (0 = P*k).  k must equal rti_basis_terms(basis) for some basis, or any
 * 1 <= k <= 16 with kernel = RTI_KERNEL_MFMA. */
int rti_fit_shared(const float* pinv, int k, int N,
                   const void* I, int in_dtype, int64_t P, int C,
                   int64_t light_stride, int64_t channel_stride,
                   float* coef, int coef_layout, int64_t coef_channel_stride,
                   int kernel, rti_stream_t stream);

/* ---- device: shared-direction fit on PIXEL-major stacks (rti_fit_pm.hip) ---------------
 * The same contraction as rti_fit_shared on the reference's own stack layout: compute_intensities
 * returns (R, R, N) arrays (analysis.py:217-219), pixel p's N intensities contiguous:
 *   coef[c][p][i] = Σ_n pinv[i][n] · I[c*channel_stride + p*pixel_stride + n]
 * (pixel_stride 0 = N, channel_stride 0 = P*pixel_stride).  pinv, coef, coef_layout and
 * coef_channel_stride as rti_fit_shared; in_dtype F32 / I32 / U8.
 * AUTO for k <= 9 (the VALU generations form): launches over a channel's 64-pixel blocks in which every wave
 * streams its units HBM -> a private LDS ring by 1-KiB LDS-DMAs (bounded buffer loads), computes one pixel per
 * lane with packed FMAs and keeps the coefficients in registers until the launch's end (one store burst per
 * wave).  AUTO for k = 16, and with RTI_KERNEL_STAGE for any k: the DIRECT form loads 16-pixel groups straight
 * into VGPRs as v_mfma_f32_16x16x4_f32 operands and writes the coefficients in LDS-staged 1-KiB bursts
 * (non-temporal for AUTO k = 16; N % 4 == 0, N <= 256).  RTI_KERNEL_MFMA: the MFMA stream through the LDS ring
 * for every k; RTI_KERNEL_TILE: a double-buffered block form.  All forms compute the same coefficients.
 * These take F32 / I32 stacks, k in {6, 9, 16}, pixel_stride = N, P·N and channel_stride multiples of 4,
 * I 16-byte aligned, coef 8- (VALU generations) or 16-byte aligned, P·k·4 < 2^31 (all but the VALU
 * generations) and N within the LDS budget (rti_fit_shared_pm_plan); RTI_KERNEL_MFMA / TILE fail with
 * RTI_ERR_UNSUPPORTED outside that, AUTO and RTI_KERNEL_VALU run one lane per pixel instead (any shape, uint8
 * included).  Tuning flags (the only bits accepted besides the selector; anything else is RTI_ERR_BAD_ARG):
 * RTI_KERNEL_TILE_WAVES(W) waves per workgroup (direct form: per CU), RTI_KERNEL_CHUNKS(n) (VALU generations:
 * at least n launches per channel; MFMA stream: n× the smallest unit; block form: 16n-pixel blocks; direct
 * form: n launch generations), RTI_KERNEL_ROTATE (VALU generations and MFMA stream: each wave one contiguous
 * run instead of interleaved units), RTI_KERNEL_NT_STORE (MFMA stream k = 16 and direct form: non-temporal
 * coefficient stores), RTI_KERNEL_STAGE (AUTO: the direct form). */
int rti_fit_shared_pm(const float* pinv, int k, int N, const void* I, int in_dtype, int64_t P, int C,
                      int64_t pixel_stride, int64_t channel_stride,
                      float* coef, int coef_layout, int64_t coef_channel_stride,
                      int kernel, rti_stream_t stream);
/* 0 if rti_fit_shared_pm runs one lane per pixel (the fallback) for this shape and kernel selection, else
 * form·10^8 + size·1000 + W: form RTI_PM_VALU_STREAM (AUTO, k <= 9: the VALU generations form) or
 * RTI_PM_MFMA_STREAM (RTI_KERNEL_MFMA) with size = KiB of LDS ring per wave and W = waves per workgroup,
 * RTI_PM_BLOCK (RTI_KERNEL_TILE, or N too small for a ring) with size = pixels per block, or RTI_PM_DIRECT
 * (AUTO k = 16, AUTO | RTI_KERNEL_STAGE) with size = 16-light steps and W = waves per CU. */
#define RTI_PM_VALU_STREAM 1
#define RTI_PM_MFMA_STREAM 2
#define RTI_PM_BLOCK       3
#define RTI_PM_DIRECT      4
int rti_fit_shared_pm_plan(int k, int N, int in_dtype, int64_t P, int C, int64_t pixel_stride,
                           int64_t channel_stride, int kernel);

/* ---- 8-bit stacks: the shared fit on the int8 matrix cores -------------------------
 * The reference's intensities are the uint8 V channel (FeatureMatcher.py:183-184, analysis.py:219).
 * rti_q8_operator (host) turns an fp64 operator pinv[k][N] (rti_pinv) into the fixed-point form the
 * kernel reads: each row scaled to 27-bit fixed point and split into four int8 digits laid out as
 * v_mfma_i32_16x16x64_i8 A fragments, plus per-row scales and sign-flip corrections (layout:
 * smartphone-based-rti_amd/csrc/rti_q8.h).  op must hold rti_q8_operator_bytes(k, N) bytes; it is copied
 * to the device by the caller (16-byte aligned).  Non-finite pinv entries (an exactly rank-deficient light
 * set without rcond) return RTI_ERR_BAD_ARG: those fits keep the fp32 path and its NaN semantics.
 * rti_fit_shared_q8 = rti_fit_shared for U8 stacks: coef[c][p][i] = Σ_n pinv[i][n]·I[c][n][p] with the
 * digit products summed exactly in int32 and combined in fp64 (|Δc_i| <= 2^-28·max_n|pinv[i][n]|·Σ_n I_n,
 * then one fp32 rounding), k ∈ {6, 9, 16}, N <= rti_fit_shared_q8_max_lights().  P, strides, I, op and
 * coef 16-byte aligned (else RTI_ERR_UNSUPPORTED).  kernel: RTI_KERNEL_ONE_LAUNCH or 0 (AUTO). */
int64_t rti_q8_operator_bytes(int k, int N);
int rti_q8_operator(const double* pinv, int k, int N, void* op);
int rti_fit_shared_q8_max_lights(void);
int rti_fit_shared_q8(const void* op, int k, int N, const uint8_t* I, int64_t P, int C,
                      int64_t light_stride, int64_t channel_stride,
                      float* coef, int coef_layout, int64_t coef_channel_stride,
                      int kernel, rti_stream_t stream);

/* ---- device: shared fit of 8-bit stacks on the fp16 matrix cores (rti_fit_h16.hip) ----
 * The same contraction as rti_fit_shared_q8 with the operator split as w·s = hi + lo in fp16 (s a power
 * of two per row: 22 significant bits) and fp32 accumulation (v_mfma_f32_16x16x32_f16): the accuracy of
 * the fp32 stream, a quarter of the q8 form's accumulator registers per pixel: 1024-pixel tiles with two
 * workgroups per CU for k <= 9 (when both fit in the LDS), else 2048-pixel tiles with one; kernel flags
 * (measurement): RTI_KERNEL_TILE_WAVES(1|2|3) forces the 2048- / 1024-pixel tile / 2048 pixels on 16 waves, RTI_KERNEL_CHUNKS(n) n tiles
 * per workgroup, RTI_KERNEL_TILE_DEPTH(1|4|8) 16-pixel groups per read/MFMA round (all bit-identical).
 * rti_h16_operator builds the operator (rti_h16_operator_bytes(k, N)
 * bytes, device copy 16-byte aligned) from the fp64 pseudo-inverse (non-finite entries -> RTI_ERR_BAD_ARG).
 * Arguments, alignment and layouts as rti_fit_shared_q8; N <= rti_fit_shared_h16_max_lights().
 * op (here and for rti_fit_shared_q8) must be the operator built for the SAME k and N: the kernel copies
 * rti_*_operator_bytes(k, N) bytes of it into LDS and the buffer carries no size the ABI could check
 * (the Python layer checks the tensor's size). */
int64_t rti_h16_operator_bytes(int k, int N);
int rti_h16_operator(const double* pinv, int k, int N, void* op);
int rti_fit_shared_h16_max_lights(void);
int rti_fit_shared_h16(const void* op, int k, int N, const uint8_t* I, int64_t P, int C,
                       int64_t light_stride, int64_t channel_stride,
                       float* coef, int coef_layout, int64_t coef_channel_stride,
                       int kernel, rti_stream_t stream);

/* ---- device: per-pixel residuals of the shared-direction fit -----------------------
 * Fit quality next to rti_fit_shared's coefficients (the reference computes the same
 * least-squares solution, analysis.py:280-298, and never reports its residual):
 *   res[c][p]     = sqrt( Σ_n (I[c][n][p] − Σ_i A[n][i]·coef[c][p][i])² / N )
 *   partial[c][b] = Σ of the squared residuals (before /N) of workgroup b's pixels, fp64
 * A: device fp32 design matrix [N][k] (rti_design_matrix rounded to fp32); k ∈ {6, 9, 16}.
 * I / coef / strides exactly as rti_fit_shared.  res: device fp32 [C][P].
 * partial: NULL, or device fp64 [C][rti_fit_residual_blocks(P)] that the caller zeroes
 * (entries past the launched grid stay 0); its sum over b is channel c's residual energy.
 * A second HBM pass over the stack (4 + 4(k+1)/N bytes per pixel·light). */
int64_t rti_fit_residual_blocks(int64_t P);
int rti_fit_residual(const float* A, int k, int N, const void* I, int in_dtype, int64_t P, int C,
                     int64_t light_stride, int64_t channel_stride, const float* coef, int coef_layout,
                     int64_t coef_channel_stride, float* res, double* partial, rti_stream_t stream);

/* ---- device: shared-direction fit + residuals in ONE pass over the stack ---------------
 * The north_star's fit with per-pixel residuals from wavefront reductions, reading the stack once
 * (analysis.py:280-298 is the solve; its residual is never reported by the reference):
 *   b = Aᵀ I[c][·][p], q = ‖I[c][·][p]‖²      accumulated in fp64 (exact fp32×fp32 products)
 *   coef[c][p] = ginv · b                      (fp32 out, layout coef_layout, as rti_fit_shared)
 *   ss = q − coefᵀ b,  res[c][p] = sqrt(ss/N), partial[c][blk] = Σ_workgroup ss (fp64)
 * A: device fp64 design matrix [N][k] (rti_design_matrix); ginv: device fp64 [k][k]
 * (rti_gram_inverse); k ∈ {6, 9, 16}.  I / strides / coef as rti_fit_shared.  res: NULL or device
 * fp32 [C][P]; partial: NULL or device fp64 [C][rti_fit_shared_residual_blocks(P)] the caller zeroes.
 * kernel: RTI_KERNEL_CHUNKS(n) overrides the chunks per lane (0 = AUTO); other bits ignored.
 * 4 + 4(k+1)/N bytes per pixel·light (one stack read + coefficients + residual map). */
int64_t rti_fit_shared_residual_blocks(int64_t P);
int rti_fit_shared_residual(const double* A, const double* ginv, int k, int N, const void* I, int in_dtype,
                            int64_t P, int C, int64_t light_stride, int64_t channel_stride,
                            float* coef, int coef_layout, int64_t coef_channel_stride,
                            float* res, double* partial, int kernel, rti_stream_t stream);
/* The same one-pass fit with the reference's SVD solve instead of the Gram form (analysis.py:295-298):
 *   y = Uᵀ I[c][·][p], q = ‖I[c][·][p]‖²      (fp64),  coef = W · y,  ss = q − yᵀ y
 * U: device fp64 [N][k], W: device fp64 [k][k] (rti_lsq_factors).  Never forms AᵀA, so coefficients
 * keep cond(A)·1e-16 relative accuracy (the Gram form: cond(A)²·1e-16) — what the reference's SVD
 * returns for ill-conditioned light sets.  Every other argument, the traffic and the speed as
 * rti_fit_shared_residual; this is the form rti.fit_with_residual uses. */
int rti_fit_shared_residual_svd(const double* U, const double* W, int k, int N, const void* I, int in_dtype,
                                int64_t P, int C, int64_t light_stride, int64_t channel_stride,
                                float* coef, int coef_layout, int64_t coef_channel_stride,
                                float* res, double* partial, int kernel, rti_stream_t stream);

/* ---- device: per-pixel PTM fit, light vectors generated in-kernel ------------------
 * Fuses compute_intensities' light vectors (analysis.py:221-231) into the
 * per-pixel PTM solve (analysis.py:280-298): for pixel (x, y) of an H×W stack
 * and camera n, l = (cam_n − (x0+x, y0+y, 0)) / ‖·‖ (fp64, rounded to fp32 as
 * the reference stores lx/ly in float32), then the 6×6 normal equations are
 * accumulated and solved in fp64 (Cholesky).  cams: device fp64 [N][3].
 * I: device light-major [N][light_stride] (0 = H*W), dtype F32/U8/I32.
 * coef: device, coef_dtype F32 or F64, layout coef_layout.
 * rcond < 0: reference semantics (exactly singular → NaN coefficients);
 * rcond >= 0: pivots <= rcond²·max_pivot are treated as singular → NaN. */
int rti_fit_perpixel_cam(const double* cams, int N,
                         const void* I, int in_dtype, int H, int W, int64_t light_stride,
                         double x0, double y0, double rcond,
                         void* coef, int coef_dtype, int coef_layout, rti_stream_t stream);

/* ---- device: per-pixel PTM fit from explicit per-pixel light vectors ---------------
 * The exact input of interpolate_intensities (analysis.py:321-363): lu, lv
 * (fp32) and I (F32/U8/I32), each PIXEL-major [P][N] as compute_intensities
 * returns them (analysis.py:217-219).  Same solve and output as above. */
int rti_fit_perpixel_dirs(const float* lu, const float* lv, const void* I, int in_dtype,
                          int N, int64_t P, double rcond,
                          void* coef, int coef_dtype, int coef_layout, rti_stream_t stream);

/* ---- host: light operators for a SHARED light set ---------------------------------
 * A light operator maps the N intensities of a pixel to E outputs: out_e = Σ_n M[e][n] I_n.
 * Both builders return it LIGHT-MAJOR, opT[n][e] (row stride E), fp64, ready for
 * rti_apply_operator after a cast to fp32.
 * rti_rbf_operator: the reference's default interpolator, SciPy Rbf(lu, lv, I,
 *   function='linear') evaluated at (qu_e, qv_e) (analysis.py:249-260):
 *   A_ij = ‖x_i − x_j‖, Φ_ej = ‖q_e − x_j‖, M = Φ A⁻¹ (LU with partial pivoting, fp64).
 *   Returns RTI_ERR_SINGULAR for a singular A (e.g. duplicate light directions), where
 *   SciPy raises LinAlgError.
 * rti_basis_operator: M = B(q) · pinv for PTM/HSH — the fit and the grid evaluation
 *   (analysis.py:293-315) fused into one operator (rcond as in rti_pinv). */
int rti_rbf_operator(const float* lu, const float* lv, int n, const double* qu, const double* qv, int E,
                     double* opT);
int rti_basis_operator(int basis, const float* lu, const float* lv, int n, const double* qu, const double* qv,
                       int E, double rcond, double* opT);

/* ---- device: apply a light operator (MFMA) -------------------------------------------
 * out[c][e][p] = Σ_n opT[n][e] · I[c][n][p]   (v_mfma_f32_16x16x4_f32, fp32 accumulate)
 * opT: device fp32 [N][op_stride] (op_stride >= E).  I as in rti_fit_shared.
 * out: device, out_dtype F32 / F64 / I32 (C truncation, NaN → INT32_MIN) / U8 (clipped),
 * element (c, e, p) at c*out_channel_stride + e*out_row_stride + p (0 = dense).
 * With the RBF operator on the 100×100 grid this is interpolate_intensities +
 * prepare_images_data for the reference's default method in one pass. */
int rti_apply_operator(const float* opT, int E, int N, int64_t op_stride,
                       const void* I, int in_dtype, int64_t P, int C,
                       int64_t light_stride, int64_t channel_stride,
                       void* out, int out_dtype, int64_t out_row_stride, int64_t out_channel_stride,
                       rti_stream_t stream);

/* ---- split-fp16 operator (v_mfma_f32_32x32x16_f16) -----------------------------------
 * The same product as rti_apply_operator at the fp16 MFMA rate: the host splits the fp64
 * operator into two fp16 halves, M·s = hi + lo (s = power of two, max|M·s| < 2^15;
 * inv_scale = 1/s), row-major [E][Kp] with Kp = N rounded up to 16 (16 <= Kp <= 256) and
 * zero padding; the device stages each 128-pixel tile of I as fp16 (a per-tile power-of-two
 * scale for values >= 2^15, plus fp16 remainders when the data is not exact in fp16) and
 * accumulates hi·I + lo·I (+ hi·I_lo) in fp32.  8-bit intensities are exact.
 * Accuracy: operator carried to 22 significant bits, fp32 accumulation (as the fp32 path).
 * op_hi / op_lo: device, 16-byte aligned.  Other arguments as rti_apply_operator. */
int rti_operator_split_f16(const double* opT, int N, int E, int64_t op_stride, int Kp,
                           uint16_t* hi, uint16_t* lo, float* inv_scale);
int rti_apply_operator_f16(const uint16_t* op_hi, const uint16_t* op_lo, int Kp, float inv_scale,
                           int E, int N, const void* I, int in_dtype, int64_t P, int C,
                           int64_t light_stride, int64_t channel_stride,
                           void* out, int out_dtype, int64_t out_row_stride, int64_t out_channel_stride,
                           rti_stream_t stream);

/* ---- device: per-pixel linear RBF (the reference's default, with its own geometry) ---
 * interpolate_intensities (analysis.py:350-363) -> _interpolate_RBF (analysis.py:249-260)
 * for every pixel: nodes x_n = (lu[p][n], lv[p][n]) and values I[p][n], PIXEL-major as
 * compute_intensities returns them; A_ij = ‖x_i − x_j‖, A w = I solved to fp64 accuracy (what
 * SciPy's LU with partial pivoting returns, to rounding: fp64 Gauss-Jordan for N <= 80, an fp32
 * Gauss-Jordan inverse + fp64 iterative refinement to 128 with an fp64 partial-pivoting fallback
 * for ill-conditioned pixels, and a blocked fp64 Cholesky of the bordered system above 128: (r06) left-looking
 * on the fp64 matrix cores to N = 1022 (two pixels per CU to 641), right-looking above),
 * f(q_e) = Σ_n w_n ‖q_e − x_n‖
 * evaluated in fp64 at luv[E][2] (device).
 * out: F64 / F32 / I32 / U8, layout RTI_OUT_PIXEL_MAJOR ([p][e], the reference's
 * [y][x][ly][lx]) or RTI_OUT_EVAL_MAJOR ([e][p], prepare_images_data's [ly][lx][y][x]).
 * status: device int the caller zeroes; set to RTI_ERR_SINGULAR when a pixel's system is
 * singular (that pixel's outputs are NaN), where SciPy raises LinAlgError.  N <= 32768 (RTI_ERR_UNSUPPORTED
 * above): above 1022 the right-looking Cholesky's panels narrow from 16 columns to 1 at N <= 4089 (the panel in
 * LDS), and above 4089 only the 32×32 diagonal block stays in LDS while the panel is solved in place in the slot.
 * Device memory: the call allocates (stream-ordered, hipMallocAsync) and frees a workspace of
 * P·N·(8 + 8) bytes (weights + nodes) plus, for N > 128, one Cholesky slot of ≈ 4·(N+pad)² bytes (L as the matrix
 * cores' 16×4 tiles plus the 64×64 diagonal blocks' factors to N = 1022, then the packed lower triangle) per
 * workgroup on min(P, 2·CUs) workgroups to N = 641, min(P, CUs) above (≈ 0.23 GB at N = 400, 3.3 GB at N = 1800, 6.7 GB at N = 2556, 17 GB at
 * N = 4089 on 256 CUs; above 4089 as many slots as fit in min(48 GiB, 90 % of the device's free memory less the
 * weights and nodes), halved again while the allocation fails, at least one; the environment variable
 * RTI_RBF_GP_WS_BYTES lowers that budget), or, for the fp32 inverses' fallback above N = 138 (reached only
 * with the RTI_RBF_LLT_MIN_N / RTI_RBF_CHOL_OLD measurement switches), 8·N·(N+1) bytes per CU (below: in LDS),
 * plus a P + 1 int list of the fallback's pixels; RTI_ERR_HIP if it cannot. */
int rti_rbf_perpixel(const float* lu, const float* lv, const void* I, int in_dtype, int N, int64_t P,
                     const double* luv, int E, void* out, int out_dtype, int out_layout, int* status,
                     rti_stream_t stream);
/* The same, and fallback_px (NULL, or a device int the caller zeroes) receives the number of pixels the
 * fp32-inverse solvers (81 <= N <= 128) handed to the fp64 partial-pivoting fallback (ill-conditioned:
 * nearly repeated light directions). */
int rti_rbf_perpixel_ex(const float* lu, const float* lv, const void* I, int in_dtype, int N, int64_t P,
                        const double* luv, int E, void* out, int out_dtype, int out_layout, int* status,
                        int* fallback_px, rti_stream_t stream);
/* Cholesky workgroups (= workspace slots) of this thread's most recent rti_rbf_perpixel call (N > 128), 0 for
 * the other solvers.  For tests and timing tools; the results do not depend on it. */
int64_t rti_rbf_last_chol_grid(void);

/* ---- device: light vectors ---------------------------------------------------------
 * The light-vector half of compute_intensities (analysis.py:221-231) for an
 * H×W ROI and N cameras: lu[p][n], lv[p][n] (fp32, pixel-major, p = y*W + x),
 * l = (cam_n − (x0+x, y0+y, 0)) / ‖·‖ in fp64 rounded to fp32. */
int rti_light_dirs(const double* cams, int N, int H, int W, double x0, double y0,
                   float* lu, float* lv, rti_stream_t stream);

/* ---- device: relight evaluator -----------------------------------------------------
 * Replaces _interpolate_PTM's grid evaluation (analysis.py:300-315), the
 * prepare_images_data transpose/truncation (analysis.py:375-411) and the
 * relighting_event lookup + clip (interactive_relighting.py:25-36):
 *   out[e][p] (or out[p][e]) = Σ_i coef[p][i] · b_i(lu_e, lv_e)
 * coef: device, coef_dtype F32 or F64 (arithmetic is done in that type; the
 * F64 PTM path sums the six terms left to right without contraction, exactly
 * as analysis.py:307-312).  luv: device fp64 [E][2] (lu, lv).
 * out_dtype: F32 / F64 value; I32 = C truncation toward zero, NaN/overflow →
 * INT32_MIN (the int32 assignment of analysis.py:407 on x86); U8 = the I32
 * value clipped to [0, 255] (interactive_relighting.py:35-36). */
int rti_relight(const void* coef, int coef_dtype, int basis, int64_t P, int coef_layout,
                const double* luv, int E,
                void* out, int out_dtype, int out_layout, rti_stream_t stream);

/* ---- device: interactive relight frame ----------------------------------------------
 * Replaces relighting_event's per-event image work (interactive_relighting.py:31-38):
 * V = clip(value, 0, 255) (the in-place clip of :35-36), img[:, :, 2] = V (:37), then
 * cv2.cvtColor(img, COLOR_HSV2BGR) (:38) for 8-bit images (OpenCV >= 4.2 HSV2RGB_b,
 * hue range 180, restated in DESIGN.md §4.4).
 *   src_dtype I32: src is the int32 table image [P] the cursor selected
 *     (interpolation_results[int_ly][int_lx]); basis, coef_layout, lu, lv ignored.
 *   src_dtype F32/F64: src is the coefficient map [P][k] / [k][P] (coef_layout) and
 *     value = relight at (lu, lv) truncated to int32 exactly as rti_relight's I32 output.
 * hsv: device uint8 [P][3] (the ROI in HSV, get_ROI(..., hsv=True)); bgr: device uint8
 * [P][3] output, may not alias hsv. */
int rti_relight_frame(const void* src, int src_dtype, int basis, int coef_layout, int64_t P,
                      double lu, double lv, const uint8_t* hsv, uint8_t* bgr, rti_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* RTI_H */
