// Batched weighted Procrustes (Kabsch) + residuals.
//
// Replaces lib/utils.py:164-256 (kabsch_transformation_estimation +
// transformation_residuals) and the batch-coupled zero-weight guard of
// lib/filtering/oanet.py:177-178.
//
// One 256-thread workgroup per pair.  The reference materialises an N x N
// diag_embed(w) and runs torch.svd; here a single pass accumulates the 16
// weighted first/second moments in fp64 (wave shuffles + one LDS round),
// one lane solves the 3x3 SVD by one-sided Jacobi in fp64, and a second pass
// (L2-resident re-read) writes the fp32 residuals.
//
// HBM bytes per pair (algorithmic): N*(24 read xyz pairs + 4 read w + 4 write res)
// (+4+4 when the guard rewrites w and its copy).
#include "common.hpp"
#include "prof.hpp"
#include <math.h>

namespace mvr {

__device__ static void jacobi_svd3(const double H[3][3], double U[3][3], double S[3], double V[3][3]) {
  double a[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) { a[i][j] = H[i][j]; V[i][j] = (i == j) ? 1.0 : 0.0; }
  const int pp[3] = {0, 0, 1}, qq[3] = {1, 2, 2};
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
    for (int r = 0; r < 3; ++r) {
      const int p = pp[r], q = qq[r];
      double al = 0, be = 0, ga = 0;
      for (int i = 0; i < 3; ++i) { al += a[i][p] * a[i][p]; be += a[i][q] * a[i][q]; ga += a[i][p] * a[i][q]; }
      if (ga == 0.0) continue;
      const double nrm = sqrt(al * be);
      if (fabs(ga) <= 1e-15 * nrm) continue;
      off = fmax(off, fabs(ga) / nrm);
      const double ze = (be - al) / (2.0 * ga);
      const double tt = (ze >= 0 ? 1.0 : -1.0) / (fabs(ze) + sqrt(1.0 + ze * ze));
      const double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
      for (int i = 0; i < 3; ++i) {
        const double ap = a[i][p], aq = a[i][q];
        a[i][p] = c * ap - s * aq; a[i][q] = s * ap + c * aq;
        const double vp = V[i][p], vq = V[i][q];
        V[i][p] = c * vp - s * vq; V[i][q] = s * vp + c * vq;
      }
    }
    if (off < 1e-15) break;
  }
  for (int j = 0; j < 3; ++j) S[j] = sqrt(a[0][j] * a[0][j] + a[1][j] * a[1][j] + a[2][j] * a[2][j]);
  // sort singular values descending (permute columns of a and V together)
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2 - i; ++j)
      if (S[j] < S[j + 1]) {
        double tmp = S[j]; S[j] = S[j + 1]; S[j + 1] = tmp;
        for (int k = 0; k < 3; ++k) {
          tmp = a[k][j]; a[k][j] = a[k][j + 1]; a[k][j + 1] = tmp;
          tmp = V[k][j]; V[k][j] = V[k][j + 1]; V[k][j + 1] = tmp;
        }
      }
  if (!(S[0] > 0.0)) {  // zero matrix: LAPACK (torch.svd) returns U = V = I
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) { U[i][j] = (i == j) ? 1.0 : 0.0; V[i][j] = U[i][j]; }
    return;
  }
  const double tiny = S[0] * 1e-13;
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 3; ++i) U[i][j] = (S[j] > tiny) ? a[i][j] / S[j] : 0.0;
  if (!(S[1] > tiny)) {  // rank 1: any unit vector orthogonal to u0
    const double x = U[0][0], y = U[1][0], z = U[2][0];
    double e[3];
    if (fabs(x) <= fabs(y) && fabs(x) <= fabs(z)) { e[0] = 0; e[1] = -z; e[2] = y; }
    else if (fabs(y) <= fabs(z)) { e[0] = -z; e[1] = 0; e[2] = x; }
    else { e[0] = -y; e[1] = x; e[2] = 0; }
    const double n = sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
    for (int i = 0; i < 3; ++i) U[i][1] = e[i] / n;
  }
  if (!(S[2] > tiny)) {  // rank <= 2: u2 = u0 x u1
    U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
    U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
    U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
  }
}

__device__ static double det3(const double M[3][3]) {
  return M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
         M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
}

template <typename T>
struct ProcrustesArgs {
  const T* x1; const T* x2; int64_t x_ps, x_ns;
  T* w; int64_t w_ps;
  const int32_t* guard_pos; T* w_copy; int64_t wc_ps;
  int P, N, normalize; T eps;
  int guard_group;   // pairs [g*G, (g+1)*G) share the guard; 0 = the whole batch
  T* R; T* t; T* res; int64_t res_ps;
  T* res_copy; int64_t rc_ps;
  int32_t* status;
};

// T = float (the fp32 OANet path) or double (fp64 inputs, as torch would compute them).
template <typename T>
__global__ __launch_bounds__(256) void procrustes_kernel(ProcrustesArgs<T> a) {
  __shared__ double red[16 * 4];
  __shared__ T sRt[12];
  __shared__ int sflag;
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
  const T* x1 = a.x1 + (int64_t)p * a.x_ps;
  const T* x2 = a.x2 + (int64_t)p * a.x_ps;
  T* w = a.w ? a.w + (int64_t)p * a.w_ps : nullptr;

  // ---- zero-weight guard (oanet.py:177-178): any pair of the batch (or of this pair's guard
  // group, see ProcrustesArgs::guard_group) with sum(w)==0
  if (tid == 0) sflag = 0;
  __syncthreads();
  if (a.guard_pos) {
    const int q0 = a.guard_group > 0 ? (p / a.guard_group) * a.guard_group : 0;
    const int q1 = a.guard_group > 0 ? min(q0 + a.guard_group, a.P) : a.P;
    int any = 0;
    for (int q = q0 + tid; q < q1; q += blockDim.x) any |= (a.guard_pos[q] == 0);
    if (any) atomicOr(&sflag, 1);
  }
  __syncthreads();
  const bool guard = sflag != 0;
  const T addw = (T)1 / (T)a.N;

  // ---- moments: W, S1[3], S2[3], S12[3][3]
  double m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = 0.0;
  for (int n = tid; n < a.N; n += blockDim.x) {
    T wi = w ? w[n] : (T)1;
    if (guard) {
      wi = wi + addw;
      w[n] = wi;
      if (a.w_copy) a.w_copy[(int64_t)p * a.wc_ps + n] = wi;
    }
    const T* p1 = x1 + (int64_t)n * a.x_ns;
    const T* p2 = x2 + (int64_t)n * a.x_ns;
    const double wd = wi;
    const double u0 = p1[0], u1 = p1[1], u2 = p1[2];
    const double v0 = p2[0], v1 = p2[1], v2 = p2[2];
    m[0] += wd;
    m[1] += wd * u0; m[2] += wd * u1; m[3] += wd * u2;
    m[4] += wd * v0; m[5] += wd * v1; m[6] += wd * v2;
    m[7] += wd * u0 * v0; m[8] += wd * u0 * v1; m[9] += wd * u0 * v2;
    m[10] += wd * u1 * v0; m[11] += wd * u1 * v1; m[12] += wd * u1 * v2;
    m[13] += wd * u2 * v0; m[14] += wd * u2 * v1; m[15] += wd * u2 * v2;
  }
  block_sum<16>(m, red);

  if (tid == 0) {
    // normalisation (utils.py:187-189): w <- w / (sum(w) + eps)
    double scale = 1.0;
    if (a.normalize) scale = 1.0 / ((double)((T)m[0] + a.eps));
    const double W = m[0] * scale;
    const double den = W + (double)a.eps;  // utils.py:203-204
    double mu1[3], mu2[3], S1[3], S2[3];
    for (int i = 0; i < 3; ++i) {
      S1[i] = m[1 + i] * scale; S2[i] = m[4 + i] * scale;
      mu1[i] = S1[i] / den; mu2[i] = S2[i] / den;
    }
    double H[3][3];
    bool finite = true;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        // sum w (x1-mu1)(x2-mu2)^T = S12 - mu1 S2^T - S1 mu2^T + W mu1 mu2^T
        H[i][j] = m[7 + 3 * i + j] * scale - mu1[i] * S2[j] - S1[i] * mu2[j] + W * mu1[i] * mu2[j];
        finite = finite && isfinite(H[i][j]);
      }
    double R[3][3], t[3];
    int st = 0;
    if (!finite) {  // torch.svd raised -> R = I, t = 0, flag (utils.py:216-223)
      st = 1;
      for (int i = 0; i < 3; ++i) { t[i] = 0.0; for (int j = 0; j < 3; ++j) R[i][j] = (i == j); }
    } else {
      double U[3][3], S[3], V[3][3];
      jacobi_svd3(H, U, S, V);
      double VUt[3][3];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) VUt[i][j] = V[i][0] * U[j][0] + V[i][1] * U[j][1] + V[i][2] * U[j][2];
      const double d = det3(VUt) < 0 ? -1.0 : 1.0;  // utils.py:225-227
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = V[i][0] * U[j][0] + V[i][1] * U[j][1] + d * V[i][2] * U[j][2];
      for (int i = 0; i < 3; ++i) t[i] = mu2[i] - (R[i][0] * mu1[0] + R[i][1] * mu1[1] + R[i][2] * mu1[2]);
    }
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) {
        sRt[3 * i + j] = (T)R[i][j];
        a.R[(int64_t)p * 9 + 3 * i + j] = (T)R[i][j];
      }
      sRt[9 + i] = (T)t[i];
      a.t[(int64_t)p * 3 + i] = (T)t[i];
    }
    if (a.status) a.status[p] = st;
  }
  __syncthreads();
  if (!a.res) return;
  T r[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) r[i] = sRt[i];
  for (int n = tid; n < a.N; n += blockDim.x) {
    const T* p1 = x1 + (int64_t)n * a.x_ns;
    const T* p2 = x2 + (int64_t)n * a.x_ns;
    const T u0 = p1[0], u1 = p1[1], u2 = p1[2];
    const T d0 = fma(r[0], u0, fma(r[1], u1, r[2] * u2)) + r[9] - p2[0];
    const T d1 = fma(r[3], u0, fma(r[4], u1, r[5] * u2)) + r[10] - p2[1];
    const T d2 = fma(r[6], u0, fma(r[7], u1, r[8] * u2)) + r[11] - p2[2];
    const T rv = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    a.res[(int64_t)p * a.res_ps + n] = rv;
    if (a.res_copy) a.res_copy[(int64_t)p * a.rc_ps + n] = rv;
  }
}

}  // namespace mvr

template <typename T>
static int procrustes_launch(const T* x1, const T* x2, int64_t x_pstride, int64_t x_nstride, T* w, int64_t w_pstride,
                             const int32_t* guard_pos, T* w_copy, int64_t wc_pstride, int P, int N, int normalize,
                             T eps, T* R, T* t, T* res, int64_t res_pstride, T* res_copy, int64_t rc_pstride,
                             int32_t* status, int guard_group, hipStream_t stream) {
  if (P < 0 || N < 0 || !x1 || !x2 || !R || !t || guard_group < 0) return MVR_EINVAL;
  if (guard_pos && !w) return MVR_EINVAL;
  if (P == 0) return MVR_OK;
  mvr::ProcrustesArgs<T> a{x1, x2, x_pstride, x_nstride, w, w_pstride, guard_pos, w_copy, wc_pstride,
                           P, N, normalize, eps, guard_group, R, t, res, res_pstride, res_copy, rc_pstride, status};
  mvr::ProfScope prof(mvr::PK_PROCRUSTES, 40.0 * P * N, (double)P * N * sizeof(T) * 8, stream);
  hipLaunchKernelGGL(mvr::procrustes_kernel<T>, dim3(P), dim3(256), 0, stream, a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_procrustes(const float* x1, const float* x2, int64_t x_pstride, int64_t x_nstride, float* w,
                              int64_t w_pstride, const int32_t* guard_pos, float* w_copy, int64_t wc_pstride, int P,
                              int N, int normalize, float eps, float* R, float* t, float* res, int64_t res_pstride,
                              float* res_copy, int64_t rc_pstride, int32_t* status, int guard_group,
                              hipStream_t stream) {
  return procrustes_launch<float>(x1, x2, x_pstride, x_nstride, w, w_pstride, guard_pos, w_copy, wc_pstride, P, N,
                                  normalize, eps, R, t, res, res_pstride, res_copy, rc_pstride, status, guard_group,
                                  stream);
}

extern "C" int mvr_procrustes_f64(const double* x1, const double* x2, int64_t x_pstride, int64_t x_nstride, double* w,
                                  int64_t w_pstride, const int32_t* guard_pos, double* w_copy, int64_t wc_pstride,
                                  int P, int N, int normalize, double eps, double* R, double* t, double* res,
                                  int64_t res_pstride, double* res_copy, int64_t rc_pstride, int32_t* status,
                                  int guard_group, hipStream_t stream) {
  return procrustes_launch<double>(x1, x2, x_pstride, x_nstride, w, w_pstride, guard_pos, w_copy, wc_pstride, P, N,
                                   normalize, eps, R, t, res, res_pstride, res_copy, rc_pstride, status, guard_group,
                                   stream);
}
