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


// ----------------------------------------------------------------------------------------------------
// RANSAC over given correspondences: lib/utils.py:671-709 run_ransac ->
// Open3D 0.9 registration_ransac_based_on_correspondence(TransformationEstimationPointToPoint(False),
// ransac_n = 4, max_correspondence_distance = 0.05, RANSACConvergenceCriteria(50000, 2500)).
// Open3D 0.9's loop (restated; oracle/ransac.py): min(max_iteration, max_validation) iterations; each draws
// ransac_n correspondences with replacement, fits R, t by Umeyama without scaling (fp64), and scores the
// fit over ALL correspondences: inlier iff |R x1 + t - x2|^2 < d^2, fitness = inliers / n,
// rmse = sqrt(sum of inlier d^2 / inliers); the result is the first hypothesis that is best by (fitness
// desc, rmse asc) among those with fitness > 0, identity when none (or n < ransac_n).  Open3D seeds
// std::rand from the clock; here draw j of iteration i for pair p is splitmix64(seed + ctr * golden) % n with
// ctr = (p << 40) | (i << 8) | j — reproducible, and the same on the host (oracle/ransac.py:draws).
//
// One thread per (pair, hypothesis): its 4 draws, the Umeyama fit (jacobi_svd3), then a sequential pass
// over the pair's correspondences staged through LDS in 256-row tiles (every thread of the workgroup reads
// the same row: LDS broadcast), in correspondence order and with rounded fp64 ops (no contraction), so the
// counts and error sums equal the host restatement's bit for bit.  A second kernel picks each pair's best.
// Work per pair: iters x n x ~15 fp64 ops (2500 x 5000: 0.19 GFLOP) — fp64 VALU-bound.
// ----------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ransac_draw(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed + ctr * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct RansacArgs {
  const double* x1; const double* x2; int64_t ps;   // [P][ps] rows of 3 doubles
  const int32_t* n;                                  // [P] correspondences per pair
  int P, iters, rn;
  double d2;                                         // max distance squared
  uint64_t seed;
  int32_t* cnt; double* err;                         // [P][iters]
  double* hyp;                                       // [P][iters][12] (R row-major, t) or null
};

constexpr int RS_TILE = 256;

__global__ __launch_bounds__(256) void ransac_eval_kernel(RansacArgs a) {
#pragma clang fp contract(off)   // hipcc contracts a * b + c into fma by default; the evaluation rounds every op
  __shared__ double tile[RS_TILE][6];
  const int p = blockIdx.y, it = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = a.n[p];
  if (n < a.rn) return;   // uniform: no hypotheses (selection returns identity)
  const double* x1 = a.x1 + (int64_t)p * a.ps;
  const double* x2 = a.x2 + (int64_t)p * a.ps;
  const bool live = it < a.iters;
  double R[3][3], t[3];
  {
    // Umeyama without scaling on the draws: sigma = sum (dst - mu_d)(src - mu_s)^T / k = U S V^T,
    // R = U diag(1, 1, sign(det U det V)) V^T, t = mu_d - R mu_s
    double s[8][3], d[8][3], ms[3] = {0, 0, 0}, md[3] = {0, 0, 0};
    const int k = a.rn;
    for (int j = 0; j < k; ++j) {
      const uint64_t ctr = ((uint64_t)p << 40) | ((uint64_t)(live ? it : 0) << 8) | (uint64_t)j;
      const int64_t c = (int64_t)(ransac_draw(a.seed, ctr) % (uint64_t)n);
      for (int e = 0; e < 3; ++e) {
        s[j][e] = x1[3 * c + e];
        d[j][e] = x2[3 * c + e];
        ms[e] = ms[e] + s[j][e];
        md[e] = md[e] + d[j][e];
      }
    }
    for (int e = 0; e < 3; ++e) {
      ms[e] = ms[e] / k;
      md[e] = md[e] / k;
    }
    double H[3][3];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double acc = 0.0;
        for (int j = 0; j < k; ++j) acc = acc + (d[j][r] - md[r]) * (s[j][c] - ms[c]);
        H[r][c] = acc / k;
      }
    double U[3][3], S[3], V[3][3];
    jacobi_svd3(H, U, S, V);
    const double sg = (det3(U) * det3(V) < 0.0) ? -1.0 : 1.0;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        R[r][c] = (U[r][0] * V[c][0] + U[r][1] * V[c][1]) + (sg * U[r][2]) * V[c][2];
    for (int r = 0; r < 3; ++r)
      t[r] = md[r] - ((R[r][0] * ms[0] + R[r][1] * ms[1]) + R[r][2] * ms[2]);
  }
  if (live && a.hyp) {
    double* h = a.hyp + ((int64_t)p * a.iters + it) * 12;
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) h[3 * r + c] = R[r][c];
      h[9 + r] = t[r];
    }
  }
  int good = 0;
  double e2 = 0.0;
  for (int b0 = 0; b0 < n; b0 += RS_TILE) {
    const int nb = min(RS_TILE, n - b0);
    __syncthreads();
    for (int i = threadIdx.x; i < nb * 6; i += blockDim.x) {
      const int r = i / 6, e = i % 6;
      tile[r][e] = e < 3 ? x1[3 * (int64_t)(b0 + r) + e] : x2[3 * (int64_t)(b0 + r) + e - 3];
    }
    __syncthreads();
    for (int r = 0; r < nb; ++r) {
      const double* q = tile[r];
      double dd = 0.0;
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const double y = ((R[e][0] * q[0] + R[e][1] * q[1]) + R[e][2] * q[2]) + t[e];
        const double df = y - q[3 + e];
        dd = dd + df * df;
      }
      if (dd < a.d2) {
        ++good;
        e2 = e2 + dd;
      }
    }
  }
  if (live) {
    a.cnt[(int64_t)p * a.iters + it] = good;
    a.err[(int64_t)p * a.iters + it] = e2;
  }
}

// best hypothesis per pair: fitness desc, rmse asc, iteration asc (= Open3D's strict-improvement loop)
__global__ __launch_bounds__(256) void ransac_select_kernel(RansacArgs a, double* T, double* fitness, double* rmse,
                                                            int32_t* best) {
  __shared__ int bi[256];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int n = a.n[p];
  auto better = [&](int i, int j) {   // hypothesis i strictly before j in the order
    if (j < 0) return i >= 0;
    if (i < 0) return false;
    const int ci = a.cnt[(int64_t)p * a.iters + i], cj = a.cnt[(int64_t)p * a.iters + j];
    if (ci != cj) return ci > cj;
    const double ri = sqrt(a.err[(int64_t)p * a.iters + i] / ci), rj = sqrt(a.err[(int64_t)p * a.iters + j] / cj);
    if (ri != rj) return ri < rj;
    return i < j;
  };
  int mine = -1;
  if (n >= a.rn)
    for (int i = tid; i < a.iters; i += blockDim.x)
      if (a.cnt[(int64_t)p * a.iters + i] > 0 && better(i, mine)) mine = i;
  bi[tid] = mine;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w && better(bi[tid + w], bi[tid])) bi[tid] = bi[tid + w];
    __syncthreads();
  }
  if (tid != 0) return;
  const int b = bi[0];
  double* Tp = T + (int64_t)p * 16;
  for (int i = 0; i < 16; ++i) Tp[i] = (i % 5 == 0) ? 1.0 : 0.0;
  best[p] = b;
  if (b < 0) {
    fitness[p] = 0.0;
    rmse[p] = 0.0;
    return;
  }
  const int c = a.cnt[(int64_t)p * a.iters + b];
  fitness[p] = (double)c / n;
  rmse[p] = sqrt(a.err[(int64_t)p * a.iters + b] / c);
  // the winner's transformation, recomputed by its own thread in ransac_eval_kernel: read it back from the
  // hypothesis buffer (always allocated by the launcher)
  const double* h = a.hyp + ((int64_t)p * a.iters + b) * 12;
  for (int r = 0; r < 3; ++r) {
    for (int cc = 0; cc < 3; ++cc) Tp[4 * r + cc] = h[3 * r + cc];
    Tp[4 * r + 3] = h[9 + r];
  }
}

}  // namespace mvr

template <typename T>
static int procrustes_launch(const T* x1, const T* x2, int64_t x_pstride, int64_t x_nstride, T* w, int64_t w_pstride,
                             const int32_t* guard_pos, T* w_copy, int64_t wc_pstride, int P, int N, int normalize,
                             T eps, T* R, T* t, T* res, int64_t res_pstride, T* res_copy, int64_t rc_pstride,
                             int32_t* status, int guard_group, hipStream_t stream) {
  if (P < 0 || N < 0 || guard_group < 0) return MVR_EINVAL;
  if (P == 0) return MVR_OK;
  if ((N > 0 && (!x1 || !x2)) || !R || !t) return MVR_EINVAL;
  if (guard_pos && N > 0 && !w) return MVR_EINVAL;
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

extern "C" size_t mvr_ransac_workspace_bytes(int P, int iters) {
  if (P <= 0 || iters <= 0) return 0;
  return (size_t)P * iters * (sizeof(int32_t) + sizeof(double) + 12 * sizeof(double)) + 256;
}

extern "C" int mvr_ransac(const double* x1, const double* x2, int64_t x_pstride, const int32_t* n, int P, int ransac_n,
                          int iters, double max_dist, uint64_t seed, double* T, double* fitness, double* rmse,
                          int32_t* best_iter, double* hyp_out, void* workspace, size_t workspace_bytes,
                          hipStream_t stream) {
  if (P < 0 || ransac_n < 3 || ransac_n > 8 || iters <= 0 || iters >= (1 << 30) || P >= (1 << 23) ||
      !(max_dist > 0.0))
    return MVR_EINVAL;
  if (P == 0) return MVR_OK;
  if (!x1 || !x2 || !n || !T || !fitness || !rmse || !best_iter) return MVR_EINVAL;
  const size_t need = mvr_ransac_workspace_bytes(P, iters) - (hyp_out ? (size_t)P * iters * 12 * sizeof(double) : 0);
  if (!workspace || workspace_bytes < need) return MVR_EINVAL;
  mvr::RansacArgs a{};
  a.x1 = x1; a.x2 = x2; a.ps = x_pstride; a.n = n;
  a.P = P; a.iters = iters; a.rn = ransac_n; a.d2 = max_dist * max_dist; a.seed = seed;
  char* w = static_cast<char*>(workspace);
  a.err = reinterpret_cast<double*>(w);
  a.cnt = reinterpret_cast<int32_t*>(w + (size_t)P * iters * sizeof(double));
  a.hyp = hyp_out ? hyp_out
                  : reinterpret_cast<double*>(w + (((size_t)P * iters * (sizeof(double) + sizeof(int32_t)) + 255) & ~(size_t)255));
  hipLaunchKernelGGL(mvr::ransac_eval_kernel, dim3((iters + 255) / 256, P), dim3(256), 0, stream, a);
  MVR_CHECK_LAUNCH();
  hipLaunchKernelGGL(mvr::ransac_select_kernel, dim3(P), dim3(256), 0, stream, a, T, fitness, rmse, best_iter);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}
