// Feature-space nearest neighbour (Soft_NN) for a batch of fragment pairs.
//
// Replaces lib/layers.py:44-88 (Soft_NN.forward) + lib/utils.py:968-992
// (pairwise_distance) + the pair gather of lib/utils.py:850-885 and the xs
// assembly of lib/utils.py:915.  The reference materialises the [P,N,M]
// distance and softmax matrices (100 MB per pair); here they never leave
// registers:
//   * S^T = Ft . Fs^T on v_mfma_f32_32x32x2_f32 (the QUERY index is the lane
//     column, so each lane owns one query's running softmax state),
//   * logits (2 fs.ft - |ft|^2) / tau^2 (|fs|^2 is constant per query and
//     cancels in the softmax / argmax),
//   * flash-style online softmax in base 2 over 32-target chunks, and the
//     3-wide weighted coordinate sum accumulated in fp32 registers,
//   * argmax tracking for the straight-through ('st') and 'hard' modes.
// Targets stream through double-buffered LDS in 128-row stages shared by the
// 4 waves (128 queries) of a workgroup.
//
// FLOPs per pair ~ 2*N*M*C (MFMA) + N*M*(exp + 5 FMA); HBM: features/coords of
// the two fragments (L2/MALL-resident across the pairs that share them).
#include "common.hpp"
#include "prof.hpp"

namespace mvr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int NN_STAGE = 128;      // targets per LDS stage
constexpr int NN_FLD = 32 + 4;     // padded LDS row (floats) for 32-dim features
constexpr float NN_NEG = -3.0e38f;

struct NNArgs {
  const float* Fq; int64_t fq_fs;    // query features [*][Nq][32], fragment stride (elements)
  const float* Ft; int64_t ft_fs;    // target features [*][Mt][32]
  const float* Xq; int64_t xq_fs;    // query coords (optional: output then holds [x_q | x_corr])
  const float* Xt; int64_t xt_fs;    // target coords [*][Mt][3]
  const int64_t* pairs;              // [P][2] (query fragment, target fragment)
  int P, Nq, Mt;
  float k2;                          // log2(e) / tau^2
  int mode;                          // 0 soft, 1 argmax (soft+st / hard)
  float* out; int64_t o_ps, o_ns;    // out(p,n,:) = [x_q(0..2) |] x_corr(0..2)
  int32_t* idx;                      // optional argmax index [P][Nq]
};

__global__ __launch_bounds__(256) void feat_nn_kernel(NNArgs a) {
  __shared__ float Fs[2][NN_STAGE][NN_FLD];
  __shared__ float4 Xs[2][NN_STAGE];   // xyz + |f|^2
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l32 = lane & 31, kh = lane >> 5;
  const int p = blockIdx.y;
  const int64_t src = a.pairs[2 * p], tgt = a.pairs[2 * p + 1];
  const float* Fq = a.Fq + src * a.fq_fs;
  const float* Ft = a.Ft + tgt * a.ft_fs;
  const float* Xt = a.Xt + tgt * a.xt_fs;
  const int j = blockIdx.x * 128 + wid * 32 + l32;  // this lane's query
  const bool jok = j < a.Nq;

  // query operand: fs[j][16*kh + e], e = 0..15 (k-order permuted identically for A and B)
  float q[16];
  {
    const float4* qp = reinterpret_cast<const float4*>(Fq + (int64_t)(jok ? j : 0) * 32 + 16 * kh);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float4 t = qp[v];
      q[4 * v] = t.x; q[4 * v + 1] = t.y; q[4 * v + 2] = t.z; q[4 * v + 3] = t.w;
    }
  }

  auto stage_load = [&](int buf, int t0) {
    // 128 targets x 32 floats = 1024 float4, 4 per thread
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      const int row = e >> 3, c4 = e & 7;
      const int gi = t0 + row;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gi < a.Mt) v = reinterpret_cast<const float4*>(Ft + (int64_t)gi * 32)[c4];
      *reinterpret_cast<float4*>(&Fs[buf][row][4 * c4]) = v;
    }
  };
  auto stage_finish = [&](int buf, int t0) {
    if (tid < NN_STAGE) {
      const int gi = t0 + tid;
      float n2 = 0.f;
#pragma unroll
      for (int c = 0; c < 32; ++c) n2 = fmaf(Fs[buf][tid][c], Fs[buf][tid][c], n2);
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gi < a.Mt) {
        const float* xp = Xt + (int64_t)gi * 3;
        x = make_float4(xp[0], xp[1], xp[2], n2);
      }
      Xs[buf][tid] = x;
    }
  };

  float run_m = NN_NEG, run_s = 0.f, ax = 0.f, ay = 0.f, az = 0.f;
  float best = NN_NEG;
  int besti = 0x7fffffff;

  const int nst = (a.Mt + NN_STAGE - 1) / NN_STAGE;
  stage_load(0, 0);
  __syncthreads();
  stage_finish(0, 0);
  __syncthreads();
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    const int t0 = st * NN_STAGE;
    if (st + 1 < nst) stage_load(cur ^ 1, t0 + NN_STAGE);
#pragma unroll 1
    for (int sub = 0; sub < NN_STAGE / 32; ++sub) {
      const int i0 = sub * 32;
      if (t0 + i0 >= a.Mt) break;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* frow = &Fs[cur][i0 + l32][16 * kh];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 f = *reinterpret_cast<const float4*>(frow + 4 * v);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.x, q[4 * v + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.y, q[4 * v + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.z, q[4 * v + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.w, q[4 * v + 3], acc, 0, 0, 0);
      }
      // acc[r] = ft[i] . fs[j],  i = i0 + (r&3) + 8(r>>2) + 4kh
      float z[16];
      float cm = NN_NEG;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int il = i0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
        const float tn = Xs[cur][il].w;
        float v = (2.f * acc[r] - tn) * a.k2;
        if (t0 + il >= a.Mt) v = NN_NEG;
        z[r] = v;
        cm = fmaxf(cm, v);
        if (a.mode == 1 && v > best) {  // strict '>' keeps the first maximum within a lane
          best = v;
          besti = t0 + il;
        }
      }
      if (a.mode == 0) {
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        const float nm = fmaxf(run_m, cm);
        const float sc = __builtin_amdgcn_exp2f(run_m - nm);
        run_s *= sc; ax *= sc; ay *= sc; az *= sc;
        run_m = nm;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int il = i0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
          const float4 xt = Xs[cur][il];
          const float pr = __builtin_amdgcn_exp2f(z[r] - nm);
          run_s += pr;
          ax = fmaf(pr, xt.x, ax);
          ay = fmaf(pr, xt.y, ay);
          az = fmaf(pr, xt.z, az);
        }
      }
    }
    __syncthreads();
    if (st + 1 < nst) {
      stage_finish(cur ^ 1, t0 + NN_STAGE);
      __syncthreads();
    }
    cur ^= 1;
  }

  float ox, oy, oz;
  if (a.mode == 0) {
    const float s = run_s + __shfl_xor(run_s, 32, 64);
    ox = (ax + __shfl_xor(ax, 32, 64)) / s;
    oy = (ay + __shfl_xor(ay, 32, 64)) / s;
    oz = (az + __shfl_xor(az, 32, 64)) / s;
  } else {
    const float ob = __shfl_xor(best, 32, 64);
    const int oi = __shfl_xor(besti, 32, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
    const float* xp = Xt + (int64_t)(besti < a.Mt ? besti : 0) * 3;
    ox = xp[0]; oy = xp[1]; oz = xp[2];
  }
  if (jok && kh == 0) {
    float* o = a.out + (int64_t)p * a.o_ps + (int64_t)j * a.o_ns;
    if (a.Xq) {
      const float* xq = a.Xq + src * a.xq_fs + (int64_t)j * 3;
      o[0] = xq[0]; o[1] = xq[1]; o[2] = xq[2];
      o += 3;
    }
    o[0] = ox; o[1] = oy; o[2] = oz;
    if (a.idx && a.mode == 1) a.idx[(int64_t)p * a.Nq + j] = besti;
  }
}

// rows gather: dst[i][:] = src[idx[i]][:]  (Sampler.forward, lib/layers.py:151-152)
__global__ void gather_rows_kernel(const float* __restrict__ src, int C, const int64_t* __restrict__ idx, int n,
                                   float* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * C) return;
  const int64_t i = e / C, c = e - i * C;
  dst[e] = src[idx[i] * C + c];
}

}  // namespace mvr

extern "C" int mvr_feat_nn(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride, const float* Xq,
                           int64_t xq_fstride, const float* Xt, int64_t xt_fstride, const int64_t* pairs, int P,
                           int Nq, int Mt, int C, float inv_tau2, int mode, float* out, int64_t out_pstride,
                           int64_t out_nstride, int32_t* idx_out, hipStream_t stream) {
  if (!Fq || !Ft || !Xt || !pairs || !out || P < 0 || Nq < 0 || Mt <= 0) return MVR_EINVAL;
  if (C != 32) return MVR_EINVAL;  // FCGF descriptor width (fcgf.py:108 out_channels=32)
  if ((reinterpret_cast<uintptr_t>(Fq) & 15) || (reinterpret_cast<uintptr_t>(Ft) & 15) || (fq_fstride & 3) ||
      (ft_fstride & 3))
    return MVR_EINVAL;
  if (mode != 0 && mode != 1) return MVR_EINVAL;
  if (P == 0 || Nq == 0) return MVR_OK;
  mvr::NNArgs a{Fq, fq_fstride, Ft, ft_fstride, Xq, xq_fstride, Xt, xt_fstride, pairs, P, Nq, Mt,
                inv_tau2 * 1.4426950408889634f, mode, out, out_pstride, out_nstride, idx_out};
  mvr::ProfScope prof(mvr::PK_FEAT_NN, 2.0 * P * (double)Nq * Mt * C, (double)P * (Nq + Mt) * (C + 3) * 4 + P * Nq * 24.0,
                      stream);
  hipLaunchKernelGGL(mvr::feat_nn_kernel, dim3((Nq + 127) / 128, P), dim3(256), 0, stream, a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_gather_rows(const float* src, int C, const int64_t* idx, int n, float* dst, hipStream_t stream) {
  if (!src || !idx || !dst || C <= 0 || n < 0) return MVR_EINVAL;
  if (n == 0) return MVR_OK;
  const int64_t tot = (int64_t)n * C;
  hipLaunchKernelGGL(mvr::gather_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, src, C, idx, n,
                     dst);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}
