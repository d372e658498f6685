/* TEST ORACLE / CPU BASELINE ONLY — never linked into the product.
 *
 * CPU restatement (C + OpenMP) of the MinkowskiEngine 0.4 sparse convolution forward that
 * lib/descriptor/fcgf.py:118-227 calls (MinkowskiEngine is not vendored in the reference and cannot run here:
 * parity unpinned, the conventions are those of oracle/fcgf.py):
 *
 *   out[o][c] = sum_k sum_ci feat[nbr[o][k]][ci] * W[k][ci][c]     (nbr = -1: no contribution)
 *
 * plus the kernel map it needs (nbr[o][k] = row of out[o] + sign * off_k * step in the input set, offset index
 * k = (dx+r) + ks (dy+r) + ks^2 (dz+r)), via an open-addressing hash of the input coordinates.  Used by
 * bench.py's cpu_baseline (the FCGF leg on the host's cores, BASELINE.md "C++/OpenMP restatement") and checked
 * against oracle/fcgf.py's numpy restatement by tests/test_oracle_fcgf.py.  fp32 accumulation per output row in
 * the order k, ci (the numpy oracle accumulates per k in a BLAS GEMM: agreement to fp32 rounding, not bits).
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KEY_BIAS (1 << 16)
#define EMPTY 0xFFFFFFFFFFFFFFFFull

static inline uint64_t pack(int b, int x, int y, int z) {
  return ((uint64_t)(uint32_t)b << 51) | ((uint64_t)((uint32_t)(x + KEY_BIAS) & 0x1FFFF) << 34) |
         ((uint64_t)((uint32_t)(y + KEY_BIAS) & 0x1FFFF) << 17) | (uint64_t)((uint32_t)(z + KEY_BIAS) & 0x1FFFF);
}
static inline uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

/* nbr [Mo][ks^3] int64 for out_coords [Mo][4] (b, x, y, z) over in_coords [Mi][4].  Returns 0, -1 on bad args,
 * -2 when out of memory. */
int mvo_kernel_map(const int32_t* in_c, int64_t Mi, const int32_t* out_c, int64_t Mo, int ks, int step,
                   int transposed, int64_t* nbr) {
  if (!in_c || !out_c || !nbr || Mi < 0 || Mo < 0 || ks <= 0 || !(ks & 1) || step <= 0) return -1;
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)(Mi > 0 ? Mi : 1)) cap <<= 1;
  uint64_t* keys = (uint64_t*)malloc(cap * sizeof(uint64_t));
  int64_t* vals = (int64_t*)malloc(cap * sizeof(int64_t));
  if (!keys || !vals) { free(keys); free(vals); return -2; }
  memset(keys, 0xFF, cap * sizeof(uint64_t));
  for (int64_t i = 0; i < Mi; ++i) {   /* first occurrence wins (the sets are distinct anyway) */
    const uint64_t k = pack(in_c[4 * i], in_c[4 * i + 1], in_c[4 * i + 2], in_c[4 * i + 3]);
    uint64_t s = mix(k) & (cap - 1);
    while (keys[s] != EMPTY && keys[s] != k) s = (s + 1) & (cap - 1);
    if (keys[s] == EMPTY) { keys[s] = k; vals[s] = i; }
  }
  const int K = ks * ks * ks, r = ks / 2, sg = transposed ? -1 : 1;
#pragma omp parallel for schedule(static)
  for (int64_t o = 0; o < Mo; ++o) {
    const int32_t* c = out_c + 4 * o;
    for (int k = 0; k < K; ++k) {
      const int dx = k % ks - r, dy = (k / ks) % ks - r, dz = k / (ks * ks) - r;
      const uint64_t key = pack(c[0], c[1] + sg * dx * step, c[2] + sg * dy * step, c[3] + sg * dz * step);
      uint64_t s = mix(key) & (cap - 1);
      int64_t v = -1;
      while (keys[s] != EMPTY) {
        if (keys[s] == key) { v = vals[s]; break; }
        s = (s + 1) & (cap - 1);
      }
      nbr[o * K + k] = v;
    }
  }
  free(keys);
  free(vals);
  return 0;
}

/* One output row of the sparse conv: acc [Cout] scratch.  The AVX2/FMA clone is chosen at load time on hosts that
 * have it (the CPU baseline's speed), the baseline-ISA one elsewhere (the library itself is built for plain x86-64,
 * so it loads on any host).  The clone is this plain function, called from the OpenMP loop body: a target_clones
 * attribute on the function holding the `omp parallel` region would not reach GCC's outlined loop body. */
__attribute__((target_clones("arch=haswell", "default")))
static void conv_row(const float* feat, int64_t Mi, int Cin, const int64_t* nrow, int K, const float* W, int Cout,
                     const float* bias, float* acc, float* dst) {
  for (int c = 0; c < Cout; ++c) acc[c] = 0.f;
  for (int k = 0; k < K; ++k) {
    const int64_t i = nrow[k];
    if (i < 0 || i >= Mi) continue;
    const float* f = feat + i * Cin;
    const float* w = W + (int64_t)k * Cin * Cout;
    for (int ci = 0; ci < Cin; ++ci) {
      const float x = f[ci];
      const float* wr = w + (int64_t)ci * Cout;
#pragma omp simd
      for (int c = 0; c < Cout; ++c) acc[c] += x * wr[c];
    }
  }
  for (int c = 0; c < Cout; ++c) dst[c] = acc[c] + (bias ? bias[c] : 0.f);
}

/* out [Mo][Cout] = sparse conv of feat [Mi][Cin] over nbr [Mo][K] with W [K][Cin][Cout] (+ bias [Cout]). */
int mvo_sparse_conv(const float* feat, int64_t Mi, int Cin, const int64_t* nbr, int64_t Mo, int K, const float* W,
                    int Cout, const float* bias, float* out) {
  if (!feat || !nbr || !W || !out || Mi < 0 || Mo < 0 || Cin <= 0 || Cout <= 0 || K <= 0) return -1;
#pragma omp parallel
  {
    float* acc = (float*)malloc(sizeof(float) * (size_t)Cout);
#pragma omp for schedule(dynamic, 256)
    for (int64_t o = 0; o < Mo; ++o) conv_row(feat, Mi, Cin, nbr + o * K, K, W, Cout, bias, acc, out + o * Cout);
    free(acc);
  }
  return 0;
}

/* The instruction set the sparse conv's clone runs at on this host: 1 AVX2 + FMA (haswell clone), 0 baseline x86-64
 * (recorded with the CPU baseline's numbers) */
int mvo_isa(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
}

/* OpenMP threads of the calls above (the CPU baseline's thread count); returns the previous maximum */
int mvo_set_threads(int n) {
  const int prev = omp_get_max_threads();
  if (n > 0) omp_set_num_threads(n);
  return prev;
}
