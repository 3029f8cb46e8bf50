// Batched NT GEMM with a sum over the batch, on MFMA: C[M, N] (fp32) = sum_b A_b . B_b^T with
// A_b = M x K and B_b = N x K row-major bf16 blocks, b < nb.  This is the filter gradient of a
// 1x1 stride-1 convolution of NCHW activations (reference: LibMatrixCuDNN.java
// conv2d_backward_filter; libmatrixdnn.cpp's per-image t(dout) %*% im2col products):
//     dW[f, c] = sum_img sum_p dout[img, f, p] * X[img, c, p]      (A = dout, B = X, K = H*W)
// Both operands are K-contiguous, so the tiles are 16-B (K % 8 == 0) or 8-B (K % 4 == 0) vector
// loads along the pixels instead of the bounds-checked 2-B gathers of dnn.hip's implicit-GEMM
// backward filter.  The (image, K step) range is the split-K axis: block z reduces its share of it
// into its own fp32 slab slice and a second pass sums the S slices (deterministic, no atomics).
// 128 x 128 tiles (64-row tiles for M or N <= 64), 4 waves of 64 x 64 (or 32 x 64), K steps of 32
// double-buffered in LDS with register prefetch: one barrier per step.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_wg {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256, BK = 32, LDK = 48;   // LDS row pitch 96 B: conflict-free for ds_read_b128's lane groups

struct WG {
  const uint16_t* A;
  const uint16_t* B;
  float* out;          // C (S == 1) or the slab S x M x N
  int M, N, K, nb, S;
  int64_t sa, sb;      // batch strides (elements)
  int tm, tn;
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// 8 consecutive k of row `row` of one operand block (rows < R, k < K), as a 16-B value
template <int VEC>
__device__ __forceinline__ uint4 load8(const uint16_t* __restrict__ base, int R, int K, int row, int k) {
  uint4 z{0, 0, 0, 0};
  if (row >= R) return z;
  const uint16_t* p = base + (int64_t)row * K + k;
  if (VEC == 8) {
    if (k + 8 <= K) return *(const uint4*)p;
  } else if (VEC == 4) {
    if (k + 8 <= K) {
      const uint2 a = *(const uint2*)p, b = *(const uint2*)(p + 4);
      return uint4{a.x, a.y, b.x, b.y};
    }
  }
  uint16_t v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (k + e < K) ? p[e] : (uint16_t)0;
  return uint4{(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
               (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
}

template <int TM, int TN, int VEC>
__global__ void __launch_bounds__(NT) wgrad_kernel(WG g) {
  constexpr int FI = TM / 32, FJ = TN / 32;            // fragments per wave (2 x 2 waves)
  constexpr int AV = TM * (BK / 8) / NT, BV = TN * (BK / 8) / NT;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][TM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][TN * LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = g.tm * g.tn;
  const int tile = wgid % ntile, z = wgid / ntile;
  const int bm = tile % g.tm, bn = tile / g.tm;
  const int m0 = bm * TM, n0 = bn * TN;
  // block z reduces the K steps [s0, s1) of the flattened (image, K step) range
  const int ksteps = (g.K + BK - 1) / BK;
  const int64_t all = (int64_t)g.nb * ksteps;
  const int s0 = (int)(z * all / g.S), s1 = (int)((z + 1) * all / g.S);
  const int total = s1 - s0;
  uint4 av[AV], bv[BV];
  auto load = [&](int s) {
    const int b = (s0 + s) / ksteps, k0 = ((s0 + s) % ksteps) * BK;
    const uint16_t* Ab = g.A + (int64_t)b * g.sa + (int64_t)m0 * g.K;
    const uint16_t* Bb = g.B + (int64_t)b * g.sb + (int64_t)n0 * g.K;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int e = v * NT + tid;
      av[v] = load8<VEC>(Ab, g.M - m0, g.K, e >> 2, k0 + (e & 3) * 8);
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int e = v * NT + tid;
      bv[v] = load8<VEC>(Bb, g.N - n0, g.K, e >> 2, k0 + (e & 3) * 8);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int e = v * NT + tid;
      *(uint4*)&As[buf][(e >> 2) * LDK + (e & 3) * 8] = av[v];
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int e = v * NT + tid;
      *(uint4*)&Bs[buf][(e >> 2) * LDK + (e & 3) * 8] = bv[v];
    }
  };
  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0, 0, 0, 0};
  if (total > 0) {
    load(0);
    store(0);
    __syncthreads();
  }
  const int kc = (lane >> 4) * 8;
  for (int s = 0; s < total; ++s) {
    const bool more = s + 1 < total;
    if (more) load(s + 1);
    const uint16_t* Ab = As[s & 1];
    const uint16_t* Bb = Bs[s & 1];
    bf8 fa[FI], fb[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i) fa[i] = *(const bf8*)&Ab[(wr * (TM / 2) + i * 16 + (lane & 15)) * LDK + kc];
#pragma unroll
    for (int j = 0; j < FJ; ++j) fb[j] = *(const bf8*)&Bb[(wc * (TN / 2) + j * 16 + (lane & 15)) * LDK + kc];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (more) {
      store((s + 1) & 1);
      __syncthreads();
    }
  }
  float* o = g.out + (int64_t)z * g.M * g.N;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wr * (TM / 2) + i * 16 + (lane >> 4) * 4 + r;
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int n = n0 + wc * (TN / 2) + j * 16 + (lane & 15);
        if (n < g.N) o[(int64_t)m * g.N + n] = acc[i][j][r];
      }
    }
}

// C[i] = sum_s slab[s, i]
__global__ void __launch_bounds__(256) slab_sum(const float* __restrict__ slab, float* __restrict__ C, int64_t n, int S) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float a = 0.f;
    for (int s = 0; s < S; ++s) a += slab[(int64_t)s * n + i];
    C[i] = a;
  }
}

// ---- 3x3 stride-1 pad-1 filter gradient -------------------------------------------------------
// dW[f, c, kh, kw] = sum_img sum_(oh, ow) dout[img, f, oh, ow] * X[img, c, oh + kh - 1, ow + kw - 1]
// M = 64 filter rows x N = 32 channels x 9 taps per block, K = output pixels.  The K axis runs over
// rows padded to Wp = the power of two >= max(W, 8) pixels (dout is zero in the padding), so that every 8-pixel
// MFMA operand run lies inside one output row at an 8-aligned column.  A chunk of RB = 64 / Wp
// output rows of one image (64 pixels, two K steps) is staged per iteration:
//   Ds[f][px]              dout rows (vector loads when W % 8 / 4 / 2 == 0)
//   Xs[kw][c][prow][owp]   the RB + 2 input rows the chunk's taps read, three copies shifted by
//                          kw - 1 columns -- so the B operand of tap (kh, kw) for a run starting at
//                          (row, owp0) is one aligned 16-B LDS read at [kw][c][row + kh][owp0]
// Channel pitch CP = (RB + 2) * Wp + 8 elements (16 B mod 128 B: the 16 channels of a fragment
// read land in distinct bank groups).  Each wave owns (TM / 2) filters x 16 channels x 9 taps
// (FI x 9 accumulators), so a K step is FI + 9 fragment reads for 9 * FI MFMAs.  Chunks (image,
// row block) are split over S blocks per tile; partial sums go to an S x F x (9C) slab.
constexpr int XIT = 3;       // X patch items (channel, row, 8-column group) per thread

struct WG3 {
  const uint16_t* X;   // N x C x H x W
  const uint16_t* D;   // N x F x H x W
  float* out;          // dW (S == 1) or the S x F x 9C slab
  int N, C, H, W, F, S;
  int Wp, RB, nrb;     // padded row width, rows per chunk, chunks per image
  int tm, tn;
};

template <int TM, int DV>
__global__ void __launch_bounds__(NT, 2) wgrad3_kernel(WG3 g) {
  constexpr int FI = TM / 32, FJ = 9;
  constexpr int DP = 64 + 8;                           // Ds pitch (64 pixels per chunk)
  constexpr int DIT = TM * 8 / NT;                     // dout items (filter row, 8-pixel group) per thread
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  uint16_t* Ds = sm;                                   // TM x DP
  const int CP = (g.RB + 2) * g.Wp + 8;
  uint16_t* Xs = sm + TM * DP;                         // 3 x 32 x CP
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = g.tm * g.tn;
  const int tile = wgid % ntile, z = wgid / ntile;
  const int bm = tile % g.tm, bn = tile / g.tm;
  const int m0 = bm * TM, c0 = bn * 32;
  const int units = g.N * g.nrb;
  const int u0 = (int)((int64_t)z * units / g.S), u1 = (int)((int64_t)(z + 1) * units / g.S);
  const int HW = g.H * g.W, Wp = g.Wp, RB = g.RB;
  const int ngx = Wp / 8, nxitems = 32 * (RB + 2) * ngx;
  // per-thread staging items, decoded once: X patch (channel, patch row, 8-column group) and
  // dout (filter row, 8-pixel group)
  int xl[XIT], xc[XIT], xr[XIT], xg[XIT];
#pragma unroll
  for (int it = 0; it < XIT; ++it) {
    const int q = it * NT + tid;
    xl[it] = -1;
    xc[it] = xr[it] = xg[it] = 0;
    if (q < nxitems) {
      const int gx = q % ngx, rest = q / ngx, prow = rest % (RB + 2), c = rest / (RB + 2);
      xl[it] = c * CP + prow * Wp + gx * 8;
      xc[it] = c; xr[it] = prow; xg[it] = gx;
    }
  }
  // chunk u (image, row block): load() fetches its X patch items and dout items into registers
  // (issued before the current chunk's MFMAs, so the loads overlap them), put() writes them to LDS
  uint32_t xv[XIT][5];                                 // input columns gx*8-1 .. gx*8+8, bf16 pairs
  uint4 dreg[DIT];
  auto load = [&](int u) {
    const int img = u / g.nrb, r0 = (u - img * g.nrb) * RB;
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      uint16_t v[10];
#pragma unroll
      for (int e = 0; e < 10; ++e) v[e] = 0;
      const int ih = r0 - 1 + xr[it];
      if (xl[it] >= 0 && c0 + xc[it] < g.C && (unsigned)ih < (unsigned)g.H) {
        const uint16_t* row = g.X + ((int64_t)img * g.C + c0 + xc[it]) * HW + (int64_t)ih * g.W;
#pragma unroll
        for (int e = 0; e < 10; ++e) {
          const int iw = xg[it] * 8 - 1 + e;
          if ((unsigned)iw < (unsigned)g.W) v[e] = row[iw];
        }
      }
#pragma unroll
      for (int e = 0; e < 5; ++e) xv[it][e] = (uint32_t)v[2 * e] | ((uint32_t)v[2 * e + 1] << 16);
    }
#pragma unroll
    for (int it = 0; it < DIT; ++it) {
      const int q = it * NT + tid, f = q >> 3, grp = q & 7;
      const int px = grp * 8, oh = r0 + px / Wp, ow0 = px % Wp;
      uint4 d{0, 0, 0, 0};
      if (m0 + f < g.F && oh < g.H) {
        const uint16_t* p = g.D + ((int64_t)img * g.F + m0 + f) * HW + (int64_t)oh * g.W + ow0;
        if (DV == 8 && ow0 + 8 <= g.W) {
          d = *(const uint4*)p;
        } else {
          uint16_t v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 0;
          if (DV >= 2) {
#pragma unroll
            for (int e = 0; e < 8; e += (DV >= 2 ? DV : 1)) {
              if (ow0 + e + DV <= g.W) {
                if (DV == 4) {
                  const uint2 w2 = *(const uint2*)(p + e);
                  v[e] = (uint16_t)w2.x; v[e + 1] = (uint16_t)(w2.x >> 16);
                  v[e + 2] = (uint16_t)w2.y; v[e + 3] = (uint16_t)(w2.y >> 16);
                } else {
                  const uint32_t w1 = *(const uint32_t*)(p + e);
                  v[e] = (uint16_t)w1; v[e + 1] = (uint16_t)(w1 >> 16);
                }
              } else {
#pragma unroll
                for (int h = 0; h < (DV >= 2 ? DV : 1); ++h)
                  if (ow0 + e + h < g.W) v[e + h] = p[e + h];
              }
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (ow0 + e < g.W) v[e] = p[e];
          }
          d = uint4{(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                    (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
        }
      }
      dreg[it] = d;
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      if (xl[it] < 0) continue;
      // copy kw holds input columns gx*8 + kw - 1 .. +8: the packed pairs shifted by kw halves
      *(uint4*)&Xs[xl[it]] = uint4{xv[it][0], xv[it][1], xv[it][2], xv[it][3]};
      *(uint4*)&Xs[32 * CP + xl[it]] =
          uint4{__builtin_amdgcn_alignbit(xv[it][1], xv[it][0], 16), __builtin_amdgcn_alignbit(xv[it][2], xv[it][1], 16),
                __builtin_amdgcn_alignbit(xv[it][3], xv[it][2], 16), __builtin_amdgcn_alignbit(xv[it][4], xv[it][3], 16)};
      *(uint4*)&Xs[64 * CP + xl[it]] = uint4{xv[it][1], xv[it][2], xv[it][3], xv[it][4]};
    }
#pragma unroll
    for (int it = 0; it < DIT; ++it) {
      const int q = it * NT + tid, f = q >> 3, grp = q & 7;
      *(uint4*)&Ds[f * DP + grp * 8] = dreg[it];
    }
  };
  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0, 0, 0, 0};
  const int grp = lane >> 4;
  if (u0 < u1) {
    load(u0);
    put();
    __syncthreads();
  }
  for (int u = u0; u < u1; ++u) {
    const bool more = u + 1 < u1;
    if (more) load(u + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int px = ks * 32 + grp * 8, prow = px / Wp, ow0 = px - prow * Wp;
      bf8 fa[FI];
#pragma unroll
      for (int i = 0; i < FI; ++i) fa[i] = *(const bf8*)&Ds[(wr * (TM / 2) + i * 16 + (lane & 15)) * DP + px];
      const uint16_t* xb = Xs + (wc * 16 + (lane & 15)) * CP + prow * Wp + ow0;
#pragma unroll
      for (int t = 0; t < FJ; ++t) {
        const bf8 fb = *(const bf8*)&xb[(t % 3) * 32 * CP + (t / 3) * Wp];
#pragma unroll
        for (int i = 0; i < FI; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][t], 0, 0, 0);
      }
    }
    if (more) {
      __syncthreads();                                 // every wave is done with this chunk
      put();
      __syncthreads();
    }
  }
  float* o = g.out + (int64_t)z * g.F * g.C * 9;
  const int c = c0 + wc * 16 + (lane & 15);
  if (c < g.C) {
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = m0 + wr * (TM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (f >= g.F) continue;
#pragma unroll
        for (int t = 0; t < FJ; ++t) o[((int64_t)f * g.C + c) * 9 + t] = acc[i][t][r];
      }
  }
}

template <int TM, int TN>
void launch(const WG& g, dim3 grid, hipStream_t st, int vec) {
  if (vec == 8) hipLaunchKernelGGL((wgrad_kernel<TM, TN, 8>), grid, dim3(NT), 0, st, g);
  else if (vec == 4) hipLaunchKernelGGL((wgrad_kernel<TM, TN, 4>), grid, dim3(NT), 0, st, g);
  else hipLaunchKernelGGL((wgrad_kernel<TM, TN, 1>), grid, dim3(NT), 0, st, g);
}

}  // namespace sysml_wg

extern "C" {

// Number of batch splits the launcher uses for this shape (the caller sizes the slab S x M x N).
int sysml_wgrad_splits(int M, int N, int K, int nb) {
  const int tm = (M + (M <= 64 ? 63 : 127)) / (M <= 64 ? 64 : 128);
  const int tn = (N + (N <= 64 ? 63 : 127)) / (N <= 64 ? 64 : 128);
  const int tiles = tm * tn;
  // ~512 blocks (two per CU) and at least 8 K steps per block; the slab (S x M x N fp32, written
  // once and read once by the reduction) at most ~32 MB
  int S = (512 + tiles - 1) / tiles;
  const int64_t ks = (K + sysml_wg::BK - 1) / sysml_wg::BK;
  const int64_t maxs = (int64_t)nb * ks / 8 > 0 ? (int64_t)nb * ks / 8 : 1;
  if (S > maxs) S = (int)maxs;
  while (S > 1 && (int64_t)S * M * N * 4 > (32LL << 20)) S >>= 1;
  if (S < 1) S = 1;
  return S;
}

// C (M x N fp32) = sum_b A_b . B_b^T; A_b = A + b*sa (M x K), B_b = B + b*sb (N x K), bf16
// row-major.  slab: S x M x N fp32 scratch when sysml_wgrad_splits(...) > 1 (may be null then not).
int sysml_wgrad_nt(const void* A, const void* B, float* C, float* slab, int M, int N, int K, int nb, int64_t sa,
                   int64_t sb, void* stream) {
  using namespace sysml_wg;
  if (M <= 0 || N <= 0 || K <= 0 || nb <= 0) return -1;
  const int S = sysml_wgrad_splits(M, N, K, nb);
  if (S > 1 && slab == nullptr) return -1;
  WG g;
  g.A = (const uint16_t*)A;
  g.B = (const uint16_t*)B;
  g.out = S > 1 ? slab : C;
  g.M = M; g.N = N; g.K = K; g.nb = nb; g.S = S;
  g.sa = sa; g.sb = sb;
  const int TMv = M <= 64 ? 64 : 128, TNv = N <= 64 ? 64 : 128;
  g.tm = (M + TMv - 1) / TMv;
  g.tn = (N + TNv - 1) / TNv;
  // vector width: every row start must be aligned to it (row stride K, batch strides)
  int vec = 1;
  if (K % 8 == 0 && sa % 8 == 0 && sb % 8 == 0) vec = 8;
  else if (K % 4 == 0 && sa % 4 == 0 && sb % 4 == 0) vec = 4;
  if (((uintptr_t)A | (uintptr_t)B) & 15) vec = 1;
  const dim3 grid((unsigned)(g.tm * g.tn * S));
  hipStream_t st = (hipStream_t)stream;
  if (TMv == 64 && TNv == 64) launch<64, 64>(g, grid, st, vec);
  else if (TMv == 64) launch<64, 128>(g, grid, st, vec);
  else if (TNv == 64) launch<128, 64>(g, grid, st, vec);
  else launch<128, 128>(g, grid, st, vec);
  if (S > 1) {
    const int64_t n = (int64_t)M * N;
    int64_t gb = (n + 255) / 256;
    if (gb > 2048) gb = 2048;
    hipLaunchKernelGGL(slab_sum, dim3((unsigned)gb), dim3(256), 0, st, (const float*)slab, C, n, S);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Batch splits of the 3x3 filter gradient for this shape (the caller sizes the S x F x 9C slab).
int sysml_wgrad3_splits(int N, int C, int H, int W, int F) {
  int Wp = 8;                                          // a power of two: RB * Wp = 64 pixels exactly
  while (Wp < W) Wp <<= 1;
  if (Wp > 64) return -1;
  const int RB = 64 / Wp, nrb = (H + RB - 1) / RB;
  const int tm = (F + 63) / 64, tn = (C + 31) / 32;
  int S = (1024 + tm * tn - 1) / (tm * tn);
  const int units = N * nrb;
  const int maxs = units / 2 > 0 ? units / 2 : 1;     // >= 2 chunks per block
  if (S > maxs) S = maxs;
  if (S < 1) S = 1;
  return S;
}

// dW (F x 9C fp32, [f][c][kh][kw]) of a 3x3 stride-1 pad-1 convolution from X (N x C x H x W) and
// dout (N x F x H x W), bf16.  slab: S x F x 9C fp32 when sysml_wgrad3_splits(...) > 1.
// -1: not covered (W > 64).
int sysml_wgrad3(const void* X, const void* D, float* dW, float* slab, int N, int C, int H, int W, int F,
                 void* stream) {
  using namespace sysml_wg;
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || F <= 0) return -1;
  if ((int64_t)N * C * H * W >= (1LL << 31) || (int64_t)N * F * H * W >= (1LL << 31)) return -1;
  const int S = sysml_wgrad3_splits(N, C, H, W, F);
  if (S < 1 || (S > 1 && slab == nullptr)) return -1;
  WG3 g;
  g.X = (const uint16_t*)X;
  g.D = (const uint16_t*)D;
  g.out = S > 1 ? slab : dW;
  g.N = N; g.C = C; g.H = H; g.W = W; g.F = F; g.S = S;
  g.Wp = 8;
  while (g.Wp < W) g.Wp <<= 1;
  g.RB = 64 / g.Wp;
  g.nrb = (H + g.RB - 1) / g.RB;
  // 64-filter tiles: the 128-row variant needs > 256 registers per lane (one wave per SIMD)
  const int TMv = 64;
  g.tm = (F + TMv - 1) / TMv;
  g.tn = (C + 31) / 32;
  if (32 * (g.RB + 2) * (g.Wp / 8) > XIT * NT) return -1;
  const size_t shm = ((size_t)TMv * (64 + 8) + (size_t)3 * 32 * ((g.RB + 2) * g.Wp + 8)) * sizeof(uint16_t);
  const int dv = (W % 8 == 0) ? 8 : (W % 4 == 0) ? 4 : (W % 2 == 0) ? 2 : 1;
  if (((uintptr_t)D) & 15) return -1;
  const dim3 grid((unsigned)(g.tm * g.tn * S)), t(NT);
  hipStream_t st = (hipStream_t)stream;
#define W3(TM_, DV_) hipLaunchKernelGGL((wgrad3_kernel<TM_, DV_>), grid, t, shm, st, g)
  if (dv == 8) W3(64, 8); else if (dv == 4) W3(64, 4); else if (dv == 2) W3(64, 2); else W3(64, 1);
#undef W3
  if (S > 1) {
    const int64_t n = (int64_t)F * C * 9;
    int64_t gb = (n + 255) / 256;
    if (gb > 2048) gb = 2048;
    hipLaunchKernelGGL(slab_sum, dim3((unsigned)gb), dim3(256), 0, st, (const float*)slab, dW, n, S);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
