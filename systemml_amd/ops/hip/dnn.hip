// CDNA4 DNN kernels for the DML deep-learning builtins (reference: LibMatrixCuDNN.java conv2d /
// conv2d_backward_filter / conv2d_backward_data, LibMatrixDNN{Conv2d,Pooling}.java and the
// bias_add / relu_backward kernels of SystemML.cu).
//
// Data layout is the DML one: images are rows of an N x (C*H*W) matrix (NCHW per row), filters
// an F x (C*Kh*Kw) matrix.
//
// Convolutions are implicit GEMMs on MFMA -- the im2col matrix is never materialised; each
// block gathers its operand tiles straight from the images into LDS:
//   forward        out[F, N*P]       = W[F, CKK]            x im2col(X)[CKK, N*P]
//   backward data  dX[C, N*H*W]      = W^T[C, F*KK]         x gather(dout)[F*KK, N*H*W]
//   backward filt. dW[F, CKK]        = dout[F, N*P] (gath.) x im2col(X)^T[N*P, CKK]   (split-K)
// Tiles are 64 x 64 per 256-thread block (4 waves, 32 x 32 each).  bf16 MFMA
// (v_mfma_f32_16x16x32_bf16, fp32 accumulate) for bf16 operands or the fast fp32 mode; exact
// v_mfma_f32_16x16x4f32 / v_mfma_f64_16x16x4f64 for fp32 / fp64.  A thread owns one output
// column (or filter row) of a tile and 8 consecutive k, so its index math (n -> image, oh, ow;
// k -> c, kh, kw) is done once per tile and advanced incrementally; its 8 values go to LDS
// with one 16-B store (bf16) in the [row][k] layout the MFMA fragments read.
// Pooling and the elementwise DNN ops are one thread per output element; max-pool backward is
// a gather over the windows covering an input cell (deterministic, no atomics).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace sysml_dnn {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d4 __attribute__((ext_vector_type(4)));

enum { FWD = 0, BWD_DATA = 1, BWD_FILTER = 2 };

struct Conv {
  const void* X;     // FWD / BWD_FILTER: images N x C*H*W;  BWD_DATA: unused
  const void* W;     // filters F x C*KK (FWD, BWD_DATA)
  const void* D;     // dout N x F*P (BWD_DATA, BWD_FILTER)
  const void* bias;  // FWD: optional F x 1 (same type as the output)
  void* out;
  int N, C, H, Wd, F, KH, KW, sh, sw, ph, pw, Ho, Wo;
  int M, Ncol, K;    // GEMM view
  int tm, tn;        // tiles along M, Ncol
  int ksplit, kper;  // BWD_FILTER split-K (kper: K elements per split, multiple of BK)
  int relu;          // FWD epilogue: max(0, .)
};

template <typename T> __device__ __forceinline__ float tof(T v) { return (float)v; }
template <> __device__ __forceinline__ float tof<__bf16>(__bf16 v) { return (float)v; }

// bijective XCD-aware remap (dispatch is round-robin over the 8 XCDs)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ---- operand gathers ------------------------------------------------------------------
// Column side ("B"): a thread owns GEMM column n and 8 consecutive k starting at k0.
template <int MODE, typename TI, int KV>
__device__ __forceinline__ void gather_b(const Conv& c, int n, int k0, float (&v)[KV]) {
  const TI* __restrict__ X = (const TI*)c.X;
  const TI* __restrict__ Dp = (const TI*)c.D;
  const int KK = c.KH * c.KW;
  if constexpr (MODE == FWD) {
    // n -> (img, oh, ow);  k -> (ci, kh, kw)
    const int P = c.Ho * c.Wo;
    const bool nv = n < c.Ncol;
    const int img = nv ? n / P : 0, p = n - img * P, oh = p / c.Wo, ow = p - oh * c.Wo;
    int ci = k0 / KK, r = k0 - ci * KK, kh = r / c.KW, kw = r - kh * c.KW;
    const int64_t ibase = (int64_t)img * c.C * c.H * c.Wd;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int ih = oh * c.sh - c.ph + kh, iw = ow * c.sw - c.pw + kw;
      const bool ok = nv && (k0 + j) < c.K && ih >= 0 && ih < c.H && iw >= 0 && iw < c.Wd;
      v[j] = ok ? tof<TI>(X[ibase + ((int64_t)ci * c.H + ih) * c.Wd + iw]) : 0.f;
      if (++kw == c.KW) { kw = 0; if (++kh == c.KH) { kh = 0; ++ci; } }
    }
  } else if constexpr (MODE == BWD_DATA) {
    // n -> (img, ih, iw);  k -> (f, kh, kw);  value dout[img, f, (ih+ph-kh)/sh, (iw+pw-kw)/sw]
    const int HW = c.H * c.Wd, P = c.Ho * c.Wo;
    const bool nv = n < c.Ncol;
    const int img = nv ? n / HW : 0, q = n - img * HW, ih = q / c.Wd, iw = q - ih * c.Wd;
    int f = k0 / KK, r = k0 - f * KK, kh = r / c.KW, kw = r - kh * c.KW;
    const int64_t dbase = (int64_t)img * c.F * P;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int th = ih + c.ph - kh, tw = iw + c.pw - kw;
      const int oh = th / c.sh, ow = tw / c.sw;
      const bool ok = nv && (k0 + j) < c.K && th >= 0 && tw >= 0 && oh * c.sh == th && ow * c.sw == tw &&
                      oh < c.Ho && ow < c.Wo;
      v[j] = ok ? tof<TI>(Dp[dbase + (int64_t)f * P + oh * c.Wo + ow]) : 0.f;
      if (++kw == c.KW) { kw = 0; if (++kh == c.KH) { kh = 0; ++f; } }
    }
  } else {
    // BWD_FILTER: n -> (ci, kh, kw);  k -> (img, p): im2col value
    const int P = c.Ho * c.Wo;
    const bool nv = n < c.Ncol;
    const int ci = nv ? n / KK : 0, r = n - ci * KK, kh = r / c.KW, kw = r - kh * c.KW;
    int img = k0 / P, p = k0 - img * P, oh = p / c.Wo, ow = p - oh * c.Wo;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int ih = oh * c.sh - c.ph + kh, iw = ow * c.sw - c.pw + kw;
      const bool ok = nv && (k0 + j) < c.K && ih >= 0 && ih < c.H && iw >= 0 && iw < c.Wd;
      v[j] = ok ? tof<TI>(X[((int64_t)img * c.C + ci) * c.H * c.Wd + (int64_t)ih * c.Wd + iw]) : 0.f;
      if (++ow == c.Wo) { ow = 0; if (++oh == c.Ho) { oh = 0; ++img; } }
    }
  }
}

// Row side ("A"): a thread owns GEMM row m and 8 consecutive k starting at k0.
template <int MODE, typename TI, int KV>
__device__ __forceinline__ void gather_a(const Conv& c, int m, int k0, float (&v)[KV]) {
  const int KK = c.KH * c.KW;
  const bool mv = m < c.M;
  if constexpr (MODE == FWD) {
    const TI* __restrict__ W = (const TI*)c.W;
    const int64_t base = (int64_t)(mv ? m : 0) * c.K;
#pragma unroll
    for (int j = 0; j < KV; ++j) v[j] = (mv && k0 + j < c.K) ? tof<TI>(W[base + k0 + j]) : 0.f;
  } else if constexpr (MODE == BWD_DATA) {
    // A(c, (f,kh,kw)) = W[f, c*KK + kh*KW + kw]
    const TI* __restrict__ W = (const TI*)c.W;
    int f = k0 / KK, r = k0 - f * KK;
    const int64_t CKK = (int64_t)c.C * KK;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      v[j] = (mv && k0 + j < c.K) ? tof<TI>(W[f * CKK + (int64_t)m * KK + r]) : 0.f;
      if (++r == KK) { r = 0; ++f; }
    }
  } else {
    // A(f, (img,p)) = dout[img, f, p]
    const TI* __restrict__ Dp = (const TI*)c.D;
    const int P = c.Ho * c.Wo;
    int img = k0 / P, p = k0 - img * P;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      v[j] = (mv && k0 + j < c.K) ? tof<TI>(Dp[((int64_t)img * c.F + m) * P + p]) : 0.f;
      if (++p == P) { p = 0; ++img; }
    }
  }
}

// output index of GEMM element (m, n)
template <int MODE>
__device__ __forceinline__ int64_t out_index(const Conv& c, int m, int n) {
  if constexpr (MODE == FWD) {
    const int P = c.Ho * c.Wo;
    const int img = n / P, p = n - img * P;
    return ((int64_t)img * c.F + m) * P + p;
  } else if constexpr (MODE == BWD_DATA) {
    const int HW = c.H * c.Wd;
    const int img = n / HW, q = n - img * HW;
    return ((int64_t)img * c.C + m) * HW + q;
  } else {
    return (int64_t)m * c.Ncol + n;
  }
}

constexpr int TM = 64, TN = 64, NT = 256;

// ---- bf16 MFMA kernel (fp32 accumulate) ---------------------------------------------------
template <int MODE, typename TI, typename TO>
__global__ void __launch_bounds__(NT) conv_bf16_kernel(Conv c) {
  constexpr int BK = 32, LDK = BK + 8;           // 80-B rows: conflict-free 16-B fragment reads
  __shared__ __attribute__((aligned(16))) __bf16 As[TM][LDK];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[TN][LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = c.tm * c.tn;
  const int tile = wg % ntile, split = wg / ntile;
  const int bm = tile % c.tm, bn = tile / c.tm;
  const int m0 = bm * TM, n0 = bn * TN;
  const int kbeg = split * c.kper;
  const int kend = min(c.K, kbeg + c.kper);
  // loader roles: A -> row tid/4, k (tid%4)*8;  B -> col tid/4, k (tid%4)*8
  const int ar = tid >> 2, ak = (tid & 3) * 8;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float va[8], vb[8];
  if (kbeg < kend) {
    gather_a<MODE, TI, 8>(c, m0 + ar, kbeg + ak, va);
    gather_b<MODE, TI, 8>(c, n0 + ar, kbeg + ak, vb);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    bf8 pa, pb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pa[j] = (__bf16)((k0 + ak + j) < kend ? va[j] : 0.f);
      pb[j] = (__bf16)((k0 + ak + j) < kend ? vb[j] : 0.f);
    }
    __syncthreads();                             // previous tile's fragment reads done
    *(bf8*)&As[ar][ak] = pa;
    *(bf8*)&Bs[ar][ak] = pb;
    __syncthreads();
    if (k0 + BK < kend) {                         // next tile's gathers overlap this tile's MFMAs
      gather_a<MODE, TI, 8>(c, m0 + ar, k0 + BK + ak, va);
      gather_b<MODE, TI, 8>(c, n0 + ar, k0 + BK + ak, vb);
    }
    const int kc = (lane >> 4) * 8;
    bf8 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = *(const bf8*)&As[wr * 32 + i * 16 + (lane & 15)][kc];
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = *(const bf8*)&Bs[wc * 32 + j * 16 + (lane & 15)][kc];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }
  // epilogue: 16x16 C/D map col = lane & 15, row = (lane >> 4) * 4 + reg
  TO* out = (TO*)c.out + (MODE == BWD_FILTER ? (int64_t)split * c.M * c.Ncol : 0);
  const TO* bias = (const TO*)c.bias;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wc * 32 + j * 16 + (lane & 15);
        if (m < c.M && n < c.Ncol) {
          float v = acc[i][j][r];
          if (MODE == FWD && bias) v += (float)bias[m];
          if (MODE == FWD && c.relu) v = v > 0.f ? v : 0.f;
          out[out_index<MODE>(c, m, n)] = (TO)v;
        }
      }
}

// ---- exact fp32 / fp64 MFMA kernel --------------------------------------------------------
template <typename T> struct Exact;
template <> struct Exact<float> {
  typedef f4 acc_t;
  static __device__ __forceinline__ acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) * 4 + r; }
};
template <> struct Exact<double> {
  typedef d4 acc_t;
  static __device__ __forceinline__ acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

// exact path: gathers produce the storage type directly (no fp32 rounding for fp64)
template <int MODE, typename T, int KV>
__device__ __forceinline__ void gather_b_x(const Conv& c, int n, int k0, T (&v)[KV]) {
  const T* __restrict__ X = (const T*)c.X;
  const T* __restrict__ Dp = (const T*)c.D;
  const int KK = c.KH * c.KW;
  const bool nv = n < c.Ncol;
  if constexpr (MODE == FWD) {
    const int P = c.Ho * c.Wo;
    const int img = nv ? n / P : 0, p = n - img * P, oh = p / c.Wo, ow = p - oh * c.Wo;
    int ci = k0 / KK, r = k0 - ci * KK, kh = r / c.KW, kw = r - kh * c.KW;
    const int64_t ibase = (int64_t)img * c.C * c.H * c.Wd;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int ih = oh * c.sh - c.ph + kh, iw = ow * c.sw - c.pw + kw;
      const bool ok = nv && (k0 + j) < c.K && ih >= 0 && ih < c.H && iw >= 0 && iw < c.Wd;
      v[j] = ok ? X[ibase + ((int64_t)ci * c.H + ih) * c.Wd + iw] : T(0);
      if (++kw == c.KW) { kw = 0; if (++kh == c.KH) { kh = 0; ++ci; } }
    }
  } else if constexpr (MODE == BWD_DATA) {
    const int HW = c.H * c.Wd, P = c.Ho * c.Wo;
    const int img = nv ? n / HW : 0, q = n - img * HW, ih = q / c.Wd, iw = q - ih * c.Wd;
    int f = k0 / KK, r = k0 - f * KK, kh = r / c.KW, kw = r - kh * c.KW;
    const int64_t dbase = (int64_t)img * c.F * P;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int th = ih + c.ph - kh, tw = iw + c.pw - kw;
      const int oh = th / c.sh, ow = tw / c.sw;
      const bool ok = nv && (k0 + j) < c.K && th >= 0 && tw >= 0 && oh * c.sh == th && ow * c.sw == tw &&
                      oh < c.Ho && ow < c.Wo;
      v[j] = ok ? Dp[dbase + (int64_t)f * P + oh * c.Wo + ow] : T(0);
      if (++kw == c.KW) { kw = 0; if (++kh == c.KH) { kh = 0; ++f; } }
    }
  } else {
    const int P = c.Ho * c.Wo;
    const int ci = nv ? n / KK : 0, r = n - ci * KK, kh = r / c.KW, kw = r - kh * c.KW;
    int img = k0 / P, p = k0 - img * P, oh = p / c.Wo, ow = p - oh * c.Wo;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int ih = oh * c.sh - c.ph + kh, iw = ow * c.sw - c.pw + kw;
      const bool ok = nv && (k0 + j) < c.K && ih >= 0 && ih < c.H && iw >= 0 && iw < c.Wd;
      v[j] = ok ? X[((int64_t)img * c.C + ci) * c.H * c.Wd + (int64_t)ih * c.Wd + iw] : T(0);
      if (++ow == c.Wo) { ow = 0; if (++oh == c.Ho) { oh = 0; ++img; } }
    }
  }
}

template <int MODE, typename T, int KV>
__device__ __forceinline__ void gather_a_x(const Conv& c, int m, int k0, T (&v)[KV]) {
  const int KK = c.KH * c.KW;
  const bool mv = m < c.M;
  if constexpr (MODE == FWD) {
    const T* __restrict__ W = (const T*)c.W;
    const int64_t base = (int64_t)(mv ? m : 0) * c.K;
#pragma unroll
    for (int j = 0; j < KV; ++j) v[j] = (mv && k0 + j < c.K) ? W[base + k0 + j] : T(0);
  } else if constexpr (MODE == BWD_DATA) {
    const T* __restrict__ W = (const T*)c.W;
    int f = k0 / KK, r = k0 - f * KK;
    const int64_t CKK = (int64_t)c.C * KK;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      v[j] = (mv && k0 + j < c.K) ? W[f * CKK + (int64_t)m * KK + r] : T(0);
      if (++r == KK) { r = 0; ++f; }
    }
  } else {
    const T* __restrict__ Dp = (const T*)c.D;
    const int P = c.Ho * c.Wo;
    int img = k0 / P, p = k0 - img * P;
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      v[j] = (mv && k0 + j < c.K) ? Dp[((int64_t)img * c.F + m) * P + p] : T(0);
      if (++p == P) { p = 0; ++img; }
    }
  }
}

template <int MODE, typename T>
__global__ void __launch_bounds__(NT) conv_exact_kernel(Conv c) {
  constexpr int BK = 16, LDK = BK + 1;           // odd row stride: conflict-free column reads
  __shared__ T As[TM][LDK];
  __shared__ T Bs[TN][LDK];
  typedef Exact<T> E;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = c.tm * c.tn;
  const int tile = wg % ntile, split = wg / ntile;
  const int bm = tile % c.tm, bn = tile / c.tm;
  const int m0 = bm * TM, n0 = bn * TN;
  const int kbeg = split * c.kper;
  const int kend = min(c.K, kbeg + c.kper);
  const int ar = tid >> 2, ak = (tid & 3) * 4;   // 64 rows x 4 groups of 4 k
  typename E::acc_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = T(0);
  T va[4], vb[4];
  if (kbeg < kend) {
    gather_a_x<MODE, T, 4>(c, m0 + ar, kbeg + ak, va);
    gather_b_x<MODE, T, 4>(c, n0 + ar, kbeg + ak, vb);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool in = (k0 + ak + j) < kend;
      As[ar][ak + j] = in ? va[j] : T(0);
      Bs[ar][ak + j] = in ? vb[j] : T(0);
    }
    __syncthreads();
    if (k0 + BK < kend) {
      gather_a_x<MODE, T, 4>(c, m0 + ar, k0 + BK + ak, va);
      gather_b_x<MODE, T, 4>(c, n0 + ar, k0 + BK + ak, vb);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      const int k = ks + (lane >> 4);
      T fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[wr * 32 + i * 16 + (lane & 15)][k];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[wc * 32 + j * 16 + (lane & 15)][k];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = E::mfma(fa[i], fb[j], acc[i][j]);
    }
  }
  T* out = (T*)c.out + (MODE == BWD_FILTER ? (int64_t)split * c.M * c.Ncol : 0);
  const T* bias = (const T*)c.bias;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + i * 16 + E::row(lane, r);
        const int n = n0 + wc * 32 + j * 16 + (lane & 15);
        if (m < c.M && n < c.Ncol) {
          T v = acc[i][j][r];
          if (MODE == FWD && bias) v += bias[m];
          if (MODE == FWD && c.relu) v = v > T(0) ? v : T(0);
          out[out_index<MODE>(c, m, n)] = v;
        }
      }
}

// split-K slabs -> output
template <typename T>
__global__ void __launch_bounds__(256) slab_sum(const T* __restrict__ s, int ks, int64_t n, T* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    T a = 0;
    for (int k = 0; k < ks; ++k) a += s[(int64_t)k * n + i];
    out[i] = a;
  }
}

// ---- pooling ----------------------------------------------------------------------------
struct Pool {
  const void* X;
  const void* D;
  void* out;
  int N, C, H, W, KH, KW, sh, sw, ph, pw, Ho, Wo;
  int avg;
};

template <typename T>
__global__ void __launch_bounds__(256) pool_fwd(Pool p) {
  const T* __restrict__ X = (const T*)p.X;
  T* __restrict__ O = (T*)p.out;
  const int64_t total = (int64_t)p.N * p.C * p.Ho * p.Wo;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int ow = (int)(i % p.Wo);
    const int oh = (int)((i / p.Wo) % p.Ho);
    const int64_t nc = i / ((int64_t)p.Wo * p.Ho);
    const T* x = X + nc * p.H * p.W;
    const int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    T m = p.avg ? T(0) : -INFINITY;
    for (int a = 0; a < p.KH; ++a) {
      const int h = h0 + a;
      if (h < 0 || h >= p.H) continue;
      for (int b = 0; b < p.KW; ++b) {
        const int w = w0 + b;
        if (w < 0 || w >= p.W) continue;
        const T v = x[h * p.W + w];
        if (p.avg) m += v;
        else m = v > m ? v : m;
      }
    }
    O[i] = p.avg ? m / T(p.KH * p.KW) : m;
  }
}

// dX[n,c,h,w] = sum over windows containing (h,w) of dout / (KH*KW) (avg) or of dout where
// (h,w) is the window's first maximum (max) -- recomputed per window, no atomics
template <typename T>
__global__ void __launch_bounds__(256) pool_bwd(Pool p) {
  const T* __restrict__ X = (const T*)p.X;
  const T* __restrict__ D = (const T*)p.D;
  T* __restrict__ O = (T*)p.out;
  const int64_t total = (int64_t)p.N * p.C * p.H * p.W;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int w = (int)(i % p.W);
    const int h = (int)((i / p.W) % p.H);
    const int64_t nc = i / ((int64_t)p.W * p.H);
    const T* x = X + nc * p.H * p.W;
    const T* d = D + nc * p.Ho * p.Wo;
    // output windows covering (h, w): oh*sh - ph <= h <= oh*sh - ph + KH - 1
    const int ohl = max(0, (h + p.ph - p.KH + p.sh) / p.sh), ohh = min(p.Ho - 1, (h + p.ph) / p.sh);
    const int owl = max(0, (w + p.pw - p.KW + p.sw) / p.sw), owh = min(p.Wo - 1, (w + p.pw) / p.sw);
    T g = 0;
    for (int oh = ohl; oh <= ohh; ++oh) {
      const int h0 = oh * p.sh - p.ph;
      if (h < h0 || h >= h0 + p.KH) continue;
      for (int ow = owl; ow <= owh; ++ow) {
        const int w0 = ow * p.sw - p.pw;
        if (w < w0 || w >= w0 + p.KW) continue;
        const T dv = d[oh * p.Wo + ow];
        if (p.avg) { g += dv / T(p.KH * p.KW); continue; }
        // first maximum of the window (row-major scan, as the forward pass)
        T m = -INFINITY;
        int ah = -1, aw = -1;
        for (int a = 0; a < p.KH; ++a) {
          const int hh = h0 + a;
          if (hh < 0 || hh >= p.H) continue;
          for (int b = 0; b < p.KW; ++b) {
            const int ww = w0 + b;
            if (ww < 0 || ww >= p.W) continue;
            const T v = x[hh * p.W + ww];
            if (v > m) { m = v; ah = hh; aw = ww; }
          }
        }
        if (ah == h && aw == w) g += dv;
      }
    }
    O[i] = g;
  }
}

// ---- elementwise: bias add / multiply (channel-wise), relu backward --------------------------
template <typename T>
__global__ void __launch_bounds__(256) bias_op(const T* __restrict__ X, const T* __restrict__ b, T* __restrict__ O,
                                                int64_t total, int C, int P, int mult, int relu) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int ch = (int)((i / P) % C);
    T v = mult ? X[i] * b[ch] : X[i] + b[ch];
    if (relu) v = v > T(0) ? v : T(0);
    O[i] = v;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) relu_bwd(const T* __restrict__ X, const T* __restrict__ D, T* __restrict__ O,
                                                 int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256)
    O[i] = X[i] > T(0) ? D[i] : T(0);
}

inline unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g < 256 * 64 ? (g < 1 ? 1 : g) : 256 * 64);
}

}  // namespace sysml_dnn

extern "C" {

// dtype: 0 bf16 in (fp32 out), 1 fp32 exact, 2 fp64 exact, 3 fp32 in / bf16 MFMA / fp32 out.
// mode: 0 forward, 1 backward data, 2 backward filter.  ws: fp32/fp64 workspace for the
// backward-filter split-K slabs (ksplit * F * C*KH*KW elements), may be null when ksplit = 1.
// Returns 0, -1 (unsupported) or a hipError_t.
int sysml_conv2d(int dtype, int mode, const void* X, const void* W, const void* D, const void* bias, void* out,
                 void* ws, int ksplit, int N, int C, int H, int Wd, int F, int KH, int KW, int sh, int sw, int ph,
                 int pw, int relu, void* stream) {
  using namespace sysml_dnn;
  Conv c;
  c.X = X; c.W = W; c.D = D; c.bias = bias; c.out = out;
  c.N = N; c.C = C; c.H = H; c.Wd = Wd; c.F = F; c.KH = KH; c.KW = KW; c.sh = sh; c.sw = sw; c.ph = ph; c.pw = pw;
  c.Ho = (H + 2 * ph - KH) / sh + 1;
  c.Wo = (Wd + 2 * pw - KW) / sw + 1;
  c.relu = relu;
  if (c.Ho <= 0 || c.Wo <= 0 || N <= 0) return -1;
  const int64_t P = (int64_t)c.Ho * c.Wo, KK = (int64_t)KH * KW;
  int64_t M, Nc, K;
  if (mode == FWD) { M = F; Nc = (int64_t)N * P; K = C * KK; }
  else if (mode == BWD_DATA) { M = C; Nc = (int64_t)N * H * Wd; K = F * KK; }
  else { M = F; Nc = C * KK; K = (int64_t)N * P; }
  if (M >= (1LL << 31) || Nc >= (1LL << 31) || K >= (1LL << 31)) return -1;
  c.M = (int)M; c.Ncol = (int)Nc; c.K = (int)K;
  c.tm = (int)((M + TM - 1) / TM);
  c.tn = (int)((Nc + TN - 1) / TN);
  const bool bfmma = dtype == 0 || dtype == 3;
  const int BK = bfmma ? 32 : 16;
  if (mode != BWD_FILTER) ksplit = 1;
  if (ksplit < 1) ksplit = 1;
  int64_t kper = (K + ksplit - 1) / ksplit;
  kper = (kper + BK - 1) / BK * BK;
  ksplit = (int)((K + kper - 1) / kper);
  c.ksplit = ksplit;
  c.kper = (int)kper;
  void* final_out = out;
  if (ksplit > 1) {
    if (!ws) return -1;
    c.out = ws;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t nwg = (int64_t)c.tm * c.tn * ksplit;
  if (nwg >= (1LL << 31)) return -1;
  dim3 g((unsigned)nwg), t(NT);
#define LAUNCH(KERN, ...)                                                                    \
  do {                                                                                       \
    if (mode == FWD) hipLaunchKernelGGL((KERN<FWD, __VA_ARGS__>), g, t, 0, s, c);            \
    else if (mode == BWD_DATA) hipLaunchKernelGGL((KERN<BWD_DATA, __VA_ARGS__>), g, t, 0, s, c); \
    else hipLaunchKernelGGL((KERN<BWD_FILTER, __VA_ARGS__>), g, t, 0, s, c);                 \
  } while (0)
  if (dtype == 0) {
    LAUNCH(conv_bf16_kernel, __bf16, float);
  } else if (dtype == 3) {
    LAUNCH(conv_bf16_kernel, float, float);
  } else if (dtype == 1) {
    LAUNCH(conv_exact_kernel, float);
  } else if (dtype == 2) {
    LAUNCH(conv_exact_kernel, double);
  } else {
    return -1;
  }
#undef LAUNCH
  if (ksplit > 1) {
    const int64_t n = M * Nc;
    if (dtype == 2)
      hipLaunchKernelGGL(slab_sum<double>, dim3(grid_for(n)), dim3(256), 0, s, (const double*)ws, ksplit, n,
                         (double*)final_out);
    else
      hipLaunchKernelGGL(slab_sum<float>, dim3(grid_for(n)), dim3(256), 0, s, (const float*)ws, ksplit, n,
                         (float*)final_out);
  }
  return (int)hipGetLastError();
}

// dtype 1 fp32, 2 fp64; backward: D = dout, out = dX
int sysml_pool2d(int dtype, int backward, int avg, const void* X, const void* D, void* out, int N, int C, int H,
                 int W, int KH, int KW, int sh, int sw, int ph, int pw, void* stream) {
  using namespace sysml_dnn;
  Pool p;
  p.X = X; p.D = D; p.out = out; p.N = N; p.C = C; p.H = H; p.W = W; p.KH = KH; p.KW = KW; p.sh = sh; p.sw = sw;
  p.ph = ph; p.pw = pw; p.avg = avg;
  p.Ho = (H + 2 * ph - KH) / sh + 1;
  p.Wo = (W + 2 * pw - KW) / sw + 1;
  if (p.Ho <= 0 || p.Wo <= 0) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = backward ? (int64_t)N * C * H * W : (int64_t)N * C * p.Ho * p.Wo;
  if (dtype == 1) {
    if (backward) hipLaunchKernelGGL(pool_bwd<float>, dim3(grid_for(n)), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(pool_fwd<float>, dim3(grid_for(n)), dim3(256), 0, s, p);
  } else if (dtype == 2) {
    if (backward) hipLaunchKernelGGL(pool_bwd<double>, dim3(grid_for(n)), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(pool_fwd<double>, dim3(grid_for(n)), dim3(256), 0, s, p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

int sysml_bias_op(int dtype, const void* X, const void* b, void* out, int64_t total, int C, int P, int mult, int relu,
                  void* stream) {
  using namespace sysml_dnn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == 1)
    hipLaunchKernelGGL(bias_op<float>, dim3(grid_for(total)), dim3(256), 0, s, (const float*)X, (const float*)b,
                       (float*)out, total, C, P, mult, relu);
  else if (dtype == 2)
    hipLaunchKernelGGL(bias_op<double>, dim3(grid_for(total)), dim3(256), 0, s, (const double*)X, (const double*)b,
                       (double*)out, total, C, P, mult, relu);
  else
    return -1;
  return (int)hipGetLastError();
}

int sysml_relu_backward(int dtype, const void* X, const void* D, void* out, int64_t total, void* stream) {
  using namespace sysml_dnn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == 1)
    hipLaunchKernelGGL(relu_bwd<float>, dim3(grid_for(total)), dim3(256), 0, s, (const float*)X, (const float*)D,
                       (float*)out, total);
  else if (dtype == 2)
    hipLaunchKernelGGL(relu_bwd<double>, dim3(grid_for(total)), dim3(256), 0, s, (const double*)X, (const double*)D,
                       (double*)out, total);
  else
    return -1;
  return (int)hipGetLastError();
}

}  // extern "C"
