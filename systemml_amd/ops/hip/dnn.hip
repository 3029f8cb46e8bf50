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
#include <type_traits>

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
  int avec;          // FWD: filter rows 16-B aligned (vector loads of W)
  void* slab;        // split-K partials (ksplit x M x Ncol, the output type) instead of atomics, or null
};

// bijective XCD-aware remap (dispatch is round-robin over the 8 XCDs)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
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

// ---- implicit-GEMM convolution ----------------------------------------------------------
// Per K-tile, BK threads decode the tile's k indices once into an LDS table (int4 per k):
//   FWD        k = (ci, kh, kw):     x = ci*H*W + kh*W + kw, y = kh, z = kw,            w = k
//   BWD_DATA   k = (f, kh, kw):      x = f*P,                y = kh, z = kw,            w = f*C*KK + kh*KW + kw
//   BWD_FILTER k = (img, oh, ow):    x = img*CHW + hs*W + ws, y = hs = oh*sh-ph, z = ws, w = img*F*P + p
// and every thread decodes its fixed GEMM column / row once per block, so gathering one
// element is two adds, two unsigned compares and a masked load (no divisions in the loop).
// Element (row side):    A[ra + w]                     (W for FWD / BWD_DATA, dout for BWD_FILTER)
// Element (column side): FWD / BWD_FILTER: X[cb + x] if (ch + y, cw + z) inside the image
//                        BWD_DATA: dout[cb + x + th*Wo + tw], th = ch - y, tw = cw - z on the stride grid
constexpr int NT = 256;

template <int PATH> struct PathCfg;                       // 0: bf16 MFMA, 1: f32, 2: f64
template <> struct PathCfg<0> { static constexpr int BK = 32; typedef f4 acc_t; };
template <> struct PathCfg<1> { static constexpr int BK = 16; typedef f4 acc_t; };
template <> struct PathCfg<2> { static constexpr int BK = 16; typedef d4 acc_t; };
// K-tile depth: 64 for the bf16 128 x 128 forward / backward-data tiles (half the barriers and
// table decodes per MFMA), the path's default otherwise (split-K rounding uses the default)
template <int PATH, int MODE, int TM_> struct KDepth {
  static constexpr int BK = (PATH == 0 && MODE != BWD_FILTER && TM_ == 128) ? 64 : PathCfg<PATH>::BK;
};

template <int MODE>
__device__ __forceinline__ int4 decode_k(const Conv& c, int k) {
  const int KK = c.KH * c.KW;
  if (MODE == FWD) {
    const int ci = k / KK, r = k - ci * KK, kh = r / c.KW, kw = r - kh * c.KW;
    return int4{ci * c.H * c.Wd + kh * c.Wd + kw, kh, kw, k};
  } else if (MODE == BWD_DATA) {
    const int f = k / KK, r = k - f * KK, kh = r / c.KW, kw = r - kh * c.KW;
    return int4{f * c.Ho * c.Wo, kh, kw, f * c.C * KK + r};
  } else {
    const int P = c.Ho * c.Wo;
    const int img = k / P, p = k - img * P, oh = p / c.Wo, ow = p - oh * c.Wo;
    const int hs = oh * c.sh - c.ph, ws = ow * c.sw - c.pw;
    return int4{img * c.C * c.H * c.Wd + hs * c.Wd + ws, hs, ws, img * c.F * P + p};
  }
}

template <int PATH, typename TI> struct Store;
template <typename TI> struct Store<0, TI> {
  template <int KV>
  static __device__ __forceinline__ void put(__bf16* row, const TI (&v)[KV]) {
#pragma unroll
    for (int h = 0; h < KV; h += 8) {
      bf8 p;
#pragma unroll
      for (int j = 0; j < 8; ++j) p[j] = (__bf16)v[h + j];
      *(bf8*)(row + h) = p;
    }
  }
};
template <int PATH, typename TI> struct Store {
  template <int KV, typename S>
  static __device__ __forceinline__ void put(S* row, const TI (&v)[KV]) {
#pragma unroll
    for (int j = 0; j < KV; ++j) row[j] = (S)v[j];
  }
};

// TM_ x TN_ output tile per 256-thread block, 2 x 2 waves of (TM_/2) x (TN_/2); 128 x 128 tiles
// (4 x 4 MFMA 16x16 accumulators per wave) halve the gathered operand bytes per MFMA against
// 64 x 64 and are used for the bf16 path whenever both GEMM dimensions reach 128.
template <int MODE, typename TI, int PATH, typename TO, int TM_, int TN_>
__global__ void __launch_bounds__(NT) conv_kernel(Conv c) {
  typedef PathCfg<PATH> Cfg;
  constexpr int BK = KDepth<PATH, MODE, TM_>::BK, KV = BK / 4;
  typedef typename std::conditional<PATH == 0, __bf16, typename std::conditional<PATH == 1, float, double>::type>::type S;
  constexpr int LDK = PATH == 0 ? BK + 8 : BK + 1;       // bf16: 80 / 144-B rows; exact: odd stride
  constexpr int FI = TM_ / 32, FJ = TN_ / 32;            // 16-wide MFMA fragments per wave
  constexpr int RS = TM_ / 64, CS = TN_ / 64;            // row / column sets of the k-run mapping
  __shared__ __attribute__((aligned(16))) S As[TM_][LDK];
  __shared__ __attribute__((aligned(16))) S Bs[TN_][LDK];
  __shared__ int4 tab[2][BK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = c.tm * c.tn;
  const int tile = wg % ntile, split = wg / ntile;
  const int bm = tile % c.tm, bn = tile / c.tm;
  const int m0 = bm * TM_, n0 = bn * TN_;
  const int kbeg = split * c.kper;
  const int kend = min(c.K, kbeg + c.kper);
  const TI* __restrict__ Ap = (const TI*)(MODE == BWD_FILTER ? c.D : c.W);
  const TI* __restrict__ Bp = (const TI*)(MODE == BWD_DATA ? c.D : c.X);
  // Load mappings (which thread fetches which tile elements), chosen so that the lanes of one
  // load instruction touch consecutive addresses:
  //   FWD / BWD_DATA  A: rows tid/4 + 64 s, k (tid%4)*KV..+KV  (W rows contiguous in k: 16-B loads)
  //                   B: columns tid%64 + 64 s, k (tid/64)*KV..  (lanes = consecutive pixels)
  //   BWD_FILTER      A, B: k = tid%BK (lanes = consecutive output pixels), RPT rows / columns each
  constexpr bool KL = MODE == BWD_FILTER;
  constexpr int RPTA = KL ? (TM_ * BK) / NT : RS;        // row slots per thread
  constexpr int RPTB = KL ? (TN_ * BK) / NT : CS;        // column slots per thread
  const int ak = KL ? tid % BK : (tid & 3) * KV;
  const int bk = KL ? tid % BK : (tid >> 6) * KV;
  auto arow = [&](int q) { return KL ? (tid / BK) * RPTA + q : (tid >> 2) + 64 * q; };
  auto bcol = [&](int q) { return KL ? (tid / BK) * RPTB + q : (tid & 63) + 64 * q; };
  // fixed per-thread row / column decode
  int ra[RPTA];
  bool mv[RPTA];
#pragma unroll
  for (int q = 0; q < RPTA; ++q) {
    const int m = m0 + arow(q);
    mv[q] = m < c.M;
    ra[q] = MODE == FWD ? m * c.K : (MODE == BWD_DATA ? m * c.KH * c.KW : m * c.Ho * c.Wo);
  }
  int cb[RPTB], ch[RPTB], cw[RPTB];
#pragma unroll
  for (int q = 0; q < RPTB; ++q) {
    const int n = n0 + bcol(q);
    cb[q] = 0; ch[q] = -(1 << 29); cw[q] = 0;
    if (n < c.Ncol) {
      if (MODE == FWD) {
        const int P = c.Ho * c.Wo, img = n / P, p = n - img * P, oh = p / c.Wo, ow = p - oh * c.Wo;
        ch[q] = oh * c.sh - c.ph;
        cw[q] = ow * c.sw - c.pw;
        cb[q] = img * c.C * c.H * c.Wd + ch[q] * c.Wd + cw[q];   // + x = image cell (ci, ch + kh, cw + kw)
      } else if (MODE == BWD_DATA) {
        const int HW = c.H * c.Wd, img = n / HW, qq = n - img * HW, ih = qq / c.Wd, iw = qq - ih * c.Wd;
        ch[q] = ih + c.ph;
        cw[q] = iw + c.pw;
        cb[q] = img * c.F * c.Ho * c.Wo;
      } else {
        const int KK = c.KH * c.KW, ci = n / KK, r = n - ci * KK, kh = r / c.KW, kw = r - kh * c.KW;
        ch[q] = kh;
        cw[q] = kw;
        cb[q] = ci * c.H * c.Wd + kh * c.Wd + kw;
      }
    }
  }
  const bool s1 = c.sh == 1 && c.sw == 1;
  constexpr int NVA = KL ? RPTA : RS * KV, NVB = KL ? RPTB : CS * KV;
  TI va[NVA], vb[NVB];
  auto build = [&](int buf, int k0) {
    if (tid < BK) {
      const int k = k0 + tid;
      tab[buf][tid] = k < kend ? decode_k<MODE>(c, k) : int4{0, -(1 << 29), -(1 << 29), -1};
    }
  };
  auto bval = [&](const int4& e, int q) -> TI {
    if (MODE != BWD_DATA) {
      const int ih = ch[q] + e.y, iw = cw[q] + e.z;
      return ((unsigned)ih < (unsigned)c.H && (unsigned)iw < (unsigned)c.Wd) ? Bp[cb[q] + e.x] : TI(0);
    } else {
      const int th = ch[q] - e.y, tw = cw[q] - e.z;
      bool ok;
      int oh, ow;
      if (s1) {
        oh = th; ow = tw;
        ok = (unsigned)th < (unsigned)c.Ho && (unsigned)tw < (unsigned)c.Wo;
      } else {
        oh = th / c.sh; ow = tw / c.sw;
        ok = th >= 0 && tw >= 0 && oh * c.sh == th && ow * c.sw == tw && oh < c.Ho && ow < c.Wo;
      }
      return ok ? Bp[cb[q] + e.x + oh * c.Wo + ow] : TI(0);
    }
  };
  auto gather = [&](int buf, int k0) {
    if constexpr (KL) {
      const int4 e = tab[buf][ak];
#pragma unroll
      for (int q = 0; q < RPTA; ++q) va[q] = (mv[q] && e.w >= 0) ? Ap[ra[q] + e.w] : TI(0);
#pragma unroll
      for (int q = 0; q < RPTB; ++q) vb[q] = bval(e, q);
    } else {
#pragma unroll
      for (int q = 0; q < RS; ++q) {
        // A: FWD rows are contiguous in k -> one 16-B load when the KV-run is in range and aligned
        bool vec = false;
        if constexpr (MODE == FWD && (sizeof(TI) * KV) % 16 == 0) vec = c.avec && mv[q] && (k0 + ak + KV) <= kend;
        if (vec) {
          typedef TI vt __attribute__((ext_vector_type(KV)));
          const vt x = *(const vt*)(Ap + ra[q] + k0 + ak);
#pragma unroll
          for (int j = 0; j < KV; ++j) va[q * KV + j] = x[j];
        } else {
#pragma unroll
          for (int j = 0; j < KV; ++j) {
            const int4 e = tab[buf][ak + j];
            va[q * KV + j] = (mv[q] && e.w >= 0) ? Ap[ra[q] + e.w] : TI(0);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < CS; ++q)
#pragma unroll
        for (int j = 0; j < KV; ++j) vb[q * KV + j] = bval(tab[buf][bk + j], q);
    }
  };
  auto store = [&]() {
    if constexpr (KL) {
#pragma unroll
      for (int q = 0; q < RPTA; ++q) As[arow(q)][ak] = (S)va[q];
#pragma unroll
      for (int q = 0; q < RPTB; ++q) Bs[bcol(q)][bk] = (S)vb[q];
    } else {
#pragma unroll
      for (int q = 0; q < RS; ++q) {
        TI r[KV];
#pragma unroll
        for (int j = 0; j < KV; ++j) r[j] = va[q * KV + j];
        Store<PATH, TI>::template put<KV>(&As[arow(q)][ak], r);
      }
#pragma unroll
      for (int q = 0; q < CS; ++q) {
        TI r[KV];
#pragma unroll
        for (int j = 0; j < KV; ++j) r[j] = vb[q * KV + j];
        Store<PATH, TI>::template put<KV>(&Bs[bcol(q)][bk], r);
      }
    }
  };
  typename Cfg::acc_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0;
  if (kbeg < kend) {
    build(0, kbeg);
    __syncthreads();
    gather(0, kbeg);
  }
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK, buf ^= 1) {
    __syncthreads();                                     // fragment reads of the previous tile done
    store();
    const bool more = k0 + BK < kend;
    if (more) build(buf ^ 1, k0 + BK);
    __syncthreads();
    if (more) gather(buf ^ 1, k0 + BK);                  // next tile's loads overlap this tile's MFMAs
    if constexpr (PATH == 0) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        const int kc = kk + (lane >> 4) * 8;
        bf8 fa[FI], fb[FJ];
#pragma unroll
        for (int i = 0; i < FI; ++i) fa[i] = *(const bf8*)&As[wr * (TM_ / 2) + i * 16 + (lane & 15)][kc];
#pragma unroll
        for (int j = 0; j < FJ; ++j) fb[j] = *(const bf8*)&Bs[wc * (TN_ / 2) + j * 16 + (lane & 15)][kc];
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK; ks += 4) {
        const int k = ks + (lane >> 4);
        S fa[FI], fb[FJ];
#pragma unroll
        for (int i = 0; i < FI; ++i) fa[i] = As[wr * (TM_ / 2) + i * 16 + (lane & 15)][k];
#pragma unroll
        for (int j = 0; j < FJ; ++j) fb[j] = Bs[wc * (TN_ / 2) + j * 16 + (lane & 15)][k];
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j) {
            if constexpr (PATH == 1) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
            else acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[i], fb[j], acc[i][j], 0, 0, 0);
          }
      }
    }
  }
  // epilogue.  C/D maps: f32 16x16: row = (lane >> 4) * 4 + reg;  f64 16x16: row = (lane >> 4) + 4 * reg
  // split-K: partial sums are added atomically into the zero-initialised output (vector
  // global atomics, fp32 / fp64); bias / relu then run as a separate pass (host).  A bf16
  // output (activations of a bf16 network) is rounded once, after bias and relu in fp32.
  constexpr bool OBF = std::is_same<TO, __bf16>::value;
  typedef typename std::conditional<OBF, float, TO>::type CT;
  const bool atomic = c.ksplit > 1;
  TO* out = (TO*)c.out;
  const CT* bias = (const CT*)c.bias;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mo = m0 + wr * (TM_ / 2) + i * 16 + (PATH == 2 ? (lane >> 4) + 4 * r : (lane >> 4) * 4 + r);
        const int no = n0 + wc * (TN_ / 2) + j * 16 + (lane & 15);
        if (mo < c.M && no < c.Ncol) {
          CT v = (CT)acc[i][j][r];
          if constexpr (!OBF) {
            if (atomic) {
              if (c.slab != nullptr)             // deterministic split-K: this split's slice
                ((TO*)c.slab)[(int64_t)split * c.M * c.Ncol + (int64_t)mo * c.Ncol + no] = (TO)v;
              else
                atomicAdd(out + out_index<MODE>(c, mo, no), v);
              continue;
            }
          }
          if (MODE == FWD && bias) v += bias[mo];
          if (MODE == FWD && c.relu) v = v > CT(0) ? v : CT(0);
          out[out_index<MODE>(c, mo, no)] = (TO)v;
        }
      }
}

// split-K slab of the backward filter: out[i] = sum_s slab[s, i] (fixed order, no atomics)
template <typename T>
__global__ void __launch_bounds__(256) slab_reduce(const T* __restrict__ slab, T* __restrict__ out, int64_t n, int S) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    T a = slab[i];
    for (int q = 1; q < S; ++q) a += slab[(int64_t)q * n + i];
    out[i] = a;
  }
}

// ---- backward data for few input channels -------------------------------------------------
// dX = conv2d_backward_data with C <= 8 (an RGB stem): the implicit GEMM's M dimension is C, so
// a 64-row MFMA tile would be > 90 % padding and, with a strided filter, most K taps are off the
// stride grid.  Direct form instead: each thread owns one dX cell and sums dout * W over the
// taps that land on the stride grid and over the filters (fp32 / fp64 accumulation).
template <typename TI, typename TA>
__global__ void __launch_bounds__(256) conv_bwd_data_direct(Conv c, TA* __restrict__ out) {
  const TI* __restrict__ Wt = (const TI*)c.W;
  const TI* __restrict__ D = (const TI*)c.D;
  const int64_t total = (int64_t)c.N * c.C * c.H * c.Wd;
  const int KK = c.KH * c.KW, P = c.Ho * c.Wo;
  const int64_t fstride_w = (int64_t)c.C * KK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    int64_t q = i / c.Wd;
    const int w = (int)(i - q * c.Wd);
    const int h = (int)(q % c.H);
    q /= c.H;
    const int ch = (int)(q % c.C);
    const int64_t n = q / c.C;
    const TI* dn = D + n * (int64_t)c.F * P;
    const TI* wc = Wt + (int64_t)ch * KK;
    TA acc = 0;
    for (int kh = 0; kh < c.KH; ++kh) {
      const int th = h + c.ph - kh;
      if (th < 0 || th % c.sh) continue;
      const int oh = th / c.sh;
      if (oh >= c.Ho) continue;
      for (int kw = 0; kw < c.KW; ++kw) {
        const int tw = w + c.pw - kw;
        if (tw < 0 || tw % c.sw) continue;
        const int ow = tw / c.sw;
        if (ow >= c.Wo) continue;
        const TI* dp = dn + oh * c.Wo + ow;
        const TI* wp = wc + kh * c.KW + kw;
        // 8 filters' loads in flight before their products are accumulated (in filter order)
        int f = 0;
        for (; f + 8 <= c.F; f += 8) {
          TA dv[8], wv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            dv[u] = (TA)dp[(int64_t)(f + u) * P];
            wv[u] = (TA)wp[(f + u) * fstride_w];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) acc += dv[u] * wv[u];
        }
        for (; f < c.F; ++f) acc += (TA)dp[(int64_t)f * P] * (TA)wp[f * fstride_w];
      }
    }
    out[i] = acc;
  }
}

// n / d for 0 <= n < 2^31 by multiply-high and shift (d fixed per launch): the flat index
// kernels below spend most of their instructions on 32-bit divisions otherwise
struct FastDiv {
  unsigned d, m, l;
};
inline FastDiv fastdiv(unsigned d) {
  unsigned l = 0;
  while ((1ull << l) < d) ++l;
  const unsigned long long m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{d, (unsigned)m, l};
}
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.l; }

// ---- pooling ----------------------------------------------------------------------------
struct Pool {
  const void* X;
  const void* D;
  void* out;
  int N, C, H, W, KH, KW, sh, sw, ph, pw, Ho, Wo;
  int avg;
  FastDiv fWo, fHo, fBw, fBh;     // divisions of the 32-bit index kernels
};

// I: index type of the flat cell loops (int below 2^31 cells: 32-bit divisions instead of the
// emulated 64-bit ones)
// storage type T, arithmetic type Acc<T>::type (bf16 activations: fp32 math, one rounding)
template <typename T> struct Acc { typedef T type; };
template <> struct Acc<__bf16> { typedef float type; };

// K > 0: K x K windows, fully unrolled with every tap loaded unconditionally (out-of-image taps
// read cell 0 and are replaced by the neutral value) so all loads of a window are in flight at
// once; K == 0: any window, taps outside the image skipped
template <typename T, typename I, int K>
__global__ void __launch_bounds__(256) pool_fwd(Pool p) {
  typedef typename Acc<T>::type A;
  const T* __restrict__ X = (const T*)p.X;
  T* __restrict__ O = (T*)p.out;
  const I total = (I)p.N * p.C * p.Ho * p.Wo;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    I q, nc;
    if constexpr (sizeof(I) == 4) {
      q = (I)fdiv((unsigned)i, p.fWo);
      nc = (I)fdiv((unsigned)q, p.fHo);
    } else {
      q = i / p.Wo;
      nc = q / p.Ho;
    }
    const int ow = (int)(i - q * p.Wo);
    const int oh = (int)(q - nc * p.Ho);
    const T* x = X + (int64_t)nc * p.H * p.W;
    const int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    A m = p.avg ? A(0) : A(-INFINITY);
    const int KH = K ? K : p.KH, KW = K ? K : p.KW;
#pragma unroll
    for (int a = 0; a < KH; ++a) {
      const int h = h0 + a;
      if (!K && (h < 0 || h >= p.H)) continue;
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        const int w = w0 + b;
        if (!K && (w < 0 || w >= p.W)) continue;
        A v;
        if (K) {
          const bool ok = (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
          const A t = (A)x[ok ? h * p.W + w : 0];
          v = ok ? t : (p.avg ? A(0) : A(-INFINITY));
        } else {
          v = (A)x[h * p.W + w];
        }
        if (p.avg) m += v;
        else m = v > m ? v : m;
      }
    }
    O[i] = (T)(p.avg ? m / A(p.KH * p.KW) : m);
  }
}

// average pooling over the whole image (global pooling, Ho = Wo = 1): one wave per (n, c)
// plane, lanes strided along the plane (coalesced), a wave reduction and one store -- the
// per-output kernel above would read each plane with one lane
template <typename T>
__global__ void __launch_bounds__(256) pool_global_avg(Pool p) {
  typedef typename Acc<T>::type A;
  const T* __restrict__ X = (const T*)p.X;
  T* __restrict__ O = (T*)p.out;
  const int64_t planes = (int64_t)p.N * p.C;
  const int HW = p.H * p.W;
  const int lane = threadIdx.x & 63;
  for (int64_t nc = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); nc < planes; nc += (int64_t)gridDim.x * 4) {
    const T* x = X + nc * HW;
    A acc = A(0);
    for (int k = lane; k < HW; k += 64) acc += (A)x[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) O[nc] = (T)(acc / A(HW));
  }
}

// max pooling backward, pass 1: position (a * KW + b) of each window's first maximum (row-major
// scan, as the forward pass), 255 for a window without a cell above -inf
template <typename T, typename I, int K>
__global__ void __launch_bounds__(256) pool_argmax(Pool p, uint8_t* __restrict__ idx) {
  typedef typename Acc<T>::type A;
  const T* __restrict__ X = (const T*)p.X;
  const I total = (I)p.N * p.C * p.Ho * p.Wo;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    I q, nc;
    if constexpr (sizeof(I) == 4) {
      q = (I)fdiv((unsigned)i, p.fWo);
      nc = (I)fdiv((unsigned)q, p.fHo);
    } else {
      q = i / p.Wo;
      nc = q / p.Ho;
    }
    const int ow = (int)(i - q * p.Wo);
    const int oh = (int)(q - nc * p.Ho);
    const T* x = X + (int64_t)nc * p.H * p.W;
    const int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    A m = A(-INFINITY);
    int am = 255;
    const int KH = K ? K : p.KH, KW = K ? K : p.KW;
#pragma unroll
    for (int a = 0; a < KH; ++a) {
      const int h = h0 + a;
      if (!K && (h < 0 || h >= p.H)) continue;
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        const int w = w0 + b;
        if (!K && (w < 0 || w >= p.W)) continue;
        A v;
        if (K) {
          const bool ok = (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
          const A t = (A)x[ok ? h * p.W + w : 0];
          v = ok ? t : A(-INFINITY);
        } else {
          v = (A)x[h * p.W + w];
        }
        if (v > m) {
          m = v;
          am = a * KW + b;
        }
      }
    }
    idx[i] = (uint8_t)am;
  }
}

// max pooling backward, pass 2: one thread per stride band cell (nc, bh, bw) -- the sh x sw input
// cells with (h + ph) / sh == bh and (w + pw) / sw == bw share their covering windows
// oh in [bh - (KH-1-dh)/sh, bh] (dh = h + ph - bh*sh), so the index arithmetic is done once per
// band instead of once per cell; each cell sums the dout of the windows whose argmax it is
template <typename T, typename I>
__global__ void __launch_bounds__(256) pool_bwd_band(Pool p, const uint8_t* __restrict__ idx) {
  typedef typename Acc<T>::type A;
  const T* __restrict__ D = (const T*)p.D;
  T* __restrict__ O = (T*)p.out;
  const int Bh = (p.H + p.ph + p.sh - 1) / p.sh, Bw = (p.W + p.pw + p.sw - 1) / p.sw;
  const I total = (I)p.N * p.C * Bh * Bw;
  for (I t = (I)blockIdx.x * 256 + threadIdx.x; t < total; t += (I)gridDim.x * 256) {
    I q, nc;
    if constexpr (sizeof(I) == 4) {
      q = (I)fdiv((unsigned)t, p.fBw);
      nc = (I)fdiv((unsigned)q, p.fBh);
    } else {
      q = t / Bw;
      nc = q / Bh;
    }
    const int bw = (int)(t - q * Bw);
    const int bh = (int)(q - nc * Bh);
    const T* d = D + (int64_t)nc * p.Ho * p.Wo;
    const uint8_t* ix = idx + (int64_t)nc * p.Ho * p.Wo;
    T* o = O + (int64_t)nc * p.H * p.W;
    for (int dh = 0; dh < p.sh; ++dh) {
      const int h = bh * p.sh + dh - p.ph;
      if (h < 0 || h >= p.H) continue;
      const int ohl = dh <= p.KH - 1 ? max(0, bh - (p.KH - 1 - dh) / p.sh) : bh + 1;
      const int ohh = min(bh, p.Ho - 1);
      for (int dw = 0; dw < p.sw; ++dw) {
        const int w = bw * p.sw + dw - p.pw;
        if (w < 0 || w >= p.W) continue;
        const int owl = dw <= p.KW - 1 ? max(0, bw - (p.KW - 1 - dw) / p.sw) : bw + 1;
        const int owh = min(bw, p.Wo - 1);
        A g = 0;
        for (int oh = ohl; oh <= ohh; ++oh) {
          const int rh = (bh - oh) * p.sh + dh;           // row of (h, w) inside window (oh, ow)
          for (int ow = owl; ow <= owh; ++ow)
            if (ix[oh * p.Wo + ow] == rh * p.KW + (bw - ow) * p.sw + dw) g += (A)d[oh * p.Wo + ow];
        }
        o[h * p.W + w] = (T)g;
      }
    }
  }
}

// 3 x 3 / stride-2 bands (the ResNet stem pooling): a band's four cells share the windows
// oh in {bh - 1, bh} x ow in {bw - 1, bw}; their positions and dout are loaded once per band
// (4 + 4 loads instead of 9 + 9 per-cell re-reads) and each cell takes the windows whose
// argmax it is (row rh = 2 (bh - oh) + dh < 3, column likewise)
template <typename T, typename I>
__global__ void __launch_bounds__(256) pool_bwd_band_k3s2(Pool p, const uint8_t* __restrict__ idx) {
  typedef typename Acc<T>::type A;
  const T* __restrict__ D = (const T*)p.D;
  T* __restrict__ O = (T*)p.out;
  const int Bh = (p.H + p.ph + 1) / 2, Bw = (p.W + p.pw + 1) / 2;
  const I total = (I)p.N * p.C * Bh * Bw;
  for (I t = (I)blockIdx.x * 256 + threadIdx.x; t < total; t += (I)gridDim.x * 256) {
    I q, nc;
    if constexpr (sizeof(I) == 4) {
      q = (I)fdiv((unsigned)t, p.fBw);
      nc = (I)fdiv((unsigned)q, p.fBh);
    } else {
      q = t / Bw;
      nc = q / Bh;
    }
    const int bw = (int)(t - q * Bw);
    const int bh = (int)(q - nc * Bh);
    const T* d = D + (int64_t)nc * p.Ho * p.Wo;
    const uint8_t* ix = idx + (int64_t)nc * p.Ho * p.Wo;
    T* o = O + (int64_t)nc * p.H * p.W;
    int wi[2][2];
    A wd[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = bh - 1 + a, ow = bw - 1 + b;
        const bool ok = (unsigned)oh < (unsigned)p.Ho && (unsigned)ow < (unsigned)p.Wo;
        const int off = ok ? oh * p.Wo + ow : 0;
        const int iv = (int)ix[off];
        const A dv = (A)d[off];
        wi[a][b] = ok ? iv : 255;
        wd[a][b] = ok ? dv : A(0);
      }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int h = bh * 2 + dh - p.ph;
      if (h < 0 || h >= p.H) continue;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int w = bw * 2 + dw - p.pw;
        if (w < 0 || w >= p.W) continue;
        A g = 0;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int rh = 2 * (1 - a) + dh;                  // row of (h, w) in window (bh - 1 + a, .)
          if (rh > 2) continue;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int rw = 2 * (1 - b) + dw;
            if (rw > 2) continue;
            if (wi[a][b] == rh * 3 + rw) g += wd[a][b];
          }
        }
        o[h * p.W + w] = (T)g;
      }
    }
  }
}

// dX[n,c,h,w] = sum over windows containing (h,w) of dout / (KH*KW) (avg) or of dout where
// (h,w) is the window's first maximum (max: from pass 1's positions, or recomputed per window
// when no position buffer is given) -- a gather, no atomics
template <typename T, typename I>
__global__ void __launch_bounds__(256) pool_bwd(Pool p, const uint8_t* __restrict__ idx) {
  typedef typename Acc<T>::type A;
  const T* __restrict__ X = (const T*)p.X;
  const T* __restrict__ D = (const T*)p.D;
  T* __restrict__ O = (T*)p.out;
  const I total = (I)p.N * p.C * p.H * p.W;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const I q = i / p.W;
    const int w = (int)(i - q * p.W);
    const I nc = q / p.H;
    const int h = (int)(q - nc * p.H);
    const T* x = X + (int64_t)nc * p.H * p.W;
    const T* d = D + (int64_t)nc * p.Ho * p.Wo;
    const uint8_t* ix = idx ? idx + (int64_t)nc * p.Ho * p.Wo : nullptr;
    // output windows covering (h, w): oh*sh - ph <= h <= oh*sh - ph + KH - 1
    const int ohl = max(0, (h + p.ph - p.KH + p.sh) / p.sh), ohh = min(p.Ho - 1, (h + p.ph) / p.sh);
    const int owl = max(0, (w + p.pw - p.KW + p.sw) / p.sw), owh = min(p.Wo - 1, (w + p.pw) / p.sw);
    A g = 0;
    for (int oh = ohl; oh <= ohh; ++oh) {
      const int h0 = oh * p.sh - p.ph;
      if (h < h0 || h >= h0 + p.KH) continue;
      for (int ow = owl; ow <= owh; ++ow) {
        const int w0 = ow * p.sw - p.pw;
        if (w < w0 || w >= w0 + p.KW) continue;
        const A dv = (A)d[oh * p.Wo + ow];
        if (p.avg) { g += dv / A(p.KH * p.KW); continue; }
        if (ix) {
          if (ix[oh * p.Wo + ow] == (h - h0) * p.KW + (w - w0)) g += dv;
          continue;
        }
        A m = A(-INFINITY);
        int ah = -1, aw = -1;
        for (int a = 0; a < p.KH; ++a) {
          const int hh = h0 + a;
          if (hh < 0 || hh >= p.H) continue;
          for (int b = 0; b < p.KW; ++b) {
            const int ww = w0 + b;
            if (ww < 0 || ww >= p.W) continue;
            const A v = (A)x[hh * p.W + ww];
            if (v > m) { m = v; ah = hh; aw = ww; }
          }
        }
        if (ah == h && aw == w) g += dv;
      }
    }
    O[i] = (T)g;
  }
}

// ---- elementwise: bias add / multiply (channel-wise), relu backward --------------------------
// one block row per (image, channel): blockIdx.x = n*C + c, threads stride over its P cells --
// the channel is known per block, no per-element index division
template <typename T>
__global__ void __launch_bounds__(256) bias_op(const T* __restrict__ X, const T* __restrict__ b, T* __restrict__ O,
                                                int C, int P, int mult, int relu) {
  const int64_t rc = blockIdx.x;
  const int ch = (int)(rc % C);
  const T bv = b ? b[ch] : (mult ? T(1) : T(0));
  const T* x = X + rc * P;
  T* o = O + rc * P;
  for (int p = blockIdx.y * 256 + threadIdx.x; p < P; p += gridDim.y * 256) {
    T v = mult ? x[p] * bv : x[p] + bv;
    if (relu) v = v > T(0) ? v : T(0);
    o[p] = v;
  }
}

// the whole N x (C*P) operand as 4-wide vectors, one per thread -- 16-B (fp32) / 32-B (fp64)
// accesses instead of one scalar per thread.  UNI (P % 4 == 0): a vector never straddles a channel
// plane, one channel per vector; otherwise the channel of each of the 4 cells.
template <typename T, bool UNI>
__global__ void __launch_bounds__(256) bias_op_v4(const T* __restrict__ X, const T* __restrict__ b, T* __restrict__ O,
                                                   int64_t nvec, int C, int P, int mult, int relu) {
  typedef T V __attribute__((ext_vector_type(4)));
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  V v = reinterpret_cast<const V*>(X)[i];
  const T dflt = mult ? T(1) : T(0);
  if (UNI) {
    const T bv = b ? b[(int)((i / (P / 4)) % C)] : dflt;
    v = mult ? v * bv : v + bv;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const T bv = b ? b[(int)(((i * 4 + k) / P) % C)] : dflt;
      v[k] = mult ? v[k] * bv : v[k] + bv;
    }
  }
  if (relu) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = v[k] > T(0) ? v[k] : T(0);
  }
  reinterpret_cast<V*>(O)[i] = v;
}

// bf16 activations: 4 cells per thread (one 8-B load / store), fp32 bias and arithmetic, one
// rounding to bf16; total % 4 == 0 and 8-B aligned operands (host checked)
__global__ void __launch_bounds__(256) bias_op_bf16(const uint2* __restrict__ X, const float* __restrict__ b,
                                                     uint2* __restrict__ O, int64_t nvec, int C, int P, int mult,
                                                     int relu) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  const uint2 q = X[i];
  const unsigned short h[4] = {(unsigned short)(q.x & 0xffff), (unsigned short)(q.x >> 16),
                               (unsigned short)(q.y & 0xffff), (unsigned short)(q.y >> 16)};
  unsigned r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float v = __uint_as_float(((unsigned)h[k]) << 16);
    const float bv = b ? b[(int)(((i * 4 + k) / P) % C)] : (mult ? 1.f : 0.f);
    v = mult ? v * bv : v + bv;
    if (relu) v = v > 0.f ? v : 0.f;
    const unsigned u = __float_as_uint(v);
    r[k] = ((u & 0x7fffffffu) > 0x7f800000u) ? ((u >> 16) | 0x40u) : ((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  }
  O[i] = make_uint2(r[0] | (r[1] << 16), r[2] | (r[3] << 16));
}

// col2im as a gather (no atomics): dX[n][c][ih][iw] = sum over the taps (kh, kw) whose output
// position oh = (ih + ph - kh) / sh, ow = (iw + pw - kw) / sw lies on the stride grid inside the
// output, of cols[n][(c*KH + kh)*KW + kw][oh*Wo + ow].  With cols = t(W) . dY[n] (a batched
// library GEMM) this is conv2d_backward_data; fp32 accumulation, one rounding.
template <typename TI, typename TO, typename I, int S2>
__global__ void __launch_bounds__(256) col2im_gather(const TI* __restrict__ cols, TO* __restrict__ dx, int N, int C,
                                                      int H, int W, int KH, int KW, int sh, int sw, int ph, int pw,
                                                      int Ho, int Wo, FastDiv fW, FastDiv fH) {
  if (S2 == 1) { sh = 2; sw = 2; }                    // stride 2: shifts instead of divisions
  if (S2 == 2) { sh = 1; sw = 1; }                    // stride 1: no divisions
  const I total = (I)N * C * H * W;
  const I P = (I)Ho * Wo;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    I q, nc;
    if constexpr (sizeof(I) == 4) {
      q = (I)fdiv((unsigned)i, fW);
      nc = (I)fdiv((unsigned)q, fH);
    } else {
      q = i / W;
      nc = q / H;
    }
    const int iw = (int)(i - q * W);
    const int ih = (int)(q - nc * H);
    const TI* cb = cols + nc * (I)(KH * KW) * P;       // (n, c) block of KH*KW rows of P
    float acc = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int th = ih + ph - kh;
      if (th < 0) break;
      const int oh = S2 == 1 ? (th >> 1) : th / sh;
      if ((S2 == 1 ? (th & 1) != 0 : oh * sh != th) || oh >= Ho) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tw = iw + pw - kw;
        if (tw < 0) break;
        const int ow = S2 == 1 ? (tw >> 1) : tw / sw;
        if ((S2 == 1 ? (tw & 1) != 0 : ow * sw != tw) || ow >= Wo) continue;
        acc += (float)cb[(I)(kh * KW + kw) * P + oh * Wo + ow];
      }
    }
    dx[i] = (TO)acc;
  }
}

// Stride-2 col2im of bf16 with even W: one thread per input-column pair (iw = 2j, 2j + 1).  A tap
// (kh, kw) lands on the stride grid for exactly one of the two columns (the one with
// iw + pw - kw even), so each tap is one load instead of two half-masked ones, and the pair is
// one 4-byte store -- half the threads and index divisions of the per-cell gather.
struct __attribute__((aligned(4))) bf16x2 { __bf16 a, b; };

__global__ void __launch_bounds__(256) col2im_s2_pair(const __bf16* __restrict__ cols, bf16x2* __restrict__ dx, int N,
                                                      int C, int H, int W, int KH, int KW, int ph, int pw, int Ho,
                                                      int Wo) {
  const int W2 = W >> 1;
  const int total = N * C * H * W2;
  const int P = Ho * Wo;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int q = i / W2;
    const int j = i - q * W2;
    const int nc = q / H;
    const int ih = q - nc * H;
    const __bf16* cb = cols + (int64_t)nc * (KH * KW) * P;
    float a0 = 0.f, a1 = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int th = ih + ph - kh;
      if (th < 0) break;
      const int oh = th >> 1;
      if ((th & 1) != 0 || oh >= Ho) continue;
      const __bf16* row = cb + (kh * KW) * P + oh * Wo;
      for (int kw = 0; kw < KW; ++kw) {
        const int e = (pw - kw) & 1;                  // the column of the pair this tap lands on
        const int tw = 2 * j + e + pw - kw;
        if (tw < 0) continue;
        const int ow = tw >> 1;
        if (ow >= Wo) continue;
        const float v = (float)row[kw * P + ow];
        if (e) a1 += v;
        else a0 += v;
      }
    }
    dx[i] = bf16x2{(__bf16)a0, (__bf16)a1};
  }
}

// im2col: cols[n][(c*KH + kh)*KW + kw][oh*Wo + ow] = X[n][c][oh*sh - ph + kh][ow*sw - pw + kw]
// (0 outside the image); one thread per cols cell, consecutive threads along the output row
// (coalesced writes, near-coalesced reads).  Feeds the batched-GEMM forward convolution.
// Rows are Pp >= P cells apart (pixels P .. Pp-1 zero): the image-blocked GEMM of gemm.hip
// reads 8-pixel pieces, so small images are padded to a multiple of 8 here, in the one write.
template <typename T, typename I>
__global__ void __launch_bounds__(256) im2col_kernel(const T* __restrict__ X, T* __restrict__ cols, int N, int C,
                                                      int H, int W, int KH, int KW, int sh, int sw, int ph, int pw,
                                                      int Ho, int Wo, FastDiv fP, FastDiv fKK, FastDiv fKW,
                                                      FastDiv fWo, int Pp) {
  const I P = Pp, KK = (I)KH * KW;
  const I total = (I)N * C * KK * P;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    I r, nc, p;
    int t, kh, kw, oh, ow;
    if constexpr (sizeof(I) == 4) {
      r = (I)fdiv((unsigned)i, fP);                  // (n, c, kh, kw) row of cols
      p = i - r * P;
      nc = (I)fdiv((unsigned)r, fKK);
      t = (int)(r - nc * KK);
      kh = (int)fdiv((unsigned)t, fKW);
      oh = (int)fdiv((unsigned)p, fWo);
    } else {
      r = i / P;
      p = i - r * P;
      nc = r / KK;
      t = (int)(r - nc * KK);
      kh = t / KW;
      oh = (int)(p / Wo);
    }
    kw = t - kh * KW;
    ow = (int)(p - (I)oh * Wo);
    const int ih = oh * sh - ph + kh, iw = ow * sw - pw + kw;
    T v = T(0);
    if (oh < Ho && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) v = X[nc * (I)H * W + (I)ih * W + iw];
    cols[i] = v;
  }
}

inline dim3 bias_grid(int64_t rows_ch, int P) {
  int64_t gy = (P + 255) / 256;
  if (gy > 1024) gy = 1024;
  return dim3((unsigned)rows_ch, (unsigned)(gy < 1 ? 1 : gy));
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

namespace sysml_dnn {
// 128 x 128 tiles only when they still give >= 2 workgroups per CU (256 CUs): a 256-filter
// 14 x 14 layer at batch 64 has 196 such tiles and runs 1.5x faster on 64 x 64 ones
inline int conv_tile(int dtype, int64_t M, int64_t Nc, int mode = 0) {
  if (!(dtype == 0 || dtype == 3 || dtype == 4) || M < 128 || Nc < 128) return 64;
  // backward filter fills the chip by splitting its deep K: the larger tile halves the
  // gathered operand loads per MFMA
  if (mode == 2) return 128;
  return ((M + 127) / 128) * ((Nc + 127) / 128) >= 512 ? 128 : 64;
}
}  // namespace sysml_dnn

namespace sysml_dnn {

template <typename T, typename I>
void pool_launch(const Pool& p, int backward, uint8_t* ws, hipStream_t s) {
  const int64_t nin = (int64_t)p.N * p.C * p.H * p.W, nout = (int64_t)p.N * p.C * p.Ho * p.Wo;
  const bool k3 = p.KH == 3 && p.KW == 3;
  if (!backward) {
    if (p.avg && p.KH == p.H && p.KW == p.W && p.ph == 0 && p.pw == 0 && p.Ho == 1 && p.Wo == 1) {
      const int64_t planes = (int64_t)p.N * p.C;
      hipLaunchKernelGGL((pool_global_avg<T>), dim3(grid_for(planes * 64)), dim3(256), 0, s, p);
      return;
    }
    if (k3) hipLaunchKernelGGL((pool_fwd<T, I, 3>), dim3(grid_for(nout)), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((pool_fwd<T, I, 0>), dim3(grid_for(nout)), dim3(256), 0, s, p);
    return;
  }
  if (ws && !p.avg) {
    const int64_t bands = (int64_t)p.N * p.C * ((p.H + p.ph + p.sh - 1) / p.sh) * ((p.W + p.pw + p.sw - 1) / p.sw);
    if (k3) hipLaunchKernelGGL((pool_argmax<T, I, 3>), dim3(grid_for(nout)), dim3(256), 0, s, p, ws);
    else hipLaunchKernelGGL((pool_argmax<T, I, 0>), dim3(grid_for(nout)), dim3(256), 0, s, p, ws);
    if (k3 && p.sh == 2 && p.sw == 2)
      hipLaunchKernelGGL((pool_bwd_band_k3s2<T, I>), dim3(grid_for(bands)), dim3(256), 0, s, p, ws);
    else
      hipLaunchKernelGGL((pool_bwd_band<T, I>), dim3(grid_for(bands)), dim3(256), 0, s, p, ws);
    return;
  }
  hipLaunchKernelGGL((pool_bwd<T, I>), dim3(grid_for(nin)), dim3(256), 0, s, p, nullptr);
}

}  // namespace sysml_dnn

extern "C" {

// Output tile edge the launcher uses for a GEMM view (the host sizes split-K from it).
int sysml_conv2d_tile(int dtype, int64_t M, int64_t Nc) { return sysml_dnn::conv_tile(dtype, M, Nc); }
int sysml_conv2d_tile_mode(int dtype, int mode, int64_t M, int64_t Nc) {
  return sysml_dnn::conv_tile(dtype, M, Nc, mode);
}

// dtype: 0 bf16 in (fp32 out), 1 fp32 exact, 2 fp64 exact, 3 fp32 in / bf16 MFMA / fp32 out,
// 4 bf16 in / bf16 out (forward and backward data, no split-K; fp32 bias).
// mode: 0 forward, 1 backward data, 2 backward filter.  ksplit > 1 splits the GEMM depth over
// blocks; the backward filter writes per-split slices into ws (ksplit x M x Ncol of the output
// type, summed by one deterministic pass) when ws is given, else every split accumulates atomically.
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
  {
    const int es = dtype == 2 ? 8 : ((dtype == 0 || dtype == 4) ? 2 : 4);
    const int64_t rowb = (int64_t)C * KH * KW * es;
    c.avec = (rowb % 16 == 0) && (reinterpret_cast<uintptr_t>(W) % 16 == 0);
  }
  if (c.Ho <= 0 || c.Wo <= 0 || N <= 0) return -1;
  const int64_t P = (int64_t)c.Ho * c.Wo, KK = (int64_t)KH * KW;
  int64_t M, Nc, K;
  if (mode == FWD) { M = F; Nc = (int64_t)N * P; K = C * KK; }
  else if (mode == BWD_DATA) { M = C; Nc = (int64_t)N * H * Wd; K = F * KK; }
  else { M = F; Nc = C * KK; K = (int64_t)N * P; }
  // 32-bit element offsets inside the kernels
  if (M >= (1LL << 31) || Nc >= (1LL << 31) || K >= (1LL << 31)) return -1;
  if ((int64_t)N * C * H * Wd >= (1LL << 31) || (int64_t)N * F * P >= (1LL << 31) || (int64_t)F * C * KK >= (1LL << 31))
    return -1;
  c.M = (int)M; c.Ncol = (int)Nc; c.K = (int)K;
  const bool bfmma = dtype == 0 || dtype == 3 || dtype == 4;
  if (dtype == 4 && (mode == BWD_FILTER || (mode == BWD_DATA && C <= 8) || ksplit > 1)) return -1;
  const int tile = conv_tile(dtype, M, Nc, mode);    // 128 x 128 (bf16, both dims >= 128) or 64 x 64
  c.tm = (int)((M + tile - 1) / tile);
  c.tn = (int)((Nc + tile - 1) / tile);
  const int BK = bfmma ? 32 : 16;
  if (ksplit < 1) ksplit = 1;
  int64_t kper = (K + ksplit - 1) / ksplit;
  kper = (kper + BK - 1) / BK * BK;
  ksplit = (int)((K + kper - 1) / kper);
  c.ksplit = ksplit;
  c.kper = (int)kper;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (mode == BWD_DATA && C <= 8) {
    const int64_t n = (int64_t)N * C * H * Wd;
    const dim3 dg((unsigned)(n / 256 + 1 < 256 * 64 ? n / 256 + 1 : 256 * 64));
    if (dtype == 0) hipLaunchKernelGGL((conv_bwd_data_direct<__bf16, float>), dg, dim3(256), 0, s, c, (float*)out);
    else if (dtype == 1 || dtype == 3)
      hipLaunchKernelGGL((conv_bwd_data_direct<float, float>), dg, dim3(256), 0, s, c, (float*)out);
    else if (dtype == 2)
      hipLaunchKernelGGL((conv_bwd_data_direct<double, double>), dg, dim3(256), 0, s, c, (double*)out);
    else
      return -1;
    return (int)hipGetLastError();
  }
  // BWD_FILTER split-K: with a slab (ws, ksplit x M x Ncol of the output type) every split writes
  // its own slice and one pass sums them in a fixed order; without one, atomics into zeroed out
  c.slab = (mode == BWD_FILTER && ksplit > 1) ? ws : nullptr;
  if (ksplit > 1 && c.slab == nullptr) {
    const int64_t n = M * Nc;
    if (hipMemsetAsync(out, 0, n * (dtype == 2 ? 8 : 4), s) != hipSuccess) return (int)hipGetLastError();
  }
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
    if (tile == 128) LAUNCH(conv_kernel, __bf16, 0, float, 128, 128);
    else LAUNCH(conv_kernel, __bf16, 0, float, 64, 64);
  } else if (dtype == 4) {
    if (mode == FWD) {
      if (tile == 128) hipLaunchKernelGGL((conv_kernel<FWD, __bf16, 0, __bf16, 128, 128>), g, t, 0, s, c);
      else hipLaunchKernelGGL((conv_kernel<FWD, __bf16, 0, __bf16, 64, 64>), g, t, 0, s, c);
    } else {
      if (tile == 128) hipLaunchKernelGGL((conv_kernel<BWD_DATA, __bf16, 0, __bf16, 128, 128>), g, t, 0, s, c);
      else hipLaunchKernelGGL((conv_kernel<BWD_DATA, __bf16, 0, __bf16, 64, 64>), g, t, 0, s, c);
    }
  } else if (dtype == 3) {
    if (tile == 128) LAUNCH(conv_kernel, float, 0, float, 128, 128);
    else LAUNCH(conv_kernel, float, 0, float, 64, 64);
  } else if (dtype == 1) {
    LAUNCH(conv_kernel, float, 1, float, 64, 64);
  } else if (dtype == 2) {
    LAUNCH(conv_kernel, double, 2, double, 64, 64);
  } else {
    return -1;
  }
#undef LAUNCH
  if (c.slab != nullptr) {
    const int64_t n = M * Nc;
    const dim3 rg((unsigned)(n / 256 + 1 < 4096 ? n / 256 + 1 : 4096));
    if (dtype == 2) hipLaunchKernelGGL(slab_reduce<double>, rg, dim3(256), 0, s, (const double*)ws, (double*)out, n, ksplit);
    else hipLaunchKernelGGL(slab_reduce<float>, rg, dim3(256), 0, s, (const float*)ws, (float*)out, n, ksplit);
  }
  if (ksplit > 1 && mode == FWD && (bias || relu)) {
    const int64_t n = M * Nc;
    const dim3 bg = bias_grid(n / P, (int)P);
    if (dtype == 2)
      hipLaunchKernelGGL(bias_op<double>, bg, dim3(256), 0, s, (const double*)out,
                         bias ? (const double*)bias : nullptr, (double*)out, F, (int)P, 0, relu);
    else
      hipLaunchKernelGGL(bias_op<float>, bg, dim3(256), 0, s, (const float*)out,
                         bias ? (const float*)bias : nullptr, (float*)out, F, (int)P, 0, relu);
  }
  return (int)hipGetLastError();
}

// dtype 1 fp32, 2 fp64, 3 bf16 (fp32 math); backward: D = dout, out = dX; ws: N*C*Ho*Wo bytes for the window argmax
// positions of max-pooling backward (nullptr: recomputed per covered window)
int sysml_pool2d_ws(int dtype, int backward, int avg, const void* X, const void* D, void* out, void* ws, int N, int C,
                    int H, int W, int KH, int KW, int sh, int sw, int ph, int pw, void* stream) {
  using namespace sysml_dnn;
  Pool p;
  p.X = X; p.D = D; p.out = out; p.N = N; p.C = C; p.H = H; p.W = W; p.KH = KH; p.KW = KW; p.sh = sh; p.sw = sw;
  p.ph = ph; p.pw = pw; p.avg = avg;
  p.Ho = (H + 2 * ph - KH) / sh + 1;
  p.Wo = (W + 2 * pw - KW) / sw + 1;
  if (p.Ho <= 0 || p.Wo <= 0) return -1;
  p.fWo = fastdiv(p.Wo);
  p.fHo = fastdiv(p.Ho);
  p.fBw = fastdiv((W + pw + sw - 1) / sw);
  p.fBh = fastdiv((H + ph + sh - 1) / sh);
  if (KH * KW > 255) ws = nullptr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool small = (int64_t)N * C * H * W < (1LL << 31) && (int64_t)N * C * p.Ho * p.Wo < (1LL << 31);
  uint8_t* w8 = static_cast<uint8_t*>(ws);
  if (dtype == 1) {
    if (small) pool_launch<float, int>(p, backward, w8, s);
    else pool_launch<float, int64_t>(p, backward, w8, s);
  } else if (dtype == 2) {
    if (small) pool_launch<double, int>(p, backward, w8, s);
    else pool_launch<double, int64_t>(p, backward, w8, s);
  } else if (dtype == 3) {
    if (small) pool_launch<__bf16, int>(p, backward, w8, s);
    else pool_launch<__bf16, int64_t>(p, backward, w8, s);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

int sysml_pool2d(int dtype, int backward, int avg, const void* X, const void* D, void* out, int N, int C, int H,
                 int W, int KH, int KW, int sh, int sw, int ph, int pw, void* stream) {
  return sysml_pool2d_ws(dtype, backward, avg, X, D, out, nullptr, N, C, H, W, KH, KW, sh, sw, ph, pw, stream);
}

int sysml_bias_op(int dtype, const void* X, const void* b, void* out, int64_t total, int C, int P, int mult, int relu,
                  void* stream) {
  using namespace sysml_dnn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (P <= 0 || total % P) return -1;
  if (dtype == 3) {                      // bf16 storage, fp32 bias (dtype 3)
    if (total % 4 || (uintptr_t)X % 8 || (uintptr_t)out % 8) return -1;
    const int64_t nvec = total / 4;
    hipLaunchKernelGGL(bias_op_bf16, dim3((unsigned)((nvec + 255) / 256)), dim3(256), 0, s, (const uint2*)X,
                       (const float*)b, (uint2*)out, nvec, C, P, mult, relu);
    return (int)hipGetLastError();
  }
  const bool v4 = total % 4 == 0 && (uintptr_t)X % (dtype == 1 ? 16 : 32) == 0 &&
                  (uintptr_t)out % (dtype == 1 ? 16 : 32) == 0 && total / 4 < (int64_t)0x7fffffff * 256;
  if (v4 && (dtype == 1 || dtype == 2)) {
    const int64_t nvec = total / 4;
    const dim3 g((unsigned)((nvec + 255) / 256));
    const bool uni = P % 4 == 0;
#define SYSML_BIAS_V4(TT, U)                                                                                  \
  hipLaunchKernelGGL((bias_op_v4<TT, U>), g, dim3(256), 0, s, (const TT*)X, (const TT*)b, (TT*)out, nvec, C, P, \
                     mult, relu)
    if (dtype == 1) {
      if (uni) SYSML_BIAS_V4(float, true);
      else SYSML_BIAS_V4(float, false);
    } else {
      if (uni) SYSML_BIAS_V4(double, true);
      else SYSML_BIAS_V4(double, false);
    }
#undef SYSML_BIAS_V4
    return (int)hipGetLastError();
  }
  const dim3 bg = bias_grid(total / P, P);
  if (dtype == 1)
    hipLaunchKernelGGL(bias_op<float>, bg, dim3(256), 0, s, (const float*)X, (const float*)b, (float*)out, C, P, mult,
                       relu);
  else if (dtype == 2)
    hipLaunchKernelGGL(bias_op<double>, bg, dim3(256), 0, s, (const double*)X, (const double*)b, (double*)out, C, P,
                       mult, relu);
  else
    return -1;
  return (int)hipGetLastError();
}

// dtype 3: bf16, 1: fp32.  X: N x C*H*W -> cols: N x (C*KH*KW) x Pp, Pp >= Ho*Wo (zero padded).
int sysml_im2col_pad(int dtype, const void* X, void* cols, int N, int C, int H, int W, int KH, int KW, int sh, int sw,
                     int ph, int pw, int Pp, void* stream) {
  using namespace sysml_dnn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int Ho = (H + 2 * ph - KH) / sh + 1, Wo = (W + 2 * pw - KW) / sw + 1;
  if (Ho <= 0 || Wo <= 0 || N <= 0 || Pp < Ho * Wo) return -1;
  const int64_t total = (int64_t)N * C * KH * KW * Pp;
  const bool small = total < (1LL << 31) && (int64_t)N * C * H * W < (1LL << 31);
  const dim3 g(grid_for(total));
  const FastDiv fP = fastdiv(Pp), fKK = fastdiv(KH * KW), fKW = fastdiv(KW), fWo = fastdiv(Wo);
  if (dtype == 3) {
    if (small) hipLaunchKernelGGL((im2col_kernel<__bf16, int>), g, dim3(256), 0, s, (const __bf16*)X, (__bf16*)cols, N, C, H, W, KH, KW, sh, sw, ph, pw, Ho, Wo, fP, fKK, fKW, fWo, Pp);
    else hipLaunchKernelGGL((im2col_kernel<__bf16, int64_t>), g, dim3(256), 0, s, (const __bf16*)X, (__bf16*)cols, N, C, H, W, KH, KW, sh, sw, ph, pw, Ho, Wo, fP, fKK, fKW, fWo, Pp);
  } else if (dtype == 1) {
    if (small) hipLaunchKernelGGL((im2col_kernel<float, int>), g, dim3(256), 0, s, (const float*)X, (float*)cols, N, C, H, W, KH, KW, sh, sw, ph, pw, Ho, Wo, fP, fKK, fKW, fWo, Pp);
    else hipLaunchKernelGGL((im2col_kernel<float, int64_t>), g, dim3(256), 0, s, (const float*)X, (float*)cols, N, C, H, W, KH, KW, sh, sw, ph, pw, Ho, Wo, fP, fKK, fKW, fWo, Pp);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

int sysml_im2col(int dtype, const void* X, void* cols, int N, int C, int H, int W, int KH, int KW, int sh, int sw,
                 int ph, int pw, void* stream) {
  const int Ho = (H + 2 * ph - KH) / sh + 1, Wo = (W + 2 * pw - KW) / sw + 1;
  return sysml_im2col_pad(dtype, X, cols, N, C, H, W, KH, KW, sh, sw, ph, pw, Ho * Wo, stream);
}

// dtype 3: bf16 cols -> bf16 dX; 1: fp32 -> fp32.  cols: N x (C*KH*KW) x (Ho*Wo), dx: N x C*H*W.
int sysml_col2im(int dtype, const void* cols, void* dx, int N, int C, int H, int W, int KH, int KW, int sh, int sw,
                 int ph, int pw, void* stream) {
  using namespace sysml_dnn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int Ho = (H + 2 * ph - KH) / sh + 1, Wo = (W + 2 * pw - KW) / sw + 1;
  if (Ho <= 0 || Wo <= 0 || N <= 0) return -1;
  const int64_t total = (int64_t)N * C * H * W, ncols = (int64_t)N * C * KH * KW * Ho * Wo;
  const bool small = total < (1LL << 31) && ncols < (1LL << 31);
  const dim3 g(grid_for(total));
  const bool s2 = sh == 2 && sw == 2;
  const FastDiv fW = fastdiv(W), fH = fastdiv(H);
#define SYSML_C2I(TI, TO)                                                                                        \
  do {                                                                                                           \
    if (small && s2)                                                                                             \
      hipLaunchKernelGGL((col2im_gather<TI, TO, int, 1>), g, dim3(256), 0, s, (const TI*)cols, (TO*)dx, N, C, H, W, \
                         KH, KW, sh, sw, ph, pw, Ho, Wo, fW, fH);                                                        \
    else if (small && sh == 1 && sw == 1)                                                                        \
      hipLaunchKernelGGL((col2im_gather<TI, TO, int, 2>), g, dim3(256), 0, s, (const TI*)cols, (TO*)dx, N, C, H, W, \
                         KH, KW, sh, sw, ph, pw, Ho, Wo, fW, fH);                                                \
    else if (small)                                                                                              \
      hipLaunchKernelGGL((col2im_gather<TI, TO, int, 0>), g, dim3(256), 0, s, (const TI*)cols, (TO*)dx, N, C, H, W, \
                         KH, KW, sh, sw, ph, pw, Ho, Wo, fW, fH);                                                        \
    else                                                                                                         \
      hipLaunchKernelGGL((col2im_gather<TI, TO, int64_t, 0>), g, dim3(256), 0, s, (const TI*)cols, (TO*)dx, N, C, H, \
                         W, KH, KW, sh, sw, ph, pw, Ho, Wo, fW, fH);                                                     \
  } while (0)
  if (dtype == 3 && small && s2 && W % 2 == 0)
    hipLaunchKernelGGL(col2im_s2_pair, dim3(grid_for(total / 2)), dim3(256), 0, s, (const __bf16*)cols, (bf16x2*)dx, N,
                       C, H, W, KH, KW, ph, pw, Ho, Wo);
  else if (dtype == 3) SYSML_C2I(__bf16, __bf16);
  else if (dtype == 1) SYSML_C2I(float, float);
  else return -1;
#undef SYSML_C2I
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
