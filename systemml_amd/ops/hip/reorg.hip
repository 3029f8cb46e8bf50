// Append and left-indexing of device matrices (reference: the cbind / rbind kernels of
// SystemML.cu:835-889 and the slice / left-index paths of LibMatrixCUDA / LibMatrixReorg).
//
//   * cbind / rbind of up to 16 row-major operands in ONE pass over the output: every thread
//     writes 4 consecutive output cells of a row and reads them from the operand that owns
//     those columns (cbind) or rows (rbind) -- no per-operand launch, no intermediate;
//   * X[r0:r1, c0:c1] = Y (or a scalar) as one pass that writes every output cell once, reading
//     it from X outside the window and from Y inside it (instead of a copy of X followed by a
//     second strided write of the window); when the output IS X (update in place, compiler/
//     loops.py) only the window is written.
// Element types: 2-byte (bf16), 4-byte (fp32) and 8-byte (fp64) cells, copied bit for bit.
//
// Right indexing / reorganisation (reference: slice_dense_dense / slice_sparse_dense_row /
// lower.tri copies of SystemML.cu:301-429, the dgeam transpose of LibMatrixCUDA.java:1593 and
// the slice paths of LibMatrixCUDA.java:1756-1834), so no ATen copy kernel touches HBM data:
//   * copy2d: a strided window (X[r0:r1, c0:c1] as a view) to a dense matrix, optionally
//     converting bf16 / fp32 / fp64 -- one pass for slices, contiguous copies and casts; narrow
//     windows (< 64 columns, the N x K vectors of the solvers) run one thread per cell with a
//     multiply-high division by the width, wide ones a wave per row;
//   * transpose: 64 x 64 tiles through LDS (row pitch 65, conflict-free for the column reads),
//     strided input; narrow (<= 16 wide / tall) shapes a thread per row / column instead;
//   * tri: lower.tri / upper.tri with or without the diagonal, values or ones, in one pass;
//   * gather_rows: out = X[idx, ] (order / removeEmpty / permutation products);
//   * slice_csr: X[r0:r1, c0:c1] of a CSR matrix into a dense window, a wave per row
//     (binary search of the first column, then the row's cells in range).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_rg {

constexpr int NT = 256;
constexpr int MAXIN = 16;

struct Cat {
  const void* src[MAXIN];
  int64_t off[MAXIN + 1];     // first output column (cbind) / row (rbind) of operand k; off[n] = total
  int64_t ld[MAXIN];          // columns of operand k
  int n;
};

template <typename T, bool ROWS>
__global__ void __launch_bounds__(NT) cat_kernel(const Cat c, T* __restrict__ out, int64_t N, int64_t D) {
  const int64_t groups = (D + 3) / 4;
  const int64_t total = N * groups;
  for (int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x; g < total; g += (int64_t)gridDim.x * NT) {
    const int64_t r = g / groups;
    const int64_t c0 = (g - r * groups) * 4;
    int k = 0;
    if (ROWS) {
      while (k + 1 < c.n && r >= c.off[k + 1]) ++k;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t col = c0 + u;
      if (col >= D) break;
      if (!ROWS) {
        while (k + 1 < c.n && col >= c.off[k + 1]) ++k;
        out[r * D + col] = static_cast<const T*>(c.src[k])[r * c.ld[k] + (col - c.off[k])];
      } else {
        out[r * D + col] = static_cast<const T*>(c.src[k])[(r - c.off[k]) * D + col];
      }
    }
  }
}

// the bit pattern of a device-resident fp64 scalar in the cell type of T (bf16: round to
// nearest even of its fp32 value)
template <typename T> __device__ __forceinline__ T dev_bits(double d);
template <> __device__ __forceinline__ uint64_t dev_bits<uint64_t>(double d) { return (uint64_t)__double_as_longlong(d); }
template <> __device__ __forceinline__ uint32_t dev_bits<uint32_t>(double d) { return __float_as_uint((float)d); }
template <> __device__ __forceinline__ uint16_t dev_bits<uint16_t>(double d) {
  uint32_t u = __float_as_uint((float)d);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <typename T>
__global__ void __launch_bounds__(NT) lix_kernel(const T* X, const T* __restrict__ Y, T* out,   // out may be X
                                                 int64_t N, int64_t D, int64_t r0, int64_t r1, int64_t c0,
                                                 int64_t c1, int scalar, T sval, int window_only,
                                                 const double* __restrict__ sdev) {
  if (sdev != nullptr) sval = dev_bits<T>(*sdev);     // a device scalar: no host round trip
  const int64_t wr = r1 - r0, wc = c1 - c0;
  const int64_t total = window_only ? wr * wc : N * D;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    int64_t r, c;
    if (window_only) {
      r = r0 + i / wc;
      c = c0 + (i % wc);
    } else {
      r = i / D;
      c = i - r * D;
    }
    const bool in = r >= r0 && r < r1 && c >= c0 && c < c1;
    T v;
    if (in) v = scalar ? sval : Y[(r - r0) * wc + (c - c0)];
    else v = X[i];
    out[r * D + c] = v;
  }
}

template <typename T>
void launch_cat(int rows, dim3 g, hipStream_t st, const Cat& c, void* out, int64_t N, int64_t D) {
  if (rows) hipLaunchKernelGGL((cat_kernel<T, true>), g, dim3(NT), 0, st, c, (T*)out, N, D);
  else hipLaunchKernelGGL((cat_kernel<T, false>), g, dim3(NT), 0, st, c, (T*)out, N, D);
}

inline int grid_for(int64_t work) {
  int64_t g = (work + NT - 1) / NT;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}


// ---------------------------------------------------------------------------------------------
// right indexing / copies / casts / transpose / tri / row gathers
// ---------------------------------------------------------------------------------------------
// storage codes: 0 = bf16 (uint16 bits), 1 = fp32, 2 = fp64
__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);   // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
template <typename To, typename Ti> __device__ __forceinline__ To cvt(Ti v);
template <> __device__ __forceinline__ uint16_t cvt<uint16_t, uint16_t>(uint16_t v) { return v; }
template <> __device__ __forceinline__ float cvt<float, uint16_t>(uint16_t v) { return bf2f(v); }
template <> __device__ __forceinline__ double cvt<double, uint16_t>(uint16_t v) { return (double)bf2f(v); }
template <> __device__ __forceinline__ uint16_t cvt<uint16_t, float>(float v) { return f2bf(v); }
template <> __device__ __forceinline__ float cvt<float, float>(float v) { return v; }
template <> __device__ __forceinline__ double cvt<double, float>(float v) { return (double)v; }
template <> __device__ __forceinline__ uint16_t cvt<uint16_t, double>(double v) { return f2bf((float)v); }
template <> __device__ __forceinline__ float cvt<float, double>(double v) { return (float)v; }
template <> __device__ __forceinline__ double cvt<double, double>(double v) { return v; }

// n / d for n < 2^31 by multiply-high (Granlund-Montgomery): q = (umulhi(n, m) + n) >> s
struct FastDiv {
  uint32_t d, m, s;
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> s; }
};
inline FastDiv make_div(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

template <typename Ti, typename To>
__global__ void __launch_bounds__(NT) copy_flat(const Ti* __restrict__ X, int64_t lds, To* __restrict__ out,
                                                 int64_t ldo, uint32_t total, FastDiv w) {
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t r = w.div(i), c = i - r * w.d;
    out[(int64_t)r * ldo + c] = cvt<To, Ti>(X[(int64_t)r * lds + c]);
  }
}

template <typename Ti, typename To>
__global__ void __launch_bounds__(NT) copy_rows(const Ti* __restrict__ X, int64_t lds, To* __restrict__ out,
                                                 int64_t ldo, int64_t nr, int64_t nc) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (NT / 64) + w; r < nr; r += (int64_t)gridDim.x * (NT / 64)) {
    const Ti* xr = X + r * lds;
    To* orow = out + r * ldo;
    int64_t c = l;
    for (; c + 192 < nc; c += 256) {
      const Ti a = xr[c], b = xr[c + 64], d = xr[c + 128], e = xr[c + 192];
      orow[c] = cvt<To, Ti>(a);
      orow[c + 64] = cvt<To, Ti>(b);
      orow[c + 128] = cvt<To, Ti>(d);
      orow[c + 192] = cvt<To, Ti>(e);
    }
    for (; c < nc; c += 64) orow[c] = cvt<To, Ti>(xr[c]);
  }
}

// out (D x N, dense) = t(X) for X N x D with row pitch lds
template <typename T>
__global__ void __launch_bounds__(NT) transpose_tile(const T* __restrict__ X, int64_t lds, T* __restrict__ out,
                                                      int64_t N, int64_t D) {
  __shared__ T tile[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t tilesD = (D + 63) / 64, tiles = ((N + 63) / 64) * tilesD;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t r0 = (t / tilesD) * 64, c0 = (t % tilesD) * 64;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int rr = ty + 4 * k;
      const int64_t r = r0 + rr, c = c0 + tx;
      if (r < N && c < D) tile[rr][tx] = X[r * lds + c];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int cc = ty + 4 * k;
      const int64_t c = c0 + cc, r = r0 + tx;
      if (c < D && r < N) out[c * N + r] = tile[tx][cc];
    }
    __syncthreads();
  }
}

// narrow X (D <= 16): a thread per input row writes its D cells into D output rows (coalesced
// writes; the row's cells come from one or two cache lines)
template <typename T>
__global__ void __launch_bounds__(NT) transpose_narrow(const T* __restrict__ X, int64_t lds, T* __restrict__ out,
                                                        int64_t N, int D) {
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < N; r += (int64_t)gridDim.x * NT) {
    const T* xr = X + r * lds;
    for (int c = 0; c < D; ++c) out[(int64_t)c * N + r] = xr[c];
  }
}

// short X (N <= 16): a thread per input column writes its N cells as one output row
template <typename T>
__global__ void __launch_bounds__(NT) transpose_short(const T* __restrict__ X, int64_t lds, T* __restrict__ out,
                                                       int N, int64_t D) {
  for (int64_t c = (int64_t)blockIdx.x * NT + threadIdx.x; c < D; c += (int64_t)gridDim.x * NT)
    for (int r = 0; r < N; ++r) out[c * N + r] = X[(int64_t)r * lds + c];
}

template <typename T> __device__ __forceinline__ T one_bits();
template <> __device__ __forceinline__ uint16_t one_bits<uint16_t>() { return 0x3f80u; }
template <> __device__ __forceinline__ uint32_t one_bits<uint32_t>() { return 0x3f800000u; }
template <> __device__ __forceinline__ uint64_t one_bits<uint64_t>() { return 0x3ff0000000000000ull; }

// lower (upper) triangle of X: cells with c <= r (c >= r), strictly without the diagonal when
// diag = 0; `values` = 0 writes ones instead of X's cells
template <typename T>
__global__ void __launch_bounds__(NT) tri_kernel(const T* __restrict__ X, T* __restrict__ out, int64_t N, int64_t D,
                                                  int lower, int diag, int values) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (NT / 64) + w; r < N; r += (int64_t)gridDim.x * (NT / 64)) {
    for (int64_t c = l; c < D; c += 64) {
      const bool in = lower ? (diag ? c <= r : c < r) : (diag ? c >= r : c > r);
      out[r * D + c] = in ? (values ? X[r * D + c] : one_bits<T>()) : (T)0;
    }
  }
}

template <typename T, typename I>
__global__ void __launch_bounds__(NT) gather_rows_kernel(const T* __restrict__ X, int64_t lds, const I* __restrict__ idx,
                                                          T* __restrict__ out, int64_t n, int64_t D) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (NT / 64) + w; r < n; r += (int64_t)gridDim.x * (NT / 64)) {
    const T* xr = X + (int64_t)idx[r] * lds;
    for (int64_t c = l; c < D; c += 64) out[r * D + c] = xr[c];
  }
}

template <typename T, typename I>
__global__ void __launch_bounds__(NT) gather_rows_narrow(const T* __restrict__ X, int64_t lds, const I* __restrict__ idx,
                                                          T* __restrict__ out, uint32_t total, FastDiv w) {
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t r = w.div(i), c = i - r * w.d;
    out[(int64_t)i] = X[(int64_t)idx[r] * lds + c];
  }
}

// X[r0:r1, c0:c1] of CSR (rowptr / col / val) into a dense zero-initialised window: a wave per row,
// first in-range column by binary search, then the lanes stride the row's cells in range
template <typename V, typename I>
__global__ void __launch_bounds__(NT) slice_csr_kernel(const I* __restrict__ rowptr, const I* __restrict__ col,
                                                        const V* __restrict__ val, V* __restrict__ out, int64_t r0,
                                                        int64_t r1, int64_t c0, int64_t c1) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t wc = c1 - c0;
  for (int64_t r = r0 + (int64_t)blockIdx.x * (NT / 64) + w; r < r1; r += (int64_t)gridDim.x * (NT / 64)) {
    int64_t lo = rowptr[r], hi = rowptr[r + 1];
    int64_t a = lo, b = hi;
    while (a < b) {                       // first cell with col >= c0
      const int64_t m = (a + b) >> 1;
      if ((int64_t)col[m] < c0) a = m + 1; else b = m;
    }
    for (int64_t k = a + l; k < hi; k += 64) {
      const int64_t c = col[k];
      if (c >= c1) break;
      out[(r - r0) * wc + (c - c0)] = val[k];
    }
  }
}

template <typename Ti, typename To>
int launch_copy(const void* X, int64_t lds, void* out, int64_t ldo, int64_t nr, int64_t nc, hipStream_t st) {
  if (nc < 64 && nr * nc < (1ll << 31)) {
    const uint32_t total = (uint32_t)(nr * nc);
    hipLaunchKernelGGL((copy_flat<Ti, To>), dim3(grid_for(total)), dim3(NT), 0, st, (const Ti*)X, lds, (To*)out, ldo,
                       total, make_div((uint32_t)nc));
  } else {
    hipLaunchKernelGGL((copy_rows<Ti, To>), dim3(grid_for(nr * 64)), dim3(NT), 0, st, (const Ti*)X, lds, (To*)out,
                       ldo, nr, nc);
  }
  return 0;
}

template <typename Ti>
int launch_copy_to(int tout, const void* X, int64_t lds, void* out, int64_t ldo, int64_t nr, int64_t nc,
                   hipStream_t st) {
  if (tout == 0) return launch_copy<Ti, uint16_t>(X, lds, out, ldo, nr, nc, st);
  if (tout == 1) return launch_copy<Ti, float>(X, lds, out, ldo, nr, nc, st);
  if (tout == 2) return launch_copy<Ti, double>(X, lds, out, ldo, nr, nc, st);
  return -1;
}

template <typename T>
void launch_transpose(const void* X, int64_t lds, void* out, int64_t N, int64_t D, hipStream_t st) {
  if (D <= 16) {
    hipLaunchKernelGGL(transpose_narrow<T>, dim3(grid_for(N)), dim3(NT), 0, st, (const T*)X, lds, (T*)out, N, (int)D);
  } else if (N <= 16) {
    hipLaunchKernelGGL(transpose_short<T>, dim3(grid_for(D)), dim3(NT), 0, st, (const T*)X, lds, (T*)out, (int)N, D);
  } else {
    const int64_t tiles = ((N + 63) / 64) * ((D + 63) / 64);
    const int g = (int)(tiles < 4096 ? tiles : 4096);
    hipLaunchKernelGGL(transpose_tile<T>, dim3(g), dim3(NT), 0, st, (const T*)X, lds, (T*)out, N, D);
  }
}

}  // namespace sysml_rg

extern "C" {

// rows = 0: cbind (operands N x ld[k], output N x D), 1: rbind (operands rows_k x D, output N x D).
// esize: bytes per cell (2, 4, 8).  off: n + 1 prefix offsets (columns for cbind, rows for rbind).
int sysml_cat(int rows, int esize, int n, const void* const* srcs, const int64_t* off, const int64_t* ld, void* out,
              int64_t N, int64_t D, void* stream) {
  using namespace sysml_rg;
  if (n < 1 || n > MAXIN || N <= 0 || D <= 0) return -1;
  Cat c;
  for (int k = 0; k < n; ++k) {
    c.src[k] = srcs[k];
    c.off[k] = off[k];
    c.ld[k] = ld[k];
  }
  c.off[n] = off[n];
  c.n = n;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid_for(N * ((D + 3) / 4)));
  if (esize == 2) launch_cat<uint16_t>(rows, g, st, c, out, N, D);
  else if (esize == 4) launch_cat<uint32_t>(rows, g, st, c, out, N, D);
  else if (esize == 8) launch_cat<uint64_t>(rows, g, st, c, out, N, D);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// out = X with out[r0:r1, c0:c1] (0-based, half-open) = Y (wr x wc row-major) or the scalar bit
// pattern `sbits`; out == X: only the window is written.
int sysml_lix2(int esize, const void* X, const void* Y, void* out, int64_t N, int64_t D, int64_t r0, int64_t r1,
               int64_t c0, int64_t c1, int scalar, uint64_t sbits, const double* sdev, void* stream);

int sysml_lix(int esize, const void* X, const void* Y, void* out, int64_t N, int64_t D, int64_t r0, int64_t r1,
              int64_t c0, int64_t c1, int scalar, uint64_t sbits, void* stream) {
  return sysml_lix2(esize, X, Y, out, N, D, r0, r1, c0, c1, scalar, sbits, nullptr, stream);
}

// as sysml_lix; sdev (scalar mode): the value is read on the device from this fp64 cell
int sysml_lix2(int esize, const void* X, const void* Y, void* out, int64_t N, int64_t D, int64_t r0, int64_t r1,
               int64_t c0, int64_t c1, int scalar, uint64_t sbits, const double* sdev, void* stream) {
  using namespace sysml_rg;
  if (N <= 0 || D <= 0 || r0 < 0 || r1 > N || c0 < 0 || c1 > D || r0 >= r1 || c0 >= c1) return -1;
  if (!scalar && Y == nullptr) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int wo = out == X ? 1 : 0;
  const dim3 g(grid_for(wo ? (r1 - r0) * (c1 - c0) : N * D));
  if (esize == 2)
    hipLaunchKernelGGL(lix_kernel<uint16_t>, g, dim3(NT), 0, st, (const uint16_t*)X, (const uint16_t*)Y,
                       (uint16_t*)out, N, D, r0, r1, c0, c1, scalar, (uint16_t)sbits, wo, sdev);
  else if (esize == 4)
    hipLaunchKernelGGL(lix_kernel<uint32_t>, g, dim3(NT), 0, st, (const uint32_t*)X, (const uint32_t*)Y,
                       (uint32_t*)out, N, D, r0, r1, c0, c1, scalar, (uint32_t)sbits, wo, sdev);
  else if (esize == 8)
    hipLaunchKernelGGL(lix_kernel<uint64_t>, g, dim3(NT), 0, st, (const uint64_t*)X, (const uint64_t*)Y,
                       (uint64_t*)out, N, D, r0, r1, c0, c1, scalar, sbits, wo, sdev);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


// window copy / cast: out[r, c] (row pitch ldo) = X[r, c] (row pitch lds), r < nr, c < nc;
// tin / tout: 0 bf16, 1 fp32, 2 fp64
int sysml_copy2d(int tin, int tout, const void* X, int64_t lds, void* out, int64_t ldo, int64_t nr, int64_t nc,
                 void* stream) {
  using namespace sysml_rg;
  if (nr <= 0 || nc <= 0) return 0;
  if (lds < nc || ldo < nc) return -1;
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if (tin == 0) rc = launch_copy_to<uint16_t>(tout, X, lds, out, ldo, nr, nc, st);
  else if (tin == 1) rc = launch_copy_to<float>(tout, X, lds, out, ldo, nr, nc, st);
  else if (tin == 2) rc = launch_copy_to<double>(tout, X, lds, out, ldo, nr, nc, st);
  else return -1;
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// out (D x N, dense) = t(X), X N x D with row pitch lds; esize 2 / 4 / 8
int sysml_transpose(int esize, const void* X, int64_t lds, void* out, int64_t N, int64_t D, void* stream) {
  using namespace sysml_rg;
  if (N <= 0 || D <= 0) return 0;
  if (lds < D) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (esize == 2) launch_transpose<uint16_t>(X, lds, out, N, D, st);
  else if (esize == 4) launch_transpose<uint32_t>(X, lds, out, N, D, st);
  else if (esize == 8) launch_transpose<uint64_t>(X, lds, out, N, D, st);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int sysml_tri(int esize, const void* X, void* out, int64_t N, int64_t D, int lower, int diag, int values,
              void* stream) {
  using namespace sysml_rg;
  if (N <= 0 || D <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid_for(N * 64));
  if (esize == 2)
    hipLaunchKernelGGL(tri_kernel<uint16_t>, g, dim3(NT), 0, st, (const uint16_t*)X, (uint16_t*)out, N, D, lower,
                       diag, values);
  else if (esize == 4)
    hipLaunchKernelGGL(tri_kernel<uint32_t>, g, dim3(NT), 0, st, (const uint32_t*)X, (uint32_t*)out, N, D, lower,
                       diag, values);
  else if (esize == 8)
    hipLaunchKernelGGL(tri_kernel<uint64_t>, g, dim3(NT), 0, st, (const uint64_t*)X, (uint64_t*)out, N, D, lower,
                       diag, values);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// out (n x D, dense) = X[idx, ] (0-based int32 / int64 row indices; X rows pitch lds)
int sysml_gather_rows(int esize, int idx64, const void* X, int64_t lds, const void* idx, void* out, int64_t n,
                      int64_t D, void* stream) {
  using namespace sysml_rg;
  if (n <= 0 || D <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
#define SYSML_GATHER(T, I)                                                                                      \
  do {                                                                                                          \
    if (D < 64 && n * D < (1ll << 31)) {                                                                        \
      const uint32_t total = (uint32_t)(n * D);                                                                 \
      hipLaunchKernelGGL((gather_rows_narrow<T, I>), dim3(grid_for(total)), dim3(NT), 0, st, (const T*)X, lds,  \
                         (const I*)idx, (T*)out, total, make_div((uint32_t)D));                                \
    } else {                                                                                                    \
      hipLaunchKernelGGL((gather_rows_kernel<T, I>), dim3(grid_for(n * 64)), dim3(NT), 0, st, (const T*)X, lds, \
                         (const I*)idx, (T*)out, n, D);                                                         \
    }                                                                                                           \
  } while (0)
  if (esize == 2) { if (idx64) SYSML_GATHER(uint16_t, int64_t); else SYSML_GATHER(uint16_t, int32_t); }
  else if (esize == 4) { if (idx64) SYSML_GATHER(uint32_t, int64_t); else SYSML_GATHER(uint32_t, int32_t); }
  else if (esize == 8) { if (idx64) SYSML_GATHER(uint64_t, int64_t); else SYSML_GATHER(uint64_t, int32_t); }
  else return -1;
#undef SYSML_GATHER
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// dense (r1-r0) x (c1-c0) window of a CSR matrix; `out` must be zero-filled by the caller.
// vcode: 1 fp32 / 2 fp64 values; idx64: int64 (else int32) row pointers and column indices
int sysml_slice_csr(int vcode, int idx64, const void* rowptr, const void* col, const void* val, void* out,
                    int64_t r0, int64_t r1, int64_t c0, int64_t c1, void* stream) {
  using namespace sysml_rg;
  if (r1 <= r0 || c1 <= c0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid_for((r1 - r0) * 64));
#define SYSML_SLICE(V, I)                                                                                   \
  hipLaunchKernelGGL((slice_csr_kernel<V, I>), g, dim3(NT), 0, st, (const I*)rowptr, (const I*)col,         \
                     (const V*)val, (V*)out, r0, r1, c0, c1)
  if (vcode == 1) { if (idx64) SYSML_SLICE(float, int64_t); else SYSML_SLICE(float, int32_t); }
  else if (vcode == 2) { if (idx64) SYSML_SLICE(double, int64_t); else SYSML_SLICE(double, int32_t); }
  else return -1;
#undef SYSML_SLICE
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
