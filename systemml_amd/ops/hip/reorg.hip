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

}  // extern "C"
