// CSR sparse x dense products for the sparse matrix-multiply path (ops/sparse.py; reference:
// LibMatrixMult.java#matrixMultSparseDense / matrixMultSparseDenseMVShortRHS and the cuSPARSE
// csrmm / csrmv calls of LibMatrixCuMatMult.java).
//
//   spmm   C[m, :] = sum_p A.val[p] * B[A.col[p], :]            (A: CSR m x n, B: n x K dense)
//   spmm_t C[j, :] += A.val[p] * B[i, :] for every non-zero p=(i,j)  (t(A) %*% B, A: CSR m x n)
//
// CDNA4 mapping.  spmm: a wavefront owns one CSR row at a time (grid-stride); its 64 lanes are
// split into groups of G lanes, G = smallest power of two >= K (capped at 64): each group
// walks its share of the row's non-zeros and each lane accumulates one output column (K > 64:
// the columns loop in chunks of 64).  The groups' partial sums are combined with xor-shuffles
// and written once.  A row's non-zeros are read once per wave (64 / G of them in flight per
// step) and every B row segment is a coalesced G-wide read -- for K = 1 (SpMV) the whole wave
// strides over the non-zeros.  spmm_t: the same traversal of A's rows, scattering
// val * B[i, :] into C[col, :] with vector global atomics (no transpose of A is materialised).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_sp {

constexpr int WAVES = 4;

template <typename T, int G>
__global__ void __launch_bounds__(WAVES * 64) spmm_kernel(const int64_t* __restrict__ crow,
                                                          const int64_t* __restrict__ col,
                                                          const T* __restrict__ val, const T* __restrict__ B,
                                                          int64_t ldb, T* __restrict__ C, int64_t ldc, int64_t m,
                                                          int K) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NG = 64 / G;
  const int g = lane / G, gl = lane & (G - 1);
  for (int64_t i = (int64_t)blockIdx.x * WAVES + w; i < m; i += (int64_t)gridDim.x * WAVES) {
    const int64_t b = crow[i], e = crow[i + 1];
    for (int k0 = 0; k0 < K; k0 += G) {
      const int k = k0 + gl;
      T acc = T(0);
      if (k < K) {
        for (int64_t p = b + g; p < e; p += NG) acc += val[p] * B[col[p] * ldb + k];
      }
#pragma unroll
      for (int o = G; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);
      if (g == 0 && k < K) C[i * ldc + k] = acc;
    }
  }
}

template <typename T, int G>
__global__ void __launch_bounds__(WAVES * 64) spmm_t_kernel(const int64_t* __restrict__ crow,
                                                            const int64_t* __restrict__ col,
                                                            const T* __restrict__ val, const T* __restrict__ B,
                                                            int64_t ldb, T* __restrict__ C, int64_t ldc, int64_t m,
                                                            int K) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NG = 64 / G;
  const int g = lane / G, gl = lane & (G - 1);
  for (int64_t i = (int64_t)blockIdx.x * WAVES + w; i < m; i += (int64_t)gridDim.x * WAVES) {
    const int64_t b = crow[i], e = crow[i + 1];
    if (b == e) continue;
    for (int k0 = 0; k0 < K; k0 += G) {
      const int k = k0 + gl;
      if (k >= K) continue;
      const T bik = B[i * ldb + k];
      for (int64_t p = b + g; p < e; p += NG) atomicAdd(C + col[p] * ldc + k, val[p] * bik);
    }
  }
}

template <typename T>
int launch(int trans, const int64_t* crow, const int64_t* col, const T* val, const T* B, int64_t ldb, T* C,
           int64_t ldc, int64_t m, int K, hipStream_t s) {
  int64_t blocks = (m + WAVES - 1) / WAVES;
  if (blocks > 256 * 64) blocks = 256 * 64;
  const dim3 g((unsigned)(blocks < 1 ? 1 : blocks)), t(WAVES * 64);
#define SP_CASE(G_)                                                                                           \
  do {                                                                                                        \
    if (trans) hipLaunchKernelGGL((spmm_t_kernel<T, G_>), g, t, 0, s, crow, col, val, B, ldb, C, ldc, m, K); \
    else hipLaunchKernelGGL((spmm_kernel<T, G_>), g, t, 0, s, crow, col, val, B, ldb, C, ldc, m, K);         \
  } while (0)
  if (K <= 1) SP_CASE(1);
  else if (K <= 2) SP_CASE(2);
  else if (K <= 4) SP_CASE(4);
  else if (K <= 8) SP_CASE(8);
  else if (K <= 16) SP_CASE(16);
  else if (K <= 32) SP_CASE(32);
  else SP_CASE(64);
#undef SP_CASE
  return (int)hipGetLastError();
}

}  // namespace sysml_sp

extern "C" {

// dtype 1 fp32, 2 fp64.  trans = 0: C (m x K) = A B;  trans = 1: C (n x K) += t(A) B (C zeroed by
// the caller).  Returns 0, -1 (unsupported) or a hipError_t.
int sysml_spmm(int dtype, int trans, const void* crow, const void* col, const void* val, const void* B, int64_t ldb,
               void* C, int64_t ldc, int64_t m, int K, void* stream) {
  using namespace sysml_sp;
  if (m <= 0 || K <= 0) return m == 0 ? 0 : -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const auto* cr = static_cast<const int64_t*>(crow);
  const auto* cl = static_cast<const int64_t*>(col);
  if (dtype == 1)
    return launch<float>(trans, cr, cl, (const float*)val, (const float*)B, ldb, (float*)C, ldc, m, K, s);
  if (dtype == 2)
    return launch<double>(trans, cr, cl, (const double*)val, (const double*)B, ldb, (double*)C, ldc, m, K, s);
  return -1;
}

}  // extern "C"
