// Sparse matrix-multiply family on CDNA4 (reference: LibMatrixMult.java
// matrixMultSparseDense :1105 / matrixMultSparseSparse :1397 / matrixMultTransposeSelfSparse
// :1839 and the cuSPARSE csrmm / csrgemm calls of LibMatrixCuMatMult.java:173).
//
//   spmm_bal  C = A B, A CSR (int32 or int64 column indices), B dense row-major: nnz-balanced.
//             The non-zeros are cut into equal chunks, one per wavefront; a wave finds its first
//             row by binary search over the row pointers and walks the rows overlapping its chunk.
//             A row that lies entirely in the chunk is written with a plain store, the (at most
//             two) rows cut by the chunk borders are added atomically -- so a skewed row (a
//             power-law user with 10^5 ratings) is shared by as many waves as it has chunks
//             instead of serialising one wave.  Lanes: G per output column group (G = next
//             power of two >= K, <= 64), 64 / G non-zeros in flight per step; B rows are
//             coalesced G-wide reads.  C is zeroed by the caller.
//   spgemm    C = A B, both CSR, Gustavson row by row with one workgroup per row of A and a
//             dense accumulator in LDS (n <= 32768 fp32 columns, 128 KiB of the 160 KiB):
//             pass 1 counts the distinct columns of each output row through an LDS bitmap;
//             the host scans the counts into C's row pointers; pass 2 accumulates
//             a_ik * b_kj with LDS float atomics and compacts the bitmap in column order, so C
//             comes out canonical (sorted columns, no duplicates).
//   tsmm_sp   C = t(X) X for CSR X (N x D, D <= 8192): one wave per row, every pair (p <= q)
//             of the row's non-zeros adds x_p x_q to C[col_p, col_q] (global float atomics on
//             the upper triangle), then the lower triangle is mirrored.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_sg {

constexpr int WAVES = 4;

template <typename I>
__device__ __forceinline__ int64_t first_row(const int64_t* __restrict__ crow, int64_t m, int64_t p) {
  // largest r with crow[r] <= p (rows with crow[r] == crow[r+1] are skipped by the caller's loop)
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (crow[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <typename T, typename I, int G>
__global__ void __launch_bounds__(WAVES * 64) spmm_bal_kernel(const int64_t* __restrict__ crow,
                                                              const I* __restrict__ col, const T* __restrict__ val,
                                                              const T* __restrict__ B, int64_t ldb,
                                                              T* __restrict__ C, int64_t ldc, int64_t m, int K,
                                                              int64_t chunk, int64_t nchunks) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NG = 64 / G;
  const int g = lane / G, gl = lane & (G - 1);
  const int64_t nnz = crow[m];
  for (int64_t c = (int64_t)blockIdx.x * WAVES + w; c < nchunks; c += (int64_t)gridDim.x * WAVES) {
    const int64_t s = c * chunk;
    const int64_t e = s + chunk < nnz ? s + chunk : nnz;
    if (s >= e) continue;
    int64_t r = first_row<I>(crow, m, s);
    while (r < m) {
      const int64_t rb = crow[r], re = crow[r + 1];
      if (rb >= e) break;
      const int64_t b = rb > s ? rb : s;
      const int64_t q = re < e ? re : e;
      if (b < q) {
        const bool whole = (rb >= s) && (re <= e);
        for (int k0 = 0; k0 < K; k0 += G) {
          const int k = k0 + gl;
          T acc = T(0);
          if (k < K) {
            // 4 non-zeros per group in flight: their indices and values first, then the 4
            // dependent B-row gathers (random rows: latency-bound without the batching)
            for (int64_t p0 = b + g; p0 < q; p0 += 4 * NG) {
              int64_t c[4];
              T v[4], bv[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int64_t p = p0 + u * NG;
                const bool in = p < q;
                c[u] = in ? (int64_t)col[p] : 0;
                v[u] = in ? val[p] : T(0);
              }
#pragma unroll
              for (int u = 0; u < 4; ++u) bv[u] = B[c[u] * ldb + k];
#pragma unroll
              for (int u = 0; u < 4; ++u) acc += v[u] * bv[u];
            }
          }
#pragma unroll
          for (int o = G; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);
          if (g == 0 && k < K) {
            if (whole) C[r * ldc + k] = acc;
            else atomicAdd(C + r * ldc + k, acc);
          }
        }
      }
      ++r;
    }
  }
}

template <typename T, typename I>
int launch_bal(const int64_t* crow, const I* col, const T* val, const T* B, int64_t ldb, T* C, int64_t ldc, int64_t m,
               int K, int64_t nnz, hipStream_t st) {
  // ~ 4 chunks per wave slot of the chip; at least 32 non-zeros per chunk
  int64_t chunk = (nnz + 256 * 16 - 1) / (256 * 16);
  if (chunk < 32) chunk = 32;
  const int64_t nchunks = (nnz + chunk - 1) / chunk;
  int64_t blocks = (nchunks + WAVES - 1) / WAVES;
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  const dim3 gr((unsigned)blocks), t(WAVES * 64);
#define SB_CASE(G_) hipLaunchKernelGGL((spmm_bal_kernel<T, I, G_>), gr, t, 0, st, crow, col, val, B, ldb, C, ldc, m, K, \
                                       chunk, nchunks)
  if (K <= 1) SB_CASE(1);
  else if (K <= 2) SB_CASE(2);
  else if (K <= 4) SB_CASE(4);
  else if (K <= 8) SB_CASE(8);
  else if (K <= 16) SB_CASE(16);
  else if (K <= 32) SB_CASE(32);
  else SB_CASE(64);
#undef SB_CASE
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------- SpGEMM
constexpr int SG_T = 256;
constexpr int SG_MAXN = 32768;

template <typename IA, typename IB>
__global__ void __launch_bounds__(SG_T) spgemm_count_kernel(const int64_t* __restrict__ acrow,
                                                            const IA* __restrict__ acol,
                                                            const int64_t* __restrict__ bcrow,
                                                            const IB* __restrict__ bcol, int64_t m, int n,
                                                            int64_t* __restrict__ cnt) {
  __shared__ unsigned bits[SG_MAXN / 32];
  __shared__ unsigned tot;
  const int nw = (n + 31) >> 5;
  for (int64_t i = blockIdx.x; i < m; i += gridDim.x) {
    for (int x = threadIdx.x; x < nw; x += SG_T) bits[x] = 0u;
    if (threadIdx.x == 0) tot = 0u;
    __syncthreads();
    const int64_t ab = acrow[i], ae = acrow[i + 1];
    for (int64_t p = ab; p < ae; ++p) {
      const int64_t k = acol[p];
      const int64_t bb = bcrow[k], be = bcrow[k + 1];
      for (int64_t q = bb + threadIdx.x; q < be; q += SG_T) {
        const unsigned j = (unsigned)bcol[q];
        atomicOr(&bits[j >> 5], 1u << (j & 31));
      }
    }
    __syncthreads();
    unsigned c = 0;
    for (int x = threadIdx.x; x < nw; x += SG_T) c += __popc(bits[x]);
    atomicAdd(&tot, c);
    __syncthreads();
    if (threadIdx.x == 0) cnt[i] = tot;
    __syncthreads();
  }
}

template <typename IA, typename IB>
__global__ void __launch_bounds__(SG_T) spgemm_fill_kernel(const int64_t* __restrict__ acrow,
                                                           const IA* __restrict__ acol,
                                                           const float* __restrict__ aval,
                                                           const int64_t* __restrict__ bcrow,
                                                           const IB* __restrict__ bcol,
                                                           const float* __restrict__ bval, int64_t m, int n,
                                                           const int64_t* __restrict__ ccrow,
                                                           int64_t* __restrict__ ccol, float* __restrict__ cval,
                                                           int64_t* __restrict__ fcnt) {
  extern __shared__ float acc[];                      // n floats, then the bitmap
  unsigned* bits = reinterpret_cast<unsigned*>(acc + n);
  const int nw = (n + 31) >> 5;
  const int lane = threadIdx.x & 63;
  for (int64_t i = blockIdx.x; i < m; i += gridDim.x) {
    const int64_t ab = acrow[i], ae = acrow[i + 1];
    for (int x = threadIdx.x; x < n; x += SG_T) acc[x] = 0.0f;
    for (int x = threadIdx.x; x < nw; x += SG_T) bits[x] = 0u;
    __syncthreads();
    for (int64_t p = ab; p < ae; ++p) {
      const int64_t k = acol[p];
      const float a = aval[p];
      const int64_t bb = bcrow[k], be = bcrow[k + 1];
      for (int64_t q = bb + threadIdx.x; q < be; q += SG_T) {
        const unsigned j = (unsigned)bcol[q];
        atomicAdd(&acc[j], a * bval[q]);
        atomicOr(&bits[j >> 5], 1u << (j & 31));
      }
    }
    __syncthreads();
    // ordered compaction by the first wave: 64 bitmap words per step, a wave-wide exclusive
    // scan of their popcounts places each lane's columns
    if (threadIdx.x < 64) {
      int64_t o = ccrow[i];
      for (int base = 0; base < nw; base += 64) {
        const int x = base + lane;
        unsigned bw = x < nw ? bits[x] : 0u;
        const int c = __popc(bw);
        int incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int v = __shfl_up(incl, d, 64);
          if (lane >= d) incl += v;
        }
        int64_t w = o + (incl - c);
        while (bw) {
          const int bit = __ffs(bw) - 1;
          bw &= bw - 1;
          const int j = (x << 5) + bit;
          ccol[w] = j;
          cval[w] = acc[j];
          ++w;
        }
        o += __shfl(incl, 63, 64);
      }
      if (lane == 0) fcnt[i] = o - ccrow[i];
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------- sparse tsmm
template <typename T, typename I>
__global__ void __launch_bounds__(WAVES * 64) tsmm_sp_kernel(const int64_t* __restrict__ crow,
                                                             const I* __restrict__ col, const T* __restrict__ val,
                                                             int64_t m, T* __restrict__ C, int64_t D) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t i = (int64_t)blockIdx.x * WAVES + w; i < m; i += (int64_t)gridDim.x * WAVES) {
    const int64_t b = crow[i], e = crow[i + 1];
    const int64_t z = e - b;
    const int64_t npairs = z * (z + 1) / 2;
    for (int64_t t = lane; t < npairs; t += 64) {
      // pair t -> (p, q), p <= q, row-major over the upper triangle of the z x z outer product
      int64_t p = (int64_t)((2.0 * z + 1.0 - sqrt((2.0 * z + 1.0) * (2.0 * z + 1.0) - 8.0 * (double)t)) * 0.5);
      if (p < 0) p = 0;
      while (p > 0 && p * (2 * z - p + 1) / 2 > t) --p;
      while ((p + 1) * (2 * z - p) / 2 <= t) ++p;
      const int64_t q = p + (t - p * (2 * z - p + 1) / 2);
      const int64_t cp = col[b + p], cq = col[b + q];
      const T v = val[b + p] * val[b + q];
      const int64_t r0 = cp < cq ? cp : cq, c0 = cp < cq ? cq : cp;
      atomicAdd(C + r0 * D + c0, v);
    }
  }
}

template <typename T>
__global__ void mirror_kernel(T* __restrict__ C, int64_t D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= D * D) return;
  const int64_t r = idx / D, c = idx - r * D;
  if (r > c) C[idx] = C[c * D + r];
}

}  // namespace sysml_sg

extern "C" {

// C (m x K) += A B over A's non-zeros (C zeroed by the caller).  dtype 1 fp32 / 2 fp64,
// idx32: A's column indices are int32.  Returns 0 or a hipError_t (-1: unsupported).
int sysml_spmm_bal(int dtype, int idx32, const void* crow, const void* col, const void* val, const void* B,
                   int64_t ldb, void* C, int64_t ldc, int64_t m, int K, int64_t nnz, void* stream) {
  using namespace sysml_sg;
  if (m <= 0 || K <= 0 || nnz <= 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const auto* cr = static_cast<const int64_t*>(crow);
  if (dtype == 1) {
    if (idx32) return launch_bal<float, int32_t>(cr, (const int32_t*)col, (const float*)val, (const float*)B, ldb,
                                                 (float*)C, ldc, m, K, nnz, s);
    return launch_bal<float, int64_t>(cr, (const int64_t*)col, (const float*)val, (const float*)B, ldb, (float*)C,
                                      ldc, m, K, nnz, s);
  }
  if (dtype == 2) {
    if (idx32) return launch_bal<double, int32_t>(cr, (const int32_t*)col, (const double*)val, (const double*)B,
                                                  ldb, (double*)C, ldc, m, K, nnz, s);
    return launch_bal<double, int64_t>(cr, (const int64_t*)col, (const double*)val, (const double*)B, ldb,
                                       (double*)C, ldc, m, K, nnz, s);
  }
  return -1;
}

// pass 1 of C = A B (A: m x k CSR, B: k x n CSR, n <= 32768): cnt[i] = nnz of C's row i.
// ia32 / ib32: int32 column indices.
int sysml_spgemm_count(int ia32, int ib32, const void* acrow, const void* acol, const void* bcrow, const void* bcol,
                       int64_t m, int n, void* cnt, void* stream) {
  using namespace sysml_sg;
  if (n > SG_MAXN || n <= 0) return -1;
  if (m <= 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned blocks = (unsigned)(m < 256 * 32 ? m : 256 * 32);
  const auto* ac = static_cast<const int64_t*>(acrow);
  const auto* bc = static_cast<const int64_t*>(bcrow);
  auto* ct = static_cast<int64_t*>(cnt);
#define SGC(IA, IB) hipLaunchKernelGGL((spgemm_count_kernel<IA, IB>), dim3(blocks), dim3(SG_T), 0, s, ac, \
                                       (const IA*)acol, bc, (const IB*)bcol, m, n, ct)
  if (ia32 && ib32) SGC(int32_t, int32_t);
  else if (ia32) SGC(int32_t, int64_t);
  else if (ib32) SGC(int64_t, int32_t);
  else SGC(int64_t, int64_t);
#undef SGC
  return (int)hipGetLastError();
}

// pass 2 (fp32 values): C's columns (int64, sorted per row) and values at ccrow's offsets;
// fcnt[i] receives the entries written for row i (checked against pass 1 by the caller).
int sysml_spgemm_fill(int ia32, int ib32, const void* acrow, const void* acol, const void* aval, const void* bcrow,
                      const void* bcol, const void* bval, int64_t m, int n, const void* ccrow, void* ccol, void* cval,
                      void* fcnt, void* stream) {
  using namespace sysml_sg;
  if (n > SG_MAXN || n <= 0) return -1;
  if (m <= 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned blocks = (unsigned)(m < 256 * 16 ? m : 256 * 16);
  const size_t lds = (size_t)n * sizeof(float) + (size_t)((n + 31) / 32) * sizeof(unsigned);
  const auto* ac = static_cast<const int64_t*>(acrow);
  const auto* bc = static_cast<const int64_t*>(bcrow);
#define SGF(IA, IB)                                                                                        \
  (void)hipFuncSetAttribute((const void*)spgemm_fill_kernel<IA, IB>,                                       \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                         \
  hipLaunchKernelGGL((spgemm_fill_kernel<IA, IB>), dim3(blocks), dim3(SG_T), lds, s, ac, (const IA*)acol, \
                     (const float*)aval, bc, (const IB*)bcol, (const float*)bval, m, n,                    \
                     (const int64_t*)ccrow, (int64_t*)ccol, (float*)cval, (int64_t*)fcnt)
  if (ia32 && ib32) { SGF(int32_t, int32_t); }
  else if (ia32) { SGF(int32_t, int64_t); }
  else if (ib32) { SGF(int64_t, int32_t); }
  else { SGF(int64_t, int64_t); }
#undef SGF
  return (int)hipGetLastError();
}

// C (D x D, zeroed by the caller) = t(X) X for CSR X (m x D).
int sysml_tsmm_sparse(int dtype, int idx32, const void* crow, const void* col, const void* val, int64_t m, void* C,
                      int64_t D, void* stream) {
  using namespace sysml_sg;
  if (m <= 0 || D <= 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int64_t blocks = (m + WAVES - 1) / WAVES;
  if (blocks > 256 * 32) blocks = 256 * 32;
  const dim3 g((unsigned)blocks), t(WAVES * 64);
  const auto* cr = static_cast<const int64_t*>(crow);
  const unsigned mb = (unsigned)((D * D + 255) / 256);
  if (dtype == 1) {
    if (idx32) hipLaunchKernelGGL((tsmm_sp_kernel<float, int32_t>), g, t, 0, s, cr, (const int32_t*)col,
                                  (const float*)val, m, (float*)C, D);
    else hipLaunchKernelGGL((tsmm_sp_kernel<float, int64_t>), g, t, 0, s, cr, (const int64_t*)col,
                            (const float*)val, m, (float*)C, D);
    hipLaunchKernelGGL((mirror_kernel<float>), dim3(mb), dim3(256), 0, s, (float*)C, D);
  } else if (dtype == 2) {
    if (idx32) hipLaunchKernelGGL((tsmm_sp_kernel<double, int32_t>), g, t, 0, s, cr, (const int32_t*)col,
                                  (const double*)val, m, (double*)C, D);
    else hipLaunchKernelGGL((tsmm_sp_kernel<double, int64_t>), g, t, 0, s, cr, (const int64_t*)col,
                            (const double*)val, m, (double*)C, D);
    hipLaunchKernelGGL((mirror_kernel<double>), dim3(mb), dim3(256), 0, s, (double*)C, D);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
