// CSR transpose plan by counting sort (reference: LibMatrixReorg.transpose of a sparse block --
// a column count pass, a prefix sum and a scatter pass), and a value gather by that plan.
//   col_count   cnt[c] = non-zeros in column c (int32 atomics), and the longest column
//   (prefix sum of cnt -> crowT, on the host side)
//   fill        one wave per row: each non-zero p = (r, c) claims a slot of column c's segment
//               (atomic cursor) and writes rowsT[slot] = r, perm[slot] = p
//   seg_sort    the claim order inside a segment is arbitrary, so each segment is sorted by row
//               (one wave per segment, bitonic sort in LDS, rows unique inside a column): the
//               result is the canonical transposed CSR -- the same arrays a stable key sort gives
//   gather      valsT[i] = vals[perm[i]]
// Segments longer than SEG_MAX are left to the caller (the launcher reports the longest one).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_ct {

constexpr int NT = 256;
constexpr int SEG_MAX = 1024;        // longest segment sorted in LDS (per wave)

template <typename I>
__global__ void __launch_bounds__(NT) col_count(const I* __restrict__ col, int64_t nnz, int* __restrict__ cnt,
                                                int* __restrict__ maxlen) {
  for (int64_t p = (int64_t)blockIdx.x * NT + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * NT) {
    const int v = atomicAdd(&cnt[(int64_t)col[p]], 1) + 1;
    if (v > SEG_MAX) atomicMax(maxlen, v);
  }
}

template <typename I>
__global__ void __launch_bounds__(NT) fill(const int64_t* __restrict__ crow, const I* __restrict__ col, int64_t m,
                                           const int64_t* __restrict__ crowT, int* __restrict__ cursor,
                                           int* __restrict__ rowsT, int64_t* __restrict__ perm) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6); r < m; r += (int64_t)gridDim.x * (NT / 64)) {
    const int64_t b = crow[r], e = crow[r + 1];
    for (int64_t p = b + lane; p < e; p += 64) {
      const int64_t c = (int64_t)col[p];
      const int64_t slot = crowT[c] + atomicAdd(&cursor[c], 1);
      rowsT[slot] = (int)r;
      perm[slot] = p;
    }
  }
}

// one wave per segment: bitonic sort of (row, perm) pairs by row in LDS
__global__ void __launch_bounds__(NT) seg_sort(const int64_t* __restrict__ crowT, int64_t n, int* __restrict__ rowsT,
                                               int64_t* __restrict__ perm) {
  __shared__ int kr[NT / 64][SEG_MAX];
  __shared__ int64_t kp[NT / 64][SEG_MAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t s = (int64_t)blockIdx.x * (NT / 64) + w; s < n; s += (int64_t)gridDim.x * (NT / 64)) {
    const int64_t b = crowT[s];
    const int L = (int)(crowT[s + 1] - b);
    if (L <= 1 || L > SEG_MAX) continue;
    // already sorted (common for short segments)?  one pass with a wave vote
    bool ok = true;
    for (int i = lane; i + 1 < L; i += 64) ok &= rowsT[b + i] < rowsT[b + i + 1];
    if (__all(ok)) continue;
    int P = 2;
    while (P < L) P <<= 1;
    for (int i = lane; i < P; i += 64) {
      kr[w][i] = i < L ? rowsT[b + i] : 0x7fffffff;
      kp[w][i] = i < L ? perm[b + i] : 0;
    }
    __builtin_amdgcn_wave_barrier();
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = lane; i < P; i += 64) {
          const int l = i ^ j;
          if (l > i) {
            const bool up = (i & k) == 0;
            const int a = kr[w][i], c = kr[w][l];
            if ((a > c) == up) {
              kr[w][i] = c;
              kr[w][l] = a;
              const int64_t t = kp[w][i];
              kp[w][i] = kp[w][l];
              kp[w][l] = t;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
    }
    for (int i = lane; i < L; i += 64) {
      rowsT[b + i] = kr[w][i];
      perm[b + i] = kp[w][i];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
}

template <typename T>
__global__ void __launch_bounds__(NT) gather(const T* __restrict__ v, const int64_t* __restrict__ perm,
                                             T* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) out[i] = v[perm[i]];
}

inline unsigned grid(int64_t work, int per) {
  int64_t g = (work + per - 1) / per;
  if (g > 16384) g = 16384;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace sysml_ct

extern "C" {

// pass 1: cnt (n ints, zeroed by the caller) = column counts of the pattern; maxlen (one int,
// zeroed): set to a count above the in-LDS sort limit when some column is longer than it.
int sysml_csrt_count(const void* col, int idx32, int64_t nnz, int* cnt, int* maxlen, void* stream) {
  using namespace sysml_ct;
  if (nnz <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (idx32) hipLaunchKernelGGL(col_count<int32_t>, dim3(grid(nnz, NT * 4)), dim3(NT), 0, st, (const int32_t*)col, nnz, cnt, maxlen);
  else hipLaunchKernelGGL(col_count<int64_t>, dim3(grid(nnz, NT * 4)), dim3(NT), 0, st, (const int64_t*)col, nnz, cnt, maxlen);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// pass 2: with crowT (n + 1, the exclusive prefix of the counts) and cursor (n ints, zeroed):
// rowsT / perm (nnz each) = the transposed pattern's column indices and the value permutation,
// sorted by row inside every segment.
int sysml_csrt_fill(const int64_t* crow, const void* col, int idx32, int64_t m, int64_t n, const int64_t* crowT,
                    int* cursor, int* rowsT, int64_t* perm, void* stream) {
  using namespace sysml_ct;
  if (m <= 0 || n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (idx32)
    hipLaunchKernelGGL(fill<int32_t>, dim3(grid(m, NT / 64)), dim3(NT), 0, st, crow, (const int32_t*)col, m, crowT,
                       cursor, rowsT, perm);
  else
    hipLaunchKernelGGL(fill<int64_t>, dim3(grid(m, NT / 64)), dim3(NT), 0, st, crow, (const int64_t*)col, m, crowT,
                       cursor, rowsT, perm);
  hipLaunchKernelGGL(seg_sort, dim3(grid(n, NT / 64)), dim3(NT), 0, st, crowT, n, rowsT, perm);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// out[i] = v[perm[i]], esize 2 / 4 / 8 bytes
int sysml_gather(int esize, const void* v, const int64_t* perm, void* out, int64_t n, void* stream) {
  using namespace sysml_ct;
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid(n, NT * 4)), t(NT);
  if (esize == 2) hipLaunchKernelGGL(gather<uint16_t>, g, t, 0, st, (const uint16_t*)v, perm, (uint16_t*)out, n);
  else if (esize == 4) hipLaunchKernelGGL(gather<uint32_t>, g, t, 0, st, (const uint32_t*)v, perm, (uint32_t*)out, n);
  else if (esize == 8) hipLaunchKernelGGL(gather<uint64_t>, g, t, 0, st, (const uint64_t*)v, perm, (uint64_t*)out, n);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
