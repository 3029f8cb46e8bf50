// Column-wise cumulative aggregates of DML (cumsum, cumprod, cummin, cummax: each column of an
// N x D matrix scanned down its rows; reference: the cumulative_scan kernels of SystemML.cu and
// LibMatrixAgg.cumaggregate).
//
// Three phases over row chunks, so that a tall matrix keeps the whole chip busy:
//   A  every workgroup reduces its chunk of rows (per column) to one value      -> tot[chunk][col]
//   B  per column, an exclusive scan of the chunk totals
//   C  every workgroup rescans its chunk from that offset and writes the result
// Two thread mappings:
//   wide   (D >= 64): a 64-column strip per workgroup, lane = column (each row read by the wave is
//          one contiguous 256-B segment for fp32), the 4 waves take consecutive quarters of the
//          chunk's rows and combine their partial results through LDS;
//   narrow (D <  64): one column per workgroup row range, 8 consecutive elements per thread, a
//          wave-level inclusive scan by __shfl_up and a block level through LDS.
// Phase B runs one workgroup per column over the chunk totals with the same block scan.
// min / max propagate NaN like torch.cummin / cummax; sums accumulate in the element type.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_scan {

enum { SUM = 0, PROD = 1, MIN = 2, MAX = 3 };

template <typename T, int OP>
__device__ __forceinline__ T ident() {
  if (OP == SUM) return T(0);
  if (OP == PROD) return T(1);
  if (OP == MIN) return (T)__builtin_inf();
  return -(T)__builtin_inf();
}

template <typename T, int OP>
__device__ __forceinline__ T comb(T a, T b) {
  if (OP == SUM) return a + b;
  if (OP == PROD) return a * b;
  if (a != a || b != b) return (T)__builtin_nan("");
  if (OP == MIN) return b < a ? b : a;
  return b > a ? b : a;
}

constexpr int NT = 256;
constexpr int UNR = 8;

// ---- wide mapping ---------------------------------------------------------------------------
// grid (nchunk, ceil(D / 64)); chunk = `rows` rows; PHASE 0: totals, 1: rescan with offsets
template <typename T, int OP, int PHASE>
__global__ void __launch_bounds__(NT) wide_kernel(const T* __restrict__ X, T* __restrict__ Y, T* __restrict__ tot,
                                                  int64_t N, int D, int64_t rows) {
  __shared__ T part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.y * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.x * rows;
  const int64_t r1 = min(N, r0 + rows);
  const int64_t q = (rows + 3) / 4;
  const int64_t w0 = min(r1, r0 + q * wave), w1 = min(r1, w0 + q);
  const bool live = col < D;
  T acc = ident<T, OP>();
  if (live) {
    // UNR independent row loads in flight per lane before they are combined in order
    int64_t r = w0;
    for (; r + UNR <= w1; r += UNR) {
      T v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = X[(r + u) * D + col];
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc = comb<T, OP>(acc, v[u]);
    }
    for (; r < w1; ++r) acc = comb<T, OP>(acc, X[r * D + col]);
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (PHASE == 0) {
    if (wave == 0 && live) {
      T t = part[0][lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) t = comb<T, OP>(t, part[w][lane]);
      tot[(int64_t)blockIdx.x * D + col] = t;
    }
    return;
  }
  if (!live) return;
  T run = tot[(int64_t)blockIdx.x * D + col];          // exclusive offset of this chunk (phase B)
  for (int w = 0; w < wave; ++w) run = comb<T, OP>(run, part[w][lane]);
  int64_t r = w0;
  for (; r + UNR <= w1; r += UNR) {
    T v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = X[(r + u) * D + col];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      run = comb<T, OP>(run, v[u]);
      Y[(r + u) * D + col] = run;
    }
  }
  for (; r < w1; ++r) {
    run = comb<T, OP>(run, X[r * D + col]);
    Y[r * D + col] = run;
  }
}

// ---- block scan of E consecutive values per thread (narrow mapping and phase B) ------------
constexpr int E = 8;            // values per thread: NT * E = 2048 rows per narrow chunk

template <typename T, int OP>
__device__ __forceinline__ T wave_incl_scan(T v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T u = __shfl_up(v, off, 64);
    if (lane >= off) v = comb<T, OP>(u, v);
  }
  return v;
}

// v[] -> inclusive prefixes within the thread; returns the exclusive prefix of this thread inside
// the workgroup and sets *total to the workgroup's total.  wsum: 4 LDS slots.
template <typename T, int OP>
__device__ __forceinline__ T block_scan(T (&v)[E], T* wsum, T* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 1; i < E; ++i) v[i] = comb<T, OP>(v[i - 1], v[i]);
  const T incl = wave_incl_scan<T, OP>(v[E - 1], lane);
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  T pre = ident<T, OP>();
  for (int w = 0; w < wave; ++w) pre = comb<T, OP>(pre, wsum[w]);
  const T excl = __shfl_up(incl, 1, 64);
  if (lane > 0) pre = comb<T, OP>(pre, excl);
  T t = wsum[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) t = comb<T, OP>(t, wsum[w]);
  *total = t;
  return pre;
}

// ---- narrow mapping -------------------------------------------------------------------------
// grid (nchunk, D); chunk = NT * E rows of one column
// VEC (a single 16-B aligned column): the thread's E consecutive values move as 16-B vectors
template <typename T>
using vec16 = T __attribute__((ext_vector_type(16 / sizeof(T))));

template <typename T, int OP, int PHASE, bool VEC>
__global__ void __launch_bounds__(NT) narrow_kernel(const T* __restrict__ X, T* __restrict__ Y, T* __restrict__ tot,
                                                    int64_t N, int D) {
  constexpr int W = 16 / sizeof(T);
  __shared__ T wsum[4];
  const int col = blockIdx.y;
  const int64_t base = (int64_t)blockIdx.x * (NT * E) + threadIdx.x * E;
  const bool full = VEC && base + E <= N;
  T v[E];
  if (full) {
    const vec16<T>* p = reinterpret_cast<const vec16<T>*>(X + base);
#pragma unroll
    for (int j = 0; j < E / W; ++j) {
      const vec16<T> q = p[j];
#pragma unroll
      for (int k = 0; k < W; ++k) v[j * W + k] = q[k];
    }
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = (base + i < N) ? X[(base + i) * D + col] : ident<T, OP>();
  }
  T total;
  T pre = block_scan<T, OP>(v, wsum, &total);
  if (PHASE == 0) {
    if (threadIdx.x == 0) tot[(int64_t)blockIdx.x * D + col] = total;
    return;
  }
  pre = comb<T, OP>(tot[(int64_t)blockIdx.x * D + col], pre);   // chunk offset (phase B)
  if (full) {
    vec16<T>* p = reinterpret_cast<vec16<T>*>(Y + base);
#pragma unroll
    for (int j = 0; j < E / W; ++j) {
      vec16<T> q;
#pragma unroll
      for (int k = 0; k < W; ++k) q[k] = comb<T, OP>(pre, v[j * W + k]);
      p[j] = q;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (base + i < N) Y[(base + i) * D + col] = comb<T, OP>(pre, v[i]);
}

// ---- phase B: exclusive scan of the chunk totals, one workgroup per column -----------------
template <typename T, int OP>
__global__ void __launch_bounds__(NT) offsets_kernel(T* __restrict__ tot, int64_t nchunk, int D) {
  __shared__ T wsum[2][4];
  const int col = blockIdx.x;
  T carry = ident<T, OP>();
  int it = 0;
  for (int64_t b0 = 0; b0 < nchunk; b0 += NT * E, ++it) {
    const int64_t base = b0 + threadIdx.x * E;
    T v[E];
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = (base + i < nchunk) ? tot[(base + i) * D + col] : ident<T, OP>();
    T total;
    const T pre = comb<T, OP>(carry, block_scan<T, OP>(v, wsum[it & 1], &total));
#pragma unroll
    for (int i = 0; i < E; ++i)     // exclusive: the prefix before element i
      if (base + i < nchunk) tot[(base + i) * D + col] = i == 0 ? pre : comb<T, OP>(pre, v[i - 1]);
    carry = comb<T, OP>(carry, total);
  }
}

template <typename T, int OP>
int launch(const T* X, T* Y, T* tot, int64_t N, int D, int64_t nchunk, int64_t rows, hipStream_t s) {
  if (D >= 64) {
    const dim3 g((unsigned)nchunk, (unsigned)((D + 63) / 64));
    hipLaunchKernelGGL((wide_kernel<T, OP, 0>), g, dim3(NT), 0, s, X, Y, tot, N, D, rows);
    hipLaunchKernelGGL((offsets_kernel<T, OP>), dim3(D), dim3(NT), 0, s, tot, nchunk, D);
    hipLaunchKernelGGL((wide_kernel<T, OP, 1>), g, dim3(NT), 0, s, X, Y, tot, N, D, rows);
  } else {
    const dim3 g((unsigned)nchunk, (unsigned)D);
    const bool vec = D == 1 && ((uintptr_t)X % 16) == 0 && ((uintptr_t)Y % 16) == 0;
    if (vec)
      hipLaunchKernelGGL((narrow_kernel<T, OP, 0, true>), g, dim3(NT), 0, s, X, Y, tot, N, D);
    else
      hipLaunchKernelGGL((narrow_kernel<T, OP, 0, false>), g, dim3(NT), 0, s, X, Y, tot, N, D);
    hipLaunchKernelGGL((offsets_kernel<T, OP>), dim3(D), dim3(NT), 0, s, tot, nchunk, D);
    if (vec)
      hipLaunchKernelGGL((narrow_kernel<T, OP, 1, true>), g, dim3(NT), 0, s, X, Y, tot, N, D);
    else
      hipLaunchKernelGGL((narrow_kernel<T, OP, 1, false>), g, dim3(NT), 0, s, X, Y, tot, N, D);
  }
  return (int)hipGetLastError();
}

}  // namespace sysml_scan

extern "C" {

// Chunking the host sizes the workspace with: returns nchunk and sets *rows (rows per chunk).
int64_t sysml_cumagg_chunks(int64_t N, int D, int64_t* rows) {
  if (D >= 64) {
    // ~2048 workgroups in total over the column strips, >= 16 rows per wave
    const int64_t strips = (D + 63) / 64;
    int64_t want = 2048 / strips;
    if (want < 1) want = 1;
    int64_t r = (N + want - 1) / want;
    if (r < 64) r = 64;
    *rows = r;
    return (N + r - 1) / r;
  }
  *rows = sysml_scan::NT * sysml_scan::E;
  return (N + *rows - 1) / *rows;
}

// dtype 0 fp32, 1 fp64; op 0 sum, 1 prod, 2 min, 3 max.  X, Y: N x D row-major; tot: nchunk x D
// workspace.  Returns 0, -1 (unsupported) or a hipError_t.
int sysml_cumagg(int dtype, int op, const void* X, void* Y, void* tot, int64_t N, int D, int64_t nchunk,
                 int64_t rows, void* stream) {
  using namespace sysml_scan;
  if (N <= 0 || D <= 0 || nchunk <= 0 || nchunk >= (1LL << 31) || op < 0 || op > 3) return -1;
  if ((D + 63) / 64 > 65535) return -1;   // grid.y of the wide mapping
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define CASE(T, OPV) return launch<T, OPV>((const T*)X, (T*)Y, (T*)tot, N, D, nchunk, rows, s)
  if (dtype == 0) {
    if (op == SUM) CASE(float, SUM);
    if (op == PROD) CASE(float, PROD);
    if (op == MIN) CASE(float, MIN);
    CASE(float, MAX);
  }
  if (dtype == 1) {
    if (op == SUM) CASE(double, SUM);
    if (op == PROD) CASE(double, PROD);
    if (op == MIN) CASE(double, MIN);
    CASE(double, MAX);
  }
#undef CASE
  return -1;
}

}  // extern "C"
