// Unary aggregates of DML over device matrices: sum, sumsq, mean, min, max, prod, var, sd over
// all cells, rows or columns, and rowIndexMax / rowIndexMin (reference: LibMatrixAgg.java
// aggregateUnaryMatrix and the reduce_{row,col}_{sum,max,min,mean} / reduce_prod kernels of
// SystemML.cu:1283-1528; the CP semantics -- fp64 accumulation, NaN propagation of min / max,
// the numerically stable variance of the CM object -- are kept).
//
// Operands are read in their storage type (bf16, fp32, fp64) and accumulated in fp64:
//   * variance: per-thread Welford (n, mean, M2) merged by Chan's pairwise update, so one pass
//     suffices and there is no sum-of-squares cancellation;
//   * rows: one wave64 per row (each lane a run of 4 consecutive cells, 256 cells per wave step),
//     rows < 16 wide one thread per row;
//   * columns: a workgroup owns a strip of columns (lane -> column, several rows per wave for
//     narrow matrices) over one chunk of rows; chunks of a tall matrix write partial states,
//     merged by a second pass -- the whole chip reduces even a 10M x 1 column;
//   * all cells: grid-stride partial states per workgroup, merged by a one-workgroup pass.
// Index aggregates return the 1-based column of the LAST extreme value (LibMatrixAgg).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sysml_ag {

enum { SUM = 0, SUMSQ = 1, MEAN = 2, MIN = 3, MAX = 4, PROD = 5, VAR = 6, SD = 7, IMAX = 8, IMIN = 9 };

struct St {
  double a, b, c;    // sum | sumsq | mean: a = sum; min/max: a; prod: a; var: a = n, b = mean, c = M2;
};                   // imax / imin: a = value, b = index

template <int OP>
__device__ __forceinline__ St st_init() {
  if (OP == MIN) return St{__builtin_inf(), 0, 0};
  if (OP == MAX) return St{-__builtin_inf(), 0, 0};
  if (OP == PROD) return St{1.0, 0, 0};
  if (OP == IMAX) return St{-__builtin_inf(), 0, 0};
  if (OP == IMIN) return St{__builtin_inf(), 0, 0};
  return St{0, 0, 0};
}

template <int OP>
__device__ __forceinline__ void st_add(St& s, double x, int64_t idx) {
  if (OP == SUM || OP == MEAN) s.a += x;
  else if (OP == SUMSQ) s.a += x * x;
  else if (OP == PROD) s.a *= x;
  else if (OP == MIN) s.a = (x != x || s.a != s.a) ? __builtin_nan("") : (x < s.a ? x : s.a);
  else if (OP == MAX) s.a = (x != x || s.a != s.a) ? __builtin_nan("") : (x > s.a ? x : s.a);
  else if (OP == IMAX) { if (x >= s.a) { s.a = x; s.b = (double)idx; } }
  else if (OP == IMIN) { if (x <= s.a) { s.a = x; s.b = (double)idx; } }
  else {  // VAR / SD: Welford
    s.a += 1.0;
    const double d = x - s.b;
    s.b += d / s.a;
    s.c += d * (x - s.b);
  }
}

// merge o into s; for the index aggregates o covers LATER columns than s on ties
template <int OP>
__device__ __forceinline__ void st_merge(St& s, const St& o) {
  if (OP == SUM || OP == MEAN || OP == SUMSQ) s.a += o.a;
  else if (OP == PROD) s.a *= o.a;
  else if (OP == MIN) s.a = (o.a != o.a || s.a != s.a) ? __builtin_nan("") : (o.a < s.a ? o.a : s.a);
  else if (OP == MAX) s.a = (o.a != o.a || s.a != s.a) ? __builtin_nan("") : (o.a > s.a ? o.a : s.a);
  else if (OP == IMAX) { if (o.a > s.a || (o.a == s.a && o.b > s.b)) { s.a = o.a; s.b = o.b; } }
  else if (OP == IMIN) { if (o.a < s.a || (o.a == s.a && o.b > s.b)) { s.a = o.a; s.b = o.b; } }
  else {
    if (o.a == 0) return;
    if (s.a == 0) { s = o; return; }
    const double n = s.a + o.a, d = o.b - s.b;
    s.c += o.c + d * d * s.a * o.a / n;
    s.b += d * o.a / n;
    s.a = n;
  }
}

template <int OP>
__device__ __forceinline__ double st_result(const St& s, int64_t n) {
  if (OP == MEAN) return s.a / (double)n;
  if (OP == VAR) return s.a > 1 ? s.c / (s.a - 1.0) : 0.0;
  if (OP == SD) return s.a > 1 ? sqrt(s.c / (s.a - 1.0)) : 0.0;
  if (OP == IMAX || OP == IMIN) return s.b + 1.0;
  return s.a;
}

__device__ __forceinline__ double ld(const float* p, int64_t i) { return (double)p[i]; }
__device__ __forceinline__ double ld(const double* p, int64_t i) { return p[i]; }
__device__ __forceinline__ double ld(const uint16_t* p, int64_t i) {
  return (double)__uint_as_float(((uint32_t)p[i]) << 16);
}

template <int OP>
__device__ __forceinline__ St st_shfl(const St& s, int off) {
  return St{__shfl_xor(s.a, off, 64), __shfl_xor(s.b, off, 64), __shfl_xor(s.c, off, 64)};
}

template <int OP>
__device__ __forceinline__ St wave_reduce(St s, int lane) {
  // index aggregates: merge the higher-lane partner (later columns) into the lower one
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const St o = st_shfl<OP>(s, off);
    if (lane & off) {
      St t = o;
      st_merge<OP>(t, s);
      s = t;
    } else {
      st_merge<OP>(s, o);
    }
  }
  return s;
}

template <typename TO>
__device__ __forceinline__ void put(TO* y, int64_t i, double v) { y[i] = (TO)v; }

constexpr int NT = 256;

// ---- rows: one wave per row, lanes stride the columns (each lane a contiguous run of 4) ----
template <typename T, typename TO, int OP>
__global__ void __launch_bounds__(NT) row_wave(const T* __restrict__ X, TO* __restrict__ Y, int64_t N, int D) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < N; r += (int64_t)gridDim.x * 4) {
    const T* row = X + r * D;
    St s = st_init<OP>();
    // lane's cells: 4-cell runs at 4 * (lane + 64 k) .. +3 (ascending column order per lane)
    for (int j0 = lane * 4; j0 < D; j0 += 256) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (j0 + u < D) ? ld(row, j0 + u) : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j0 + u < D) st_add<OP>(s, v[u], j0 + u);
    }
    s = wave_reduce<OP>(s, lane);
    if (lane == 0) put(Y, r, st_result<OP>(s, D));
  }
}

// ---- narrow rows: one thread per row ---------------------------------------------------------
template <typename T, typename TO, int OP>
__global__ void __launch_bounds__(NT) row_thread(const T* __restrict__ X, TO* __restrict__ Y, int64_t N, int D) {
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < N; r += (int64_t)gridDim.x * NT) {
    St s = st_init<OP>();
    for (int j = 0; j < D; ++j) st_add<OP>(s, ld(X, r * D + j), j);
    put(Y, r, st_result<OP>(s, D));
  }
}

// ---- columns: grid (column strips, row chunks); lane -> column within a CW-wide strip, the
// 64 / CW lane groups and the 4 waves interleave rows; partial states per (chunk, column) ----
template <typename T, int OP, int CW>
__global__ void __launch_bounds__(NT) col_part(const T* __restrict__ X, St* __restrict__ part, int64_t N, int D,
                                               int64_t rows) {
  constexpr int RPW = 64 / CW;          // row phases per wave
  __shared__ St red[NT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * CW + (lane % CW);
  const int phase = wave * RPW + lane / CW;
  const int64_t r0 = (int64_t)blockIdx.y * rows, r1 = min(N, r0 + rows);
  St s = st_init<OP>();
  if (col < D) {
    int64_t r = r0 + phase;
    for (; r + 3 * 4 * RPW < r1; r += 4 * 4 * RPW) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld(X, (r + (int64_t)u * 4 * RPW) * D + col);
#pragma unroll
      for (int u = 0; u < 4; ++u) st_add<OP>(s, v[u], r + (int64_t)u * 4 * RPW);
    }
    for (; r < r1; r += 4 * RPW) st_add<OP>(s, ld(X, r * D + col), r);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < CW) {
    // merge the row phases of this column in row order (phase p covers rows p, p + 4 RPW, ...:
    // every phase's rows interleave, so only order-free merges are exact for the index
    // aggregates -- those are row-direction only)
    St t = red[threadIdx.x];
    for (int p = 1; p < 4 * RPW; ++p) {
      const int w = p / RPW, l = (p % RPW) * CW + threadIdx.x;
      st_merge<OP>(t, red[w * 64 + l]);
    }
    const int c = blockIdx.x * CW + threadIdx.x;
    if (c < D) part[(int64_t)blockIdx.y * D + c] = t;
  }
}

// ---- columns, 16-B loads (sum / sumsq / mean of bf16 or fp32 with D a multiple of 8 / 4): lane ->
// a run of VW consecutive columns (one 16-B load per row), the 4 waves interleave rows, so a wave
// reads 1 KiB of every row it visits; fp64 accumulation as in col_part ----
template <typename T, int OP>
__global__ void __launch_bounds__(NT) col_vec(const T* __restrict__ X, St* __restrict__ part, int64_t N, int D,
                                              int64_t rows) {
  constexpr int VW = 16 / sizeof(T);
  __shared__ double red[3][64][VW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x * 64 + lane;            // column group
  const int col = g * VW;
  const int64_t r0 = (int64_t)blockIdx.y * rows, r1 = min(N, r0 + rows);
  double acc[VW];
#pragma unroll
  for (int v = 0; v < VW; ++v) acc[v] = 0.0;
  if (col < D) {
    const T* p = X + col;
    int64_t r = r0 + wave;
    for (; r + 12 < r1; r += 16) {
      uint4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = *(const uint4*)(p + (r + 4 * u) * D);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
        for (int v = 0; v < VW; ++v) {
          double x;
          if constexpr (sizeof(T) == 2) x = (double)__uint_as_float(v & 1 ? (w[v >> 1] & 0xffff0000u) : (w[v >> 1] << 16));
          else x = (double)__uint_as_float(w[v]);
          acc[v] += OP == SUMSQ ? x * x : x;
        }
      }
    }
    for (; r < r1; r += 4) {
      const uint4 q = *(const uint4*)(p + r * D);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int v = 0; v < VW; ++v) {
        double x;
        if constexpr (sizeof(T) == 2) x = (double)__uint_as_float(v & 1 ? (w[v >> 1] & 0xffff0000u) : (w[v >> 1] << 16));
        else x = (double)__uint_as_float(w[v]);
        acc[v] += OP == SUMSQ ? x * x : x;
      }
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int v = 0; v < VW; ++v) red[wave - 1][lane][v] = acc[v];
  }
  __syncthreads();
  if (wave == 0 && col < D) {
#pragma unroll
    for (int v = 0; v < VW; ++v) {
      const double t = acc[v] + red[0][lane][v] + red[1][lane][v] + red[2][lane][v];
      part[(int64_t)blockIdx.y * D + col + v] = St{t, 0, 0};
    }
  }
}

template <typename TO, int OP>
__global__ void __launch_bounds__(NT) col_final(const St* __restrict__ part, TO* __restrict__ Y, int64_t N, int D,
                                                int nchunk) {
  for (int c = blockIdx.x * NT + threadIdx.x; c < D; c += gridDim.x * NT) {
    St s = part[c];
    for (int k = 1; k < nchunk; ++k) st_merge<OP>(s, part[(int64_t)k * D + c]);
    put(Y, c, st_result<OP>(s, N));
  }
}

// ---- all cells -----------------------------------------------------------------------------
template <typename T, int OP>
__global__ void __launch_bounds__(NT) all_part(const T* __restrict__ X, St* __restrict__ part, int64_t n) {
  __shared__ St red[NT / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  St s = st_init<OP>();
  const int64_t stride = (int64_t)gridDim.x * NT;
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(X, i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) st_add<OP>(s, v[u], 0);
  }
  for (; i < n; i += stride) st_add<OP>(s, ld(X, i), 0);
  s = wave_reduce<OP>(s, lane);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    St t = red[0];
    for (int w = 1; w < NT / 64; ++w) st_merge<OP>(t, red[w]);
    part[blockIdx.x] = t;
  }
}

template <int OP>
__global__ void __launch_bounds__(64) all_final(const St* __restrict__ part, double* __restrict__ y, int nb,
                                                int64_t n) {
  const int lane = threadIdx.x;
  St s = st_init<OP>();
  for (int k = lane; k < nb; k += 64) st_merge<OP>(s, part[k]);
  s = wave_reduce<OP>(s, lane);
  if (lane == 0) *y = st_result<OP>(s, n);
}

// ---- fold of row-block partials: y[j] = op_b part[b, j] (fp64 partials of a column aggregate) --
template <typename TO, int OP>
__global__ void __launch_bounds__(NT) fold_rows(const double* __restrict__ part, TO* __restrict__ y, int nb, int64_t n) {
  for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (int64_t)gridDim.x * NT) {
    double a = part[j];
    for (int b = 1; b < nb; ++b) {
      const double v = part[(int64_t)b * n + j];
      a = OP == MIN ? (v < a ? v : a) : (OP == MAX ? (v > a ? v : a) : a + v);
    }
    y[j] = (TO)a;
  }
}

// ---- dot product sum(a * b) (TernaryAggregate tak+*) -------------------------------------
template <typename T>
__global__ void __launch_bounds__(NT) dot_part(const T* __restrict__ A, const T* __restrict__ B, St* __restrict__ part,
                                               int64_t n) {
  __shared__ St red[NT / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  St s = st_init<SUM>();
  const int64_t stride = (int64_t)gridDim.x * NT;
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(A, i + u * stride) * ld(B, i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) s.a += v[u];
  }
  for (; i < n; i += stride) s.a += ld(A, i) * ld(B, i);
  s = wave_reduce<SUM>(s, lane);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    St t = red[0];
    for (int w = 1; w < NT / 64; ++w) st_merge<SUM>(t, red[w]);
    part[blockIdx.x] = t;
  }
}

inline int grid_for(int64_t work, int per) {
  int64_t g = (work + per - 1) / per;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

template <typename T, int OP>
inline bool vec_cols(const void* X, int D) {
  if constexpr ((OP == SUM || OP == SUMSQ || OP == MEAN) && (sizeof(T) == 2 || sizeof(T) == 4)) {
    constexpr int VW = 16 / sizeof(T);
    return D >= 64 && D % VW == 0 && ((uintptr_t)X & 15) == 0;
  }
  return false;
}

// row chunks of a column aggregate: enough workgroups for the chip (>= 1024) and >= 64 rows each
inline void col_chunks(int64_t N, int strips, int64_t& nch, int64_t& rows) {
  nch = (1024 + strips - 1) / strips;
  const int64_t maxch = (N + 63) / 64;
  if (nch > maxch) nch = maxch;
  if (nch < 1) nch = 1;
  rows = (N + nch - 1) / nch;
  nch = (N + rows - 1) / rows;
}

template <typename T, typename TO, int OP>
int run(int dir, const void* X, void* Y, void* scratch, int64_t N, int D, hipStream_t st) {
  if (dir == 0) {   // all
    const int64_t n = N * D;
    const int nb = grid_for(n, NT * 8) > 1024 ? 1024 : grid_for(n, NT * 8);
    hipLaunchKernelGGL((all_part<T, OP>), dim3(nb), dim3(NT), 0, st, (const T*)X, (St*)scratch, n);
    hipLaunchKernelGGL((all_final<OP>), dim3(1), dim3(64), 0, st, (const St*)scratch, (double*)Y, nb, n);
  } else if (dir == 1) {   // rows
    if (D < 16)
      hipLaunchKernelGGL((row_thread<T, TO, OP>), dim3(grid_for(N, NT)), dim3(NT), 0, st, (const T*)X, (TO*)Y, N, D);
    else
      hipLaunchKernelGGL((row_wave<T, TO, OP>), dim3(grid_for(N, 4)), dim3(NT), 0, st, (const T*)X, (TO*)Y, N, D);
  } else if (vec_cols<T, OP>(X, D)) {   // columns, 16-B loads
    constexpr int VW = 16 / sizeof(T);
    const int strips = (D / VW + 63) / 64;
    int64_t nch, rows;
    col_chunks(N, strips, nch, rows);
    hipLaunchKernelGGL((col_vec<T, OP>), dim3(strips, (unsigned)nch), dim3(NT), 0, st, (const T*)X, (St*)scratch, N, D,
                       rows);
    hipLaunchKernelGGL((col_final<TO, OP>), dim3(grid_for(D, NT)), dim3(NT), 0, st, (const St*)scratch, (TO*)Y, N, D,
                       (int)nch);
  } else {   // columns
    const int cw = D >= 64 ? 64 : (D > 16 ? 32 : (D > 4 ? 16 : 4));
    const int strips = (D + cw - 1) / cw;
    // chunks: enough workgroups for the chip (>= 1024) and >= 256 rows each
    int64_t nch = (1024 + strips - 1) / strips;
    const int64_t maxch = (N + 255) / 256;
    if (nch > maxch) nch = maxch;
    if (nch < 1) nch = 1;
    const int64_t rows = (N + nch - 1) / nch;
    nch = (N + rows - 1) / rows;
    const dim3 g(strips, (unsigned)nch);
    switch (cw) {
      case 64: hipLaunchKernelGGL((col_part<T, OP, 64>), g, dim3(NT), 0, st, (const T*)X, (St*)scratch, N, D, rows); break;
      case 32: hipLaunchKernelGGL((col_part<T, OP, 32>), g, dim3(NT), 0, st, (const T*)X, (St*)scratch, N, D, rows); break;
      case 16: hipLaunchKernelGGL((col_part<T, OP, 16>), g, dim3(NT), 0, st, (const T*)X, (St*)scratch, N, D, rows); break;
      default: hipLaunchKernelGGL((col_part<T, OP, 4>), g, dim3(NT), 0, st, (const T*)X, (St*)scratch, N, D, rows); break;
    }
    hipLaunchKernelGGL((col_final<TO, OP>), dim3(grid_for(D, NT)), dim3(NT), 0, st, (const St*)scratch, (TO*)Y, N, D,
                       (int)nch);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <typename T, typename TO>
int by_op(int op, int dir, const void* X, void* Y, void* scratch, int64_t N, int D, hipStream_t st) {
  switch (op) {
    case SUM: return run<T, TO, SUM>(dir, X, Y, scratch, N, D, st);
    case SUMSQ: return run<T, TO, SUMSQ>(dir, X, Y, scratch, N, D, st);
    case MEAN: return run<T, TO, MEAN>(dir, X, Y, scratch, N, D, st);
    case MIN: return run<T, TO, MIN>(dir, X, Y, scratch, N, D, st);
    case MAX: return run<T, TO, MAX>(dir, X, Y, scratch, N, D, st);
    case PROD: return run<T, TO, PROD>(dir, X, Y, scratch, N, D, st);
    case VAR: return run<T, TO, VAR>(dir, X, Y, scratch, N, D, st);
    case SD: return run<T, TO, SD>(dir, X, Y, scratch, N, D, st);
    case IMAX: return dir == 1 ? run<T, TO, IMAX>(dir, X, Y, scratch, N, D, st) : -1;
    case IMIN: return dir == 1 ? run<T, TO, IMIN>(dir, X, Y, scratch, N, D, st) : -1;
    default: return -1;
  }
}

}  // namespace sysml_ag

extern "C" {

// Scratch bytes the aggregate needs (partial states): all -> 1024 states, columns -> chunks x D.
int64_t sysml_agg_scratch(int dir, int64_t N, int D) {
  using namespace sysml_ag;
  if (dir == 0) return 1024 * (int64_t)sizeof(St);
  if (dir == 1) return 0;
  const int cw = D >= 64 ? 64 : (D > 16 ? 32 : (D > 4 ? 16 : 4));
  int strips = (D + cw - 1) / cw;
  const int vstrips = ((D + 7) / 8 + 63) / 64;    // col_vec with 8-wide bf16 runs: the fewest strips
  if (vstrips < strips) strips = vstrips;
  int64_t nch, rows;
  col_chunks(N, strips, nch, rows);
  return nch * (int64_t)D * (int64_t)sizeof(St);
}

// op: 0 sum 1 sumsq 2 mean 3 min 4 max 5 prod 6 var 7 sd 8 rowIndexMax 9 rowIndexMin;
// dir: 0 all (Y: one double), 1 rows (Y: N values), 2 columns (Y: D values);
// xdt: 0 bf16, 1 fp32, 2 fp64 (X row-major N x D, contiguous); ydt: 1 fp32, 2 fp64.
int sysml_agg(int op, int dir, int xdt, int ydt, const void* X, void* Y, void* scratch, int64_t N, int D,
              void* stream) {
  using namespace sysml_ag;
  hipStream_t st = (hipStream_t)stream;
  if (N <= 0 || D <= 0 || dir < 0 || dir > 2) return -1;
  if (xdt == 0) return ydt == 1 ? by_op<uint16_t, float>(op, dir, X, Y, scratch, N, D, st)
                                : by_op<uint16_t, double>(op, dir, X, Y, scratch, N, D, st);
  if (xdt == 1) return ydt == 1 ? by_op<float, float>(op, dir, X, Y, scratch, N, D, st)
                                : by_op<float, double>(op, dir, X, Y, scratch, N, D, st);
  if (xdt == 2) return ydt == 1 ? by_op<double, float>(op, dir, X, Y, scratch, N, D, st)
                                : by_op<double, double>(op, dir, X, Y, scratch, N, D, st);
  return -1;
}

// y (one double, device) = sum(A .* B) over n cells of two same-typed dense arrays (dt: 0 bf16,
// 1 fp32, 2 fp64), fp64 accumulation; scratch: sysml_agg_scratch(0, n, 1) bytes.
int sysml_dot(int dt, const void* A, const void* B, double* y, void* scratch, int64_t n, void* stream) {
  using namespace sysml_ag;
  if (n <= 0) return -1;
  hipStream_t st = (hipStream_t)stream;
  int nb = grid_for(n, NT * 8);
  if (nb > 1024) nb = 1024;                      // the scratch holds 1024 partials
  St* part = (St*)scratch;
  if (dt == 0) hipLaunchKernelGGL(dot_part<uint16_t>, dim3(nb), dim3(NT), 0, st, (const uint16_t*)A, (const uint16_t*)B, part, n);
  else if (dt == 1) hipLaunchKernelGGL(dot_part<float>, dim3(nb), dim3(NT), 0, st, (const float*)A, (const float*)B, part, n);
  else if (dt == 2) hipLaunchKernelGGL(dot_part<double>, dim3(nb), dim3(NT), 0, st, (const double*)A, (const double*)B, part, n);
  else return -1;
  hipLaunchKernelGGL(all_final<SUM>, dim3(1), dim3(64), 0, st, (const St*)part, y, nb, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// y (n values, fp32 when ydt == 1 else fp64) = sum / min / max (op 0 / 3 / 4) over the nb rows of
// an nb x n fp64 partial block -- one pass, the last step of a blocked column aggregate.
int sysml_fold_rows(int op, int ydt, const double* part, void* y, int nb, int64_t n, void* stream) {
  using namespace sysml_ag;
  if (nb <= 0 || n <= 0) return -1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid_for(n, NT * 4)), t(NT);
#define FOLD(TO_, OP_) hipLaunchKernelGGL((fold_rows<TO_, OP_>), g, t, 0, st, part, (TO_*)y, nb, n)
  if (op == SUM) { if (ydt == 1) FOLD(float, SUM); else FOLD(double, SUM); }
  else if (op == MIN) { if (ydt == 1) FOLD(float, MIN); else FOLD(double, MIN); }
  else if (op == MAX) { if (ydt == 1) FOLD(float, MAX); else FOLD(double, MAX); }
  else return -1;
#undef FOLD
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
