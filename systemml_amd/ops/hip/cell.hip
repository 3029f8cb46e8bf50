// Fused cellwise operator ("cell template"): one kernel evaluates a whole DAG of elementwise
// binary / unary operators -- optionally followed by a full, row or column aggregate -- per
// output cell, reading every input once and writing only the result (reference:
// hops/codegen/template/TemplateCell.java + runtime/codegen/SpoofCellwise.java, which generate
// and javac-compile a Java class per fused DAG).
//
// MI355X design: no run-time code generation.  The compiler (compiler/codegen.py) lowers each
// fused DAG to a short register program (<= 40 instructions over 16 registers) that travels
// in the kernel arguments; the opcode and register indices are wave-uniform, so the
// interpreter's dispatch is scalar branching (SALU, s_cbranch) and only the selected
// operation issues vector instructions.  Each thread evaluates V = 4 adjacent cells at a
// time, so every dispatch is amortised over four cells and contiguous inputs / the output
// move as 16-byte vector loads / stores.  Inputs broadcast as full matrices, row vectors,
// column vectors or scalars (host literal or a device-resident value), in fp32 / fp64 / bf16
// storage; computation runs in the output type T (fp32 or fp64) with FMA contraction off, so
// every cell is rounded exactly as the unfused torch operators round it.
//
// Aggregates: sum / sumsq / min / max over all cells (per-block partials, reduced on the
// host side by one tiny op -- no atomics, deterministic), per row (lane groups of G lanes
// per row, xor-shuffle reduction) and per column (column tiles x row chunks, LDS reduction,
// per-chunk partials).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#pragma clang fp contract(off)

namespace sysml_cl {

constexpr int MAXIN = 12;
constexpr int MAXOPS = 40;
constexpr int NR = 16;
constexpr int THREADS = 256;

enum : int {
  ADD = 1, SUB, MUL, DIV, POW, MOD, INTDIV, EQ, NE, LT, LE, GT, GE, AND, OR, XOR, MIN, MAX, LOGB, SQ,
  NEG = 32, NOT, ABS, EXP, LOG, SQRT, ROUND, FLOOR, CEIL, SIGN, SIN, COS, TAN, ASIN, ACOS, ATAN, SINH, COSH,
  TANH, SIGMOID
};
enum : int { FULL = 0, ROWV = 1, COLV = 2, HSCALAR = 3, DSCALAR = 4 };
enum : int { A_SUM = 0, A_SUMSQ = 1, A_MIN = 2, A_MAX = 3 };

struct In {
  const void* p;
  double s;
  int mode;    // FULL / ROWV / COLV / HSCALAR / DSCALAR
  int dtype;   // 0 fp32, 1 fp64, 2 bf16
  int vec;     // FULL input whose base is 16-byte aligned (vector loads)
  int pad;
};

struct Prog {
  In in[MAXIN];
  int64_t rows, cols, total;
  int n_in, n_ops, out, aggop;
  int need_ij, pad;
};

static_assert(sizeof(In) == 32, "In layout");
static_assert(sizeof(Prog) == MAXIN * 32 + 24 + 24, "Prog layout");

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

template <typename T>
__device__ __forceinline__ T ld(const In& in, int64_t off) {
  if (in.dtype == 0) return (T)static_cast<const float*>(in.p)[off];
  if (in.dtype == 1) return (T)static_cast<const double*>(in.p)[off];
  return (T)bf2f(static_cast<const uint16_t*>(in.p)[off]);
}

// V adjacent cells starting at flat index e0 (row i[v], column j[v])
template <typename T, int V>
__device__ __forceinline__ void load_in(const In& in, int64_t e0, const int64_t (&i)[V], const int64_t (&j)[V],
                                        bool whole, int64_t total, T (&r)[V]) {
  switch (in.mode) {
    case FULL:
      if constexpr (V == 4) {
        if (whole && in.vec) {
        if (in.dtype == 0) {
          const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(in.p) + e0);
          r[0] = (T)q.x; r[1] = (T)q.y; r[2] = (T)q.z; r[3] = (T)q.w;
        } else if (in.dtype == 1) {
          const double2 q0 = *reinterpret_cast<const double2*>(static_cast<const double*>(in.p) + e0);
          const double2 q1 = *reinterpret_cast<const double2*>(static_cast<const double*>(in.p) + e0 + 2);
          r[0] = (T)q0.x; r[1] = (T)q0.y; r[2] = (T)q1.x; r[3] = (T)q1.y;
        } else {
          const uint2 q = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(in.p) + e0);
          r[0] = (T)bf2f(q.x & 0xffff); r[1] = (T)bf2f(q.x >> 16);
          r[2] = (T)bf2f(q.y & 0xffff); r[3] = (T)bf2f(q.y >> 16);
        }
        break;
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v) r[v] = (e0 + v < total) ? ld<T>(in, e0 + v) : T(0);
      break;
    case ROWV:
#pragma unroll
      for (int v = 0; v < V; ++v) r[v] = ld<T>(in, j[v]);
      break;
    case COLV:
#pragma unroll
      for (int v = 0; v < V; ++v) r[v] = ld<T>(in, i[v]);
      break;
    case HSCALAR: {
      const T s = (T)in.s;
#pragma unroll
      for (int v = 0; v < V; ++v) r[v] = s;
      break;
    }
    default: {
      const T s = ld<T>(in, 0);
#pragma unroll
      for (int v = 0; v < V; ++v) r[v] = s;
    }
  }
}

// The register file is V separate NR-entry arrays (one per cell of the thread's group):
// indexed by a wave-uniform register number, each is promoted to a VGPR vector and read /
// written with v_movrel (a single 4 x NR array would not be promoted and would live in scratch).
template <typename T, int V>
__device__ __forceinline__ void getr(T* const (&rf)[V], int idx, T (&o)[V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) o[v] = rf[v][idx];
}

template <typename T, int V>
__device__ __forceinline__ void setr(T* const (&rf)[V], int idx, const T (&o)[V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) rf[v][idx] = o[v];
}

template <typename T>
__device__ __forceinline__ T t_nan() { return (T)NAN; }

// torch.remainder: fmod adjusted to the divisor's sign
template <typename T>
__device__ __forceinline__ T rem(T a, T b) {
  T m = fmod(a, b);
  if (m != T(0) && ((b < T(0)) != (m < T(0)))) m += b;
  return m;
}

template <typename T, int V>
__device__ __forceinline__ void run(const Prog& P, const int4* __restrict__ code, T* const (&r)[V]) {
  for (int q = 0; q < P.n_ops; ++q) {
    const int4 c = code[q];        // wave-uniform: scalar loads
    const int op = c.x;
    T x[V], y[V], z[V];
    getr<T, V>(r, c.z, x);
    if (op < NEG) getr<T, V>(r, c.w, y);
#define SYSML_OP(code, expr)                  \
  case code:                                  \
    _Pragma("unroll") for (int v = 0; v < V; ++v) { \
      const T a = x[v];                       \
      const T b = y[v];                       \
      (void)b;                                \
      z[v] = (expr);                          \
    }                                         \
    break;
    switch (op) {
      SYSML_OP(ADD, a + b)
      SYSML_OP(SUB, a - b)
      SYSML_OP(MUL, a * b)
      SYSML_OP(DIV, a / b)
      SYSML_OP(POW, pow(a, b))
      SYSML_OP(MOD, rem(a, b))
      SYSML_OP(INTDIV, floor(a / b))
      SYSML_OP(EQ, a == b ? T(1) : T(0))
      SYSML_OP(NE, a != b ? T(1) : T(0))
      SYSML_OP(LT, a < b ? T(1) : T(0))
      SYSML_OP(LE, a <= b ? T(1) : T(0))
      SYSML_OP(GT, a > b ? T(1) : T(0))
      SYSML_OP(GE, a >= b ? T(1) : T(0))
      SYSML_OP(AND, (a != T(0) && b != T(0)) ? T(1) : T(0))
      SYSML_OP(OR, (a != T(0) || b != T(0)) ? T(1) : T(0))
      SYSML_OP(XOR, ((a != T(0)) != (b != T(0))) ? T(1) : T(0))
      SYSML_OP(MIN, (a != a || b != b) ? t_nan<T>() : (a < b ? a : b))
      SYSML_OP(MAX, (a != a || b != b) ? t_nan<T>() : (a > b ? a : b))
      SYSML_OP(LOGB, log(a) / log(b))
      SYSML_OP(SQ, a * a)
      SYSML_OP(NEG, -a)
      SYSML_OP(NOT, a == T(0) ? T(1) : T(0))
      SYSML_OP(ABS, fabs(a))
      SYSML_OP(EXP, exp(a))
      SYSML_OP(LOG, log(a))
      SYSML_OP(SQRT, sqrt(a))
      SYSML_OP(ROUND, floor(a + T(0.5)))
      SYSML_OP(FLOOR, floor(a))
      SYSML_OP(CEIL, ceil(a))
      SYSML_OP(SIGN, (T)((a > T(0)) - (a < T(0))))
      SYSML_OP(SIN, sin(a))
      SYSML_OP(COS, cos(a))
      SYSML_OP(TAN, tan(a))
      SYSML_OP(ASIN, asin(a))
      SYSML_OP(ACOS, acos(a))
      SYSML_OP(ATAN, atan(a))
      SYSML_OP(SINH, sinh(a))
      SYSML_OP(COSH, cosh(a))
      SYSML_OP(TANH, tanh(a))
      SYSML_OP(SIGMOID, T(1) / (T(1) + exp(-a)))
      default:
#pragma unroll
        for (int v = 0; v < V; ++v) z[v] = t_nan<T>();
    }
#undef SYSML_OP
    setr<T, V>(r, c.y, z);
  }
}

// V cells starting at (i0, j0) / flat e0: inputs -> registers -> program -> output register
template <typename T, int V>
__device__ __forceinline__ void eval(const Prog& P, const int4* __restrict__ code, int64_t e0, int64_t i0, int64_t j0, bool whole, T (&o)[V]) {
  int64_t i[V], j[V];
  i[0] = i0;
  j[0] = j0;
#pragma unroll
  for (int v = 1; v < V; ++v) {
    i[v] = i[v - 1];
    j[v] = j[v - 1] + 1;
    while (j[v] >= P.cols) {
      j[v] -= P.cols;
      ++i[v];
    }
    if (i[v] >= P.rows) i[v] = P.rows - 1;     // cells past the end: clamped, never stored
  }
  T r0[NR], r1[NR], r2[NR], r3[NR];
  T* const rf_all[4] = {r0, r1, r2, r3};
  T* const (&r)[V] = reinterpret_cast<T* const (&)[V]>(rf_all);
#pragma unroll
  for (int k = 0; k < MAXIN; ++k) {
    if (k >= P.n_in) break;
    T x[V];
    load_in<T, V>(P.in[k], e0, i, j, whole, P.total, x);
#pragma unroll
    for (int v = 0; v < V; ++v) r[v][k] = x[v];
  }
  run<T, V>(P, code, r);
  getr<T, V>(r, P.out, o);
}

template <typename T>
__device__ __forceinline__ double acc_init(int aggop) {
  return aggop == A_MIN ? INFINITY : (aggop == A_MAX ? -INFINITY : 0.0);
}

__device__ __forceinline__ double acc_add(int aggop, double acc, double v) {
  switch (aggop) {
    case A_SUM: return acc + v;
    case A_SUMSQ: return acc + v * v;
    case A_MIN: return (v != v || v < acc) ? v : acc;
    default: return (v != v || v > acc) ? v : acc;
  }
}

__device__ __forceinline__ double acc_comb(int aggop, double a, double b) {
  if (aggop == A_SUM || aggop == A_SUMSQ) return a + b;
  if (a != a) return a;
  if (b != b) return b;
  return aggop == A_MIN ? (a < b ? a : b) : (a > b ? a : b);
}

// ---- no aggregate (AGG = 0) / full aggregate (AGG = 1): flat traversal, 4 cells per thread
template <typename T, int AGG>
__global__ void __launch_bounds__(THREADS) cell_flat(const Prog P, const int4* __restrict__ code, T* __restrict__ out, double* __restrict__ part) {
  constexpr int V = 4;
  const int64_t groups = (P.total + V - 1) / V;
  double acc = acc_init<T>(P.aggop);
  for (int64_t g = (int64_t)blockIdx.x * THREADS + threadIdx.x; g < groups; g += (int64_t)gridDim.x * THREADS) {
    const int64_t e0 = g * V;
    const bool whole = e0 + V <= P.total;
    int64_t i0 = 0, j0 = 0;
    if (P.need_ij) {
      i0 = e0 / P.cols;
      j0 = e0 - i0 * P.cols;
    }
    T o[V];
    eval<T, V>(P, code, e0, i0, j0, whole, o);
    if (AGG == 0) {
      if constexpr (sizeof(T) == 4) {
        if (whole) {
          *reinterpret_cast<float4*>(out + e0) = make_float4(o[0], o[1], o[2], o[3]);
          continue;
        }
      } else {
        if (whole) {
          *reinterpret_cast<double2*>(out + e0) = make_double2(o[0], o[1]);
          *reinterpret_cast<double2*>(out + e0 + 2) = make_double2(o[2], o[3]);
          continue;
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (e0 + v < P.total) out[e0 + v] = o[v];
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (e0 + v < P.total) acc = acc_add(P.aggop, acc, (double)o[v]);
    }
  }
  if (AGG == 1) {
    __shared__ double red[THREADS / 64];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc = acc_comb(P.aggop, acc, __shfl_xor(acc, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double a = red[0];
#pragma unroll
      for (int w = 1; w < THREADS / 64; ++w) a = acc_comb(P.aggop, a, red[w]);
      part[blockIdx.x] = a;
    }
  }
}

// ---- row aggregate: G lanes per row (G = 1 for narrow rows ... 64 for wide ones)
template <typename T, int G>
__global__ void __launch_bounds__(THREADS) cell_row(const Prog P, const int4* __restrict__ code, T* __restrict__ out) {
  constexpr int RPB = THREADS / G;            // rows per block per step
  const int gl = threadIdx.x % G;
  for (int64_t i = (int64_t)blockIdx.x * RPB + threadIdx.x / G; i - threadIdx.x / G < P.rows;
       i += (int64_t)gridDim.x * RPB) {
    const bool live = i < P.rows;
    const int64_t ii = live ? i : P.rows - 1;
    double acc = acc_init<T>(P.aggop);
    for (int64_t j = gl; j < P.cols; j += G) {
      T o[1];
      eval<T, 1>(P, code, ii * P.cols + j, ii, j, true, o);
      acc = acc_add(P.aggop, acc, (double)o[0]);
    }
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) acc = acc_comb(P.aggop, acc, __shfl_xor(acc, off, 64));
    if (live && gl == 0) out[i] = (T)acc;
  }
}

// ---- column aggregate: CW columns x (THREADS / CW) row phases per block; blockIdx.y = row chunk
template <typename T, int CW>
__global__ void __launch_bounds__(THREADS) cell_col(const Prog P, const int4* __restrict__ code, int64_t chunk, double* __restrict__ part) {
  constexpr int RPH = THREADS / CW;
  __shared__ double red[THREADS];
  const int c = threadIdx.x % CW, ph = threadIdx.x / CW;
  const int64_t j = (int64_t)blockIdx.x * CW + c;
  const int64_t r0 = (int64_t)blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < P.rows ? r0 + chunk : P.rows;
  double acc = acc_init<T>(P.aggop);
  if (j < P.cols) {
    for (int64_t i = r0 + ph; i < r1; i += RPH) {
      T o[1];
      eval<T, 1>(P, code, i * P.cols + j, i, j, true, o);
      acc = acc_add(P.aggop, acc, (double)o[0]);
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (ph == 0 && j < P.cols) {
    double a = acc;
    for (int p = 1; p < RPH; ++p) a = acc_comb(P.aggop, a, red[p * CW + c]);
    part[(int64_t)blockIdx.y * P.cols + j] = a;
  }
}

template <typename T>
int launch(int agg, const Prog& P, const int4* code, void* out, void* part, int64_t nblk, hipStream_t s) {
  const dim3 t(THREADS);
  if (agg == 0 || agg == 1) {
    const dim3 g((unsigned)nblk);
    if (agg == 0) hipLaunchKernelGGL((cell_flat<T, 0>), g, t, 0, s, P, code, (T*)out, (double*)nullptr);
    else hipLaunchKernelGGL((cell_flat<T, 1>), g, t, 0, s, P, code, (T*)nullptr, (double*)part);
  } else if (agg == 2) {
    const dim3 g((unsigned)nblk);
    if (P.cols <= 8) hipLaunchKernelGGL((cell_row<T, 1>), g, t, 0, s, P, code, (T*)out);
    else if (P.cols <= 32) hipLaunchKernelGGL((cell_row<T, 4>), g, t, 0, s, P, code, (T*)out);
    else if (P.cols <= 128) hipLaunchKernelGGL((cell_row<T, 16>), g, t, 0, s, P, code, (T*)out);
    else hipLaunchKernelGGL((cell_row<T, 64>), g, t, 0, s, P, code, (T*)out);
  } else {
    const int cw = P.cols <= 8 ? 8 : 64;
    const dim3 g((unsigned)((P.cols + cw - 1) / cw), (unsigned)nblk);
    const int64_t chunk = (P.rows + nblk - 1) / nblk;
    if (cw == 8) hipLaunchKernelGGL((cell_col<T, 8>), g, t, 0, s, P, code, chunk, (double*)part);
    else hipLaunchKernelGGL((cell_col<T, 64>), g, t, 0, s, P, code, chunk, (double*)part);
  }
  return (int)hipGetLastError();
}

}  // namespace sysml_cl

extern "C" {

int sysml_cell_prog_size() { return (int)sizeof(sysml_cl::Prog); }

// Number of blocks (flat / row kernels) or row chunks (column kernel) the launch will use;
// the caller sizes the partials buffer (agg 1: nblk doubles, agg 3: nblk x cols doubles).
int64_t sysml_cell_blocks(int agg, int64_t rows, int64_t cols) {
  using namespace sysml_cl;
  if (agg == 0 || agg == 1) {
    const int64_t groups = (rows * cols + 3) / 4;
    int64_t b = (groups + THREADS - 1) / THREADS;
    const int64_t cap = agg == 1 ? 2048 : 16384;
    return b < 1 ? 1 : (b > cap ? cap : b);
  }
  if (agg == 2) {
    const int G = cols <= 8 ? 1 : (cols <= 32 ? 4 : (cols <= 128 ? 16 : 64));
    int64_t b = (rows + THREADS / G - 1) / (THREADS / G);
    return b < 1 ? 1 : (b > 16384 ? 16384 : b);
  }
  // >= 32 rows per thread (SYSML_COL_RPT; ResNet-50 at 16 / 32 / 64: 5046 / 5101 / 5077 img/s):
  // a batch-norm column aggregate (256 image rows x C*H*W columns) then has 2 row blocks per
  // column strip -- one block per strip left ~3 blocks per CU
  static const int rpt = [] { const char* e = getenv("SYSML_COL_RPT"); return e ? atoi(e) : 32; }();
  const int cw = cols <= 8 ? 8 : 64;
  const int64_t rph = THREADS / cw;
  int64_t b = (rows + rph * rpt - 1) / (rph * rpt);
  return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

// prog: host Prog (inputs, sizes); code: DEVICE array of n_ops int4 (opcode, dst, a, b) with
// register indices < 16, validated by the caller (ops/cell.py) when it uploads the program.
// dtype 0: fp32 compute / output, 1: fp64.  agg 0 none (out: rows x cols), 1 all (part:
// nblk partials), 2 row (out: rows), 3 col (part: nblk x cols partials).  Returns 0, -1
// (invalid program) or a hipError_t.
int sysml_cell(int dtype, int agg, const void* prog, const void* code, void* out, void* part, int64_t nblk, void* stream) {
  using namespace sysml_cl;
  Prog P = *static_cast<const Prog*>(prog);
  if (P.n_in < 1 || P.n_in > MAXIN || P.n_ops < 0 || P.n_ops > MAXOPS || P.out < 0 || P.out >= NR) return -1;
  if (P.rows <= 0 || P.cols <= 0 || P.total != P.rows * P.cols) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == 0) return launch<float>(agg, P, (const int4*)code, out, part, nblk, s);
  if (dtype == 1) return launch<double>(agg, P, (const int4*)code, out, part, nblk, s);
  return -1;
}

}  // extern "C"
