// Row-streaming kernels for tall-skinny linear algebra on MI355X (gfx950).
//
// One launch reads a tall matrix X [N x D] (row-major; bf16, fp32 or fp64) exactly
// once from HBM and performs one of:
//   XV      : U[N x K]  = X %*% V                         (ba+* matrix-vector / skinny)
//   XTG     : R[D x K]  = t(X) %*% G                      (ba+* with transposed LHS)
//   XTXV    : R         = t(X) %*% (X %*% V)              (mmchain XtXv)
//   XTWXV   : R         = t(X) %*% (w * (X %*% V))        (mmchain XtwXv)
//   XTXVY   : R         = t(X) %*% ((X %*% V) - Y)        (mmchain XtXvy)
//   XTPSXV  : R         = t(X) %*% (Q - P*rowSums(Q)),  Q = P*(X %*% V)
//                                                         (multinomial logreg H*v, row template)
//   XTSMG   : U = X %*% V and R = t(X) %*% (softmax([U, 0])[, 1:K] - Y)
//                                                         (multinomial logreg gradient at a candidate
//                                                          point, two outputs, one pass)
//   ROWSSQ  : U[N x 1]  = rowSums(X^2)
//   COLSSQ  : R[D x 1]  = colSums(X^2)
//   COLSUM  : R[D x 1]  = colSums(X)
//   ROWSUM  : U[N x 1]  = rowSums(X)
//
// Reference semantics: LibMatrixMult.matrixMultChain / matrixMult (CP) and the
// codegen Row template (hops/codegen/template/TemplateRow.java); here fused so X
// streams through the CU once (memory-bound: 1 byte of X per ~K FMAs).
//
// Mapping (wave64): a wave owns one row at a time.  Lane l owns the 8-column
// chunks c = (j*64 + l)*8 .. +7, j < J (so D <= 512*J).  Row loads are 16-byte
// vector loads (one 1-KiB coalesced wave-instruction per chunk for bf16); the next
// row of the wave is prefetched into registers before the current row's wave
// reductions so HBM latency overlaps the shuffle/FMA work.  V is staged once per
// block in LDS; t(X)-side accumulators live in registers (J*8 x K per lane) and are
// combined across the 4 waves through LDS, then one partial [D x K] per block is
// written (reduced over blocks by the host wrapper).  Accumulation is fp32 for
// bf16/fp32 X and fp64 for fp64 X.
#include <hip/hip_runtime.h>
#include <unordered_set>
#include <stdint.h>

// cache policy of the streamed X rows' LDS-DMA (aux of global_load_lds): 2 = non-temporal -- each
// X row is read once per pass and X is far larger than the 256 MB MALL, so the default policy
// only evicts the small operands (MI355X_MICROARCH.md: LDS-DMA streams 6.4 -> 6.5-6.8 TB/s nt)
#ifndef SYSML_X_AUX
#define SYSML_X_AUX 2
#endif

namespace sysml {

enum Mode { XV = 0, XTG = 1, XTXV = 2, XTWXV = 3, XTXVY = 4, XTPSXV = 5,
            ROWSSQ = 6, COLSSQ = 7, COLSUM = 8, ROWSUM = 9, XTSMG = 10 };

constexpr int WAVES = 4;
constexpr int BLOCK = 64 * WAVES;

template <int M> struct ModeInfo {
  static constexpr bool needV   = (M == XV || M == XTXV || M == XTWXV || M == XTXVY || M == XTPSXV ||
                                   M == XTSMG);
  static constexpr bool accum   = (M == XTG || M == XTXV || M == XTWXV || M == XTXVY || M == XTPSXV ||
                                   M == COLSSQ || M == COLSUM || M == XTSMG);
  static constexpr bool rowOut  = (M == XV || M == ROWSSQ || M == ROWSUM);
};

// ---------------------------------------------------------------------------
// element loads: 8 consecutive elements of one row into accumulator type A
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }

template <typename T> struct Raw8;
template <> struct Raw8<uint16_t> { uint4 v; };
template <> struct Raw8<float>    { float4 v[2]; };
template <> struct Raw8<double>   { double2 v[4]; };

template <typename T>
__device__ __forceinline__ void load_raw(Raw8<T>& r, const T* __restrict__ row, int c0, int D, bool vec);

typedef unsigned int sysml_u4v __attribute__((ext_vector_type(4)));

// a bf16 X row piece, non-temporal (X streams once per pass, SYSML_X_AUX above)
__device__ __forceinline__ uint4 ld_x16(const uint16_t* p) {
#if SYSML_X_AUX
  const sysml_u4v t = __builtin_nontemporal_load(reinterpret_cast<const sysml_u4v*>(p));
  return make_uint4(t.x, t.y, t.z, t.w);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}

template <>
__device__ __forceinline__ void load_raw<uint16_t>(Raw8<uint16_t>& r, const uint16_t* __restrict__ row,
                                                   int c0, int D, bool vec) {
  if (vec && c0 + 8 <= D) {
    r.v = ld_x16(row + c0);
  } else {
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = (c0 + i < D) ? row[c0 + i] : 0u;
    r.v.x = e[0] | (e[1] << 16); r.v.y = e[2] | (e[3] << 16);
    r.v.z = e[4] | (e[5] << 16); r.v.w = e[6] | (e[7] << 16);
  }
}

template <>
__device__ __forceinline__ void load_raw<float>(Raw8<float>& r, const float* __restrict__ row,
                                                int c0, int D, bool vec) {
  if (vec && c0 + 8 <= D) {
    r.v[0] = *reinterpret_cast<const float4*>(row + c0);
    r.v[1] = *reinterpret_cast<const float4*>(row + c0 + 4);
  } else {
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = (c0 + i < D) ? row[c0 + i] : 0.f;
    r.v[0] = make_float4(e[0], e[1], e[2], e[3]);
    r.v[1] = make_float4(e[4], e[5], e[6], e[7]);
  }
}

template <>
__device__ __forceinline__ void load_raw<double>(Raw8<double>& r, const double* __restrict__ row,
                                                 int c0, int D, bool vec) {
  if (vec && c0 + 8 <= D) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = *reinterpret_cast<const double2*>(row + c0 + 2 * i);
  } else {
    double e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = (c0 + i < D) ? row[c0 + i] : 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = make_double2(e[2 * i], e[2 * i + 1]);
  }
}

// unconditional 16-B-aligned loads of 8 elements (vector path of the packed kernel)
template <typename T>
__device__ __forceinline__ void load_vec(Raw8<T>& r, const T* __restrict__ p);
template <>
__device__ __forceinline__ void load_vec<uint16_t>(Raw8<uint16_t>& r, const uint16_t* __restrict__ p) {
  r.v = ld_x16(p);
}
template <>
__device__ __forceinline__ void load_vec<float>(Raw8<float>& r, const float* __restrict__ p) {
  r.v[0] = *reinterpret_cast<const float4*>(p);
  r.v[1] = *reinterpret_cast<const float4*>(p + 4);
}
template <>
__device__ __forceinline__ void load_vec<double>(Raw8<double>& r, const double* __restrict__ p) {
#pragma unroll
  for (int i = 0; i < 4; ++i) r.v[i] = *reinterpret_cast<const double2*>(p + 2 * i);
}

template <typename A>
__device__ __forceinline__ void unpack(const Raw8<uint16_t>& r, A* x) {
  x[0] = bf2f(r.v.x & 0xffffu); x[1] = bf2f(r.v.x >> 16);
  x[2] = bf2f(r.v.y & 0xffffu); x[3] = bf2f(r.v.y >> 16);
  x[4] = bf2f(r.v.z & 0xffffu); x[5] = bf2f(r.v.z >> 16);
  x[6] = bf2f(r.v.w & 0xffffu); x[7] = bf2f(r.v.w >> 16);
}
template <typename A>
__device__ __forceinline__ void unpack(const Raw8<float>& r, A* x) {
  x[0] = r.v[0].x; x[1] = r.v[0].y; x[2] = r.v[0].z; x[3] = r.v[0].w;
  x[4] = r.v[1].x; x[5] = r.v[1].y; x[6] = r.v[1].z; x[7] = r.v[1].w;
}
template <typename A>
__device__ __forceinline__ void unpack(const Raw8<double>& r, A* x) {
#pragma unroll
  for (int i = 0; i < 4; ++i) { x[2 * i] = r.v[i].x; x[2 * i + 1] = r.v[i].y; }
}

// Wave-wide sum whose result is wave-uniform.  fp32: DPP butterflies inside each
// 16-lane row (quad_perm xor1 / xor2, row_half_mirror, row_mirror: pure VALU, no LDS
// crossbar) + 4 v_readlane for the cross-row total.  fp64 keeps the generic shuffle.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror  -> every lane holds its 16-lane row sum
  const int iv = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(iv, 0)) + __int_as_float(__builtin_amdgcn_readlane(iv, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(iv, 32)) + __int_as_float(__builtin_amdgcn_readlane(iv, 48)));
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------------------
// main kernel: each wave streams R rows per iteration (rows r + i*WAVES), so R
// independent reduction chains interleave and 2*R row loads are in flight.
// ---------------------------------------------------------------------------
template <typename T, typename A, int K, int J, int MODE, int R>
__global__ void __launch_bounds__(BLOCK)
rowstream_kernel(const T* __restrict__ X, int64_t N, int D, int vec,
                 const A* __restrict__ V, int ldv,          // D x K (row-major, ld ldv)
                 const A* __restrict__ S, int lds, int sbc, // side input rows (G / w / Y / P)
                 A* __restrict__ out, int ldo,              // U rows, or per-block partials
                 int64_t rows_per_block) {
  using MI = ModeInfo<MODE>;
  constexpr int C = J * 8;                       // columns owned per lane
  extern __shared__ __attribute__((aligned(16))) char smem[];
  A* sV = reinterpret_cast<A*>(smem);            // [J*512][K] (zero padded)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Dp = J * 512;

  if constexpr (MI::needV) {
    for (int i = threadIdx.x; i < Dp * K; i += BLOCK) {
      int d = i / K, k = i - d * K;
      sV[i] = (d < D) ? V[(int64_t)d * ldv + k] : A(0);
    }
    __syncthreads();
  }

  A acc[MI::accum ? C : 1][MI::accum ? K : 1];
  if constexpr (MI::accum) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < K; ++k) acc[c][k] = A(0);
  }

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < N) ? r0 + rows_per_block : N;
  constexpr int STEP = WAVES * R;

  Raw8<T> nxt[R][J];
  int64_t r = r0 + wave;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int64_t ri = r + i * WAVES;
    if (ri < r1) {
#pragma unroll
      for (int j = 0; j < J; ++j) load_raw<T>(nxt[i][j], X + ri * (int64_t)D, (j * 64 + lane) * 8, D, vec);
    } else {
#pragma unroll
      for (int j = 0; j < J; ++j) nxt[i][j] = Raw8<T>{};   // rows past the block: zeros, never garbage
    }
  }
  for (; r < r1; r += STEP) {
    A x[R][C];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j) unpack<A>(nxt[i][j], x[i] + j * 8);
    // prefetch the wave's next R rows before the reductions below
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t rn = r + STEP + i * WAVES;
      if (rn < r1) {
#pragma unroll
        for (int j = 0; j < J; ++j) load_raw<T>(nxt[i][j], X + rn * (int64_t)D, (j * 64 + lane) * 8, D, vec);
      } else {
#pragma unroll
        for (int j = 0; j < J; ++j) nxt[i][j] = Raw8<T>{};
      }
    }
    bool valid[R];
#pragma unroll
    for (int i = 0; i < R; ++i) valid[i] = (r + i * WAVES) < r1;   // wave-uniform

    if constexpr (MODE == ROWSSQ || MODE == ROWSUM) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        A s = A(0);
#pragma unroll
        for (int c = 0; c < C; ++c) s += (MODE == ROWSSQ) ? x[i][c] * x[i][c] : x[i][c];
        s = wave_sum(s);
        if (valid[i] && lane == 0) out[(r + i * WAVES) * (int64_t)ldo] = s;
      }
      continue;
    }
    if constexpr (MODE == COLSSQ || MODE == COLSUM) {
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c][0] += (MODE == COLSSQ) ? x[i][c] * x[i][c] : x[i][c];
      continue;
    }

    A g[R][K];
    if constexpr (MI::needV) {
      A u[R][K];
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int k = 0; k < K; ++k) u[i][k] = A(0);
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const A* vrow = sV + ((j * 64 + lane) * 8) * K;
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const A vv = vrow[e * K + k];
#pragma unroll
            for (int i = 0; i < R; ++i) u[i][k] += x[i][j * 8 + e] * vv;
          }
      }
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int i = 0; i < R; ++i) u[i][k] = wave_sum(u[i][k]);
      if constexpr (MODE == XV) {
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int k = 0; k < K; ++k)
            if (valid[i] && lane == k) out[(r + i * WAVES) * (int64_t)ldo + k] = u[i][k];
        continue;
      } else {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const int64_t ri = r + i * WAVES;
          const bool ok = valid[i];
          if constexpr (MODE == XTXV) {
#pragma unroll
            for (int k = 0; k < K; ++k) g[i][k] = ok ? u[i][k] : A(0);
          } else if constexpr (MODE == XTWXV) {
#pragma unroll
            for (int k = 0; k < K; ++k) g[i][k] = ok ? S[ri * (int64_t)lds + (sbc ? 0 : k)] * u[i][k] : A(0);
          } else if constexpr (MODE == XTXVY) {
#pragma unroll
            for (int k = 0; k < K; ++k) g[i][k] = ok ? u[i][k] - S[ri * (int64_t)lds + (sbc ? 0 : k)] : A(0);
          } else if constexpr (MODE == XTPSXV) {
            A p[K], q[K], sq = A(0);
#pragma unroll
            for (int k = 0; k < K; ++k) { p[k] = ok ? S[ri * (int64_t)lds + k] : A(0); q[k] = p[k] * u[i][k]; sq += q[k]; }
#pragma unroll
            for (int k = 0; k < K; ++k) g[i][k] = q[k] - p[k] * sq;
          }
        }
      }
    } else {  // XTG
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int64_t ri = r + i * WAVES;
#pragma unroll
        for (int k = 0; k < K; ++k) g[i][k] = valid[i] ? S[ri * (int64_t)lds + k] : A(0);
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[c][k] += x[i][c] * g[i][k];
  }

  if constexpr (MI::accum) {
    constexpr int KO = (MODE == COLSSQ || MODE == COLSUM) ? 1 : K;
    // combine the 4 waves' register accumulators through LDS, then one partial per block
    __syncthreads();
    A* red = reinterpret_cast<A*>(smem);          // reuse: [J*512][KO]
    for (int w = 0; w < WAVES; ++w) {
      if (wave == w) {
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int k = 0; k < KO; ++k) {
              int idx = ((j * 64 + lane) * 8 + e) * KO + k;
              red[idx] = (w == 0) ? acc[j * 8 + e][k] : red[idx] + acc[j * 8 + e][k];
            }
      }
      __syncthreads();
    }
    A* dst = out + (int64_t)blockIdx.x * D * KO;
    for (int i = threadIdx.x; i < D * KO; i += BLOCK) dst[i] = red[i];
  }
}

// ---------------------------------------------------------------------------
// Packed-fp32 kernels for K in {2,4,8} (fp32 accumulate: bf16 / fp32 X), vector rows
// only (D % 8 == 0, 16-B aligned; the host routes everything else to rowstream_kernel).
//
// The k dimension is carried in float2 pairs so every dot-product / accumulate FMA is a
// v_pk_fma_f32 (2 FMAs per lane per instruction), and for C*K <= 64 the lane's slice of
// V lives in registers for the whole launch (no per-row LDS traffic).  Row-side values
// (g) are wave-uniform after the DPP reduction.  The per-row math lives in RowOps and is
// shared by the two streaming front ends:
//
//  * rowstream_dma_kernel (every accumulating mode: XTG and the fused chains) — each wave
//    owns an R-slot ring in LDS that is filled by LDS-DMA (global_load_lds_dwordx4 for the
//    X row, global_load_lds_dword for the row-side operand S) and drained with a COUNTED
//    s_waitcnt vmcnt((R-1) * loads_per_row): R rows per wave stay in flight across the
//    whole loop.  The LDS reads are inline asm (data and lgkmcnt wait in one statement) so
//    hipcc's waitcnt pass, which would otherwise drain vmcnt(0) before any ds_read while
//    an LDS-DMA is outstanding, sees no LDS access to protect.  (Register-staged rings do
//    not survive hipcc: it sinks the prefetch loads into the consuming iteration and waits
//    vmcnt(0) there — profiles/mfma_chain_experiments.md.)
//  * rowstream_pk_kernel (XV, whose per-row stores would share vmcnt with the ring) —
//    register prefetch ring with unconditional (clamped) loads.
//
// Out-of-range handling without branches: a row index past the block's range re-reads
// the block's last row, a column chunk past D re-reads the row's last chunk.  Those values
// meet zero V rows (phase 1), a zero row weight (phase 2) or accumulator columns that are
// never written out.
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) char lds_char;

template <typename T, int K, int J, int MODE>
struct RowOps {
  using MI = ModeInfo<MODE>;
  static constexpr int C = J * 8;
  static constexpr int K2 = K / 2;
  static constexpr bool VREG = MI::needV && (C * K <= 64);
  static constexpr bool NEEDS = (MODE == XTWXV || MODE == XTXVY || MODE == XTPSXV || MODE == XTG ||
                                 MODE == XTSMG);

  f2 vreg[VREG ? C : 1][VREG ? K2 : 1];
  f2 acc[MI::accum ? C : 1][MI::accum ? K2 : 1];
  float ulast[MODE == XTSMG ? K : 1];   // XTSMG: U row of the last processed row (wave-uniform)
  const float* sV;
  int lane;

  // stage V (D x K, zero-padded to J*512 rows) in LDS, then the lane's slice in registers
  __device__ __forceinline__ void init(const float* __restrict__ V, int ldv, int D, float* smemV, int ln) {
    lane = ln;
    sV = smemV;
    constexpr int Dp = J * 512;
    if constexpr (MI::needV) {
      for (int i = threadIdx.x; i < Dp * K; i += BLOCK) {
        int d = i / K, k = i - d * K;
        smemV[i] = (d < D) ? V[(int64_t)d * ldv + k] : 0.f;
      }
      __syncthreads();
      if constexpr (VREG) {
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int kk = 0; kk < K2; ++kk) {
              const float* p = smemV + (((j * 64 + lane) * 8 + e) * K + 2 * kk);
              vreg[j * 8 + e][kk] = f2{p[0], p[1]};
            }
      }
    }
    if constexpr (MI::accum) {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) acc[c][kk] = f2{0.f, 0.f};
    }
  }

  // one row: cur = the lane's 8*J elements, sl = lane k's S[r][k]
  // XTSMG: out/ldo = the U output, kact = number of real (unpadded) columns
  __device__ __forceinline__ void process(const Raw8<T> (&cur)[J], const float sl, const int64_t r,
                                          const bool valid, float* __restrict__ out, int ldo, int kact = 0) {
    float x[C];
#pragma unroll
    for (int j = 0; j < J; ++j) unpack<float>(cur[j], x + j * 8);
    float sv[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
      sv[k] = NEEDS ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sl), k)) : 0.f;
    f2 g[K2];
    if constexpr (MI::needV) {
      // two partial sums per k pair: halves the dependent-FMA chain of the dot products
      f2 u0[K2], u1[K2];
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) { u0[kk] = f2{0.f, 0.f}; u1[kk] = f2{0.f, 0.f}; }
#pragma unroll
      for (int c = 0; c < C; ++c) {
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) {
          f2 vv;
          if constexpr (VREG) {
            vv = vreg[c][kk];
          } else {
            const float* pv = sV + ((((c >> 3) * 64 + lane) * 8 + (c & 7)) * K + 2 * kk);
            vv = f2{pv[0], pv[1]};
          }
          if (c & 1) u1[kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, vv, u1[kk]);
          else       u0[kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, vv, u0[kk]);
        }
      }
      float us[K];
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) {
        const f2 u = u0[kk] + u1[kk];
        us[2 * kk] = wave_sum(u.x);
        us[2 * kk + 1] = wave_sum(u.y);
      }
      if constexpr (MODE == XV) {
        if (valid) {
#pragma unroll
          for (int k = 0; k < K; ++k)
            if (lane == k) out[r * (int64_t)ldo + k] = us[k];
        }
        return;
      } else {
        float gs[K];
        if constexpr (MODE == XTXV) {
#pragma unroll
          for (int k = 0; k < K; ++k) gs[k] = us[k];
        } else if constexpr (MODE == XTWXV) {
#pragma unroll
          for (int k = 0; k < K; ++k) gs[k] = sv[k] * us[k];
        } else if constexpr (MODE == XTXVY) {
#pragma unroll
          for (int k = 0; k < K; ++k) gs[k] = us[k] - sv[k];
        } else if constexpr (MODE == XTPSXV) {
          float pr[K], q[K], sq = 0.f;
#pragma unroll
          for (int k = 0; k < K; ++k) { pr[k] = sv[k]; q[k] = pr[k] * us[k]; sq += q[k]; }
#pragma unroll
          for (int k = 0; k < K; ++k) gs[k] = q[k] - pr[k] * sq;
        } else if constexpr (MODE == XTSMG) {
          // softmax over [u_1..u_kact, 0] (the baseline class has linear term 0)
          float m = 0.f;
#pragma unroll
          for (int k = 0; k < K; ++k) m = (k < kact) ? fmaxf(m, us[k]) : m;
          float e[K], s = __expf(-m);
#pragma unroll
          for (int k = 0; k < K; ++k) { e[k] = (k < kact) ? __expf(us[k] - m) : 0.f; s += e[k]; }
          const float inv = 1.f / s;
#pragma unroll
          for (int k = 0; k < K; ++k) gs[k] = (k < kact) ? e[k] * inv - sv[k] : 0.f;
          // U is not stored here: the DMA front end batches the row outputs of a whole ring
          // round into one store (a per-row store would share vmcnt with the LDS-DMA ring)
#pragma unroll
          for (int k = 0; k < K; ++k) ulast[k] = us[k];
        }
#pragma unroll
        for (int kk = 0; kk < K2; ++kk)
          g[kk] = valid ? f2{gs[2 * kk], gs[2 * kk + 1]} : f2{0.f, 0.f};
      }
    } else {  // XTG
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) g[kk] = valid ? f2{sv[2 * kk], sv[2 * kk + 1]} : f2{0.f, 0.f};
    }
    if constexpr (MI::accum) {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int kk = 0; kk < K2; ++kk)
          acc[c][kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, g[kk], acc[c][kk]);
    }
  }

  // combine the 4 waves' accumulators through LDS (red: J*512*K floats), one partial per block
  __device__ __forceinline__ void reduce(float* red, int wave, float* __restrict__ out, int D) {
    if constexpr (MI::accum) {
      __syncthreads();
      for (int w = 0; w < WAVES; ++w) {
        if (wave == w) {
#pragma unroll
          for (int j = 0; j < J; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e)
#pragma unroll
              for (int kk = 0; kk < K2; ++kk) {
                int idx = ((j * 64 + lane) * 8 + e) * K + 2 * kk;
                f2 a = acc[j * 8 + e][kk];
                if (w == 0) { red[idx] = a.x; red[idx + 1] = a.y; }
                else { red[idx] += a.x; red[idx + 1] += a.y; }
              }
        }
        __syncthreads();
      }
      float* dst = out + (int64_t)blockIdx.x * D * K;
      for (int i = threadIdx.x; i < D * K; i += BLOCK) dst[i] = red[i];
    }
  }
};

// lane's clamped element offset of its 8-element chunk j (D % 8 == 0)
__device__ __forceinline__ int chunk_off(int j, int lane, int D) {
  const int c0 = (j * 64 + lane) * 8;
  return (c0 < D) ? c0 : D - 8;
}

// ---------------------------------------------------------------------------
// register-ring front end (XV)
// ---------------------------------------------------------------------------
template <typename T, int K, int J, int MODE, int R>
__global__ void __launch_bounds__(BLOCK)
rowstream_pk_kernel(const T* __restrict__ X, int64_t N, int D,
                    const float* __restrict__ V, int ldv,
                    const float* __restrict__ S, int lds, int sbc,
                    float* __restrict__ out, int ldo, int64_t rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using OPS = RowOps<T, K, J, MODE>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OPS ops;
  ops.init(V, ldv, D, reinterpret_cast<float*>(smem), lane);

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < N) ? r0 + rows_per_block : N;
  const int64_t rlast = r1 - 1;
  constexpr int STEP = WAVES * R;
  int coff[J];
#pragma unroll
  for (int j = 0; j < J; ++j) coff[j] = chunk_off(j, lane, D);
  const int scol = ((MODE == XTWXV || MODE == XTXVY) && sbc) ? 0 : (lane < K ? lane : K - 1);

  Raw8<T> ring[R][J];
  float sring[R];
  auto fetch = [&](Raw8<T> (&dst)[J], float& sdst, int64_t rr) {
    rr = (rr < rlast) ? rr : rlast;
    const T* row = X + rr * (int64_t)D;
#pragma unroll
    for (int j = 0; j < J; ++j) load_vec<T>(dst[j], row + coff[j]);
    if constexpr (OPS::NEEDS) {
      sdst = S[rr * (int64_t)lds + scol];
    } else {
      sdst = 0.f;
    }
  };
  int64_t base = r0 + wave;
#pragma unroll
  for (int p = 0; p < R; ++p) fetch(ring[p], sring[p], base + p * WAVES);

  for (; base < r1; base += STEP) {
#pragma unroll
    for (int p = 0; p < R; ++p) {
      const int64_t r = base + p * WAVES;   // wave-uniform
      Raw8<T> cur[J];
#pragma unroll
      for (int j = 0; j < J; ++j) cur[j] = ring[p][j];
      const float sl = sring[p];
      fetch(ring[p], sring[p], r + STEP);
      ops.process(cur, sl, r, r < r1, out, ldo);
    }
  }
  ops.reduce(reinterpret_cast<float*>(smem), wave, out, D);
}

// ---------------------------------------------------------------------------
// LDS-DMA front end (XTG and the fused chains)
// ---------------------------------------------------------------------------
template <typename T> struct DmaShape {
  static constexpr int PIECES = (int)sizeof(T) / 2;   // 16-B pieces per 8-element chunk
};

__device__ __forceinline__ uint4 lds_read_b128(uint32_t addr) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ void lds_read_row_bf16(Raw8<uint16_t> (&cur)[1], float& s, uint32_t xa, uint32_t sa) {
  uint4 v;
  uint32_t t;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(v), "=&v"(t) : "v"(xa), "v"(sa) : "memory");
  cur[0].v = v;
  s = __uint_as_float(t);
}
__device__ __forceinline__ void lds_read_row_bf16(Raw8<uint16_t> (&cur)[2], float& s, uint32_t xa, uint32_t sa) {
  uint4 v0, v1;
  uint32_t t;
  asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:1024\n\tds_read_b32 %2, %4\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(v0), "=&v"(v1), "=&v"(t) : "v"(xa), "v"(sa) : "memory");
  cur[0].v = v0;
  cur[1].v = v1;
  s = __uint_as_float(t);
}
template <int J>
__device__ __forceinline__ void lds_read_row_f32(Raw8<float> (&cur)[J], float& s, uint32_t xa, uint32_t sa) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint4 a = lds_read_b128(xa + (2 * j) * 1024);
    const uint4 b = lds_read_b128(xa + (2 * j + 1) * 1024);
    cur[j].v[0] = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
    cur[j].v[1] = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w));
  }
  uint32_t t;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(t) : "v"(sa) : "memory");
  s = __uint_as_float(t);
}

template <int N> __device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// LDS bytes of the DMA front end: reduction / V region + WAVES rings of R slots
template <typename T, int K, int J, int R>
constexpr size_t dma_lds_bytes() {
  return (size_t)J * 512 * K * 4 + (size_t)WAVES * R * (J * DmaShape<T>::PIECES * 1024 + 256);
}

template <typename T, int K, int J, int MODE, int R>
__global__ void __launch_bounds__(BLOCK)
rowstream_dma_kernel(const T* __restrict__ X, int64_t N, int D,
                     const float* __restrict__ V, int ldv,
                     const float* __restrict__ S, int lds, int sbc,
                     float* __restrict__ out, int64_t rows_per_block,
                     float* __restrict__ uout, int ldu) {
  static_assert(MODE != XV, "row-output mode uses the register-ring front end");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using OPS = RowOps<T, K, J, MODE>;
  constexpr int PIECES = DmaShape<T>::PIECES;
  constexpr int XB = J * PIECES * 1024;       // X bytes of one slot (lane-linear 16-B pieces)
  constexpr int SLOT = XB + 256;              // + S: 64 lanes x 4 B
  constexpr int NPR = J * PIECES + (OPS::NEEDS ? 1 : 0);   // LDS-DMA instructions per row
  constexpr int STEP = WAVES * R;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OPS ops;
  ops.init(V, ldv, D, reinterpret_cast<float*>(smem), lane);

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < N) ? r0 + rows_per_block : N;
  const int64_t rlast = r1 - 1;
  int coff[J];
#pragma unroll
  for (int j = 0; j < J; ++j) coff[j] = chunk_off(j, lane, D);
  int scol = ((MODE == XTWXV || MODE == XTXVY) && sbc) ? 0 : (lane < K ? lane : K - 1);
  if constexpr (MODE == XTSMG) scol = lane < sbc ? lane : sbc - 1;   // Y has only kact columns

  const int ring_off = J * 512 * K * 4 + wave * (R * SLOT);
  lds_char* ring = (lds_char*)(smem) + ring_off;
  const uint32_t ring_addr = (uint32_t)(uintptr_t)ring;

  auto fetch = [&](int slot, int64_t rr) {
    rr = (rr < rlast) ? rr : rlast;
    const T* row = X + rr * (int64_t)D;
    lds_char* sb = ring + slot * SLOT;
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int h = 0; h < PIECES; ++h)
        __builtin_amdgcn_global_load_lds((const void*)(row + coff[j] + h * (8 / PIECES)),
                                         (void __attribute__((address_space(3)))*)(sb + (j * PIECES + h) * 1024),
                                         16, 0, SYSML_X_AUX);
    if constexpr (OPS::NEEDS)
      __builtin_amdgcn_global_load_lds((const void*)(S + rr * (int64_t)lds + scol),
                                       (void __attribute__((address_space(3)))*)(sb + XB), 4, 0, 0);
  };

  int64_t base = r0 + wave;
#pragma unroll
  for (int p = 0; p < R; ++p) fetch(p, base + p * WAVES);

  // XTSMG: lane p*K + k collects U[row of slot p][k] over a ring round; one store per round
  // (to U's pad row N for lanes without a valid cell, so it is never skipped).  Invariant for
  // the counted wait: exactly one store is younger than the loads of the slot being waited
  // on, hence the dummy store after the prologue.
  constexpr bool SMG = (MODE == XTSMG);
  constexpr int NST = SMG ? 1 : 0;
  float ureg = 0.f;
  float* const upad = uout + N * (int64_t)ldu;
  if constexpr (SMG) *upad = 0.f;

  for (; base < r1; base += STEP) {
#pragma unroll
    for (int p = 0; p < R; ++p) {
      const int64_t r = base + p * WAVES;   // wave-uniform
      wait_vmcnt<(R - 1) * NPR + NST>();    // slot p landed; R-1 rows stay in flight
      Raw8<T> cur[J];
      float sl;
      const uint32_t xa = ring_addr + p * SLOT + lane * 16;
      const uint32_t sa = ring_addr + p * SLOT + XB + lane * 4;
      if constexpr (sizeof(T) == 2) {
        lds_read_row_bf16(cur, sl, xa, sa);
      } else {
        lds_read_row_f32<J>(cur, sl, xa, sa);
      }
      if constexpr (!OPS::NEEDS) sl = 0.f;
      fetch(p, r + STEP);                   // refill the slot (its LDS reads have retired)
      ops.process(cur, sl, r, r < r1, uout, ldu, sbc);
      if constexpr (SMG) {
#pragma unroll
        for (int k = 0; k < K; ++k) ureg = (lane == p * K + k) ? ops.ulast[k] : ureg;
      }
    }
    if constexpr (SMG) {
      const int sl_ = lane / K, kl = lane - (lane / K) * K;
      const int64_t row = base + (int64_t)sl_ * WAVES;
      const bool ok = (lane < R * K) && (kl < sbc) && (row < r1);
      float* dst = ok ? uout + row * (int64_t)ldu + kl : upad;
      *dst = ureg;
    }
  }
  wait_vmcnt<0>();                          // no LDS-DMA may outlive the block's LDS
  ops.reduce(reinterpret_cast<float*>(smem), wave, out, D);
}

}  // namespace sysml

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
using namespace sysml;

static int g_rows_per_iter = 0;   // 0 = auto, else rows per iteration (generic) / prefetch depth (pk)
static int g_variant = 0;         // 0 = auto (packed fp32 where applicable), 1 = generic scalar kernel
static float* g_uout = nullptr;   // XTSMG: row output U (set by sysml_rowstream_smg around the launch)
static int g_ldu = 0;

// dynamic LDS above 64 KiB must be allowed per kernel (once)
static void allow_lds(const void* fn, size_t bytes) {
  static std::unordered_set<const void*> done;
  if (bytes <= 65536 || done.count(fn)) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  done.insert(fn);
}

template <typename T, typename A, int K, int J, int MODE>
static int launch_t(const void* X, int64_t N, int D, int vec, const void* V, int ldv, const void* S,
                    int lds, int sbc, void* out, int ldo, int grid, int64_t rpb, hipStream_t st) {
  using MI = ModeInfo<MODE>;
  if constexpr (sizeof(A) == 8 && K == 8 && J == 2 && MODE >= XTXV && MODE <= XTPSXV) {
    return -1;  // fp64 x 8 columns x 1024 cols would spill: caller falls back to XV + XTG passes
  } else if constexpr (MODE == XTSMG && (sizeof(A) != 4 || K < 2 || K > 4)) {
    return -1;  // fused softmax gradient: packed-fp32 LDS-DMA kernel only (caller runs it unfused)
  } else {
  constexpr int KO = (MODE == COLSSQ || MODE == COLSUM) ? 1 : K;
  size_t shv = MI::needV ? (size_t)J * 512 * K * sizeof(A) : 0;
  size_t shr = MI::accum ? (size_t)J * 512 * KO * sizeof(A) : 0;
  size_t sh = shv > shr ? shv : shr;
  const bool two = (g_rows_per_iter == 2) ||
                   (g_rows_per_iter == 0 && sizeof(A) == 4 && (MODE == XV || MODE == XTXV || MODE == ROWSSQ ||
                                                               MODE == ROWSUM || (K == 1 && MI::accum)));
  if constexpr (sizeof(A) == 4 && K >= 2 && (MODE <= XTPSXV || MODE == XTSMG)) {
    if (g_variant != 1 && vec && (D % 8) == 0) {   // packed-fp32 kernels (vector rows only)
      // rows in flight per wave: knob (1-2 -> 2, 3+ -> 4), else bf16 4 / fp32 2 (same bytes)
      const int knob = g_rows_per_iter;
      const bool deep = knob ? (knob > 2) : (sizeof(T) == 2);
      if constexpr (MODE == XV) {
#define SYSML_PK(PF) hipLaunchKernelGGL((rowstream_pk_kernel<T, K, J, MODE, PF>), dim3(grid), dim3(BLOCK), sh, st, \
          (const T*)X, N, D, (const float*)V, ldv, (const float*)S, lds, sbc, (float*)out, ldo, rpb)
        if (deep) SYSML_PK(4); else SYSML_PK(2);
#undef SYSML_PK
      } else {
        // LDS-DMA ring depth R (rows in flight per wave).  The ring is LDS, so R costs no
        // VGPRs; what bounds it is the LDS of the co-resident blocks.  The K >= 4 kernels run 2
        // waves/SIMD (XTSMG 1) by VGPRs, so they get deeper rings to keep ~96 KiB of X in
        // flight per CU (profiles/rowstream_ring_depth_r2.txt); narrower modes are LDS-limited
        // at R = 4 (bf16) / 2 (fp32) with 3 blocks per CU.
        int R = deep ? 4 : 2;
        if (!knob) {
          if (MODE == XTSMG) R = sizeof(T) == 2 ? 12 : 6;
          else if (K >= 4) R = sizeof(T) == 2 ? 6 : 3;
        }
#define SYSML_DMA(PF) do { \
          auto kfn = rowstream_dma_kernel<T, K, J, MODE, PF>; \
          const size_t shb = dma_lds_bytes<T, K, J, PF>(); \
          allow_lds(reinterpret_cast<const void*>(kfn), shb); \
          hipLaunchKernelGGL(kfn, dim3(grid), dim3(BLOCK), shb, st, (const T*)X, N, D, \
                             (const float*)V, ldv, (const float*)S, lds, sbc, (float*)out, rpb, g_uout, g_ldu); \
        } while (0)
        if constexpr (MODE == XTSMG) {
          if constexpr (sizeof(T) == 2) { if (R == 12) SYSML_DMA(12); else if (R == 4) SYSML_DMA(4); else SYSML_DMA(2); }
          else { if (R == 6) SYSML_DMA(6); else if (R == 4) SYSML_DMA(4); else SYSML_DMA(2); }
        } else if constexpr (K >= 4) {
          if constexpr (sizeof(T) == 2) { if (R == 6) SYSML_DMA(6); else if (R == 4) SYSML_DMA(4); else SYSML_DMA(2); }
          else { if (R == 3) SYSML_DMA(3); else if (R == 4) SYSML_DMA(4); else SYSML_DMA(2); }
        } else {
          if (R == 4) SYSML_DMA(4); else SYSML_DMA(2);
        }
#undef SYSML_DMA
      }
      return hipGetLastError() == hipSuccess ? 0 : -2;
    }
  }
  if constexpr (MODE == XTSMG) {
    return -1;  // no generic-kernel variant of the two-output mode
  } else {
  if (sizeof(A) == 4 && K <= 4 && two) {
    hipLaunchKernelGGL((rowstream_kernel<T, A, K, J, MODE, 2>), dim3(grid), dim3(BLOCK), sh, st,
                       (const T*)X, N, D, vec, (const A*)V, ldv, (const A*)S, lds, sbc, (A*)out, ldo, rpb);
  } else {
    hipLaunchKernelGGL((rowstream_kernel<T, A, K, J, MODE, 1>), dim3(grid), dim3(BLOCK), sh, st,
                       (const T*)X, N, D, vec, (const A*)V, ldv, (const A*)S, lds, sbc, (A*)out, ldo, rpb);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  }
}

template <typename T, typename A, int J, int MODE>
static int launch_k(int K, const void* X, int64_t N, int D, int vec, const void* V, int ldv, const void* S,
                    int lds, int sbc, void* out, int ldo, int grid, int64_t rpb, hipStream_t st) {
  switch (K) {
    case 1: return launch_t<T, A, 1, J, MODE>(X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    case 2: return launch_t<T, A, 2, J, MODE>(X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    case 4: return launch_t<T, A, 4, J, MODE>(X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    case 8: return launch_t<T, A, 8, J, MODE>(X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    default: return -1;
  }
}

template <typename T, typename A, int MODE>
static int launch_j(int J, int K, const void* X, int64_t N, int D, int vec, const void* V, int ldv,
                    const void* S, int lds, int sbc, void* out, int ldo, int grid, int64_t rpb, hipStream_t st) {
  if (J == 1) return launch_k<T, A, 1, MODE>(K, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
  if (J == 2) return launch_k<T, A, 2, MODE>(K, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
  return -1;
}

template <typename T, typename A>
static int launch_mode(int mode, int J, int K, const void* X, int64_t N, int D, int vec, const void* V,
                       int ldv, const void* S, int lds, int sbc, void* out, int ldo, int grid, int64_t rpb,
                       hipStream_t st) {
#define SYSML_CASE(M) case M: return launch_j<T, A, M>(J, K, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
  switch (mode) {
    SYSML_CASE(XV) SYSML_CASE(XTG) SYSML_CASE(XTXV) SYSML_CASE(XTWXV) SYSML_CASE(XTXVY) SYSML_CASE(XTPSXV)
    default: break;
  }
#undef SYSML_CASE
  if (K != 1) return -1;
  switch (mode) {
    case ROWSSQ: return launch_j<T, A, ROWSSQ>(J, 1, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    case COLSSQ: return launch_j<T, A, COLSSQ>(J, 1, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    case COLSUM: return launch_j<T, A, COLSUM>(J, 1, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    case ROWSUM: return launch_j<T, A, ROWSUM>(J, 1, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid, rpb, st);
    default: return -1;
  }
}

extern "C" {

// xdtype: 0 = bf16 (fp32 accumulate), 1 = fp32, 2 = fp64.   Returns 0 on success.
int sysml_rowstream(int mode, int xdtype, const void* X, int64_t N, int D, const void* V, int ldv,
                    const void* S, int lds, int sbc, void* out, int ldo, int K, int grid,
                    int64_t rows_per_block, void* stream) {
  if (D <= 0 || D > 1024 || N <= 0 || grid <= 0) return -1;
  const int J = (D <= 512) ? 1 : 2;
  hipStream_t st = (hipStream_t)stream;
  int vec;
  if (xdtype == 0) {
    vec = ((D % 8) == 0 && (((uintptr_t)X) & 15) == 0) ? 1 : 0;
    return launch_mode<uint16_t, float>(mode, J, K, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid,
                                        rows_per_block, st);
  }
  if (xdtype == 1) {
    vec = ((D % 4) == 0 && (((uintptr_t)X) & 15) == 0) ? 1 : 0;
    return launch_mode<float, float>(mode, J, K, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid,
                                     rows_per_block, st);
  }
  if (xdtype == 2) {
    vec = ((D % 2) == 0 && (((uintptr_t)X) & 15) == 0) ? 1 : 0;
    return launch_mode<double, double>(mode, J, K, X, N, D, vec, V, ldv, S, lds, sbc, out, ldo, grid,
                                       rows_per_block, st);
  }
  return -1;
}

// Fused multinomial-logreg candidate evaluation (mode XTSMG): U = X %*% V (N x kact, written; U
// must have N + 1 rows: row N is a scratch pad the kernel stores into
// to U with leading dimension ldu) and partial[grid][D x K] of t(X) %*% (softmax([U,0])[,1:kact]
// - Y[,1:kact]) in one pass over X.  V is D x K (K = kact padded to 2 or 4, zero columns),
// Y is N x >= kact (leading dimension ldy).  bf16 / fp32 X only.  Returns 0 on success.
int sysml_rowstream_smg(int xdtype, const void* X, int64_t N, int D, const void* V, int ldv,
                        const void* Y, int ldy, int kact, void* U, int ldu, void* partial, int K,
                        int grid, int64_t rows_per_block, void* stream) {
  if (D <= 0 || D > 1024 || N <= 0 || grid <= 0 || kact < 1 || kact > K || (xdtype != 0 && xdtype != 1))
    return -1;
  const int J = (D <= 512) ? 1 : 2;
  const int align = xdtype == 0 ? 8 : 4;
  const int vec = ((D % align) == 0 && (((uintptr_t)X) & 15) == 0) ? 1 : 0;
  g_uout = (float*)U;
  g_ldu = ldu;
  int rc;
  if (xdtype == 0)
    rc = launch_j<uint16_t, float, XTSMG>(J, K, X, N, D, vec, V, ldv, Y, ldy, kact, partial, 0, grid,
                                          rows_per_block, (hipStream_t)stream);
  else
    rc = launch_j<float, float, XTSMG>(J, K, X, N, D, vec, V, ldv, Y, ldy, kact, partial, 0, grid,
                                       rows_per_block, (hipStream_t)stream);
  g_uout = nullptr;
  g_ldu = 0;
  return rc;
}

int sysml_abi_version() { return 3; }

// tuning knob for A/B runs: 0 = automatic, 1 or 2 rows per wave iteration
void sysml_set_rows_per_iter(int r) { g_rows_per_iter = r; }
void sysml_set_variant(int v) { g_variant = v; }

}  // extern "C"
