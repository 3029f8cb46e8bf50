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
#include <stdint.h>

namespace sysml {

enum Mode { XV = 0, XTG = 1, XTXV = 2, XTWXV = 3, XTXVY = 4, XTPSXV = 5,
            ROWSSQ = 6, COLSSQ = 7, COLSUM = 8, ROWSUM = 9 };

constexpr int WAVES = 4;
constexpr int BLOCK = 64 * WAVES;

template <int M> struct ModeInfo {
  static constexpr bool needV   = (M == XV || M == XTXV || M == XTWXV || M == XTXVY || M == XTPSXV);
  static constexpr bool accum   = (M == XTG || M == XTXV || M == XTWXV || M == XTXVY || M == XTPSXV ||
                                   M == COLSSQ || M == COLSUM);
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

template <>
__device__ __forceinline__ void load_raw<uint16_t>(Raw8<uint16_t>& r, const uint16_t* __restrict__ row,
                                                   int c0, int D, bool vec) {
  if (vec && c0 + 8 <= D) {
    r.v = *reinterpret_cast<const uint4*>(row + c0);
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
// Packed-fp32 variant for K in {2,4,8} (fp32 accumulate: bf16 / fp32 X).
// The k dimension is carried in float2 pairs so every dot-product / accumulate
// FMA is a v_pk_fma_f32 (2 FMAs per lane per instruction), and for C*K <= 64 the
// lane's slice of V lives in registers for the whole launch (no per-row LDS
// traffic).  Row-side values (g) are wave-uniform after the DPP reduction.
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

template <typename T, int K, int J, int MODE, int R>
__global__ void __launch_bounds__(BLOCK)
rowstream_pk_kernel(const T* __restrict__ X, int64_t N, int D, int vec,
                    const float* __restrict__ V, int ldv,
                    const float* __restrict__ S, int lds, int sbc,
                    float* __restrict__ out, int ldo, int64_t rows_per_block) {
  using MI = ModeInfo<MODE>;
  constexpr int C = J * 8;
  constexpr int K2 = K / 2;
  constexpr bool VREG = MI::needV && (C * K <= 64);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sV = reinterpret_cast<float*>(smem);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Dp = J * 512;

  f2 vreg[VREG ? C : 1][VREG ? K2 : 1];
  if constexpr (MI::needV) {
    for (int i = threadIdx.x; i < Dp * K; i += BLOCK) {
      int d = i / K, k = i - d * K;
      sV[i] = (d < D) ? V[(int64_t)d * ldv + k] : 0.f;
    }
    __syncthreads();
    if constexpr (VREG) {
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int kk = 0; kk < K2; ++kk) {
            const float* p = sV + (((j * 64 + lane) * 8 + e) * K + 2 * kk);
            vreg[j * 8 + e][kk] = f2{p[0], p[1]};
          }
    }
  }

  f2 acc[MI::accum ? C : 1][MI::accum ? K2 : 1];
  if constexpr (MI::accum) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) acc[c][kk] = f2{0.f, 0.f};
  }

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < N) ? r0 + rows_per_block : N;
  // R = prefetch depth: each wave keeps R of its future rows in flight (packed, so a
  // prefetched bf16 row costs 4*J VGPRs) while it processes one row; deeper rings put
  // more bytes in flight per SIMD (Little's law at ~6 TB/s needs ~10 MB chip-wide).
  constexpr int STEP = WAVES * R;

  // row-side operand (weights / targets / probabilities / g) for the same rows rides in
  // the ring too, so its (wave-uniform) load latency is hidden behind R-1 rows of work
  constexpr bool NEEDS = (MODE == XTWXV || MODE == XTXVY || MODE == XTPSXV || MODE == XTG);
  constexpr int KS = NEEDS ? K : 1;
  Raw8<T> ring[R][J];
  float sring[R][KS];
  auto load_s = [&](float (&dst)[KS], const int64_t rr) {
    if constexpr (NEEDS) {
#pragma unroll
      for (int k = 0; k < K; ++k) dst[k] = S[rr * (int64_t)lds + (((MODE == XTWXV || MODE == XTXVY) && sbc) ? 0 : k)];
    }
  };
  int64_t base = r0 + wave;
#pragma unroll
  for (int p = 0; p < R; ++p) {
    const int64_t rp = base + p * WAVES;
    if (rp < r1) {
#pragma unroll
      for (int j = 0; j < J; ++j) load_raw<T>(ring[p][j], X + rp * (int64_t)D, (j * 64 + lane) * 8, D, vec);
      load_s(sring[p], rp);
    }
  }

  auto process = [&](const Raw8<T> (&cur)[J], const float (&sv)[KS], const int64_t r) {
    float x[C];
#pragma unroll
    for (int j = 0; j < J; ++j) unpack<float>(cur[j], x + j * 8);
    f2 g[K2];
    if constexpr (MI::needV) {
      f2 u[K2];
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) u[kk] = f2{0.f, 0.f};
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
          u[kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, vv, u[kk]);
        }
      }
      float us[K];
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) {
        us[2 * kk] = wave_sum(u[kk].x);
        us[2 * kk + 1] = wave_sum(u[kk].y);
      }
      if constexpr (MODE == XV) {
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (lane == k) out[r * (int64_t)ldo + k] = us[k];
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
        }
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) g[kk] = f2{gs[2 * kk], gs[2 * kk + 1]};
      }
    } else {  // XTG
#pragma unroll
      for (int kk = 0; kk < K2; ++kk) g[kk] = f2{sv[2 * kk], sv[2 * kk + 1]};
    }
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int kk = 0; kk < K2; ++kk)
        acc[c][kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, g[kk], acc[c][kk]);
  };

  for (; base < r1; base += STEP) {
#pragma unroll
    for (int p = 0; p < R; ++p) {
      const int64_t r = base + p * WAVES;   // wave-uniform
      if (r < r1) {
        Raw8<T> cur[J];
#pragma unroll
        for (int j = 0; j < J; ++j) cur[j] = ring[p][j];
        float sv[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) sv[k] = sring[p][k];
        const int64_t rn = r + STEP;
        if (rn < r1) {
#pragma unroll
          for (int j = 0; j < J; ++j) load_raw<T>(ring[p][j], X + rn * (int64_t)D, (j * 64 + lane) * 8, D, vec);
          load_s(sring[p], rn);
        }
        process(cur, sv, r);
      }
    }
  }

  if constexpr (MI::accum) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
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

}  // namespace sysml

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
using namespace sysml;

static int g_rows_per_iter = 0;   // 0 = auto, else rows per iteration (generic) / prefetch depth (pk)
#ifndef PF_DEFAULT_BF16
#define PF_DEFAULT_BF16 4
#endif
#ifndef PF_DEFAULT_F32
#define PF_DEFAULT_F32 1
#endif
static int g_variant = 0;         // 0 = auto (packed fp32 where applicable), 1 = generic scalar kernel

template <typename T, typename A, int K, int J, int MODE>
static int launch_t(const void* X, int64_t N, int D, int vec, const void* V, int ldv, const void* S,
                    int lds, int sbc, void* out, int ldo, int grid, int64_t rpb, hipStream_t st) {
  using MI = ModeInfo<MODE>;
  if constexpr (sizeof(A) == 8 && K == 8 && J == 2 && MODE >= XTXV && MODE <= XTPSXV) {
    return -1;  // fp64 x 8 columns x 1024 cols would spill: caller falls back to XV + XTG passes
  } else {
  constexpr int KO = (MODE == COLSSQ || MODE == COLSUM) ? 1 : K;
  size_t shv = MI::needV ? (size_t)J * 512 * K * sizeof(A) : 0;
  size_t shr = MI::accum ? (size_t)J * 512 * KO * sizeof(A) : 0;
  size_t sh = shv > shr ? shv : shr;
  const bool two = (g_rows_per_iter == 2) ||
                   (g_rows_per_iter == 0 && sizeof(A) == 4 && (MODE == XV || MODE == XTXV || MODE == ROWSSQ ||
                                                               MODE == ROWSUM || (K == 1 && MI::accum)));
  if constexpr (sizeof(A) == 4 && K >= 2 && MODE <= XTPSXV) {
    if (g_variant != 1) {   // packed-fp32 kernel (default)
      // prefetch-ring depth: knob 1..4, else tuned default (bf16 rows are half the bytes,
      // so they need twice the rows in flight for the same HBM occupancy)
      // measured (profiles/rowstream_kbench_r1_prefetch.txt): bf16 chains like 4 rows in
      // flight per wave, bf16 XV / XTG 3; fp32 rows are twice the bytes, 1 suffices
      int depth = g_rows_per_iter ? g_rows_per_iter
                                  : (sizeof(T) == 2 ? ((MODE == XV || MODE == XTG) ? 3 : PF_DEFAULT_BF16)
                                                    : PF_DEFAULT_F32);
#define SYSML_PK(PF) hipLaunchKernelGGL((rowstream_pk_kernel<T, K, J, MODE, PF>), dim3(grid), dim3(BLOCK), sh, st, \
          (const T*)X, N, D, vec, (const float*)V, ldv, (const float*)S, lds, sbc, (float*)out, ldo, rpb)
      switch (depth) {
        case 1: SYSML_PK(1); break;
        case 2: SYSML_PK(2); break;
        case 3: SYSML_PK(3); break;
        default: SYSML_PK(4); break;
      }
#undef SYSML_PK
      return hipGetLastError() == hipSuccess ? 0 : -2;
    }
  }
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

int sysml_abi_version() { return 2; }

// tuning knob for A/B runs: 0 = automatic, 1 or 2 rows per wave iteration
void sysml_set_rows_per_iter(int r) { g_rows_per_iter = r; }
void sysml_set_variant(int v) { g_variant = v; }

}  // extern "C"
