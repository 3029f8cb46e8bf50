// Fused tall-skinny matrix-chain kernels on the CDNA4 matrix cores (gfx950).
//
// Reference semantics: runtime/matrix/data/LibMatrixMult.matrixMultChain (XtXv, XtwXv,
// XtXvy) and the MultiLogReg inner-loop chain t(X) %*% (P[,1:K] * (X %*% V) - P[,1:K] *
// rowSums(P[,1:K] * (X %*% V)))  (scripts/algorithms/MultiLogReg.dml); plus plain
// X %*% V and t(X) %*% G for skinny V / G.  The reference runs these on the CPU
// (multi-threaded row blocks) or cuBLAS; here one kernel streams X from HBM exactly once.
//
// Design (one 512-thread block = 8 wave64, X in bf16, everything accumulated in fp32):
//   * X is staged through LDS in 16-row tiles (register staging: the NEXT tile's global
//     loads are issued before the current tile is computed, so HBM latency hides behind
//     two MFMA phases).  LDS row pitch = 2*Dp + 16 bytes -> conflict-free row reads.
//   * phase 1  U^T = V3^T * X^T  on v_mfma_f32_16x16x32_bf16.  V is split on the host into
//     three bf16 planes (hi, lo, lo2 = successive rounding residuals) stacked in the 16-row
//     M dimension (K <= 4 columns -> rows 4s+k), so a bf16 MFMA delivers ~fp32-accurate
//     X*V (X itself is exact bf16).  Each wave owns a Dp/8 column slice; the eight partial
//     16x16 tiles are summed through LDS.
//   * row epilogue (per mode) in fp32: G = U | w.*U | U-y | P.*U - P.*rowSums(P.*U) | given.
//   * phase 2  out[d][k'] += X^T[d][r] * G3[r][k']  on v_mfma_f32_16x16x16_bf16, with X^T
//     read straight from the same LDS tile by ds_read_b64_tr_b16 (hardware transpose) and
//     G again split hi/lo/lo2 into the N dimension.  Accumulators live in VGPRs/AGPRs for
//     the wave's whole row range; per-block partials are reduced by a tiny torch sum.
// This removes every cross-lane DPP reduction of the VALU row-streaming kernel (which was
// instruction-issue bound at ~3.9 TB/s for K=4) and leaves HBM as the only limiter.
#include <hip/hip_runtime.h>
#include <stdint.h>

const double* sysml_live_flag();   // chain4.hip: run-ahead flag of the calling host thread

// run-ahead live flag (see chain4.hip sysml_set_live): true when the queued iteration is dead
__device__ __forceinline__ bool sysml_dead(const double* live) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(live);
  if (a == 0) return false;
  const double f = *reinterpret_cast<const double*>(a & ~(uintptr_t)1);
  return (f == 0.0) != ((a & 1) != 0);
}

namespace sysml_mc {

typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

enum Mode { XV = 0, XTG = 1, XTXV = 2, XTWXV = 3, XTXVY = 4, XTPSXV = 5,  // = rowstream.hip
            XTSMG = 10, XTSMGO = 11 };                                      // = chain4.hip (wide kernel only)

constexpr int WAVES = 8;
constexpr int BLOCK = 64 * WAVES;
constexpr int MIN_WAVES_PER_SIMD = 4;   // <= 128 VGPR+AGPR: two blocks (16 waves) per CU
constexpr int TR = 16;  // rows per tile

__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ s4 tr_read(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p));
}

template <int MODE, int KS>
__global__ void __launch_bounds__(BLOCK, MIN_WAVES_PER_SIMD)
mchain_kernel(const uint16_t* __restrict__ X, int64_t N, int D,
              const uint16_t* __restrict__ V3T,  // [16][Dp] bf16 (row 4s+k = plane s of V[:,k])
              const float* __restrict__ S, int lds, int sbc, int K,
              float* __restrict__ out, int ldo, int64_t tiles_per_block, const double* __restrict__ live) {
  if (sysml_dead(live)) return;    // dead run-ahead iteration (runtime/program.py)
  constexpr int Dp = KS * 32 * WAVES;   // KS = 32-column k-steps per wave
  constexpr int ROWB = Dp * 2 + 16;      // LDS pitch of one X row (bytes)
  constexpr int CH = Dp / 8;             // 16-byte chunks per row
  constexpr int NST = TR * CH / BLOCK;   // staging chunks per thread (= KS)
  constexpr int NB = KS * 2;             // 16-column d-blocks per wave (phase 2)
  static_assert(Dp / WAVES == 32 * KS, "wave slice = KS k-steps");
  constexpr bool P1 = (MODE != XTG);
  constexpr bool P2 = (MODE != XV);
  static_assert(NST * BLOCK == TR * CH, "tile must split evenly over the block");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Xs = smem;
  float* Ured = reinterpret_cast<float*>(smem + TR * ROWB);            // [WAVES][TR][16]
  uint16_t* G3 = reinterpret_cast<uint16_t*>(Ured + WAVES * TR * 16);  // [WAVES][TR][16]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;     // 16-lane group
  const int i16 = lane & 15;
  const int q = i16 >> 2, p = i16 & 3;
  const int dsl = wave * (Dp / WAVES);

  bf8 afr[P1 ? KS : 1];
  if constexpr (P1) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      afr[ks] = *reinterpret_cast<const bf8*>(V3T + (int64_t)i16 * Dp + dsl + ks * 32 + 8 * g);
  }
  f4 acc[P2 ? NB : 1];
#pragma unroll
  for (int b = 0; b < (P2 ? NB : 1); ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};

  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_block;
  const int64_t t1 = (t0 + tiles_per_block < ntiles) ? t0 + tiles_per_block : ntiles;

  // staging: loads are unconditional (out-of-range chunks re-read a valid address) and the
  // zero-fill is applied at LDS-write time, so no branch sits between a load and its use
  // and the waitcnt pass can keep the next tile's loads in flight through both MFMA phases.
  u4 st[NST];
  uint32_t stok = 0;
  auto gload = [&](int64_t t) {
    stok = 0;
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int id = j * BLOCK + tid;
      const int row = id / CH, ch = id - (id / CH) * CH;
      const int64_t r = t * TR + row;
      const bool ok = (r < N) && (ch * 8 < D);
      stok |= (ok ? 1u : 0u) << j;
      const int64_t off = ok ? r * (int64_t)D + ch * 8 : 0;
      st[j] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(X + off));
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int id = j * BLOCK + tid;
      const int row = id / CH, ch = id - (id / CH) * CH;
      const u4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u4*>(Xs + row * ROWB + ch * 16) = ((stok >> j) & 1u) ? st[j] : z;
    }
  };
  // row-side operand of this lane's (row i16, column g) for a tile
  auto sload = [&](int64_t t, float (&sv)[2]) {
    const int64_t r = t * TR + i16;
    sv[0] = sv[1] = 0.f;
    const bool ok = (r < N) && (g < K);
    const int64_t off = ok ? r * (int64_t)lds + (((MODE == XTWXV || MODE == XTXVY) && sbc) ? 0 : g) : 0;
    if constexpr (MODE == XTWXV || MODE == XTXVY || MODE == XTPSXV || MODE == XTG) sv[0] = S[off];
  };

  if (t0 < t1) {
    gload(t0);
    swrite();
  }
  __builtin_amdgcn_s_waitcnt(0);   // V fragments + first tile retired before the pipelined loop
  __syncthreads();

  for (int64_t t = t0; t < t1; ++t) {
    float sv[2];
    sload(t, sv);
    if (t + 1 < t1) gload(t + 1);
    const int64_t r = t * TR + i16;
    const bool ok = (r < N) && (g < K);

    float gval = 0.f;
    if constexpr (P1) {
      f4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf8 b = *reinterpret_cast<const bf8*>(Xs + i16 * ROWB + (dsl + ks * 32 + 8 * g) * 2);
        u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[ks], b, u, 0, 0, 0);
      }
      // u[i] = partial U^T[k' = 4g+i][row i16]
      *reinterpret_cast<f4*>(Ured + (wave * TR + i16) * 16 + 4 * g) = u;
      __syncthreads();
      float uu = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w)
#pragma unroll
        for (int s = 0; s < 3; ++s) uu += Ured[(w * TR + i16) * 16 + 4 * s + g];
      if constexpr (MODE == XV) {
        if (ok) out[r * (int64_t)ldo + g] = uu;
      } else if constexpr (MODE == XTXV) {
        gval = uu;
      } else if constexpr (MODE == XTWXV) {
        gval = sv[0] * uu;
      } else if constexpr (MODE == XTXVY) {
        gval = uu - sv[0];
      } else if constexpr (MODE == XTPSXV) {
        const float qv = sv[0] * uu;
        float sq = qv + __shfl_xor(qv, 16);
        sq += __shfl_xor(sq, 32);
        gval = qv - sv[0] * sq;
      }
    } else {
      gval = sv[0];
    }
    if (!ok) gval = 0.f;

    if constexpr (P2) {
      uint16_t* Gw = G3 + wave * TR * 16;
      const uint16_t h = f2bf(gval);
      float rem = gval - bf2f(h);
      const uint16_t l1 = f2bf(rem);
      rem -= bf2f(l1);
      const uint16_t l2 = f2bf(rem);
      Gw[i16 * 16 + g] = h;
      Gw[i16 * 16 + 4 + g] = l1;
      Gw[i16 * 16 + 8 + g] = l2;
      Gw[i16 * 16 + 12 + g] = 0;
      __syncthreads();
      const s4 bfr = tr_read(Gw + (4 * g + q) * 16 + 4 * p);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int dblk = dsl + b * 16;
        const s4 a = tr_read(Xs + (4 * g + q) * ROWB + (dblk + 4 * p) * 2);
        acc[b] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bfr, acc[b], 0, 0, 0);
      }
    }
    __syncthreads();
    if (t + 1 < t1) {
      swrite();
      __syncthreads();
    }
  }

  if constexpr (P2) {
    // acc[b][i] = out[d = dsl + 16b + 4g + i][k' = i16]; fold the three bf16 planes of G
    float* dst = out + (int64_t)blockIdx.x * D * K;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[b][i];
        v += __shfl_down(v, 4) + __shfl_down(v, 8);
        const int d = dsl + b * 16 + 4 * g + i;
        if (i16 < K && d < D) dst[(int64_t)d * K + i16] = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Wide products (up to 16 columns): U = X %*% V and R = t(X) %*% G for 5..16 classes (the
// 10-class MultiLogReg of BASELINE config #3).  Same tile pipeline as mchain_kernel, but the
// three bf16 rounding planes of V / G are separate MFMAs accumulating into one tile whose M / N
// dimension holds the 16 columns themselves (mchain_kernel stacks the planes in the spare rows,
// which caps it at 4 columns).
// Waves per block: the fused chains at D > 768 hold V's planes, the R accumulators and the
// staged X tile at once, which at 8 waves exceeds 128 VGPRs; 16 waves halve each wave's slice.
template <int MODE, int KS>
constexpr int wide_waves() { return (MODE != XV && MODE != XTG && KS == 4) ? 16 : WAVES; }

template <int MODE, int KS>
__global__ void __launch_bounds__((64 * wide_waves<MODE, KS>()), MIN_WAVES_PER_SIMD)
wide_kernel(const uint16_t* __restrict__ X, int64_t N, int D,
            const uint16_t* __restrict__ VW,   // [3][16][Dp] bf16: plane p of V[:, k] in row 16p + k
            const float* __restrict__ S, int lds, int K,
            float* __restrict__ out, int ldo, int64_t tiles_per_block,
            float* __restrict__ U, int ldu, double* __restrict__ obj, const double* __restrict__ live) {
  if (sysml_dead(live)) return;    // dead run-ahead iteration (runtime/program.py)
  constexpr int WV = wide_waves<MODE, KS>();
  constexpr int BLK = 64 * WV;
  constexpr int Dp = KS * 256;
  constexpr int ROWB = Dp * 2 + 16;
  constexpr int CH = Dp / 8;
  constexpr int NST = TR * CH / BLK;
  constexpr int KC = Dp / (32 * WV);  // 32-column chunks of this wave's slice (phase 1)
  constexpr int NB = Dp / (16 * WV);  // 16-column blocks of this wave's slice (phase 2)
  static_assert(NST * BLK == TR * CH && KC * 32 * WV == Dp, "wide tile shape");
  // phase 1: U = X V on the tile (XV and the chains); phase 2: R += t(X_tile) G (XTG and chains)
  constexpr bool P1 = (MODE != XTG);
  constexpr bool P2 = (MODE != XV);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Xs = smem;
  float* Ured = reinterpret_cast<float*>(smem + TR * ROWB);         // [WV][TR][16]
  uint16_t* G3 = reinterpret_cast<uint16_t*>(Ured + WV * TR * 16);  // [3][TR][16]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int i16 = lane & 15;
  const int q = i16 >> 2, p = i16 & 3;
  const int dsl = wave * (Dp / WV);

  bf8 afr[P1 ? 3 : 1][P1 ? KC : 1];
  if constexpr (P1) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int ks = 0; ks < KC; ++ks)
        afr[pl][ks] = *reinterpret_cast<const bf8*>(VW + ((int64_t)pl * 16 + i16) * Dp + dsl + ks * 32 + 8 * g);
  }
  f4 acc[P2 ? NB : 1];
#pragma unroll
  for (int b = 0; b < (P2 ? NB : 1); ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};

  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_block;
  const int64_t t1 = (t0 + tiles_per_block < ntiles) ? t0 + tiles_per_block : ntiles;

  u4 st[NST];
  uint32_t stok = 0;
  auto gload = [&](int64_t t) {
    stok = 0;
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int id = j * BLK + tid;
      const int row = id / CH, ch = id - (id / CH) * CH;
      const int64_t r = t * TR + row;
      const bool ok = (r < N) && (ch * 8 < D);
      stok |= (ok ? 1u : 0u) << j;
      const int64_t off = ok ? r * (int64_t)D + ch * 8 : 0;
      st[j] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(X + off));
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int id = j * BLK + tid;
      const int row = id / CH, ch = id - (id / CH) * CH;
      const u4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u4*>(Xs + row * ROWB + ch * 16) = ((stok >> j) & 1u) ? st[j] : z;
    }
  };
  // this thread's S value of the tile (threads 0..255: row tid / 16, column tid % 16):
  // G for XTG, w for XTWXV (one column), y for XTXVY, P for XTPSXV, Y for the softmax modes
  // (XTSMGO reads Y's K + 1 columns)
  constexpr int SX = (MODE == XTSMGO) ? 1 : 0;
  auto svals = [&](int64_t t) -> float {
    if (tid >= TR * 16) return 0.f;
    const int row = tid >> 4, col = tid & 15;
    const int64_t r = t * TR + row;
    if constexpr (MODE == XTWXV) return (r < N && col < K) ? S[r * (int64_t)lds] : 0.f;
    return (r < N && col < K + SX) ? S[r * (int64_t)lds + col] : 0.f;
  };
  float o1 = 0.f, o2 = 0.f;   // XTSMGO objective terms of this thread's rows

  if (t0 < t1) {
    gload(t0);
    swrite();
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  for (int64_t t = t0; t < t1; ++t) {
    float gv = 0.f;
    if constexpr (MODE != XV && MODE != XTXV) gv = svals(t);
    if (t + 1 < t1) gload(t + 1);

    if constexpr (P1) {
      f4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KC; ++ks) {
        const bf8 b = *reinterpret_cast<const bf8*>(Xs + i16 * ROWB + (dsl + ks * 32 + 8 * g) * 2);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[pl][ks], b, u, 0, 0, 0);
      }
      // u[i] = partial U[row i16][column 4g + i] over this wave's columns of X
      *reinterpret_cast<f4*>(Ured + (wave * TR + i16) * 16 + 4 * g) = u;
      __syncthreads();
      if (tid < TR * 16) {
        const int row = tid >> 4, col = tid & 15;
        float uu = 0.f;
#pragma unroll
        for (int w = 0; w < WV; ++w) uu += Ured[(w * TR + row) * 16 + col];
        if constexpr (MODE == XV) {
          const int64_t r = t * TR + row;
          if (r < N && col < K) out[r * (int64_t)ldo + col] = uu;
        } else if constexpr (MODE == XTXV) {
          gv = uu;
        } else if constexpr (MODE == XTWXV) {
          gv *= uu;
        } else if constexpr (MODE == XTXVY) {
          gv = uu - gv;
        } else if constexpr (MODE == XTPSXV) {
          // g = P * u - P * rowSums(P * u): the 16 columns of a row are 16 consecutive lanes
          const float qv = gv * uu;
          float rs = qv;
#pragma unroll
          for (int m = 1; m < 16; m <<= 1) rs += __shfl_xor(rs, m, 16);
          gv = qv - gv * rs;
        } else {
          // softmax over L = [u_0 .. u_{K-1}, 0] (K <= 15: the zero class is column K)
          const int64_t r = t * TR + row;
          const bool rv = r < N;
          const float lv = col < K ? uu : 0.f;
          float m = col <= K ? lv : -INFINITY;
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 16));
          const float e = col <= K ? __expf(lv - m) : 0.f;
          float se = e;
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) se += __shfl_xor(se, o, 16);
          const float pr = e / se;
          if constexpr (MODE == XTSMG) {
            if (rv && col < K) U[r * (int64_t)ldu + col] = uu;
          } else {
            if (rv && col <= K) U[r * (int64_t)ldu + col] = pr;
            if (rv && col <= K) o1 += gv * (lv - m);
            if (rv && col == 0) o2 += __logf(se);
          }
          gv = (rv && col < K) ? pr - gv : 0.f;
        }
        // padded rows / columns stay zero: U's padding is zero and S is read as zero there
      }
    }
    if constexpr (P2) {
      if (tid < TR * 16) {
        const uint16_t h = f2bf(gv);
        float rem = gv - bf2f(h);
        const uint16_t l1 = f2bf(rem);
        rem -= bf2f(l1);
        const uint16_t l2 = f2bf(rem);
        G3[tid] = h;
        G3[TR * 16 + tid] = l1;
        G3[2 * TR * 16 + tid] = l2;
      }
      __syncthreads();
      s4 bfr[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bfr[pl] = tr_read(G3 + pl * TR * 16 + (4 * g + q) * 16 + 4 * p);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int dblk = dsl + b * 16;
        const s4 a = tr_read(Xs + (4 * g + q) * ROWB + (dblk + 4 * p) * 2);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) acc[b] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bfr[pl], acc[b], 0, 0, 0);
      }
    }
    __syncthreads();
    if (t + 1 < t1) {
      swrite();
      __syncthreads();
    }
  }

  if constexpr (MODE == XTSMGO) {
    double d1 = o1, d2 = o2;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      d1 += __shfl_xor(d1, o, 64);
      d2 += __shfl_xor(d2, o, 64);
    }
    if (lane == 0) {
      obj[((int64_t)blockIdx.x * WV + wave) * 2] = d1;
      obj[((int64_t)blockIdx.x * WV + wave) * 2 + 1] = d2;
    }
  }
  if constexpr (P2) {
    // acc[b][i] = R[d = dsl + 16b + 4g + i][column i16]
    float* dst = out + (int64_t)blockIdx.x * D * K;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = dsl + b * 16 + 4 * g + i;
        if (i16 < K && d < D) dst[(int64_t)d * K + i16] = acc[b][i];
      }
  }
}

template <int MODE, int KS>
static size_t lds_bytes_wide() {
  return (size_t)TR * (KS * 512 + 16) + wide_waves<MODE, KS>() * TR * 16 * 4 + 3 * TR * 16 * 2;
}

template <int MODE, int KS>
static int launch_wide(bool occ, const void* X, int64_t N, int D, const void* VW, const float* S, int lds, int K,
                       float* out, int ldo, int grid, hipStream_t st, float* U, int ldu, double* obj) {
  const size_t sh = lds_bytes_wide<MODE, KS>();
  constexpr int blk = 64 * wide_waves<MODE, KS>();
  if (occ) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, wide_kernel<MODE, KS>, blk, sh) != hipSuccess) return -1;
    return nb;
  }
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t tpb = (ntiles + grid - 1) / grid;
  hipLaunchKernelGGL((wide_kernel<MODE, KS>), dim3(grid), dim3(blk), sh, st, (const uint16_t*)X, N, D,
                     (const uint16_t*)VW, S, lds, K, out, ldo, tpb, U, ldu, obj, sysml_live_flag());
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int MODE>
static int dispatch_wide(int ks, bool occ, const void* X, int64_t N, int D, const void* VW, const float* S, int lds,
                         int K, float* out, int ldo, int grid, hipStream_t st, float* U, int ldu, double* obj) {
  switch (ks) {
    case 1: return launch_wide<MODE, 1>(occ, X, N, D, VW, S, lds, K, out, ldo, grid, st, U, ldu, obj);
    case 2: return launch_wide<MODE, 2>(occ, X, N, D, VW, S, lds, K, out, ldo, grid, st, U, ldu, obj);
    case 3: return launch_wide<MODE, 3>(occ, X, N, D, VW, S, lds, K, out, ldo, grid, st, U, ldu, obj);
    case 4: return launch_wide<MODE, 4>(occ, X, N, D, VW, S, lds, K, out, ldo, grid, st, U, ldu, obj);
    default: return -1;
  }
}

template <int MODE, int KS>
static size_t lds_bytes() {
  return (size_t)TR * (KS * 64 * WAVES + 16) + WAVES * TR * 16 * 4 + WAVES * TR * 16 * 2;
}

template <int MODE, int KS>
static int launch(const void* X, int64_t N, int D, const void* V3T, const float* S, int lds, int sbc, int K,
                  float* out, int ldo, int grid, hipStream_t st) {
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t tpb = (ntiles + grid - 1) / grid;
  const size_t sh = lds_bytes<MODE, KS>();
  hipLaunchKernelGGL((mchain_kernel<MODE, KS>), dim3(grid), dim3(BLOCK), sh, st,
                     (const uint16_t*)X, N, D, (const uint16_t*)V3T, S, lds, sbc, K, out, ldo, tpb, sysml_live_flag());
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int MODE, int KS>
static int occupancy() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, mchain_kernel<MODE, KS>, BLOCK, lds_bytes<MODE, KS>()) !=
      hipSuccess)
    return -1;
  return nb;
}

template <int MODE>
static int dispatch(int ks, bool occ, const void* X, int64_t N, int D, const void* V3T, const float* S, int lds,
                    int sbc, int K, float* out, int ldo, int grid, hipStream_t st) {
#define SYSML_MC_CASE(KV)                                                                          \
  case KV:                                                                                         \
    return occ ? occupancy<MODE, KV>() : launch<MODE, KV>(X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
  switch (ks) {
    SYSML_MC_CASE(1)
    SYSML_MC_CASE(2)
    SYSML_MC_CASE(3)
    SYSML_MC_CASE(4)
    default: return -1;
  }
#undef SYSML_MC_CASE
}

static int route(int mode, int ks, bool occ, const void* X, int64_t N, int D, const void* V3T, const float* S,
                 int lds, int sbc, int K, float* out, int ldo, int grid, hipStream_t st) {
  switch (mode) {
    case XV: return dispatch<XV>(ks, occ, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
    case XTG: return dispatch<XTG>(ks, occ, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
    case XTXV: return dispatch<XTXV>(ks, occ, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
    case XTWXV: return dispatch<XTWXV>(ks, occ, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
    case XTXVY: return dispatch<XTXVY>(ks, occ, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
    case XTPSXV: return dispatch<XTPSXV>(ks, occ, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, st);
    default: return -1;
  }
}

}  // namespace sysml_mc

extern "C" {

// Number of co-resident blocks per CU for (mode, D); the host sizes the grid as CUs x this.
int sysml_mchain_occupancy(int mode, int D) {
  if (D <= 0 || D > 1024) return -1;
  return sysml_mc::route(mode, (D + 255) / 256, true, nullptr, 0, D, nullptr, nullptr, 0, 0, 0, nullptr, 0, 0,
                         nullptr);
}

// X: N x D bf16 row-major (D % 8 == 0, 16-B aligned); V3T: [16][Dp] bf16 split planes of V
// (Dp = 256*ceil(D/256)); S: row-side fp32 operand (weights / targets / probabilities / G);
// out: XV -> N x ldo fp32; other modes -> grid x (D*K) fp32 partials.  K in {1, 2, 4}.
int sysml_mchain(int mode, const void* X, int64_t N, int D, const void* V3T, const float* S, int lds, int sbc, int K,
                 float* out, int ldo, int grid, hipStream_t stream) {
  if (D <= 0 || D > 1024 || (D & 7) || K < 1 || K > 4 || grid <= 0) return -1;
  return sysml_mc::route(mode, (D + 255) / 256, false, X, N, D, V3T, S, lds, sbc, K, out, ldo, grid, stream);
}

// Wide products and chains (K <= 16 columns; V as [3][16][Dp] bf16 planes).
static int wide_route(int mode, int ks, bool occ, const void* X, int64_t N, int D, const void* VW, const float* S,
                      int lds, int K, float* out, int ldo, int grid, hipStream_t st, float* U, int ldu, double* obj) {
  using namespace sysml_mc;
#define SYSML_WIDE(M) return dispatch_wide<M>(ks, occ, X, N, D, VW, S, lds, K, out, ldo, grid, st, U, ldu, obj)
  switch (mode) {
    case XV: SYSML_WIDE(XV);
    case XTG: SYSML_WIDE(XTG);
    case XTXV: SYSML_WIDE(XTXV);
    case XTWXV: SYSML_WIDE(XTWXV);
    case XTXVY: SYSML_WIDE(XTXVY);
    case XTPSXV: SYSML_WIDE(XTPSXV);
    case XTSMG: SYSML_WIDE(XTSMG);
    case XTSMGO: SYSML_WIDE(XTSMGO);
    default: return -1;
  }
#undef SYSML_WIDE
}

int sysml_mwide_occupancy(int mode, int D) {
  if (D <= 0 || D > 1024) return -1;
  return wide_route(mode, (D + 255) / 256, true, nullptr, 0, D, nullptr, nullptr, 0, 0, nullptr, 0, 0, nullptr,
                    nullptr, 0, nullptr);
}

// Wide products and chains (K <= 16 columns; V as [3][16][Dp] bf16 planes).  Mode XV: out N x ldo;
// XTG and the chains (XTXV, XTWXV w: N x 1, XTXVY y: N x K, XTPSXV P: N x K; lds = leading
// dimension of S): out grid x (D*K) per-block partials of the D x K result.  Softmax modes
// (K <= 15, S = Y): XTSMG writes U = X V to U (N x ldu); XTSMGO reads Y's K + 1 columns, writes
// the K + 1 class probabilities to U and per-wave objective partials to obj (grid * waves x 2).
int sysml_mwide(int mode, const void* X, int64_t N, int D, const void* VW, const float* S, int lds, int K, float* out,
                int ldo, int grid, hipStream_t stream, float* U, int ldu, double* obj) {
  using namespace sysml_mc;
  if (D <= 0 || D > 1024 || (D & 7) || K < 1 || K > 16 || grid <= 0 || N <= 0) return -1;
  if (mode != XTG && VW == nullptr) return -1;
  const int scols = mode == XTWXV ? 1 : mode == XTSMGO ? K + 1 : K;
  if (mode != XV && mode != XTXV && (S == nullptr || lds < scols)) return -1;
  if (mode == XTSMG || mode == XTSMGO) {
    if (K > 15 || U == nullptr || ldu < scols || (mode == XTSMGO && obj == nullptr)) return -1;
  }
  return wide_route(mode, (D + 255) / 256, false, X, N, D, VW, S, lds, K, out, ldo, grid, stream, U, ldu, obj);
}

}  // extern "C"
