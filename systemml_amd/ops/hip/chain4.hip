// Row-group fused chain kernels: t(X) %*% g(X %*% V) for tall X (N x D, D <= 1024) and skinny V
// (D x K, K in {1, 2, 4}) in ONE pass over X, with the cross-lane work batched over groups of
// four rows.
//
// Reference semantics: LibMatrixMult.matrixMultChain (XtXv, XtwXv, XtXvy) and the MultiLogReg
// inner-loop chain t(X) %*% (P * (X %*% V) - P * rowSums(P * (X %*% V))) plus the fused
// softmax gradient (U = X %*% V, t(X) %*% (softmax([U, 0])[, 1:K] - Y)) that
// compiler/rewrites.py forms from MultiLogReg's line search (scripts/algorithms/MultiLogReg.dml).
//
// Why a second front end next to rowstream.hip's per-row RowOps: with one row at a time every
// dot product needs its own 64-lane reduction (4 DPP steps + 4 readlanes each, a long dependent
// chain), so the K = 4 chains were VALU-latency bound (149 VALU/row for XtPSXv, 290 for the
// softmax gradient at one wave per SIMD; profiles/pmc_chain_r2.txt).  Here a wave takes four
// rows, leaving 4K partial dot products per lane, and reduces all of them together with a
// *transposing* butterfly: each step exchanges half of the remaining values with a partner
// lane and adds (v_permlane32_swap / v_permlane16_swap for lane bits 5 / 4, DPP row_mirror /
// row_half_mirror for bits 3 / 2), so the 16 sums of a K = 4 group cost ~35 VALU instead of
// ~190, and each lane ends up owning one (row, k) value.  The row epilogue (Hessian weights,
// softmax) then runs on 16 lanes at once, and its results reach the accumulate phase as
// wave-uniform SGPR operands of v_pk_fma_f32.
//
// Streaming: X rows arrive by LDS-DMA (global_load_lds_dwordx4; the row-side operand by
// global_load_lds_dword) into a per-wave ring of R = 8 row slots (two groups) retired with a
// counted s_waitcnt vmcnt, exactly as rowstream_dma_kernel; the fused-softmax U output is one
// store per group (lane-selected address, never skipped) and enters the vmcnt count.
#include <hip/hip_runtime.h>
#include <stdint.h>

// cache policy of the streamed X rows' LDS-DMA (aux of global_load_lds): 2 = non-temporal -- each
// X row is read once per pass and X is far larger than the 256 MB MALL, so the default policy
// only evicts the small operands (MI355X_MICROARCH.md: LDS-DMA streams 6.4 -> 6.5-6.8 TB/s nt)
#ifndef SYSML_X_AUX
#define SYSML_X_AUX 2
#endif
#include <unordered_set>

// Run-ahead loops (runtime/program.py _exec_while_runahead): the device address of the fp64
// flag a speculatively queued iteration's streaming kernels read first (0.0 = dead iteration:
// return at once).  Set per host thread by the executor, read by every launch below.
// Bit 0 of the address selects the sense: clear -> live while the flag is non-zero (a `while (p)`
// predicate), set -> live while it is zero (`while (!p)`: the flag is p itself, no negation op).
static thread_local const double* g_live_flag = nullptr;
const double* sysml_live_flag() { return g_live_flag; }
extern "C" void sysml_set_live(const void* p) { g_live_flag = static_cast<const double*>(p); }

// run-ahead live flag (see chain4.hip sysml_set_live): true when the queued iteration is dead
__device__ __forceinline__ bool sysml_dead(const double* live) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(live);
  if (a == 0) return false;
  const double f = *reinterpret_cast<const double*>(a & ~(uintptr_t)1);
  return (f == 0.0) != ((a & 1) != 0);
}

namespace sysml_c4 {

enum Mode { XTXV = 2, XTWXV = 3, XTXVY = 4, XTPSXV = 5, XTSMG = 10, XTSMGO = 11 };   // = rowstream.hip
// XTSMGO (chain4m only): the softmax gradient plus the multinomial-logreg objective terms and
// the full probability matrix -- P = softmax(cbind(X V, 0)) (N x (K+1)), G = t(X) (P[,1:K] -
// Y[,1:K]), sum(Y * (L - rowMaxs(L))) and sum(log(rowSums(exp(L - rowMaxs(L))))), L = cbind(X V, 0)
constexpr int WAVES = 4;
constexpr int BLOCK = 64 * WAVES;
constexpr int G = 4;     // rows per group
constexpr int R = 8;     // ring slots per wave (two groups)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) char lds_char;

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }

template <typename T> struct Pieces { static constexpr int P = (int)sizeof(T) / 2; };   // 16-B pieces / 8 elements

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int QP_X1 = 0xB1, QP_X2 = 0x4E, ROW_HALF_MIRROR = 0x141, ROW_MIRROR = 0x140;

// partner value for butterfly step s: s = 0 lane ^ 32, 1 lane ^ 16, 2 lane ^ 15 (row_mirror),
// 3 lane ^ 7 (row_half_mirror), 4 lane ^ 1, 5 lane ^ 2 (quad_perm)
template <int S>
__device__ __forceinline__ float partner(float v) {
  if constexpr (S == 0) return __shfl_xor(v, 32, 64);
  else if constexpr (S == 1) return __shfl_xor(v, 16, 64);
  else if constexpr (S == 2) return dpp<ROW_MIRROR>(v);
  else if constexpr (S == 3) return dpp<ROW_HALF_MIRROR>(v);
  else if constexpr (S == 4) return dpp<QP_X1>(v);
  else return dpp<QP_X2>(v);
}

// one halving step over the lane bit of step S: values [0, n/2) are kept by lanes whose bit
// is 0, [n/2, n) by lanes whose bit is 1; the partner's copy of the kept half is added
template <int S, int N>
__device__ __forceinline__ void halve(float (&v)[16], int lane) {
  constexpr int H = N / 2;
  if constexpr (S == 0 || S == 1) {
#pragma unroll
    for (int i = 0; i < H; ++i) {
      // v_permlane{32,16}_swap: lanes with the bit clear get {own a, partner a}, lanes with
      // it set get {partner b, own b}  (tools/probe/permlane_probe.hip)
      uint32_t a = __float_as_uint(v[i]), b = __float_as_uint(v[i + H]);
      if constexpr (S == 0) {
        auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      } else {
        auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
    }
  } else {
    const bool hi = (lane >> (S == 2 ? 3 : 2)) & 1;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float keep = hi ? v[i + H] : v[i];
      const float send = hi ? v[i] : v[i + H];
      v[i] = keep + partner<S>(send);
    }
  }
}

// reduce NV = 4K per-lane partials over the wave; afterwards lane l owns value
// (l >> (6 - log2 NV)) & (NV - 1), replicated on 64 / NV lanes.
template <int NV>
__device__ __forceinline__ float transpose_reduce(float (&v)[16], int lane) {
  static_assert(NV == 4 || NV == 8 || NV == 16, "NV");
  halve<0, NV>(v, lane);
  halve<1, NV / 2>(v, lane);
  if constexpr (NV >= 8) halve<2, NV / 4>(v, lane);
  if constexpr (NV >= 16) halve<3, NV / 8>(v, lane);
  float x = v[0];
  if constexpr (NV < 8) x += partner<2>(x);
  if constexpr (NV < 16) x += partner<3>(x);
  x += partner<4>(x);
  x += partner<5>(x);
  return x;
}

template <int N> __device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one X row of the ring slot -> 8J fp32 values of this lane.  All of the row's LDS reads and
// their lgkmcnt wait sit in ONE asm statement: hipcc must not see an LDS read it would order
// behind the pending LDS-DMA with vmcnt(0), and the wait must not be separable from the reads.
__device__ __forceinline__ void unpack_bf16(uint4 r, float* o) {
  o[0] = bf2f(r.x & 0xffffu); o[1] = bf2f(r.x >> 16);
  o[2] = bf2f(r.y & 0xffffu); o[3] = bf2f(r.y >> 16);
  o[4] = bf2f(r.z & 0xffffu); o[5] = bf2f(r.z >> 16);
  o[6] = bf2f(r.w & 0xffffu); o[7] = bf2f(r.w >> 16);
}
__device__ __forceinline__ void unpack_f32(uint4 r, float* o) {
  o[0] = __uint_as_float(r.x); o[1] = __uint_as_float(r.y);
  o[2] = __uint_as_float(r.z); o[3] = __uint_as_float(r.w);
}

template <typename T, int J>
__device__ __forceinline__ void lds_row(const lds_char* slot, int lane, float (&x)[J * 8]) {
  const uint32_t a = (uint32_t)(uintptr_t)(slot + lane * 16);
  if constexpr (sizeof(T) == 2 && J == 1) {
    uint4 r0;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r0) : "v"(a) : "memory");
    unpack_bf16(r0, x);
  } else if constexpr (sizeof(T) == 2 && J == 2) {
    uint4 r0, r1;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(r0), "=&v"(r1) : "v"(a) : "memory");
    unpack_bf16(r0, x);
    unpack_bf16(r1, x + 8);
  } else if constexpr (J == 1) {
    uint4 r0, r1;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(r0), "=&v"(r1) : "v"(a) : "memory");
    unpack_f32(r0, x);
    unpack_f32(r1, x + 4);
  } else {
    uint4 r0, r1, r2, r3;
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\tds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(a) : "memory");
    unpack_f32(r0, x);
    unpack_f32(r1, x + 4);
    unpack_f32(r2, x + 8);
    unpack_f32(r3, x + 12);
  }
}

__device__ __forceinline__ float lds_f32(const lds_char* p) {
  uint32_t t;
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(t) : "v"(a) : "memory");
  return __uint_as_float(t);
}

template <typename T, int K, int J>
constexpr size_t lds_bytes() {
  constexpr size_t ring = (size_t)WAVES * R * (J * Pieces<T>::P * 1024 + 256);
  constexpr size_t red = (size_t)J * 512 * K * 4;
  return ring > red ? ring : red;
}

template <typename T, int K, int J, int MODE>
__global__ void __launch_bounds__(BLOCK, 2)
chain4_kernel(const T* __restrict__ X, int64_t N, int D, const float* __restrict__ V, int ldv,
              const float* __restrict__ S, int lds, int sbc, float* __restrict__ out,
              float* __restrict__ U, int ldu, int64_t rows_per_block, const double* __restrict__ live) {
  if (sysml_dead(live)) return;    // dead run-ahead iteration (runtime/program.py)
  constexpr int C = J * 8;
  constexpr int K2 = (K + 1) / 2;
  constexpr int NV = G * K;
  constexpr int LSH = (NV == 16) ? 2 : (NV == 8) ? 3 : 4;   // lanes per value = 1 << LSH
  constexpr int P = Pieces<T>::P;
  constexpr int XB = J * P * 1024;
  constexpr int SLOT = XB + 256;
  constexpr int NPR = J * P + 1;                  // DMA instructions per row (X pieces + S)
  constexpr bool SMG = (MODE == XTSMG);
  constexpr int NSTG = SMG ? 1 : 0;               // stores per group
  constexpr int NGR = R / G;                      // groups in the ring
  constexpr int WAITN = (NGR - 1) * (G * NPR + NSTG);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- V slice in registers: vreg[c][kk] = V[d(c)][2kk .. 2kk+1], d(c) = (j*64 + lane)*8 + e
  f2 vreg[C][K2];
  {
    float* sV = reinterpret_cast<float*>(smem);
    constexpr int Dp = J * 512;
    for (int i = threadIdx.x; i < Dp * K; i += BLOCK) {
      const int d = i / K, k = i - d * K;
      sV[i] = (d < D) ? V[(int64_t)d * ldv + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) {
          const float* p = sV + ((j * 64 + lane) * 8 + e) * K + 2 * kk;
          vreg[j * 8 + e][kk] = f2{p[0], (2 * kk + 1 < K) ? p[1] : 0.f};
        }
    __syncthreads();   // the ring overlays the V staging area
  }
  f2 acc[C][K2];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int kk = 0; kk < K2; ++kk) acc[c][kk] = f2{0.f, 0.f};

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < N) ? r0 + rows_per_block : N;
  const int64_t rlast = r1 - 1;
  int coff[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    coff[j] = (c0 < D) ? c0 : D - 8;
  }
  int scol;
  if constexpr (SMG) scol = lane < sbc ? lane : sbc - 1;
  else if constexpr (MODE == XTWXV || MODE == XTXVY) scol = sbc ? 0 : (lane < K ? lane : K - 1);
  else scol = lane < K ? lane : K - 1;

  lds_char* ring = (lds_char*)smem + wave * (R * SLOT);
  float* const upad = U + N * (int64_t)ldu;

  auto fetch = [&](int slot, int64_t rr) {
    rr = (rr < rlast) ? rr : rlast;
    const T* row = X + rr * (int64_t)D;
    lds_char* sb = ring + slot * SLOT;
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int h = 0; h < P; ++h)
        __builtin_amdgcn_global_load_lds((const void*)(row + coff[j] + h * (8 / P)),
                                         (void __attribute__((address_space(3)))*)(sb + (j * P + h) * 1024), 16, 0,
                                         SYSML_X_AUX);
    __builtin_amdgcn_global_load_lds((const void*)(S + rr * (int64_t)lds + scol),
                                     (void __attribute__((address_space(3)))*)(sb + XB), 4, 0, 0);
  };

  // rows of the wave: base + (slot) * WAVES; group q = slots [4q, 4q + 4)
  constexpr int STEP = WAVES * R;
  int64_t base = r0 + wave;
#pragma unroll
  for (int q = 0; q < NGR; ++q) {
    // round-0 invariant of the counted wait: every group sees NGR-1 younger (store + refill)
    // sets, so groups after the first are preceded by a dummy store
    if constexpr (SMG) if (q > 0) *upad = 0.f;
#pragma unroll
    for (int s = 0; s < G; ++s) fetch(q * G + s, base + (q * G + s) * WAVES);
  }

  const int myv = (lane >> LSH) & (NV - 1);   // (row, k) value this lane owns after the reduce
  const int myrho = myv / K, myk = myv - (myv / K) * K;

  for (; base < r1; base += STEP) {
#pragma unroll
    for (int q = 0; q < NGR; ++q) {
      wait_vmcnt<WAITN>();
      // ---- phase 1: 4K partial dot products per lane
      float pv[16];
#pragma unroll
      for (int rho = 0; rho < G; ++rho) {
        float x[C];
        lds_row<T, J>(ring + (q * G + rho) * SLOT, lane, x);
        f2 u0[K2];
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) u0[kk] = f2{0.f, 0.f};
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int kk = 0; kk < K2; ++kk) u0[kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, vreg[c][kk], u0[kk]);
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) {
          const f2 u = u0[kk];
          pv[rho * K + 2 * kk] = u.x;
          if (2 * kk + 1 < K) pv[rho * K + 2 * kk + 1] = u.y;
        }
      }
      // ---- transposing butterfly: lane owns u = (X V)[row myrho][myk]
      const float u = transpose_reduce<NV>(pv, lane);
      const int64_t myrow = base + (int64_t)(q * G + myrho) * WAVES;
      const bool rvalid = myrow < r1;
      const float sval = lds_f32(ring + (q * G + myrho) * SLOT + XB + 4 * myk);
      // ---- row epilogue on the (row, k) lanes
      float g;
      if constexpr (MODE == XTXV) {
        g = u;
      } else if constexpr (MODE == XTWXV) {
        g = sval * u;
      } else if constexpr (MODE == XTXVY) {
        g = u - sval;
      } else if constexpr (MODE == XTPSXV) {
        const float qv = sval * u;
        float sq = qv;
        if constexpr (K >= 2) sq += (K == 2) ? partner<2>(sq) : partner<3>(sq);
        if constexpr (K >= 4) sq += partner<2>(sq);
        g = qv - sval * sq;
      } else {   // XTSMG: softmax over [u_1 .. u_kact, 0]
        const bool act = myk < sbc;
        float m = act ? u : 0.f;
        if constexpr (K >= 2) m = fmaxf(m, (K == 2) ? partner<2>(m) : partner<3>(m));
        if constexpr (K >= 4) m = fmaxf(m, partner<2>(m));
        m = fmaxf(m, 0.f);
        const float e = act ? __expf(u - m) : 0.f;
        float s = e;
        if constexpr (K >= 2) s += (K == 2) ? partner<2>(s) : partner<3>(s);
        if constexpr (K >= 4) s += partner<2>(s);
        s += __expf(-m);
        g = act ? e / s - sval : 0.f;
        // U output: one store per group (replica 0 of each valid cell, else the pad row)
        const bool st = act && rvalid && ((lane & ((1 << LSH) - 1)) == 0);
        float* dst = st ? U + myrow * (int64_t)ldu + myk : upad;
        *dst = u;
      }
      g = rvalid ? g : 0.f;
      // ---- phase 2: acc[c][k] += x[row][c] * g[row][k] (g wave-uniform from SGPRs)
#pragma unroll
      for (int rho = 0; rho < G; ++rho) {
        f2 gk[K2];
#pragma unroll
        for (int kk = 0; kk < K2; ++kk) {
          const int v0 = rho * K + 2 * kk;
          const float ga = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), v0 << LSH));
          const float gb = (2 * kk + 1 < K)
                               ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), (v0 + 1) << LSH))
                               : 0.f;
          gk[kk] = f2{ga, gb};
        }
        float x[C];
        lds_row<T, J>(ring + (q * G + rho) * SLOT, lane, x);
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int kk = 0; kk < K2; ++kk) acc[c][kk] = __builtin_elementwise_fma(f2{x[c], x[c]}, gk[kk], acc[c][kk]);
      }
      // ---- refill the group's slots (their LDS reads have retired)
#pragma unroll
      for (int s = 0; s < G; ++s) fetch(q * G + s, base + STEP + (q * G + s) * WAVES);
    }
  }
  wait_vmcnt<0>();   // no LDS-DMA may outlive the ring

  // ---- combine the 4 waves' accumulators through LDS, one partial per block
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int kk = 0; kk < K2; ++kk) {
            const int idx = ((j * 64 + lane) * 8 + e) * K + 2 * kk;
            const f2 a = acc[j * 8 + e][kk];
            if (w == 0) {
              red[idx] = a.x;
              if (2 * kk + 1 < K) red[idx + 1] = a.y;
            } else {
              red[idx] += a.x;
              if (2 * kk + 1 < K) red[idx + 1] += a.y;
            }
          }
    }
    __syncthreads();
  }
  float* dst = out + (int64_t)blockIdx.x * D * K;
  for (int i = threadIdx.x; i < D * K; i += BLOCK) dst[i] = red[i];
}

// ---------------------------------------------------------------------------------------------
// Matrix-core variant for bf16 X and K = 4 (chain4m): both products of the chain run on
// v_mfma_f32_4x4x4bf16_1k (16 independent 4x4x4 blocks per instruction), so the per-element VALU
// work of the kernel above (bf16 unpack + 2 packed FMAs per element and phase) disappears.
//   phase 1  U[row][k] = sum_d X[row][d] V[d][k]: block b of step s takes d = 64s + 4b .. +3
//            (A: lane 4b+i = row i of the group, a plain ds_read_b64 of 4 bf16 of that row;
//            B: lane 4b+j = V[d][j], V split into three exact bf16 planes h + l1 + l2 held in
//            registers), the 16 block partials are summed by a transposing butterfly.
//   phase 2  acc[d][k] += sum_rows X[row][d] G[row][k]: block b of step s owns d = 64s + 4b .. +3
//            (A: lane 4b+i = X[rows 0..3][64s + 4b + i], one ds_read_b64_tr_b16 hardware-transposed
//            read; B: lane 4b+j = G[rows 0..3][j], G split into three bf16 planes through a
//            per-wave LDS scratch), accumulated in 4 fp32 registers per step.
// Every operand product is exact in fp32 (bf16 x bf16), so the result matches the VALU kernel's
// fp32 accumulation.  Ring, row-side operand and counted vmcnt are the kernel above's.
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s4 as_s4(u2 v) {
  s4 r;
  __builtin_memcpy(&r, &v, 8);
  return r;
}

// exact three-plane bf16 split by truncation: v = h + l1 + l2 (each residual fits 8 bits)
__device__ __forceinline__ void split3(float v, uint32_t& h, uint32_t& l1, uint32_t& l2) {
  const uint32_t hb = __float_as_uint(v) & 0xffff0000u;
  const float r1 = v - __uint_as_float(hb);
  const uint32_t b1 = __float_as_uint(r1) & 0xffff0000u;
  const float r2 = r1 - __uint_as_float(b1);
  h = hb >> 16;
  l1 = b1 >> 16;
  l2 = __float_as_uint(r2) >> 16;
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int ROW_ROR4 = 0x124, ROW_ROR8 = 0x128;

// 8 ds_read_b64 (plain or transposed) from one base address at immediate offsets o + 128 s, with
// their lgkmcnt wait in the same asm statement (see lds_row)
#define C4M_READ8(OP, dst, addr, o)                                                                      \
  asm volatile(OP " %0, %8 offset:" #o "\n\t" OP " %1, %8 offset:" #o "+128\n\t" OP " %2, %8 offset:" #o \
               "+256\n\t" OP " %3, %8 offset:" #o "+384\n\t" OP " %4, %8 offset:" #o "+512\n\t" OP       \
               " %5, %8 offset:" #o "+640\n\t" OP " %6, %8 offset:" #o "+768\n\t" OP " %7, %8 offset:" #o  \
               "+896\n\ts_waitcnt lgkmcnt(0)"                                                            \
               : "=&v"(dst[0]), "=&v"(dst[1]), "=&v"(dst[2]), "=&v"(dst[3]), "=&v"(dst[4]), "=&v"(dst[5]), \
                 "=&v"(dst[6]), "=&v"(dst[7])                                                            \
               : "v"(addr)                                                                               \
               : "memory")

template <int J>
constexpr size_t lds_bytes_m() {
  constexpr size_t ring = (size_t)WAVES * R * (J * 1024 + 256 + 64);
  constexpr size_t red = (size_t)J * 512 * 4 * 4;
  return ring > red ? ring : red;
}

template <int J, int MODE, int VAR>
__global__ void __launch_bounds__(BLOCK, 2)
chain4m_kernel(const uint16_t* __restrict__ X, int64_t N, int D, const float* __restrict__ V, int ldv,
               const float* __restrict__ S, int lds, int sbc, float* __restrict__ out,
               float* __restrict__ U, int ldu, int64_t rows_per_block, double* __restrict__ obj,
               const double* __restrict__ live) {
  if (sysml_dead(live)) return;    // dead run-ahead iteration (runtime/program.py)
  constexpr int K = 4;
  constexpr int NS = J * 8;                       // 64-column steps per row
  constexpr int XB = J * 1024;
  constexpr int SLOT = XB + 256 + 64;             // pitch = 16 banks mod 64: conflict-free 4-row reads
  constexpr int NPR = J + 1;
  constexpr bool OBJ = (MODE == XTSMGO);
  constexpr bool SMG = (MODE == XTSMG) || OBJ;
  constexpr int NSTG = OBJ ? 2 : SMG ? 1 : 0;
  constexpr int NGR = R / G;
  constexpr int WAITN = (NGR - 1) * (G * NPR + NSTG);
  static_assert(NS % 8 == 0, "steps come in batches of 8");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int blk = lane >> 2, li = lane & 3;

  // ---- V planes: bv[s][p] = plane p of V[64s + 4blk + e][li], e = 0..3 (zero past D)
  s4 bv[NS][3];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    uint32_t h[4], l1[4], l2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int d = 64 * s + 4 * blk + e;
      split3(d < D ? V[(int64_t)d * ldv + li] : 0.f, h[e], l1[e], l2[e]);
    }
    bv[s][0] = as_s4(u2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)});
    bv[s][1] = as_s4(u2{l1[0] | (l1[1] << 16), l1[2] | (l1[3] << 16)});
    bv[s][2] = as_s4(u2{l2[0] | (l2[1] << 16), l2[2] | (l2[3] << 16)});
  }
  f4 acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = f4{0.f, 0.f, 0.f, 0.f};

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < N) ? r0 + rows_per_block : N;
  const int64_t rlast = r1 - 1;
  int coff[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    coff[j] = (c0 < D) ? c0 : D - 8;
  }
  int scol;
  if constexpr (OBJ) scol = lane <= sbc ? lane : sbc;       // Y[, 1 .. K+1]
  else if constexpr (SMG) scol = lane < sbc ? lane : sbc - 1;
  else if constexpr (MODE == XTWXV || MODE == XTXVY) scol = sbc ? 0 : (lane < K ? lane : K - 1);
  else scol = lane < K ? lane : K - 1;

  lds_char* ring = (lds_char*)smem + wave * (R * SLOT);
  float* const upad = U + N * (int64_t)ldu;
  float o1 = 0.f, o2 = 0.f;     // XTSMGO: this lane's share of sum(Y * LT) and sum(log(rowSums(E)))

  auto fetch = [&](int slot, int64_t rr) {
    rr = (rr < rlast) ? rr : rlast;
    const uint16_t* row = X + rr * (int64_t)D;
    lds_char* sb = ring + slot * SLOT;
#pragma unroll
    for (int j = 0; j < J; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(row + coff[j]),
                                       (void __attribute__((address_space(3)))*)(sb + j * 1024), 16, 0, SYSML_X_AUX);
    __builtin_amdgcn_global_load_lds((const void*)(S + rr * (int64_t)lds + scol),
                                     (void __attribute__((address_space(3)))*)(sb + XB), 4, 0, 0);
  };

  constexpr int STEP = WAVES * R;
  int64_t base = r0 + wave;
#pragma unroll
  for (int q = 0; q < NGR; ++q) {
    if constexpr (SMG) if (q > 0) *upad = 0.f;
    if constexpr (OBJ) if (q > 0) *upad = 0.f;
#pragma unroll
    for (int s = 0; s < G; ++s) fetch(q * G + s, base + (q * G + s) * WAVES);
  }

  const int myrho = (lane >> 4) & 3, myk = lane & 3;   // (row, class) this lane owns after phase 1
  // per-lane LDS addresses (bytes) relative to a group's first slot
  const uint32_t a1 = (uint32_t)(li * SLOT + 8 * blk);                         // phase 1 row reads
  const int tq = (lane >> 2) & 3, tp = lane & 3, tg = lane >> 4;
  const uint32_t a2 = (uint32_t)(tq * SLOT + 32 * tg + 8 * tp);                // phase 2 transposed reads
  const uint32_t gsw = (uint32_t)(XB + 64 + ((myk * 4 + myrho) * 2));          // G scratch write (plane 0)
  const uint32_t gsr = (uint32_t)(XB + 64 + li * 8);                            // G scratch read (plane 0)
  const uint32_t asv = (uint32_t)(myrho * SLOT + XB + 4 * myk);                 // row-side value

  for (; base < r1; base += STEP) {
#pragma unroll
    for (int q = 0; q < NGR; ++q) {
      wait_vmcnt<WAITN>();
      const uint32_t gb = (uint32_t)(uintptr_t)(ring + q * G * SLOT);
      // ---- phase 1: three plane accumulators, 16 steps of 64 columns; the first batch of
      // row reads also fetches this lane's row-side value (one lgkmcnt wait for both)
      f4 cu[3] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
      float sval;
#pragma unroll
      for (int h8 = 0; h8 < NS / 8; ++h8) {
        u2 ar[8];
        const uint32_t ad = gb + a1 + h8 * 1024;
        if (VAR == 1 && h8 == 0) {
          uint32_t sv;
          asm volatile(
              "ds_read_b64 %0, %9\n\tds_read_b64 %1, %9 offset:128\n\tds_read_b64 %2, %9 offset:256\n\t"
              "ds_read_b64 %3, %9 offset:384\n\tds_read_b64 %4, %9 offset:512\n\tds_read_b64 %5, %9 offset:640\n\t"
              "ds_read_b64 %6, %9 offset:768\n\tds_read_b64 %7, %9 offset:896\n\tds_read_b32 %8, %10\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(ar[0]), "=&v"(ar[1]), "=&v"(ar[2]), "=&v"(ar[3]), "=&v"(ar[4]), "=&v"(ar[5]), "=&v"(ar[6]),
                "=&v"(ar[7]), "=&v"(sv)
              : "v"(ad), "v"(gb + asv)
              : "memory");
          sval = __uint_as_float(sv);
        } else {
          C4M_READ8("ds_read_b64", ar, ad, 0);
          if (VAR != 1 && h8 == 0) sval = lds_f32(ring + (q * G + myrho) * SLOT + XB + 4 * myk);
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            cu[p] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(as_s4(ar[s]), bv[h8 * 8 + s][p], cu[p], 0, 0, 0);
      }
      // cu[p][i] on lane 4b+j: partial U[row i][class j] over block b's columns
      float v4[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = cu[0][i] + cu[1][i] + cu[2][i];
      halve<0, 4>(v4, lane);            // lane bit 5 picks rows {0,1} / {2,3}
      halve<1, 2>(v4, lane);            // lane bit 4 picks the row within the pair
      float u = v4[0];
      u += dppf<ROW_ROR8>(u);           // sum over lane bits 2, 3 (the remaining blocks)
      u += dppf<ROW_ROR4>(u);
      // row of this lane's (row, class) value as a 32-bit offset from the wave-uniform base
      // (64-bit address math stays scalar: it is register-pressure critical here)
      const int roff = (q * G + myrho) * WAVES;
      const int64_t left = r1 - base;
      const bool rvalid = roff < (left < (int64_t)0x7fffffff ? (int)left : 0x7fffffff);
      float* const ub = U + base * (int64_t)ldu;
      float g;
      if constexpr (MODE == XTXV) {
        g = u;
      } else if constexpr (MODE == XTWXV) {
        g = sval * u;
      } else if constexpr (MODE == XTXVY) {
        g = u - sval;
      } else if constexpr (MODE == XTPSXV) {
        const float qv = sval * u;
        float sq = qv + dpp<QP_X1>(qv);
        sq += dpp<QP_X2>(sq);
        g = qv - sval * sq;
      } else {   // XTSMG: softmax over [u_1 .. u_kact, 0]
        const bool act = myk < sbc;
        if constexpr (!OBJ) {
          const bool st = act && rvalid && (((lane >> 2) & 3) == 0);
          float* dst = st ? ub + (roff * ldu + myk) : upad;
          *dst = u;
          asm volatile("" ::: "memory");
        }
        float m = act ? u : 0.f;
        m = fmaxf(m, dpp<QP_X1>(m));
        m = fmaxf(m, dpp<QP_X2>(m));
        m = fmaxf(m, 0.f);
        const float e = act ? __expf(u - m) : 0.f;
        float sm = e + dpp<QP_X1>(e);
        sm += dpp<QP_X2>(sm);
        sm += __expf(-m);
        g = act ? e / sm - sval : 0.f;
        if constexpr (OBJ) {
          const bool rep0 = rvalid && (((lane >> 2) & 3) == 0);
          // probabilities of the K + 1 classes (the last one is the zero column of L) and the
          // row's objective terms sum_k Y[r,k] (L[r,k] - max) and log(sum_k exp(L[r,k] - max))
          const float rs = 1.f / sm;
          const float ylast = lds_f32(ring + (q * G + myrho) * SLOT + XB + 4 * sbc);
          float* d1 = (act && rep0) ? ub + (roff * ldu + myk) : upad;
          *d1 = e * rs;
          float* d2 = (myk == 0 && rep0) ? ub + (roff * ldu + sbc) : upad;
          *d2 = __expf(-m) * rs;
          float t1 = act ? sval * (u - m) : 0.f;
          if (myk == 0) t1 -= ylast * m;
          if (rep0) {
            o1 += t1;
            if (myk == 0) o2 += __logf(sm);
          }
        }
      }
      g = rvalid ? g : 0.f;
      __builtin_amdgcn_sched_barrier(0);   // keep phase-2 work from being hoisted (register pressure)
      // ---- G planes through the group's LDS scratch: Gs[p][class][row] bf16
      {
        uint32_t h, l1, l2;
        split3(g, h, l1, l2);
        const uint32_t w = gb + gsw;
        asm volatile("ds_write_b16 %0, %1\n\tds_write_b16 %0, %2 offset:32\n\tds_write_b16 %0, %3 offset:64"
                     :: "v"(w), "v"(h), "v"(l1), "v"(l2) : "memory");
      }
      // ---- phase 2: acc[s] += X^T[64s + ..][rows] G[rows][class]; the G planes are read back
      // together with the first batch of transposed X reads (one wait)
      u2 bg0, bg1, bg2;
      s4 bg[3];
#pragma unroll
      for (int h8 = 0; h8 < NS / 8; ++h8) {
        u2 ar[8];
        const uint32_t ad = gb + a2 + h8 * 1024;
        if (VAR == 1 && h8 == 0) {
          asm volatile(
              "ds_read_b64 %8, %11\n\tds_read_b64 %9, %11 offset:32\n\tds_read_b64 %10, %11 offset:64\n\t"
              "ds_read_b64_tr_b16 %0, %12\n\tds_read_b64_tr_b16 %1, %12 offset:128\n\t"
              "ds_read_b64_tr_b16 %2, %12 offset:256\n\tds_read_b64_tr_b16 %3, %12 offset:384\n\t"
              "ds_read_b64_tr_b16 %4, %12 offset:512\n\tds_read_b64_tr_b16 %5, %12 offset:640\n\t"
              "ds_read_b64_tr_b16 %6, %12 offset:768\n\tds_read_b64_tr_b16 %7, %12 offset:896\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(ar[0]), "=&v"(ar[1]), "=&v"(ar[2]), "=&v"(ar[3]), "=&v"(ar[4]), "=&v"(ar[5]), "=&v"(ar[6]),
                "=&v"(ar[7]), "=&v"(bg0), "=&v"(bg1), "=&v"(bg2)
              : "v"(gb + gsr), "v"(ad)
              : "memory");
          bg[0] = as_s4(bg0);
          bg[1] = as_s4(bg1);
          bg[2] = as_s4(bg2);
        } else {
          if (VAR != 1 && h8 == 0) {
            asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %3 offset:32\n\tds_read_b64 %2, %3 offset:64\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(bg0), "=&v"(bg1), "=&v"(bg2) : "v"(gb + gsr) : "memory");
            bg[0] = as_s4(bg0);
            bg[1] = as_s4(bg1);
            bg[2] = as_s4(bg2);
          }
          C4M_READ8("ds_read_b64_tr_b16", ar, ad, 0);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int s = 0; s < 8; ++s)
            acc[h8 * 8 + s] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(as_s4(ar[s]), bg[p], acc[h8 * 8 + s], 0, 0, 0);
      }
      // ---- refill the group's slots (their LDS reads have retired)
#pragma unroll
      for (int s = 0; s < G; ++s) fetch(q * G + s, base + STEP + (q * G + s) * WAVES);
    }
  }
  wait_vmcnt<0>();

  // ---- combine the 4 waves' accumulators: acc[s][i] on lane 4b+j = out[64s + 4b + i][j]
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = (64 * s + 4 * blk + i) * K + li;
          if (w == 0) red[idx] = acc[s][i];
          else red[idx] += acc[s][i];
        }
    }
    __syncthreads();
  }
  float* dst = out + (int64_t)blockIdx.x * D * K;
  for (int i = threadIdx.x; i < D * K; i += BLOCK) dst[i] = red[i];
  if constexpr (OBJ) {
    double d1 = o1, d2 = o2;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      d1 += __shfl_xor(d1, o, 64);
      d2 += __shfl_xor(d2, o, 64);
    }
    if (lane == 0) {
      obj[((int64_t)blockIdx.x * WAVES + wave) * 2] = d1;
      obj[((int64_t)blockIdx.x * WAVES + wave) * 2 + 1] = d2;
    }
  }
}


static void allow_lds(const void* fn, size_t bytes) {
  static std::unordered_set<const void*> done;
  if (bytes <= 65536 || done.count(fn)) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  done.insert(fn);
}

template <typename T, int K, int J, int MODE>
static int launch(bool occ, const void* X, int64_t N, int D, const float* V, int ldv, const float* S, int lds,
                  int sbc, float* out, float* U, int ldu, int grid, int64_t rpb, hipStream_t st) {
  auto kfn = chain4_kernel<T, K, J, MODE>;
  const size_t sh = lds_bytes<T, K, J>();
  allow_lds(reinterpret_cast<const void*>(kfn), sh);
  if (occ) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, BLOCK, sh) != hipSuccess) return -1;
    return nb;
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(BLOCK), sh, st, (const T*)X, N, D, V, ldv, S, lds, sbc, out, U, ldu,
                     rpb, sysml_live_flag());
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <typename T, int MODE>
static int route_kj(int K, int J, bool occ, const void* X, int64_t N, int D, const float* V, int ldv, const float* S,
                    int lds, int sbc, float* out, float* U, int ldu, int grid, int64_t rpb, hipStream_t st) {
#define C4_CASE(KV, JV)                                                                                    \
  if (K == KV && J == JV) return launch<T, KV, JV, MODE>(occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st);
  C4_CASE(1, 1) C4_CASE(1, 2) C4_CASE(2, 1) C4_CASE(2, 2) C4_CASE(4, 1) C4_CASE(4, 2)
#undef C4_CASE
  return -1;
}

template <typename T>
static int route(int mode, int K, int J, bool occ, const void* X, int64_t N, int D, const float* V, int ldv,
                 const float* S, int lds, int sbc, float* out, float* U, int ldu, int grid, int64_t rpb,
                 hipStream_t st) {
  switch (mode) {
    case XTXV: return route_kj<T, XTXV>(K, J, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st);
    case XTWXV: return route_kj<T, XTWXV>(K, J, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st);
    case XTXVY: return route_kj<T, XTXVY>(K, J, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st);
    case XTPSXV: return route_kj<T, XTPSXV>(K, J, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st);
    case XTSMG: return route_kj<T, XTSMG>(K, J, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st);
    default: return -1;
  }
}

template <int J, int MODE>
static int launch_m(int var, bool occ, const void* X, int64_t N, int D, const float* V, int ldv, const float* S,
                    int lds, int sbc, float* out, float* U, int ldu, int grid, int64_t rpb, hipStream_t st,
                    double* obj) {
  auto kfn = var == 1 ? chain4m_kernel<J, MODE, 1> : chain4m_kernel<J, MODE, 0>;
  const size_t sh = lds_bytes_m<J>();
  allow_lds(reinterpret_cast<const void*>(kfn), sh);
  if (occ) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, BLOCK, sh) != hipSuccess) return -1;
    return nb;
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(BLOCK), sh, st, (const uint16_t*)X, N, D, V, ldv, S, lds, sbc, out, U,
                     ldu, rpb, obj, sysml_live_flag());
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

static int route_m(int var, int mode, int J, bool occ, const void* X, int64_t N, int D, const float* V, int ldv,
                   const float* S, int lds, int sbc, float* out, float* U, int ldu, int grid, int64_t rpb,
                   hipStream_t st, double* obj) {
#define C4M_CASE(MV)                                                                                       \
  case MV:                                                                                                 \
    return J == 1 ? launch_m<1, MV>(var, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st, obj) \
                  : launch_m<2, MV>(var, occ, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rpb, st, obj);
  switch (mode) {
    C4M_CASE(XTXV) C4M_CASE(XTWXV) C4M_CASE(XTXVY) C4M_CASE(XTPSXV) C4M_CASE(XTSMG) C4M_CASE(XTSMGO)
    default: return -1;
  }
#undef C4M_CASE
}

// live flag of the iteration after a queued one in a k-deep run-ahead loop: live only when
// the queued iteration was live AND its predicate continues the loop.  A dead iteration skips
// its kernels and leaves its predicate unwritten, so its successor must not read that value.
__global__ void __launch_bounds__(64) live_and_kernel(const double* prev, const double* q, double* out) {
  if (threadIdx.x == 0) out[threadIdx.x] = (!sysml_dead(prev) && !sysml_dead(q)) ? 1.0 : 0.0;
}

// commit of a graph-replayed run-ahead iteration (runtime/program.py _GraphLoop): copy each
// (src -> dst) pair of the iteration's loop state into the loop's static buffers, only when
// the iteration is live -- a dead (speculative) replay leaves the last live state in place.
constexpr int COMMIT_MAX = 16;
struct CommitTab {
  const void* src[COMMIT_MAX];
  void* dst[COMMIT_MAX];
  long long nbytes[COMMIT_MAX];
  int n;
};

__global__ void __launch_bounds__(256) commit_live_kernel(const CommitTab T, const double* live) {
  if (sysml_dead(live)) return;
  const long long tid = (long long)blockIdx.x * 256 + threadIdx.x, step = (long long)gridDim.x * 256;
  for (int p = 0; p < T.n; ++p) {
    const long long nb = T.nbytes[p];
    const bool words = ((nb | (long long)(uintptr_t)T.src[p] | (long long)(uintptr_t)T.dst[p]) & 3) == 0;
    if (words) {
      const uint32_t* s = (const uint32_t*)T.src[p];
      uint32_t* d = (uint32_t*)T.dst[p];
      for (long long i = tid; i < (nb >> 2); i += step) d[i] = s[i];
    } else {
      const uint8_t* s = (const uint8_t*)T.src[p];
      uint8_t* d = (uint8_t*)T.dst[p];
      for (long long i = tid; i < nb; i += step) d[i] = s[i];
    }
  }
}

}  // namespace sysml_c4

extern "C" {

// n <= COMMIT_MAX pairs; live: encoded run-ahead flag (address | inverted-sense bit)
int sysml_commit_live(int n, const void* const* src, void* const* dst, const long long* nbytes, const void* live,
                      void* stream) {
  using namespace sysml_c4;
  if (n < 0 || n > COMMIT_MAX || live == nullptr) return -1;
  CommitTab T;
  long long mx = 0;
  for (int p = 0; p < n; ++p) {
    if (nbytes[p] < 0 || (nbytes[p] > 0 && (src[p] == nullptr || dst[p] == nullptr))) return -1;
    T.src[p] = src[p];
    T.dst[p] = dst[p];
    T.nbytes[p] = nbytes[p];
    mx = nbytes[p] > mx ? nbytes[p] : mx;
  }
  T.n = n;
  long long g = (mx / 4 + 255) / 256;
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(commit_live_kernel, dim3((int)g), dim3(256), 0, (hipStream_t)stream, T, (const double*)live);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// out (fp64) = 1.0 when neither encoded live flag (address | inverted-sense bit, 0 = none) is
// dead, else 0.0
int sysml_live_and(const void* prev, const void* q, void* out, void* stream) {
  if (out == nullptr) return -1;
  hipLaunchKernelGGL(sysml_c4::live_and_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const double*)prev,
                     (const double*)q, (double*)out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Matrix-core chain (bf16 X, K = 4): blocks per CU, and the launch (arguments as sysml_chain4).
int sysml_chain4m_occupancy(int mode, int D) {
  using namespace sysml_c4;
  if (D <= 0 || D > 1024) return -1;
  return route_m(0, mode, D <= 512 ? 1 : 2, true, nullptr, 0, D, nullptr, 0, nullptr, 0, 0, nullptr, nullptr, 0, 0, 0,
                 nullptr, nullptr);
}

// XTSMGO: U receives P ((N + 1) x ldu, ldu >= sbc + 1, row N a scratch pad), S = Y with sbc + 1
// columns, obj = grid x 4 x 2 doubles of per-wave objective partials.
int sysml_chain4m(int mode, const void* X, int64_t N, int D, const float* V, int ldv, const float* S, int lds,
                  int sbc, float* out, float* U, int ldu, int grid, int64_t rows_per_block, void* stream, int variant,
                  double* obj) {
  using namespace sysml_c4;
  if (D <= 0 || D > 1024 || (D & 7) || N <= 0 || grid <= 0 || (((uintptr_t)X) & 15)) return -1;
  if (mode == XTSMG && (U == nullptr || sbc < 1 || sbc > 4)) return -1;
  if (mode == XTSMGO && (U == nullptr || obj == nullptr || sbc < 1 || sbc > 4 || ldu < sbc + 1 || lds < sbc + 1))
    return -1;
  return route_m(variant, mode, D <= 512 ? 1 : 2, false, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rows_per_block,
                 (hipStream_t)stream, obj);
}


// Blocks per CU of the kernel for (mode, xdtype, K, D) (the host sizes the grid from it).
int sysml_chain4_occupancy(int mode, int xdtype, int K, int D) {
  using namespace sysml_c4;
  if (D <= 0 || D > 1024) return -1;
  const int J = D <= 512 ? 1 : 2;
  if (xdtype == 0)
    return route<uint16_t>(mode, K, J, true, nullptr, 0, D, nullptr, 0, nullptr, 0, 0, nullptr, nullptr, 0, 0, 0,
                           nullptr);
  if (xdtype == 1)
    return route<float>(mode, K, J, true, nullptr, 0, D, nullptr, 0, nullptr, 0, 0, nullptr, nullptr, 0, 0, 0,
                        nullptr);
  return -1;
}

// X: N x D (bf16 xdtype 0 / fp32 xdtype 1), D % 8 == 0, 16-B aligned; V: D x K fp32 (ldv);
// S: row-side operand (N x ., leading dim lds; sbc: broadcast column for XtwXv/XtXvy, number
// of real classes for the softmax gradient); out: grid x (D*K) fp32 partials; U (softmax
// gradient only): (N + 1) x ldu fp32, row N is a scratch pad.  K in {1, 2, 4}.
int sysml_chain4(int mode, int xdtype, const void* X, int64_t N, int D, const float* V, int ldv, const float* S,
                 int lds, int sbc, float* out, float* U, int ldu, int K, int grid, int64_t rows_per_block,
                 void* stream) {
  using namespace sysml_c4;
  if (D <= 0 || D > 1024 || (D & 7) || N <= 0 || grid <= 0 || (((uintptr_t)X) & 15)) return -1;
  if (mode == XTSMG && (U == nullptr || sbc < 1 || sbc > K)) return -1;
  const int J = D <= 512 ? 1 : 2;
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == 0)
    return route<uint16_t>(mode, K, J, false, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rows_per_block, st);
  if (xdtype == 1)
    return route<float>(mode, K, J, false, X, N, D, V, ldv, S, lds, sbc, out, U, ldu, grid, rows_per_block, st);
  return -1;
}

}  // extern "C"
