// General dense matrix multiply (ba+*), transpose-self multiply (tsmm) and their split-K
// reductions on the CDNA4 matrix cores (gfx950).
//
// Reference semantics: runtime/matrix/data/LibMatrixMult.java:86 (matrixMult, ba+*) and :331
// (matrixMultTransposeSelf, tsmm), GPU path LibMatrixCUDA.java:477 (matmultTSMM) and
// LibMatrixCuMatMult (cuBLAS dgemm).  The reference hands these to cuBLAS/MKL; here they are
// hand-written for gfx950:
//
//   * bf16 operands -> v_mfma_f32_16x16x32_bf16, fp32 accumulation / output.
//     256x256x64 block tile, 512 threads = 8 wave64 (2 x 4), each wave owns a 128 x 64 output
//     sub-tile = 8 x 4 MFMA tiles (128 accumulator registers).  Both operands are staged
//     HBM -> LDS by LDS-DMA (global_load_lds_dwordx4), double-buffered: the DMA of K-tile t+1
//     is in flight while tile t is read and multiplied.
//   * Each operand is consumed in whichever orientation it is stored in, with no transpose
//     pass: a K-contiguous operand ("K-major": A of A%*%B, or B of A%*%t(B)) lands as a
//     [rows][64] image (128-B rows) read by ds_read_b128; an M/N-contiguous operand
//     ("MN-major": B of A%*%B, A of t(A)%*%B) lands as a [64][256] image (512-B rows) read
//     with the hardware transpose ds_read_b64_tr_b16.  Both images are XOR-swizzled in 16-B
//     granules so every fragment read is bank-conflict free; glds writes LDS lane-linearly,
//     so the swizzle is applied to the per-lane GLOBAL source address (the inverse
//     permutation) and again on the read.
//   * tsmm = t(X) %*% X runs the same kernel with both operands MN-major and only the
//     upper-triangular block tiles scheduled; a finishing pass mirrors the result.
//   * Tall reductions (K >> M, N: t(X) %*% Y, tsmm on 10M-row X) are split over K into fp32
//     slabs summed by a separate pass (deterministic, no float atomics).
//   * Block ids are remapped so each XCD (own L2) receives a contiguous run of output tiles.
//   * fp32 / fp64 operands -> exact-precision MFMA (v_mfma_f32_32x32x2_f32,
//     v_mfma_f64_16x16x4_f64) in a register-staged 128x128 tile kernel (gemm_fp_kernel).
//
// Edges: rows/columns past M/N read a clamped valid address and are never stored; the
// K-tail tile zeroes fragment elements with k >= K in registers.  The host guarantees that
// the contiguous dimension of every operand is a multiple of 8 elements (bf16) / 16 bytes
// (fp32, fp64) and 16-B aligned (ops/gemm.py pads otherwise).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <cstdlib>

namespace sysml_gk {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;
typedef __attribute__((address_space(3))) s8 lds_s8;
typedef __attribute__((address_space(3))) char lds_char;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHR = 512;
constexpr int OPB = BM * BK * 2;    // bytes of one operand image (32 KiB)
constexpr int LDS_BYTES = 4 * OPB;  // 2 buffers x (A, B) = 128 KiB

struct Args {
  const void* A;
  const void* B;
  float* C;          // output (fp32 for bf16 operands; T for the fp kernel)
  int64_t lda, ldb, ldc;
  int64_t slab;      // elements between split-K slabs (0: write C directly)
  int M, N, K;
  int tm, tn;        // block tiles along M, N
  int ntiles;        // scheduled output tiles (upper triangle only when tri)
  int ksplit, ktps;  // K splits, K-tiles per split
  int tri, beta;
  int veca, vecb;    // fp kernel: operand rows are 16-B aligned (vector loads allowed)
  // image-blocked columns (convolutions lowered to ONE GEMM over all images, bf16 kernel):
  // hwb > 0 -> column j of B and C is pixel j % hwb of image j / hwb; B image n starts at
  // simgB * n (pixels contiguous, k stride ldb), C image n at simgC * n (pixels contiguous,
  // row stride ldc); pixels >= hwr are padding (read as data, never stored)
  int hwb, hwr;
  int64_t simgB, simgC;
  int obf16, relu;   // C stored bf16 (round to nearest even); relu after the bias
  const float* bias; // C[row][*] += bias[row] (null: none)
  int vec;           // 4-column vector stores are aligned (C / slab rows, image strides, base)
};

__device__ __forceinline__ int swz_k(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz_t(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }

// bijective XCD-aware remap: blocks b and b+8 share an XCD (dispatch round-robin), give each
// XCD a contiguous range of logical work-group ids (cdna_hip_programming.md T1)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// logical tile -> (bm, bn): groups of 8 tile-rows for L2 reuse; upper triangle for tsmm
__device__ __forceinline__ void tile_coords(const Args& a, int t, int& bm, int& bn) {
  if (a.tri) {
    int r = 0, rem = t;
    while (rem >= a.tm - r) { rem -= a.tm - r; ++r; }
    bm = r;
    bn = r + rem;
    return;
  }
  const int per = 8 * a.tn;
  const int grp = t / per, first = grp * 8;
  const int gsz = (a.tm - first) < 8 ? (a.tm - first) : 8;
  const int w = t - grp * per;
  bm = first + w % gsz;
  bn = w / gsz;
}

// ---------------------------------------------------------------------------------------
// bf16 kernel
// ---------------------------------------------------------------------------------------
// Per-lane staging source for one operand: BKT/16 DMA instructions per wave per K-tile.
// KMAJ: image [256 rows][BKT k] (operand stored [rows][ld], k contiguous)
// else: image [BKT k][256 cols] (operand stored [k][ld], cols contiguous, 512-B rows)
// Lane offsets are 32-bit and relative to the block's (scalar) base pointer, so the
// staging state costs BKT/16 VGPRs per operand (host guarantees 256 * ld < 2^31).
template <int BKT> __device__ __forceinline__ int swz_kb(int row) {
  // XOR on the 16-B chunk index of a K-major row, conflict-free for the ds_read_b128 lane
  // groups (tools/lds_bank_sim.py): 128-B rows -> 8 chunks, 64-B rows -> 4 chunks
  if constexpr (BKT == 64) return (row >> 1) & 7;
  else return (row & 1) | ((row >> 1) & 2);
}

// LDS-DMA of one 16-B piece per lane: global_load_lds_dwordx4 in the saddr form (scalar tile
// base + 32-bit lane byte offset), LDS destination M0 + lane * 16.  Issued from inline asm so
// the compiler's waitcnt pass does not see an LDS write it would order every later ds_read
// behind with vmcnt(0) (that drains the DMA pipeline each K-tile); the kernel retires the
// DMAs itself with counted s_waitcnt vmcnt(N) + s_barrier.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const uint16_t* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory", "m0");
}
#pragma clang diagnostic pop

template <bool KMAJ, int BKT, int ROWS = 256, int NW = 8>   // NW: waves sharing the DMAs
struct Stager {
  static_assert(KMAJ || ROWS == 256, "MN-major images are 256 columns wide");
  static constexpr int NJ = ROWS * BKT * 2 / (1024 * NW); // DMA instructions per wave per K-tile (NW waves)
  static constexpr int RPI = 1024 / (BKT * 2);   // K-major rows per 1-KiB instruction
  static constexpr int CPR = BKT / 8;            // 16-B chunks per K-major row
  int off[NJ];
  const uint16_t* base;   // block base: operand + r0 * ld (KMAJ) or operand + r0 (MN-major)
  int64_t ld;
  // hw > 0 (MN-major only): image-blocked columns (Args::hwb), images simg elements apart
  __device__ __forceinline__ void init(const uint16_t* op, int wave, int lane, int r0, int R, int64_t ld_,
                                       int hw = 0, int64_t simg = 0) {
    ld = ld_;
    const int img0 = hw > 0 ? r0 / hw : 0;
    base = KMAJ ? op + (int64_t)r0 * ld_ : (hw > 0 ? op + (int64_t)img0 * simg : op + r0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gi = wave * NJ + j;
      if constexpr (KMAJ) {
        const int row = gi * RPI + lane / CPR;
        const int c = (lane % CPR) ^ swz_kb<BKT>(row);
        const int gr = (r0 + row < R) ? row : R - 1 - r0;
        off[j] = gr * (int)ld_ + 8 * c;
      } else {
        const int krow = gi * 2 + (lane >> 5);
        const int g = (lane & 31) ^ swz_t(krow);
        const int R8 = (R + 7) & ~7;                   // ld >= R8: columns up to R8 are in bounds
        const int gc = (r0 + 8 * g < R8 - 8) ? 8 * g : R8 - 8 - r0;
        if (hw > 0) {
          // hw % 8 == 0: an 8-column piece never straddles two images
          const int col = r0 + gc, img = col / hw;
          off[j] = (int)((int64_t)(img - img0) * simg) + krow * (int)ld_ + (col - img * hw);
        } else {
          off[j] = krow * (int)ld_ + gc;
        }
      }
    }
  }
  // issue the DMAs of the K-tile starting at k0 into image `dst`
  __device__ __forceinline__ void issue(int k0, int K, bool tail, lds_char* dst, int wave, int lane) const {
    const uint16_t* tb = KMAJ ? base + k0 : base + (int64_t)k0 * ld;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      int o = off[j];
      if (tail) {
        const int gi = wave * NJ + j;
        if constexpr (KMAJ) {
          const int kc = 8 * ((lane % CPR) ^ swz_kb<BKT>(gi * RPI + lane / CPR));
          const int K8 = (K + 7) & ~7;                 // ld >= K8: the chunk at K8-8 is in bounds
          if (k0 + kc >= K8) o += (K8 - 8 - k0) - kc;  // any valid chunk; masked in registers
        } else {
          const int krow = gi * 2 + (lane >> 5);
          if (k0 + krow >= K) o += (K - 1 - k0 - krow) * (int)ld;
        }
      }
      glds16(tb, (uint32_t)o * 2u, (uint32_t)(uintptr_t)(dst + (wave * NJ + j) * 1024));
    }
  }
};

__device__ __forceinline__ s8 cat(s4 a, s4 b) { return s8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }

// fragment of 16 rows (or cols) x 32 k for MFMA 16x16x32, from an operand image.
// r0: first row/col of the 16 within the 256-wide image; kk: 32-deep k step in the tile
template <bool KMAJ, int BKT>
__device__ __forceinline__ s8 frag(const lds_char* img, int r0, int kk, int lane) {
  if constexpr (KMAJ) {
    const int row = r0 + (lane & 15);
    const int c = (kk * 4 + (lane >> 4)) ^ swz_kb<BKT>(row);
    return *(const lds_s8*)(img + row * (BKT * 2) + c * 16);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int G = (r0 >> 3) + (p >> 1);
    const int k0 = kk * 32 + 8 * g + q;
    const int k1 = k0 + 4;
    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + k0 * 512 + ((G ^ swz_t(k0)) * 16) + 8 * (p & 1)));
    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + k1 * 512 + ((G ^ swz_t(k1)) * 16) + 8 * (p & 1)));
    return cat(lo, hi);
  }
}

__device__ __forceinline__ s8 mask_k(s8 v, int kbase, int K) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (kbase + j < K) ? v[j] : (short)0;
  return v;
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// Workgroup barrier that does NOT drain the LDS-DMA queue (a __syncthreads() fence would emit
// vmcnt(0)): own LDS reads retired, then s_barrier.
__device__ __forceinline__ void bar_keep_dma() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// BKT = 64: two LDS stages (DMA of tile t+1 overlaps tile t; drain + barrier per tile).
// BKT = 32: four LDS stages of 32 KiB, three K-tiles in flight; per tile a COUNTED vmcnt
//           (own DMAs of tile t retired, later tiles keep streaming) + a raw s_barrier.
// BMT = rows of A per block: 256 (waves 2 x 4 of 128 x 64), 128 (2 x 4 of 64 x 64: twice the
// workgroups for GEMMs whose 256-row tiles leave CUs idle) or 64 (waves 2 x 4 of 32 x 64, for GEMMs
// with few rows -- convolutions with 64 filters / channels); the smaller tiles K-major A, BKT 64
template <bool TA, bool TB, int BKT, int BMT = 256>
__global__ void __launch_bounds__(NTHR, 2)
gemm_bf16_kernel(Args a) {
  constexpr bool AK = !TA;   // A K-major
  constexpr bool BKM = TB;   // B K-major
  static_assert(BMT == 256 || ((BMT == 64 || BMT == 128) && !TA && BKT == 64), "row-tile variants");
  constexpr int WM = BMT / 2;                    // rows per wave
  constexpr int MI = WM / 16;                    // 16-row MFMA tiles per wave
  constexpr int NST = BKT == 64 ? 2 : 4;         // LDS stages
  constexpr int OPA = BMT * BKT * 2;             // bytes of the A image
  constexpr int OPI = BM * BKT * 2;              // bytes of the B image (256 columns)
  constexpr int STG = OPA + OPI;                 // bytes per stage (A + B images)
  constexpr int KK = BKT / 32;                   // 32-deep MFMA steps per tile
  constexpr int DPT = (BMT * BKT * 2 + BM * BKT * 2) / 8192;   // DMA instructions per wave per tile (A + B)
  static_assert(NST * STG <= LDS_BYTES, "LDS budget");
  extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % a.ntiles, split = wg / a.ntiles;
  int bm, bn;
  tile_coords(a, tile, bm, bn);
  const int ktiles = (a.K + BKT - 1) / BKT;
  const int kt0 = split * a.ktps;
  const int kt1 = (kt0 + a.ktps < ktiles) ? kt0 + a.ktps : ktiles;

  Stager<AK, BKT, BMT> sa;
  Stager<BKM, BKT> sb;
  sa.init((const uint16_t*)a.A, wave, lane, bm * BMT, a.M, a.lda);
  sb.init((const uint16_t*)a.B, wave, lane, bn * BN, a.N, a.ldb, BKM ? 0 : a.hwb, a.simgB);

  f4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // one K-tile from LDS: per 32-deep step read the wave's 4 B fragments, then stream its 8 A
  // fragments through 4 MFMAs each (keeps the live fragment set at ~24 VGPRs)
  auto compute = [&](const lds_char* Ai, const lds_char* Bi, int k0, auto tailtag) {
    constexpr bool TAIL = decltype(tailtag)::value;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int kb = k0 + kk * 32 + 8 * (lane >> 4);
      s8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bfr[j] = frag<BKM, BKT>(Bi, wc * 64 + j * 16, kk, lane);
        if constexpr (TAIL) bfr[j] = mask_k(bfr[j], kb, a.K);
      }
      s8 af = frag<AK, BKT>(Ai, wr * WM, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        // next A fragment in flight while this one's 4 MFMAs issue
        s8 an = af;
        if (i < MI - 1) an = frag<AK, BKT>(Ai, wr * WM + (i + 1) * 16, kk, lane);
        if constexpr (TAIL) af = mask_k(af, kb, a.K);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          // operands swapped: the accumulator holds C^T, so a lane's 4 values are 4 consecutive
          // C columns of one row (vector stores in the epilogue)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf8)bfr[j], (bf8)af, acc[i][j], 0, 0, 0);
        af = an;
      }
    }
  };
  auto issue = [&](int kt, int ktail, lds_char* st) {
    sa.issue(kt * BKT, a.K, kt == ktail, st, wave, lane);
    sb.issue(kt * BKT, a.K, kt == ktail, st + OPA, wave, lane);
  };

  if (kt0 < kt1) {
    const bool has_tail = (kt1 == ktiles) && (a.K % BKT) != 0;
    const int ktail = has_tail ? kt1 - 1 : -1;
    if constexpr (NST == 2) {
      const int ktf = has_tail ? kt1 - 1 : kt1;   // full tiles: [kt0, ktf)
      issue(kt0, ktail, smem);
      wait_vm<0>();
      __syncthreads();
      int cur = 0;
      for (int kt = kt0; kt < ktf; ++kt) {
        lds_char* St = smem + cur * STG;
        if (kt + 1 < kt1) issue(kt + 1, ktail, smem + (cur ^ 1) * STG);
        compute(St, St + OPA, kt * BKT, std::false_type{});
        wait_vm<0>();
        __syncthreads();
        cur ^= 1;
      }
      if (has_tail) {
        lds_char* St = smem + cur * STG;
        compute(St, St + OPA, ktf * BKT, std::true_type{});
      }
    } else {
      // prologue: tiles kt0 .. kt0+2 in flight
#pragma unroll
      for (int p = 0; p < NST - 1; ++p)
        if (kt0 + p < kt1) issue(kt0 + p, ktail, smem + p * STG);
      int slot = 0;
      const int ktf = has_tail ? kt1 - 1 : kt1;   // full tiles: [kt0, ktf)
      for (int kt = kt0; kt < ktf; ++kt) {
        // tile kt landed for this wave: the DMAs of up to two later tiles stay in flight
        const int later = kt1 - 1 - kt;
        if (later >= 2) wait_vm<2 * DPT>();
        else if (later == 1) wait_vm<DPT>();
        else wait_vm<0>();
        bar_keep_dma();   // every wave's tile-kt DMAs retired; every wave done reading tile kt-1
        if (kt + NST - 1 < kt1) issue(kt + NST - 1, ktail, smem + ((slot + NST - 1) & (NST - 1)) * STG);
        lds_char* St = smem + slot * STG;
        compute(St, St + OPA, kt * BKT, std::false_type{});
        slot = (slot + 1) & (NST - 1);
      }
      if (has_tail) {
        wait_vm<0>();
        bar_keep_dma();
        lds_char* St = smem + slot * STG;
        compute(St, St + OPA, ktf * BKT, std::true_type{});
      }
    }
  }

  // epilogue.  C^T map of 16x16x32 with swapped operands: C row = lane & 15 (+ 16 i), C columns
  // (lane >> 4) * 4 + reg (+ 16 j) -- four consecutive columns per lane
  const int64_t ldc = a.ldc;
  const int rbase = bm * BMT + wr * WM + (lane & 15);
  const int cbase = bn * BN + wc * 64 + (lane >> 4) * 4;
  if (a.slab || (!a.obf16 && a.hwb == 0 && a.bias == nullptr && !a.relu)) {
    // plain fp32 C (or a split-K slab: the reduction pass applies the epilogue)
    float* dst = (float*)a.C + (a.slab ? (int64_t)split * a.slab : 0);
    const bool acc_in = a.beta && !a.slab;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = rbase + i * 16;
      if (row >= a.M) continue;
      float* prow = dst + (int64_t)row * ldc;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = cbase + j * 16;
        if (a.vec && col + 3 < a.N) {
          f4 v = acc[i][j];
          if (acc_in) v += *(const f4*)(prow + col);
          *(f4*)(prow + col) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col + r < a.N) prow[col + r] = acc_in ? prow[col + r] + acc[i][j][r] : acc[i][j][r];
        }
      }
    }
    return;
  }
  // DNN epilogue: image-blocked columns (4 consecutive columns never straddle two images: hwb %
  // 8 == 0), per-row bias, relu, bf16 or fp32 C
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = rbase + i * 16;
    if (row >= a.M) continue;
    const float bv = a.bias != nullptr ? a.bias[row] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cbase + j * 16;
      if (col >= a.N) continue;
      int64_t cofs = col;
      int nv = a.N - col < 4 ? a.N - col : 4;
      if (a.hwb > 0) {
        const int img = col / a.hwb, px = col - img * a.hwb;
        nv = a.hwr - px < nv ? a.hwr - px : nv;
        cofs = (int64_t)img * a.simgC + px;
      }
      if (nv <= 0) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bv;
        if (a.relu) v[r] = v[r] > 0.f ? v[r] : 0.f;
      }
      const int64_t o = (int64_t)row * ldc + cofs;
      if (a.obf16) {
        uint16_t h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          uint32_t u = __float_as_uint(v[r]);
          u += 0x7fffu + ((u >> 16) & 1u);
          h[r] = (uint16_t)(u >> 16);
        }
        uint16_t* p = (uint16_t*)a.C + o;
        if (a.vec && nv == 4) {
          *(uint2*)p = uint2{(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r < nv) p[r] = h[r];
        }
      } else {
        float* p = (float*)a.C + o;
        if (a.vec && nv == 4) *(f4*)p = f4{v[0], v[1], v[2], v[3]};
        else
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r < nv) p[r] = v[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// bf16 kernel, register-pipelined (K a multiple of 64; plain, split-K slab and DNN epilogues): the same
// 256x256x64 block tile, LDS images and 2-stage LDS-DMA as gemm_bf16_kernel, but the MFMA
// fragments are software-pipelined one 32-deep step ahead ACROSS the K-tile boundary:
//   step kk=1 of tile t is read from LDS while the 32 MFMAs of step kk=0 issue; after the
//   barrier that publishes tile t+1, step kk=0 of tile t+1 is read while kk=1's MFMAs issue,
//   and the DMA of tile t+2 goes into tile t's buffer right there (its fragments already sit
//   in registers) -- so every ds_read has a full step of MFMAs (512 cycles per wave) to land,
//   and every DMA about a whole tile.  Two fragment sets: 2 x 48 VGPRs + 128 accumulators.
// ---------------------------------------------------------------------------------------
template <bool TA, bool TB, bool DNN>
__global__ void __launch_bounds__(NTHR, 1)
gemm_bf16_pf(Args a) {
  constexpr bool AK = !TA, BKM = TB;
  constexpr int BKT = 64, WM = 128, MI = 8, OPA = BM * BKT * 2, STG = 2 * OPA;
  extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % a.ntiles, split = wg / a.ntiles;
  int bm, bn;
  tile_coords(a, tile, bm, bn);
  const int ktiles = a.K / BKT;
  const int kt0 = split * a.ktps;
  const int kt1 = (kt0 + a.ktps < ktiles) ? kt0 + a.ktps : ktiles;
  Stager<AK, BKT> sa;
  Stager<BKM, BKT> sb;
  sa.init((const uint16_t*)a.A, wave, lane, bm * BM, a.M, a.lda);
  sb.init((const uint16_t*)a.B, wave, lane, bn * BN, a.N, a.ldb, DNN ? a.hwb : 0, DNN ? a.simgB : 0);
  f4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  s8 fa0[MI], fb0[4], fa1[MI], fb1[4];
  auto issue = [&](int kt) {
    lds_char* st = smem + (kt & 1) * STG;
    sa.issue(kt * BKT, a.K, false, st, wave, lane);
    sb.issue(kt * BKT, a.K, false, st + OPA, wave, lane);
  };
  auto load = [&](int kt, int kk, s8 (&fa)[MI], s8 (&fb)[4]) {
    const lds_char* st = smem + (kt & 1) * STG;
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag<BKM, BKT>(st + OPA, wc * 64 + j * 16, kk, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = frag<AK, BKT>(st, wr * WM + i * 16, kk, lane);
  };
  auto mma = [&](const s8 (&fa)[MI], const s8 (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf8)fb[j], (bf8)fa[i], acc[i][j], 0, 0, 0);
  };
  if (kt0 < kt1) {
    issue(kt0);
    wait_vm<0>();
    __syncthreads();
    load(kt0, 0, fa0, fb0);
    if (kt0 + 1 < kt1) issue(kt0 + 1);
    for (int kt = kt0; kt < kt1; ++kt) {
      load(kt, 1, fa1, fb1);
      mma(fa0, fb0);
      if (kt + 1 < kt1) {
        wait_vm<0>();          // this wave's DMA of tile kt+1 landed
        bar_keep_dma();        // ... every wave's; and every read of tile kt's buffer retired
        load(kt + 1, 0, fa0, fb0);
        if (kt + 2 < kt1) issue(kt + 2);    // into tile kt's buffer: its fragments are in registers
      }
      mma(fa1, fb1);
    }
  }
  const int64_t ldc = a.ldc;
  const int rbase = bm * BM + wr * WM + (lane & 15);
  const int cbase = bn * BN + wc * 64 + (lane >> 4) * 4;
  if (!DNN || a.slab) {   // plain fp32 C, or split-K slabs (the reduction pass applies the DNN epilogue)
    float* dst = (float*)a.C + (a.slab ? (int64_t)split * a.slab : 0);
    const bool acc_in = a.beta && !a.slab;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = rbase + i * 16;
      if (row >= a.M) continue;
      float* prow = dst + (int64_t)row * ldc;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = cbase + j * 16;
        if (a.vec && col + 3 < a.N) {
          f4 v = acc[i][j];
          if (acc_in) v += *(const f4*)(prow + col);
          *(f4*)(prow + col) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col + r < a.N) prow[col + r] = acc_in ? prow[col + r] + acc[i][j][r] : acc[i][j][r];
        }
      }
    }
    return;
  }
  // DNN epilogue (as gemm_bf16_kernel): image-blocked columns, per-row bias, relu, bf16 / fp32 C
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = rbase + i * 16;
    if (row >= a.M) continue;
    const float bv = a.bias != nullptr ? a.bias[row] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cbase + j * 16;
      if (col >= a.N) continue;
      int64_t cofs = col;
      int nv = a.N - col < 4 ? a.N - col : 4;
      if (a.hwb > 0) {
        const int img = col / a.hwb, px = col - img * a.hwb;
        nv = a.hwr - px < nv ? a.hwr - px : nv;
        cofs = (int64_t)img * a.simgC + px;
      }
      if (nv <= 0) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bv;
        if (a.relu) v[r] = v[r] > 0.f ? v[r] : 0.f;
      }
      const int64_t o = (int64_t)row * ldc + cofs;
      if (a.obf16) {
        uint16_t h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          uint32_t u = __float_as_uint(v[r]);
          u += 0x7fffu + ((u >> 16) & 1u);
          h[r] = (uint16_t)(u >> 16);
        }
        uint16_t* p = (uint16_t*)a.C + o;
        if (a.vec && nv == 4) {
          *(uint2*)p = uint2{(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r < nv) p[r] = h[r];
        }
      } else {
        float* p = (float*)a.C + o;
        if (a.vec && nv == 4) *(f4*)p = f4{v[0], v[1], v[2], v[3]};
        else
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r < nv) p[r] = v[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// fp32 / fp64 kernel: 128x128x16 tile, 256 threads (2 x 2 waves of 64 x 64), register-staged
// double-buffered LDS images [16][128 + PAD] in M/N-contiguous order for both operands.
// ---------------------------------------------------------------------------------------
template <typename T> struct FpCfg;
template <> struct FpCfg<float> { static constexpr int PAD = 2; };
template <> struct FpCfg<double> { static constexpr int PAD = 1; };

constexpr int FBM = 128, FBK = 16, FNTHR = 256;

template <typename T>
__device__ __forceinline__ void ld8(const T* p, int64_t n_ok, bool vec, T (&v)[8]) {
  // 8 contiguous elements, the first n_ok of them valid; 16-B vector loads when the whole
  // chunk is valid and aligned (vec: row pitch and base are 16-B multiples)
  if (n_ok >= 8 && vec) {
    if constexpr (sizeof(T) == 4) {
      const float4 x0 = *(const float4*)p;
      const float4 x1 = *(const float4*)(p + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
      v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    } else {
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const double2 x = *(const double2*)(p + 2 * h);
        v[2 * h] = x.x;
        v[2 * h + 1] = x.y;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (i < n_ok) ? p[i] : (T)0;
  }
}

template <typename T, bool TA, bool TB>
__global__ void __launch_bounds__(FNTHR, 2)
gemm_fp_kernel(Args a) {
  constexpr int PAD = FpCfg<T>::PAD;
  constexpr int LD = FBM + PAD;
  __shared__ T As[2][FBK][LD];
  __shared__ T Bs[2][FBK][LD];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % a.ntiles, split = wg / a.ntiles;
  int bm, bn;
  tile_coords(a, tile, bm, bn);
  const int ktiles = (a.K + FBK - 1) / FBK;
  const int kt0 = split * a.ktps;
  const int kt1 = (kt0 + a.ktps < ktiles) ? kt0 + a.ktps : ktiles;
  const T* A = (const T*)a.A;
  const T* B = (const T*)a.B;
  const int m0 = bm * FBM, n0 = bn * FBM;

  T ra[8], rb[8];
  // stage one operand tile into registers.  MN-major source [k][ld]: thread -> (k = t/16,
  // 8 contiguous cols); K-major source [rows][ld]: thread -> (row = t/2, 8 contiguous k)
  auto gload = [&](const T* base, int64_t ld, bool kmaj, int r0, int R, int k0, bool vec, T (&v)[8]) {
    if (!kmaj) {
      const int k = k0 + (tid >> 4), c = r0 + (tid & 15) * 8;
      const int64_t nok = (k < a.K) ? (int64_t)R - c : 0;
      ld8<T>(base + (int64_t)(k < a.K ? k : 0) * ld + (c < R ? c : 0), nok, vec, v);
    } else {
      const int r = r0 + (tid >> 1), k = k0 + (tid & 1) * 8;
      const int64_t nok = (r < R) ? (int64_t)a.K - k : 0;
      ld8<T>(base + (int64_t)(r < R ? r : 0) * ld + (k < a.K ? k : 0), nok, vec, v);
    }
  };
  auto swrite = [&](T (*S)[LD], bool kmaj, const T (&v)[8]) {
    if (!kmaj) {
      const int k = tid >> 4, c = (tid & 15) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) S[k][c + i] = v[i];
    } else {
      const int r = tid >> 1, k = (tid & 1) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) S[k + i][r] = v[i];
    }
  };

  constexpr bool F32 = sizeof(T) == 4;
  // fp32: 2 x 2 tiles of 32x32 (16 acc regs each); fp64: 4 x 4 tiles of 16x16 (4 acc each)
  f16v accf[2][2];
  d4 accd[4][4];
  if constexpr (F32) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) accf[i][j][r] = 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accd[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  }

  if (kt0 < kt1) {
    gload(A, a.lda, !TA, m0, a.M, kt0 * FBK, a.veca, ra);
    gload(B, a.ldb, TB, n0, a.N, kt0 * FBK, a.vecb, rb);
    swrite(As[0], !TA, ra);
    swrite(Bs[0], TB, rb);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) {
        gload(A, a.lda, !TA, m0, a.M, (kt + 1) * FBK, a.veca, ra);
        gload(B, a.ldb, TB, n0, a.N, (kt + 1) * FBK, a.vecb, rb);
      }
      if constexpr (F32) {
#pragma unroll
        for (int ks = 0; ks < FBK; ks += 2) {
          const int k = ks + (lane >> 5);
          float av[2], bv[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) av[i] = As[cur][k][wr * 64 + i * 32 + (lane & 31)];
#pragma unroll
          for (int j = 0; j < 2; ++j) bv[j] = Bs[cur][k][wc * 64 + j * 32 + (lane & 31)];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              accf[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], accf[i][j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < FBK; ks += 4) {
          const int k = ks + (lane >> 4);
          double av[4], bv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) av[i] = As[cur][k][wr * 64 + i * 16 + (lane & 15)];
#pragma unroll
          for (int j = 0; j < 4; ++j) bv[j] = Bs[cur][k][wc * 64 + j * 16 + (lane & 15)];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              accd[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], accd[i][j], 0, 0, 0);
        }
      }
      if (more) {
        swrite(As[cur ^ 1], !TA, ra);
        swrite(Bs[cur ^ 1], TB, rb);
      }
      __syncthreads();
    }
  }

  T* dst = (T*)a.C + (a.slab ? (int64_t)split * a.slab : 0);
  const bool acc_in = a.beta && !a.slab;
  auto put = [&](int row, int col, T v) {
    if (row < a.M && col < a.N) {
      T* p = dst + (int64_t)row * a.ldc + col;
      *p = acc_in ? *p + v : v;
    }
  };
  if constexpr (F32) {
    // 32x32 C/D: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          put(m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), n0 + wc * 64 + j * 32 + (lane & 31),
              accf[i][j][r]);
  } else {
    // f64 16x16: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          put(m0 + wr * 64 + i * 16 + (lane >> 4) + 4 * r, n0 + wc * 64 + j * 16 + (lane & 15), accd[i][j][r]);
  }
}

// ---------------------------------------------------------------------------------------
// split-K reduction (+ triangle mirror) and in-place mirror
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
splitk_reduce(const T* __restrict__ slab, int64_t stride, int ks, T* __restrict__ C, int64_t ldc, int M, int N,
              int tri, int tb, int beta) {
  const int64_t total = (int64_t)M * N;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(idx / N), j = (int)(idx - (int64_t)i * N);
    int si = i, sj = j;
    if (tri && (i / tb) > (j / tb)) { si = j; sj = i; }
    T s = 0;
    const T* p = slab + (int64_t)si * N + sj;
    for (int k = 0; k < ks; ++k) s += p[(int64_t)k * stride];
    T* o = C + (int64_t)i * ldc + j;
    *o = beta ? *o + s : s;
  }
}

// split-K reduction with the DNN epilogue (image-blocked columns, bias, relu, bf16 / fp32 C)
__global__ void __launch_bounds__(256)
splitk_reduce_dnn(const float* __restrict__ slab, int64_t stride, int ks, void* __restrict__ C, int64_t ldc, int M,
                  int N, int hwb, int hwr, int64_t simgC, const float* __restrict__ bias, int relu, int obf16) {
  const int64_t total = (int64_t)M * N;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(idx / N), j = (int)(idx - (int64_t)i * N);
    int64_t cofs = j;
    if (hwb > 0) {
      const int img = j / hwb, px = j - img * hwb;
      if (px >= hwr) continue;
      cofs = (int64_t)img * simgC + px;
    }
    float v = 0.f;
    for (int k = 0; k < ks; ++k) v += slab[idx + (int64_t)k * stride];
    if (bias != nullptr) v += bias[i];
    if (relu) v = v > 0.f ? v : 0.f;
    const int64_t o = (int64_t)i * ldc + cofs;
    if (obf16) {
      uint32_t u = __float_as_uint(v);
      u += 0x7fffu + ((u >> 16) & 1u);
      ((uint16_t*)C)[o] = (uint16_t)(u >> 16);
    } else {
      ((float*)C)[o] = v;
    }
  }
}

// B [N][C][hw] -> [N][C][hwp] (zero padding): image-blocked GEMM operands need 8-pixel pieces.
// One thread per 8 output pixels (one 16-B store); the source run is read with the widest loads
// its alignment allows (VEC = 4: hw % 4 == 0, 8-B loads; 2: 4-B loads; 1: 2-B loads).
template <int VEC>
__global__ void __launch_bounds__(256)
pad_pixels(const uint16_t* __restrict__ X, uint16_t* __restrict__ Y, int64_t planes, int hw, int hwp) {
  const int gpp = hwp >> 3;                       // 8-pixel groups per plane
  const int64_t total = planes * gpp;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pl = g / gpp;
    const int px = (int)(g - pl * gpp) * 8;
    const uint16_t* src = X + pl * hw + px;
    uint16_t v[8];
    if (px + 8 <= hw) {
      if (VEC == 4) {
        const uint2 a = *(const uint2*)src, b = *(const uint2*)(src + 4);
        v[0] = (uint16_t)a.x; v[1] = (uint16_t)(a.x >> 16); v[2] = (uint16_t)a.y; v[3] = (uint16_t)(a.y >> 16);
        v[4] = (uint16_t)b.x; v[5] = (uint16_t)(b.x >> 16); v[6] = (uint16_t)b.y; v[7] = (uint16_t)(b.y >> 16);
      } else if (VEC == 2) {
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const uint32_t a = *(const uint32_t*)(src + e);
          v[e] = (uint16_t)a; v[e + 1] = (uint16_t)(a >> 16);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = src[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = px + e < hw ? src[e] : (uint16_t)0;
    }
    *(uint4*)(Y + pl * hwp + px) = uint4{(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                                         (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
  }
}

// fp32 M x K filter -> bf16 (round to nearest even) R x Cp, R x C = W or t(W), columns C..Cp-1
// zero: the GEMM's A operand (16-B aligned rows) in ONE pass instead of cast + transpose + pad
__global__ void __launch_bounds__(256)
cast_weight(const float* __restrict__ W, uint16_t* __restrict__ Y, int M, int K, int trans, int cp) {
  const int R = trans ? K : M, C = trans ? M : K;
  const int64_t total = (int64_t)R * cp;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(idx / cp), c = (int)(idx - (int64_t)r * cp);
    uint16_t h = 0;
    if (c < C) {
      uint32_t u = __float_as_uint(trans ? W[(int64_t)c * K + r] : W[(int64_t)r * K + c]);
      u += 0x7fffu + ((u >> 16) & 1u);
      h = (uint16_t)(u >> 16);
    }
    Y[idx] = h;
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
mirror_lower(T* __restrict__ C, int64_t ldc, int M, int tb) {
  const int64_t total = (int64_t)M * M;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(idx / M), j = (int)(idx - (int64_t)i * M);
    if ((i / tb) > (j / tb)) C[(int64_t)i * ldc + j] = C[(int64_t)j * ldc + i];
  }
}

template <typename K>
static int launch_kernel(K kern, const Args& a, int threads, size_t lds, hipStream_t st) {
  const int grid = a.ntiles * a.ksplit;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace sysml_gk

using namespace sysml_gk;

static int g_bk = 0;    // bf16 K-tile override: 0 = auto, 32 (4-stage, counted vmcnt), 64 (2-stage)

template <bool TA, bool TB, int BKT, int BMT = 256>
static int launch_bf16_t(const Args& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_kernel<TA, TB, BKT, BMT>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) != hipSuccess)
      return -3;
    attr = true;
  }
  return launch_kernel(gemm_bf16_kernel<TA, TB, BKT, BMT>, a, NTHR, LDS_BYTES, st);
}

// register-pipelined bf16 kernel (gemm_bf16_pf): 1 = on for plain GEMMs with K % 64 == 0 and a
// 64-deep K tile, 0 = off, 2 = also the image-blocked DNN GEMMs (SYSML_GEMM_PF / sysml_gemm_set_pf).
// The DNN route is opt-in: ResNet-50 b256 measured 51.6 ms/step with it vs 51.2 without
// (profiles/gemm_pf_dnn_r6.txt) -- its 1x1 GEMMs are HBM-bound, not issue-bound
static int g_pf = [] { const char* e = getenv("SYSML_GEMM_PF"); return e ? atoi(e) : 1; }();

template <bool TA, bool TB, bool DNN = false>
static int launch_bf16_pf(const Args& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_pf<TA, TB, DNN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES) != hipSuccess)
      return -3;
    attr = true;
  }
  return launch_kernel(gemm_bf16_pf<TA, TB, DNN>, a, NTHR, LDS_BYTES, st);
}

template <bool TA, bool TB>
static int launch_bf16(const Args& a, int bk, hipStream_t st) {
  if (g_pf && bk == 64 && a.K % 64 == 0 && a.hwb == 0 && !a.obf16 && !a.relu && a.bias == nullptr)
    return launch_bf16_pf<TA, TB>(a, st);
  return bk == 64 ? launch_bf16_t<TA, TB, 64>(a, st) : launch_bf16_t<TA, TB, 32>(a, st);
}

template <typename T>
static int launch_fp(int ta, int tb, const Args& a, hipStream_t st) {
  if (!ta && !tb) return launch_kernel(gemm_fp_kernel<T, false, false>, a, FNTHR, 0, st);
  if (!ta && tb) return launch_kernel(gemm_fp_kernel<T, false, true>, a, FNTHR, 0, st);
  if (ta && !tb) return launch_kernel(gemm_fp_kernel<T, true, false>, a, FNTHR, 0, st);
  return launch_kernel(gemm_fp_kernel<T, true, true>, a, FNTHR, 0, st);
}

template <typename T>
static int reduce_into(const T* slab, int64_t stride, int ks, T* C, int64_t ldc, int M, int N, int tri, int tb,
                       int beta, hipStream_t st) {
  const int64_t total = (int64_t)M * N;
  int g = (int)((total + 255) / 256);
  g = g < 16384 ? g : 16384;
  hipLaunchKernelGGL(splitk_reduce<T>, dim3(g), dim3(256), 0, st, slab, stride, ks, C, ldc, M, N, tri, tb, beta);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <typename T>
static int mirror(T* C, int64_t ldc, int M, int tb, hipStream_t st) {
  const int64_t total = (int64_t)M * M;
  int g = (int)((total + 255) / 256);
  g = g < 16384 ? g : 16384;
  hipLaunchKernelGGL(mirror_lower<T>, dim3(g), dim3(256), 0, st, C, ldc, M, tb);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" {

// Block-tile edge of each kernel (the host sizes split-K and slabs from it).
int sysml_gemm_tile(int dtype) { return dtype == 2 ? BM : FBM; }
int sysml_gemm_ktile(int dtype) { return dtype == 2 ? 64 : FBK; }
void sysml_gemm_set_bk(int bk) { g_bk = (bk == 64 || bk == 32) ? bk : 0; }
// 0: the 8-wave kernel, 1: register-pipelined (gemm_bf16_pf).  A 4-wave 128 x 128-per-wave
// variant was measured slower (993 vs 1,181 TF nn 8192^3: 256 VGPRs + 256 AGPRs spill at one wave
// per SIMD) and dropped.
void sysml_gemm_set_pf(int on) { g_pf = on < 0 ? 0 : (on > 2 ? 2 : on); }

// C[M][N] (+)= op(A) op(B), op(A) = A (ta=0, A stored [M][lda]) or A^T (ta=1, A stored [K][lda]);
// op(B) = B (tb=0, B stored [K][ldb]) or B^T (tb=1, B stored [N][ldb]).
// dtype: 2 = bf16 operands / fp32 C, 4 = fp32, 8 = fp64.  tri: tsmm (A^T A, M == N, only the
// upper block triangle computed, then mirrored).  ksplit > 1: `slab` holds ksplit x M x N
// partials (ld N) that are summed into C.  beta: accumulate into C.
int sysml_gemm(int dtype, const void* A, int64_t lda, int ta, const void* B, int64_t ldb, int tb, void* C,
               int64_t ldc, int M, int N, int K, int ksplit, void* slab, int tri, int beta, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || ksplit < 1 || (tri && M != N)) return -1;
  const int tile = dtype == 2 ? BM : FBM;
  // bf16 K-tile by measurement: the 2-stage BK=64 kernel wins on square shapes, the 4-stage BK=32
  // one on split-K tall reductions (profiles/gemm_kbench_r2.json) -- unless the register-pipelined
  // BK=64 kernel applies (K % 64 == 0), which wins there too (tn 1000 x 1000 x 1M: 1,103 vs 1,076
  // TF, profiles/gemm_kbench_r6b.json)
  const int bk = g_bk ? g_bk : ((ksplit > 1 && !(g_pf && K % 64 == 0)) ? 32 : 64);
  const int kt = dtype == 2 ? bk : FBK;
  Args a;
  a.veca = a.vecb = 0;
  a.hwb = a.hwr = 0;
  a.simgB = a.simgC = 0;
  a.obf16 = a.relu = 0;
  a.bias = nullptr;
  a.vec = 0;
  a.A = A; a.B = B;
  a.lda = lda; a.ldb = ldb;
  a.M = M; a.N = N; a.K = K;
  a.tm = (M + tile - 1) / tile;
  a.tn = (N + tile - 1) / tile;
  a.ntiles = tri ? a.tm * (a.tm + 1) / 2 : a.tm * a.tn;
  const int ktiles = (K + kt - 1) / kt;
  if (ksplit > ktiles) ksplit = ktiles;
  a.ktps = (ktiles + ksplit - 1) / ksplit;
  a.ksplit = (ktiles + a.ktps - 1) / a.ktps;
  a.tri = tri;
  a.beta = beta;
  const bool use_slab = a.ksplit > 1;
  if (use_slab && !slab) return -1;
  a.C = (float*)(use_slab ? slab : C);
  a.ldc = use_slab ? N : ldc;
  a.slab = use_slab ? (int64_t)M * N : 0;
  if (use_slab) a.beta = 0;
  a.vec = (a.ldc % 4 == 0) && (((uintptr_t)a.C & 15) == 0) && (!use_slab || (a.slab % 4 == 0));
  int rc;
  if (dtype == 2) {
    if ((lda & 7) || (ldb & 7) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return -4;
    if (lda < (ta ? ((M + 7) & ~7) : ((K + 7) & ~7)) || ldb < (tb ? ((K + 7) & ~7) : ((N + 7) & ~7))) return -4;
    if (lda * 256 >= (int64_t)1 << 31 || ldb * 256 >= (int64_t)1 << 31) return -4;
    if (!ta && !tb) rc = launch_bf16<false, false>(a, bk, st);
    else if (!ta && tb) rc = launch_bf16<false, true>(a, bk, st);
    else if (ta && !tb) rc = launch_bf16<true, false>(a, bk, st);
    else rc = launch_bf16<true, true>(a, bk, st);
    if (rc) return rc;
    if (use_slab) return reduce_into<float>((const float*)slab, a.slab, a.ksplit, (float*)C, ldc, M, N, tri, tile,
                                            beta, st);
    return tri ? mirror<float>((float*)C, ldc, M, tile, st) : 0;
  }
  const int vec = 16 / (dtype == 4 ? 4 : 8);
  a.veca = (lda % vec) == 0 && ((uintptr_t)A & 15) == 0;
  a.vecb = (ldb % vec) == 0 && ((uintptr_t)B & 15) == 0;
  if (dtype == 4) {
    rc = launch_fp<float>(ta, tb, a, st);
    if (rc) return rc;
    if (use_slab) return reduce_into<float>((const float*)slab, a.slab, a.ksplit, (float*)C, ldc, M, N, tri, tile,
                                            beta, st);
    return tri ? mirror<float>((float*)C, ldc, M, tile, st) : 0;
  }
  if (dtype == 8) {
    rc = launch_fp<double>(ta, tb, a, st);
    if (rc) return rc;
    if (use_slab) return reduce_into<double>((const double*)slab, a.slab, a.ksplit, (double*)C, ldc, M, N, tri,
                                             tile, beta, st);
    return tri ? mirror<double>((double*)C, ldc, M, tile, st) : 0;
  }
  return -1;
}

// Convolution GEMMs over ALL images as one launch (bf16 operands, fp32 accumulation):
//   C[m][img, px] = bias[m] + sum_k A[m][k] B_img[k][px]   (relu optional, C bf16 or fp32)
// A: K-major [M][lda] (filters; the host transposes W for backward data).  B: images of
// [K][hwb] pixels (hwb % 8 == 0), image n at B + n * simgB, k stride ldb.  C: images of
// [M][hwr] pixels at C + n * simgC (row stride ldc), pixels >= hwr of B's blocks are padding.
// N = images * hwb.  rowtile: 64 or 256 rows of A per workgroup.  ksplit > 1: fp32 slabs
// (ksplit x M x N) reduced by the epilogue pass.
int sysml_gemm_dnn(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t simgB, void* C, int64_t ldc,
                   int64_t simgC, int M, int N, int K, int hwb, int hwr, const float* bias, int relu, int obf16,
                   int ksplit, void* slab, int rowtile, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || ksplit < 1 || hwb <= 0 || (hwb & 7) || hwr > hwb || N % hwb) return -1;
  if ((lda & 7) || (ldb & 7) || (simgB & 7) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return -4;
  if (lda < ((K + 7) & ~7) || ldb < hwb) return -4;
  // 32-bit lane offsets: a 256-column tile spans at most 256 / hwb + 2 images
  if (((int64_t)(256 / hwb + 2) * simgB + (int64_t)BK * ldb) * 2 >= ((int64_t)1 << 31)) return -4;
  if (lda * 256 >= (int64_t)1 << 31) return -4;
  const bool small = rowtile == 64 || rowtile == 128;   // the host picks the row tile (ops/kernels.py _gemm_img)
  const int tile = small ? rowtile : BM;
  const int bk = small ? 64 : (g_bk ? g_bk : (ksplit > 1 ? 32 : 64));
  Args a;
  a.veca = a.vecb = 0;
  a.A = A; a.B = B;
  a.lda = lda; a.ldb = ldb;
  a.M = M; a.N = N; a.K = K;
  a.tm = (M + tile - 1) / tile;
  a.tn = (N + BN - 1) / BN;
  a.ntiles = a.tm * a.tn;
  const int ktiles = (K + bk - 1) / bk;
  if (ksplit > ktiles) ksplit = ktiles;
  a.ktps = (ktiles + ksplit - 1) / ksplit;
  a.ksplit = (ktiles + a.ktps - 1) / a.ktps;
  a.tri = 0;
  a.beta = 0;
  a.hwb = hwb; a.hwr = hwr;
  a.simgB = simgB; a.simgC = simgC;
  a.bias = bias; a.relu = relu; a.obf16 = obf16;
  const bool use_slab = a.ksplit > 1;
  if (use_slab && !slab) return -1;
  a.C = (float*)(use_slab ? slab : C);
  a.ldc = use_slab ? N : ldc;
  a.slab = use_slab ? (int64_t)M * N : 0;
  a.vec = use_slab ? ((N % 4 == 0) && (((uintptr_t)slab & 15) == 0) && (a.slab % 4 == 0))
                   : ((ldc % 4 == 0) && (simgC % 4 == 0) && (((uintptr_t)C & (obf16 ? 7 : 15)) == 0));
  int rc;
  if (small) rc = rowtile == 64 ? launch_bf16_t<false, false, 64, 64>(a, st) : launch_bf16_t<false, false, 64, 128>(a, st);
  else if (g_pf > 1 && bk == 64 && K % 64 == 0) rc = launch_bf16_pf<false, false, true>(a, st);
  else rc = bk == 64 ? launch_bf16_t<false, false, 64>(a, st) : launch_bf16_t<false, false, 32>(a, st);
  if (rc || !use_slab) return rc;
  const int64_t total = (int64_t)M * N;
  int g = (int)((total + 255) / 256);
  g = g < 16384 ? g : 16384;
  hipLaunchKernelGGL(splitk_reduce_dnn, dim3(g), dim3(256), 0, st, (const float*)slab, a.slab, a.ksplit, C, ldc, M, N,
                     hwb, hwr, simgC, bias, relu, obf16);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Y[planes][hwp] = X[planes][hw] zero-padded to hwp pixels (bf16)
int sysml_pad_pixels(const void* X, void* Y, int64_t planes, int hw, int hwp, void* stream) {
  if (planes <= 0 || hw <= 0 || hwp < hw || (hwp & 7) || ((uintptr_t)Y & 15)) return -1;
  const int64_t total = planes * (hwp >> 3);
  int g = (int)((total + 255) / 256);
  g = g < 65536 ? g : 65536;
  const bool a8 = ((uintptr_t)X & 7) == 0, a4 = ((uintptr_t)X & 3) == 0;
  hipStream_t st = (hipStream_t)stream;
  if (hw % 4 == 0 && a8)
    hipLaunchKernelGGL(pad_pixels<4>, dim3(g), dim3(256), 0, st, (const uint16_t*)X, (uint16_t*)Y, planes, hw, hwp);
  else if (hw % 2 == 0 && a4)
    hipLaunchKernelGGL(pad_pixels<2>, dim3(g), dim3(256), 0, st, (const uint16_t*)X, (uint16_t*)Y, planes, hw, hwp);
  else
    hipLaunchKernelGGL(pad_pixels<1>, dim3(g), dim3(256), 0, st, (const uint16_t*)X, (uint16_t*)Y, planes, hw, hwp);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Y (bf16, (trans ? K : M) x cp) = W (fp32 M x K) or its transpose, zero-padded to cp columns
int sysml_cast_weight(const void* W, void* Y, int M, int K, int trans, int cp, void* stream) {
  if (M <= 0 || K <= 0 || cp < (trans ? M : K)) return -1;
  const int64_t total = (int64_t)(trans ? K : M) * cp;
  int g = (int)((total + 255) / 256);
  g = g < 65536 ? g : 65536;
  hipLaunchKernelGGL(cast_weight, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)W, (uint16_t*)Y, M, K,
                     trans, cp);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
