// Sampled dense-dense product for the weighted quaternary operators (ops/quaternary.py;
// reference: LibMatrixMult.java#matrixMultWSLossSparseDense / wdivmm / wcemm, which loop over
// the non-zeros of W and compute dotProduct(U[i], V[j]) per non-zero).
//
// out[k] = <U[i_k], V[j_k]> for every non-zero k of a CSR pattern (crow/col int64), in fp32 or
// fp64 (the engine's default precision is fp64; the result is accumulated in the operand type).
//
// CDNA4 mapping: one 64-lane wavefront per CSR row (grid-stride over rows).  The wave is split
// into groups of G lanes; a group owns one non-zero at a time and reads the whole V[j] row with
// one 16-byte load per lane (G * 16 B = r * sizeof(T): r=64 fp32 -> G=16, 4 non-zeros per wave
// instruction, each a fully coalesced 256 B segment), multiplies with the matching slice of
// U[i] that the lane keeps in registers for the whole row, and reduces over the group with
// xor-shuffles.  V traffic is exactly r*sizeof(T) per non-zero in whole cache lines; U[i] is
// read once per row.  Rows that need more than 64 lanes (r*sizeof(T) > 1 KiB) loop over chunks.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>

namespace sysml_sd {

constexpr int WAVES = 4;

template <typename T, int NV>
__device__ __forceinline__ void load_vec(const T* p, T (&v)[NV]) {
  if constexpr (NV == 4) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else if constexpr (NV == 2) {
    const double2 x = *reinterpret_cast<const double2*>(p);
    v[0] = x.x; v[1] = x.y;
  } else {
    v[0] = *p;
  }
}

// G lanes per non-zero, NV elements per lane per chunk (16 B when vectorised), NCH chunks
template <typename T, int G, int NV, int NCH, typename I>
__global__ __launch_bounds__(WAVES * 64) void sddmm_kernel(const int64_t* __restrict__ crow,
                                                           const I* __restrict__ col,
                                                           const T* __restrict__ U, const T* __restrict__ V,
                                                           int64_t m, int r, T* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int gl = lane & (G - 1);          // lane within its group
  const int grp = lane / G;               // group within the wave
  constexpr int NG = 64 / G;
  for (int64_t i = (int64_t)blockIdx.x * WAVES + w; i < m; i += (int64_t)gridDim.x * WAVES) {
    const int64_t b = crow[i], e = crow[i + 1];
    if (b == e) continue;                 // wave-uniform
    T u[NCH][NV];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = (c * G + gl) * NV;
      if (k < r) load_vec<T, NV>(U + i * r + k, u[c]);
      else
#pragma unroll
        for (int j = 0; j < NV; ++j) u[c][j] = T(0);
    }
    // UN steps of NG non-zeros per iteration: the column indices first, then every V-row
    // gather of the batch (random rows), then the dot products
    constexpr int UN = NCH == 1 ? 4 : 1;
    for (int64_t p0 = b; p0 < e; p0 += NG * UN) {
      int64_t cc[UN];
#pragma unroll
      for (int s2 = 0; s2 < UN; ++s2) {
        const int64_t p = p0 + s2 * NG + grp;
        cc[s2] = p < e ? (int64_t)col[p] : 0;
      }
      T acc[UN];
      T vv[UN][NCH][NV];
#pragma unroll
      for (int s2 = 0; s2 < UN; ++s2) {
        const T* vr = V + cc[s2] * (int64_t)r;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int k = (c * G + gl) * NV;
          if (k < r) load_vec<T, NV>(vr + k, vv[s2][c]);
          else
#pragma unroll
            for (int j = 0; j < NV; ++j) vv[s2][c][j] = T(0);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < UN; ++s2) {
        acc[s2] = T(0);
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < NV; ++j) acc[s2] += u[c][j] * vv[s2][c][j];
#pragma unroll
        for (int o = G / 2; o >= 1; o >>= 1) acc[s2] += __shfl_xor(acc[s2], o, 64);
        const int64_t p = p0 + s2 * NG + grp;
        if (gl == 0 && p < e) out[p] = acc[s2];
      }
    }
  }
}

template <typename T, int NV, typename I>
int launch(const int64_t* crow, const I* col, const T* U, const T* V, int64_t m, int r, T* out,
           hipStream_t s) {
  int64_t blocks = (m + WAVES - 1) / WAVES;
  if (blocks > 256 * 64) blocks = 256 * 64;     // 8 XCDs x 32 CUs x 64: grid-stride beyond that
  const int lanes = (r + NV - 1) / NV;          // lanes needed to cover one row once
  dim3 g((unsigned)blocks), t(WAVES * 64);
#define SD_CASE(G_, NCH_) hipLaunchKernelGGL((sddmm_kernel<T, G_, NV, NCH_, I>), g, t, 0, s, crow, col, U, V, m, r, out)
  if (lanes <= 1) SD_CASE(1, 1);
  else if (lanes <= 2) SD_CASE(2, 1);
  else if (lanes <= 4) SD_CASE(4, 1);
  else if (lanes <= 8) SD_CASE(8, 1);
  else if (lanes <= 16) SD_CASE(16, 1);
  else if (lanes <= 32) SD_CASE(32, 1);
  else if (lanes <= 64) SD_CASE(64, 1);
  else if (lanes <= 128) SD_CASE(64, 2);
  else if (lanes <= 256) SD_CASE(64, 4);
  else return -1;
#undef SD_CASE
  return (int)hipGetLastError();
}

}  // namespace sysml_sd

namespace sysml_sd {

// ---- fused weighted divide / multiply matrix multiplication (wdivmm right form) ----------------
// out[i, :] = sum over the non-zeros p = (i, j) of q_p * V[j, :] with q_p = f(w_p, <U[i, :], V[j, :]>,
// x_p):  mode 0: w * uv,  1: w * (uv - x),  2: w / (uv + eps).  One pass over the pattern: the V[j]
// row gathered for the dot product is the row that is accumulated (the separate sampled product
// + SpMM read it twice and wrote / read the sampled values).  Non-zeros are split into equal
// chunks over the waves (rows spanning chunks finish with atomics, as spmm_bal); a group of G
// lanes owns one non-zero, lane k its factor column k (K <= 64); the group reduces the dot
// product with xor-shuffles, every lane then accumulates q * V[j, k].  w == nullptr: w = 1.
template <typename I>
__device__ __forceinline__ int64_t wd_first_row(const int64_t* __restrict__ crow, int64_t m, int64_t p) {
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (crow[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Column-blocked passes (rbp != nullptr): V is gathered one column block at a time so the block's
// rows stay resident in the 256 MB MALL instead of missing to HBM (a 10M x 10 fp32 V is 400 MB).
// rbp[r * (nb + 1) + k] is the first non-zero of row r in column block k (columns sorted within a
// row); pass `blk` visits only [rbp[..blk], rbp[..blk + 1]) of each row and ADDS into out (zeroed
// before the first pass), so the CSR arrays are never permuted or copied.
template <typename T, typename I, int G, int UN, bool BLK>
__global__ void __launch_bounds__(WAVES * 64, 8) wdivmm_kernel(const int64_t* __restrict__ crow,
                                                            const I* __restrict__ col, const T* __restrict__ wv,
                                                            const T* __restrict__ xv, const T* __restrict__ U,
                                                            const T* __restrict__ V, T* __restrict__ out, int64_t m,
                                                            int K, int mode, T eps, int64_t chunk, int64_t nchunks,
                                                            const int64_t* __restrict__ rbp, int nb, int blk,
                                                            int64_t ldv) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NG = 64 / G;
  const int g = lane / G, gl = lane & (G - 1);
  const int64_t nnz = crow[m];
  const bool kin = gl < K;
  for (int64_t c = (int64_t)blockIdx.x * WAVES + w; c < nchunks; c += (int64_t)gridDim.x * WAVES) {
    const int64_t s = c * chunk;
    const int64_t e = s + chunk < nnz ? s + chunk : nnz;
    if (s >= e) continue;
    int64_t r = wd_first_row<I>(crow, m, s);
    while (r < m) {
      int64_t rb = crow[r], re = crow[r + 1];
      if (rb >= e) break;
      if constexpr (BLK) {         // this pass's column block of the row
        rb = rbp[r * (nb + 1) + blk];
        re = rbp[r * (nb + 1) + blk + 1];
      }
      const int64_t b = rb > s ? rb : s;
      const int64_t q = re < e ? re : e;
      if (b < q) {
        const bool whole = (rb >= s) && (re <= e);
        const T u = kin ? U[r * K + gl] : T(0);
        T acc = T(0);
        // UN non-zeros per group in flight: indices, weights and the 4 V-row gathers first
        for (int64_t p0 = b + g; p0 < q; p0 += UN * NG) {
          int64_t cj[UN];
          T wt[UN], xt[UN], bv[UN], dt[UN];
#pragma unroll
          // (non-temporal loads of the pattern measured slower: ALS-CG 10M 1.57 vs 1.48 s,
          // profiles/als_pad_r6.txt)
          for (int t = 0; t < UN; ++t) {
            const int64_t p = p0 + t * NG;
            const bool in = p < q;
            cj[t] = in ? (int64_t)col[p] : 0;
            wt[t] = in ? (wv != nullptr ? wv[p] : T(1)) : T(0);
            xt[t] = (in && mode == 1) ? xv[p] : T(0);
          }
#pragma unroll
          for (int t = 0; t < UN; ++t) bv[t] = kin ? V[cj[t] * ldv + gl] : T(0);
#pragma unroll
          for (int t = 0; t < UN; ++t) dt[t] = u * bv[t];
#pragma unroll
          for (int off = G / 2; off >= 1; off >>= 1)
#pragma unroll
            for (int t = 0; t < UN; ++t) dt[t] += __shfl_xor(dt[t], off, G);
#pragma unroll
          for (int t = 0; t < UN; ++t) {
            T qv;
            if (mode == 0) qv = wt[t] * dt[t];
            else if (mode == 1) qv = wt[t] * (dt[t] - xt[t]);
            else qv = wt[t] / (dt[t] + eps);
            if (wt[t] == T(0)) qv = T(0);          // outside the pattern / padding slots
            acc += qv * bv[t];
          }
        }
#pragma unroll
        for (int o = G; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);
        if (g == 0 && kin) {
          if (whole) out[r * K + gl] = BLK ? out[r * K + gl] + acc : acc;
          else atomicAdd(out + r * K + gl, acc);
        }
      }
      ++r;
    }
  }
}

template <typename T, typename I>
int launch_wd(const int64_t* crow, const I* col, const T* wv, const T* xv, const T* U, const T* V, T* out, int64_t m,
              int K, int mode, double eps, int64_t nnz, hipStream_t st, const int64_t* rbp = nullptr, int nb = 0,
              int blk = 0, int64_t ldv = 0) {
  if (ldv < K) ldv = K;
  // the kernel is bound by the latency of its random V-row gathers: one chunk per wave and
  // enough waves for a full CU (8 per SIMD at <= 64 VGPRs), each with UN gathers per group in
  // flight.  SYSML_WD_WAVES / SYSML_WD_UNROLL override (tuning).
  static const int wps = [] { const char* e = getenv("SYSML_WD_WAVES"); return e ? atoi(e) : 32; }();
  static const int un = [] { const char* e = getenv("SYSML_WD_UNROLL"); return e ? atoi(e) : 4; }();
  int64_t chunk = (nnz + 256LL * wps - 1) / (256LL * wps);
  if (chunk < 32) chunk = 32;
  const int64_t nchunks = (nnz + chunk - 1) / chunk;
  int64_t blocks = (nchunks + WAVES - 1) / WAVES;
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  const dim3 gr((unsigned)blocks), t(WAVES * 64);
#define WD_LAUNCH(G_, U_)                                                                                       \
  do {                                                                                                          \
    if (rbp != nullptr)                                                                                         \
      hipLaunchKernelGGL((wdivmm_kernel<T, I, G_, U_, true>), gr, t, 0, st, crow, col, wv, xv, U, V, out, m, K,  \
                         mode, (T)eps, chunk, nchunks, rbp, nb, blk, ldv);                                      \
    else                                                                                                        \
      hipLaunchKernelGGL((wdivmm_kernel<T, I, G_, U_, false>), gr, t, 0, st, crow, col, wv, xv, U, V, out, m, K, \
                         mode, (T)eps, chunk, nchunks, rbp, nb, blk, ldv);                                      \
  } while (0)
#define WD_CASE(G_) \
  if (un >= 8) WD_LAUNCH(G_, 8); \
  else WD_LAUNCH(G_, 4)
  if (K <= 4) { WD_CASE(4); }
  else if (K <= 8) { WD_CASE(8); }
  else if (K <= 16) { WD_CASE(16); }
  else if (K <= 32) { WD_CASE(32); }
  else if (K <= 64) { WD_CASE(64); }
  else return -1;
#undef WD_LAUNCH
#undef WD_CASE
  return (int)hipGetLastError();
}

// rbp[r * (nb + 1) + k] = first non-zero of row r with column >= k * cb (k = 0 .. nb), by binary
// search in the row's sorted column indices; a thread per (row, boundary)
template <typename I>
__global__ void __launch_bounds__(256) block_offsets_kernel(const int64_t* __restrict__ crow, const I* __restrict__ col,
                                                            int64_t m, int nb, int64_t cb, int64_t* __restrict__ rbp) {
  const int64_t total = m * (nb + 1);
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / (nb + 1);
    const int k = (int)(t - r * (nb + 1));
    int64_t lo = crow[r], hi = crow[r + 1];
    if (k == nb) {
      rbp[t] = hi;
      continue;
    }
    const int64_t c0 = (int64_t)k * cb;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)col[mid] < c0) lo = mid + 1;
      else hi = mid;
    }
    rbp[t] = lo;
  }
}

}  // namespace sysml_sd

extern "C" {

// per-row column-block offsets of a CSR pattern (see wdivmm_kernel): rbp m x (nb + 1) int64
int sysml_csr_block_offsets(int idx32, const void* crow, const void* col, int64_t m, int nb, int64_t cb, void* rbp,
                            void* stream) {
  if (m <= 0 || nb < 1 || cb < 1) return -1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t g = (m * (nb + 1) + 255) / 256;
  if (g > 65536) g = 65536;
  if (idx32)
    hipLaunchKernelGGL(sysml_sd::block_offsets_kernel<int32_t>, dim3((unsigned)g), dim3(256), 0, st,
                       static_cast<const int64_t*>(crow), static_cast<const int32_t*>(col), m, nb, cb,
                       static_cast<int64_t*>(rbp));
  else
    hipLaunchKernelGGL(sysml_sd::block_offsets_kernel<int64_t>, dim3((unsigned)g), dim3(256), 0, st,
                       static_cast<const int64_t*>(crow), static_cast<const int64_t*>(col), m, nb, cb,
                       static_cast<int64_t*>(rbp));
  return (int)hipGetLastError();
}

// wdivmm (as sysml_wdivmm) in nb column-block passes over the offsets rbp, V block k = columns
// [k * cb, (k + 1) * cb): each pass's V rows fit the MALL.  out zeroed by the caller.
int sysml_wdivmm_blocked(int dtype, int idx32, const void* crow, const void* col, const void* wv, const void* xv,
                         const void* U, const void* V, void* out, int64_t m, int K, int mode, double eps, int64_t nnz,
                         const void* rbp, int nb, int64_t ldv, void* stream) {
  if (K < 1 || K > 64 || nnz <= 0 || nb < 1 || rbp == nullptr || (mode == 1 && xv == nullptr)) return -1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const auto* cr = static_cast<const int64_t*>(crow);
  const auto* rb = static_cast<const int64_t*>(rbp);
  for (int k = 0; k < nb; ++k) {
    int rc;
#define WDB_T(T_)                                                                                              \
  (idx32 ? sysml_sd::launch_wd<T_, int32_t>(cr, static_cast<const int32_t*>(col), static_cast<const T_*>(wv),   \
                                            static_cast<const T_*>(xv), static_cast<const T_*>(U),              \
                                            static_cast<const T_*>(V), static_cast<T_*>(out), m, K, mode, eps,  \
                                            nnz, st, rb, nb, k, ldv)                                            \
         : sysml_sd::launch_wd<T_, int64_t>(cr, static_cast<const int64_t*>(col), static_cast<const T_*>(wv),   \
                                            static_cast<const T_*>(xv), static_cast<const T_*>(U),              \
                                            static_cast<const T_*>(V), static_cast<T_*>(out), m, K, mode, eps,  \
                                            nnz, st, rb, nb, k, ldv))
    if (dtype == 0) rc = WDB_T(float);
    else if (dtype == 1) rc = WDB_T(double);
    else return -1;
#undef WDB_T
    if (rc != 0) return rc;
  }
  return 0;
}

// Fused wdivmm (right form, see wdivmm_kernel): out (m x K, zeroed by the caller) for a CSR pattern
// (crow int64, col int32 if idx32 else int64), weights wv (nullptr: 1), x values xv (mode 1, the
// pattern's order), factors U (m x K), V (n x K).  dtype 0 fp32, 1 fp64.  -1: unsupported.
// ldv: row pitch of V in elements (>= K; a padded copy keeps every gathered row in one 64-B
// segment -- K = 10 fp32 rows of 40 B straddle two segments 60 % of the time)
int sysml_wdivmm(int dtype, int idx32, const void* crow, const void* col, const void* wv, const void* xv,
                 const void* U, const void* V, void* out, int64_t m, int K, int mode, double eps, int64_t nnz,
                 int64_t ldv, void* stream) {
  if (K < 1 || K > 64 || nnz <= 0 || (mode == 1 && xv == nullptr)) return -1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const auto* cr = static_cast<const int64_t*>(crow);
#define WD_T(T_)                                                                                             \
  (idx32 ? sysml_sd::launch_wd<T_, int32_t>(cr, static_cast<const int32_t*>(col), static_cast<const T_*>(wv),           \
                                  static_cast<const T_*>(xv), static_cast<const T_*>(U), static_cast<const T_*>(V), \
                                  static_cast<T_*>(out), m, K, mode, eps, nnz, st, nullptr, 0, 0, ldv)       \
         : sysml_sd::launch_wd<T_, int64_t>(cr, static_cast<const int64_t*>(col), static_cast<const T_*>(wv),           \
                                  static_cast<const T_*>(xv), static_cast<const T_*>(U), static_cast<const T_*>(V), \
                                  static_cast<T_*>(out), m, K, mode, eps, nnz, st, nullptr, 0, 0, ldv))
  if (dtype == 0) return WD_T(float);
  if (dtype == 1) return WD_T(double);
#undef WD_T
  return -1;
}

// dtype 0 = fp32, 1 = fp64.  Returns 0 on success, -1 on unsupported shape, else a hipError_t.
// idx32: the column indices are int32 (half the index bytes of the pass).
int sysml_sddmm2(int dtype, int idx32, const void* crow, const void* col, const void* U, const void* V, int64_t m,
                 int r, void* out, void* stream) {
  using namespace sysml_sd;
  if (r <= 0 || m <= 0) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const auto* cr = static_cast<const int64_t*>(crow);
  const bool aligned = (reinterpret_cast<uintptr_t>(U) % 16) == 0 && (reinterpret_cast<uintptr_t>(V) % 16) == 0;
#define SD_IDX(T_, NV_, u_, v_, o_)                                                                   \
  (idx32 ? launch<T_, NV_, int32_t>(cr, static_cast<const int32_t*>(col), u_, v_, m, r, o_, s)        \
         : launch<T_, NV_, int64_t>(cr, static_cast<const int64_t*>(col), u_, v_, m, r, o_, s))
  if (dtype == 0) {
    const auto* u = static_cast<const float*>(U);
    const auto* v = static_cast<const float*>(V);
    auto* o = static_cast<float*>(out);
    if (aligned && r % 4 == 0) return SD_IDX(float, 4, u, v, o);
    return SD_IDX(float, 1, u, v, o);
  }
  if (dtype == 1) {
    const auto* u = static_cast<const double*>(U);
    const auto* v = static_cast<const double*>(V);
    auto* o = static_cast<double*>(out);
    if (aligned && r % 2 == 0) return SD_IDX(double, 2, u, v, o);
    return SD_IDX(double, 1, u, v, o);
  }
#undef SD_IDX
  return -1;
}

int sysml_sddmm(int dtype, const void* crow, const void* col, const void* U, const void* V, int64_t m, int r,
                void* out, void* stream) {
  return sysml_sddmm2(dtype, 0, crow, col, U, V, m, r, out, stream);
}

}  // extern "C"
