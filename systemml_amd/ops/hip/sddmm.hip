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

extern "C" {

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
