// Sampled dense-dense product for the weighted quaternary operators (ops/quaternary.py;
// reference: LibMatrixMult.java#matrixMultWSLossSparseDense / wdivmm / wcemm, which loop over
// the non-zeros of W and compute dotProduct(U[i], V[j]) per non-zero).
//
// out[k] = <U[i_k], V[j_k]> for every non-zero k of a CSR pattern (crow/col int64).
// CDNA4 mapping: one 64-lane wavefront per CSR row (grid-stride over rows).  The wave stages
// U[i] (r <= 256 fp32) in its LDS slice once; then each lane owns one non-zero of the row
// and reads V[j] with 16-byte loads (r % 4 == 0) while the U values come from LDS as
// broadcast reads (every lane reads the same address -> no bank conflicts).  The kernel is a
// gather: its bound is HBM/L2 traffic of the V rows (r*4 bytes per non-zero), so U is read
// once per row instead of once per non-zero.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sysml_sd {

constexpr int WAVES = 4;
constexpr int RMAX = 256;

template <bool VEC4>
__global__ __launch_bounds__(WAVES * 64) void sddmm_kernel(const int64_t* __restrict__ crow,
                                                           const int64_t* __restrict__ col,
                                                           const float* __restrict__ U,
                                                           const float* __restrict__ V, int64_t m, int r,
                                                           float* __restrict__ out) {
  __shared__ float su[WAVES][RMAX];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  for (int64_t i = (int64_t)blockIdx.x * WAVES + w; i < m; i += (int64_t)gridDim.x * WAVES) {
    const int64_t b = crow[i], e = crow[i + 1];
    if (b == e) continue;                       // wave-uniform: whole wave skips empty rows
    for (int k = lane; k < r; k += 64) su[w][k] = U[i * r + k];
    __builtin_amdgcn_wave_barrier();            // LDS ops of one wave complete in order
    for (int64_t p = b + lane; p < e; p += 64) {
      const float* vr = V + col[p] * (int64_t)r;
      float acc = 0.f;
      if (VEC4) {
        for (int k = 0; k < r; k += 4) {
          const float4 v = *reinterpret_cast<const float4*>(vr + k);
          acc += su[w][k] * v.x + su[w][k + 1] * v.y + su[w][k + 2] * v.z + su[w][k + 3] * v.w;
        }
      } else {
        for (int k = 0; k < r; ++k) acc += su[w][k] * vr[k];
      }
      out[p] = acc;
    }
    __builtin_amdgcn_wave_barrier();            // LDS slice reused by this wave's next row
  }
}

}  // namespace sysml_sd

extern "C" {

// Returns 0 on success, -1 on unsupported shape, otherwise a hipError_t.
int sysml_sddmm(const void* crow, const void* col, const float* U, const float* V, int64_t m, int r,
                float* out, void* stream) {
  using namespace sysml_sd;
  if (r <= 0 || r > RMAX || m <= 0) return -1;
  int64_t blocks = (m + WAVES - 1) / WAVES;
  if (blocks > 256 * 64) blocks = 256 * 64;     // 8 XCDs x 32 CUs x 64: grid-stride beyond that
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool vec = (r % 4) == 0 && (reinterpret_cast<uintptr_t>(V) % 16) == 0;
  if (vec)
    hipLaunchKernelGGL(sddmm_kernel<true>, dim3((unsigned)blocks), dim3(WAVES * 64), 0, s,
                       (const int64_t*)crow, (const int64_t*)col, U, V, m, r, out);
  else
    hipLaunchKernelGGL(sddmm_kernel<false>, dim3((unsigned)blocks), dim3(WAVES * 64), 0, s,
                       (const int64_t*)crow, (const int64_t*)col, U, V, m, r, out);
  return (int)hipGetLastError();
}

}  // extern "C"
