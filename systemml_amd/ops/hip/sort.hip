// Device sorts for order() / sort-based quantiles (reference: LibMatrixReorg.sort and the
// order() of ReorgOp -- the reference's GPU backend has no sort and falls back to the CPU).
//
//   * keys: one column of a (bf16 / fp32 / fp64) matrix, optionally gathered through a
//     permutation (multi-key order = stable passes from the last key to the first), widened to
//     fp64 in one pass (sort_keys_prep);
//   * sort: LSD radix sort of (fp64 key, int32 row) pairs on the device (rocPRIM's onesweep
//     radix sort, stable -- ties keep input order, as order() requires -- ascending or
//     descending) into caller-owned buffers; the scratch size is queried once per size;
//   * perm_compose: perm = base[perm] (a later, more significant key pass refines the order of
//     the earlier ones) and the 1-based index.return output in the matrix's value type.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

namespace sysml_st {

constexpr int NT = 256;

inline int grid_for(int64_t work) {
  int64_t g = (work + NT - 1) / NT;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

__device__ __forceinline__ double load_as_double(const void* X, int code, int64_t i) {
  if (code == 0) return (double)__uint_as_float(((uint32_t)((const uint16_t*)X)[i]) << 16);
  if (code == 1) return (double)((const float*)X)[i];
  return ((const double*)X)[i];
}

// keys[i] = X[perm[i] (or i), col]; iota (optional) = 0..n-1
__global__ void __launch_bounds__(NT) keys_kernel(const void* __restrict__ X, int code, int64_t lds, int64_t col,
                                                  const int32_t* __restrict__ perm, double* __restrict__ keys,
                                                  int32_t* __restrict__ iota, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t r = perm ? (int64_t)perm[i] : i;
    double v = load_as_double(X, code, r * lds + col);
    if (v == 0.0) v = 0.0;          // -0 sorts with +0 (a stable order must not split them)
    keys[i] = v;
    if (iota) iota[i] = (int32_t)i;
  }
}

// out_perm[i] = base[perm[i]] (base null: perm[i]); idx (optional, value type code) = out_perm + 1
__global__ void __launch_bounds__(NT) compose_kernel(const int32_t* __restrict__ perm, const int32_t* __restrict__ base,
                                                     int32_t* __restrict__ out_perm, void* __restrict__ idx, int code,
                                                     int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int32_t p = base ? base[perm[i]] : perm[i];
    if (out_perm) out_perm[i] = p;
    if (idx) {
      const double v = (double)p + 1.0;
      if (code == 2) ((double*)idx)[i] = v;
      else if (code == 1) ((float*)idx)[i] = (float)v;
      else {
        uint32_t u = __float_as_uint((float)v);
        u += 0x7fffu + ((u >> 16) & 1u);
        ((uint16_t*)idx)[i] = (uint16_t)(u >> 16);
      }
    }
  }
}

}  // namespace sysml_st

extern "C" {

int sysml_sort_keys_prep(int code, const void* X, int64_t lds, int64_t col, const int32_t* perm, double* keys,
                         int32_t* iota, int64_t n, void* stream) {
  using namespace sysml_st;
  if (n <= 0) return 0;
  if (code < 0 || code > 2 || col < 0 || col >= lds) return -1;
  hipLaunchKernelGGL(keys_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, X, code, lds, col, perm, keys,
                     iota, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// scratch bytes the pair sort of n elements needs
int64_t sysml_sort_pairs_scratch(int64_t n) {
  size_t bytes = 0;
  if (n <= 0) return 0;
  if (rocprim::radix_sort_pairs((void*)nullptr, bytes, (const double*)nullptr, (double*)nullptr,
                                (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n) != hipSuccess)
    return -1;
  return (int64_t)bytes;
}

// stable sort of (kin, vin) pairs by key into (kout, vout); desc = 1: descending
int sysml_sort_pairs(const double* kin, double* kout, const int32_t* vin, int32_t* vout, int64_t n, int desc,
                     void* scratch, int64_t scratch_bytes, void* stream) {
  if (n <= 0) return 0;
  if (n >= (1ll << 31)) return -1;
  size_t bytes = (size_t)scratch_bytes;
  hipError_t e;
  if (desc)
    e = rocprim::radix_sort_pairs_desc(scratch, bytes, kin, kout, vin, vout, (size_t)n, 0, 64,
                                       (hipStream_t)stream);
  else
    e = rocprim::radix_sort_pairs(scratch, bytes, kin, kout, vin, vout, (size_t)n, 0, 64, (hipStream_t)stream);
  return e == hipSuccess ? 0 : -2;
}

int sysml_perm_compose(const int32_t* perm, const int32_t* base, int32_t* out_perm, void* idx, int code, int64_t n,
                       void* stream) {
  using namespace sysml_st;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(compose_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, perm, base, out_perm, idx,
                     code, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
