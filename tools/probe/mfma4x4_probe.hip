// Operand / result layout of v_mfma_f32_4x4x4bf16_1k (16 independent 4x4x4 blocks) on gfx950:
// one-hot A with all-ones B (and the reverse) shows which lane / element feeds which output
// lane / register.  Also times a dependent-free stream of these MFMAs and of ds_read_b64_tr_b16.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out, int which) {
  const int cfg = blockIdx.x;          // one-hot source: lane cfg / 4, element cfg % 4
  const int l = threadIdx.x;
  const short one = 0x3f80;            // bf16 1.0
  s4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
  for (int e = 0; e < 4; ++e) {
    const bool hot = (l == cfg / 4) && (e == cfg % 4);
    if (which == 0) { a[e] = hot ? one : 0; b[e] = one; }
    else { a[e] = one; b[e] = hot ? one : 0; }
  }
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[(cfg * 64 + l) * 4 + r] = c[r];
}

__global__ void rate(float* out, int n) {
  s4 a = {(short)threadIdx.x, 1, 2, 3}, b = {1, 2, 3, (short)threadIdx.x};
  f4 c[8];
  for (int i = 0; i < 8; ++i) c[i] = f4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < n; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, b, c[i], 0, 0, 0);
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 64 * 4 * sizeof(float));
  float* h = new float[256 * 64 * 4];
  for (int which = 0; which < 2; ++which) {
    probe<<<256, 64>>>(d, which);
    hipMemcpy(h, d, 256 * 64 * 4 * sizeof(float), hipMemcpyDeviceToHost);
    printf("%s one-hot:\n", which == 0 ? "A" : "B");
    for (int cfg = 0; cfg < 256; ++cfg) {
      printf("  src lane %2d elem %d ->", cfg / 4, cfg % 4);
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
          if (h[(cfg * 64 + l) * 4 + r] != 0.f) printf(" (%d,%d)", l, r);
      printf("\n");
    }
  }
  // throughput: 1024 CUs' worth of waves, 8 independent accumulators per wave
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int n = 4096, blocks = 256 * 4;
  rate<<<blocks, 64>>>(d, 16);
  hipEventRecord(e0);
  rate<<<blocks, 64>>>(d, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfmas_per_simd = (double)n * 8;    // one wave per SIMD (1024 waves on 1024 SIMDs)
  printf("4x4x4bf16_1k: %.3f ms for %.0f MFMAs per SIMD -> %.2f ns per MFMA per SIMD\n", ms, mfmas_per_simd,
         ms * 1e6 / mfmas_per_simd);
  return 0;
}
