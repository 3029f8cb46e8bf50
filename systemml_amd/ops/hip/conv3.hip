// Direct 3x3 / stride-1 / pad-1 convolution on MFMA for bf16 activations (the thirteen 3x3
// layers of ResNet-50 that keep their resolution, forward and backward data).  Reference:
// LibMatrixCuDNN.java conv2d / conv2d_backward_data (cuDNN) and libmatrixdnn.cpp's im2col + GEMM.
//
// out[img, m, oh, ow] = sum_{tap, ci} A[m, tap, ci] * in[img, ci, oh + kh - 1, ow + kw - 1]
//   forward        in = X (Cin = C),    A[f, tap, c] = W[f, c, kh, kw]                     (M = F)
//   backward data  in = dout (Cin = F), A[c, tap, f] = W[f, c, 2 - kh, 2 - kw]             (M = C)
// (the backward-data convolution of a 3x3 stride-1 pad-1 layer is the forward convolution of
// dout with the flipped, transposed filter).
//
// Unlike the implicit GEMM of dnn.hip, which gathers every (pixel, tap, channel) operand element
// from HBM with a bounds check (9 gathers per input element), a block here stages the input
// PATCH its 128 output pixels need -- the padded rows they touch, all columns, 32 channels --
// into LDS once per channel chunk, transposed to [position][channel] (96-B position pitch:
// the 16 positions one MFMA fragment reads fall in distinct bank groups).  The nine taps are
// then address offsets into that patch: each tap is one K=32 step whose B fragments are single
// 16-B LDS reads, with no index math and no bounds checks in the MFMA loop.  The filter tile of
// the next tap is loaded into registers while the current tap's MFMAs run and the next chunk's
// patch while the current chunk's nine taps run; one barrier per tap.
// Pixel tiles are 128 consecutive output pixels in (img, oh, ow) order and may span images:
// the patch rows are "padded rows" g = img * (H + 2) + ph, so the rows of consecutive images
// are consecutive and the zero padding between them comes for free from the bounds test of the
// staging pass.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>

namespace sysml_c3 {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;      // 4 waves, 2 x 2 over the output tile
constexpr int TN = 128;      // output pixels per tile
constexpr int CB = 32;       // channels per chunk (one MFMA K step per tap)
constexpr int CBP = 48;      // LDS pitch of a position / filter row, bf16 (96 B: conflict-free for ds_read_b128's lane groups)
constexpr int MAXIT = 8;     // patch items (position x 8 channels) per thread
constexpr int MAXPOS = NT * MAXIT / (CB / 8);

struct C3 {
  const uint16_t* in;   // N x Cin x H x W
  const uint16_t* A;    // M x 9 x Cin
  const float* bias;    // M, or null
  void* out;            // N x M x H x W (bf16, or fp32 when out_f32)
  int N, Cin, H, W, M, relu;
  int NP;               // N * H * W output pixels
  int PR;               // padded rows per patch
  int tm, tn;           // tiles along M and pixels
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <int TM, typename TO>
__global__ void __launch_bounds__(NT, 2) conv3_kernel(C3 c) {
  constexpr int FI = TM / 32;                          // 16-row fragments per wave (TM / 2 rows)
  constexpr int FJ = 4;                                // 16-column fragments per wave (64 pixels)
  constexpr int AV = TM * (CB / 8) / NT;               // 16-B filter vectors per thread per tap
  __shared__ __attribute__((aligned(16))) uint16_t As[2][TM * CBP];
  extern __shared__ __attribute__((aligned(16))) uint16_t patch[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = wg % c.tm, bn = wg / c.tm;            // the M tiles of one pixel tile are neighbours
  const int m0 = bm * TM, n0 = bn * TN;
  const int HW = c.H * c.W, W2 = c.W + 2, H2 = c.H + 2;
  const int g0 = (n0 / HW) * H2 + (n0 % HW) / c.W;     // first padded row (tap row 0)
  const int npos = c.PR * W2;
  const int nch = c.Cin / CB;
  // B fragment positions of this lane's four output columns
  int bpos[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    bpos[j] = 0;
    if (n < c.NP) {
      const int img = n / HW, p = n - img * HW, oh = p / c.W, ow = p - oh * c.W;
      bpos[j] = ((img * H2 + oh) - g0) * W2 + ow;
    }
  }
  // patch items of this thread: (position, 8-channel group); global offset of the position's
  // pixel without the channel term (-1: padding / past the last image), LDS offset (-1: none)
  int goff[MAXIT], loff[MAXIT];
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int q = it * NT + tid;
    goff[it] = -1;
    loff[it] = -1;
    if (q < npos * (CB / 8)) {
      const int c8 = q / npos, pos = q - c8 * npos;
      const int gr = g0 + pos / W2, pc = pos - (pos / W2) * W2;
      const int img = gr / H2, ih = gr - img * H2 - 1, iw = pc - 1;
      loff[it] = pos * CBP + c8 * 8;
      if (img < c.N && (unsigned)ih < (unsigned)c.H && (unsigned)iw < (unsigned)c.W)
        goff[it] = (img * c.Cin + c8 * 8) * HW + ih * c.W + iw;
    }
  }
  uint32_t pv[MAXIT][4];                               // staged patch values (bf16 pairs)
  auto load_patch = [&](int ch) {
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      uint16_t v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0;
      if (goff[it] >= 0) {
        const uint16_t* p = c.in + (int64_t)goff[it] + (int64_t)ch * CB * HW;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = p[(int64_t)e * HW];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) pv[it][e] = (uint32_t)v[2 * e] | ((uint32_t)v[2 * e + 1] << 16);
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int it = 0; it < MAXIT; ++it)
      if (loff[it] >= 0) *(uint4*)&patch[loff[it]] = uint4{pv[it][0], pv[it][1], pv[it][2], pv[it][3]};
  };
  // filter tile of step s = (chunk, tap): rows m0.., channels chunk*CB.. of the tap
  uint4 av[AV];
  auto load_a = [&](int s) {
    const int ch = s / 9, tap = s - ch * 9;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int e = v * NT + tid, r = e >> 2, part = e & 3;
      av[v] = uint4{0, 0, 0, 0};
      if (m0 + r < c.M)
        av[v] = *(const uint4*)(c.A + ((int64_t)(m0 + r) * 9 + tap) * c.Cin + ch * CB + part * 8);
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int e = v * NT + tid, r = e >> 2, part = e & 3;
      *(uint4*)&As[buf][r * CBP + part * 8] = av[v];
    }
  };
  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0, 0, 0, 0};
  const int S = nch * 9;
  load_patch(0);
  load_a(0);
  store_patch();
  store_a(0);
  __syncthreads();
  if (nch > 1) load_patch(1);
  const int kc = (lane >> 4) * 8;
  for (int s = 0; s < S; ++s) {
    const int ch = s / 9, tap = s - ch * 9;
    const bool more = s + 1 < S;
    if (more) load_a(s + 1);
    const uint16_t* Ab = As[s & 1];
    const int toff = (tap / 3) * W2 + (tap % 3);
    bf8 fa[FI], fb[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i) fa[i] = *(const bf8*)&Ab[(wr * (TM / 2) + i * 16 + (lane & 15)) * CBP + kc];
#pragma unroll
    for (int j = 0; j < FJ; ++j) fb[j] = *(const bf8*)&patch[(bpos[j] + toff) * CBP + kc];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (more) {
      if (tap == 8) {                                  // the next step starts a new channel chunk
        __syncthreads();                               // every wave is done with this patch
        store_patch();
        store_a((s + 1) & 1);
        __syncthreads();
        if (ch + 2 < nch) load_patch(ch + 2);
      } else {
        store_a((s + 1) & 1);
        __syncthreads();
      }
    }
  }
  // epilogue: bias, relu, NCHW store
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    if (n >= c.NP) continue;
    const int img = n / HW, p = n - img * HW;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * (TM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (m >= c.M) continue;
        float v = acc[i][j][r];
        if (c.bias != nullptr) v += c.bias[m];
        if (c.relu) v = v > 0.f ? v : 0.f;
        const int64_t o = ((int64_t)img * c.M + m) * HW + p;
        if constexpr (sizeof(TO) == 2) ((uint16_t*)c.out)[o] = f2bf(v);
        else ((float*)c.out)[o] = v;
      }
  }
}

// fp32 F x (C*9) filter -> bf16 tap-major operand: forward A[f, t, c] = W[f, c, t]; backward
// data (flip = 1) A[c, t, f] = W[f, c, 8 - t]
__global__ void __launch_bounds__(256) conv3_weight(const float* __restrict__ W, uint16_t* __restrict__ A, int F,
                                                    int C, int flip) {
  const int64_t total = (int64_t)F * C * 9;
  const int Cin = flip ? F : C;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(idx / (9 * Cin)), rem = (int)(idx - (int64_t)m * 9 * Cin);
    const int t = rem / Cin, ci = rem - t * Cin;
    const float w = flip ? W[((int64_t)ci * C + m) * 9 + (8 - t)] : W[((int64_t)m * C + ci) * 9 + t];
    A[idx] = f2bf(w);
  }
}

// padded rows a pixel tile spans (+ the two tap rows), cached per (N, H, W)
int patch_rows(int N, int H, int W) {
  static std::mutex mu;
  static int key[16][3], val[16], used = 0;
  std::lock_guard<std::mutex> g(mu);
  for (int i = 0; i < used; ++i)
    if (key[i][0] == N && key[i][1] == H && key[i][2] == W) return val[i];
  const int64_t HW = (int64_t)H * W, NP = (int64_t)N * HW;
  auto grow = [&](int64_t n) { return (n / HW) * (H + 2) + (n % HW) / W; };
  int64_t mx = 0;
  for (int64_t n0 = 0; n0 < NP; n0 += TN) {
    const int64_t n1 = n0 + TN - 1 < NP ? n0 + TN - 1 : NP - 1;
    const int64_t d = grow(n1) - grow(n0);
    if (d > mx) mx = d;
  }
  const int pr = (int)mx + 3;
  const int slot = used < 16 ? used++ : 15;
  key[slot][0] = N; key[slot][1] = H; key[slot][2] = W;
  val[slot] = pr;
  return pr;
}

}  // namespace sysml_c3

extern "C" {

// out (N x M x H x W; bf16, or fp32 when out_f32) = 3x3 stride-1 pad-1 convolution of `in`
// (N x Cin x H x W bf16) with the tap-major bf16 operand A (M x 9 x Cin), + bias (fp32 M, may be
// null), relu.  -1: shape not covered (Cin % 32, patch larger than MAXPOS positions).
int sysml_conv3s1(const void* in, const void* A, const float* bias, void* out, int out_f32, int N, int Cin, int H,
                  int W, int M, int relu, void* stream) {
  using namespace sysml_c3;
  if (N <= 0 || Cin <= 0 || Cin % CB || H <= 0 || W <= 0 || M <= 0) return -1;
  if ((int64_t)N * Cin * H * W >= (1LL << 31) || (int64_t)N * M * H * W >= (1LL << 40)) return -1;
  const int PR = patch_rows(N, H, W);
  if (PR * (W + 2) > MAXPOS) return -1;
  C3 c;
  c.in = (const uint16_t*)in;
  c.A = (const uint16_t*)A;
  c.bias = bias;
  c.out = out;
  c.N = N; c.Cin = Cin; c.H = H; c.W = W; c.M = M; c.relu = relu;
  c.NP = N * H * W;
  c.PR = PR;
  const int tmE = M <= 64 ? 64 : 128;
  c.tm = (M + tmE - 1) / tmE;
  c.tn = (c.NP + TN - 1) / TN;
  const size_t shm = (size_t)PR * (W + 2) * CBP * sizeof(uint16_t);
  const dim3 g((unsigned)(c.tm * c.tn)), t(NT);
  hipStream_t st = (hipStream_t)stream;
  if (tmE == 64) {
    if (out_f32) hipLaunchKernelGGL((conv3_kernel<64, float>), g, t, shm, st, c);
    else hipLaunchKernelGGL((conv3_kernel<64, uint16_t>), g, t, shm, st, c);
  } else {
    if (out_f32) hipLaunchKernelGGL((conv3_kernel<128, float>), g, t, shm, st, c);
    else hipLaunchKernelGGL((conv3_kernel<128, uint16_t>), g, t, shm, st, c);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int sysml_conv3_weight(const void* W, void* A, int F, int C, int flip, void* stream) {
  using namespace sysml_c3;
  const int64_t total = (int64_t)F * C * 9;
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(conv3_weight, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, (const float*)W,
                     (uint16_t*)A, F, C, flip);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
