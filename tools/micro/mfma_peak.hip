// Micro-benchmark: v_mfma_f32_32x32x16_bf16 throughput with operands in registers, in the conv
// kernels' accumulation pattern (2 channel blocks x NPB pixel blocks, 3 products per pair), random
// operands, 1 or 2 waves per SIMD.  Prints TF/s (bf16 MFMA flops) and the f32-accurate equivalent.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NPB>
__global__ __launch_bounds__(256, 2) void mfma_loop(const bf16x8* in, float* out, int iters) {
  const int lane = threadIdx.x;
  bf16x8 ah[2], al[2], bh[NPB], bl[NPB];
  for (int i = 0; i < 2; ++i) {
    ah[i] = in[(lane + 64 * i) & 255];
    al[i] = in[(lane + 64 * i + 7) & 255];
  }
  for (int i = 0; i < NPB; ++i) {
    bh[i] = in[(lane + 13 * i) & 255];
    bl[i] = in[(lane + 29 * i) & 255];
  }
  floatx16 acc[2][NPB];
  for (int c = 0; c < 2; ++c)
    for (int p = 0; p < NPB; ++p)
      for (int e = 0; e < 16; ++e) acc[c][p][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int p = 0; p < NPB; ++p)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        acc[c][p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], bh[p], acc[c][p], 0, 0, 0);
        acc[c][p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], bl[p], acc[c][p], 0, 0, 0);
        acc[c][p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[c], bh[p], acc[c][p], 0, 0, 0);
      }
  }
  float s = 0.f;
  for (int c = 0; c < 2; ++c)
    for (int p = 0; p < NPB; ++p)
      for (int e = 0; e < 16; ++e) s += acc[c][p][e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Same work with v_mfma_f32_16x16x32_bf16: 4 channel blocks of 16 x 12 pixel blocks of 16 (the
// same 64 x 192 output tile), 3 products per pair.
__global__ __launch_bounds__(256, 2) void mfma_loop16(const bf16x8* in, float* out, int iters) {
  const int lane = threadIdx.x;
  bf16x8 ah[4], al[4], bh[2], bl[2];
  for (int i = 0; i < 4; ++i) {
    ah[i] = in[(lane + 64 * i) & 255];
    al[i] = in[(lane + 64 * i + 7) & 255];
  }
  for (int i = 0; i < 2; ++i) {
    bh[i] = in[(lane + 13 * i) & 255];
    bl[i] = in[(lane + 29 * i) & 255];
  }
  floatx4 acc[4][12];
  for (int c = 0; c < 4; ++c)
    for (int p = 0; p < 12; ++p)
      for (int e = 0; e < 4; ++e) acc[c][p][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int p = 0; p < 12; ++p)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c], bh[p & 1], acc[c][p], 0, 0, 0);
        acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c], bl[p & 1], acc[c][p], 0, 0, 0);
        acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[c], bh[p & 1], acc[c][p], 0, 0, 0);
      }
  }
  float s = 0.f;
  for (int c = 0; c < 4; ++c)
    for (int p = 0; p < 12; ++p)
      for (int e = 0; e < 4; ++e) s += acc[c][p][e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = 2000, blocks = 256 * 2 * (argc > 1 ? atoi(argv[1]) : 4);
  bf16x8* in;
  float* out;
  hipMalloc(&in, 256 * sizeof(bf16x8));
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  bf16x8 h[256];
  srand(1);
  for (int i = 0; i < 256; ++i)
    for (int j = 0; j < 8; ++j) h[i][j] = (__bf16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL(mfma_loop<6>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double flops = (double)blocks * 4 /*waves*/ * iters * 6 * 2 * 3 * (32.0 * 32 * 16 * 2);
    printf("blocks %d: %.3f ms  %.1f TF/s bf16 MFMA  (= %.1f TF/s f32-accurate bf16x3)\n", blocks, ms,
           flops / ms / 1e9, flops / ms / 1e9 / 3);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL(mfma_loop16, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double flops = (double)blocks * 4 * iters * 48 * 3 * (16.0 * 16 * 32 * 2);
    printf("16x16x32 blocks %d: %.3f ms  %.1f TF/s bf16 MFMA  (= %.1f TF/s f32-accurate bf16x3)\n", blocks, ms,
           flops / ms / 1e9, flops / ms / 1e9 / 3);
  }
  return 0;
}
