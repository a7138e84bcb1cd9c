// Micro-benchmark (round 4): throughput of v_mfma_f32_16x16x16_bf16 against v_mfma_f32_16x16x32_bf16
// on gfx950, operands in registers, 2 waves per SIMD, 8 independent accumulators per wave (the 7x7
// kernel's odd 49th tap would run at K = 16 instead of pairing with a zero tap).
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/mfma_k16 tools/micro/mfma_k16.hip && tools/micro/mfma_k16
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <bool K32>
__global__ __launch_bounds__(512, 1) void mfma_loop(const float* in, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int e = 0; e < 8; ++e) {
    a8[e] = (__bf16)(in[(lane + e) & 63]);
    b8[e] = (__bf16)(in[(lane * 3 + e) & 63]);
  }
  for (int e = 0; e < 4; ++e) {
    a4[e] = a8[e];
    b4[e] = b8[e];
  }
  floatx4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (K32) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[i], 0, 0, 0);
      else acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool K32>
static void run(int cus, const float* in, float* out) {
  const int iters = 20000;
  hipLaunchKernelGGL(mfma_loop<K32>, dim3(cus), dim3(512), 0, 0, in, out, 100);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL(mfma_loop<K32>, dim3(cus), dim3(512), 0, 0, in, out, iters);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double n_mfma = (double)cus * 8 * iters * 8;  // waves x iters x 8
  const double flop = n_mfma * 2.0 * 16 * 16 * (K32 ? 32 : 16);
  printf("%s: %.3f ns per MFMA per SIMD (%.1f TF/s bf16)\n", K32 ? "16x16x32_bf16" : "16x16x16_bf16",
         ms * 1e6 / (n_mfma / (cus * 4)), flop / (ms * 1e-3) / 1e12);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  float *in, *out;
  (void)hipMalloc(&in, 64 * 4);
  (void)hipMalloc(&out, (size_t)p.multiProcessorCount * 512 * 4);
  float h[64];
  for (int i = 0; i < 64; ++i) h[i] = 0.25f + 0.01f * i;
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  run<true>(p.multiProcessorCount, in, out);
  run<false>(p.multiProcessorCount, in, out);
  run<true>(p.multiProcessorCount, in, out);
  run<false>(p.multiProcessorCount, in, out);
  return 0;
}
