// Micro-benchmark: the 7x7 kernel's inner loop (LDS fragment reads + v_mfma_f32_16x16x32_bf16,
// 3 products per pair, random data) for two wave shapes, to decide whether a larger wave tile pays:
//   w64  : 8 waves / CU (2 per SIMD), wave = 64 co x NPX 16-px blocks  (the product kernel's shape:
//          8 A + 2 NPX B fragment reads per 12 NPX MFMAs)
//   w128 : 4 waves / CU (1 per SIMD, up to 512 registers), wave = 128 co x NPX blocks
//          (16 A + 2 NPX B reads per 24 NPX MFMAs)
// No barriers, no global traffic after the prologue.  Prints TF/s of bf16 MFMA work and the
// f32-accurate equivalent (/3).  Timing-only tool; never part of the product library.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_mfma tools/micro/lds_mfma.hip && /tmp/lds_mfma
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int LDS_BYTES = 150 * 1024;

template <int CB, int NPX, bool FROM_LDS>
__device__ __forceinline__ void body(const char* lds, int lane, int pairs, float* out) {
  const int l16 = lane & 15, kg = lane >> 4;
  floatx4 acc[CB][NPX];
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int p = 0; p < NPX; ++p) acc[c][p] = floatx4{0.f, 0.f, 0.f, 0.f};
  // A: 4 ring slots of [2 planes][CB*16 co][16 B]; B: a halo of 4 planes x 1700 16-B slots
  constexpr int PLANE_W = CB * 16 * 16;
  constexpr int SLOT_W = 4 * PLANE_W;  // planes 2 khalf + {hi, lo}, as the product kernel's ring
  const char* wbase = lds + 2 * (kg & 1) * PLANE_W + l16 * 16;
  const char* hbase = lds + 4 * SLOT_W + 2 * (kg & 1) * 1700 * 16;
  const int hplane = 1700 * 16;
  bf16x8 ah[CB], al[CB];
  if (!FROM_LDS) {
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      ah[c] = *(const bf16x8*)(wbase + c * 256);
      al[c] = *(const bf16x8*)(wbase + PLANE_W + c * 256);
    }
  }
  bf16x8 bh0 = *(const bf16x8*)(hbase + l16 * 16), bl0 = *(const bf16x8*)(hbase + hplane + l16 * 16);
#pragma unroll 1
  for (int t = 0; t < pairs; ++t) {
    const char* wsl = wbase + ((t + (kg >> 1)) & 3) * SLOT_W;  // lanes 32-63: the pair's second tap
    const int toff = (t * 7) % 49 + (kg >> 1);                // halo slot offset of the tap
    bf16x8 bh[2], bl[2];
    if (FROM_LDS) {
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        ah[c] = *(const bf16x8*)(wsl + c * 256);
        al[c] = *(const bf16x8*)(wsl + PLANE_W + c * 256);
      }
      bh[0] = *(const bf16x8*)(hbase + (l16 + toff) * 16);
      bl[0] = *(const bf16x8*)(hbase + hplane + (l16 + toff) * 16);
    } else {
      bh[0] = bh0;
      bl[0] = bl0;
    }
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) {
      const int cur = pb & 1;
      if (pb + 1 < NPX) {
        if (FROM_LDS) {
          bh[cur ^ 1] = *(const bf16x8*)(hbase + ((pb + 1) * 16 + l16 + toff) * 16);
          bl[cur ^ 1] = *(const bf16x8*)(hbase + hplane + ((pb + 1) * 16 + l16 + toff) * 16);
        } else {
          bh[cur ^ 1] = bh[cur];
          bl[cur ^ 1] = bl[cur];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        acc[c][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c], bh[cur], acc[c][pb], 0, 0, 0);
        acc[c][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c], bl[cur], acc[c][pb], 0, 0, 0);
        acc[c][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[c], bh[cur], acc[c][pb], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int p = 0; p < NPX; ++p) s += acc[c][p][0] + acc[c][p][1] + acc[c][p][2] + acc[c][p][3];
  out[(blockIdx.x * blockDim.x + threadIdx.x)] = s;
}

__device__ void fill(char* lds, const uint4* src) {
  for (int i = threadIdx.x; i < LDS_BYTES / 16; i += blockDim.x) ((uint4*)lds)[i] = src[i & 4095];
  __syncthreads();
}

template <int NPX, bool FROM_LDS>
__global__ __launch_bounds__(512, 1) void k_w64(const uint4* src, float* out, int pairs) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fill(lds, src);
  body<4, NPX, FROM_LDS>(lds, threadIdx.x & 63, pairs, out);
}

template <int NPX, bool FROM_LDS>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_w128(const uint4* src, float* out,
                                                                                            int pairs) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fill(lds, src);
  body<8, NPX, FROM_LDS>(lds, threadIdx.x & 63, pairs, out);
}

template <class K>
static void run(const char* name, K kern, int threads, int cb, int npx, const uint4* src, float* out, int blocks = 1024,
                int pairs = 2000) {
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // warm up ~1.5 s so the clock settles under load, then time 10 launches
  const int warm = 60 * 1024 * 2000 / (blocks * pairs);
  for (int i = 0; i < warm; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), LDS_BYTES, 0, src, out, pairs);
  hipEventRecord(a);
  const int reps = 20 * 1024 * 2000 / (blocks * pairs);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), LDS_BYTES, 0, src, out, pairs);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double waves = (double)blocks * threads / 64;
  const double flops = waves * pairs * cb * npx * 3.0 * 2 * 16 * 16 * 32 * reps;
  printf("%-34s %7.3f ms/launch  %7.1f TF/s bf16  %6.1f TF/s f32-accurate\n", name, ms / reps, flops / (ms * 1e-3) / 1e12,
         flops / 3 / (ms * 1e-3) / 1e12);
}

int main() {
  uint4* src;
  float* out;
  hipMalloc(&src, 4096 * 16);
  hipMalloc(&out, 256 * 4 * 512 * 4);
  uint4* h = (uint4*)malloc(4096 * 16);
  srand(1);
  for (int i = 0; i < 4096; ++i) {
    unsigned w[4];
    for (int j = 0; j < 4; ++j) {
      // two bf16 values of magnitude ~1 with random mantissas and signs
      unsigned lo = 0x3f00u | (rand() & 0x7f) | ((rand() & 1) << 15) | ((rand() & 1) << 7);
      unsigned hi = 0x3f00u | (rand() & 0x7f) | ((rand() & 1) << 15) | ((rand() & 1) << 7);
      w[j] = lo | (hi << 16);
    }
    h[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  hipMemcpy(src, h, 4096 * 16, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run("w64  npx10 regs (8 waves/CU)", k_w64<10, false>, 512, 4, 10, src, out);
    run("w64  npx10 LDS  (8 waves/CU)", k_w64<10, true>, 512, 4, 10, src, out);
    run("w128 npx10 regs (4 waves/CU)", k_w128<10, false>, 256, 8, 10, src, out);
    run("w128 npx10 LDS  (4 waves/CU)", k_w128<10, true>, 256, 8, 10, src, out);
    run("w128 npx8  LDS  (4 waves/CU)", k_w128<8, true>, 256, 8, 8, src, out);
    run("w128 npx6  LDS  (4 waves/CU)", k_w128<6, true>, 256, 8, 6, src, out);
    run("w64  npx12 LDS  (8 waves/CU)", k_w64<12, true>, 512, 4, 12, src, out);
    // the product kernel's launch shape: one round of 252 workgroups x 196 tap pairs (~0.5 ms)
    run("w64  npx10 LDS  252 WG x 196 pairs", k_w64<10, true>, 512, 4, 10, src, out, 252, 196);
    run("w64  npx10 LDS  256 WG x 196 pairs", k_w64<10, true>, 512, 4, 10, src, out, 256, 196);
    run("w64  npx10 LDS  256 WG x 784 pairs", k_w64<10, true>, 512, 4, 10, src, out, 256, 784);
  }
  return 0;
}
