// Micro-benchmark (round 4, the Winograd F(2x2,3x3) costing of DESIGN.md §9): how fast can the
// MFMA pipe run when every wave must also stream its A operand (weights) from L2 into VGPRs, at the
// bytes-per-MFMA ratio a kernel design implies?
//
// Each wave repeats: issue NLOAD 16-B loads per lane (1 KiB pieces of a weight window that stays
// L2/MALL-resident, walked like a conv's weight stream: consecutive pieces, wrapping in the window),
// then NMFMA v_mfma_f32_16x16x32_bf16 on the previous iteration's fragments (double-buffered, so
// the loads have a whole iteration to land), 3 products per pair like the bf16x3 convs.
// Design points (per wave, per step):
//   direct 3x3 conv_m16r: 32 co x 12 px blocks, one tap: 4 pieces / 72 MFMAs
//   Winograd F(2x2,3x3), wave = 32 co x 48 tiles, one position: 4 pieces / 18 MFMAs
//   Winograd, wave = 64 co x 16 tiles (U shared by 2 waves via LDS, counted as 4): 4 / 24 ...
// Prints, per point, the bf16 MFMA TF/s, the L2 bytes/clk/CU it moved, and what a Winograd
// F(2x2,3x3) kernel at that MFMA rate would give as f32-accurate direct-equivalent TF/s
// (x 2.25 / 3).  Operand registers only: no LDS, no transforms -- an UPPER bound for the fused
// Winograd kernel.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/l2s tools/micro/l2_mfma_stream.hip && /tmp/l2s
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) (void)(x)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NLOAD, int NMFMA, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void l2_mfma(const bf16x8* __restrict__ w, long window_pieces,
                                                         float* out, int iters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // each wave starts at its own offset of the window (different output-channel slices)
  long piece = ((long)blockIdx.x * WAVES + wave) * 97 % window_pieces;
  bf16x8 a[2][NLOAD];
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) a[0][i] = w[((piece + i) % window_pieces) * 64 + lane];
  piece += NLOAD;
  bf16x8 bh = a[0][0], bl = a[0][NLOAD - 1];
  floatx4 acc[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](bf16x8(&use)[NLOAD], bf16x8(&fill)[NLOAD]) {
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) {
      long p = piece + i;
      if (p >= window_pieces) p -= window_pieces;
      fill[i] = w[p * 64 + lane];
    }
    piece += NLOAD;
    if (piece >= window_pieces) piece -= window_pieces;
#pragma unroll
    for (int m = 0; m < NMFMA; m += 3) {
      const int k = (m / 3) % NLOAD, q = (m / 3) % 6;
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(use[k], bh, acc[q], 0, 0, 0);
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(use[k], bl, acc[q], 0, 0, 0);
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(use[(k + 1) % NLOAD], bh, acc[q], 0, 0, 0);
    }
  };
  for (int it = 0; it < iters; it += 2) {  // double-buffered: a step's loads feed the next step
    step(a[0], a[1]);
    step(a[1], a[0]);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NLOAD, int NMFMA, int WAVES>
static void run(const char* name, int blocks_per_cu, const bf16x8* w, long window_pieces, float* out, int cus) {
  const int iters = 4000;
  const int blocks = cus * blocks_per_cu;
  hipLaunchKernelGGL((l2_mfma<NLOAD, NMFMA, WAVES>), dim3(blocks), dim3(WAVES * 64), 0, 0, w, window_pieces, out, 10);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  hipLaunchKernelGGL((l2_mfma<NLOAD, NMFMA, WAVES>), dim3(blocks), dim3(WAVES * 64), 0, 0, w, window_pieces, out, iters);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double waves = (double)blocks * WAVES;
  const double mfma = waves * iters * (NMFMA / 3 * 3);
  const double tf = mfma * 16384.0 / (ms * 1e-3) / 1e12;
  const double bytes = waves * iters * NLOAD * 1024.0;
  // clock: assume the MFMA pipe's own rate under load is unknown; report bytes per CU per microsecond
  printf("%-44s waves/CU %2d  %5.1f KiB/%3d MFMA per wave-step: %7.1f TF/s bf16 (%.3f of 2500), "
         "L2->CU %6.1f GB/s/CU, Winograd-equiv (x2.25/3) %6.1f TF/s f32-accurate, direct-equiv (/3) %6.1f\n",
         name, (int)(waves / cus), NLOAD * 1.0, NMFMA, tf, tf / 2500.0, bytes / cus / (ms * 1e-3) / 1e9,
         tf * 2.25 / 3.0, tf / 3.0);
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const long window_bytes = argc > 1 ? atol(argv[1]) : 4L << 20;  // 4 MiB: one 256x256 layer's U
  const long window_pieces = window_bytes / 1024;
  bf16x8* w;
  float* out;
  CK(hipMalloc(&w, window_pieces * 1024));
  CK(hipMalloc(&out, (size_t)cus * 2 * 256 * 4));
  CK(hipMemset(w, 0x3c, window_pieces * 1024));
  printf("CUs %d, weight window %.1f MiB\n", cus, window_bytes / 1048576.0);
  // 2 blocks of 4 waves per CU = 2 waves per SIMD (conv_m16r's occupancy); 1 = one per SIMD (a
  // fused Winograd kernel holding 16 positions' accumulators needs the whole register file)
  run<4, 72, 4>("direct 3x3 (conv_m16r wave: 32co x 12blk)", 2, w, window_pieces, out, cus);
  run<4, 72, 4>("direct 3x3, one wave per SIMD", 1, w, window_pieces, out, cus);
  run<4, 36, 4>("4 pieces / 36 MFMA", 1, w, window_pieces, out, cus);
  run<4, 24, 4>("Winograd 64co x 16 tiles, U shared x2", 1, w, window_pieces, out, cus);
  run<4, 18, 4>("Winograd wave 32co x 48 tiles", 1, w, window_pieces, out, cus);
  run<4, 12, 4>("Winograd wave 32co x 32 tiles", 1, w, window_pieces, out, cus);
  run<8, 24, 4>("Winograd wave 64co x 16 tiles", 1, w, window_pieces, out, cus);
  run<2, 18, 4>("Winograd 32co x 48 tiles, U shared x2", 1, w, window_pieces, out, cus);
  return 0;
}
