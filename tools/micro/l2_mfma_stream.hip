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

// The fused Winograd F(2x2,3x3) design of DESIGN.md §9, as its two phases per 32-channel input
// chunk of one workgroup (4 waves, one per SIMD; wave = 32 output channels x 48 tiles, the
// workgroup's 4 waves share the 48 tiles' V through LDS):
//  * GEMM phase: per transform position (16): A = U fragments (2 channel blocks x hi/lo = 4 x 16 B
//    per lane) streamed from an L2-resident window, B = V fragments (3 tile blocks x hi/lo = 6
//    ds_read_b128) from LDS, 18 MFMAs (2 x 3 blocks x 3 split products) into 96 accumulators;
//  * transform phase: 192 work items (tile, 8 input channels) over the workgroup's 256 lanes, each
//    reading its 4x4 x 8-channel f32 input window from LDS (32 ds_read_b128, one 4-channel half at
//    a time), B^T d B in place (32 add/sub per channel), the hi/lo bf16 split of the 128 values,
//    and 64 ds_write_b64 into V.
// Timed separately and together (serialised by barriers, as with one V buffer): the direct-
// equivalent TF/s of the whole chunk is what a real kernel could at best reach.
typedef float floatx4v __attribute__((ext_vector_type(4)));
template <bool GEMM, bool XFORM, int TB>
__global__ __launch_bounds__(256, 1) void wino_core(const bf16x8* __restrict__ w, long window_pieces, float* out,
                                                   int iters) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const halo = lds;               // 48 KiB of f32 input window
  char* const vbuf = lds + 48 * 1024;   // 96 KiB: V [16 pos][48 tiles][32 ci] hi/lo
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  long piece = ((long)blockIdx.x * 4 + wave) * 97 % window_pieces;
  for (int i = tid; i < 144 * 1024 / 16; i += 256) ((floatx4v*)lds)[i] = floatx4v{0.5f, 0.25f, 0.125f, 1.f};
  __syncthreads();
  floatx4 acc[16][2 * TB];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int i = 0; i < 2 * TB; ++i) acc[p][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  float sink = 0.f;
  for (int it = 0; it < iters; ++it) {
    if (XFORM && tid < 64 * TB) {
      // item: 4x4 window of 8 channels (16 px x 32 B), one 4-channel half at a time (16 floatx4 in
      // place: with 384 accumulator registers live, a whole item's window does not fit)
      const char* src = halo + (tid * 32) % (48 * 1024 - 512);
      char* dst = vbuf + (tid % (16 * TB)) * 64 + (tid / (16 * TB)) * 16;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        floatx4v d[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) d[i] = *(const floatx4v*)(src + i * 32 * 48 % 8192 + 16 * h);
        // B^T d B in place: columns (r0-r2, r1+r2, r2-r1, r1-r3), then rows the same way
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const floatx4v x0 = d[c], x1 = d[4 + c], x2 = d[8 + c], x3 = d[12 + c];
          d[c] = x0 - x2;
          d[4 + c] = x1 + x2;
          d[8 + c] = x2 - x1;
          d[12 + c] = x1 - x3;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const floatx4v x0 = d[4 * r], x1 = d[4 * r + 1], x2 = d[4 * r + 2], x3 = d[4 * r + 3];
          d[4 * r] = x0 - x2;
          d[4 * r + 1] = x1 + x2;
          d[4 * r + 2] = x2 - x1;
          d[4 * r + 3] = x1 - x3;
        }
        // hi/lo split of each position's 4 channels -> 8 B into the hi plane, 8 B into the lo plane
#pragma unroll
        for (int p = 0; p < 16; ++p) {
          __bf16 hb[4], lb[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hb[e] = (__bf16)d[p][e];
            lb[e] = (__bf16)(d[p][e] - (float)hb[e]);
          }
          uint2 qh, ql;
          qh.x = *(unsigned short*)&hb[0] | ((unsigned)*(unsigned short*)&hb[1] << 16);
          qh.y = *(unsigned short*)&hb[2] | ((unsigned)*(unsigned short*)&hb[3] << 16);
          ql.x = *(unsigned short*)&lb[0] | ((unsigned)*(unsigned short*)&lb[1] << 16);
          ql.y = *(unsigned short*)&lb[2] | ((unsigned)*(unsigned short*)&lb[3] << 16);
          *(uint2*)(dst + p * 6144 + 8 * h) = qh;
          *(uint2*)(dst + p * 6144 + 3072 + 8 * h) = ql;
        }
      }
    }
    if (XFORM) __syncthreads();
    if (GEMM) {
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        __builtin_amdgcn_sched_barrier(0);  // one position's loads at a time (no hoisting: spills)
        bf16x8 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          long q = piece + i;
          if (q >= window_pieces) q -= window_pieces;
          a[i] = w[q * 64 + lane];
        }
        piece += 4;
        if (piece >= window_pieces) piece -= window_pieces;
        const char* vb = vbuf + p * 6144 + lane * 16;
        bf16x8 b[2 * TB];
#pragma unroll
        for (int i = 0; i < 2 * TB; ++i) b[i] = *(const bf16x8*)(vb + i * 1024);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int tb = 0; tb < TB; ++tb) {
            floatx4& c = acc[p][cb * TB + tb];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], b[2 * tb], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], b[2 * tb + 1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb + 1], b[2 * tb], c, 0, 0, 0);
          }
      }
    }
    if (XFORM) __syncthreads();
  }
  float s = sink;
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int i = 0; i < 2 * TB; ++i) s += acc[p][i][0] + acc[p][i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool GEMM, bool XFORM, int TB>
static void run_wino(const char* name, const bf16x8* w, long window_pieces, float* out, int cus) {
  const int iters = 2000;
  auto k = wino_core<GEMM, XFORM, TB>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024));
  hipLaunchKernelGGL(k, dim3(cus), dim3(256), 144 * 1024, 0, w, window_pieces, out, 10);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(k, dim3(cus), dim3(256), 144 * 1024, 0, w, window_pieces, out, iters);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  // direct-equivalent work of one chunk of one workgroup: 128 co x (16 TB tiles x 4 px) x 32 ci x 9 taps x 2
  const double fl = (double)cus * iters * 128.0 * (64 * TB) * 32 * 9 * 2;
  printf("%-52s %8.3f us per chunk  direct-equivalent %7.1f TF/s f32-accurate\n", name, ms * 1e3 / iters,
         fl / (ms * 1e-3) / 1e12);
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
  // the fused F(2x2,3x3) chunk, phase by phase (one workgroup of 4 waves per CU)
  run_wino<true, false, 3>("Winograd chunk, 48 tiles/wave: GEMM phase (spills)", w, window_pieces, out, cus);
  run_wino<false, true, 3>("Winograd chunk, 48 tiles/wave: transform phase", w, window_pieces, out, cus);
  run_wino<true, true, 3>("Winograd chunk, 48 tiles/wave: both (spills)", w, window_pieces, out, cus);
  run_wino<true, false, 2>("Winograd chunk, 32 tiles/wave: GEMM phase (U L2, V LDS)", w, window_pieces, out, cus);
  run_wino<false, true, 2>("Winograd chunk, 32 tiles/wave: transform phase", w, window_pieces, out, cus);
  run_wino<true, true, 2>("Winograd chunk, 32 tiles/wave: both", w, window_pieces, out, cus);
  return 0;
}
