// FETCH_SIZE calibration for the conv kernels' own HBM access patterns.
// MI355X_MICROARCH.md §HBM calibrates only the contiguous 16-B/lane stream (FETCH_SIZE = half the
// bytes); the halo loads of conv_m16_bf16x3 read one 64-B channel chunk of every 256-1024-B pixel
// record (4 waves = the chunk's four 16-B planes, 64 consecutive records per wave instruction) and
// conv_m16k_bf16x3 a 128-B chunk pair.  Each case below reads a known byte count into LDS with the
// same global_load_lds_dwordx4 and is run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`:
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip && ./fetch_calib
// Buffers are >= 512 MiB and each is read once, so the 256 MiB Infinity Cache cannot serve them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

// REC: record bytes; CHUNK: bytes read per record (CHUNK / 16 waves, wave w reads bytes
// [16w, 16w + 16) of 64 consecutive records per instruction).
template <int REC, int CHUNK>
__global__ __launch_bounds__(CHUNK / 16 * 64) void fetch_case(const char* src, long nrec) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long groups = nrec / 64;
  for (long g = blockIdx.x; g < groups; g += gridDim.x) {
    const char* p = src + (g * 64 + lane) * (long)REC + wave * 16;
    __builtin_amdgcn_global_load_lds(p, (__attribute__((address_space(3))) void*)(lds + wave * 1024), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// chunk-planar halo (round 3, conv_m16_bf16x3's stage buffers): wave w reads 64 consecutive 16-B
// pieces of plane w, the 4 planes `plane` bytes apart (a 1-KiB run per wave instruction)
__global__ __launch_bounds__(256) void fetch_planar(const char* src, long plane, long groups) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (long g = blockIdx.x; g < groups; g += gridDim.x) {
    const char* p = src + wave * plane + (g * 64 + lane) * 16L;
    __builtin_amdgcn_global_load_lds(p, (__attribute__((address_space(3))) void*)(lds + wave * 1024), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// streams a separate 1 GiB buffer between cases (evicts the Infinity Cache)
__global__ __launch_bounds__(256) void flush(const float4* p, long n, float* sink) {
  float4 a = {0, 0, 0, 0};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) {
    const float4 v = p[i];
    a.x += v.x;
  }
  if (a.x == 12345.0f) sink[0] = a.x;
}

static char* g_flush = nullptr;
static float* g_sink = nullptr;

template <int REC, int CHUNK>
static void run(const char* buf, size_t known) {
  const long nflush = (1L << 30) / 16;
  hipLaunchKernelGGL(flush, dim3(4096), dim3(256), 0, 0, (const float4*)g_flush, nflush, g_sink);
  CK(hipDeviceSynchronize());
  const long nrec = (long)(known / CHUNK);
  hipLaunchKernelGGL((fetch_case<REC, CHUNK>), dim3(2048), dim3(CHUNK / 16 * 64), CHUNK / 16 * 1024, 0, buf, nrec);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("fetch_case<%d, %d>: records %ld, known bytes %zu (%.1f MB), buffer span %.1f MB\n", REC, CHUNK, nrec,
         known, known / 1e6, (double)nrec * REC / 1e6);
}

int main() {
  const size_t known = (size_t)512 << 20;  // bytes actually read per case
  const size_t span = known * 8;           // largest case: 64 B of every 512-B record
  char* buf = nullptr;
  CK(hipMalloc(&buf, span));
  CK(hipMemset(buf, 1, span));
  CK(hipMalloc(&g_flush, 1L << 30));
  CK(hipMemset(g_flush, 0, 1L << 30));
  CK(hipMalloc(&g_sink, 64));
  CK(hipDeviceSynchronize());
  run<16, 16>(buf, known);     // the guide's calibrated case: contiguous 16-B/lane stream
  run<64, 64>(buf, known);     // whole 64-B records, strided per instruction, contiguous per 4 waves
  run<512, 64>(buf, known);    // 7x7 halo: 64-B chunk of a 512-B (128-channel) pixel
  run<256, 64>(buf, known / 2);  // 64-B chunk of a 256-B (64-channel) pixel
  run<512, 128>(buf, known / 2);  // 3x3 halo: 128-B chunk pair of a 512-B pixel
  {
    const long nflush = (1L << 30) / 16;
    hipLaunchKernelGGL(flush, dim3(4096), dim3(256), 0, 0, (const float4*)g_flush, nflush, g_sink);
    CK(hipDeviceSynchronize());
    const long plane = (long)(known / 4), groups = plane / 1024;
    hipLaunchKernelGGL(fetch_planar, dim3(2048), dim3(256), 4096, 0, buf, plane, groups);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    printf("fetch_planar: 4 planes x %ld B, known bytes %zu (%.1f MB)\n", plane, known, known / 1e6);
  }
  CK(hipFree(buf));
  CK(hipFree(g_flush));
  return 0;
}
