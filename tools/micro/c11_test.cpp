// Standalone check of launch_conv11_split (X0 path) against a CPU f64 conv (debugging aid).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../chainer_realtime_multi-person_pose_estimation_amd/csrc/common.hpp"
namespace op {
void set_error(const std::string&) {}
bool g_debug_sync = false;
int debug_after_launch(const char*, hipStream_t) { return 0; }
}
static unsigned short bf(float f) {  // round-to-nearest-even bf16
  unsigned u; memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return (unsigned short)(u >> 16);
}
static float fb(unsigned short s) { unsigned u = (unsigned)s << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
  const int h = 32, w = 48;
  std::vector<float> x(3 * h * w), wt(9 * 3 * 64), b(64);
  srand(3);
  for (auto& v : x) v = rand() / (float)RAND_MAX - 0.5f;
  for (auto& v : wt) v = (rand() / (float)RAND_MAX - 0.5f) * 0.5f;
  for (auto& v : b) v = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  if (getenv("PROBE")) {  // co = k*... : identity probes
    for (auto& v : wt) v = 0;
    for (auto& v : b) v = 1.0f;
    wt[(4 * 3 + 0) * 64 + 0] = 1.0f;   // co0 = x_c0 (center) + 1
    wt[(4 * 3 + 1) * 64 + 1] = 1.0f;   // co1 = x_c1 + 1
    wt[(0 * 3 + 0) * 64 + 2] = 1.0f;   // co2 = x_c0(y-1,x-1) + 1
    wt[(8 * 3 + 2) * 64 + 3] = 1.0f;   // co3 = x_c2(y+1,x+1) + 1
  }
  std::vector<unsigned short> x0((size_t)(h + 2) * (w + 2) * 32, 0);
  std::vector<float> xr(3 * h * w);
  for (int y = 0; y < h; ++y)
    for (int xx = 0; xx < w; ++xx)
      for (int c = 0; c < 3; ++c) {
        const float v = x[(c * h + y) * w + xx];
        const unsigned short hi = bf(v), lo = bf(v - fb(hi));
        unsigned short* p = &x0[((size_t)(y + 1) * (w + 2) + xx + 1) * 32];
        p[c] = hi;
        p[8 + c] = lo;
        xr[(c * h + y) * w + xx] = fb(hi) + fb(lo);
      }
  void *dx, *dw, *db, *dout;
  const size_t ob = (size_t)(h + 2) * (w + 2) * 256;
  hipMalloc(&dx, x0.size() * 2); hipMalloc(&dw, wt.size() * 4); hipMalloc(&db, 256); hipMalloc(&dout, ob);
  hipMemcpy(dx, x0.data(), x0.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dw, wt.data(), wt.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 256, hipMemcpyHostToDevice);
  hipMemset(dout, 0, ob);
  int rc = op::launch_conv11_split(nullptr, 0, 0, 0, 0, (const float*)dx, 1, h, w, (const float*)dw, (const float*)db,
                                   (float*)dout, 0);
  hipDeviceSynchronize();
  std::vector<unsigned short> out(ob / 2);
  hipMemcpy(out.data(), dout, ob, hipMemcpyDeviceToHost);
  double maxe = 0; int bad = 0;
  for (int y = 0; y < h; ++y)
    for (int xx = 0; xx < w; ++xx)
      for (int co = 0; co < 64; ++co) {
        double r = b[co];
        for (int t = 0; t < 9; ++t)
          for (int c = 0; c < 3; ++c) {
            const int yy = y - 1 + t / 3, xq = xx - 1 + t % 3;
            if (yy < 0 || yy >= h || xq < 0 || xq >= w) continue;
            r += (double)xr[(c * h + yy) * w + xq] * wt[(t * 3 + c) * 64 + co];
          }
        r = r > 0 ? r : 0;
        const unsigned short* p = &out[((size_t)(y + 1) * (w + 2) + xx + 1) * 128 + (co / 8) * 16];
        const double g = (double)fb(p[co % 8]) + fb(p[8 + co % 8]);
        const double e = fabs(g - r);
        if (e > maxe) maxe = e;
        if (e > 1e-4) ++bad;
      }
  printf("rc %d max err %.3g bad %d of %d\n", rc, maxe, bad, h * w * 64);
  for (int co = 0; co < 6; ++co) {
    printf("co %d:", co);
    for (int xx = 0; xx < 6; ++xx) {
      const unsigned short* p = &out[((size_t)(5 + 1) * (w + 2) + xx + 1) * 128 + (co / 8) * 16];
      printf(" %.4f", (double)fb(p[co % 8]) + fb(p[8 + co % 8]));
    }
    printf("\n");
  }
  printf("x c0 row5:");
  for (int xx = 0; xx < 6; ++xx) printf(" %.4f", xr[(0 * h + 5) * w + xx] + 1);
  printf("\nx c1 row5:");
  for (int xx = 0; xx < 6; ++xx) printf(" %.4f", xr[(1 * h + 5) * w + xx] + 1);
  printf("\n");
  return 0;
}
