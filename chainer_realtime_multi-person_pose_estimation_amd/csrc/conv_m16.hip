// 7x7 stage convs on v_mfma_f32_16x16x32_bf16 (the default 7x7 kernel; see conv_big.hip for the
// shared halo / weight-ring scheme).  Own translation unit: built with the Makefile's FLAGS_conv_m16.
#include "conv_big.hpp"

// Round 5: the weight ring is staged by waves 0-3 only (one wave per SIMD, 4 pieces per tap pair),
// so on every SIMD one wave issues the LDS-DMA while its partner keeps issuing MFMAs; with all 8
// waves staging 2 pieces each, both waves of a SIMD paused for the DMA issue after the same ring
// barrier.  7x7 class -0.6..-1.1 % in 6 interleaved rounds on two boxes
// (profiles/r05/ab_r05c_7x7_dma_placement.log, ab_r05d_dmahalf.log); -DM16_DMA_HALF=0 restores it.
#ifndef M16_DMA_HALF
#define M16_DMA_HALF 1
#endif
// taps of the staggered kernel's weight ring: 6 (three pair slots, 28-KiB halo planes) by default;
// 4 (32-KiB planes) for A/Bs
#ifndef M16_STAG_RING
#define M16_STAG_RING 6
#endif
static_assert(M16_STAG_RING == 6 || M16_STAG_RING == 4, "staggered ring: 4 or 6 taps");
// M16_PF_L2 (round 6, A/B): waves 4-7 (the staggered half that stages no weights) pull chunk c + 1's
// halo lines into L2 during pairs kPfPair .. kPfPair + 3 of chunk c, by 4-byte LDS-DMAs into a
// spare KiB of their plane (nh < 28), so the chunk-boundary DMA reads L2 instead of MALL / HBM.
#ifndef M16_PF_L2
#define M16_PF_L2 0
#endif

namespace op {

#if M16_STAMPS
// Diagnostic build only (tools/build_variant.sh ... -DM16_STAMPS=1; never the product library):
// per-wave s_memtime sums over each 7x7 launch, added into these counters by vector atomics and
// read back by launch_m16_7x7 (OP_M16_STAMPS=1): [0] whole wave, [1] chunk boundaries (halo
// reload: two barriers + DMA wait), [2] pair starts (vmcnt wait, ring barrier, DMA issue, A / B
// fragment reads up to the first MFMA's issue), [3] pair loops incl. boundaries, [4] epilogue,
// [5] pairs, [6] waves, [7] after the pair loop before the epilogue (final vmcnt wait); pair start
// split: [8] the ring vmcnt wait, [9] the ring barrier, [10] the weight DMA issue
// [11] chunk boundaries' first barrier, [12] their halo DMA issue (the rest of [1]: DMA wait + barrier)
__device__ unsigned long long g_m16_st[14];
#define M16_T() __builtin_amdgcn_s_memtime()
#endif

// ---- 7x7 on v_mfma_f32_16x16x32_bf16, raster tiles (the default 7x7 kernel) ----
// K = 32 of the 16x16x32 form is fed with a tap PAIR of one 16-channel chunk: lane group
// g = lane / 16 holds k = 8g..8g+7 = tap t + g/2, channel half g%2, so halo and weight ring keep
// the layout above (the odd last tap pairs with zero weights).  Under the power limit this MFMA
// sustains ~15 % more FLOP/s than 32x32x16 on random data (tools/micro/mfma_peak.hip); in the
// network it runs the 7x7 layers 6.7 % faster per frame than conv_big_bf16x3<7,..,RASTER>.  Wave:
// 64 channels (4 blocks of 16) x NPX 16-pixel blocks of a raster tile; D rows are channels (4
// consecutive per lane), columns pixels.  Halo, 4-slot weight ring (one barrier per tap pair, 2
// taps ahead) and XCD-aware block order as conv_big_bf16x3<7,..,RASTER>.
// DEEP (small tiles, halo planes <= 16 KiB): a 12-slot weight ring staged 5 tap pairs ahead instead
// of 4 slots / 1 pair.  A small tile's workgroup does little MFMA work per tap pair, so with one pair
// of prefetch it waits on the weight fetch (L2 / HBM latency) every pair: the single-frame and
// single-crop launches.
// STAG (round 5): the two waves of a SIMD run half a tap pair apart.  Waves 0-3 (which stage the
// ring) meet the ring barrier at the start of their pair p, waves 4-7 in the middle of their pair
// p - 1 (after block NPX / 2), so when one half starts a pair -- vmcnt wait, barrier, DMA issue, A / B
// fragment reads, the 28 % of a wave's time before its first MFMA (profiles/r05/m16_stamps_*) -- its
// SIMD partner is halfway through its MFMA stream.  The slot staged at the barrier held pair p - 1,
// whose A fragments waves 4-7 read into registers when they started it, so the 4-tap ring would
// do; measured, the 32-KiB-plane form is faster with a 6-tap ring (three pair slots) in 28-KiB halo
// planes (7x7 -1.8 %, profiles/r05/ab_r05l_*) than with the 4-tap ring (+1.4 %, ab_r05o_*), so it
// takes that where nh <= 28 (the 46 x 46 batch rasters: 27); the deep 12-tap ring (small tiles:
// one frame's split-K launches) is staggered as it is (one frame's 7x7 -4.7 %).
// CIRC (round 6): no chunk-boundary drain for tiles of one frame.  Each halo
// plane is a circular buffer of CP = HPLANE / 1 KiB pieces; chunk c's np pieces sit at physical
// pieces cbase_c .. cbase_c + np - 1 (mod CP), chunk c + 1 right after them, and a B fragment's
// slot is wrapped (one v_min_u32 per block) on its way into the LDS address.  Waves 4-7 (which
// stage no weights) each stream one plane of chunk c + 1 in the background, one 1-KiB piece at a
// time, in three regions: R1, the pieces that overlay no live data, during pairs 2-20 of chunk c;
// R2, those overlaying chunk c's halo rows 0-5 (read only by taps with ky <= 5, i.e. pairs <= 20),
// during pairs 21-22; R3, those overlaying chunk c's later rows, during pairs 0-1 of chunk c + 1 --
// allowed only when R3 holds rows that chunk c + 1 first reads with ky >= 1 (pair 3 on).  A piece
// issued by waves 4-7 at the start of pair p is waited for (vmcnt) at their start of pair p + 1 and
// ordered by the ring barrier they meet in its middle, so every wave may read it from pair p + 2;
// the staggered ring barriers then run on across chunk boundaries.  Tiles that cross a frame
// border (two row sets, ~30 % at 640 px on 46 x 46 maps) or whose R3 would hold early rows keep
// the drain.  Bit-identical: the same MFMAs on the same data in the same order.
// LIN (round 6): chunk-planar input whose halo pitch is the padded width (pad = R, the tight
// pitch): a halo slot's source is one linear pixel index (a compare + select per piece where the
// tile crosses a frame) instead of the row / column cursor with its per-piece carry loop.
// One tile (block id lin) of the launch; the kernel below runs one, or (PERS) a loop of them.
template <int KS, int NPX, bool DEEP, bool STAG, bool CIRC, bool LIN>
__device__ __forceinline__ void m16_tile(const SplitConvShape& s, const SplitConvGroup& g0, const SplitConvGroup& g1,
                                         const BigTiling& tl, const int lin) {
  static_assert(!STAG || M16_DMA_HALF, "staggered halves: waves 4-7 must not stage the ring");
  static_assert(!CIRC || (STAG && !DEEP && KS == 7), "circular halo: the staggered 7x7 ring kernel only");
  static_assert(!LIN || (!DEEP && !CIRC), "linear halo sources: the drained 4- / 6-tap ring kernels");
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  constexpr int CW = 128, PG = 4;        // 2 channel halves x 4 pixel groups = 8 waves
  constexpr int PLANE_W = CW * 16;
  constexpr int SLOT_W = 4 * PLANE_W;
  constexpr int RING = DEEP ? 12 : (STAG ? M16_STAG_RING : 4);  // taps; even, so a pair never wraps
  constexpr int AHEAD = DEEP ? 5 : 1;               // tap pairs staged ahead of the one being computed
  constexpr int CAP = PG * NPX * 16;
  // halo planes at a fixed stride (raster_tiling keeps nh <= 32; DEEP: nh <= 16; STAG: nh <= 28),
  // placed first so a lane's lo-plane read is its hi-plane address + an immediate offset; the
  // weight ring follows
  constexpr int HPLANE = (DEEP ? 16 : (STAG ? (M16_STAG_RING == 6 ? 28 : 32) : 32)) * 1024;
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [halo: 4 planes][W ring]

  int unit, widx;
  if (tl.xpu) {
    // XCD set su runs weight sets su*P .. su*P+P-1 (P = tl.pair, default 1); with P > 1 (Mconv1: its
    // two channel tiles read the same 192-channel input) one pixel tile's P channel tiles are
    // consecutive slots of one XCD, so its halo is fetched once into that XCD's L2
    const int xcd = lin & 7, slot = lin >> 3;
    const int P = tl.pair > 1 ? tl.pair : 1;
    const int su = xcd / tl.xpu, q = slot / P, xo = xcd - su * tl.xpu;
    unit = su * P + (slot - q * P);
    widx = q * tl.xpu + xo;
  } else {
    unit = lin / tl.per_unit;
    widx = lin - unit * tl.per_unit;
  }
  if (unit >= tl.units || widx >= tl.per_unit) return;
  const int grp = unit / tl.co_tiles;
  const int co0 = (unit - grp * tl.co_tiles) * CW;
  const SplitConvGroup g = grp == 0 ? g0 : g1;
  if (co0 >= g.cop) return;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ch = wave / PG, pg = wave % PG;
  const int l16 = lane & 15, kg = lane >> 4;  // k group: tap t + kg/2, channel half kg%2
  const int tsel = kg >> 1, khalf = kg & 1;
  char* const halo = lds;
  char* const ring = lds + 4 * HPLANE;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  // a chunk's 4 halo planes: 16-B pieces of each pixel record, or (chunk-planar input) 4 planes of
  // contiguous rows, so each wave's 64 x 16 B read is one 1-KiB run
  const int64_t in_pc = split_piece_stride(s.in_planar, hp_in, wp_in);
  const int64_t in_px = split_pixel_stride(s.in_planar, s.cs_in);

  // weights: wave w copies piece w: plane w / 2, channels co0 + 64*(w % 2) + 0..63
  const int64_t wplane = (int64_t)g.cop * 16;
  const int64_t wstep = 4 * wplane;
  const char* const wsrc = (const char*)g.w + (wave / 2) * wplane + ((int64_t)co0 + 64 * (wave % 2) + lane) * 16;
  const int wdst = (wave / 2) * PLANE_W + (wave % 2) * 1024;
#if M16_DMA_HALF  // waves 0-3 (one per SIMD) copy pieces w and w + 4, waves 4-7 only compute
  const char* const wsrc4 = (const char*)g.w + ((wave + 4) / 2) * wplane + ((int64_t)co0 + 64 * (wave % 2) + lane) * 16;
  const int wdst4 = ((wave + 4) / 2) * PLANE_W + (wave % 2) * 1024;
#endif
  // split-K (tl.ksplit > 1): this workgroup runs input chunks [cb0, cb1)
  const int nsplit = tl.ksplit > 1 ? tl.ksplit : 1;
  const int split = nsplit > 1 ? (int)blockIdx.y : 0;
  const int cb0 = split * (s.c16 / nsplit), cb1 = cb0 + s.c16 / nsplit;
  // ring index it = chunk * KSQP + tap over an even tap count per chunk: the odd 49th tap pairs with
  // a padding tap whose weights are staged from device zeros, so every pair is a full K = 32 step
  // (no per-pair masking of the A fragments)
  constexpr int KSQP = KSQ + (KSQ & 1);
  constexpr int kDmaPerPair = M16_DMA_HALF ? 4 : 2;  // weight pieces a (staging) wave issues per tap pair
  const int n_it = cb1 * KSQP;
  const char* const zsrc = (const char*)tl.zeros + lane * 16;
  auto stage_w = [&](int it) {
    char* dst = ring + ((unsigned)it % RING) * SLOT_W;
    if (it >= n_it) it = n_it - 1;
    const int c = it / KSQP, tp = it - c * KSQP;
#if M16_DMA_HALF
    if (wave < 4) {
      glds16(tp < KSQ ? (const void*)(wsrc + (int64_t)(c * KSQ + tp) * wstep) : (const void*)zsrc, dst + wdst);
      glds16(tp < KSQ ? (const void*)(wsrc4 + (int64_t)(c * KSQ + tp) * wstep) : (const void*)zsrc, dst + wdst4);
    }
#else
    glds16(tp < KSQ ? (const void*)(wsrc + (int64_t)(c * KSQ + tp) * wstep) : (const void*)zsrc, dst + wdst);
#endif
  };

  // the tile's geometry: pixels [P0, P1] of the batch, frame / first row, the second frame's rows
  struct Tile {
    int P0, P1, frame, y0, fb, rowsA;
  };
  auto tile_of = [&](int widx) {
    Tile T;
    if (tl.fa_tiles) {  // frame-aligned raster tiles (wide maps): one frame per tile, last one partial
      const int f = widx / tl.fa_tiles;
      T.P0 = f * tl.hw + (widx - f * tl.fa_tiles) * CAP;
      T.P1 = min(T.P0 + CAP, (f + 1) * tl.hw) - 1;
    } else {
      T.P0 = widx * CAP;
      T.P1 = min(T.P0 + CAP, tl.total) - 1;
    }
    T.frame = T.P0 / tl.hw;
    T.y0 = (T.P0 - T.frame * tl.hw) / s.w;
    T.fb = T.P1 / tl.hw;
    T.rowsA = T.fb != T.frame ? s.h - T.y0 + 2 * R : (1 << 30);
    // wave-uniform: keep them in SGPRs (the compiler divides on the VALU)
    T.P0 = __builtin_amdgcn_readfirstlane(T.P0);
    T.P1 = __builtin_amdgcn_readfirstlane(T.P1);
    T.frame = __builtin_amdgcn_readfirstlane(T.frame);
    T.y0 = __builtin_amdgcn_readfirstlane(T.y0);
    T.fb = __builtin_amdgcn_readfirstlane(T.fb);
    T.rowsA = __builtin_amdgcn_readfirstlane(T.rowsA);
    return T;
  };
  const int h_plane = wave & 3, h_i0 = wave >> 2;
  const int h_sl0 = h_i0 * 64 + lane;
  const int h_r0 = h_sl0 / tl.pitch, h_c0 = h_sl0 - (h_sl0 / tl.pitch) * tl.pitch;
  // CIRC: this lane's row / column in piece 0 of a plane (the background cursor's start)
  const int hq_r0 = lane / tl.pitch, hq_c0 = lane - (lane / tl.pitch) * tl.pitch;
  // LIN (the launcher checks chunk-planar input, pitch == padded width, pad == R): halo slot sl of
  // the tile is linear pixel y0 * wp_in + sl of frame A's plane (sl < splitA), else pixel
  // sl - splitA of frame B's
  auto lin_src = [&](const char* a0, const char* b0, int sl, int splitA, int lastA) -> const char* {
    return sl < splitA ? a0 + (int64_t)min(sl, lastA) * 16 : b0 + (int64_t)min(sl - splitA, hp_in * wp_in - 1) * 16;
  };
  // this wave's pieces of chunk c's halo (LDS-DMA)
  auto issue_halo = [&](int c, const Tile& T) {
    const char* const fbase = (const char*)g.in + (int64_t)T.frame * hp_in * wp_in * pix_bytes;
    const char* const fbase_b = (const char*)g.in + (int64_t)T.fb * hp_in * wp_in * pix_bytes;
    const char* src0 = fbase + (int64_t)(c * 4 + h_plane) * in_pc;
    const char* src0_b = fbase_b + (int64_t)(c * 4 + h_plane) * in_pc;
    if constexpr (LIN) {
      const int splitA = T.rowsA < (1 << 29) ? T.rowsA * tl.pitch : (1 << 30);
      const int lastA = (hp_in - T.y0) * wp_in - 1;
      const char* const a0 = src0 + (int64_t)T.y0 * wp_in * 16;
      char* dst = halo + h_plane * HPLANE + h_i0 * 1024;
      // halo_trim: a tile reads halo slots < its rows x pitch only (its output rows + 2R, or for a tile
      // that crosses a frame both row sets; block q = (y - y0) * pitch + x plus tap offsets < 2R * pitch
      // + 2R): the pieces past them (the plane is sized for the launch's largest tile) are not loaded
      int np = tl.nh;
      if (tl.halo_trim) {  // a tile that crosses a frame: frame A's rowsA rows, then frame B's rows 0..yb + 2R
        const int yb = (T.P1 - T.fb * tl.hw) / s.w;
        const int rows = T.fb == T.frame ? yb - T.y0 + 1 + 2 * R : T.rowsA + yb + 1 + 2 * R;
        np = min(np, (rows * tl.pitch + 63) / 64);
      }
      for (int i = h_i0; i < np; i += 2) {
        glds16((const void*)lin_src(a0, src0_b, i * 64 + lane, splitA, lastA), dst);
        dst += 2 * 1024;
      }
      return;
    }
    int hr = h_r0, hc = h_c0;
    char* dst = halo + h_plane * HPLANE + h_i0 * 1024;
    for (int i = h_i0; i < tl.nh; i += 2) {
      const bool in_a = hr < T.rowsA;
      const int yy = min((in_a ? T.y0 - R + hr : hr - T.rowsA - R) + s.pin, hp_in - 1);
      const int xx = min(hc - R + s.pin, wp_in - 1);
      glds16((const void*)((in_a ? src0 : src0_b) + (int64_t)(yy * wp_in + xx) * in_px), dst);
      dst += 2 * 1024;
      hc += 2 * 64;
      while (hc >= tl.pitch) {
        hc -= tl.pitch;
        ++hr;
      }
    }
  };
  const int wlane = (2 * khalf) * PLANE_W + (ch * 64 + l16) * 16;     // A: channel ch*64 + cb*16 + l16

#if M16_STAMPS
  const unsigned long long st_t0 = M16_T();
#endif
  const Tile T = tile_of(widx);
  // CIRC schedule of this tile (wave-uniform): np pieces per chunk and its regions R1 / R2 / R3
  constexpr int CP = HPLANE / 1024;
  int c_np = 0, c_r1 = 0, c_r2 = 0, c_r3 = 0;
  bool circ = false;
  if constexpr (CIRC) {
    if (T.fb == T.frame && cb1 - cb0 > 1) {
      const int rows = (T.P1 - T.frame * tl.hw) / s.w - T.y0 + 1 + 2 * R;  // output rows + the 2R border
      const int np = (rows * tl.pitch + 63) / 64;
      const int op = max(2 * np - CP, 0);         // pieces of chunk c + 1 that overlay chunk c's
      const int early = (6 * tl.pitch) / 64;      // chunk c's pieces inside its rows 0-5
      c_np = np;
      c_r2 = min(op, early);
      c_r3 = op - c_r2;
      c_r1 = np - op;
      // R3's first row must be read by taps with ky >= 1 only: row >= the tile's output rows
      circ = np <= CP && (c_r3 == 0 || ((np - c_r3) * 64) / tl.pitch >= rows - 2 * R);
    }
    c_np = __builtin_amdgcn_readfirstlane(c_np);
    c_r1 = __builtin_amdgcn_readfirstlane(c_r1);
    c_r2 = __builtin_amdgcn_readfirstlane(c_r2);
    c_r3 = __builtin_amdgcn_readfirstlane(c_r3);
  }
#pragma unroll
  for (int j = 0; j < 2 * AHEAD; ++j) stage_w(cb0 * KSQP + j);
  {
    // this lane's pixel of each block -> byte offset of its halo slot in its hi plane (2 khalf), so
    // a B fragment address is qb[pb] + the tap's offset: one VALU add per block
    int qb[NPX];
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) {
      const int P = T.P0 + (pg * NPX + pb) * 16 + l16;
      int q = 0;
      if (P <= T.P1) {
        const int f = P / tl.hw, pp = P - (P / tl.hw) * tl.hw;
        const int y = pp / s.w, x = pp - (pp / s.w) * s.w;
        q = (f == T.frame ? y - T.y0 : T.rowsA + y) * tl.pitch + x;
      }
      qb[pb] = CIRC ? q * 16 : (2 * khalf) * HPLANE + q * 16;  // CIRC: the plane base is added per read
    }
    const int pbase = (2 * khalf) * HPLANE;  // CIRC: this lane's hi plane
    // CIRC: a lane's byte offset of block pb's slot + the tap offset, wrapped into the plane
    auto bofs = [&](int pb, int toff) -> int {
      if constexpr (CIRC) {
        const unsigned a = (unsigned)(qb[pb] + toff);
        return (int)min(a, a - (unsigned)HPLANE) + pbase;
      } else {
        return qb[pb] + toff;
      }
    };
    // CIRC: waves 4-7's background halo stream of plane wave - 4: pieces [jlo, jhi) of chunk cc into
    // physical pieces base + j (mod CP); the cursor (hq_r, hq_c) is the lane's row / column of piece jlo
    int hq_r = 0, hq_c = 0;
    const int hq_pl = wave & 3;
    auto circ_issue = [&](int cc, int jlo, int jhi, int base) {
      const char* const src0 = (const char*)g.in + (int64_t)T.frame * hp_in * wp_in * pix_bytes +
                               (int64_t)(cc * 4 + hq_pl) * in_pc;
      for (int j = jlo; j < jhi; ++j) {
        const int yy = min(T.y0 - R + hq_r + s.pin, hp_in - 1);
        const int xx = min(hq_c - R + s.pin, wp_in - 1);
        int ph = base + j;
        ph = ph >= CP ? ph - CP : ph;
        glds16((const void*)(src0 + (int64_t)(yy * wp_in + xx) * in_px), halo + hq_pl * HPLANE + ph * 1024);
        hq_c += 64;
        while (hq_c >= tl.pitch) {
          hq_c -= tl.pitch;
          ++hq_r;
        }
      }
    };
    int cbase = 0;  // CIRC: the current chunk's first physical piece

    floatx4 acc[4][NPX];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int pb = 0; pb < NPX; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

    int it = cb0 * KSQP;
#if M16_STAMPS
    unsigned long long st_b = 0, st_p = 0, st_np = 0, st_v = 0, st_bar = 0, st_dma = 0, st_b1 = 0, st_b2 = 0;
    const unsigned long long st_loop0 = M16_T();
#endif
    for (int c = cb0; c < cb1; ++c) {
#if M16_STAMPS
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long tb0 = M16_T();
      __builtin_amdgcn_sched_barrier(0);
#endif
      // the chunk-boundary drain (CIRC tiles: only before their first chunk)
      const bool cont = CIRC && circ && c > cb0;  // the ring barriers run on from the previous chunk
      if (!cont) {
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#if M16_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long tb1 = M16_T();
        __builtin_amdgcn_sched_barrier(0);
#endif
#if M16_PROBE_NOHALO  // timing probe only (wrong results): the halo is loaded for the first chunk only
        if (c == cb0) issue_halo(c, T);
#else
        issue_halo(c, T);
#endif
#if M16_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long tb2 = M16_T();
        __builtin_amdgcn_sched_barrier(0);
        st_b1 += tb1 - tb0;
        st_b2 += tb2 - tb1;
#endif
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      int nbase = cbase + c_np;  // CIRC: the next chunk's first physical piece
      nbase = nbase >= CP ? nbase - CP : nbase;
      const bool has_next = c + 1 < cb1;
      const bool cont_next = CIRC && circ;  // the next chunk continues without a drain
#if M16_STAMPS
      __builtin_amdgcn_sched_barrier(0);
      st_b += M16_T() - tb0;
      __builtin_amdgcn_sched_barrier(0);
#endif
      bf16x8g ah[4], al[4];
#if M16_PROBE_NOPAD  // timing probe only (wrong results): the padding pair of the odd 49th tap skipped
      constexpr int kPairsEnd = KSQ - 1;
#else
      constexpr int kPairsEnd = KSQP;
#endif
#pragma unroll 1
      for (int t = 0; t < kPairsEnd; t += 2, it += 2) {
#if M16_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long tp0 = M16_T();
        __builtin_amdgcn_sched_barrier(0);
        ++st_np;
#endif
        wait_vmcnt<kDmaPerPair * (AHEAD - 1)>();  // W(it), W(it+1) (issued AHEAD pairs back) ...
#if M16_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long tp1 = M16_T();
        __builtin_amdgcn_sched_barrier(0);
#endif
#if !M16_PROBE_NOBAR  // timing probe only (racy ring): no per-pair barrier
        if (!STAG) {
          __builtin_amdgcn_s_barrier();  // ... landed for every wave; the previous pair's slots are free
        } else if (wave < 4 && (t > 0 || cont)) {
          // waves 0-3 at the start of pair p, waves 4-7 in the middle of pair p - 1 (below): pair p's
          // pieces landed for every wave; the slot staged next (pair p - 1's) is free -- waves 4-7
          // hold pair p - 1's A fragments in registers since they started it.  The chunk's first
          // pair needs none after a drain: the chunk barriers above ordered everything
          __builtin_amdgcn_s_barrier();
        }
#endif
        asm volatile("" ::: "memory");
#if M16_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long tp2 = M16_T();
        __builtin_amdgcn_sched_barrier(0);
#endif
        stage_w(it + 2 * AHEAD);
        stage_w(it + 2 * AHEAD + 1);
#if M16_PF_L2
        if constexpr (LIN) {
          constexpr int kPfPair = 8;
          const int pk = (t >> 1) - kPfPair;
          if (wave >= 4 && tl.nh < 28 && c + 1 < cb1 && pk >= 0 && pk * 64 * 8 < tl.nh * 64) {
            // lane l: 128-B line pk * 64 + l of plane wave - 4 of chunk c + 1 (slots 8 apart)
            const int pl = wave - 4;
            const char* const pa = (const char*)g.in + (int64_t)T.frame * hp_in * wp_in * pix_bytes +
                                   (int64_t)((c + 1) * 4 + pl) * in_pc;
            const char* const pb0 = (const char*)g.in + (int64_t)T.fb * hp_in * wp_in * pix_bytes +
                                    (int64_t)((c + 1) * 4 + pl) * in_pc;
            const int splitA = T.rowsA < (1 << 29) ? T.rowsA * tl.pitch : (1 << 30);
            const int sl = min((pk * 64 + lane) * 8, tl.nh * 64 - 1);
            __builtin_amdgcn_global_load_lds(
                (const void*)lin_src(pa + (int64_t)T.y0 * wp_in * 16, pb0, sl, splitA, (hp_in - T.y0) * wp_in - 1),
                (__attribute__((address_space(3))) void*)(halo + pl * HPLANE + 27 * 1024), 4, 0, 0);
          }
        }
#endif
        if constexpr (CIRC) {
          if (circ && wave >= 4) {  // the background halo stream (see CIRC above), pair p = t / 2
            const int p = t >> 1;
            int cc = c + 1, jlo = 0, jhi = 0, base = nbase;
            if (p < 2) {  // R3 of this chunk, half per pair
              const int j0 = c_np - c_r3, jm = j0 + (c_r3 + 1) / 2;
              cc = c;
              base = cbase;
              jlo = p == 0 ? j0 : jm;
              jhi = c > cb0 ? (p == 0 ? jm : c_np) : jlo;
            } else if (p <= 20) {  // R1 of the next chunk over pairs 2-20
              jlo = (p - 2) * c_r1 / 19;
              jhi = has_next ? (p - 1) * c_r1 / 19 : jlo;
            } else if (p <= 22) {  // R2 over pairs 21-22
              const int jm = c_r1 + (c_r2 + 1) / 2;
              jlo = p == 21 ? c_r1 : jm;
              jhi = has_next ? (p == 21 ? jm : c_r1 + c_r2) : jlo;
            }
            if (p == 2) {
              hq_r = hq_r0;
              hq_c = hq_c0;
            }
            circ_issue(cc, jlo, jhi, base);
          }
        }
#if M16_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long tp3 = M16_T();
        __builtin_amdgcn_sched_barrier(0);
        st_v += tp1 - tp0;
        st_bar += tp2 - tp1;
        st_dma += tp3 - tp2;
#endif
        // tap offsets of the pair (uniform: scalar), then one select per lane (tsel); the padding
        // tap (zero weights) reads tap t's pixels: finite values, times zero
        const int t1 = t + 1 < KSQ ? t + 1 : t;
        const int toff0 = ((t / KS) * tl.pitch + (t - (t / KS) * KS)) * 16;
        const int toff1 = ((t1 / KS) * tl.pitch + (t1 - (t1 / KS) * KS)) * 16;
        const int toff = tsel ? toff1 : toff0;
        const char* wsl = ring + ((unsigned)it % RING + tsel) * SLOT_W + wlane;  // it even: no wrap
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          ah[cb] = *(const bf16x8g*)(wsl + cb * 256);
          al[cb] = *(const bf16x8g*)(wsl + PLANE_W + cb * 256);
        }
        bf16x8g bh[2], bl[2];
        {
          const char* bp = halo + bofs(0, toff);
          bh[0] = *(const bf16x8g*)bp;
          bl[0] = *(const bf16x8g*)(bp + HPLANE);
        }
#pragma unroll
        for (int pb = 0; pb < NPX; ++pb) {
          const int cur = pb & 1;
          if (STAG && pb == NPX / 2 && wave >= 4 && (t + 2 < kPairsEnd || (cont_next && has_next))) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();  // waves 0-3's barrier at the start of pair p + 1 (above)
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
          }
          if (pb + 1 < NPX) {
            const char* bp = halo + bofs(pb + 1, toff);
            bh[cur ^ 1] = *(const bf16x8g*)bp;
            bl[cur ^ 1] = *(const bf16x8g*)(bp + HPLANE);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[cb], bh[cur], acc[cb][pb], 0, 0, 0);
#if M16_STAMPS
            if (pb == 0 && cb == 0) {
              __builtin_amdgcn_sched_barrier(0);
              st_p += M16_T() - tp0;
              __builtin_amdgcn_sched_barrier(0);
            }
#endif
            acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[cb], bl[cur], acc[cb][pb], 0, 0, 0);
            acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[cb], bh[cur], acc[cb][pb], 0, 0, 0);
          }
        }
      }
      if constexpr (CIRC) {
        if (circ) {  // the next chunk's pieces start where this chunk's end: move every block's slot
          cbase = nbase;
#pragma unroll
          for (int pb = 0; pb < NPX; ++pb) {
            const unsigned a = (unsigned)(qb[pb] + c_np * 1024);
            qb[pb] = (int)min(a, a - (unsigned)HPLANE);
          }
        }
      }
    }
#if M16_STAMPS
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long st_loop1 = M16_T();
    __builtin_amdgcn_sched_barrier(0);
#endif
    wait_vmcnt<0>();
#if M16_STAMPS
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long st_wait1 = M16_T();
    __builtin_amdgcn_sched_barrier(0);
#endif

    if (nsplit > 1) {  // raw partial sums; conv_m16_splitk_reduce adds the splits, bias and ReLU
      const int wsc = max(g0.cop, g1.cop);  // partial row stride (the launcher sizes ws with it)
      float* const wsg = tl.ws + ((int64_t)split * s.groups + grp) * (int64_t)tl.total * wsc;
#pragma unroll
      for (int pb = 0; pb < NPX; ++pb) {
        const int P = T.P0 + (pg * NPX + pb) * 16 + l16;
        if (P > T.P1) continue;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int co = co0 + ch * 64 + cb * 16 + 4 * kg;
          if (co < g.cop) *(floatx4*)(wsg + (int64_t)P * wsc + co) = acc[cb][pb];
        }
      }
    } else {
      const int wp_out = s.w + 2 * s.pout;
      const int hp_out = s.h + 2 * s.pout;
      const int64_t out_pc = split_piece_stride(s.out_planar, hp_out, wp_out);
      const int64_t out_px = split_pixel_stride(s.out_planar, s.cs_out);
#pragma unroll
      for (int pb = 0; pb < NPX; ++pb) {
        const int P = T.P0 + (pg * NPX + pb) * 16 + l16;
        const int f = P / tl.hw, pp = P - f * tl.hw;
        const int y = pp / s.w, x = pp - y * s.w;
        char* optr = (char*)g.out + (int64_t)f * hp_out * wp_out * s.cs_out * 4 +
                     ((int64_t)(y + s.pout) * wp_out + (x + s.pout)) * out_px;
        float* o32 = g.out32 ? g.out32 + ((int64_t)(f * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int co = co0 + ch * 64 + cb * 16 + 4 * kg;
          floatx4 v;
          uint32_t own[4], w[4];
          split_pair_swap(acc[cb][pb], co < g.cop ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f},
                          s.relu, v, own, w);
          if (P > T.P1 || co >= g.cout_store) continue;
          store_split_group(optr, co, kg, g.cout_store, own, w, out_pc);
          if (o32) *(floatx4*)(o32 + co) = v;
        }
      }
    }
#if M16_STAMPS
    wait_vmcnt<0>();
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long st_end = M16_T();
    if (lane == 0) {
      atomicAdd(&g_m16_st[0], st_end - st_t0);
      atomicAdd(&g_m16_st[1], st_b);
      atomicAdd(&g_m16_st[2], st_p);
      atomicAdd(&g_m16_st[3], st_loop1 - st_loop0);
      atomicAdd(&g_m16_st[4], st_end - st_wait1);
      atomicAdd(&g_m16_st[5], st_np);
      atomicAdd(&g_m16_st[6], 1ull);
      atomicAdd(&g_m16_st[7], st_wait1 - st_loop1);
      atomicAdd(&g_m16_st[8], st_v);
      atomicAdd(&g_m16_st[9], st_bar);
      atomicAdd(&g_m16_st[10], st_dma);
      atomicAdd(&g_m16_st[11], st_b1);
      atomicAdd(&g_m16_st[12], st_b2);
    }
#endif
  }
}

// PERS (round 6): a persistent grid of one workgroup per CU, each running the
// tiles lin = blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8, so every tile keeps its XCD
// and its place in the XCD-aware order): tile i's epilogue stores drain while tile i + 1 stages its
// ring and first halo, instead of every CU writing its outputs in the same burst at the end of a
// round of workgroups.  A barrier between tiles keeps the staggered half's last pair ahead of the
// next tile's ring staging.
template <int KS, int NPX, bool DEEP = false, bool STAG = false, bool CIRC = false, bool LIN = false, bool PERS = false>
__global__ __launch_bounds__(512, 1) void conv_m16_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                          BigTiling tl) {
  static_assert(!PERS || (LIN && !DEEP), "persistent tiles: the linear-halo kernel");
  if constexpr (PERS) {
#pragma unroll 1
    for (int lin = blockIdx.x; lin < tl.pers_blocks; lin += gridDim.x) {
      if (lin != (int)blockIdx.x) __syncthreads();
      m16_tile<KS, NPX, DEEP, STAG, CIRC, LIN>(s, g0, g1, tl, lin);
    }
  } else {
    m16_tile<KS, NPX, DEEP, STAG, CIRC, LIN>(s, g0, g1, tl, blockIdx.x);
  }
}

int launch_m16_7x7(int npx, hipStream_t st, const SplitConvShape& s, const SplitConvGroup& g0,
                   const SplitConvGroup& g1, const BigTiling& tl) {
  static bool attr = false;
  if (!attr) {
    const void* fns[] = {(const void*)conv_m16_bf16x3<7, 10>, (const void*)conv_m16_bf16x3<7, 9>,
                         (const void*)conv_m16_bf16x3<7, 8>,  (const void*)conv_m16_bf16x3<7, 7>,
                         (const void*)conv_m16_bf16x3<7, 6>,
                         (const void*)conv_m16_bf16x3<7, 5>,  (const void*)conv_m16_bf16x3<7, 4>,
                         (const void*)conv_m16_bf16x3<7, 3>,  (const void*)conv_m16_bf16x3<7, 2>,
                         (const void*)conv_m16_bf16x3<7, 5, true>, (const void*)conv_m16_bf16x3<7, 4, true>,
                         (const void*)conv_m16_bf16x3<7, 3, true>, (const void*)conv_m16_bf16x3<7, 2, true>,
                         (const void*)conv_m16_bf16x3<7, 10, false, true>, (const void*)conv_m16_bf16x3<7, 9, false, true>,
                         (const void*)conv_m16_bf16x3<7, 8, false, true>, (const void*)conv_m16_bf16x3<7, 7, false, true>,
                         (const void*)conv_m16_bf16x3<7, 6, false, true>, (const void*)conv_m16_bf16x3<7, 5, false, true>,
                         (const void*)conv_m16_bf16x3<7, 4, false, true>, (const void*)conv_m16_bf16x3<7, 3, false, true>,
                         (const void*)conv_m16_bf16x3<7, 2, false, true>,
                         (const void*)conv_m16_bf16x3<7, 5, true, true>, (const void*)conv_m16_bf16x3<7, 4, true, true>,
                         (const void*)conv_m16_bf16x3<7, 3, true, true>, (const void*)conv_m16_bf16x3<7, 2, true, true>,
                         (const void*)conv_m16_bf16x3<7, 10, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 9, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 8, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 7, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 6, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 10, false, true, false, true>,
                         (const void*)conv_m16_bf16x3<7, 9, false, true, false, true>,
                         (const void*)conv_m16_bf16x3<7, 8, false, true, false, true>,
                         (const void*)conv_m16_bf16x3<7, 7, false, true, false, true>,
                         (const void*)conv_m16_bf16x3<7, 6, false, true, false, true>,
                         (const void*)conv_m16_bf16x3<7, 10, false, true, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 9, false, true, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 8, false, true, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 7, false, true, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 6, false, true, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 10, false, false, false, true>,
                         (const void*)conv_m16_bf16x3<7, 9, false, false, false, true>,
                         (const void*)conv_m16_bf16x3<7, 8, false, false, false, true>,
                         (const void*)conv_m16_bf16x3<7, 7, false, false, false, true>,
                         (const void*)conv_m16_bf16x3<7, 6, false, false, false, true>,
                         (const void*)conv_m16_bf16x3<7, 10, false, false, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 9, false, false, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 8, false, false, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 7, false, false, false, true, true>,
                         (const void*)conv_m16_bf16x3<7, 6, false, false, false, true, true>};
    for (const void* f : fns)
      OP_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (tl.nh > 32) {
    set_error("conv_m16_bf16x3: halo plane over 32 KiB");
    return OP_ERR_INVALID;
  }

  // small tiles whose halo planes fit 16 KiB take the deep weight ring (12 taps, 5 pairs ahead)
  static const bool no_deep = getenv("OP_M16_NODEEP") && atoi(getenv("OP_M16_NODEEP")) != 0;  // A/B aid
  const bool deep = npx <= 5 && tl.nh <= 16 && !no_deep;
  // the staggered halves (OP_M16_STAG=0: one barrier per pair for all 8 waves; read per call)
  const char* stag_env = getenv("OP_M16_STAG");
  // not on frame-aligned raster tiles (the wide multi-scale maps): C4's 7x7 79.2 ms staggered
  // everywhere, 78.5 never, 77.8 except those (profiles/r05/ab_r05p_7x7_stag_c4_modes.log)
  const bool stag = M16_DMA_HALF && (deep || tl.nh <= (M16_STAG_RING == 6 ? 28 : 32)) && tl.fa_tiles == 0 &&
                    !(stag_env && atoi(stag_env) == 0);
  const int lds = deep ? 12 * 4 * 128 * 16 + 4 * 16 * 1024   // ring + 4 halo planes (16-KiB stride)
                  : stag ? (M16_STAG_RING == 6 ? 6 * 4 * 128 * 16 + 4 * 28 * 1024  // 6-tap ring + 4 planes (28-KiB stride)
                                               : 4 * 4 * 128 * 16 + 4 * 32 * 1024)
                         : 4 * 4 * 128 * 16 + 4 * 32 * 1024;  // ring + 4 halo planes (32-KiB stride)
  const unsigned blocks = tl.xpu ? 8u * (unsigned)((tl.per_unit + tl.xpu - 1) / tl.xpu * std::max(tl.pair, 1))
                                 : (unsigned)(tl.units * tl.per_unit);
  const dim3 grid(blocks, (unsigned)tl.ksplit);
  // round 6: the staggered kernel with circular halo planes (no chunk-boundary drain for tiles of
  // one frame) -- bit-identical, measured SLOWER and opt-in (OP_M16_CIRC=1, read per call): the 7x7
  // class 77.2 -> 79.8 ms per headline step, and 79.6 with the circular kernel's drain on every tile
  // (profiles/r06/ab_r06b_*): the pair loop is that sensitive to added per-pair instructions (its
  // per-block slot wrap and the background schedule); so is it to fewer scalar but more vector ones
  // (incremental staging cursor: 76.0 -> 80.4 ms, profiles/r06/ab_r06c_incr_scalar_cursor_not_kept.log)
  const char* circ_env = getenv("OP_M16_CIRC");
  const bool circ = stag && !deep && npx >= 6 && circ_env && atoi(circ_env) == 1;
  // round 6: linear halo sources (LIN) on chunk-planar input with the tight pitch, by default
  // (OP_M16_LIN=0, read per call, keeps the row / column cursor): with the halo trimmed to a tile's own
  // rows (conv_big.hip halo_trim) the headline's 7x7 class 74.9 -> 74.4 ms per step, C5's 39.6 ->
  // 38.0, C4's within noise (profiles/r06/ab_r06t_7x7_lin_trim_pers_*.log); bit-identical
  const char* lin_env = getenv("OP_M16_LIN");
  const bool lin = !deep && !circ && npx >= 6 && s.in_planar && s.pin == 3 && tl.pitch == s.w + 2 * s.pin &&
                   !(lin_env && atoi(lin_env) == 0);
  // round 6: persistent tiles (PERS) for LIN launches of more than one round, unsplit (opt-in
  // OP_M16_PERS=1, read per call): bit-identical, measured SLOWER -- the headline's 7x7 class 74.4 ->
  // 77.4 ms per step, C5 38.0 -> 38.8 (profiles/r06/ab_r06t_7x7_lin_trim_pers_*.log)
  const char* pers_env = getenv("OP_M16_PERS");
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    OP_HIP_CHECK(hipGetDevice(&dev));
    OP_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const unsigned pgrid = (unsigned)(n_cu / 8 * 8);
  const bool pers = lin && tl.ksplit == 1 && pgrid >= 8 && blocks > pgrid && pers_env && atoi(pers_env) == 1;
  BigTiling tlp = tl;
  tlp.pers_blocks = (int)blocks;
#define M16_LAUNCH(N, D, S) hipLaunchKernelGGL((conv_m16_bf16x3<7, N, D, S>), grid, dim3(512), lds, st, s, g0, g1, tl)
#define M16_LAUNCH_C(N) hipLaunchKernelGGL((conv_m16_bf16x3<7, N, false, true, true>), grid, dim3(512), lds, st, s, g0, g1, tl)
#define M16_LAUNCH_L(N, S)                                                                                            \
  do {                                                                                                                \
    if (pers)                                                                                                         \
      hipLaunchKernelGGL((conv_m16_bf16x3<7, N, false, S, false, true, true>), dim3(pgrid), dim3(512), lds, st, s,    \
                         g0, g1, tlp);                                                                                \
    else                                                                                                              \
      hipLaunchKernelGGL((conv_m16_bf16x3<7, N, false, S, false, true>), grid, dim3(512), lds, st, s, g0, g1, tl);    \
  } while (0)
#define M16_CASE(N)                                  \
  case N:                                            \
    if (deep && N <= 5) {                            \
      if (stag) M16_LAUNCH(N, (N <= 5), true);       \
      else M16_LAUNCH(N, (N <= 5), false);           \
    } else if (stag) {                               \
      if (circ && N >= 6) M16_LAUNCH_C((N >= 6 ? N : 6)); \
      else if (lin && N >= 6) M16_LAUNCH_L((N >= 6 ? N : 6), true); \
      else M16_LAUNCH(N, false, true);               \
    } else {                                         \
      if (lin && N >= 6) M16_LAUNCH_L((N >= 6 ? N : 6), false); \
      else M16_LAUNCH(N, false, false);              \
    }                                                \
    break;
  switch (npx) {
    M16_CASE(9)
    M16_CASE(8)
    M16_CASE(7)
    M16_CASE(6)
    M16_CASE(5)
    M16_CASE(4)
    M16_CASE(3)
    M16_CASE(2)
    default:
      if (circ) M16_LAUNCH_C(10);
      else if (lin) {
        if (stag) M16_LAUNCH_L(10, true);
        else M16_LAUNCH_L(10, false);
      } else if (stag) M16_LAUNCH(10, false, true);
      else M16_LAUNCH(10, false, false);
  }
#undef M16_CASE
#undef M16_LAUNCH
#undef M16_LAUNCH_C
#undef M16_LAUNCH_L
  census_add(stag ? OP_CENSUS_7X7_STAG : OP_CENSUS_7X7_PLAIN_RING);
  if (circ) census_add(OP_CENSUS_7X7_CIRC);
  if (lin) census_add(OP_CENSUS_7X7_LIN);
  if (pers) census_add(OP_CENSUS_7X7_PERS);
#if M16_STAMPS
  static const bool dump = getenv("OP_M16_STAMPS") != nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (dump && hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone && tl.ksplit == 1) {
    static unsigned long long tot[14] = {};
    static int launches = 0;
    unsigned long long h[14];
    OP_HIP_CHECK(hipStreamSynchronize(st));
    OP_HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_m16_st), sizeof(h)));
    const unsigned long long z[14] = {};
    OP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_m16_st), z, sizeof(z)));
    for (int i = 0; i < 14; ++i) tot[i] += h[i];
    if (++launches % 25 == 0) {
      const double w = (double)tot[0];
      fprintf(stderr,
              "M16_STAMPS npx %d launches %d waves %llu pairs/wave %.1f | per wave cycles %.0f | chunk boundary %.4f "
              "pair start %.4f (vmcnt %.4f barrier %.4f dma %.4f) pair loop %.4f (pure pairs %.4f) final wait %.4f "
              "epilogue %.4f prologue %.4f | chunk boundary: first barrier %.4f halo issue %.4f\n",
              npx, launches, tot[6], (double)tot[5] / tot[6], w / tot[6], tot[1] / w, tot[2] / w, tot[8] / w, tot[9] / w,
              tot[10] / w, tot[3] / w,
              (tot[3] - tot[1] - tot[2]) / w, tot[7] / w, tot[4] / w, (w - tot[3] - tot[7] - tot[4]) / w, tot[11] / w,
              tot[12] / w);
    }
  }
#endif
  return OP_OK;
}

}  // namespace op
