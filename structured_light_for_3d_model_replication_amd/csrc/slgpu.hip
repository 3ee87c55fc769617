// slgpu.hip — MI355X (gfx950, CDNA4) kernels for the structured-light hot path.
//
// Path (reference): Gray-code decode  server/processing.py:28-124, server/sl_system.py:516-588
//                   ray-plane triangulation  server/processing.py:127-234, sl_system.py:592-661
// C ABI: include/slgpu.h.  Design and rooflines: DESIGN.md.
//
// Kernels
//   stats_kernel      white/black histograms (+ max contrast) -> last-arriving workgroup turns
//                     them into integer mask thresholds (Otsu as OpenCV, or NumPy percentile);
//                     also zeroes the compaction state of the next main launch.
//   main3_kernel<...> fused decode + triangulate + ordered compaction, one 4096-pixel tile per
//                     workgroup (512 lanes x 8 pixels), up to 16 views per launch: the mask
//                     first (white/black), then the used pattern frames only in lanes holding a
//                     valid pixel, with 8-byte-per-lane coalesced loads (instances specialised on
//                     the common decode plans issue them all unconditionally), SWAR byte compares,
//                     packed 16-bit Gray->binary, wave-private LDS compaction of valid pixels,
//                     fp64 ray-plane intersection, decoupled look-back over static tile ids,
//                     compacted stores straight from registers; the grid's first workgroups
//                     can turn a carried batch's Otsu partials into thresholds.
//   decode_maps_kernel  the decode alone, to correspondence maps (slg_decode).
//   row_tail_kernel   row_mode 2: moves the row cloud behind the column cloud.
//   pinhole_kernel    bitwise Nc == pinhole(cam_K) test.
//
// Numerics: every floating-point expression follows NumPy's operation order with
// -ffp-contract=off (no FMA contraction), IEEE-correct f64 division and sqrt, so the fp64
// results equal the reference bit for bit; integer/byte work is exact by construction.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>
#include <limits.h>
#include <type_traits>
#include <utility>
#include <stdlib.h>
#include <math.h>
#include <string>
#include <errno.h>
#include <fcntl.h>
#include <unistd.h>
#include <thread>
#include <vector>
#include <algorithm>
#include <mutex>
#include <dlfcn.h>

#include "../../include/slgpu.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBlock = 256;                 // 4 waves of 64
constexpr int kPx = 8;                      // pixels per lane (one 8-byte load per frame)
#ifndef SLG_TILE_BLOCK
#define SLG_TILE_BLOCK 512
#endif
constexpr int kTileBlock = SLG_TILE_BLOCK;  // main3 workgroup: 512 lanes, 322.6 vs 331.3 us per
                                            // 12-view launch with 256 (half the look-backs per pixel)
constexpr int kTilePx = kTileBlock * kPx;   // 4096 pixels per main3 tile (one look-back entry)
constexpr int kMapsPx = kBlock * kPx;       // 2048 pixels per decode_maps workgroup
constexpr int kMaxBits = 15;                // packed 16-bit code lanes
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;

// ------------------------------------------------------------------ workspace layout
struct WsHeader {
  uint32_t hist[3][256];   // otsu: 0 white, 1 clip(white-black,0,255); percentile: 0 black
  uint32_t max_diff_enc;   // max(white-black) + 256 (0 = none yet)
  uint32_t ticket;         // stats_kernel arrival counter
  uint32_t lb_ticket;      // main3 tiles that published their column-stream aggregate (lookback_scan)
  uint32_t error;          // bit 0: look-back spin timeout; 1: a look-back helper ran
  int32_t smin;            // mask: white >= smin
  int32_t cmin;            //       (white - black) >= cmin
  uint32_t lb_ticket_row;  // the same for the row stream (row_mode 2)
  int32_t pad0;
  double thr_s;            // float thresholds (for inspection / tests)
  double thr_c;
  int64_t totals[2];       // column / row stream point totals
  // Otsu only: pixels with white >= smin, and with white - black >= cmin (n_px when cmin <= 0,
  // which the clipped histogram cannot count); their minimum bounds the valid pixels, so the
  // point count of row_mode 0/1 (resident jobs size their clouds with it).  n_px otherwise.
  int64_t above[2];
  // Resident-job arena (slg_workspace_set_arena; NULL cursor: none).  The Otsu tail that sets a
  // view's thresholds also reserves its cloud's region: arena_off = atomicAdd(cursor, need),
  // need = min(above) * arena_mult (an upper bound of its points), or -1 when the arena has no
  // room left (the fused launch then stores nothing for it; the host re-runs it).
  int64_t arena_off;
  int32_t arena_mult;      // points per valid pixel at most: 1 (row_mode 0/1) or 2 (row_mode 2)
  int32_t pad4;
  unsigned long long* arena_cursor;
  int64_t arena_cap;       // points the arena holds
  uint64_t pad3[2];
};
constexpr int kHistCopies = 16;            // partial histograms: blocks spread their atomics
constexpr int64_t kHistPartOff = 8192;      // uint32 [kHistCopies][2][256] after the header
constexpr int64_t kHeaderBytes = 65536;
static_assert(sizeof(WsHeader) <= kHistPartOff, "header");
static_assert(offsetof(WsHeader, error) == 3084 && offsetof(WsHeader, totals) == 3120 && offsetof(WsHeader, above) == 3136 &&
              offsetof(WsHeader, arena_off) == 3152,
              "header offsets the host reads (engine.py: error word, WS_TOTALS_OFF, WS_ABOVE_OFF)");

__host__ __device__ inline int64_t n_tiles_of(int64_t n_px) { return (n_px + kTilePx - 1) / kTilePx; }
__host__ __device__ inline int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
__host__ __device__ inline int64_t states_off(int64_t) { return kHeaderBytes; }
__host__ __device__ inline int64_t n_state_words(int64_t n_px) { return 2 * n_tiles_of(n_px); }   // [stream][tile]
__host__ __device__ inline int64_t states_bytes(int64_t n_px) { return align_up(n_state_words(n_px) * 8, 256); }
__host__ __device__ inline int64_t scratch_xyz_off(int64_t n_px) { return kHeaderBytes + states_bytes(n_px); }
__host__ __device__ inline int64_t scratch_bgr_off(int64_t n_px) { return scratch_xyz_off(n_px) + align_up(n_px * 24, 256); }
__host__ __device__ inline int64_t parts_off(int64_t n_px) { return scratch_bgr_off(n_px) + align_up(n_px * 3, 256); }
// per tile: the Otsu histograms of the batch after next over the tile's pixels, u16 [2][256]
constexpr int64_t kPartWords = 256;         // packed u16 pairs per tile
__host__ __device__ inline int64_t ws_total(int64_t n_px) { return parts_off(n_px) + align_up(n_tiles_of(n_px) * kPartWords * 4, 256); }

// ------------------------------------------------------------------ small helpers
__device__ inline uint64_t ld_state(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_state(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifndef SLG_FRAME_BUFFER_LOADS
#define SLG_FRAME_BUFFER_LOADS 1           // frame loads as buffer loads (scalar base, 32-bit lane offset)
#endif
#ifndef SLG_NT_LOADS
#define SLG_NT_LOADS 1                     // frames / texture are read once: non-temporal loads
#endif
// Once-read stream (frames, texture): non-temporal 8-byte load (global_load_dwordx2 nt).
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ inline uint2 ld_once8(const void* ptr) {
#if SLG_NT_LOADS
  const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(ptr));
  return make_uint2(v.x, v.y);
#else
  return *reinterpret_cast<const uint2*>(ptr);
#endif
}

template <class T>
__device__ inline T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
__device__ inline int wave_min_i(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o));
  return x;
}

// Per-byte unsigned p > i on 4 packed bytes: 0x80 in every byte lane where p > i.
__device__ inline uint32_t gt_u8x4(uint32_t p, uint32_t i) {
  // per byte p > i in bit 7 (other bits garbage: callers mask with 0x80808080):
  // f(p, i, d) = (p & ~i) | (~(p ^ i) & ~d), d = (i | 0x80) - (p & 0x7f) per byte, one v_bitop3
  const uint32_t d = (i | 0x80808080u) - (p & 0x7f7f7f7fu);
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x71" : "=v"(r) : "v"(p), "v"(i), "v"(d));
  return r;
}

// Gray -> binary on two packed 16-bit lanes (values < 2^15): prefix XOR from the top.
__device__ inline uint32_t gray2bin_x2(uint32_t x) {
  x ^= (x >> 1) & 0x7fff7fffu;
  x ^= (x >> 2) & 0x3fff3fffu;
  x ^= (x >> 4) & 0x0fff0fffu;
  x ^= (x >> 8) & 0x00ff00ffu;
  return x;
}

// ------------------------------------------------------------------ stats kernel
constexpr int kMaxBatch = 16;               // views per batched stats launch (blockIdx.y)
constexpr int kStatsPx = 32;                // pixels per lane per stats iteration
constexpr int kStatsBlocks = 64;            // stats workgroups per view (at most), percentile path
#ifndef SLG_STATS_OTSU_BLOCKS
#define SLG_STATS_OTSU_BLOCKS 64                 // 128: 2.6% and 256: 10% slower bench (slot contention)
#endif
constexpr int kStatsBlocksOtsu = SLG_STATS_OTSU_BLOCKS;   // matrix-core Otsu path
#ifndef SLG_STATS_BLOCKS_ONE
#define SLG_STATS_BLOCKS_ONE 256   // r3ao: 64 -> 51.7, 128 -> 42.2, 256 -> 40.0, 512 -> 39.9 us (1080p, Otsu)
#endif
constexpr int kStatsBlocksOne = SLG_STATS_BLOCKS_ONE;   // one-view launches (nothing runs beside them)
#ifndef SLG_OTSU_ONE_CHUNKS
#define SLG_OTSU_ONE_CHUNKS 2
#endif
constexpr int kOtsuOneChunks = SLG_OTSU_ONE_CHUNKS;

struct StatsParams {
  const uint8_t* white[kMaxBatch];
  const uint8_t* black[kMaxBatch];
  WsHeader* wsv[kMaxBatch];
  int64_t n_px;
  int64_t n_state_words;   // look-back words zeroed here for the next main launch
  int32_t thresh_mode;
  int32_t pad;
  double shadow_val;
  double contrast_val;
  int32_t pad2[2];
  const uint32_t* parts[kMaxBatch];   // parts_kernel: per-tile partial histograms of each view
  int64_t n_parts;                    // tiles per view
  int64_t pad_zero;                   // zero pixels counted past n_px (removed from bin 0)
  uint32_t* hist_out;                 // one view, histograms only (slg_decode_histograms): no thresholds
};

// a / b correctly rounded from y = RN(1/b) (Markstein): with y correctly rounded and q1
// faithful, q2 = RN(q1 + (a - b*q1) * y) = RN(a / b); q0 = RN(a*y) is within 1.5 ulp, so one
// correction makes q1 faithful and the second one is exact (tools/markstein_check.c checks it
// against IEEE division).  Valid while nothing over/underflows: div_rn_ok() vets a, the
// caller vets b and y.
__device__ inline double div_rn(double a, double b, double y) {
  const double q0 = a * y;
  const double q1 = fma(fma(-b, q0, a), y, q0);
  return fma(fma(-b, q1, a), y, q1);
}
__device__ inline bool div_rn_ok(double a) {
  const double m = fabs(a);
  return m == 0.0 || (m > 0x1p-900 && m < 0x1p900);
}

// OpenCV getThreshVal_Otsu_8u (see oracle/sl_oracle.py:otsu_from_hist) evaluated by one wave.
// Bit-exact with the sequential fp64 loop: only order-independent pieces run in parallel.
//  * mu = sum(i*h[i]) of exact integers (< 2^53) == OpenCV's sequential double sum;
//  * q1 (running sum of p_i = h[i]*scale) is one sequential add chain (same rounding as the
//    loop); it alone decides which bins OpenCV skips, so the skip flags, i*p_i and
//    y = RN(1/q1) are then computed lane-parallel, bin i on lane i/4;
//  * the remaining chain mu1 = (mu1*q1_prev + i*p_i)/q1 runs on wave-uniform registers up to
//    the last unskipped bin, each division as the Markstein pair div_rn(., q1, y) (IEEE
//    division when div_rn_ok refuses the numerator): 7 dependent fp64 ops per bin instead of a
//    full IEEE division sequence;
//  * sigma per bin and the first-maximum argmax (strict '>' from 0) are lane-parallel.
__device__ inline double readlane_f64(double v, int l) {
  const uint64_t b = uint64_t(__double_as_longlong(v));
  const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(b), l);
  const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(b >> 32), l);
  return __longlong_as_double((long long)((uint64_t(hi) << 32) | lo));
}

// otsu_wave's exact mu1 run over bins [lo, hi] (the rerun when the speculative chain misses):
// each quotient as the Markstein pair div_rn(a, q1, y).
__device__ inline void mu1_run_exact(int lo, int hi, const double (&ip)[4], const double (&q1r)[4],
                                     const double (&yr)[4], double (&m1r)[4]) {
  const int lane = threadIdx.x & 63;
  double mu1 = 0.0, q_prev = 0.0;                    // bin i's previous q1 is bin i-1's q1 (mu1 = 0 at lo)
  for (int l = lo >> 2; l <= (hi >> 2); ++l) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * l + j;
      if (i < lo || i > hi) continue;                // scalar: first and last lane only
      const double a = mu1 * q_prev + readlane_f64(ip[j], l);
      q_prev = readlane_f64(q1r[j], l);
      mu1 = div_rn(a, q_prev, readlane_f64(yr[j], l));
      if (lane == l) m1r[j] = mu1;
    }
  }
}

// Pixels of a 256-bin histogram at or above bin m (the wave's sum).  n when m <= 0: the clipped
// difference histogram puts every negative white - black into bin 0, so it cannot tell which of
// them reach a threshold below 1 (for white, m <= 0 is every pixel anyway).
__device__ __attribute__((always_inline)) inline int64_t hist_at_least_wave(const uint32_t* h, int m, int64_t n) {
  if (m <= 0) return n;
  const int lane = threadIdx.x & 63;
  uint64_t a = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = 64 * j + lane;
    if (b >= m) a += h[b];
  }
  return int64_t(wave_sum(a));
}

// The resident-job arena reservation of one view, by the thread that finishes its thresholds,
// from its two `above` counts: see WsHeader::arena_off.
__device__ inline void arena_reserve(WsHeader* ws, int64_t a0, int64_t a1) {
  unsigned long long* cur = ws->arena_cursor;
  if (!cur) return;
  const int64_t need = (a0 < a1 ? a0 : a1) * int64_t(ws->arena_mult);
  const int64_t off = int64_t(atomicAdd(cur, (unsigned long long)need));
  ws->arena_off = off + need <= ws->arena_cap ? off : -1;
}

// The two serial chains of otsu_wave (q1, then mu1) run on wave-uniform registers fed from LDS:
// every lane computes the same chain, its per-bin operands read as broadcast LDS words, and only
// the value after each lane's four bins is captured (one 64-bit select per four steps); each
// lane then redoes its own four steps from its left neighbour's capture -- the same operations on
// the same values in the same order, so the same bits.  A dependent fp64 op costs ~5 clocks
// (tools/dp_latency_probe.hip), so a step costs its instruction count (profiles/r5y: 7.8 us for
// one 1080p histogram).  lds: kOtsuLds doubles of this wave's own.
#ifndef SLG_OTSU_MARK
#define SLG_OTSU_MARK(k)                   // tools/otsu_probe.hip: a timestamp per part of otsu_wave
#endif
#ifndef SLG_OTSU_UNROLL
#define SLG_OTSU_UNROLL 2                  // the chain loops: steps per loop body
#endif
constexpr int kOtsuLds = 5 * 256;          // p_i [256] + the mu1 chain's {q1[i-1], ip, y, c} [256][4]

__device__ __attribute__((always_inline)) inline double otsu_wave(const uint32_t* h, int64_t n, double* lds) {
  SLG_OTSU_MARK(0);
  const int lane = threadIdx.x & 63;
  const double scale = 1.0 / double(n);
  const double eps = double(__FLT_EPSILON__);
  double* sp = lds;                 // p_i
  double pv[4], ip[4], q1r[4], yr[4], m1r[4], ar[4];
  uint64_t isum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = 4 * lane + j;
    pv[j] = double(h[i]) * scale;
    ip[j] = double(i) * pv[j];
    isum += uint64_t(i) * h[i];
    q1r[j] = yr[j] = m1r[j] = ar[j] = 0.0;
    sp[i] = pv[j];
  }
  isum = wave_sum(isum);
  const double mu = double(isum) * scale;
  SLG_OTSU_MARK(1);
  // 1. the q1 chain (OpenCV's order) from broadcast LDS reads (wave-local: the wave's own LDS ops
  // are in order, the fence only keeps the compiler from moving them)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    double q1 = 0.0, qcap = 0.0;
#pragma unroll SLG_OTSU_UNROLL
    for (int l0 = 0; l0 < 64; l0 += 4) {
      double pp[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) pp[k] = sp[4 * l0 + k];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) q1 = q1 + pp[4 * t + j];
        qcap = lane == l0 + t ? q1 : qcap;
      }
    }
    double q = __shfl_up(qcap, 1);
    if (lane == 0) q = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q = q + pv[j];
      q1r[j] = q;
    }
  }
  SLG_OTSU_MARK(2);
  uint32_t okr = 0;                                  // 2. bit j: bin 4*lane+j not skipped
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double q2 = 1.0 - q1r[j];
    if (!(fmin(q1r[j], q2) < eps || fmax(q1r[j], q2) > 1.0 - eps)) {
      okr |= 1u << j;
      yr[j] = 1.0 / q1r[j];
    }
  }
  // 3. the mu1 chain.  The unskipped bins form one run [lo, hi]: q1 never decreases and
  // q2 = RN(1 - q1) never increases, so each skip test holds on a prefix plus a suffix of the
  // bins, and mu1 is still 0 at lo.  Over the run every bin is the same few dependent ops,
  // each quotient taken speculatively as fma(a, y, a * c) with c = fma(-q1, y, 1) * y (y + c
  // is 1/q1 to ~2^-105): faithful, and RN(a / q1) unless a / q1 sits within ~2^-105 of a
  // rounding boundary -- so every bin is checked afterwards (Markstein: RN(m + (a - q1 m) y)
  // = RN(a / q1) for faithful m) and the run is redone exactly on a miss.  That needs every
  // numerator to suit div_rn: a is 0, or at least ~1/n (an empty bin's mu1 *= q1 then / q1
  // moves a by ulps), so n <= 2^52 keeps a far inside its range.  Anything else (never seen)
  // takes the general loop: per-bin skip flags, IEEE division when refused.
  SLG_OTSU_MARK(3);
  const uint64_t lanes_ok = __ballot(okr != 0);
  int lo = 256, hi = -1, n_ok = 0;
  if (lanes_ok) {
    const int l_lo = __builtin_ctzll(lanes_ok), l_hi = 63 - __builtin_clzll(lanes_ok);
    lo = 4 * l_lo + __builtin_ctz(__builtin_amdgcn_readlane(okr, l_lo));
    hi = 4 * l_hi + 31 - __builtin_clz(__builtin_amdgcn_readlane(okr, l_hi));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) n_ok += __popcll(__ballot((okr >> j) & 1u));
  double mu1 = 0.0;
  SLG_OTSU_MARK(4);
  if (n_ok == hi - lo + 1 && n <= (int64_t(1) << 52)) {
    {                                                // per bin {q1[i-1], ip, y, c}, 32 bytes
      double* sops = lds + 256;
      const double qprev0 = __shfl_up(q1r[3], 1);
      double cr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double* o = sops + 4 * (4 * lane + j);
        cr[j] = fma(-q1r[j], yr[j], 1.0) * yr[j];
        o[0] = j == 0 ? qprev0 : q1r[j - 1];
        o[1] = ip[j];
        o[2] = yr[j];
        o[3] = cr[j];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // the chain over [lo, hi] (mu1 is 0 at lo, whatever q1[lo-1]), one capture per 4 bins:
      // mcap of lane l = mu1 after bin min(4l + 3, hi)
      double mu1c = 0.0, mcap = 0.0;
      const int g_lo = lo >> 2, g_hi = hi >> 2;
      // the edge groups (partial) apart, so the middle ones are one straight-line body the
      // scheduler can unroll and issue the next group's LDS reads ahead in (an explicitly
      // double-buffered form measured no faster: the buffers were shuffled through extra
      // registers, profiles/r5x)
      auto edge = [&](int l) {
        double o[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) o[k] = sops[16 * l + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * l + j;
          if (i >= lo && i <= hi) {                  // (wave-uniform)
            const double a = mu1c * o[4 * j] + o[4 * j + 1];
            mu1c = fma(a, o[4 * j + 2], a * o[4 * j + 3]);
          }
        }
        mcap = lane == l ? mu1c : mcap;
      };
      edge(g_lo);
#pragma unroll SLG_OTSU_UNROLL
      for (int l = g_lo + 1; l < g_hi; ++l) {
        double o[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) o[k] = sops[16 * l + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double a = mu1c * o[4 * j] + o[4 * j + 1];
          mu1c = fma(a, o[4 * j + 2], a * o[4 * j + 3]);
        }
        mcap = lane == l ? mu1c : mcap;
      }
      if (g_hi > g_lo) edge(g_hi);
      // every lane redoes its own bins from its left neighbour's capture (0 before g_lo)
      double m = __shfl_up(mcap, 1);
      if (lane <= g_lo) m = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * lane + j;
        const double qp = j == 0 ? qprev0 : q1r[j - 1];
        const double a = m * qp + ip[j];
        const double mj = fma(a, yr[j], a * cr[j]);
        if (i >= lo && i <= hi) {
          m = mj;
          m1r[j] = mj;
          ar[j] = a;
        }
      }
    }
    SLG_OTSU_MARK(5);
    uint32_t miss = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double r = fma(-q1r[j], m1r[j], ar[j]);   // exact remainder
      if ((okr >> j) & 1u) miss |= uint32_t(fma(r, yr[j], m1r[j]) != m1r[j]);
    }
    if (__ballot(miss != 0)) mu1_run_exact(lo, hi, ip, q1r, yr, m1r);
  } else {
    const int l_end = 64 - __builtin_clzll(lanes_ok | 1ull);   // lanes with work: [0, l_end)
    double q_prev = 0.0;
    for (int l = 0; l < l_end; ++l) {
      const uint32_t okl = __builtin_amdgcn_readlane(okr, l);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mu1 *= q_prev;                               // mu1 *= q1 (previous q1)
        const double q = readlane_f64(q1r[j], l);
        if (okl & (1u << j)) {
          const double a = mu1 + readlane_f64(ip[j], l);
          mu1 = div_rn_ok(a) ? div_rn(a, q, readlane_f64(yr[j], l)) : a / q;
          if (lane == l) m1r[j] = mu1;
        }
        q_prev = q;
      }
    }
  }
  SLG_OTSU_MARK(6);
  double best = 0.0;
  int best_i = INT_MAX;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!(okr & (1u << j))) continue;
    const double q1j = q1r[j], q2 = 1.0 - q1j, mu1j = m1r[j];
    const double mu2 = (mu - q1j * mu1j) / q2;
    const double sigma = q1j * q2 * (mu1j - mu2) * (mu1j - mu2);
    if (sigma > best) { best = sigma; best_i = 4 * lane + j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(best_i, o);
    if (ob > best || (ob == best && oi < best_i)) { best = ob; best_i = oi; }
  }
  SLG_OTSU_MARK(7);
  return best_i == INT_MAX ? 0.0 : double(best_i);
}

// smallest integer x in [lo, 256] with double(x) > thr (256 = none reachable)
__device__ inline int int_threshold(double thr, int lo) {
  if (!(thr == thr)) return 256;                 // NaN: comparison always false
  if (thr < double(lo)) return lo;
  if (thr >= 256.0) return 256;
  return int(floor(thr)) + 1;
}

// k-th smallest value (0-based) from a 256-bin histogram.
__device__ __attribute__((always_inline)) inline int kth_from_hist(const uint32_t* h, int64_t k) {
  int64_t c = 0;
  for (int v = 0; v < 256; ++v) {
    c += h[v];
    if (c > k) return v;
  }
  return 255;
}

// np.percentile(float32 image, 95) with method 'linear' (numpy 2.x _quantile/_lerp, float32).
__device__ __attribute__((always_inline)) inline float percentile95_from_hist(const uint32_t* h, int64_t n) {
  const float q = 95.0f / 100.0f;                       // np.true_divide(95, float32(100))
  const float vi = float(n - 1) * q;                    // (n-1) * quantiles, float32
  float prev = floorf(vi);
  float next = prev + 1.0f;
  const float gamma = vi - prev;
  int64_t pi = int64_t(prev), ni = int64_t(next);
  if (vi >= float(n - 1)) { pi = n - 1; ni = n - 1; }   // index -1 -> last element
  const float a = float(kth_from_hist(h, pi));
  const float b = float(kth_from_hist(h, ni));
  const float diff = b - a;
  float r = a + diff * gamma;
  if (gamma >= 0.5f) r = b - diff * (1.0f - gamma);
  return r;
}

// ---- Otsu histograms on the i8 matrix cores.  For 64 pixels v_k (k = 16 * lane-group + byte),
// A[m][k] = 16 * [v_k >> 4 == m] and B[k][n] = 16 * [v_k & 15 == n], so one
// v_mfma_i32_16x16x64_i8 adds 256 x the count of every value v = 16m + n: no LDS atomics (which
// retire about one lane per clock).  The 16 lanes of a row group (lane >> 4) hold the same 16
// pixels, each against its own m or n = lane & 15.  Operand dwords are built in two VALU ops:
// ((nib ^ (m ^ 15)) + 1) & 0x10 = 16 - (nib ^ m) masked to bit 4, i.e. 0x10 iff nib == m (no
// carries between bytes: every byte stays in 1..16).  Lane maps checked by
// tools/mfma_hist_probe.hip; C/D: col = lane & 15, row = 4 * (lane >> 4) + r.
//
// main3's carried count (hist_next_count: other waves' pixels) stages nibble planes in LDS and
// reads them with broadcast ds_read_b128.  stats_kernel counts each wave's own pixels
// (hist_chunk_dpp): MFMA step i takes row group g's pixels from lane 16 g + i by a DPP
// row_newbcast folded into the operand's add, so no LDS at all -- the LDS form read 4 KB per wave
// and step through the CU's LDS port, four waves per CU, which bounded the count.  The folded
// add cannot also take the xor, so those operands are step functions, 0x10 iff nib >= m
// ((nib + 16 - m) & 0x10), the MFMA sums S[m][n] = #{hi >= m, lo >= n}, and the wave's
// histogram is the 2-D difference S[m][n] - S[m+1][n] - S[m][n+1] + S[m+1][n+1] taken once on
// the accumulators (hist_from_cumulative).
typedef int v4i32 __attribute__((ext_vector_type(4)));
constexpr int kHistChunk = 1024;            // pixels per wave and MFMA chunk (16 per lane)
constexpr int64_t kHistMaxChunks = 8000;    // per wave: 8000 * 1024 * 256 < 2^31 (i32 accumulators)

__device__ inline uint32_t sub_sat_u8x4(uint32_t w, uint32_t b) {   // per byte max(w - b, 0)
  const uint32_t dl = ((w & 0x00ff00ffu) | 0x01000100u) - (b & 0x00ff00ffu);   // 256 + w - b
  const uint32_t dh = (((w >> 8) & 0x00ff00ffu) | 0x01000100u) - ((b >> 8) & 0x00ff00ffu);
  const uint32_t ml = ((dl >> 8) & 0x00010001u) * 0xffu, mh = ((dh >> 8) & 0x00010001u) * 0xffu;
  return (dl & ml) | ((dh & mh) << 8);
}

__device__ inline int onehot16(uint32_t nib, uint32_t repx) {      // bytes: 0x10 iff nib == m
  return int(((nib ^ repx) + 0x01010101u) & 0x10101010u);
}

// Step I of a chunk: per byte 0x10 iff the nibble of lane 16 * (lane >> 4) + I >= m, where
// c = (16 - m) per byte, m = lane & 15.  Bytes stay in 1..31: no carries.
template <int I>
__device__ inline int ge16_bcast(uint32_t plane, uint32_t c) {
  const uint32_t b = uint32_t(__builtin_amdgcn_update_dpp(0, int(plane), 0x150 + I, 0xf, 0xf, false));  // row_newbcast:I
  return int((b + c) & 0x10101010u);
}

// pl: the lane's 16 pixels as nibble planes {hi(w)[4], lo(w)[4], hi(d)[4], lo(d)[4]}
template <int I>
__device__ inline void hist_step_dpp(const uint32_t (&pl)[16], uint32_t c, v4i32& acc_w, v4i32& acc_d) {
  const v4i32 aw = {ge16_bcast<I>(pl[0], c), ge16_bcast<I>(pl[1], c), ge16_bcast<I>(pl[2], c), ge16_bcast<I>(pl[3], c)};
  const v4i32 bw = {ge16_bcast<I>(pl[4], c), ge16_bcast<I>(pl[5], c), ge16_bcast<I>(pl[6], c), ge16_bcast<I>(pl[7], c)};
  const v4i32 ad = {ge16_bcast<I>(pl[8], c), ge16_bcast<I>(pl[9], c), ge16_bcast<I>(pl[10], c), ge16_bcast<I>(pl[11], c)};
  const v4i32 bd = {ge16_bcast<I>(pl[12], c), ge16_bcast<I>(pl[13], c), ge16_bcast<I>(pl[14], c), ge16_bcast<I>(pl[15], c)};
  acc_w = __builtin_amdgcn_mfma_i32_16x16x64_i8(aw, bw, acc_w, 0, 0, 0);
  acc_d = __builtin_amdgcn_mfma_i32_16x16x64_i8(ad, bd, acc_d, 0, 0, 0);
}

template <int... Is>
__device__ inline void hist_steps_dpp(std::integer_sequence<int, Is...>, const uint32_t (&pl)[16], uint32_t c,
                                      v4i32& acc_w, v4i32& acc_d) {
  (hist_step_dpp<Is>(pl, c, acc_w, acc_d), ...);
}

// One wave adds its 1024 pixels (pixel c + 16 * lane + byte: white w[], clip(white - black) d[])
// into its cumulative accumulators S_w, S_d (256 x #{hi >= m, lo >= n}).
__device__ inline void hist_chunk_dpp(const uint32_t (&w)[4], const uint32_t (&d)[4], v4i32& acc_w, v4i32& acc_d) {
  const uint32_t m4 = 0x0f0f0f0fu;
  const uint32_t c = (16u - uint32_t(threadIdx.x & 15)) * 0x01010101u;
  uint32_t pl[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pl[q] = (w[q] >> 4) & m4; pl[4 + q] = w[q] & m4;
    pl[8 + q] = (d[q] >> 4) & m4; pl[12 + q] = d[q] & m4;
  }
  hist_steps_dpp(std::make_integer_sequence<int, 16>(), pl, c, acc_w, acc_d);
}

// S (this lane's C/D entries: row 4 * (lane >> 4) + r, col lane & 15) -> the histogram entries
// S[m][n] - S[m+1][n] - S[m][n+1] + S[m+1][n+1], S past row / column 15 being 0.
__device__ inline v4i32 hist_from_cumulative(v4i32 s) {
  const int lane = threadIdx.x & 63;
  const int below = __shfl_down(s[0], 16);        // row 4 * (g + 1): lane + 16, same column
  v4i32 dm;
  dm[0] = s[0] - s[1]; dm[1] = s[1] - s[2]; dm[2] = s[2] - s[3]; dm[3] = s[3] - (lane < 48 ? below : 0);
  v4i32 h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int right = __shfl_down(dm[r], 1);       // column n + 1: lane + 1
    h[r] = dm[r] - ((lane & 15) != 15 ? right : 0);
  }
  return h;
}

// 16 pixels of white and clip(white - black) for lane `lane` of the chunk at c; bytes at or
// past n_px read as 0 (the last arriver removes them from bin 0).
__device__ inline void hist_load(const uint8_t* white, const uint8_t* black, int64_t c, int64_t n_px,
                                 uint32_t (&w)[4], uint32_t (&d)[4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int h = 0; h < 2; ++h) {             // two 8-byte loads
    const int64_t o = c + 16 * lane + 8 * h;
    const int64_t so = o < n_px ? o : 0;    // frames readable to round_up(n, 8)
    uint2 wq = ld_once8(white + so);
    uint2 bq = ld_once8(black + so);
    if (o + 8 > n_px) {                     // tail: zero the bytes at or past n_px
      const int64_t keep = n_px - o;        // <= 0: none
      const uint64_t mk = keep <= 0 ? 0 : (~0ull >> (64 - 8 * keep));
      wq.x &= uint32_t(mk); wq.y &= uint32_t(mk >> 32);
      bq.x &= uint32_t(mk); bq.y &= uint32_t(mk >> 32);
    }
    w[2 * h] = wq.x; w[2 * h + 1] = wq.y;
    d[2 * h] = sub_sat_u8x4(wq.x, bq.x); d[2 * h + 1] = sub_sat_u8x4(wq.y, bq.y);
  }
}

// The mask thresholds of a view from its summed histograms into ws (stats_kernel's last arriver,
// hist_thresholds_kernel): Otsu of hg[0..255] (white) and hg[256..511] (clip(white - black)) by
// waves 0 and 1 concurrently, with the bound of the valid pixels (WsHeader::above); or the
// percentile rule from hg[0..255] (black) and maxd = max(white - black) + 256.  otsu_lds: two
// waves' kOtsuLds doubles.  Then the resident-job arena reservation (no cursor: nothing).
__device__ __attribute__((always_inline)) inline void set_thresholds(const uint32_t* hg, uint32_t maxd, int64_t n_px,
                                                                     bool otsu, WsHeader* ws, double* otsu_lds,
                                                                     int64_t* s_above) {
  const int tid = threadIdx.x, wave = tid >> 6;
  if (otsu) {
    if (wave < 2) {                            // wave 0: white, wave 1: clip(w-b); concurrently
      const double thr = otsu_wave(hg + 256 * wave, n_px, otsu_lds + wave * kOtsuLds);
      const int m = int_threshold(thr, wave == 0 ? 0 : -255);
      const int64_t above = hist_at_least_wave(hg + 256 * wave, m, n_px);
      if ((tid & 63) == 0) {
        if (wave == 0) { ws->smin = m; ws->thr_s = thr; } else { ws->cmin = m; ws->thr_c = thr; }
        ws->above[wave] = above;
        s_above[wave] = above;
      }
    }
  } else if (tid < 2) {
    double thr;
    if (tid == 0) {
      const float nf = percentile95_from_hist(hg, n_px);
      thr = double(nf * 1.5f);                           // noise_floor * 1.5 (float32)
    } else {
      const float dr = float(int(maxd) - 256);           // np.max(contrast)
      thr = double(dr * 0.05f);                          // dynamic_range * 0.05 (float32)
    }
    const int m = int_threshold(thr, tid == 0 ? 0 : -255);
    if (tid == 0) { ws->smin = m; ws->thr_s = thr; } else { ws->cmin = m; ws->thr_c = thr; }
    ws->above[tid] = n_px;                     // (the percentile histogram is black's: no bound)
    s_above[tid] = n_px;
  }
  __syncthreads();
  if (tid == 0) arena_reserve(ws, s_above[0], s_above[1]);
}

#ifndef SLG_STATS_MINB
#define SLG_STATS_MINB 1     // stats_kernel workgroups per CU its registers are budgeted for
#endif

// The view's histogram copies summed into hg[0..511] by 256 lanes (lane t: bins t and t + 256),
// every copy of both bins loaded before any is summed: one round trip (a loop over the two bins
// took two, 1.6 us of a one-view call's stats launch).  pad: the zero padding past n_px, taken
// off bins 0 and 256.  Agent-scope atomic loads: see stats_kernel's ticket.
__device__ __attribute__((always_inline)) inline void sum_hist_copies(const uint32_t* hist_part, int tid, uint32_t pad,
                                                                     uint32_t* hg) {
  uint32_t v[2][kHistCopies];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < kHistCopies; ++c)
      v[r][c] = __hip_atomic_load(hist_part + c * 512 + tid + 256 * r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < kHistCopies; ++c) acc += v[r][c];
    hg[tid + 256 * r] = acc - (tid == 0 ? pad : 0u);
  }
}

__global__ __launch_bounds__(kBlock, SLG_STATS_MINB) void stats_kernel(StatsParams p) {
  // 16 sub-histograms per kind (wave x lane&3), rows padded to 257 words so the copies of one
  // bin sit in different banks: a flat background costs at most 16-way same-address adds.
  constexpr int kRow = 257;
  __shared__ __attribute__((aligned(16))) uint32_t sh[16 * 2 * kRow];
  static_assert(512 * 4 + 2 * kOtsuLds * 8 <= 16 * 2 * kRow * 4, "Otsu tail: histograms + two waves' LDS");
  __shared__ uint32_t s_maxd;
  __shared__ uint32_t s_last;
  __shared__ int64_t s_above[2];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int view = blockIdx.y;               // batched launches: one grid row per view
  WsHeader* ws = p.wsv[view];
  const uint8_t* white = p.white[view];
  const uint8_t* black = p.black[view];
  uint32_t* hist_part = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws) + kHistPartOff);
  uint64_t* states = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ws) + states_off(p.n_px));

  // Arm the compaction state of the following main launch (ordered by the kernel boundary).
  for (int64_t i = int64_t(blockIdx.x) * kBlock + tid; i < p.n_state_words; i += int64_t(gridDim.x) * kBlock)
    states[i] = 0;
  if (blockIdx.x == 0 && tid == 0) ws->lb_ticket = ws->lb_ticket_row = 0;

  if (p.thresh_mode == SLG_THRESH_MANUAL) {
    if (blockIdx.x == 0 && tid < 2) {
      const double thr = tid == 0 ? p.shadow_val : p.contrast_val;
      const int m = int_threshold(thr, tid == 0 ? 0 : -255);
      if (tid == 0) { ws->smin = m; ws->thr_s = thr; } else { ws->cmin = m; ws->thr_c = thr; }
      ws->above[tid] = p.n_px;                 // manual thresholds: no histogram, no bound
    }
    if (blockIdx.x == 0 && tid == 0) arena_reserve(ws, p.n_px, p.n_px);
    return;
  }

  for (int i = tid; i < 16 * 2 * kRow; i += kBlock) sh[i] = 0;
  if (tid == 0) s_maxd = 0;
  __syncthreads();

  // hist kinds: otsu -> [0] white, [1] clip(white-black); percentile -> [0] black.
  const bool otsu = p.thresh_mode == SLG_THRESH_OTSU;
  if (otsu) {                                  // matrix-core histograms (hist_chunk_dpp)
    v4i32 acc_w = {0, 0, 0, 0}, acc_d = {0, 0, 0, 0};
    const int lane = tid & 63;
    const int64_t step = int64_t(gridDim.x) * (kBlock / 64) * kHistChunk;
    int64_t c = (int64_t(blockIdx.x) * (kBlock / 64) + wave) * kHistChunk;
    uint32_t w[4], d[4];
    if (c < p.n_px) hist_load(white, black, c, p.n_px, w, d);
    for (; c < p.n_px; c += step) {            // next chunk's loads in flight during the MFMAs
      uint32_t wn[4], dn[4];
      const bool more = c + step < p.n_px;
      if (more) hist_load(white, black, c + step, p.n_px, wn, dn);
      hist_chunk_dpp(w, d, acc_w, acc_d);
      if (more) {
#pragma unroll
        for (int q = 0; q < 4; ++q) { w[q] = wn[q]; d[q] = dn[q]; }
      }
    }
    acc_w = hist_from_cumulative(acc_w);
    acc_d = hist_from_cumulative(acc_d);
#pragma unroll
    for (int r = 0; r < 4; ++r) {              // wave sub-histograms: row-major bins 16*row + col
      const int bin = 16 * (4 * (lane >> 4) + r) + (lane & 15);
      if (acc_w[r]) atomicAdd(&sh[(2 * wave) * kRow + bin], uint32_t(acc_w[r]) >> 8);
      if (acc_d[r]) atomicAdd(&sh[(2 * wave + 1) * kRow + bin], uint32_t(acc_d[r]) >> 8);
    }
  }
  // percentile: LDS adds into 16 sub-histograms, kStatsPx consecutive pixels per lane and step
  uint32_t local_max = 0;
  if (!otsu) {
    uint32_t* h0 = sh + (4 * wave + (tid & 3)) * 2 * kRow;
    const int64_t per_block = int64_t(kBlock) * kStatsPx;
    for (int64_t b0 = int64_t(blockIdx.x) * per_block; b0 < p.n_px; b0 += int64_t(gridDim.x) * per_block) {
      const int64_t px0 = b0 + int64_t(tid) * kStatsPx;
      uint2 w[kStatsPx / 8], b[kStatsPx / 8];
#pragma unroll
      for (int q = 0; q < kStatsPx / 8; ++q) {
        const int64_t o = px0 + 8 * q < p.n_px ? px0 + 8 * q : 0;   // frames readable to round_up(n, 8)
        w[q] = *reinterpret_cast<const uint2*>(white + o);
        b[q] = *reinterpret_cast<const uint2*>(black + o);
      }
      // (a guard, not a break: with the break the loop stayed rolled and w[] / b[] went to
      // scratch, indexed at run time)
#pragma unroll
      for (int k = 0; k < kStatsPx; ++k) {
        if (px0 + k < p.n_px) {
          const uint2 wq = w[k >> 3], bq = b[k >> 3];
          const int wv = (((k & 7) < 4 ? wq.x : wq.y) >> (8 * (k & 3))) & 0xff;
          const int bv = (((k & 7) < 4 ? bq.x : bq.y) >> (8 * (k & 3))) & 0xff;
          atomicAdd(&h0[bv], 1u);
          local_max = max(local_max, uint32_t(wv - bv + 256));
        }
      }
    }
  }
  if (!otsu) atomicMax(&s_maxd, local_max);
  __syncthreads();
  for (int i = tid; i < 2 * 256; i += kBlock) {
    const int kind = i >> 8, bin = i & 255;
    uint32_t v = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) v += sh[(2 * c + kind) * kRow + bin];
    if (v) atomicAdd(hist_part + (blockIdx.x % kHistCopies) * 512 + i, v);
  }
  if (!otsu && tid == 0 && s_maxd) atomicMax(&ws->max_diff_enc, s_maxd);

  // Publish (every wave drains its atomics, barrier) then take a ticket.  Hardware assumption
  // (no release / acquire fences): what the last arriver reads -- the histogram copies,
  // max_diff_enc -- is written and read by agent-scope atomics only, which gfx950 performs at
  // the L2 that owns the address (the device's point of coherence for agent scope, whichever
  // XCD issues them); a returned vmcnt means the add has been performed there, so a ticket
  // taken after vmcnt(0) orders every earlier add before the last arriver's atomic loads.  No
  // L2 write-back or invalidate is needed (an agent-scope fence is one of each, per workgroup).
  // tests/test_gpu_configs.py::test_concurrent_stats_thresholds checks the thresholds of many
  // concurrent multi-view launches against the oracle.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t t = __hip_atomic_fetch_add(&ws->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == gridDim.x - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;

  // Last arriver: read the global histograms, compute thresholds, reset for reuse.
  uint32_t* hg = sh;                           // reuse the sub-histograms for the global ones
  sum_hist_copies(hist_part, tid, otsu ? uint32_t(p.pad_zero) : 0u, hg);
  if (tid == 0) s_maxd = __hip_atomic_load(&ws->max_diff_enc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (p.hist_out) {                            // histograms only: a band of a view split over ranks
    for (int i = tid; i < 512; i += kBlock) p.hist_out[i] = hg[i];
    if (tid == 0) p.hist_out[512] = s_maxd;
  } else {
    set_thresholds(hg, s_maxd, p.n_px, otsu, ws, reinterpret_cast<double*>(sh + 512), s_above);
  }
  for (int i = tid; i < kHistCopies * 512; i += kBlock) hist_part[i] = 0;
  if (tid == 0) { ws->max_diff_enc = 0; ws->ticket = 0; }
}

// Thresholds of a view whose histograms were summed over the bands of rows the ranks hold
// (slg_thresholds_from_histograms; SURVEY 8(e), the one exchange step of a single-view split):
// block 0 runs set_thresholds on hist[513] (as slg_decode_histograms wrote it, summed), every
// block zeroes this band's look-back words for the following fused launch (kernel boundary).
__global__ __launch_bounds__(kBlock) void hist_thresholds_kernel(const uint32_t* hist, WsHeader* ws, int64_t n_px,
                                                                 int32_t thresh_mode, int64_t n_state_words) {
  __shared__ __attribute__((aligned(16))) uint32_t hg[512 + 4 * kOtsuLds];
  __shared__ int64_t s_above[2];
  const int tid = threadIdx.x;
  uint64_t* states = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ws) + states_off(0));
  for (int64_t i = int64_t(blockIdx.x) * kBlock + tid; i < n_state_words; i += int64_t(gridDim.x) * kBlock)
    states[i] = 0;
  if (blockIdx.x != 0) return;
  if (tid == 0) ws->lb_ticket = ws->lb_ticket_row = 0;
  for (int i = tid; i < 512; i += kBlock) hg[i] = hist[i];
  __syncthreads();
  set_thresholds(hg, hist[512], n_px, thresh_mode == SLG_THRESH_OTSU, ws, reinterpret_cast<double*>(hg + 512), s_above);
}

// Otsu thresholds from the per-tile partial histograms a fused launch left in each view's
// workspace slice (the carried "batch after next", hist_next_*): the lean counterpart of
// stats_kernel for the streaming pipeline.  It runs on a side stream BESIDE a fused launch, so
// it holds as few CU resources as it can: 2 KB of LDS, no frame reads, every partial of a
// workgroup's tile range in flight at once (kPartsInFlight loads per lane), then <= 512 global
// adds, a ticket, and the same Otsu tail as stats_kernel in the last arriver.
constexpr int kPartsInFlight = 16;
constexpr int kPartsLdsWords = 512 + 4 * kOtsuLds + 4;
constexpr int kPartsBlocksMax = 64;         // workgroups per view (each sums a contiguous tile range)

// One workgroup's share of "thresholds from partials" for one view: workgroup `block` of
// `n_blocks` sums its contiguous range of the view's n_parts per-tile partials, adds them into
// the view's histogram copies, takes a ticket; the last arriver runs Otsu, writes the mask
// thresholds and resets the histogram state.  Also zeroes the view's look-back words (arming
// the main launch that will use these thresholds; ordered by the kernel boundary).  256 lanes;
// hg: kPartsLdsWords words of LDS (512 histogram words + 2 x kOtsuLds doubles + 2 int64,
// 16-byte aligned), s_last: one.  Used by parts_kernel and by main3's finishing workgroups.
__device__ __attribute__((always_inline)) inline void otsu_from_parts(const uint32_t* pp, WsHeader* ws, int64_t n_parts, int64_t n_px,
                                int64_t n_state_words, int64_t pad_zero, int block, int n_blocks,
                                uint32_t* hg, uint32_t* s_last) {
  const int tid = threadIdx.x, wave = tid >> 6;
  int64_t* s_above = reinterpret_cast<int64_t*>(hg + 512 + 4 * kOtsuLds);
  const bool act = tid < kBlock;               // the work is laid out for 256 lanes (a 512-lane
  uint32_t* hist_part = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws) + kHistPartOff);
  uint64_t* states = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ws) + states_off(n_px));
  if (act) {                                   // main3 workgroup's upper half only syncs)
    for (int64_t i = int64_t(block) * kBlock + tid; i < n_state_words; i += int64_t(n_blocks) * kBlock)
      states[i] = 0;
    if (block == 0 && tid == 0) ws->lb_ticket = ws->lb_ticket_row = 0;

    // thread t owns packed word t (bins 2t, 2t+1 of [white 0..255 | clip 256..511])
    const int64_t per = (n_parts + n_blocks - 1) / n_blocks;
    const int64_t t0 = int64_t(block) * per, t1 = t0 + per < n_parts ? t0 + per : n_parts;
    uint32_t a0 = 0, a1 = 0;
    for (int64_t k0 = t0; k0 < t1; k0 += kPartsInFlight) {
      uint32_t v[kPartsInFlight];
#pragma unroll
      for (int j = 0; j < kPartsInFlight; ++j)
        v[j] = k0 + j < t1 ? pp[(k0 + j) * kPartWords + tid] : 0u;
#pragma unroll
      for (int j = 0; j < kPartsInFlight; ++j) { a0 += v[j] & 0xffffu; a1 += v[j] >> 16; }
    }
    uint32_t* dst = hist_part + (block % kHistCopies) * 512 + 2 * tid;
    if (a0) atomicAdd(dst, a0);
    if (a1) atomicAdd(dst + 1, a1);
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (atomics only: see stats_kernel)
  __syncthreads();
  if (tid == 0) {
    const uint32_t t = __hip_atomic_fetch_add(&ws->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = (t == uint32_t(n_blocks) - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!*s_last) return;
  if (act) sum_hist_copies(hist_part, tid, uint32_t(pad_zero), hg);
  __syncthreads();
  if (wave < 2) {                              // wave 0: white, wave 1: clip(w-b); concurrently
    const double thr = otsu_wave(hg + 256 * wave, n_px, reinterpret_cast<double*>(hg + 512) + wave * kOtsuLds);
    const int m = int_threshold(thr, wave == 0 ? 0 : -255);
    const int64_t above = hist_at_least_wave(hg + 256 * wave, m, n_px);
    if ((tid & 63) == 0) {
      if (wave == 0) { ws->smin = m; ws->thr_s = thr; } else { ws->cmin = m; ws->thr_c = thr; }
      ws->above[wave] = above;
      s_above[wave] = above;
    }
  }
  __syncthreads();
  if (tid == 0) arena_reserve(ws, s_above[0], s_above[1]);
  for (int i = tid; act && i < kHistCopies * 512; i += kBlock) hist_part[i] = 0;
  if (tid == 0) { ws->max_diff_enc = 0; ws->ticket = 0; }
}

__global__ __launch_bounds__(kBlock) void parts_kernel(StatsParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t hg[kPartsLdsWords];   // + the Otsu tail's LDS
  __shared__ uint32_t s_last;
  otsu_from_parts(p.parts[blockIdx.y], p.wsv[blockIdx.y], p.n_parts, p.n_px, p.n_state_words, p.pad_zero,
                  int(blockIdx.x), int(gridDim.x), hg, &s_last);
}

// ------------------------------------------------------------------ main kernel
struct MainParams {
  // frames source
  const uint8_t* frames;
  int64_t stride;
  // maps source
  const int32_t* in_col;
  const int32_t* in_row;
  const uint8_t* in_mask;
  // common
  const uint8_t* texture;
  int64_t n_px;
  int32_t width;
  // decode plan (frame index of first pattern, pairs to read, pre-shift, post-shift)
  int32_t col_first, col_pairs, col_pre, col_post;
  int32_t row_first, row_pairs, row_pre, row_post;
  // maps output
  int32_t* out_col;
  int32_t* out_row;
  uint8_t* out_mask;
  // calibration
  const double* rays;
  double fx, fy, cx, cy;
  double rfx, rfy;            // RN(1/fx), RN(1/fy) when div_fast (Markstein divisions)
  int32_t div_fast;
  int32_t rays_fast;          // host-verified: every pixel's ray takes the Markstein path (tri_item FAST)
  double o0, o1, o2;
  int32_t num_pre;            // pcol (and prow in row_mode 2): split pair planes with numer, not d
  int32_t pad_np;
  const double* pcol;
  int32_t n_pcol;
  const double* prow;
  int32_t n_prow;
  double tol;
  // outputs
  void* xyz;
  uint8_t* bgr;
  int64_t* count;
  WsHeader* ws;
  uint64_t* states;        // [2][n_tiles]
  int64_t n_tiles;
  void* scratch_xyz;       // row_mode 2 row cloud
  uint8_t* scratch_bgr;
  int32_t dbg;             // env SLG_DBG; read only by the profiling instance (PROF): bit0 no
                           // look-back wait, bit1 trivial triangulation, bit2 no output stores,
                           // bit3 no BGR stores, bit6 per-workgroup phase records, bit7 no XYZ stores
  uint32_t help_after;     // look-back: s_sleep(2) units before a silent predecessor is helped
                           // (kHelpAfter; env SLG_HELP_AFTER=0 forces the helper path in tests)
};

// ------------------------------------------------------------------ decode (shared by the kernels)
// Bit planes of 4 pixels accumulate one byte per pixel: plane b's compare mask (bit 7 of each
// byte: pattern > inverse) enters at bit 7 while the earlier planes shift down, two VALU ops per
// word per plane.  Planes 0-7 go to word A, planes 8-14 to word B.  After n planes, bit-reversing
// the word (v_bfrev: bits within a byte AND the byte order) leaves pixel k's code MSB-first in
// byte 3-k: A' byte = code >> m, B' byte = code & (2^m - 1), m = max(n - 8, 0).
struct PlaneAcc {
  uint32_t a[2], b[2];       // [pixels 0-3, 4-7]
};

__device__ inline void acc_plane(uint32_t& w, uint32_t m) { w = (w >> 1) | (m & 0x80808080u); }

template <bool HI>
__device__ inline void acc_pair(PlaneAcc& q, uint2 pv, uint2 iv) {
  const uint32_t m0 = gt_u8x4(pv.x, iv.x);
  const uint32_t m1 = gt_u8x4(pv.y, iv.y);
  if (HI) { acc_plane(q.b[0], m0); acc_plane(q.b[1], m1); }
  else { acc_plane(q.a[0], m0); acc_plane(q.a[1], m1); }
}

// The n-plane Gray codes of the lane's 8 pixels as two per word (16-bit halves), converted
// like gray2bin_x2(code << pre) << post: w[2h] = pixels (4h, 4h+2) in (high, low) halves,
// w[2h+1] = pixels (4h+1, 4h+3).
__device__ inline void acc_codes(const PlaneAcc& q, int n, int pre, int post, uint32_t (&w)[4]) {
  const int m = n > 8 ? n - 8 : 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t A = __builtin_bitreverse32(q.a[h]), B = __builtin_bitreverse32(q.b[h]);
    const uint32_t hi = (((A >> 8) & 0x00ff00ffu) << m) | ((B >> 8) & 0x00ff00ffu);
    const uint32_t lo = ((A & 0x00ff00ffu) << m) | (B & 0x00ff00ffu);
    w[2 * h] = gray2bin_x2(hi << pre) << post;
    w[2 * h + 1] = gray2bin_x2(lo << pre) << post;
  }
}

// code of pixel k (0..7) from acc_codes' words
__device__ inline int unpack_code(const uint32_t (&w)[4], int k) {
  const uint32_t a = w[((k >> 2) << 1) | (k & 1)];
  return int((a >> (16 * (1 - ((k >> 1) & 1)))) & 0xffffu);
}

// 8 once-read bytes at base + off as a buffer load (scalar descriptor, 32-bit lane offset).
__device__ inline uint2 ld_once8_buf(const uint8_t* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, 0xffffffff, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, SLG_NT_LOADS ? 2 : 0);   // aux 2: nt
  return make_uint2(v[0], v[1]);
}

// A wave-uniform 64-bit value pinned to SGPRs: the compiler cannot fold a lane offset into it
// first, so frame f's address is (frames + lane offset) + one scalar term -- one VALU add per
// load instead of a 64-bit vector multiply-add.
__device__ inline int64_t sgpr64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(uint64_t(v)));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(uint64_t(v) >> 32));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// 8 frame bytes at pixel lp (clamped in-bounds by the caller; rows are padded to >= 8 px).
// As a buffer load: the frame's base lives in a scalar resource descriptor and the lane offset
// is a 32-bit VGPR (buffer_load_dwordx2 ... offen nt), so the address costs no VALU at all.
__device__ inline uint2 ld_frame8(const MainParams& p, int frame, int64_t lp) {
#if SLG_FRAME_BUFFER_LOADS
  // one descriptor for the whole stack, the frame's offset in the scalar soffset (a capture's
  // frames span < 4 GiB: check_capture)
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.frames), 0, 0xffffffff, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, uint32_t(lp), uint32_t(frame) * uint32_t(p.stride),
                                                      SLG_NT_LOADS ? 2 : 0);   // aux 2: nt
  return make_uint2(v[0], v[1]);
#else
  return ld_once8(p.frames + sgpr64(int64_t(frame) * p.stride) + uint32_t(lp));
#endif
}

// Paired 16-byte frame loads (two-axis decodes): lanes 2j and 2j+1 own pixels [q, q + 16) of the
// tile (q = the even lane's px0, a multiple of 16).  For a frame pair (a, a + 1) -- white / black,
// or a pattern / inverse pair -- the even lane reads 16 bytes of frame a and the odd lane 16 bytes
// of frame a + 1 at q, then the two trade halves (DPP quad_perm [1,0,3,2]), so each holds its own
// 8 pixels of both frames.  Half the vector-memory instructions of two 8-byte loads per lane and
// the same 128-byte lines (tools/fetch_probe.hip: C2's mask-gated reads 11.1 vs 12.1-12.4 us;
// the bench's C2 step 305.5 vs 309.8 us, f64 neutral, profiles/r7l).  Pairing the texture and the
// carried white / black loads too measured slower or neutral (306.2 / 310.6 us; as buffer loads
// 311.2 vs 310.5, profiles/r7l).  An unaligned caller stack keeps the 8-byte loads (GPU test).
// Needs 16-byte aligned frames and stride (else the 8-byte loads run) and both lanes of a pair
// active at the trade.

struct PairLd {
  uint32_t v[4];
};
__device__ inline PairLd ld_pair16(const MainParams& p, int frame_a, uint32_t voff) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.frames), 0, 0xffffffff, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, uint32_t(frame_a) * uint32_t(p.stride),
                                                       SLG_NT_LOADS ? 2 : 0);   // aux 2: nt
  return {{v[0], v[1], v[2], v[3]}};
}
// a = this lane's 8 bytes of frame a, b = of frame a + 1
__device__ inline void pair_split(const PairLd& L, bool odd, uint2& a, uint2& b) {
  const uint32_t s0 = odd ? L.v[0] : L.v[2], s1 = odd ? L.v[1] : L.v[3];
  const uint32_t r0 = uint32_t(__builtin_amdgcn_update_dpp(0, int(s0), 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  const uint32_t r1 = uint32_t(__builtin_amdgcn_update_dpp(0, int(s1), 0xB1, 0xf, 0xf, false));
  a = odd ? make_uint2(r0, r1) : make_uint2(L.v[0], L.v[1]);
  b = odd ? make_uint2(L.v[2], L.v[3]) : make_uint2(r0, r1);
}

// Decode the 8 pixels of one lane: mask bits + column / row codes.  Frame loads of both axes
// are issued up to kBatch pairs at a time before any is consumed (memory-level parallelism).
// `tail` (wave-uniform) is set only in the last tile, where map/texture reads need guards;
// frame reads never do: the frame stride is >= round_up(H*W, 8) and out-of-image lanes read
// pixel 0 (their mask bits are cleared).
// MF (mask first, the fused reconstruction only): the mask is computed from white / black before
// any pattern frame is read, and a lane none of whose 8 pixels is valid reads no pattern frame at
// all (its codes are never used: the reference masks them out, processing.py:121-124,157).  The
// memory system then fetches only the 64-byte segments a valid pixel lies in.  `pre()` runs once
// the lane is known to hold a valid pixel, before its pattern loads (the texture loads).
struct NoPre {
  __device__ void operator()(uint2) const {}
};

// PLAN: (col_pairs << 4) | row_pairs as compile-time constants (main3's specialised instances for
// the common capture layouts, SLG_PLAN_*; every view of such a launch has that plan), or 0: the
// counts come from the view's plan at run time.
// Constant counts make every frame load unconditional, so the decode consumes each pair as it
// lands (vmcnt(n) in issue order) instead of after a vmcnt(0) for the whole batch, and drop the
// per-pair branches (243.3 vs 259.8 us per 12-view launch, profiles/r3m).
template <int ROW_MODE, int SRC_FRAMES, int kBatch, bool MF = false, int PLAN = 0, class Pre = NoPre>
__device__ inline void decode_lane(const MainParams& p, int64_t px0, bool tail, uint32_t& valid,
                                   int (&col)[kPx], int (&row)[kPx], Pre pre = Pre()) {
  valid = 0;
  if (SRC_FRAMES) {
    const int smin = p.ws->smin, cmin = p.ws->cmin;
    const int64_t lp = px0 < p.n_px ? px0 : 0;
    // paired 16-byte loads (wave-uniform choice): the pair's base pixel, clamped like lp
    // (column-only decodes -- row_mode 0, C1's 10 pairs -- measured 2-5 % slower paired: there the
    // lanes a partner drags into the decode cost more than the halved loads save)
    const bool paired = ROW_MODE != 0 &&
                        ((reinterpret_cast<uintptr_t>(p.frames) | uint64_t(p.stride)) & 15) == 0;
    const bool odd = (threadIdx.x & 1) != 0;
    const int64_t q = px0 & ~int64_t(15);
    const uint32_t vo = uint32_t(q < p.n_px ? q : 0) + (odd ? uint32_t(p.stride) : 0u);
    uint2 w, bl;
    if (paired) pair_split(ld_pair16(p, 0, vo), odd, w, bl);
    else { w = ld_frame8(p, 0, lp); bl = ld_frame8(p, 1, lp); }
    if constexpr (MF) {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const int wv = ((k < 4 ? w.x : w.y) >> (8 * (k & 3))) & 0xff;
        const int bv = ((k < 4 ? bl.x : bl.y) >> (8 * (k & 3))) & 0xff;
        valid |= uint32_t((wv >= smin) & ((wv - bv) >= cmin) & (px0 + k < p.n_px)) << k;
        col[k] = 0;
        row[k] = 0;
      }
      // paired: a pair reads its pattern frames if either lane has a valid pixel (both must
      // take part in the trades); the other lane's codes are never used
      const uint32_t go = paired ? (valid | uint32_t(__builtin_amdgcn_update_dpp(0, int(valid), 0xB1, 0xf, 0xf, false)))
                                 : valid;
      if (go == 0u) return;
      if (valid != 0u) pre(w);                    // (white bytes: a gray capture's texture)
    }
    PlaneAcc qc = {{0, 0}, {0, 0}}, qr = {{0, 0}, {0, 0}};
    const int np_c = PLAN ? ((PLAN >> 4) & 15) : p.col_pairs;
    const int np_r = ROW_MODE == 0 ? 0 : (PLAN ? (PLAN & 15) : p.row_pairs);
    // compile-time trip count (kMaxBits pairs max), fully unrolled: only forward, wave-uniform
    // branches remain, so the loads of a batch stay in flight together (no vmcnt(0) per load)
    if (paired) {
#pragma unroll
      for (int b0 = 0; b0 < kMaxBits; b0 += kBatch) {
        PairLd cl[kBatch], rl[kBatch];
#pragma unroll
        for (int g = 0; g < kBatch; ++g)
          if (b0 + g < np_c) cl[g] = ld_pair16(p, p.col_first + 2 * (b0 + g), vo);
#pragma unroll
        for (int g = 0; g < kBatch; ++g)
          if (b0 + g < np_r) rl[g] = ld_pair16(p, p.row_first + 2 * (b0 + g), vo);
#pragma unroll
        for (int g = 0; g < kBatch; ++g)
          if (b0 + g < np_c) {
            uint2 pv, iv;
            pair_split(cl[g], odd, pv, iv);
            if (b0 + g < 8) acc_pair<false>(qc, pv, iv);
            else acc_pair<true>(qc, pv, iv);
          }
#pragma unroll
        for (int g = 0; g < kBatch; ++g)
          if (b0 + g < np_r) {
            uint2 pv, iv;
            pair_split(rl[g], odd, pv, iv);
            if (b0 + g < 8) acc_pair<false>(qr, pv, iv);
            else acc_pair<true>(qr, pv, iv);
          }
      }
    } else {
#pragma unroll
    for (int b0 = 0; b0 < kMaxBits; b0 += kBatch) {
      uint2 cp[kBatch], ci[kBatch], rp[kBatch], ri[kBatch];
#pragma unroll
      for (int g = 0; g < kBatch; ++g)
        if (b0 + g < np_c) {
          cp[g] = ld_frame8(p, p.col_first + 2 * (b0 + g), lp);
          ci[g] = ld_frame8(p, p.col_first + 2 * (b0 + g) + 1, lp);
        }
#pragma unroll
      for (int g = 0; g < kBatch; ++g)
        if (b0 + g < np_r) {
          rp[g] = ld_frame8(p, p.row_first + 2 * (b0 + g), lp);
          ri[g] = ld_frame8(p, p.row_first + 2 * (b0 + g) + 1, lp);
        }
#pragma unroll
      for (int g = 0; g < kBatch; ++g)
        if (b0 + g < np_c) {
          if (b0 + g < 8) acc_pair<false>(qc, cp[g], ci[g]);
          else acc_pair<true>(qc, cp[g], ci[g]);
        }
#pragma unroll
      for (int g = 0; g < kBatch; ++g)
        if (b0 + g < np_r) {
          if (b0 + g < 8) acc_pair<false>(qr, rp[g], ri[g]);
          else acc_pair<true>(qr, rp[g], ri[g]);
        }
    }
    }
    uint32_t ac[4], ar[4];
    acc_codes(qc, np_c, p.col_pre, p.col_post, ac);
    acc_codes(qr, np_r, p.row_pre, p.row_post, ar);
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      if constexpr (!MF) {
        const int wv = ((k < 4 ? w.x : w.y) >> (8 * (k & 3))) & 0xff;
        const int bv = ((k < 4 ? bl.x : bl.y) >> (8 * (k & 3))) & 0xff;
        valid |= uint32_t((wv >= smin) & ((wv - bv) >= cmin) & (px0 + k < p.n_px)) << k;
      }
      col[k] = unpack_code(ac, k);
      row[k] = ROW_MODE != 0 ? unpack_code(ar, k) : 0;
    }
  } else {
    if (!tail) {
      const uint2 mv = *reinterpret_cast<const uint2*>(p.in_mask + px0);
      const int4* ic = reinterpret_cast<const int4*>(p.in_col + px0);
      const int4 c0 = ic[0], c1 = ic[1];
      col[0] = c0.x; col[1] = c0.y; col[2] = c0.z; col[3] = c0.w;
      col[4] = c1.x; col[5] = c1.y; col[6] = c1.z; col[7] = c1.w;
      if constexpr (ROW_MODE != 0) {
        const int4* ir = reinterpret_cast<const int4*>(p.in_row + px0);
        const int4 r0 = ir[0], r1 = ir[1];
        row[0] = r0.x; row[1] = r0.y; row[2] = r0.z; row[3] = r0.w;
        row[4] = r1.x; row[5] = r1.y; row[6] = r1.z; row[7] = r1.w;
      } else {
#pragma unroll
        for (int k = 0; k < kPx; ++k) row[k] = 0;
      }
#pragma unroll
      for (int k = 0; k < kPx; ++k) valid |= uint32_t((((k < 4 ? mv.x : mv.y) >> (8 * (k & 3))) & 0xff) != 0) << k;
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const bool in = px0 + k < p.n_px;
        col[k] = in ? p.in_col[px0 + k] : 0;
        row[k] = (in && ROW_MODE != 0) ? p.in_row[px0 + k] : 0;
        valid |= uint32_t(in && p.in_mask[px0 + k] != 0) << k;
      }
    }
  }
}

// clamp like np.clip(idx, 0, n-1) (processing.py:159,189) and pack col | row << 16
template <int ROW_MODE>
__device__ inline uint32_t pack_code(const MainParams& p, int c, int r) {
  c = c < 0 ? 0 : (c > p.n_pcol - 1 ? p.n_pcol - 1 : c);
  r = ROW_MODE == 0 ? 0 : (r < 0 ? 0 : (r > p.n_prow - 1 ? p.n_prow - 1 : r));
  return uint32_t(c) | (uint32_t(r) << 16);
}

struct TriOut {
  double x, y, z;      // column-stream point (row_mode 0/1), or column point (row_mode 2)
  double rx, ry, rz;   // row-stream point (row_mode 2)
  double t, tr;        // their ray parameters: (x, y, z) = Oc + r * t, (rx, ry, rz) = Oc + r * tr
  uint32_t keep;       // bit 0 column stream, bit 1 row stream
};

// Ray-plane intersection of one valid pixel (processing.py:143-234), fp64 in NumPy's order, in
// three parts so phase B can issue an item's plane gathers, compute its ray while they are in
// flight, and only then combine (tri_item chains them for the other callers).
struct TriPlanes {
  double2 pc01, pc23;  // column plane: (n0, n1), (n2, d or numer)
  double2 pr01, pr23;  // row plane (row_mode 1/2)
};

// Plane rows: (n0, n1, n2, d) row-major, or -- with the precomputed-numerator tables -- split
// in pair planes [0][c] = (n0, n1), [1][c] = (n2, numer): a wave's consecutive column codes
// then read consecutive 16-byte pairs (8 per cache line) instead of every other 16 bytes of
// 32-byte rows.
// NP: 0 reads p.num_pre at run time, 1 / 2 take it as set / clear (phase B picks per workgroup).
template <int NP = 0>
__device__ inline void tri_planes_col(const MainParams& p, uint32_t code, double2& pc01, double2& pc23) {
  if (NP == 1 || (NP == 0 && p.num_pre)) {
    const double2* qc = reinterpret_cast<const double2*>(p.pcol);
    const uint32_t cc = code & 0xffffu;
    pc01 = qc[cc];
    pc23 = qc[p.n_pcol + cc];
  } else {
    const double2* qc = reinterpret_cast<const double2*>(p.pcol + 4 * int64_t(code & 0xffffu));
    pc01 = qc[0];
    pc23 = qc[1];
  }
}

template <int ROW_MODE, int NP = 0>
__device__ inline void tri_planes_row(const MainParams& p, uint32_t code, double2& pr01, double2& pr23) {
  pr01 = make_double2(0, 0);
  pr23 = make_double2(0, 0);
  if constexpr (ROW_MODE == 2) {
    if (NP == 1 || (NP == 0 && p.num_pre)) {
      const double2* qr = reinterpret_cast<const double2*>(p.prow);
      pr01 = qr[code >> 16];
      pr23 = qr[p.n_prow + (code >> 16)];
    } else {
      const double2* qr = reinterpret_cast<const double2*>(p.prow + 4 * int64_t(code >> 16));
      pr01 = qr[0];
      pr23 = qr[1];
    }
  } else if constexpr (ROW_MODE != 0) {
    const double2* qr = reinterpret_cast<const double2*>(p.prow + 4 * int64_t(code >> 16));
    pr01 = qr[0];
    pr23 = qr[1];
  }
}

template <int ROW_MODE, int NP = 0>
__device__ inline TriPlanes tri_planes(const MainParams& p, uint32_t code) {
  TriPlanes t;
  tri_planes_col<NP>(p, code, t.pc01, t.pc23);
  tri_planes_row<ROW_MODE, NP>(p, code, t.pr01, t.pr23);
  return t;
}


// sqrt and 1/x of a double in [1, 2^900): the same fma sequences the compiler's IEEE-correct
// expansions run (v_rsq_f64 + two Newton/correction rounds; v_rcp_f64 + two Newton rounds +
// one correction, as v_div_scale/v_div_fmas/v_div_fixup compute them when nothing needs
// scaling), without the range scaling and special-case selects that cannot trigger here: the
// same bits, 11 fewer VALU instructions per pixel.
__device__ inline double sqrt_ge1(double x) {
  const double g = __builtin_amdgcn_rsq(x);
  double s = x * g, h = g * 0.5;
  const double r = __builtin_fma(-h, s, 0.5);
  s = __builtin_fma(s, r, s);
  double d = __builtin_fma(-s, s, x);
  h = __builtin_fma(h, r, h);
  s = __builtin_fma(d, h, s);
  d = __builtin_fma(-s, s, x);
  return __builtin_fma(d, h, s);
}

__device__ inline double rcp_ge1(double n) {
  double y = __builtin_amdgcn_rcp(n);
  y = __builtin_fma(y, __builtin_fma(-n, y, 1.0), y);
  y = __builtin_fma(y, __builtin_fma(-n, y, 1.0), y);
  return __builtin_fma(__builtin_fma(-n, y, 1.0), y, y);
}

// The pixel's unit ray (processing.py:143-156).  FAST (p.rays_fast, checked on the host for
// every column and row of the image): the Markstein conditions hold for every pixel, so the
// code is one straight-line block with no per-lane fallback branches -- the same values.
template <int RAYS, bool FAST = false>
__device__ inline void tri_ray(const MainParams& p, int u, int v, double& r0, double& r1, double& r2) {
  if (RAYS == SLG_RAYS_PINHOLE) {
    // The same IEEE quotients as the reference, with the divisions by fx, fy (per camera)
    // and by the norm (three per pixel) done as Markstein corrections of one reciprocal.
    // (Per-column / per-row tables of x and y measured 8 % slower: two more L2 gathers per
    // point cost more than the fp64 they replace.)
    const double ax = double(u) - p.cx, ay = double(v) - p.cy;
    double x, y;
    if constexpr (FAST) {
      x = div_rn(ax, p.fx, p.rfx);                         // processing.py:150
      y = div_rn(ay, p.fy, p.rfy);                         // processing.py:151
    } else {
      x = p.div_fast && div_rn_ok(ax) ? div_rn(ax, p.fx, p.rfx) : ax / p.fx;
      y = p.div_fast && div_rn_ok(ay) ? div_rn(ay, p.fy, p.rfy) : ay / p.fy;
    }
    // np.linalg.norm(rays, axis=0), then rays /= norms; FAST: n in [1, 2^450) (host check)
    const double s2 = (x * x + y * y) + 1.0;
    const double n = FAST ? sqrt_ge1(s2) : sqrt(s2);
    r2 = FAST ? rcp_ge1(n) : 1.0 / n;
    if (FAST || (n < 0x1p900 && div_rn_ok(x) && div_rn_ok(y))) {   // n >= 1: its reciprocal is normal
      r0 = div_rn(x, n, r2); r1 = div_rn(y, n, r2);
    } else {
      r0 = x / n; r1 = y / n;
    }
  } else {
    const int64_t px = int64_t(v) * p.width + u;
    r0 = p.rays[px]; r1 = p.rays[p.n_px + px]; r2 = p.rays[2 * p.n_px + px];
  }
}

template <int ROW_MODE, bool FAST = false, int NP = 0>
__device__ inline TriOut tri_combine(const MainParams& p, const TriPlanes& pl, double r0, double r1, double r2) {
  const bool num_pre = NP == 1 || (NP == 0 && p.num_pre);
  const double2 pc01 = pl.pc01, pc23 = pl.pc23, pr01 = pl.pr01, pr23 = pl.pr23;
  TriOut o;
  const double den = (pc01.x * r0 + pc01.y * r1) + pc23.x * r2;          // np.sum(N*rays, 0)
  // numer = n.Oc + d (processing.py:163-165): precomputed per plane by the caller (column 3 of
  // the table) or computed here
  const double num = num_pre ? pc23.y : ((pc01.x * p.o0 + pc01.y * p.o1) + pc23.x * p.o2) + pc23.y;
  const bool okc = fabs(den) > 1e-6;
  double t;
  if constexpr (FAST) {
    const double q = (-num) / den;                         // unconditional: a select, not a branch
    t = okc ? q : 0.0;
  } else {
    t = okc ? (-num) / den : 0.0;
  }
  o.x = p.o0 + r0 * t; o.y = p.o1 + r1 * t; o.z = p.o2 + r2 * t;
  o.t = t;
  o.tr = 0.0;
  o.keep = okc;
  o.rx = o.ry = o.rz = 0.0;
  if constexpr (ROW_MODE == 1) {                          // epipolar filter, processing.py:197-201
    const double dist = fabs(((pr01.x * o.x + pr01.y * o.y) + pr23.x * o.z) + pr23.y);
    o.keep = okc && (dist < p.tol);
  }
  if constexpr (ROW_MODE == 2) {                          // independent row cloud, :218-228
    const double dr = (pr01.x * r0 + pr01.y * r1) + pr23.x * r2;
    const double nr = num_pre ? pr23.y : ((pr01.x * p.o0 + pr01.y * p.o1) + pr23.x * p.o2) + pr23.y;
    const bool okr = fabs(dr) > 1e-6;
    double tr;
    if constexpr (FAST) {
      const double q = (-nr) / dr;
      tr = okr ? q : 0.0;
    } else {
      tr = okr ? (-nr) / dr : 0.0;
    }
    o.rx = p.o0 + r0 * tr; o.ry = p.o1 + r1 * tr; o.rz = p.o2 + r2 * tr;
    o.tr = tr;
    o.keep |= uint32_t(okr) << 1;
  }
  return o;
}

template <int ROW_MODE, int RAYS, bool FAST = false>
__device__ inline TriOut tri_item(const MainParams& p, uint32_t code, int u, int v) {
  const TriPlanes pl = tri_planes<ROW_MODE>(p, code);
  double r0, r1, r2;
  tri_ray<RAYS, FAST>(p, u, v, r0, r1, r2);
  return tri_combine<ROW_MODE, FAST>(p, pl, r0, r1, r2);
}

// One pixel decoded exactly as decode_lane decodes it, with byte loads and few registers
// (the look-back helper path only).
template <int ROW_MODE, int SRC_FRAMES>
__device__ inline bool decode_px(const MainParams& p, int64_t px, int& col, int& row) {
  if (SRC_FRAMES) {
    const uint8_t* f = p.frames + px;
    const int wv = f[0], bv = f[p.stride];
    uint32_t c = 0, r = 0;
    for (int b = 0; b < p.col_pairs; ++b)
      c = (c << 1) | uint32_t(f[int64_t(p.col_first + 2 * b) * p.stride] > f[int64_t(p.col_first + 2 * b + 1) * p.stride]);
    col = int(gray2bin_x2(c << p.col_pre) << p.col_post);
    if (ROW_MODE != 0) {
      for (int b = 0; b < p.row_pairs; ++b)
        r = (r << 1) | uint32_t(f[int64_t(p.row_first + 2 * b) * p.stride] > f[int64_t(p.row_first + 2 * b + 1) * p.stride]);
      r = gray2bin_x2(r << p.row_pre) << p.row_post;
    }
    row = int(r);
    return (wv >= p.ws->smin) & ((wv - bv) >= p.ws->cmin);
  }
  col = p.in_col[px];
  row = ROW_MODE != 0 ? p.in_row[px] : 0;
  return p.in_mask[px] != 0;
}

// Keep-count of another tile of the same view, computed by the calling wave alone: the
// aggregate a predecessor that has not published for a long time would publish (it may not
// have been dispatched yet).  Same arithmetic as main3's phases A/B => same value.
template <int ROW_MODE, int SRC_FRAMES, int RAYS>
__device__ int tile_keep_count_wave(const MainParams& p, int tile, int stream) {
  const int lane = threadIdx.x & 63;
  int cnt = 0;
  const int64_t tile_px = int64_t(tile) * kTilePx;
#pragma unroll 1
  for (int i = lane; i < kTilePx; i += 64) {
    const int64_t px = tile_px + i;
    int col, row;
    if (px < p.n_px && decode_px<ROW_MODE, SRC_FRAMES>(p, px, col, row)) {
      const int v = int(px / p.width), u = int(px - int64_t(v) * p.width);
      const TriOut o = tri_item<ROW_MODE, RAYS>(p, pack_code<ROW_MODE>(p, col, row), u, v);
      cnt += (o.keep >> stream) & 1u;
    }
  }
  return wave_sum(cnt);
}

__device__ inline void publish_agg(uint64_t* w, int agg) {   // unless a helper already did
  unsigned long long expect = 0;
  __hip_atomic_compare_exchange_strong(reinterpret_cast<unsigned long long*>(w), &expect,
                                       (unsigned long long)(kFlagAgg | uint64_t(agg)), __ATOMIC_RELAXED,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned kNapCap = 8;         // back-off cap: 8 x s_sleep(2) ~ 1k clocks between re-polls
constexpr unsigned kHelpAfter = 2048;   // s_sleep(2) units (~0.1 ms) before asking for help

// Look-back words st[b .. b+7] read by one scalar load that misses the scalar cache (glc): the
// poll goes to L2 without queueing behind the co-resident workgroup's frame stream in the
// CU's vector-memory pipeline (a vector poll waits behind up to ~180 KB of streaming loads).
__device__ inline void ld_state8_scalar(const uint64_t* p, uint64_t (&v)[8]) {
  typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
  u32x16 r;
  const uint64_t a = reinterpret_cast<uint64_t>(p);   // uniform: pinned to SGPRs for the "s" operand
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));          // (the builtin returns int:
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));    //  widen only as uint32)
  const uint64_t sa = (uint64_t(hi) << 32) | lo;
  asm volatile("s_load_dwordx16 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(sa) : "memory");
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = uint64_t(r[2 * k]) | (uint64_t(r[2 * k + 1]) << 32);
}

// Decoupled look-back over static tile ids (wave 0 calls it, lane 0 publishes).  Returns true
// with the exclusive prefix of `agg` over the view's tiles before `tile`, or false with the
// nearest predecessor that has not published for p.help_after (it may not be dispatched yet:
// dispatch order is not guaranteed): the caller then computes that tile's aggregate itself
// (tile_keep_count_wave) and retries, so waiting always ends.  Polled 8 predecessors at a time
// with wave-uniform scalar loads, newest first: aggregates are summed as they appear and the
// walk stops at the first inclusive prefix; an unpublished entry is re-polled after a capped
// back-off.  Published values never change (0 -> aggregate -> inclusive), so a stale read only
// delays the walk, never changes the sum.
template <bool PROF>
__device__ bool lookback_scalar(const MainParams& p, uint64_t* st, int tile, int agg, bool published,
                                uint64_t& excl_out, int& help_tile, uint32_t& polls, uint32_t& naps) {
  const int lane = threadIdx.x & 63;
  if (PROF && (p.dbg & 1)) { excl_out = uint64_t(tile) * kTilePx; return true; }   // ablation: no wait
  if (tile == 0) {
    if (lane == 0 && !published) st_state(&st[0], kFlagInc | uint64_t(agg));
    excl_out = 0;
    return true;
  }
  if (lane == 0 && !published) st_state(&st[tile], kFlagAgg | uint64_t(agg));
  uint64_t excl = 0;
  int j = tile - 1;                          // newest predecessor not summed yet
  unsigned slept = 0, nap = 1;
  for (;;) {
    ++polls;
    const int b = j >= 7 ? j - 7 : 0;
    uint64_t v[8];
    ld_state8_scalar(st + b, v);
    bool done = false, stall = false;
#pragma unroll
    for (int k = 7; k >= 0; --k) {
      if (done || stall || b + k > j) continue;
      const uint64_t f = v[k] >> 62;
      if (f == 0) { stall = true; continue; }
      excl += v[k] & kValMask;
      j = b + k - 1;
      done = f == 2;
    }
    if (done || j < 0) break;
    if (stall) {
      if (slept >= p.help_after) {
        help_tile = j;
        return false;
      }
      for (unsigned z = 0; z < nap; ++z) __builtin_amdgcn_s_sleep(2);
      slept += nap;
      naps += nap;
      nap = nap < kNapCap ? nap * 2 : kNapCap;
    }
  }
  if (lane == 0) st_state(&st[tile], kFlagInc | (excl + uint64_t(agg)));
  excl_out = excl;
  return true;
}

// Publishes this tile's aggregate (tile 0: its inclusive prefix) and takes a ticket.  The last of
// the view's tiles to do so finds every tile's word published: it scans them all, 8 consecutive
// tiles per lane (a segmented scan: an inclusive word restarts the running sum), publishes every
// tile's inclusive prefix, and returns true with its own exclusive prefix.  The others return
// false and walk back (lookback_scalar) as before; a walk that is still polling when the scan
// lands meets an inclusive prefix at its next poll.  A lone view's launch has every tile in
// flight at once, so without the scan its walks are ~6.7 polls of ~0.8 us each
// (profiles/r7w).  The values written are the ones the walks compute, so a word only ever
// goes 0 -> aggregate -> inclusive prefix, whichever writer gets there first.
constexpr int kScanPer = 8;                // lookback_scan: consecutive tiles per lane
constexpr int kScanTiles = 2 * 64 * kScanPer;   // lone views up to 1024 tiles (4.2 MP) take the scan
template <bool PROF>
__device__ bool lookback_scan(const MainParams& p, uint64_t* st, int tile, int tiles, int agg, uint32_t* ticket,
                              uint64_t& excl_out) {
  const int lane = threadIdx.x & 63;
  if (PROF && (p.dbg & 1)) return false;     // ablation (lookback_scalar): no wait
  // (no release / acquire fences: on gfx950 an agent-scope one writes back or invalidates the
  // L2 -- the bench shape took 716 instead of 313 us per step with them.  The words and the
  // ticket are agent-scope atomics, performed at the L2 that owns the address, and the ticket is
  // taken after vmcnt(0): the hardware assumption of stats_kernel's ticket)
  uint32_t t = 0;
  if (lane == 0) {
    st_state(&st[tile], (tile == 0 ? kFlagInc : kFlagAgg) | uint64_t(agg));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  t = __builtin_amdgcn_readfirstlane(t);
  if (t != uint32_t(tiles - 1)) return false;
  // kScanPer consecutive tiles per lane: their words loaded at once, summed in the lane, then one
  // wave-wide segmented scan of the lane totals; blocks of 64 * kScanPer tiles in order
  uint64_t carry = 0, mine = 0;
  for (int c0 = 0; c0 < tiles; c0 += 64 * kScanPer) {
    const int i0 = c0 + kScanPer * lane;
    uint64_t w[kScanPer];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) w[k] = i0 + k < tiles ? ld_state(&st[i0 + k]) : 0;
    uint64_t x = 0;                          // the lane's running segmented sum
    bool f = false;                          // an inclusive word seen in the lane so far
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      const bool inc = (w[k] >> 62) == 2;
      x = inc ? (w[k] & kValMask) : x + (w[k] & kValMask);
      f = f || inc;
    }
    uint64_t sx = x;                         // inclusive segmented scan of the lane totals
    bool sf = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t xo = __shfl_up(sx, o);
      const bool fo = __shfl_up(int(sf), o) != 0;
      if (lane >= o && !sf) { sx += xo; sf = fo; }
    }
    uint64_t ex = __shfl_up(sx, 1);          // the lanes before this one (+ carry unless they hold
    const bool ef = lane > 0 && __shfl_up(int(sf), 1) != 0;   //  an inclusive word)
    ex = (lane == 0 ? 0 : ex) + (ef ? 0 : carry);
    x = ex;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      const bool inc = (w[k] >> 62) == 2;
      x = inc ? (w[k] & kValMask) : x + (w[k] & kValMask);
      if (i0 + k < tiles && !inc) st_state(&st[i0 + k], kFlagInc | x);
      if (i0 + k == tile) mine = x;
    }
    carry = __shfl(x, 63);
  }
  mine = __builtin_amdgcn_readlane(uint32_t(mine), (tile % (64 * kScanPer)) / kScanPer) |
         (uint64_t(__builtin_amdgcn_readlane(uint32_t(mine >> 32), (tile % (64 * kScanPer)) / kScanPer)) << 32);
  excl_out = mine - uint64_t(agg);
  return true;
}

// Correspondence maps of 2048 pixels per workgroup (slg_decode): col/row int32, mask uint8.
// (Plan-specialised instances as main3's measured the same: 21.3 vs 21.4 us at 1080p, r3an2.)
__global__ __launch_bounds__(kBlock) void decode_maps_kernel(MainParams p) {
  const int64_t px0 = int64_t(blockIdx.x) * kMapsPx + int64_t(threadIdx.x) * kPx;
  const bool tail = px0 + kPx > p.n_px;       // lane-level guard for the ragged end
  uint32_t valid;
  int col[kPx], row[kPx];
  decode_lane<1, 1, 8>(p, px0, tail, valid, col, row);
  if (px0 + kPx <= p.n_px) {
    int4* oc = reinterpret_cast<int4*>(p.out_col + px0);
    int4* orr = reinterpret_cast<int4*>(p.out_row + px0);
    oc[0] = make_int4(col[0], col[1], col[2], col[3]);
    oc[1] = make_int4(col[4], col[5], col[6], col[7]);
    orr[0] = make_int4(row[0], row[1], row[2], row[3]);
    orr[1] = make_int4(row[4], row[5], row[6], row[7]);
    uint32_t m0 = 0, m1 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m0 |= ((valid >> k) & 1u) << (8 * k);
      m1 |= ((valid >> (k + 4)) & 1u) << (8 * k);
    }
    *reinterpret_cast<uint2*>(p.out_mask + px0) = make_uint2(m0, m1);
  } else {
    for (int k = 0; k < kPx; ++k)
      if (px0 + k < p.n_px) {
        p.out_col[px0 + k] = col[k];
        p.out_row[px0 + k] = row[k];
        p.out_mask[px0 + k] = uint8_t((valid >> k) & 1u);
      }
  }
}

// ------------------------------------------------------------------ main3: occupancy-first fused kernel
// One launch covers up to kMaxViews views of one geometry (grid = tiles x views, views
// interleaved).  Per kTileBlock-lane workgroup and kTilePx-pixel tile:
//  A  every lane decodes its 8 pixels (all used frames in flight, 8-byte coalesced loads); a
//     block scan compacts the tile's valid pixels into LDS items (code, BGR, pixel offset);
//  B  the lanes triangulate the items one workgroup-width at a time (fp64, NumPy order) --
//     balanced over the waves whatever the foreground layout; points stay in registers and one ballot
//     per wave and round gives every kept point its rank;
//  C  one barrier shares the per-(round, wave) counts, wave 0 resolves the tile's offset by
//     decoupled look-back (helping a long-silent predecessor, so waiting always ends);
//  D  each lane stores its points at offset + rank: consecutive lanes write consecutive
//     points, so the compacted stores coalesce without an LDS staging copy.
// 49 KB of LDS (24 KB at 256 lanes) and no point staging keep two 512-lane workgroups per CU
// resident, so one tile's decode stream overlaps another's fp64 work and look-back.
constexpr int kMaxViews = 16;
#ifndef SLG_DECODE_BATCH
#define SLG_DECODE_BATCH 11                // pairs per axis in flight per lane (4/6/8/11: 31.7/30.3/28.7/27.5 us/view)
#endif
#ifndef SLG_TRI_GROUP
#define SLG_TRI_GROUP 4                    // phase B: rounds (items per lane) whose gathers are in flight together
#endif
#ifndef SLG_M3_WAVES
#define SLG_M3_WAVES 4                     // waves per SIMD main3 is register-budgeted for
#endif

struct ViewIO {
  const uint8_t* frames;      // SRC_FRAMES: [F][stride]
  const uint8_t* texture;     // [n_px][3] BGR
  const int32_t* in_col;      // !SRC_FRAMES: maps
  const int32_t* in_row;
  const uint8_t* in_mask;
  void* xyz;
  uint8_t* bgr;
  int64_t* count;
  WsHeader* ws;
  uint64_t* states;           // [2][n_tiles]
  void* scratch_xyz;          // row_mode 2 row cloud
  uint8_t* scratch_bgr;
  int64_t stride;             // frame stride of this view
  int32_t col_first, col_pairs, col_pre, col_post;   // decode plan of this view (frames present)
  int32_t row_first, row_pairs, row_pre, row_post;
  const uint8_t* hn_white;    // batch after next: white / black of the view in this slot, whose
  const uint8_t* hn_black;    // Otsu histograms this launch computes per tile (NULL: none)
  uint32_t* hn_part;          // -> [n_tiles][kPartWords] of this view's workspace slice
};

// A view whose Otsu partials (carried by an EARLIER launch on the same stream) this launch
// turns into thresholds, with finishing workgroups placed at the front of its grid: the
// streaming pipeline's stats pass then costs no kernel and no cross-stream wait of its own.
struct FinIO {
  const uint32_t* parts;      // [n_tiles][kPartWords] partials in the view's workspace slice
  WsHeader* ws;               // the slice: thresholds out, look-back words armed
};

struct Main3Params {
  MainParams c;               // geometry, decode plan, calibration (per-view pointers unused)
  int32_t n_views;
  int32_t n_fin;              // views finished by this launch (FinIO), 0: none
  int32_t fin_blocks;         // finishing workgroups per such view (the grid's first n_fin*fin_blocks)
  int32_t pad_m3;
  int64_t n_state_words;      // look-back words per view slice (finishing arms them)
  int64_t pad_zero;           // zero bytes the last tile's partial counted past n_px
  ViewIO v[kMaxViews];
  FinIO fin[kMaxViews];
};

static_assert(sizeof(Main3Params) <= 4096, "kernel arguments");

__device__ inline MainParams view_params(const Main3Params& P, int view) {
  MainParams q = P.c;
  const ViewIO& io = P.v[view];
  q.frames = io.frames; q.texture = io.texture;
  q.in_col = io.in_col; q.in_row = io.in_row; q.in_mask = io.in_mask;
  q.xyz = io.xyz; q.bgr = io.bgr; q.count = io.count;
  q.ws = io.ws; q.states = io.states;
  q.scratch_xyz = io.scratch_xyz; q.scratch_bgr = io.scratch_bgr;
  q.stride = io.stride;
  q.col_first = io.col_first; q.col_pairs = io.col_pairs; q.col_pre = io.col_pre; q.col_post = io.col_post;
  q.row_first = io.row_first; q.row_pairs = io.row_pairs; q.row_pre = io.row_pre; q.row_post = io.row_post;
  return q;
}

// BGR bytes of pixel k (0..7) from the lane's 24 texture bytes t[0..5].
__device__ inline uint32_t bgr_of(const uint32_t (&t)[6], int k) {
  const int b = 3 * k, w = b >> 2, s = 8 * (b & 3);
  const uint64_t pair = uint64_t(t[w]) | (uint64_t(w + 1 < 6 ? t[w + 1] : 0u) << 32);
  return uint32_t(pair >> s) & 0xffffffu;
}

// The Otsu histograms (white, clip(white - black)) of another capture over this tile's pixel
// range, as u16 counts [2][256] packed in pairs (1 KB per tile) -- the stats pass of the batch
// after next, carried by this fused launch (stats_kernel's partials mode sums the tiles).
// Split so it costs neither latency nor chain time: the loads are issued when the workgroup
// starts (hist_next_load), the nibble planes staged once the points are computed
// (hist_next_stage), the matrix-core counting done by waves 1..3 while wave 0 runs the
// look-back (hist_next_count, as mfma_hist_chunk) and the partial written after it
// (hist_next_write).  Bytes past n_px count as 0 (pad_zero).
__device__ inline void hist_next_load(const uint8_t* white, const uint8_t* black, int64_t n_px, int64_t o,
                                      uint2& wq, uint2& bq) {
  wq = make_uint2(0, 0);
  bq = make_uint2(0, 0);
  if (o < n_px) {                            // frames readable to round_up(n, 8)
    wq = ld_once8_buf(white, uint32_t(o));     // o < n_px < 2^31
    bq = ld_once8_buf(black, uint32_t(o));
  }
}

// stage: [wave][hi_w, lo_w, hi_d, lo_d][64 lanes] uint2 (the lane's 8 pixels per plane)
__device__ inline void hist_next_stage(uint2 wq, uint2 bq, int64_t n_px, int64_t o, uint2* stage) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (o + 8 > n_px) {                        // tail: zero the bytes at or past n_px
    const uint64_t mk = o >= n_px ? 0ull : (~0ull >> (64 - 8 * (n_px - o)));
    wq.x &= uint32_t(mk); wq.y &= uint32_t(mk >> 32);
    bq.x &= uint32_t(mk); bq.y &= uint32_t(mk >> 32);
  }
  const uint32_t m4 = 0x0f0f0f0fu;
  const uint32_t d0 = sub_sat_u8x4(wq.x, bq.x), d1 = sub_sat_u8x4(wq.y, bq.y);
  uint2* st = stage + wave * 256;
  st[lane] = make_uint2((wq.x >> 4) & m4, (wq.y >> 4) & m4);
  st[64 + lane] = make_uint2(wq.x & m4, wq.y & m4);
  st[128 + lane] = make_uint2((d0 >> 4) & m4, (d1 >> 4) & m4);
  st[192 + lane] = make_uint2(d0 & m4, d1 & m4);
}

// Steps h, h + n_help, ... of the tile's kTilePx / 64 MFMA steps (64 pixels each), added to
// s_h[512] (zeroed beforehand) with LDS atomics.
__device__ inline void hist_next_count(const uint2* stage, uint32_t* s_h, int h, int n_help) {
  const int lane = threadIdx.x & 63;
  const uint32_t repx = (uint32_t(lane & 15) * 0x01010101u) ^ 0x0f0f0f0fu;
  v4i32 acc_w = {0, 0, 0, 0}, acc_d = {0, 0, 0, 0};
  for (int step = h; step < kTilePx / 64; step += n_help) {
    const uint2* st = stage + (step >> 3) * 256 + 8 * (step & 7) + 2 * (lane >> 4);   // lanes src, src+1
    const uint4 hw = *reinterpret_cast<const uint4*>(st);
    const uint4 lw = *reinterpret_cast<const uint4*>(st + 64);
    const uint4 hd = *reinterpret_cast<const uint4*>(st + 128);
    const uint4 ld = *reinterpret_cast<const uint4*>(st + 192);
    const v4i32 aw = {onehot16(hw.x, repx), onehot16(hw.y, repx), onehot16(hw.z, repx), onehot16(hw.w, repx)};
    const v4i32 bw = {onehot16(lw.x, repx), onehot16(lw.y, repx), onehot16(lw.z, repx), onehot16(lw.w, repx)};
    const v4i32 ad = {onehot16(hd.x, repx), onehot16(hd.y, repx), onehot16(hd.z, repx), onehot16(hd.w, repx)};
    const v4i32 bd = {onehot16(ld.x, repx), onehot16(ld.y, repx), onehot16(ld.z, repx), onehot16(ld.w, repx)};
    acc_w = __builtin_amdgcn_mfma_i32_16x16x64_i8(aw, bw, acc_w, 0, 0, 0);
    acc_d = __builtin_amdgcn_mfma_i32_16x16x64_i8(ad, bd, acc_d, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int bin = 16 * (4 * (lane >> 4) + r) + (lane & 15);
    if (acc_w[r]) atomicAdd(&s_h[bin], uint32_t(acc_w[r]) >> 8);
    if (acc_d[r]) atomicAdd(&s_h[256 + bin], uint32_t(acc_d[r]) >> 8);
  }
}

__device__ inline void hist_next_write(const uint32_t* s_h, uint32_t* part) {
  for (int i = threadIdx.x; i < kPartWords; i += kTileBlock) part[i] = s_h[2 * i] | (s_h[2 * i + 1] << 16);
}

// Block-wide exclusive scan of one int per lane: (exclusive prefix, block total).
__device__ inline int2 block_scan(int x, int* s_wtot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wtot[wave] = incl;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kTileBlock / 64; ++w) {
    off += w < wave ? s_wtot[w] : 0;
    tot += s_wtot[w];
  }
  return make_int2(off + incl - x, tot);
}

// LDS slots of compacted item m: phase A writes lane L's items at m = prefix(L) + j, a stride of
// up to 8 items between neighbouring lanes (16 words for the 8-byte records: 16 lanes per
// bank); one pad slot per 16 records (per 8 BGR words) makes that stride odd in words.
#ifndef SLG_ITEM_PAD
#define SLG_ITEM_PAD 4                     // one pad record per 2^SLG_ITEM_PAD items
#endif
#ifndef SLG_BGR_PAD
#define SLG_BGR_PAD 3                      // one pad word per 2^SLG_BGR_PAD BGR words
#endif
constexpr int kItemSlots = kTilePx + (kTilePx >> SLG_ITEM_PAD), kBgrSlots = kTilePx + (kTilePx >> SLG_BGR_PAD);
__device__ inline int item_slot(int m) { return m + (m >> SLG_ITEM_PAD); }
__device__ inline int bgr_slot(int m) { return m + (m >> SLG_BGR_PAD); }

#ifndef SLG_X64_KEEP_T
#define SLG_X64_KEEP_T 1                   // f64 XYZ, pinhole rays: t in registers, ray recomputed in phase D
#endif
// Phase B of main3 for rounds [i, i + G) (item m = tid + 256 * round), FAST path: the G items'
// loads and fp64 chains are independent, so their plane gathers are in flight together.
// tri_rounds: i is a compile-time multiple of G (the unrolled group loop); tri_rounds_at: any i.
template <int G, int ROW_MODE, int RAYS, typename XT, int NS, int kIt, int NP = 0, int NC = 3>
__device__ inline void tri_rounds_at(const MainParams& p, int i, int n_items, const uint2* s_item,
                                     XT (&pts)[NS][kIt][NC], uint64_t (&km)[NS][kIt]) {
  const int tid = threadIdx.x;
  TriOut o[G];
  TriPlanes pl[G];
  double ra[G][3];
  bool in[G];
  uint32_t uvs[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {                    // the G items' plane gathers, all in flight ...
    const int m = tid + kTileBlock * (i + h);
    in[h] = m < n_items;
    const uint2 it = s_item[item_slot(m)];          // m < kTilePx; garbage past n_items masked
    const uint32_t sc = it.x, suv = it.y;
    const uint32_t code = in[h] ? sc : 0u;
    uvs[h] = in[h] ? suv : 0u;
    pl[h] = tri_planes<ROW_MODE, NP>(p, code);
  }
#pragma unroll
  for (int h = 0; h < G; ++h)                      // ... while the rays are computed
    tri_ray<RAYS, true>(p, int(uvs[h] & 0xffffu), int(uvs[h] >> 16), ra[h][0], ra[h][1], ra[h][2]);
  __builtin_amdgcn_sched_barrier(0);               // keep the combine (first use of the planes) after them
#pragma unroll
  for (int h = 0; h < G; ++h) o[h] = tri_combine<ROW_MODE, true, NP>(p, pl[h], ra[h][0], ra[h][1], ra[h][2]);
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const uint32_t keep = in[h] ? o[h].keep : 0u;
    // runtime round index: select into the register arrays (unrolled compares, no scratch)
#pragma unroll
    for (int r = 0; r < kIt; ++r)
      if (r == i + h) {
        if constexpr (NC == 1) {                   // the ray parameters only (x64_keep_t)
          pts[0][r][0] = o[h].t;
          if constexpr (ROW_MODE == 2) pts[NS - 1][r][0] = o[h].tr;
        } else {
          pts[0][r][0] = XT(o[h].x); pts[0][r][1] = XT(o[h].y); pts[0][r][2] = XT(o[h].z);
          if constexpr (ROW_MODE == 2) {
            pts[NS - 1][r][0] = XT(o[h].rx); pts[NS - 1][r][1] = XT(o[h].ry); pts[NS - 1][r][2] = XT(o[h].rz);
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) km[s][r] = __ballot((keep >> s) & 1u);
      }
  }
}

template <int G, int ROW_MODE, int RAYS, typename XT, int NS, int kIt, int NP = 0, int NC = 3>
__device__ inline void tri_rounds(const MainParams& p, int i, int n_items, const uint2* s_item,
                                  XT (&pts)[NS][kIt][NC], uint64_t (&km)[NS][kIt]) {
  tri_rounds_at<G, ROW_MODE, RAYS, XT, NS, kIt, NP, NC>(p, i, n_items, s_item, pts, km);
}

// PROF: the profiling instance (SLG_DBG set): honours the ablation bits of MainParams::dbg and
// writes per-workgroup phase records; the production instances carry none of that code.
constexpr int kPlanGray = 0x100;           // PLAN bit: every view of the launch is a gray capture

template <int ROW_MODE, int XYZ64, int SRC_FRAMES, int RAYS, bool PROF, int PLAN = 0>
__global__ __launch_bounds__(kTileBlock, ROW_MODE == 2 && XYZ64 ? 2 : SLG_M3_WAVES) void main3_kernel(Main3Params P) {
  using XT = typename std::conditional<XYZ64 != 0, double, float>::type;
  constexpr int NS = ROW_MODE == 2 ? 2 : 1;
  constexpr int kB = kTileBlock;
  constexpr int kIt = kTilePx / kB;        // 8 item rounds of one workgroup at most
  __shared__ __attribute__((aligned(16))) uint2 s_item[kItemSlots];  // valid item: (col | row << 16, u | v << 16)
  __shared__ uint32_t s_bgr[kBgrSlots];    // its BGR (24 bits)
  __shared__ int s_wtot[kB / 64];
  __shared__ int s_cnt[NS][kIt][kB / 64];  // kept points per (round, wave)
  __shared__ int s_loc[NS][kIt][kB / 64];  // their exclusive offsets within the tile (phase C)
  __shared__ uint64_t s_excl[NS];
  // the carried batch's nibble planes and histograms in LDS of their own (68 KB per workgroup,
  // two per CU): each wave stages its lane data as soon as phase A ends, no extra barrier
  // (289.7 vs 291.6 us per launch against aliasing the item arrays after phase B)
  __shared__ __attribute__((aligned(16))) uint2 s_hstage[(kB / 64) * 256];   // [wave][4 planes][64 lanes]
  __shared__ uint32_t s_hn[512];                                      // histograms

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles = int(P.c.n_tiles);
  const int n_fin_wg = P.n_fin * P.fin_blocks;      // finishing workgroups come first
  if (int(blockIdx.x) < n_fin_wg) {
    const int fv = int(blockIdx.x) / P.fin_blocks;
    otsu_from_parts(P.fin[fv].parts, P.fin[fv].ws, tiles, P.c.n_px, P.n_state_words, P.pad_zero,
                    int(blockIdx.x) - fv * P.fin_blocks, P.fin_blocks, reinterpret_cast<uint32_t*>(s_item), s_bgr);
    static_assert(kPartsLdsWords * 4 <= sizeof(s_item), "the finishing workgroups' Otsu LDS");
    return;
  }
  const int bid = int(blockIdx.x) - n_fin_wg;
  // Views interleaved in dispatch order: each view's look-back chain has only ~1/n_views of
  // the resident workgroups in flight, so a tile waits on fewer, similar predecessors.
  const int tile = bid / P.n_views;
  const int view = bid - tile * P.n_views;
  const MainParams p = view_params(P, view);
  // resident-job arena (WsHeader::arena_off, set with the thresholds by an earlier kernel): the
  // view's column cloud starts at aoff in the arena the cloud pointers name; -1: no room, store nothing
  const int64_t aoff = p.ws->arena_cursor ? p.ws->arena_off : 0;
  const int64_t tile_px = int64_t(tile) * kTilePx;
  const int64_t px0 = tile_px + int64_t(tid) * kPx;
  const bool tail = tile == tiles - 1;               // block-uniform: guarded reads only here
  const int tile_v0 = int(tile_px / p.width);
  // PROF, SLG_DBG bit 6: per workgroup one 32-byte record {A decode, B triangulate, C
  // look-back, D stores (100 MHz ticks), look-back polls, sleep units, items, start} written to
  // view 0's partials region (tools/kbench.py "phases"; the host refuses it when a batch is
  // carried, whose partials live there).
  const bool prof = PROF && (p.dbg & 64) != 0;
  uint64_t t_phase = prof ? __builtin_amdgcn_s_memrealtime() : 0;
  // the record lives in LDS (tid 0 writes it): as a register array it pushed the profiling
  // instance into VGPR spills once the production decode reached the register limit
  __shared__ uint32_t s_rec[8];
  if (prof && tid == 0) s_rec[7] = uint32_t(t_phase);                // start time (low 32 bits)
  uint32_t polls = 0, naps = 0;
  auto stamp = [&](int k) {
    if (prof && tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      s_rec[k] = uint32_t(t - t_phase);
      t_phase = t;
    }
  };

  // stats pass of the batch after next (hist_next_*): loads now, counting during phase C
  const bool hn = P.v[view].hn_part != nullptr;     // block-uniform
  uint2 hn_w, hn_b;
  if (hn) {
    hist_next_load(P.v[view].hn_white, P.v[view].hn_black, p.n_px, px0, hn_w, hn_b);
  }
  // ------------------------------------------------------------ A: decode + tile compaction
  int n_items;
  {
    uint32_t tex[6] = {0, 0, 0, 0, 0, 0};
    // texture NULL: a gray capture, whose cv2.imread(files[0]) is frame 0 replicated -- the white
    // bytes decode_lane has already read give the colour, no texture bytes are read at all.
    // Plan instances fix it at compile time (kPlanGray set: gray; clear: colour, the texture code
    // exactly as before -- a run-time test cost colour captures 1.4 %, profiles/r4r); the generic
    // instance tests each view.
    const bool gray = (PLAN & kPlanGray) != 0 || ((PLAN & 0xff) == 0 && p.texture == nullptr);
    auto load_tex = [&](uint2 white) {
      if (gray) {
        tex[0] = white.x;
        tex[1] = white.y;
      } else if (!tail) {
        const uint32_t tq = uint32_t(px0) * 3u;   // n_px * 3 < 2^32 (host: slg_capture checks)
        const uint2 t0 = ld_once8_buf(p.texture, tq), t1 = ld_once8_buf(p.texture, tq + 8u),
                    t2 = ld_once8_buf(p.texture, tq + 16u);
        tex[0] = t0.x; tex[1] = t0.y; tex[2] = t1.x; tex[3] = t1.y; tex[4] = t2.x; tex[5] = t2.y;
      } else {
        for (int k = 0; k < 3 * kPx; ++k)
          if (px0 * 3 + k < p.n_px * 3) tex[k >> 2] |= uint32_t(p.texture[px0 * 3 + k]) << (8 * (k & 3));
      }
    };
    uint32_t valid;
    int col[kPx], row[kPx];
    if constexpr (SRC_FRAMES) {
      // mask first: a lane with a valid pixel issues its texture loads, then its pattern loads
      decode_lane<ROW_MODE, SRC_FRAMES, SLG_DECODE_BATCH, true, PLAN>(p, px0, tail, valid, col, row, load_tex);
    } else {
      // maps source (slg_triangulate): only lanes with a valid pixel read their 24 texture
      // bytes, once the mask is known (the block scan's barrier covers part of the latency)
      decode_lane<ROW_MODE, SRC_FRAMES, SLG_DECODE_BATCH, false, PLAN>(p, px0, tail, valid, col, row);
      if (valid != 0u) load_tex(make_uint2(0u, 0u));
    }
    const int2 sc = block_scan(__popc(valid), s_wtot);
    n_items = sc.y;
    int m = sc.x;
    int u = int(tile_px - int64_t(tile_v0) * p.width) + tid * kPx, v = tile_v0;   // lane's first pixel
    while (u >= p.width) { u -= p.width; ++v; }
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      if (valid & (1u << k)) {
        s_item[item_slot(m)] = make_uint2(pack_code<ROW_MODE>(p, col[k], row[k]), uint32_t(u) | (uint32_t(v) << 16));
        s_bgr[bgr_slot(m)] = gray ? ((tex[k >> 2] >> (8 * (k & 3))) & 0xffu) * 0x010101u : bgr_of(tex, k);
        ++m;
      }
      if (++u == p.width) { u = 0; ++v; }
    }
  }
  __syncthreads();

  stamp(0);
  if (hn) {                                          // block-uniform; counted in phase C
    for (int i = tid; i < 512; i += kB) s_hn[i] = 0;
    hist_next_stage(hn_w, hn_b, p.n_px, px0, s_hstage);
  }
  // ------------------------------------------------------------ B: triangulate, balanced
  // Item m = tid + kB * i: every wave gets an equal share of the tile's valid pixels.
  // Points stay in registers across the look-back (recomputing them after it instead frees
  // ~15 VGPRs for a fifth wave per SIMD but measured 6% slower).
  // f64 XYZ with pinhole rays (x64_keep_t): only t (and tr) stay in registers across the look-back
  // -- 48 VGPRs of points pushed the instance past 128 VGPRs into scratch -- and phase D
  // recomputes the ray from the item's (u, v): the same code on the same inputs, the same bits.
  constexpr bool KT = XYZ64 && RAYS == SLG_RAYS_PINHOLE && SLG_X64_KEEP_T;
  constexpr int NC = KT ? 1 : 3;
  XT pts[NS][kIt][NC];
  uint64_t km[NS][kIt];
  // full groups, then a pair, then a single round: the tail takes at most 3 rounds, so groups
  // of 1, 2 or 4 (8 left rounds 4..7 of a tile uncomputed: wrong counts, caught by bench verify)
  static_assert(kIt % SLG_TRI_GROUP == 0 && (SLG_TRI_GROUP == 1 || SLG_TRI_GROUP == 2 || SLG_TRI_GROUP == 4),
                "grouped rounds");
  const bool trivial = PROF && (p.dbg & 2);          // ablation: no triangulation arithmetic
  if (p.rays_fast && !trivial) {
    // Several rounds per step: independent straight-line fp64 chains per lane whose plane
    // gathers (L2, high latency under the streaming load) are all in flight together.  The
    // tile's round count is block-uniform: full groups of SLG_TRI_GROUP rounds, then a pair,
    // then a single round, so no empty round is computed.
    const int rounds = (n_items + kB - 1) / kB;
    int i = 0;
    auto all_rounds = [&](auto np) {
      constexpr int NP = decltype(np)::value;
#pragma unroll
      for (int g = 0; g + SLG_TRI_GROUP <= kIt; g += SLG_TRI_GROUP)
        if (i + SLG_TRI_GROUP <= rounds) {
          tri_rounds<SLG_TRI_GROUP, ROW_MODE, RAYS, XT, NS, kIt, NP>(p, g, n_items, s_item, pts, km);
          i = g + SLG_TRI_GROUP;
        }
      if (SLG_TRI_GROUP > 2 && i + 2 <= rounds) {
        tri_rounds_at<2, ROW_MODE, RAYS, XT, NS, kIt, NP>(p, i, n_items, s_item, pts, km);
        i += 2;
      }
      if (i < rounds) {
        tri_rounds_at<1, ROW_MODE, RAYS, XT, NS, kIt, NP>(p, i, n_items, s_item, pts, km);
        i += 1;
      }
    };
    // numerator tables or not: a block-uniform choice between two straight-line instances,
    // so neither computes the other's numerator and selects
    if (p.num_pre) all_rounds(std::integral_constant<int, 1>());
    else all_rounds(std::integral_constant<int, 2>());
#pragma unroll
    for (int r = 0; r < kIt; ++r)
      if (r >= i) {
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) km[s2][r] = 0;
      }
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < kIt; ++r) {
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) s_cnt[s2][r][wave] = __popcll(km[s2][r]);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
#pragma unroll
      for (int s = 0; s < NS; ++s) km[s][i] = 0;
      if (i * kB < n_items) {                          // block-uniform
        const int m = tid + kB * i;
        const bool in = m < n_items;
        const uint2 it = s_item[item_slot(m)];          // read unconditionally (m < kTilePx) ...
        const uint32_t sc = it.x, suv = it.y;
        const uint32_t code = in ? sc : 0u, uv = in ? suv : 0u;   // ... garbage past n_items masked
        const int u = int(uv & 0xffffu), v = int(uv >> 16);
        uint32_t keep;
        if (trivial) {
          keep = in ? (ROW_MODE == 2 ? 3u : 1u) : 0u;
          if constexpr (NC == 3) {
            pts[0][i][0] = XT(code & 0xffff); pts[0][i][1] = XT(code >> 16); pts[0][i][2] = XT(u);
            if constexpr (ROW_MODE == 2) { pts[NS - 1][i][0] = XT(v); pts[NS - 1][i][1] = 0; pts[NS - 1][i][2] = 0; }
          }
        } else {
          const TriOut o = tri_item<ROW_MODE, RAYS>(p, code, u, v);
          keep = in ? o.keep : 0u;
          if constexpr (NC == 1) {
            pts[0][i][0] = o.t;
            if constexpr (ROW_MODE == 2) pts[NS - 1][i][0] = o.tr;
          } else {
            pts[0][i][0] = XT(o.x); pts[0][i][1] = XT(o.y); pts[0][i][2] = XT(o.z);
            if constexpr (ROW_MODE == 2) { pts[NS - 1][i][0] = XT(o.rx); pts[NS - 1][i][1] = XT(o.ry); pts[NS - 1][i][2] = XT(o.rz); }
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) km[s][i] = __ballot((keep >> s) & 1u);
      }
      if (lane == 0) {
#pragma unroll
        for (int s = 0; s < NS; ++s) s_cnt[s][i][wave] = __popcll(km[s][i]);
      }
    }
  }
  __syncthreads();

  stamp(1);
  // ------------------------------------------------------------ C: tile offset (look-back)
  if (wave == 0) {
#pragma unroll 1
    for (int s = 0; s < NS; ++s) {
      // one lane per (round, wave) count: the tile aggregate and, for phase D, each (round,
      // wave)'s offset within the tile -- one wave-wide scan instead of per-round sums later
      constexpr int kEnt = kIt * (kB / 64);           // 64 for 512-lane tiles, 32 for 256
      static_assert(kEnt <= 64, "one lane per (round, wave)");
      const int cnt = lane < kEnt ? (&s_cnt[s][0][0])[lane] : 0;
      int incl = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (lane < kEnt) (&s_loc[s][0][0])[lane] = incl - cnt;
      const int agg = __shfl(incl, 63);
      uint64_t* st = p.states + int64_t(s) * tiles;
      uint64_t excl;
      int ht;
      // a lone view's launch: the last tile to publish scans them all (lookback_scan: 1.3 us
      // off a one-view call; in 16-view launches the walks are hidden and the scan cost 1.3 %;
      // views of more than kScanTiles tiles span several waves of workgroups, whose staggered
      // walks end sooner, while the scan of every tile would delay the last one)
      const bool lone = P.n_views == 1 && tiles <= kScanTiles;
      if (!(lone && lookback_scan<PROF>(p, st, tile, tiles, agg, s == 0 ? &p.ws->lb_ticket : &p.ws->lb_ticket_row, excl)))
      while (!lookback_scalar<PROF>(p, st, tile, agg, lone, excl, ht, polls, naps)) {
        // a predecessor has not published for long (it may not be dispatched yet): publish
        // its aggregate for it, computed by this wave, and look back again
        const int hagg = tile_keep_count_wave<ROW_MODE, SRC_FRAMES, RAYS>(p, ht, s);
        if (lane == 0) {
          publish_agg(&st[ht], hagg);
          atomicOr(&p.ws->error, 2u);                // diagnostic: a helper ran (not an error)
        }
      }
      if (lane == 0) {
        s_excl[s] = excl;
        if (tail) {
          p.ws->totals[s] = int64_t(excl) + agg;
          if (ROW_MODE != 2) *p.count = int64_t(excl) + agg;
          if (s == 0 && p.ws->arena_cursor) p.count[1] = aoff;   // arena mode: count[2]
        }
      }
    }
  } else if (hn) {                                   // waves 1..: next-batch histograms meanwhile
    hist_next_count(s_hstage, s_hn, wave - 1, kB / 64 - 1);
  }
  __syncthreads();
  if (hn) hist_next_write(s_hn, P.v[view].hn_part + int64_t(tile) * kPartWords);

  stamp(2);
  // ------------------------------------------------------------ D: ordered stores from registers
  if (PROF && (p.dbg & 4)) return;                   // ablation: no output stores
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // the point of round i, stream s: from registers, or (KT) Oc + r * t with the ray recomputed
  auto point_of = [&](int s, int i, XT& x, XT& y, XT& z) {
    if constexpr (KT) {
      const uint32_t uv = s_item[item_slot(tid + kB * i)].y;
      double r0, r1, r2;
      if (p.rays_fast) tri_ray<RAYS, true>(p, int(uv & 0xffffu), int(uv >> 16), r0, r1, r2);
      else tri_ray<RAYS, false>(p, int(uv & 0xffffu), int(uv >> 16), r0, r1, r2);
      const double t = pts[s][i][0];
      x = p.o0 + r0 * t; y = p.o1 + r1 * t; z = p.o2 + r2 * t;
    } else {
      x = pts[s][i][0]; y = pts[s][i][NC - 1 < 1 ? 0 : 1]; z = pts[s][i][NC - 1];
    }
  };
  // (tried and measured no faster, in git history: BGR staged through LDS as 16-byte stores,
  // phase D's LDS reads hoisted, non-temporal stores, f64 XYZ through a per-wave LDS window or
  // as 16 + 8-byte stores -- DESIGN.md §4)
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int64_t base = int64_t(s_excl[s]) + (s == 0 ? aoff : 0);
    XT* gx = reinterpret_cast<XT*>(s == 0 ? p.xyz : p.scratch_xyz);
    uint8_t* gb = s == 0 ? p.bgr : p.scratch_bgr;
    if (s == 0 && aoff < 0) continue;                // arena without room for the view
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
      if ((km[s][i] >> lane) & 1ull) {
        const int l = s_loc[s][i][wave] + __popcll(km[s][i] & lt);
        const int64_t q = base + l;
        const uint32_t c = s_bgr[bgr_slot(tid + kB * i)];
        if (!(PROF && (p.dbg & 128))) {              // PROF ablation bit 7: no XYZ stores
          XT x, y, z;
          point_of(s, i, x, y, z);
          gx[3 * q] = x; gx[3 * q + 1] = y; gx[3 * q + 2] = z;
        }
        if (!(PROF && (p.dbg & 8))) {                // PROF ablation bit 3: no BGR stores
          gb[3 * q] = uint8_t(c); gb[3 * q + 1] = uint8_t(c >> 8); gb[3 * q + 2] = uint8_t(c >> 16);
        }
      }
    }
  }
  if (prof) {
    __syncthreads();
    stamp(3);
    if (tid == 0) {
      s_rec[4] = polls; s_rec[5] = naps; s_rec[6] = uint32_t(n_items);
      uint4* out = reinterpret_cast<uint4*>(reinterpret_cast<char*>(P.v[0].ws) + parts_off(p.n_px)) + 2 * bid;
      out[0] = make_uint4(s_rec[0], s_rec[1], s_rec[2], s_rec[3]);
      out[1] = make_uint4(s_rec[4], s_rec[5], s_rec[6], s_rec[7]);
    }
  }
}

// row_mode 2: append the row cloud (workspace scratch) behind the column cloud.
template <int XYZ64>
__global__ __launch_bounds__(kBlock) void row_tail_kernel(WsHeader* ws, const void* sx, const uint8_t* sb,
                                                          void* xyz, uint8_t* bgr, int64_t* count) {
  using XT = typename std::conditional<XYZ64 != 0, double, float>::type;
  const int64_t nc = ws->totals[0], nr = ws->totals[1];
  const int64_t aoff = ws->arena_cursor ? ws->arena_off : 0;     // resident-job arena (main3)
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i == 0) *count = nc + nr;
  if (i >= nr || aoff < 0) return;
  const XT* s = reinterpret_cast<const XT*>(sx);
  XT* d = reinterpret_cast<XT*>(xyz);
  const int64_t q = aoff + nc + i;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    d[q * 3 + c] = s[i * 3 + c];
    bgr[q * 3 + c] = sb[i * 3 + c];
  }
}

// Colour captures (the reference's phone path uploads canvas PNGs, frontend/App.tsx:234-247,
// saved as-is by server/server.py:86): cv2.imread(f, 0) turns each frame to gray and
// cv2.imread(files[0]) gives frame 0 as BGR.  One upload of the decoded RGB(A) frames feeds
// both: gray planes into the frame stack and frame 0's BGR texture.  PNG: libpng's
// png_do_rgb_to_gray for an 8-bit file without gamma tables (OpenCV's png_set_rgb_to_gray(png,
// 1, 0.299, 0.587)): (9797 r + 19234 g + 3737 b) >> 15, truncated, r where r == g == b --
// pinned to libpng 1.6.37 (tests/test_png_color.py); gAMA / sRGB / iCCP files never come here
// (slg_png_zstream refuses them; the host decodes them).  BMP: OpenCV's BGR2GRAY 14-bit weights,
// restated (parity unpinned: no OpenCV here).  16 pixels per lane: channel bytes are read as
// 16 x C contiguous bytes.
constexpr int kRgbPx = 16;
__global__ __launch_bounds__(kBlock) void rgb_gray_kernel(const uint8_t* rgb, int32_t channels, int64_t n_px,
                                                          int64_t src_stride, uint8_t* gray, int64_t gray_stride,
                                                          uint8_t* bgr0, int32_t bmp) {
  const int f = blockIdx.y;
  const int64_t px0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) * kRgbPx;
  if (px0 >= n_px) return;
  const uint8_t* src = rgb + int64_t(f) * src_stride + px0 * channels;
  uint8_t* dst = gray + int64_t(f) * gray_stride + px0;
  const int n = n_px - px0 < kRgbPx ? int(n_px - px0) : kRgbPx;
  uint32_t g4[kRgbPx / 4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kRgbPx; ++k) {
    if (k >= n) continue;
    const uint32_t r = src[k * channels], g = src[k * channels + 1], b = src[k * channels + 2];
    const uint32_t y = bmp ? (b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14
                           : (r == g && r == b) ? r : (r * 9797u + g * 19234u + b * 3737u) >> 15;
    g4[k >> 2] |= (y & 0xffu) << (8 * (k & 3));
    if (bgr0 && f == 0) {
      bgr0[(px0 + k) * 3] = uint8_t(b);
      bgr0[(px0 + k) * 3 + 1] = uint8_t(g);
      bgr0[(px0 + k) * 3 + 2] = uint8_t(r);
    }
  }
  if (n == kRgbPx && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    *reinterpret_cast<uint4*>(dst) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
  } else {
    for (int k = 0; k < n; ++k) dst[k] = uint8_t(g4[k >> 2] >> (8 * (k & 3)));
  }
}

// slg_workspace_set_arena: the arena words of n slices' headers.
__global__ __launch_bounds__(64) void set_arena_kernel(char* ws, int64_t stride, int n, unsigned long long* cursor,
                                                       int64_t cap, int mult) {
  const int v = int(blockIdx.x) * 64 + int(threadIdx.x);
  if (v >= n) return;
  WsHeader* h = reinterpret_cast<WsHeader*>(ws + int64_t(v) * stride);
  h->arena_cursor = cursor;
  h->arena_cap = cap;
  h->arena_mult = mult;
  h->arena_off = 0;
}

// Gray frame stack whose texture is frame 0 replicated (cv2.imread(f) of an 8-bit gray PNG):
// bgr[i] = (g, g, g) with g = frame0[i].
__global__ __launch_bounds__(kBlock) void gray_texture_kernel(const uint8_t* frame0, int64_t n_px, uint8_t* bgr) {
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n_px) return;
  const uint8_t g = frame0[i];
  bgr[3 * i] = g; bgr[3 * i + 1] = g; bgr[3 * i + 2] = g;
}

__global__ __launch_bounds__(kBlock) void pinhole_kernel(const double* rays, int64_t n_px, int width, double fx,
                                                         double fy, double cx, double cy,
                                                         unsigned long long* mismatches) {
  const int64_t px = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  unsigned bad = 0;
  if (px < n_px) {
    const int v = int(px / width), u = int(px - int64_t(v) * width);
    const double x = (double(u) - cx) / fx;
    const double y = (double(v) - cy) / fy;
    const double n = sqrt((x * x + y * y) + 1.0);
    const double r[3] = {x / n, y / n, 1.0 / n};
#pragma unroll
    for (int c = 0; c < 3; ++c)
      bad += __double_as_longlong(r[c]) != __double_as_longlong(rays[c * n_px + px]);
  }
  bad = wave_sum(bad);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(mismatches, (unsigned long long)bad);
}

// ------------------------------------------------------------------ host side
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SLG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return SLG_OK;
}

int ceil_log2(int n) {
  int b = 0;
  while ((1ll << b) < (long long)n) ++b;
  return b;
}

struct Plan {
  int col_first, col_pairs, col_pre, col_post;
  int row_first, row_pairs, row_pre, row_post;
};

// Which frames each axis reads and how the code is shifted (processing.py:80-122,
// sl_system.py:546-585).
int make_plan(const slg_capture* cap, const slg_decode_params* dp, Plan* out) {   // out may be NULL
  Plan tmp;
  Plan* pl = out ? out : &tmp;
  if (cap->n_frames < 4)
    return fail(SLG_ERR_NOT_ENOUGH, "Not enough images (got %d, need at least 4).", cap->n_frames);
  if (dp->proj_cols < 1 || dp->proj_rows < 1) return fail(SLG_ERR_INVALID, "projector size must be positive");
  const int Bc = ceil_log2(dp->proj_cols), Br = ceil_log2(dp->proj_rows);
  if (Bc > kMaxBits || Br > kMaxBits)
    return fail(SLG_ERR_UNSUPPORTED, "at most %d code bits per axis (got %d, %d)", kMaxBits, Bc, Br);
  const int n = cap->n_frames;
  if (dp->variant == SLG_VARIANT_PROCESSING) {
    const int nc = dp->n_sets_col < 1 ? 1 : (dp->n_sets_col > Bc ? Bc : dp->n_sets_col);
    const int nr = dp->n_sets_row < 1 ? 1 : (dp->n_sets_row > Br ? Br : dp->n_sets_row);
    int kc = 0, kr = 0;
    for (int b = 0; b < nc; ++b) kc += (2 + 2 * b + 1 < n);          // processing.py:94
    for (int b = 0; b < nr; ++b) kr += (2 + 2 * Bc + 2 * b + 1 < n);
    *pl = {2, kc, nc - kc, Bc - nc, 2 + 2 * Bc, kr, nr - kr, Br - nr};
  } else if (dp->variant == SLG_VARIANT_SLSYSTEM) {
    int idx = 2, kc = 0, kr = 0;
    for (int b = 0; b < Bc; ++b) {                                  // sl_system.py:557-562
      if (idx >= n) break;
      if (idx + 1 >= n) return fail(SLG_ERR_INDEX, "list index out of range");
      idx += 2; ++kc;
    }
    const int row_first = idx;
    for (int b = 0; b < Br; ++b) {
      if (idx >= n) break;
      if (idx + 1 >= n) return fail(SLG_ERR_INDEX, "list index out of range");
      idx += 2; ++kr;
    }
    *pl = {2, kc, Bc - kc, 0, row_first, kr, Br - kr, 0};
  } else {
    return fail(SLG_ERR_INVALID, "unknown variant %d", dp->variant);
  }
  return SLG_OK;
}

int check_capture(const slg_capture* cap) {
  if (!cap || !cap->frames) return fail(SLG_ERR_INVALID, "capture frames is NULL");
  if (cap->height < 1 || cap->width < 1) return fail(SLG_ERR_INVALID, "bad image size %dx%d", cap->width, cap->height);
  const int64_t n_px = int64_t(cap->height) * cap->width;
  if (n_px >= (int64_t(1) << 31)) return fail(SLG_ERR_UNSUPPORTED, "image larger than 2^31 pixels");
  if (n_px * 3 + 64 >= (int64_t(1) << 32))        // texture reads take 32-bit byte offsets
    return fail(SLG_ERR_UNSUPPORTED, "image larger than 1.43e9 pixels");
  if (cap->height > 65535 || cap->width > 65535) return fail(SLG_ERR_UNSUPPORTED, "image side above 65535 pixels");
  if (cap->frame_stride < ((n_px + 7) & ~int64_t(7)) || (cap->frame_stride & 7))
    return fail(SLG_ERR_INVALID, "frame_stride must be >= round_up(H*W, 8) and a multiple of 8");
  if (reinterpret_cast<uintptr_t>(cap->frames) & 7) return fail(SLG_ERR_INVALID, "frames must be 8-byte aligned");
  if (int64_t(cap->n_frames > 0 ? cap->n_frames : 0) * cap->frame_stride >= (int64_t(1) << 32))
    return fail(SLG_ERR_UNSUPPORTED, "frame stack larger than 4 GiB");   // 32-bit buffer offsets
  return SLG_OK;
}

int debug_flags();

// One stats launch for n_views views (<= kMaxBatch) of one geometry; view v reads white/black
// from whites[v] / blacks[v] and owns the workspace slice at workspace + v * ws_stride.
// from_parts: Otsu from the per-tile partial histograms in each slice (written by a fused
// launch's next-batch pass) instead of from white/black frames.
int stats_launch_batch(const uint8_t* const* whites, const uint8_t* const* blacks, int n_views, int64_t n_px,
                       const slg_decode_params* dp, char* workspace, int64_t ws_stride, hipStream_t s,
                       bool from_parts = false, uint32_t* hist_out = nullptr) {
  StatsParams sp{};
  sp.hist_out = hist_out;
  for (int v = 0; v < n_views; ++v) {
    sp.white[v] = whites ? whites[v] : nullptr;
    sp.black[v] = blacks ? blacks[v] : nullptr;
    sp.wsv[v] = reinterpret_cast<WsHeader*>(workspace + int64_t(v) * ws_stride);
    if (from_parts) sp.parts[v] = reinterpret_cast<const uint32_t*>(workspace + int64_t(v) * ws_stride + parts_off(n_px));
  }
  sp.n_parts = n_tiles_of(n_px);
  sp.pad_zero = from_parts ? sp.n_parts * kTilePx - n_px : align_up(n_px, kHistChunk) - n_px;
  sp.n_px = n_px;
  sp.n_state_words = n_state_words(n_px);
  sp.thresh_mode = dp ? dp->thresh_mode : SLG_THRESH_MANUAL;
  sp.shadow_val = dp ? dp->shadow_val : 0.0;
  sp.contrast_val = dp ? dp->contrast_val : 0.0;
  // Few fat workgroups per view: each merges its sub-histograms into the view's histogram with
  // <= 512 global atomics, and a batch's stats pass takes few CU slots next to a fused launch.
  // One-view Otsu launches: kOtsuOneChunks MFMA chunks per wave.
  const bool otsu_one = n_views == 1 && sp.thresh_mode == SLG_THRESH_OTSU;
  const int64_t px_per_block = otsu_one ? int64_t(kBlock / 64) * kHistChunk * kOtsuOneChunks : int64_t(kBlock) * kStatsPx;
  int64_t grid = (n_px + px_per_block - 1) / px_per_block;
  const int64_t cap = otsu_one ? 4 * kStatsBlocksOne : n_views == 1 ? kStatsBlocksOne
                    : sp.thresh_mode == SLG_THRESH_OTSU ? kStatsBlocksOtsu : kStatsBlocks;
  if (grid > cap) grid = cap;
  if (sp.thresh_mode == SLG_THRESH_OTSU) {   // bound chunks per wave (i32 MFMA accumulators)
    const int64_t per_block = int64_t(kBlock / 64) * kHistChunk * kHistMaxChunks;
    const int64_t need = (n_px + per_block - 1) / per_block;
    if (grid < need) grid = need;
  }
  if (from_parts) {   // ~2 x kPartsInFlight tiles per workgroup: one or two rounds of loads
    grid = (sp.n_parts + 2 * kPartsInFlight - 1) / (2 * kPartsInFlight);
    grid = grid < 1 ? 1 : (grid > kPartsBlocksMax ? kPartsBlocksMax : grid);
    hipLaunchKernelGGL(parts_kernel, dim3(unsigned(grid), unsigned(n_views)), dim3(kBlock), 0, s, sp);
    return check_launch("parts_kernel");
  }
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(stats_kernel, dim3(unsigned(grid), unsigned(n_views)), dim3(kBlock), 0, s, sp);
  return check_launch("stats_kernel");
}

int stats_launch(const uint8_t* white, const uint8_t* black, int64_t n_px, const slg_decode_params* dp,
                 void* workspace, hipStream_t s) {
  return stats_launch_batch(&white, &black, 1, n_px, dp, static_cast<char*>(workspace), 0, s);
}

int fill_calib(MainParams& mp, const slg_calib* c, const slg_tri_params* tp, int64_t n_px, int width) {
  if (!c || !tp) return fail(SLG_ERR_INVALID, "calib/tri params NULL");
  if (tp->row_mode < 0 || tp->row_mode > 2) return fail(SLG_ERR_INVALID, "row_mode must be 0, 1 or 2");
  if (c->ray_mode == SLG_RAYS_TABLE && !c->rays) return fail(SLG_ERR_INVALID, "ray table is NULL");
  if (c->ray_mode != SLG_RAYS_TABLE && c->ray_mode != SLG_RAYS_PINHOLE) return fail(SLG_ERR_INVALID, "bad ray_mode");
  if (!c->col_planes || c->n_col_planes < 1) return fail(SLG_ERR_INVALID, "column planes missing");
  if (tp->row_mode != 0 && (!c->row_planes || c->n_row_planes < 1)) return fail(SLG_ERR_INVALID, "row planes missing");
  if ((reinterpret_cast<uintptr_t>(c->col_planes) | reinterpret_cast<uintptr_t>(c->row_planes)) & 15)
    return fail(SLG_ERR_INVALID, "plane tables must be 16-byte aligned");
  mp.rays = c->rays;
  mp.fx = c->fx; mp.fy = c->fy; mp.cx = c->cx; mp.cy = c->cy;
  auto vetted = [](double b) {                     // b and RN(1/b) normal, far from over/underflow
    const double m = fabs(b);
    return std::isfinite(b) && m > 0x1p-900 && m < 0x1p900;
  };
  mp.rfx = 1.0 / c->fx;
  mp.rfy = 1.0 / c->fy;
  mp.div_fast = vetted(c->fx) && vetted(c->fy) ? 1 : 0;
  // rays_fast: tri_item's Markstein conditions hold for every column and row of the image
  // (x = (u-cx)/fx and y = (v-cy)/fy in range, so n = |(x, y, 1)| < 2^450 as well).
  auto ok_num = [](double a) { const double m = fabs(a); return m == 0.0 || (m > 0x1p-900 && m < 0x1p900); };
  bool fast = c->ray_mode == SLG_RAYS_TABLE || mp.div_fast;
  const int64_t height = width > 0 ? n_px / width : 0;
  for (int64_t u = 0; fast && c->ray_mode == SLG_RAYS_PINHOLE && u < width; ++u) {
    const double ax = double(u) - c->cx, x = ax / c->fx;
    fast = ok_num(ax) && ok_num(x) && fabs(x) < 0x1p449;
  }
  for (int64_t v = 0; fast && c->ray_mode == SLG_RAYS_PINHOLE && v < height; ++v) {
    const double ay = double(v) - c->cy, y = ay / c->fy;
    fast = ok_num(ay) && ok_num(y) && fabs(y) < 0x1p449;
  }
  mp.rays_fast = fast ? 1 : 0;
  mp.o0 = c->oc[0]; mp.o1 = c->oc[1]; mp.o2 = c->oc[2];
  mp.pcol = c->col_planes; mp.n_pcol = c->n_col_planes;
  mp.prow = c->row_planes; mp.n_prow = c->n_row_planes;
  // optional per-plane numerators (slg_calib, ABI 2)
  mp.num_pre = c->col_planes_num && (tp->row_mode != 2 || c->row_planes_num) ? 1 : 0;
  if (mp.num_pre) {
    mp.pcol = c->col_planes_num;
    if (tp->row_mode == 2) mp.prow = c->row_planes_num;
  }
  if ((reinterpret_cast<uintptr_t>(c->col_planes_num) | reinterpret_cast<uintptr_t>(c->row_planes_num)) & 15)
    return fail(SLG_ERR_INVALID, "numerator plane tables must be 16-byte aligned");
  mp.tol = tp->epipolar_tol;
  mp.n_px = n_px;
  mp.width = width;
  return SLG_OK;
}

int fill_out(MainParams& mp, const slg_cloud* out, const slg_tri_params* tp, int64_t n_px, void* ws) {
  if (!out || !out->xyz || !out->bgr || !out->count) return fail(SLG_ERR_INVALID, "output cloud buffers NULL");
  const int64_t need = tp->row_mode == 2 ? 2 * n_px : n_px;
  if (out->capacity < need) return fail(SLG_ERR_INVALID, "cloud capacity %lld < %lld", (long long)out->capacity, (long long)need);
  mp.xyz = out->xyz;
  mp.bgr = out->bgr;
  mp.count = out->count;
  mp.ws = reinterpret_cast<WsHeader*>(ws);
  mp.states = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + states_off(n_px));
  mp.n_tiles = n_tiles_of(n_px);
  mp.scratch_xyz = static_cast<char*>(ws) + scratch_xyz_off(n_px);
  mp.scratch_bgr = reinterpret_cast<uint8_t*>(static_cast<char*>(ws) + scratch_bgr_off(n_px));
  return SLG_OK;
}

int debug_flags() {   // profiling ablations only; unset in production
  const char* e = getenv("SLG_DBG");
  return e ? atoi(e) : 0;
}

constexpr int kMainDbgBits = 1 | 2 | 4 | 8 | 64 | 128 | 512;   // 512: the instance alone   // bits main3's profiling instance reads

uint32_t help_after() {   // look-back helper delay; SLG_HELP_AFTER=0 forces the helper (tests)
  const char* e = getenv("SLG_HELP_AFTER");
  return e ? uint32_t(atoi(e)) : kHelpAfter;
}

using Main3Fn = void (*)(Main3Params);

// Production instances for every (source, row_mode, xyz, ray) case; the profiling instance
// (SLG_DBG with any main3 bit) exists for the benchmark shape only: row_mode 1, f32 XYZ, frames,
// pinhole rays (tools/kbench.py).
// Decode plans main3 has specialised instances for (PLAN = (col_pairs << 4) | row_pairs), with
// row_mode 1 and pinhole rays: C2's 11 + 10 bits (1920x1080 projector, row_scale 2), the
// reference's default 11 + 11 (processing.py:29-30; C3, C5) and C4's 12 + 12; row_mode 0: C1's
// 10 column bits.
#define SLG_PLAN_C2 0xBA
#define SLG_PLAN_1080P 0xBB
#define SLG_PLAN_C4 0xCC
#define SLG_PLAN_C1 0xA0           // row_mode 0, 10 column bits (1024-wide projector), no row pairs

// Every main3 instance the library can launch, one table: pick_main only returns pointers from
// it, and only those whose device code is in the library's gfx950 code object
// (device_symbols): the HIP runtime aborts the process on a launch -- or any query -- of a kernel
// whose code object lacks it (a round-5 run ended that way: DESIGN.md §4), so a missing
// instance must be caught before the runtime sees it.
struct Main3Inst {
  int src, row_mode, x64, rays, plan;
  bool prof;
  Main3Fn fn;
};
#define SLG_M3(S, RM, X, R, P, PL) {S, RM, X, R, PL, P, main3_kernel<RM, X, S, R, P, PL>},
#define SLG_M3_GENERIC(S)                                                                          \
  SLG_M3(S, 0, 0, 0, false, 0) SLG_M3(S, 0, 0, 1, false, 0) SLG_M3(S, 0, 1, 0, false, 0)          \
  SLG_M3(S, 0, 1, 1, false, 0) SLG_M3(S, 1, 0, 0, false, 0) SLG_M3(S, 1, 0, 1, false, 0)          \
  SLG_M3(S, 1, 1, 0, false, 0) SLG_M3(S, 1, 1, 1, false, 0) SLG_M3(S, 2, 0, 0, false, 0)          \
  SLG_M3(S, 2, 0, 1, false, 0) SLG_M3(S, 2, 1, 0, false, 0) SLG_M3(S, 2, 1, 1, false, 0)
#define SLG_M3_PLAN(RM, PL) SLG_M3(1, RM, 0, 1, false, PL) SLG_M3(1, RM, 1, 1, false, PL)         \
  SLG_M3(1, RM, 0, 1, false, (PL) | kPlanGray) SLG_M3(1, RM, 1, 1, false, (PL) | kPlanGray)
const Main3Inst kMain3Table[] = {
#ifdef SLG_FAST_BUILD   // register/spill inspection builds only: the benchmark's instances alone
    SLG_M3(1, 1, 0, 1, false, SLG_PLAN_C2) SLG_M3(1, 1, 0, 1, false, 0)
#else
    SLG_M3_GENERIC(0) SLG_M3_GENERIC(1)
    SLG_M3_PLAN(1, SLG_PLAN_C2) SLG_M3_PLAN(1, SLG_PLAN_1080P) SLG_M3_PLAN(1, SLG_PLAN_C4)
    SLG_M3_PLAN(0, SLG_PLAN_C1)
    SLG_M3(1, 1, 0, 1, true, SLG_PLAN_C2) SLG_M3(1, 1, 0, 1, true, 0)
#endif
};
#undef SLG_M3_PLAN
#undef SLG_M3_GENERIC
#undef SLG_M3

// Itanium name of main3_kernel<RM, X, S, R, P, PL> (anonymous namespace), as the code object and
// the runtime's registration spell it.
std::string main3_symbol(const Main3Inst& k) {
  auto li = [](int v) { return "Li" + (v < 0 ? "n" + std::to_string(-v) : std::to_string(v)) + "E"; };
  return "_ZN12_GLOBAL__N_112main3_kernelI" + li(k.row_mode) + li(k.x64) + li(k.src) + li(k.rays) +
         std::string(k.prof ? "Lb1E" : "Lb0E") + li(k.plan) + "EEvNS_11Main3ParamsE";
}

// Symbol names of this library's gfx950 code objects: the clang offload bundles in its own file
// (found by dladdr), each gfx950 entry an ELF whose symbol tables are read.  File reads only --
// no HIP call, so nothing here can trip the runtime's abort.  Empty when the file cannot be read.
const std::vector<std::string>& device_symbols() {
  static std::vector<std::string> names;
  static std::once_flag once;
  std::call_once(once, [] {
    Dl_info info{};
    if (!dladdr(reinterpret_cast<void*>(&slg_version), &info) || !info.dli_fname) return;
    FILE* f = fopen(info.dli_fname, "rb");
    if (!f) return;
    std::vector<uint8_t> b;
    if (fseek(f, 0, SEEK_END) == 0) {
      const long n = ftell(f);
      if (n > 0 && fseek(f, 0, SEEK_SET) == 0) {
        b.resize(size_t(n));
        if (fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
      }
    }
    fclose(f);
    auto u16 = [&](size_t o) { uint16_t v; memcpy(&v, &b[o], 2); return v; };
    auto u32 = [&](size_t o) { uint32_t v; memcpy(&v, &b[o], 4); return v; };
    auto u64 = [&](size_t o) { uint64_t v; memcpy(&v, &b[o], 8); return v; };
    static const char kMagic[] = "__CLANG_OFFLOAD_BUNDLE__";
    const size_t ml = sizeof(kMagic) - 1;
    for (size_t at = 0; at + ml + 8 <= b.size(); ++at) {
      if (b[at] != '_' || memcmp(&b[at], kMagic, ml) != 0) continue;
      size_t e = at + ml;
      const uint64_t n_ent = u64(e);
      e += 8;
      for (uint64_t k = 0; k < n_ent && e + 24 <= b.size(); ++k) {
        const uint64_t off = u64(e), size = u64(e + 8), tl = u64(e + 16);
        e += 24;
        if (e + tl > b.size()) break;
        const std::string triple(reinterpret_cast<const char*>(&b[e]), size_t(tl));
        e += tl;
        const size_t o = at + off;                 // the entry: an ELF64 code object
        if (triple.find("gfx950") == std::string::npos || o + 64 > b.size() || off + size > b.size() - at ||
            memcmp(&b[o], "\x7f" "ELF", 4) != 0)
          continue;
        const uint64_t shoff = u64(o + 0x28);
        const uint16_t shentsize = u16(o + 0x3a), shnum = u16(o + 0x3c);
        if (shentsize < 64 || o + shoff + uint64_t(shnum) * shentsize > b.size()) continue;
        for (uint16_t si = 0; si < shnum; ++si) {
          const size_t sh = o + shoff + size_t(si) * shentsize;
          const uint32_t type = u32(sh + 4);
          if (type != 2 && type != 11) continue;   // SHT_SYMTAB, SHT_DYNSYM
          const uint64_t sym_off = u64(sh + 24), sym_size = u64(sh + 32), ent = u64(sh + 56);
          const uint32_t link = u32(sh + 40);
          if (ent < 24 || link >= shnum) continue;
          const size_t strh = o + shoff + size_t(link) * shentsize;
          const uint64_t str_off = u64(strh + 24), str_size = u64(strh + 32);
          if (o + sym_off + sym_size > b.size() || o + str_off + str_size > b.size()) continue;
          for (uint64_t q = 0; q + ent <= sym_size; q += ent) {
            const uint32_t nm = u32(o + sym_off + q);
            if (nm == 0 || nm >= str_size) continue;
            const char* c = reinterpret_cast<const char*>(&b[o + str_off + nm]);
            names.emplace_back(c, strnlen(c, size_t(str_size - nm)));
          }
        }
      }
    }
    std::sort(names.begin(), names.end());
  });
  return names;
}

bool device_has(const std::string& name) {
  const auto& v = device_symbols();
  return std::binary_search(v.begin(), v.end(), name);
}

// The instance the calling thread's last pick_main returned (slg_last_kernel; NULL: none).
thread_local const Main3Inst* g_last_main = nullptr;

// The kernel of a (source, row_mode, xyz, rays, plan) launch: the plan's specialised instance
// if the table has one, else the generic one; the profiling instance when SLG_DBG asks for it.
// NULL (and *why set) when the table has none or its device code is missing.
Main3Fn pick_main(int src, int row_mode, int x64, int rays, int plan, const char** why) {
  g_last_main = nullptr;
  const bool prof = (debug_flags() & kMainDbgBits) != 0;
  const Main3Inst* hit = nullptr;
  for (int pass = 0; pass < 2 && !hit; ++pass) {
    const int want = pass == 0 ? plan : 0;
    if (pass == 1 && plan == 0) break;
    for (const Main3Inst& k : kMain3Table)
      if (k.src == src && k.row_mode == row_mode && k.x64 == x64 && k.rays == rays && k.plan == want && k.prof == prof) {
        hit = &k;
        break;
      }
  }
  if (!hit) {
    *why = prof ? "no kernel for this configuration (SLG_DBG profiling: row_mode 1, f32, frames, pinhole only)"
                : "no kernel for this configuration";
    return nullptr;
  }
  if (!device_has(main3_symbol(*hit))) {
    *why = "the library's code object lacks this kernel instance (rebuild libslgpu.so)";
    return nullptr;
  }
  g_last_main = hit;
  return hit->fn;
}

// Output + workspace pointers of one view (the per-view half of fill_out).
int fill_view(ViewIO& io, const slg_cloud* out, const slg_tri_params* tp, int64_t n_px, void* ws) {
  MainParams mp{};
  const int rc = fill_out(mp, out, tp, n_px, ws);
  if (rc) return rc;
  io.xyz = mp.xyz; io.bgr = mp.bgr; io.count = mp.count; io.ws = mp.ws; io.states = mp.states;
  io.scratch_xyz = mp.scratch_xyz; io.scratch_bgr = mp.scratch_bgr;
  return SLG_OK;
}

// One main3 launch over mp.n_views views (<= kMaxViews), then the row_mode-2 tails.
int launch_main3(Main3Fn fn, const char* why, Main3Params& mp, const slg_tri_params* tp, const slg_cloud* outs,
                 hipStream_t s) {
  if (!fn) return fail(SLG_ERR_UNSUPPORTED, "%s", why ? why : "no kernel for this configuration");
  mp.c.dbg = debug_flags();
  mp.c.help_after = help_after();
  const int64_t grid = int64_t(mp.n_fin) * mp.fin_blocks + mp.c.n_tiles * mp.n_views;
  if (grid > INT_MAX) return fail(SLG_ERR_UNSUPPORTED, "batch too large for one launch");
  hipLaunchKernelGGL(fn, dim3(unsigned(grid)), dim3(kTileBlock), 0, s, mp);
  int rc = check_launch("main kernel");
  if (rc || !tp || tp->row_mode != 2) return rc;
  const unsigned tg = unsigned((mp.c.n_px + kBlock - 1) / kBlock);
  for (int v = 0; v < mp.n_views; ++v) {
    const ViewIO& io = mp.v[v];
    if (tp->xyz_f64)
      hipLaunchKernelGGL(row_tail_kernel<1>, dim3(tg), dim3(kBlock), 0, s, io.ws, io.scratch_xyz, io.scratch_bgr, outs[v].xyz, outs[v].bgr, outs[v].count);
    else
      hipLaunchKernelGGL(row_tail_kernel<0>, dim3(tg), dim3(kBlock), 0, s, io.ws, io.scratch_xyz, io.scratch_bgr, outs[v].xyz, outs[v].bgr, outs[v].count);
    rc = check_launch("row_tail_kernel");
    if (rc) return rc;
  }
  return SLG_OK;
}

// Views of one batch must share the launch-wide parameters.
int check_batch(const slg_capture* caps, int n_views) {
  for (int v = 0; v < n_views; ++v) {
    const int rc = check_capture(&caps[v]);
    if (rc) return rc;
    if (reinterpret_cast<uintptr_t>(caps[v].texture) & 7) return fail(SLG_ERR_INVALID, "texture must be 8-byte aligned");
    if (caps[v].height != caps[0].height || caps[v].width != caps[0].width)
      return fail(SLG_ERR_INVALID, "all views of a batch must share one geometry");
  }
  return SLG_OK;
}

// Fused decode + triangulate of n_views views (thresholds already in each view's workspace
// slice): one main3 launch per kMaxViews views.  timing_events: 2 per launch, or NULL.
int fused_batch(const slg_capture* caps, int n_views, const slg_decode_params* dp, const slg_calib* calib,
                const slg_tri_params* tp, char* ws, int64_t ws_stride, const slg_cloud* outs,
                void* const* timing_events, hipStream_t s, const slg_capture* next = nullptr, int n_next = 0,
                char* fin_ws = nullptr, int n_fin = 0) {
  if (!caps || n_views < 1 || !dp || !ws || !outs) return fail(SLG_ERR_INVALID, "NULL argument");
  int rc = check_batch(caps, n_views);
  if (rc) return rc;
  if (n_fin) {                                      // finish thresholds carried by an earlier launch
    if (!fin_ws || n_fin < 0 || n_fin > kMaxViews) return fail(SLG_ERR_INVALID, "finish: NULL or more than 16 views");
    if (dp->thresh_mode != SLG_THRESH_OTSU) return fail(SLG_ERR_UNSUPPORTED, "carried histograms need thresh_mode OTSU");
  }
  if (n_next) {                                     // the batch after next rides along (Otsu only)
    if (!next || n_next < 0 || n_next > n_views) return fail(SLG_ERR_INVALID, "next batch: NULL or more views than this batch");
    if (dp->thresh_mode != SLG_THRESH_OTSU) return fail(SLG_ERR_UNSUPPORTED, "next-batch histograms need thresh_mode OTSU");
    if (debug_flags() & 64)   // the phase records would land on the carried partials
      return fail(SLG_ERR_UNSUPPORTED, "SLG_DBG phase records cannot run with a carried batch");
    for (int v = 0; v < n_next; ++v) {
      rc = check_capture(&next[v]);
      if (rc) return rc;
      if (next[v].n_frames < 4)
        return fail(SLG_ERR_NOT_ENOUGH, "Not enough images (got %d, need at least 4).", next[v].n_frames);
      if (next[v].height != caps[0].height || next[v].width != caps[0].width)
        return fail(SLG_ERR_INVALID, "next batch must share this batch's geometry");
    }
  }
  for (int v = 0; v < n_views; ++v) {
    rc = make_plan(&caps[v], dp, nullptr);
    if (rc) return rc;
  }
  const int64_t n_px = int64_t(caps[0].height) * caps[0].width;
  // every slice of this launch (its views, the carried next batch, the finished batch) is
  // ws_stride apart; the finished batch's slices are read with THIS batch's geometry and
  // decode parameters (include/slgpu.h, slg_decode_triangulate_batch_carry)
  if ((n_views > 1 || n_next > 1 || n_fin > 1) && (ws_stride < ws_total(n_px) || (ws_stride & 255)))
    return fail(SLG_ERR_INVALID, "ws_stride too small or not 256-aligned");
  Main3Params mp{};
  rc = fill_calib(mp.c, calib, tp, n_px, caps[0].width);
  if (rc) return rc;
  mp.c.n_tiles = n_tiles_of(n_px);
  for (int v0 = 0, launch = 0; v0 < n_views; v0 += kMaxViews, ++launch) {
    mp.n_views = n_views - v0 < kMaxViews ? n_views - v0 : kMaxViews;
    int plan = -1;                                  // the views' common pair counts, else 0
    bool all_gray = true, any_gray = false;         // gray captures (texture NULL)
    for (int k = 0; k < mp.n_views; ++k) {
      Plan pl;
      make_plan(&caps[v0 + k], dp, &pl);
      const int rp = tp->row_mode == 0 ? 0 : pl.row_pairs;     // row_mode 0 reads no row frame
      const int key = pl.col_pairs <= 15 && rp <= 15 ? (pl.col_pairs << 4) | rp : 0;
      plan = plan < 0 || plan == key ? key : 0;
      all_gray = all_gray && !caps[v0 + k].texture;
      any_gray = any_gray || !caps[v0 + k].texture;
    }
    // a mixed launch runs the generic instance (per-view test); a plan instance is all one kind
    if (plan > 0 && any_gray) plan = all_gray ? (plan | kPlanGray) : 0;
    const char* why = nullptr;
    const Main3Fn fn = pick_main(1, tp->row_mode, tp->xyz_f64 ? 1 : 0, calib->ray_mode, plan < 0 ? 0 : plan, &why);
    for (int k = 0; k < mp.n_views; ++k) {
      const int v = v0 + k;
      ViewIO& io = mp.v[k];
      io = ViewIO{};
      rc = fill_view(io, &outs[v], tp, n_px, ws + int64_t(v) * ws_stride);
      if (rc) return rc;
      io.frames = caps[v].frames;
      io.texture = caps[v].texture;
      io.stride = caps[v].frame_stride;
      Plan pl;
      make_plan(&caps[v], dp, &pl);
      io.col_first = pl.col_first; io.col_pairs = pl.col_pairs; io.col_pre = pl.col_pre; io.col_post = pl.col_post;
      io.row_first = pl.row_first; io.row_pairs = pl.row_pairs; io.row_pre = pl.row_pre; io.row_post = pl.row_post;
      if (v < n_next) {
        io.hn_white = next[v].frames;
        io.hn_black = next[v].frames + next[v].frame_stride;
        io.hn_part = reinterpret_cast<uint32_t*>(ws + int64_t(v) * ws_stride + parts_off(n_px));
      }
    }
    mp.n_fin = launch == 0 ? n_fin : 0;             // the first launch finishes them all
    if (mp.n_fin) {
      const int64_t nb = (mp.c.n_tiles + 127) / 128;   // ~128 partials (128 KB) per workgroup
      mp.fin_blocks = int(nb < 1 ? 1 : (nb > kPartsBlocksMax ? kPartsBlocksMax : nb));
      mp.n_state_words = n_state_words(n_px);
      mp.pad_zero = mp.c.n_tiles * kTilePx - n_px;
      for (int k = 0; k < n_fin; ++k) {
        char* slice = fin_ws + int64_t(k) * ws_stride;
        mp.fin[k].parts = reinterpret_cast<const uint32_t*>(slice + parts_off(n_px));
        mp.fin[k].ws = reinterpret_cast<WsHeader*>(slice);
      }
    }
    if (timing_events && timing_events[2 * launch]) (void)hipEventRecord(static_cast<hipEvent_t>(timing_events[2 * launch]), s);
    rc = launch_main3(fn, why, mp, tp, &outs[v0], s);
    if (rc) return rc;
    if (timing_events && timing_events[2 * launch + 1]) (void)hipEventRecord(static_cast<hipEvent_t>(timing_events[2 * launch + 1]), s);
  }
  return SLG_OK;
}

// Stats of n_views views (one launch per kMaxBatch views).
int stats_batch(const slg_capture* caps, int n_views, const slg_decode_params* dp, char* ws, int64_t ws_stride,
                hipStream_t s) {
  if (!caps || n_views < 1 || !dp || !ws) return fail(SLG_ERR_INVALID, "NULL argument");
  if (dp->thresh_mode < 0 || dp->thresh_mode > 2) return fail(SLG_ERR_INVALID, "bad thresh_mode");
  for (int v = 0; v < n_views; ++v) {
    const int rc = check_capture(&caps[v]);
    if (rc) return rc;
    if (caps[v].n_frames < 4)
      return fail(SLG_ERR_NOT_ENOUGH, "Not enough images (got %d, need at least 4).", caps[v].n_frames);
    if (caps[v].height != caps[0].height || caps[v].width != caps[0].width)
      return fail(SLG_ERR_INVALID, "all views of a batch must share one geometry");
  }
  const int64_t n_px = int64_t(caps[0].height) * caps[0].width;
  if (n_views > 1 && (ws_stride < ws_total(n_px) || (ws_stride & 255)))
    return fail(SLG_ERR_INVALID, "ws_stride too small or not 256-aligned");
  for (int v0 = 0; v0 < n_views; v0 += kMaxBatch) {
    const int nb = n_views - v0 < kMaxBatch ? n_views - v0 : kMaxBatch;
    const uint8_t* wh[kMaxBatch];
    const uint8_t* bl[kMaxBatch];
    for (int v = 0; v < nb; ++v) {
      wh[v] = caps[v0 + v].frames;
      bl[v] = caps[v0 + v].frames + caps[v0 + v].frame_stride;
    }
    const int rc = stats_launch_batch(wh, bl, nb, n_px, dp, ws + int64_t(v0) * ws_stride, ws_stride, s);
    if (rc) return rc;
  }
  return SLG_OK;
}

// ------------------------------------------------------------------ ASCII PLY (host)
// "%.4f" of a double exactly as Python formats it (correctly rounded, ties to even, sign of
// negative zero kept, 'nan' / 'inf' / '-inf'): the value m*2^e times 10^4 is rounded with
// 128-bit integer arithmetic and its digits are emitted directly (no printf: ~10x faster);
// magnitudes >= 9.2e14 fall back to glibc's exact printf.  Writes at most kFmtMax chars at p.
constexpr int kFmtMax = 400;
char* fmt4(double x, char* p) {
  if (isnan(x)) { memcpy(p, "nan", 3); return p + 3; }
  if (isinf(x)) {
    if (x < 0) { memcpy(p, "-inf", 4); return p + 4; }
    memcpy(p, "inf", 3); return p + 3;
  }
  uint64_t bits;
  memcpy(&bits, &x, 8);
  const bool neg = bits >> 63;
  const double ax = fabs(x);
  if (ax >= 9.2e14) return p + snprintf(p, kFmtMax, "%.4f", x);
  const int bexp = int((bits >> 52) & 0x7ff);
  uint64_t m = bits & ((uint64_t(1) << 52) - 1);
  int e;
  if (bexp == 0) { e = -1074; } else { m |= uint64_t(1) << 52; e = bexp - 1075; }
  unsigned __int128 v = (unsigned __int128)m * 10000u;
  uint64_t n;                                   // round(|x| * 10^4), ties to even
  if (e >= 0) {
    n = uint64_t(v << e);
  } else {
    const int k = -e;
    if (k >= 127) {
      n = 0;
    } else {
      const unsigned __int128 q = v >> k;
      const unsigned __int128 rem = v - (q << k);
      const unsigned __int128 half = (unsigned __int128)1 << (k - 1);
      n = uint64_t(q) + ((rem > half || (rem == half && (q & 1))) ? 1 : 0);
    }
  }
  if (neg) *p++ = '-';
  uint64_t ip = n / 10000u;
  unsigned fr = unsigned(n % 10000u);
  char tmp[24];
  int t = 0;
  do { tmp[t++] = char('0' + ip % 10); ip /= 10; } while (ip);
  while (t) *p++ = tmp[--t];
  p[0] = '.';
  p[1] = char('0' + fr / 1000);
  p[2] = char('0' + (fr / 100) % 10);
  p[3] = char('0' + (fr / 10) % 10);
  p[4] = char('0' + fr % 10);
  return p + 5;
}

char* fmt_u8(unsigned v, char* p) {
  if (v >= 100) *p++ = char('0' + v / 100);
  if (v >= 10) *p++ = char('0' + (v / 10) % 10);
  *p++ = char('0' + v % 10);
  return p;
}

// ------------------------------------------------------------------ ASCII PLY on the device
// The body of ProcessingLogic._save_ply (server/processing.py:245-248): one line per point,
// f"{x:.4f} {y:.4f} {z:.4f} {r} {g} {b}\n", formatted by the GPU so the cloud never leaves HBM
// as numbers and the host only writes bytes.  The same exact rounding as fmt4 (round(|x|*10^4)
// on the exact binary value, ties to even, '-' from the sign bit); magnitudes >= 9.2e14 (the
// host path prints those through glibc) raise the `bad` flag so the caller formats on the host.
constexpr int kPlyBlock = 256;             // threads per workgroup
constexpr int kPlyPts = 4;                 // consecutive points per thread
constexpr int kPlyChunk = kPlyBlock * kPlyPts;
constexpr int kPlyNumMax = 21;             // '-' + 15 integer digits + '.' + 4
constexpr int kPlyLineMax = 3 * kPlyNumMax + 3 * 3 + 6;

struct PlyWs {                              // device workspace header (include/slgpu.h)
  int64_t total;                            // body bytes
  int32_t bad;                              // a value the device cannot format exactly
  int32_t pad;
};

// |x| * 10^4 rounded exactly; false when |x| >= 9.2e14, NaN or inf (handled by the caller)
__device__ inline uint64_t fixed4(double x, bool& neg) {
  const uint64_t bits = uint64_t(__double_as_longlong(x));
  neg = bits >> 63;
  const int bexp = int((bits >> 52) & 0x7ff);
  uint64_t m = bits & ((uint64_t(1) << 52) - 1);
  int e;
  if (bexp == 0) { e = -1074; } else { m |= uint64_t(1) << 52; e = bexp - 1075; }
  const unsigned __int128 v = (unsigned __int128)m * 10000u;   // < 2^67; e <= -3 below 9.2e14
  const int k = -e;
  if (k >= 127) return 0;
  const unsigned __int128 q = v >> k;
  const unsigned __int128 rem = v - (q << k);
  const unsigned __int128 half = (unsigned __int128)1 << (k - 1);
  return uint64_t(q) + ((rem > half || (rem == half && (uint64_t(q) & 1))) ? 1 : 0);
}

// the line of point i into o (kPlyLineMax bytes), its length; -1: not formattable here
__device__ inline int ply_line(const double* xyz, const uint8_t* bgr, int64_t i, char* o) {
  int len = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double x = xyz[3 * i + c];
    if (!(fabs(x) < 9.2e14)) return -1;          // NaN, inf, or beyond the exact fast path
    bool neg;
    const uint64_t n = fixed4(x, neg);
    if (neg) o[len++] = '-';
    uint64_t ip = n / 10000u;
    const unsigned fr = unsigned(n - ip * 10000u);
    char tmp[16];
    int t = 0;
    do { tmp[t++] = char('0' + ip % 10u); ip /= 10u; } while (ip);
    while (t) o[len++] = tmp[--t];
    o[len++] = '.';
    o[len++] = char('0' + fr / 1000u);
    o[len++] = char('0' + (fr / 100u) % 10u);
    o[len++] = char('0' + (fr / 10u) % 10u);
    o[len++] = char('0' + fr % 10u);
    o[len++] = ' ';
  }
#pragma unroll
  for (int c = 2; c >= 0; --c) {                 // BGR -> "R G B"
    const unsigned v = bgr[3 * i + c];
    if (v >= 100) o[len++] = char('0' + v / 100);
    if (v >= 10) o[len++] = char('0' + (v / 10) % 10);
    o[len++] = char('0' + v % 10);
    o[len++] = c ? ' ' : '\n';
  }
  return len;
}

__device__ inline int ply_thread_bytes(const double* xyz, const uint8_t* bgr, int64_t n, int64_t i0, int* bad) {
  char line[kPlyLineMax];
  int sum = 0;
  for (int j = 0; j < kPlyPts; ++j) {
    const int64_t i = i0 + j;
    if (i >= n) break;
    const int l = ply_line(xyz, bgr, i, line);
    if (l < 0) { atomicOr(bad, 1); return 0; }
    sum += l;
  }
  return sum;
}

// Block-wide exclusive scan of one int per thread (kPlyBlock threads): (prefix, total).
__device__ inline int2 ply_block_scan(int x, int* s_w) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kPlyBlock / 64; ++w) {
    off += w < wave ? s_w[w] : 0;
    tot += s_w[w];
  }
  return make_int2(off + incl - x, tot);
}

// pass 1: bytes per chunk
__global__ __launch_bounds__(kPlyBlock) void ply_len_kernel(const double* xyz, const uint8_t* bgr, int64_t n,
                                                           int64_t* chunk, PlyWs* hdr) {
  __shared__ int s_w[kPlyBlock / 64];
  const int64_t i0 = int64_t(blockIdx.x) * kPlyChunk + int64_t(threadIdx.x) * kPlyPts;
  const int b = ply_thread_bytes(xyz, bgr, n, i0, &hdr->bad);
  const int2 sc = ply_block_scan(b, s_w);
  if (threadIdx.x == 0) chunk[blockIdx.x] = sc.y;
}

// pass 2: exclusive offsets of the chunks (one workgroup, serial over 1024-chunk strides)
__global__ __launch_bounds__(1024) void ply_scan_kernel(int64_t* chunk, int64_t n_chunks, PlyWs* hdr) {
  __shared__ int64_t s_w[16];
  __shared__ int64_t s_carry;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n_chunks; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t x = i < n_chunks ? chunk[i] : 0;
    int64_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int64_t off = s_carry;
    for (int w = 0; w < wave; ++w) off += s_w[w];
    if (i < n_chunks) chunk[i] = off + incl - x;
    __syncthreads();
    if (threadIdx.x == 1023) s_carry = off + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) hdr->total = s_carry;
}

// pass 3: every thread writes its points' lines at the chunk offset + its prefix
__global__ __launch_bounds__(kPlyBlock) void ply_write_kernel(const double* xyz, const uint8_t* bgr, int64_t n,
                                                             const int64_t* chunk, char* text, PlyWs* hdr) {
  __shared__ int s_w[kPlyBlock / 64];
  if (hdr->bad) return;                                      // the caller formats on the host
  const int64_t i0 = int64_t(blockIdx.x) * kPlyChunk + int64_t(threadIdx.x) * kPlyPts;
  const int b = ply_thread_bytes(xyz, bgr, n, i0, &hdr->bad);
  const int2 sc = ply_block_scan(b, s_w);
  char* o = text + chunk[blockIdx.x] + sc.x;
  char line[kPlyLineMax];
  for (int j = 0; j < kPlyPts; ++j) {
    const int64_t i = i0 + j;
    if (i >= n) break;
    const int l = ply_line(xyz, bgr, i, line);
    for (int k = 0; k < l; ++k) o[k] = line[k];
    o += l;
  }
}

}  // namespace

// Error entry for the library's other translation units (csrc/gather.cpp).
int slg_internal_fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// ==================================================================== C ABI
extern "C" {

int32_t slg_version(void) { return SLG_ABI_VERSION; }

#ifndef SLG_BUILD_ID
#define SLG_BUILD_ID "unknown"
#endif
const char* slg_build_id(void) { return SLG_BUILD_ID; }

int32_t slg_kernel_table(char* buf, int64_t cap) {
  if (!buf || cap < 1) return -fail(SLG_ERR_INVALID, "buf NULL or cap < 1");
  int64_t at = 0;
  int32_t missing = 0;
  buf[0] = 0;
  for (const Main3Inst& k : kMain3Table) {
    const std::string name = main3_symbol(k);
    const bool has = device_has(name);
    missing += has ? 0 : 1;
    const std::string line = name + (has ? "\t1\n" : "\t0\n");
    if (at + int64_t(line.size()) < cap) {
      memcpy(buf + at, line.data(), line.size());
      at += int64_t(line.size());
      buf[at] = 0;
    }
  }
  return missing;
}

int32_t slg_last_kernel(char* buf, int64_t cap) {
  if (!buf || cap < 1) return fail(SLG_ERR_INVALID, "buf NULL or cap < 1");
  buf[0] = 0;
  if (!g_last_main) return 0;
  const std::string name = main3_symbol(*g_last_main);
  if (int64_t(name.size()) >= cap) return fail(SLG_ERR_INVALID, "buf too small for the symbol");
  memcpy(buf, name.c_str(), name.size() + 1);
  return 0;
}

const char* slg_last_error(void) { return g_err; }

int64_t slg_workspace_bytes(int64_t n_pixels) { return n_pixels > 0 ? ws_total(n_pixels) : kHeaderBytes; }

int32_t slg_workspace_init(void* workspace, int64_t workspace_bytes, void* stream) {
  if (!workspace) return fail(SLG_ERR_INVALID, "workspace NULL");
  const int64_t n = workspace_bytes < kHeaderBytes ? workspace_bytes : kHeaderBytes;
  if (hipMemsetAsync(workspace, 0, size_t(n), static_cast<hipStream_t>(stream)) != hipSuccess)
    return fail(SLG_ERR_HIP, "hipMemsetAsync failed");
  return SLG_OK;
}

int32_t slg_decode_stats(const slg_capture* cap, const slg_decode_params* dp, void* workspace, void* stream) {
  int rc = check_capture(cap);
  if (rc) return rc;
  if (!dp || !workspace) return fail(SLG_ERR_INVALID, "NULL argument");
  if (cap->n_frames < 4)
    return fail(SLG_ERR_NOT_ENOUGH, "Not enough images (got %d, need at least 4).", cap->n_frames);
  if (dp->thresh_mode < 0 || dp->thresh_mode > 2) return fail(SLG_ERR_INVALID, "bad thresh_mode");
  const int64_t n_px = int64_t(cap->height) * cap->width;
  return stats_launch(cap->frames, cap->frames + cap->frame_stride, n_px, dp, workspace,
                      static_cast<hipStream_t>(stream));
}

int32_t slg_decode_histograms(const slg_capture* cap, const slg_decode_params* dp, void* workspace,
                              uint32_t* hist_out, void* stream) {
  int rc = check_capture(cap);
  if (rc) return rc;
  if (!dp || !workspace || !hist_out) return fail(SLG_ERR_INVALID, "NULL argument");
  if (cap->n_frames < 4)
    return fail(SLG_ERR_NOT_ENOUGH, "Not enough images (got %d, need at least 4).", cap->n_frames);
  if (dp->thresh_mode != SLG_THRESH_OTSU && dp->thresh_mode != SLG_THRESH_PERCENTILE)
    return fail(SLG_ERR_INVALID, "histograms serve Otsu / percentile thresholds (manual ones need none)");
  if (reinterpret_cast<uintptr_t>(hist_out) & 3) return fail(SLG_ERR_INVALID, "hist_out must be 4-byte aligned");
  const int64_t n_px = int64_t(cap->height) * cap->width;
  const uint8_t* white = cap->frames;
  const uint8_t* black = cap->frames + cap->frame_stride;
  return stats_launch_batch(&white, &black, 1, n_px, dp, static_cast<char*>(workspace), 0,
                            static_cast<hipStream_t>(stream), false, hist_out);
}

int32_t slg_thresholds_from_histograms(const uint32_t* hist, int64_t n_pixels, const slg_decode_params* dp,
                                       void* workspace, int64_t n_band_pixels, void* stream) {
  if (!hist || !dp || !workspace) return fail(SLG_ERR_INVALID, "NULL argument");
  if (n_pixels < 1 || n_band_pixels < 1 || n_band_pixels > n_pixels || n_pixels >= (int64_t(1) << 31))
    return fail(SLG_ERR_INVALID, "need 1 <= n_band_pixels <= n_pixels < 2^31");
  if (dp->thresh_mode != SLG_THRESH_OTSU && dp->thresh_mode != SLG_THRESH_PERCENTILE)
    return fail(SLG_ERR_INVALID, "histograms serve Otsu / percentile thresholds (manual ones need none)");
  if (reinterpret_cast<uintptr_t>(hist) & 3) return fail(SLG_ERR_INVALID, "hist must be 4-byte aligned");
  const int64_t nsw = n_state_words(n_band_pixels);
  int64_t grid = (nsw + kBlock - 1) / kBlock;
  grid = grid < 1 ? 1 : (grid > 64 ? 64 : grid);
  hipLaunchKernelGGL(hist_thresholds_kernel, dim3(unsigned(grid)), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     hist, reinterpret_cast<WsHeader*>(workspace), n_pixels, dp->thresh_mode, nsw);
  return check_launch("hist_thresholds_kernel");
}

int32_t slg_decode(const slg_capture* cap, const slg_decode_params* dp, void* workspace, int32_t* col_out,
                   int32_t* row_out, uint8_t* mask_out, void* stream) {
  int rc = check_capture(cap);
  if (rc) return rc;
  if (!dp || !workspace || !col_out || !row_out || !mask_out) return fail(SLG_ERR_INVALID, "NULL argument");
  if ((reinterpret_cast<uintptr_t>(col_out) | reinterpret_cast<uintptr_t>(row_out)) & 15 ||
      reinterpret_cast<uintptr_t>(mask_out) & 7)
    return fail(SLG_ERR_INVALID, "map outputs must be 16-byte (col,row) / 8-byte (mask) aligned");
  Plan pl;
  rc = make_plan(cap, dp, &pl);
  if (rc) return rc;
  const int64_t n_px = int64_t(cap->height) * cap->width;
  MainParams mp{};
  mp.frames = cap->frames;
  mp.stride = cap->frame_stride;
  mp.n_px = n_px;
  mp.width = cap->width;
  mp.col_first = pl.col_first; mp.col_pairs = pl.col_pairs; mp.col_pre = pl.col_pre; mp.col_post = pl.col_post;
  mp.row_first = pl.row_first; mp.row_pairs = pl.row_pairs; mp.row_pre = pl.row_pre; mp.row_post = pl.row_post;
  mp.out_col = col_out; mp.out_row = row_out; mp.out_mask = mask_out;
  mp.ws = reinterpret_cast<WsHeader*>(workspace);
  mp.n_tiles = n_tiles_of(n_px);
  hipLaunchKernelGGL(decode_maps_kernel, dim3(unsigned((n_px + kMapsPx - 1) / kMapsPx)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), mp);
  return check_launch("decode_maps_kernel");
}

int32_t slg_triangulate(const slg_maps* maps, const slg_calib* calib, const slg_tri_params* tp, void* workspace,
                        const slg_cloud* out, void* stream) {
  if (!maps || !maps->col || !maps->mask || !maps->texture || !workspace) return fail(SLG_ERR_INVALID, "NULL argument");
  if (maps->height < 1 || maps->width < 1) return fail(SLG_ERR_INVALID, "bad map size");
  if (tp && tp->row_mode != 0 && !maps->row) return fail(SLG_ERR_INVALID, "row map required for row_mode 1/2");
  if ((reinterpret_cast<uintptr_t>(maps->col) | reinterpret_cast<uintptr_t>(maps->row)) & 15 ||
      (reinterpret_cast<uintptr_t>(maps->mask) | reinterpret_cast<uintptr_t>(maps->texture)) & 7)
    return fail(SLG_ERR_INVALID, "maps must be 16-byte (col,row) / 8-byte (mask,texture) aligned");
  const int64_t n_px = int64_t(maps->height) * maps->width;
  MainParams mp{};
  int rc = fill_calib(mp, calib, tp, n_px, maps->width);
  if (rc) return rc;
  rc = fill_out(mp, out, tp, n_px, workspace);
  if (rc) return rc;
  mp.in_col = maps->col; mp.in_row = maps->row; mp.in_mask = maps->mask; mp.texture = maps->texture;
  hipStream_t s = static_cast<hipStream_t>(stream);
  rc = stats_launch(nullptr, nullptr, n_px, nullptr, workspace, s);   // arms states only (manual mode)
  if (rc) return rc;
  Main3Params m3{};
  m3.c = mp;
  m3.n_views = 1;
  rc = fill_view(m3.v[0], out, tp, n_px, workspace);
  if (rc) return rc;
  m3.v[0].in_col = maps->col; m3.v[0].in_row = maps->row; m3.v[0].in_mask = maps->mask;
  m3.v[0].texture = maps->texture;
  const char* why = nullptr;
  const Main3Fn fn = pick_main(0, tp->row_mode, tp->xyz_f64 ? 1 : 0, calib->ray_mode, 0, &why);
  return launch_main3(fn, why, m3, tp, out, s);
}

static int reconstruct_impl(const slg_capture* cap, const slg_decode_params* dp, const slg_calib* calib,
                            const slg_tri_params* tp, void* workspace, const slg_cloud* out, void* stream,
                            bool with_stats) {
  if (!cap || !dp || !workspace) return fail(SLG_ERR_INVALID, "NULL argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (with_stats) {
    int rc = check_batch(cap, 1);
    if (!rc) rc = make_plan(cap, dp, nullptr);
    if (!rc) rc = stats_batch(cap, 1, dp, static_cast<char*>(workspace), 0, s);
    if (rc) return rc;
  }
  return fused_batch(cap, 1, dp, calib, tp, static_cast<char*>(workspace), 0, out, nullptr, s);
}

int32_t slg_reconstruct(const slg_capture* cap, const slg_decode_params* dp, const slg_calib* calib,
                        const slg_tri_params* tp, void* workspace, const slg_cloud* out, void* stream) {
  return reconstruct_impl(cap, dp, calib, tp, workspace, out, stream, true);
}

int32_t slg_decode_triangulate(const slg_capture* cap, const slg_decode_params* dp, const slg_calib* calib,
                               const slg_tri_params* tp, void* workspace, const slg_cloud* out, void* stream) {
  return reconstruct_impl(cap, dp, calib, tp, workspace, out, stream, false);
}

int64_t slg_ply_format_bound(int64_t n) { return n < 0 ? -fail(SLG_ERR_INVALID, "n < 0") : n * kPlyLineMax; }

int64_t slg_ply_format_ws_bytes(int64_t n) {
  if (n < 0) return -fail(SLG_ERR_INVALID, "n < 0");
  return int64_t(sizeof(PlyWs)) + 8 * ((n + kPlyChunk - 1) / kPlyChunk + 1);
}

int32_t slg_ply_format(const double* xyz, const uint8_t* bgr, int64_t n, char* text, void* ws, void* stream) {
  if (n < 0 || !ws || (n > 0 && (!xyz || !bgr || !text))) return fail(SLG_ERR_INVALID, "bad argument");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  PlyWs* hdr = static_cast<PlyWs*>(ws);
  int64_t* chunk = reinterpret_cast<int64_t*>(hdr + 1);
  if (hipMemsetAsync(hdr, 0, sizeof(PlyWs), s) != hipSuccess) return fail(SLG_ERR_HIP, "hipMemsetAsync");
  if (n == 0) return SLG_OK;
  const int64_t nc = (n + kPlyChunk - 1) / kPlyChunk;
  if (nc > INT_MAX) return fail(SLG_ERR_UNSUPPORTED, "cloud too large");
  hipLaunchKernelGGL(ply_len_kernel, dim3(unsigned(nc)), dim3(kPlyBlock), 0, s, xyz, bgr, n, chunk, hdr);
  int rc = check_launch("ply_len_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(ply_scan_kernel, dim3(1), dim3(1024), 0, s, chunk, nc, hdr);
  rc = check_launch("ply_scan_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(ply_write_kernel, dim3(unsigned(nc)), dim3(kPlyBlock), 0, s, xyz, bgr, n, chunk, text, hdr);
  return check_launch("ply_write_kernel");
}

int64_t slg_ply_write(const char* path, const double* xyz, const uint8_t* bgr, int64_t n, int32_t n_threads) {
  if (!path || n < 0 || (n > 0 && (!xyz || !bgr))) return -fail(SLG_ERR_INVALID, "bad argument");
  // default: the CPUs this process may run on, at most 16 (the formatter is ~60 ns per point
  // per thread; more threads only contend with the frame decoders of the batch pipeline)
  int nt = n_threads > 0 ? n_threads : std::min(16, int(std::thread::hardware_concurrency()));
  if (nt < 1) nt = 1;
  if (int64_t(nt) * 4096 > n) nt = int(n / 4096) + 1;
  std::vector<std::string> parts(static_cast<size_t>(nt));
  auto work = [&](int t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    std::string& o = parts[size_t(t)];
    o.reserve(size_t(hi - lo) * 40);
    char line[3 * kFmtMax + 32];
    for (int64_t i = lo; i < hi; ++i) {
      char* p = line;
      p = fmt4(xyz[3 * i], p); *p++ = ' ';
      p = fmt4(xyz[3 * i + 1], p); *p++ = ' ';
      p = fmt4(xyz[3 * i + 2], p); *p++ = ' ';
      p = fmt_u8(bgr[3 * i + 2], p); *p++ = ' ';  // BGR -> "R G B" (processing.py:248)
      p = fmt_u8(bgr[3 * i + 1], p); *p++ = ' ';
      p = fmt_u8(bgr[3 * i], p); *p++ = '\n';
      o.append(line, size_t(p - line));
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  char hdr[320];
  const int hlen = snprintf(hdr, sizeof(hdr), "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\n"
                            "property float y\nproperty float z\nproperty uchar red\nproperty uchar green\n"
                            "property uchar blue\nend_header\n", (long long)n);
  // Each thread's part goes to its own offset with pwrite, in parallel (no serial copy through
  // a stdio buffer: ~45 MB per C2 view).
  std::vector<int64_t> off(size_t(nt) + 1);
  off[0] = hlen;
  for (int t = 0; t < nt; ++t) off[size_t(t) + 1] = off[size_t(t)] + int64_t(parts[size_t(t)].size());
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) return -fail(SLG_ERR_INVALID, "cannot open %s", path);
  auto put = [fd](const char* b, int64_t len, int64_t at) {
    while (len > 0) {
      const ssize_t w = pwrite(fd, b, size_t(len), off_t(at));
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return false;
      b += w; len -= w; at += w;
    }
    return true;
  };
  std::vector<char> ok(size_t(nt) + 1, 1);
  ok[size_t(nt)] = put(hdr, hlen, 0);
  th.clear();
  for (int t = 1; t < nt; ++t)
    th.emplace_back([&, t] { ok[size_t(t)] = put(parts[size_t(t)].data(), int64_t(parts[size_t(t)].size()), off[size_t(t)]); });
  ok[0] = put(parts[0].data(), int64_t(parts[0].size()), off[0]);
  for (auto& x : th) x.join();
  const bool closed = close(fd) == 0;
  for (char c : ok)
    if (!c) return -fail(SLG_ERR_INVALID, "write failed: %s", path);
  if (!closed) return -fail(SLG_ERR_INVALID, "write failed: %s", path);
  return off[size_t(nt)];
}

int32_t slg_reconstruct_batch(const slg_capture* caps, int32_t n_views, const slg_decode_params* dp,
                              const slg_calib* calib, const slg_tri_params* tp, void* workspace,
                              int64_t ws_stride, const slg_cloud* outs, void* const* timing_events,
                              void* stream) {
  if (!caps || n_views < 1 || !dp || !workspace || !outs) return fail(SLG_ERR_INVALID, "NULL argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* ws = static_cast<char*>(workspace);
  int rc = check_batch(caps, n_views);              // validate everything before enqueueing
  for (int v = 0; v < n_views && !rc; ++v) rc = make_plan(&caps[v], dp, nullptr);
  if (rc) return rc;
  for (int v0 = 0, launch = 0; v0 < n_views; v0 += kMaxViews, ++launch) {
    const int nb = n_views - v0 < kMaxViews ? n_views - v0 : kMaxViews;
    rc = stats_batch(caps + v0, nb, dp, ws + int64_t(v0) * ws_stride, ws_stride, s);
    if (rc) return rc;
    rc = fused_batch(caps + v0, nb, dp, calib, tp, ws + int64_t(v0) * ws_stride, ws_stride, outs + v0,
                     timing_events ? timing_events + 2 * launch : nullptr, s);
    if (rc) return rc;
  }
  return SLG_OK;
}

int32_t slg_decode_stats_batch(const slg_capture* caps, int32_t n_views, const slg_decode_params* dp,
                               void* workspace, int64_t ws_stride, void* stream) {
  return stats_batch(caps, n_views, dp, static_cast<char*>(workspace), ws_stride, static_cast<hipStream_t>(stream));
}

int32_t slg_decode_triangulate_batch(const slg_capture* caps, int32_t n_views, const slg_decode_params* dp,
                                     const slg_calib* calib, const slg_tri_params* tp, void* workspace,
                                     int64_t ws_stride, const slg_cloud* outs, void* const* timing_events,
                                     void* stream) {
  return fused_batch(caps, n_views, dp, calib, tp, static_cast<char*>(workspace), ws_stride, outs, timing_events,
                     static_cast<hipStream_t>(stream));
}

int32_t slg_decode_triangulate_batch_next(const slg_capture* caps, int32_t n_views, const slg_decode_params* dp,
                                          const slg_calib* calib, const slg_tri_params* tp, void* workspace,
                                          int64_t ws_stride, const slg_cloud* outs, const slg_capture* next,
                                          int32_t n_next, void* const* timing_events, void* stream) {
  return fused_batch(caps, n_views, dp, calib, tp, static_cast<char*>(workspace), ws_stride, outs, timing_events,
                     static_cast<hipStream_t>(stream), next, next ? n_next : 0);
}

int32_t slg_decode_triangulate_batch_carry(const slg_capture* caps, int32_t n_views, const slg_decode_params* dp,
                                           const slg_calib* calib, const slg_tri_params* tp, void* workspace,
                                           int64_t ws_stride, const slg_cloud* outs, const slg_capture* next,
                                           int32_t n_next, void* fin_workspace, int32_t n_fin,
                                           void* const* timing_events, void* stream) {
  return fused_batch(caps, n_views, dp, calib, tp, static_cast<char*>(workspace), ws_stride, outs, timing_events,
                     static_cast<hipStream_t>(stream), next, next ? n_next : 0, static_cast<char*>(fin_workspace),
                     fin_workspace ? n_fin : 0);
}

int32_t slg_decode_stats_partials_batch(int32_t n_views, int32_t height, int32_t width, const slg_decode_params* dp,
                                        void* workspace, int64_t ws_stride, void* stream) {
  if (n_views < 1 || !dp || !workspace || height < 1 || width < 1) return fail(SLG_ERR_INVALID, "bad argument");
  if (dp->thresh_mode != SLG_THRESH_OTSU) return fail(SLG_ERR_UNSUPPORTED, "partial histograms are Otsu only");
  const int64_t n_px = int64_t(height) * width;
  if (n_views > 1 && (ws_stride < ws_total(n_px) || (ws_stride & 255)))
    return fail(SLG_ERR_INVALID, "ws_stride too small or not 256-aligned");
  char* ws = static_cast<char*>(workspace);
  for (int v0 = 0; v0 < n_views; v0 += kMaxBatch) {
    const int nb = n_views - v0 < kMaxBatch ? n_views - v0 : kMaxBatch;
    const int rc = stats_launch_batch(nullptr, nullptr, nb, n_px, dp, ws + int64_t(v0) * ws_stride, ws_stride,
                                      static_cast<hipStream_t>(stream), true);
    if (rc) return rc;
  }
  return SLG_OK;
}

int32_t slg_rgb_to_gray(const uint8_t* rgb, int32_t channels, int64_t n_pixels, int64_t src_stride, int32_t n_frames,
                        uint8_t* gray, int64_t gray_stride, uint8_t* bgr0, int32_t weights, void* stream) {
  if (!rgb || !gray || n_pixels < 1 || n_frames < 1 || (channels != 3 && channels != 4))
    return fail(SLG_ERR_INVALID, "bad rgb_to_gray argument");
  if (src_stride < n_pixels * channels || gray_stride < n_pixels)
    return fail(SLG_ERR_INVALID, "strides smaller than a frame");
  if (weights != SLG_GRAY_PNG && weights != SLG_GRAY_BMP) return fail(SLG_ERR_INVALID, "bad weights");
  const int64_t per_block = int64_t(kBlock) * kRgbPx;
  hipLaunchKernelGGL(rgb_gray_kernel, dim3(unsigned((n_pixels + per_block - 1) / per_block), unsigned(n_frames)),
                     dim3(kBlock), 0, static_cast<hipStream_t>(stream), rgb, channels, n_pixels, src_stride, gray,
                     gray_stride, bgr0, weights == SLG_GRAY_BMP ? 1 : 0);
  return check_launch("rgb_gray_kernel");
}

int32_t slg_workspace_set_arena(void* workspace, int64_t ws_stride, int32_t n_slices, int64_t* cursor,
                                int64_t capacity_points, int32_t points_per_valid, void* stream) {
  if (!workspace || n_slices < 1 || (n_slices > 1 && (ws_stride < kHeaderBytes || (ws_stride & 255))))
    return fail(SLG_ERR_INVALID, "bad workspace / stride");
  if (cursor && (capacity_points < 0 || (points_per_valid != 1 && points_per_valid != 2)))
    return fail(SLG_ERR_INVALID, "arena capacity < 0 or points_per_valid not 1 / 2");
  if (reinterpret_cast<uintptr_t>(cursor) & 7) return fail(SLG_ERR_INVALID, "cursor must be 8-byte aligned");
  hipLaunchKernelGGL(set_arena_kernel, dim3(unsigned((n_slices + 63) / 64)), dim3(64), 0, static_cast<hipStream_t>(stream),
                     static_cast<char*>(workspace), ws_stride, int(n_slices),
                     reinterpret_cast<unsigned long long*>(cursor), cursor ? capacity_points : 0,
                     cursor ? points_per_valid : 0);
  return check_launch("set_arena_kernel");
}

int32_t slg_gray_texture(const uint8_t* frame0, int64_t n_pixels, uint8_t* bgr, void* stream) {
  if (!frame0 || !bgr || n_pixels < 1) return fail(SLG_ERR_INVALID, "bad gray_texture argument");
  hipLaunchKernelGGL(gray_texture_kernel, dim3(unsigned((n_pixels + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), frame0, n_pixels, bgr);
  return check_launch("gray_texture_kernel");
}

int32_t slg_rays_match_pinhole(const double* rays, int32_t height, int32_t width, double fx, double fy, double cx,
                               double cy, int64_t* mismatches, void* stream) {
  if (!rays || !mismatches || height < 1 || width < 1) return fail(SLG_ERR_INVALID, "bad argument");
  const int64_t n_px = int64_t(height) * width;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(mismatches, 0, sizeof(int64_t), s) != hipSuccess) return fail(SLG_ERR_HIP, "hipMemsetAsync failed");
  hipLaunchKernelGGL(pinhole_kernel, dim3(unsigned((n_px + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rays, n_px,
                     int(width), fx, fy, cx, cy, reinterpret_cast<unsigned long long*>(mismatches));
  return check_launch("pinhole_kernel");
}

}  // extern "C"
