// png_device.hip -- PNG decode on the device for the batch file path (include/slgpu.h,
// slg_png_decode_device): the cv2.imread(f, 0) of every used capture frame
// (server/processing.py:59-60,98-99; captures written by server/sl_system.py:444-476 or uploaded
// by the phone, server/server.py:86) with the host left only reading files.  Two kernels per
// batch of frames:
//
// png_inflate_kernel -- one 64-lane wave per zlib stream.  The symbol decode is inherently
//   serial, so it runs wave-uniform (bit buffer in SGPRs, Huffman tables -- one of them giving
//   up to 4 literals per lookup -- and the 32 KB history ring in LDS, 50 KB per wave: 3 streams
//   per CU, 768 in flight); literal runs are written by 4 lanes, LZ77 copies by all 64
//   lanes (a copy whose distance is under 64 repeats its period, so no lane reads a byte the
//   copy itself has yet to write).  Inflated scanlines go to the frame's raw scratch.
// png_unfilter_kernel -- one wave per frame undoes the five scanline filters (PNG §9) over
//   bands of 64 rows as a wavefront: lane L holds row y0 + L and at step t reconstructs its byte
//   x = t - L, so the byte above (x of row L - 1) was made by lane L - 1 one step earlier and
//   arrives by a lane shift, the bytes to the left come from the lane's own last `bpp` steps.
//   Every filter type (Sub / Up / Average / Paeth) is then one data-parallel step, where a row
//   at a time is serial for Average and Paeth.  The same pass sums the Adler-32 of the inflated
//   bytes and checks it against the stream's trailer.
// A frame that fails any check gets a non-zero status and is decoded on the host by the caller.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "../../include/slgpu.h"

int slg_internal_fail(int code, const char* fmt, ...);

namespace {

constexpr int kRing = 36864;                // LDS output ring: the 32 KB deflate window + what is
constexpr int kFlush = 2048;                //   not yet flushed to the frame's raw scratch (flushed
                                            //   2 KB at a time by the whole wave; < 2048 + 258
                                            //   unflushed bytes).  50 KB of LDS per wave with the
                                            //   tables: 3 streams per CU, 768 in flight
constexpr int kFastBits = 10;               // primary Huffman table index bits
constexpr int kAdlerMod = 65521;
constexpr int kMaxRowBytes = 24576;         // device un-filter: rows up to 24 KB (6000 px RGBA: host)

// RFC 1951 §3.2.5 length / distance bases and extra bits, computed (SALU) rather than read from
// tables: a table read is a vector-memory round trip on every match's serial chain.
// Length code 257 + s: s < 8 -> 3 + s; s == 28 -> 258; else e = (s - 4) / 4 extra bits on
// ((4 + s % 4) << e) + 3.  Distance code d: d < 4 -> d + 1; else e = d / 2 - 1 on
// ((2 + d % 2) << e) + 1.
__device__ inline uint32_t len_extra(uint32_t s) { return (s < 8u || s == 28u) ? 0u : (s - 4u) >> 2; }
__device__ inline uint32_t len_base(uint32_t s) {
  return s < 8u ? s + 3u : s == 28u ? 258u : ((4u + (s & 3u)) << len_extra(s)) + 3u;
}
__device__ inline uint32_t dist_extra(uint32_t d) { return d < 4u ? 0u : (d >> 1) - 1u; }
__device__ inline uint32_t dist_base(uint32_t d) { return d < 4u ? d + 1u : ((2u + (d & 1u)) << dist_extra(d)) + 1u; }
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// PNG_PROF builds (tools/png_device_bench.py --prof): per-launch sums of event counts and
// 100 MHz timer intervals over all streams, read back by slg_png_prof_read; PNG_ABL bits switch
// parts off for timing (the output is then wrong): 1 literal LDS writes, 2 match copies,
// 4 ring flushes.
#ifndef PNG_PROF
#define PNG_PROF 0
#endif
#ifndef PNG_ABL
#define PNG_ABL 0
#endif
enum { kPfTotal, kPfBuild, kPfHeader, kPfCopy, kPfFlush, kPfLit, kPfMatch, kPfMatchBytes, kPfBlocks,
       kPfRuns, kPfSymbols, kPfN = 16 };
#if PNG_PROF
__device__ unsigned long long g_png_prof[kPfN];
#endif
__device__ inline uint64_t pf_now() { return PNG_PROF ? __builtin_amdgcn_s_memrealtime() : 0; }

// Canonical Huffman code in LDS: a 2^kFastBits table for codes up to kFastBits bits (entry =
// symbol | length << 9, 0 = longer code or none) and the counts + sorted symbols the slow
// (bit at a time, canonical) decode walks for the rest.
struct Huff {
  uint16_t fast[1 << kFastBits];
  uint32_t count[16];
  uint16_t sym[288];
};

constexpr uint32_t kRsrcFlags = 0x00020000;  // buffer descriptor word 3 (as the frame loads use)

__device__ inline uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// A buffer descriptor over [p, p + n) built from wave-uniform (SGPR) values: the frame
// descriptor is a per-workgroup load the compiler cannot prove uniform, and a descriptor left in
// VGPRs turns every buffer access into a readfirstlane waterfall loop.
__device__ inline __amdgpu_buffer_rsrc_t uni_rsrc(const void* p, uint32_t n) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t u = uint64_t(uni(uint32_t(a))) | (uint64_t(uni(uint32_t(a >> 32))) << 32);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), 0, uni(n), kRsrcFlags);
}

// Wave-uniform LSB-first bit reader over the zlib stream.  The stream arrives 256 bytes at a time
// by ONE vector buffer load (lane i holds word i of the chunk) issued a chunk ahead, and a refill
// takes the next word with v_readlane (an SGPR): no load sits on the decode's critical path, and
// no flat access whose completion every LDS wait (lgkmcnt) would also have to await.  Reads past
// the stream come back 0 (buffer bounds).

struct Bits {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t cur, next;       // this chunk / the next one, one word per lane (VGPRs)
  uint32_t base;            // byte offset of `cur` in the stream
  int k;                    // next word of `cur`
  uint64_t buf;
  int cnt;
};

__device__ inline void bits_init(Bits& b, const uint8_t* z, int64_t zlen) {
  // zlen + 8: slg_png_zstream leaves 8 readable (zeroed) bytes behind every stream, so the dword
  // holding the stream's last bytes is read whole (with zlen alone, a dword that straddled zlen
  // would come back 0; only the Adler-32 trailer after the deflate data kept that harmless)
  b.rsrc = uni_rsrc(z, uint32_t(zlen + 8));
  const int lane = threadIdx.x;
  b.cur = __builtin_amdgcn_raw_buffer_load_b32(b.rsrc, lane * 4, 0, 0);
  b.next = __builtin_amdgcn_raw_buffer_load_b32(b.rsrc, lane * 4, 256, 0);
  b.base = 0;
  b.k = 0;
  b.buf = 0;
  b.cnt = 0;
}

__device__ inline void refill(Bits& b) {
  if (b.cnt <= 32) {
    const uint32_t w = __builtin_amdgcn_readlane(b.cur, b.k);
    b.buf |= uint64_t(w) << b.cnt;
    b.cnt += 32;
    if (++b.k == 64) {                                   // the next chunk (loaded 64 words ago)
      b.cur = b.next;
      b.base += 256;
      b.k = 0;
      __builtin_amdgcn_sched_barrier(0);                 // (so the load may land in `next` itself)
      b.next = __builtin_amdgcn_raw_buffer_load_b32(b.rsrc, int(threadIdx.x) * 4, int(b.base + 256), 0);
    }
  }
}

__device__ inline int64_t bits_consumed(const Bits& b) { return int64_t(b.base) * 8 + int64_t(b.k) * 32 - b.cnt; }

__device__ inline uint32_t getbits(Bits& b, int n) {        // n <= 16
  refill(b);
  const uint32_t v = uint32_t(b.buf) & ((1u << n) - 1u);
  b.buf >>= n;
  b.cnt -= n;
  return v;
}

// Codes longer than kFastBits: canonical decode a bit at a time (rare; kept out of line so the
// decode loop stays small).  Returns symbol | bits << 16, or ~0u for an invalid code.  Takes and
// returns plain values: the caller re-reads the result with readfirstlane, so the symbol stays
// wave-uniform (SGPRs, scalar branches) on both paths.
__device__ __attribute__((noinline)) uint32_t decode_slow(uint64_t buf, const Huff& h) {
  int code = 0, first = 0, index = 0;
#pragma unroll 1
  for (int len = 1; len <= 15; ++len) {
    code |= int(buf & 1u);
    buf >>= 1;
    const int count = int(h.count[len]);
    if (code - count < first) return uint32_t(h.sym[index + (code - first)]) | (uint32_t(len) << 16);
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return ~0u;
}

__device__ inline int decode(Bits& b, const Huff& h) {
  refill(b);                                                 // (cnt > 32 >= 15 bits after it)
  const uint32_t e = uni(h.fast[uint32_t(b.buf) & ((1u << kFastBits) - 1u)]);
  const uint32_t r = (e >> 9) ? ((e & 511u) | ((e >> 9) << 16)) : uni(decode_slow(b.buf, h));
  if (r == ~0u) return -1;
  const int len = int(r >> 16);
  b.buf >>= len;
  b.cnt -= len;
  return int(r & 0xffffu);
}

// Literal runs: lit4[i] holds the literals that the next kLitBits stream bits i decode to in a
// row, as long as each code fits the bits still known (at most kLitMax), with their count and the
// bits they use; a count of 0 (the first code is a length / end-of-block symbol, or longer than
// kFastBits) falls back to decode().  PNG scanline residuals code in ~4 bits a byte, so one LDS
// lookup on the serial chain yields ~2.5 literals instead of one.
#ifndef PNG_LIT11
#define PNG_LIT11 1   // 11-bit index, 4-byte entries, <= 3 literals: 14.07 vs 16.28 ms/view for the
                      // 10-bit, 8-byte, <= 4 form (profiles/r4n/png_lit11_ab.log)
#endif
#if PNG_LIT11
constexpr int kLitBits = 11, kLitMax = 3;
typedef uint32_t LitEntry;                   // bytes 0-23, count in 24-25, bits used in 26-29
constexpr int kLitCountShift = 24;
#else
constexpr int kLitBits = kFastBits, kLitMax = 4;
typedef uint64_t LitEntry;                   // bytes 0-31, count in 32-35, bits used in 36-39
constexpr int kLitCountShift = 32;
#endif

__device__ inline void build_lit4(LitEntry* lit4, const Huff& h) {
  for (int i = int(threadIdx.x); i < (1 << kLitBits); i += 64) {
    uint32_t idx = uint32_t(i), used = 0, n = 0, lits = 0;
    while (n < uint32_t(kLitMax)) {
      const uint32_t e = h.fast[idx & ((1u << kFastBits) - 1u)];
      const uint32_t l = e >> 9, sym = e & 511u;
      if (l == 0 || used + l > uint32_t(kLitBits) || sym >= 256u) break;
      lits |= sym << (8 * n);
      ++n;
      used += l;
      idx >>= l;
    }
    lit4[i] = LitEntry(lits) | (LitEntry(n | (used << 4)) << kLitCountShift);
  }
}

// Build `h` from code lengths lens[0..n) (LDS); all 64 lanes call it.  False for an
// over-subscribed set (an incomplete one decodes only its codes: a missing code fails decode()).
// w: LDS work words [48] (start of each length in the sorted symbols, its first canonical code,
// a running cursor).
__device__ __attribute__((noinline)) bool build(Huff& h, const uint8_t* lens, int n, uint32_t* w) {
  const int lane = threadIdx.x;
  uint32_t* offs = w;
  uint32_t* first = w + 16;
  uint32_t* cur = w + 32;
  if (lane < 16) h.count[lane] = 0;
  for (int i = lane; i < (1 << kFastBits); i += 64) h.fast[i] = 0;
  __syncthreads();
  for (int s = lane; s < n; s += 64)
    if (lens[s]) atomicAdd(&h.count[lens[s]], 1u);
  __syncthreads();
  if (lane == 0) {
    int left = 1;
    uint32_t off = 0, code = 0;
    offs[0] = first[0] = 0;
    for (int l = 1; l < 16; ++l) {
      left = (left << 1) - int(h.count[l]);
      offs[l] = cur[l] = off;                    // start of length l in the sorted symbols
      off += h.count[l];
      code = (code + (l > 1 ? h.count[l - 1] : 0u)) << 1;
      first[l] = code;                           // canonical code of its first symbol
    }
    cur[0] = left < 0 ? 1u : 0u;                 // over-subscribed
    for (int s = 0; s < n; ++s)
      if (lens[s]) h.sym[cur[lens[s]]++] = uint16_t(s);
  }
  __syncthreads();
  const bool bad = uni(cur[0]) != 0;
  const uint32_t total = offs[15] + h.count[15];
  for (uint32_t i = lane; i < total; i += 64) {  // the fast entries of every code <= kFastBits bits
    const int s = h.sym[i];
    const int l = lens[s];
    if (l > kFastBits) continue;
    const uint32_t c = first[l] + (i - offs[l]);
    const uint32_t rev = __builtin_bitreverse32(c) >> (32 - l);
    for (uint32_t k = 0; k < (1u << (kFastBits - l)); ++k) h.fast[rev | (k << l)] = uint16_t(s | (l << 9));
  }
  __syncthreads();
  return !bad;
}

#ifndef PNG_LIT_WORD
#define PNG_LIT_WORD 1                       // literal runs stored as one unaligned LDS word by lane 0
#endif

struct InflateLds {
  alignas(16) uint8_t ring[kRing + 4];    // + 4 slack bytes: a literal-run word at the ring's end
  LitEntry lit4[1 << kLitBits];
  Huff lit, dist;
  uint8_t lens[320];                      // litlen code lengths at [0, 288), distance at [288, 320)
  uint32_t work[48];
};

// Ring bytes [flushed, flushed + n) -> raw[flushed ...], by all lanes: whole kFlush blocks as
// 16-byte moves, the final ragged part byte by byte.
__device__ inline void flush_ring(const uint8_t* ring, __amdgpu_buffer_rsrc_t out, int64_t flushed, int n) {
  const int lane = threadIdx.x;
  const int fr = int(flushed % kRing);
  __builtin_amdgcn_wave_barrier();
  if (n == kFlush) {
#pragma unroll
    for (int q = 0; q < kFlush / (64 * 16); ++q) {
      const int o = (q * 64 + lane) * 16;
      const uint4 v = *reinterpret_cast<const uint4*>(ring + fr + o);
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 w = {v.x, v.y, v.z, v.w};
      __builtin_amdgcn_raw_buffer_store_b128(w, out, o, int(flushed), 0);
    }
  } else {
    for (int o = lane; o < n; o += 64) {
      int r = fr + o;
      if (r >= kRing) r -= kRing;
      __builtin_amdgcn_raw_buffer_store_b8(ring[r], out, o, int(flushed), 0);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64) void png_inflate_kernel(const slg_png_frame* frames, int32_t* status) {
  __shared__ InflateLds L;
  const int lane = threadIdx.x;
  const slg_png_frame f = frames[blockIdx.x];
  // (the descriptor is a vector load: its sizes re-read as wave-uniform SGPR values)
  const int64_t row = 1 + int64_t(int32_t(uni(uint32_t(f.width)))) * int32_t(uni(uint32_t(f.channels)));
  const int64_t n_out64 = int64_t(int32_t(uni(uint32_t(f.height)))) * row;
  const int32_t n_out = n_out64 < INT32_MAX ? int32_t(n_out64) : 0;    // (32-bit positions: SALU compares)
  Bits b;
  bits_init(b, f.z, f.zlen);
  const __amdgpu_buffer_rsrc_t out = uni_rsrc(f.raw, uint32_t(n_out));
  int err = 0;
  int32_t pos = 0, flushed = 0;
  if (n_out64 >= INT32_MAX) err = SLG_PNG_E_UNSUPPORTED;
  int ridx = 0;                                            // pos % kRing
  uint64_t pf[kPfN] = {};
  const uint64_t pf_t0 = pf_now();
  auto flush4k = [&]() {
    const uint64_t t = pf_now();
    if (!(PNG_ABL & 4)) flush_ring(L.ring, out, flushed, kFlush);
    flushed += kFlush;
    if (PNG_PROF) pf[kPfFlush] += pf_now() - t;
  };
  auto put = [&](uint8_t v) {                              // one literal byte (lane 0 writes)
    if (lane == 0 && !(PNG_ABL & 1)) L.ring[ridx] = v;
    ++pos;
    if (++ridx == kRing) ridx = 0;
    if (pos - flushed >= kFlush) flush4k();
  };
  // zlib header: deflate, 32 KB window at most, no preset dictionary, check bits
  const uint32_t cmf = getbits(b, 8), flg = getbits(b, 8);
  if ((cmf & 15u) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20u)) err = SLG_PNG_E_STREAM;
  bool last = false;
  while (!err && !last) {
    if (PNG_PROF) ++pf[kPfBlocks];
    const uint64_t pf_th = pf_now();
    last = getbits(b, 1) != 0;
    const uint32_t type = getbits(b, 2);
    if (type == 0) {                                         // stored block
      const int drop = b.cnt & 7;
      b.buf >>= drop;
      b.cnt -= drop;
      const uint32_t len = getbits(b, 16), nlen = getbits(b, 16);
      if ((len ^ 0xffffu) != nlen || pos + int32_t(len) > n_out) { err = SLG_PNG_E_STREAM; break; }
      for (uint32_t k = 0; k < len; ++k) {
        put(uint8_t(getbits(b, 8)));
      }
      continue;
    }
    if (type == 3) { err = SLG_PNG_E_STREAM; break; }
    int hlit = 288, hdist = 30;
    if (type == 1) {                                         // fixed codes
      for (int s = lane; s < 320; s += 64)
        L.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
      __syncthreads();
    } else {                                                 // dynamic codes
      hlit = int(getbits(b, 5)) + 257;
      hdist = int(getbits(b, 5)) + 1;
      const int hclen = int(getbits(b, 4)) + 4;
      if (hlit > 286 || hdist > 30) { err = SLG_PNG_E_STREAM; break; }
      uint32_t cl[19];
      for (int k = 0; k < 19; ++k) cl[k] = 0;
      for (int k = 0; k < hclen; ++k) {
        const uint32_t v = getbits(b, 3);
#pragma unroll
        for (int j = 0; j < 19; ++j) if (j == kClOrder[k]) cl[j] = v;
      }
      if (lane < 19) L.lens[lane] = uint8_t(cl[lane]);
      __syncthreads();
      if (!uni(build(L.dist, L.lens, 19, L.work))) { err = SLG_PNG_E_STREAM; break; }   // code-length code
      // the HLIT + HDIST code lengths (wave-uniform), written over the code-length code's own
      // lengths (no longer needed: its table is built) -- litlen at [0, hlit), distance at 288
      int i = 0;
      uint32_t prev = 0;
      while (i < hlit + hdist) {
        const int s = decode(b, L.dist);
        if (s < 0) { err = SLG_PNG_E_STREAM; break; }
        int rep = 1;
        uint32_t v = uint32_t(s);
        if (s == 16) {
          if (i == 0) { err = SLG_PNG_E_STREAM; break; }
          rep = 3 + int(getbits(b, 2));
          v = prev;
        } else if (s == 17) {
          rep = 3 + int(getbits(b, 3));
          v = 0;
        } else if (s == 18) {
          rep = 11 + int(getbits(b, 7));
          v = 0;
        }
        if (i + rep > hlit + hdist) { err = SLG_PNG_E_STREAM; break; }
        if (lane == 0)
          for (int k = i; k < i + rep; ++k) L.lens[k < hlit ? k : 288 + k - hlit] = uint8_t(v);
        i += rep;
        prev = v;
      }
      if (err) break;
      __syncthreads();
      if (L.lens[256] == 0) { err = SLG_PNG_E_STREAM; break; }
    }
    const uint64_t pf_tb = pf_now();
    if (!uni(build(L.lit, L.lens, hlit, L.work)) || !uni(build(L.dist, L.lens + 288, hdist, L.work))) {
      err = SLG_PNG_E_STREAM;
      break;
    }
    if (PNG_PROF) { pf[kPfBuild] += pf_now() - pf_tb; pf[kPfHeader] += pf_tb - pf_th; }
    build_lit4(L.lit4, L.lit);
    __syncthreads();
    for (;;) {                                               // the block's symbols
      refill(b);
      const LitEntry e4 = L.lit4[uint32_t(b.buf) & ((1u << kLitBits) - 1u)];
      const uint32_t cu = uni(uint32_t(e4 >> kLitCountShift));
      const uint32_t n4 = cu & 15u;
      if (n4) {                                              // a run of 1..kLitMax literals
        const uint32_t used = (cu >> 4) & 15u;
        b.buf >>= used;
        b.cnt -= int(used);
        if (pos + int32_t(n4) > n_out) { err = SLG_PNG_E_SIZE; break; }
#if PNG_LIT_WORD
        // lane 0 stores the run as one unaligned LDS word (bytes past the run land on positions
        // not yet written, or in the ring's 4 slack bytes); a run that wraps also writes its
        // wrapped bytes at the ring's start (rare)
        if (lane == 0 && !(PNG_ABL & 1)) {
          const uint32_t word = uint32_t(e4);
          __builtin_memcpy(&L.ring[ridx], &word, 4);
        }
        if (__builtin_expect(ridx + int(n4) > kRing, 0)) {   // (uniform: a scalar branch)
          __builtin_amdgcn_wave_barrier();
          if (lane < int(n4) && ridx + lane >= kRing) L.ring[ridx + lane - kRing] = uint8_t(uint32_t(e4) >> (8 * lane));
        }
#else
        if (lane < int(n4) && !(PNG_ABL & 1)) {              // lane k writes literal k
          int r = ridx + lane;
          if (r >= kRing) r -= kRing;
          L.ring[r] = uint8_t(uint32_t(e4) >> (8 * lane));
        }
#endif
        pos += int32_t(n4);
        ridx += int(n4);
        if (ridx >= kRing) ridx -= kRing;
        if (pos - flushed >= kFlush) flush4k();
        if (PNG_PROF) { pf[kPfLit] += n4; ++pf[kPfRuns]; }
        continue;
      }
      int s = decode(b, L.lit);
      if (s < 0) { err = SLG_PNG_E_STREAM; break; }
      if (s < 256) {
        if (pos >= n_out) { err = SLG_PNG_E_SIZE; break; }
        put(uint8_t(s));
        if (PNG_PROF) ++pf[kPfLit];
        continue;
      }
      if (s == 256) break;
      s -= 257;
      if (s >= 29) { err = SLG_PNG_E_STREAM; break; }
      const int len = int(len_base(uint32_t(s))) + int(getbits(b, int(len_extra(uint32_t(s)))));
      const int ds = decode(b, L.dist);
      if (ds < 0 || ds >= 30) { err = SLG_PNG_E_STREAM; break; }
      const int dist = int(dist_base(uint32_t(ds))) + int(getbits(b, int(dist_extra(uint32_t(ds)))));
      if (dist > pos) { err = SLG_PNG_E_STREAM; break; }
      if (pos + len > n_out) { err = SLG_PNG_E_SIZE; break; }
      __builtin_amdgcn_wave_barrier();
      const uint64_t pf_tc = pf_now();
      const int sbase = ridx >= dist ? ridx - dist : ridx - dist + kRing;
      for (int c = 0; c < ((PNG_ABL & 2) ? 0 : len); c += 64) {   // all lanes; 64 bytes per step
        const int i = c + lane;
        if (i < len) {
          int si = sbase + (dist >= 64 ? i : i % dist), di = ridx + i;
          if (si >= kRing) si -= kRing;
          if (di >= kRing) di -= kRing;
          L.ring[di] = L.ring[si];
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (PNG_PROF) { pf[kPfCopy] += pf_now() - pf_tc; ++pf[kPfMatch]; pf[kPfMatchBytes] += len; }
      pos += len;
      ridx += len;
      if (ridx >= kRing) ridx -= kRing;
      if (pos - flushed >= kFlush) flush4k();                // (len <= 258: at most one block)
    }
  }
  if (!err && pos != n_out) err = SLG_PNG_E_SIZE;
  if (!err && pos > flushed) flush_ring(L.ring, out, flushed, int(pos - flushed));
  uint32_t adler = 0;
  if (!err) {                                                // the trailer: next byte boundary
    const int64_t at = (bits_consumed(b) + 7) / 8;
    if (at + 4 > f.zlen) err = SLG_PNG_E_STREAM;
    else adler = (uint32_t(f.z[at]) << 24) | (uint32_t(f.z[at + 1]) << 16) | (uint32_t(f.z[at + 2]) << 8) | f.z[at + 3];
  }
  if (lane == 0) {
    status[2 * blockIdx.x] = err;
    status[2 * blockIdx.x + 1] = int32_t(adler);
  }
#if PNG_PROF
  pf[kPfTotal] = pf_now() - pf_t0;
  pf[kPfSymbols] = pf[kPfLit] + pf[kPfMatch];                // (literals, not lookups)
  if (lane == 0)
    for (int k = 0; k < kPfN; ++k) atomicAdd(&g_png_prof[k], (unsigned long long)pf[k]);
#endif
}

// Wavefront un-filter + Adler-32 check of one frame (status from png_inflate_kernel).
template <int BPP>
__device__ void unfilter_frame(const slg_png_frame& f, int32_t* st, uint8_t* lastrow) {
  const int lane = threadIdx.x;
  const int rb = f.width * BPP;                               // bytes per row (without filter byte)
  const int64_t n = int64_t(f.height) * (rb + 1);
  uint64_t A = 0, B = 0;
  int bad = 0;
  for (int y0 = 0; y0 < f.height; y0 += 64) {
    const int row = y0 + lane;
    const bool live = row < f.height;
    const int rows = f.height - y0 < 64 ? f.height - y0 : 64;
    const uint8_t* src = f.raw + int64_t(row) * (rb + 1);
    const int ft = live ? src[0] : 0;
    if (ft > 4) bad = 1;
    const uint64_t i0 = uint64_t(row) * uint64_t(rb + 1);
    if (live) { A += uint64_t(ft); B += uint64_t(n - int64_t(i0)) * uint64_t(ft); }
    uint8_t* dst = f.out + int64_t(row) * f.out_pitch;
    uint32_t ho[BPP], hu[BPP];                                // last BPP outputs / bytes above
#pragma unroll
    for (int k = 0; k < BPP; ++k) ho[k] = hu[k] = 0;
    uint32_t o_prev = 0;
    const int steps = rb + rows - 1;
    uint32_t sbuf[16], nbuf[16];
    auto load16 = [&](int t0, uint32_t (&v)[16]) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int x = t0 + k - lane;
        v[k] = (live && x >= 0 && x < rb) ? src[1 + x] : 0u;
      }
    };
    load16(0, sbuf);
    for (int t0 = 0; t0 < steps; t0 += 16) {
      load16(t0 + 16, nbuf);                                  // next 16 steps' bytes, in flight
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int t = t0 + k;
        const int x = t - lane;
        const uint32_t from_left_lane = uint32_t(__shfl_up(int(o_prev), 1));
        uint32_t up;
        if (lane == 0) up = (y0 > 0 && x >= 0 && x < rb) ? lastrow[x] : 0u;
        else up = from_left_lane;
        const bool act = live && x >= 0 && x < rb && t < steps;
        const uint32_t a = ho[BPP - 1], c = hu[BPP - 1];
        // every lane's own row filter, as selects (no divergent branch)
        const int db = int(up) - int(c), da = int(a) - int(c);
        const int pa = abs(db), pb = abs(da), pc = abs(db + da);
        const uint32_t paeth = (pa <= pb && pa <= pc) ? a : (pb <= pc ? up : c);
        uint32_t pred = ft == 1 ? a : 0u;
        pred = ft == 2 ? up : pred;
        pred = ft == 3 ? (a + up) >> 1 : pred;
        pred = ft == 4 ? paeth : pred;
        const uint32_t s = sbuf[k];
        const uint32_t o = (s + pred) & 255u;
        if (act) {
          dst[x] = uint8_t(o);
          if (lane == 63) lastrow[x] = uint8_t(o);
          A += s;
          B += uint64_t(n - int64_t(i0) - 1 - x) * s;
        }
#pragma unroll
        for (int q = BPP - 1; q > 0; --q) { ho[q] = ho[q - 1]; hu[q] = hu[q - 1]; }
        ho[0] = act ? o : 0u;
        hu[0] = act ? up : 0u;
        o_prev = act ? o : 0u;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) sbuf[k] = nbuf[k];
    }
    A %= kAdlerMod;
    B %= kAdlerMod;
    __syncthreads();                                          // lastrow complete for the next band
  }
  // wave sums of the lanes' Adler parts
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    A += uint64_t(__shfl_xor(int64_t(A), o));
    B += uint64_t(__shfl_xor(int64_t(B), o));
    bad |= __shfl_xor(bad, o);
  }
  const uint32_t a32 = uint32_t((1 + A) % kAdlerMod), b32 = uint32_t((B + uint64_t(n)) % kAdlerMod);
  if (lane == 0) {
    if (bad) st[0] = SLG_PNG_E_FILTER;
    else if (((b32 << 16) | a32) != uint32_t(st[1])) st[0] = SLG_PNG_E_ADLER;
  }
}

__global__ __launch_bounds__(64) void png_unfilter_kernel(const slg_png_frame* frames, int32_t* status) {
  const slg_png_frame f = frames[blockIdx.x];
  __shared__ uint8_t lastrow[kMaxRowBytes];                   // a band's last row, for the next band
  int32_t* st = status + 2 * blockIdx.x;
  if (st[0] != 0) return;                                     // inflate failed: host decodes it
  if (int64_t(f.width) * f.channels > kMaxRowBytes) {         // (uniform) too wide for the LDS row
    if (threadIdx.x == 0) st[0] = SLG_PNG_E_UNSUPPORTED;
    return;
  }
  switch (f.channels) {
    case 1: unfilter_frame<1>(f, st, lastrow); break;
    case 2: unfilter_frame<2>(f, st, lastrow); break;
    case 3: unfilter_frame<3>(f, st, lastrow); break;
    default: unfilter_frame<4>(f, st, lastrow); break;
  }
}

}  // namespace

extern "C" {

int64_t slg_png_raw_bytes(int32_t width, int32_t height, int32_t channels) {
  if (width <= 0 || height <= 0 || channels < 1 || channels > 4) return -SLG_ERR_INVALID;
  return (int64_t(height) * (1 + int64_t(width) * channels) + 15) / 16 * 16;
}

// PNG_PROF builds only (not in include/slgpu.h): copy the counters out, optionally zero them.
#if PNG_PROF
int32_t slg_png_prof_read(uint64_t* out, int32_t reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_png_prof), sizeof(uint64_t) * kPfN) != hipSuccess) return SLG_ERR_HIP;
  if (reset) {
    static const uint64_t zero[kPfN] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_png_prof), zero, sizeof(zero)) != hipSuccess) return SLG_ERR_HIP;
  }
  return SLG_OK;
}
#endif

int32_t slg_png_decode_device(const slg_png_frame* frames, int32_t n, int32_t* status, void* stream) {
  if (n < 0 || (n > 0 && (!frames || !status))) return slg_internal_fail(SLG_ERR_INVALID, "slg_png_decode_device: bad argument");
  if (n == 0) return SLG_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(png_inflate_kernel, dim3(unsigned(n)), dim3(64), 0, s, frames, status);
  if (hipGetLastError() != hipSuccess) return slg_internal_fail(SLG_ERR_HIP, "png_inflate_kernel launch failed");
  hipLaunchKernelGGL(png_unfilter_kernel, dim3(unsigned(n)), dim3(64), 0, s, frames, status);
  if (hipGetLastError() != hipSuccess) return slg_internal_fail(SLG_ERR_HIP, "png_unfilter_kernel launch failed");
  return SLG_OK;
}

}  // extern "C"

extern "C" int32_t slg_stream_create_reserving(int32_t reserve_every, void** stream) {
  if (!stream || reserve_every < 2) return SLG_ERR_INVALID;
  int dev = 0, n_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1)
    return SLG_ERR_HIP;
  const int n_words = (n_cu + 31) / 32;
  uint32_t mask[64] = {};
  if (n_words > 64) return SLG_ERR_UNSUPPORTED;
  for (int cu = 0; cu < n_cu; ++cu)
    if (cu % reserve_every != reserve_every - 1) mask[cu / 32] |= 1u << (cu % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, uint32_t(n_words), mask) != hipSuccess) return SLG_ERR_HIP;
  *stream = s;
  return SLG_OK;
}

extern "C" int32_t slg_stream_destroy(void* stream) {
  return hipStreamDestroy(static_cast<hipStream_t>(stream)) == hipSuccess ? SLG_OK : SLG_ERR_HIP;
}
