// Host-side PNG fast path for the frame ingest of the hot path (server/processing.py:59-60,98-99:
// cv2.imread(f, 0) of every used frame).  Captures are 8-bit grayscale, non-interlaced PNGs:
// for them cv2.imread(f, 0) is the identity on the stored samples, so decoding is inflate +
// the five PNG row filters.  Anything else (colour, 16-bit, palette, interlaced, a bad CRC or
// a truncated stream) returns a non-zero status and the caller decodes it the general way
// (frames.py), so error behaviour stays that of the general decoder.
//
// Inflate uses libdeflate when the image has it (dlopen, ~2-3x zlib's speed), else zlib.
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include <emmintrin.h>

#include <mutex>
#include <vector>

namespace {

constexpr int kOk = 0, kInvalid = 1, kUnsupported = 3;

uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

bool read_file(const char* path, std::vector<uint8_t>& buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return false; }
  const long n = ftell(f);
  if (n < 0 || fseek(f, 0, SEEK_SET) != 0) { fclose(f); return false; }
  buf.resize(size_t(n));
  const bool ok = fread(buf.data(), 1, size_t(n), f) == size_t(n);
  fclose(f);
  return ok;
}

uint32_t chunk_crc(const uint8_t* p, size_t n);

struct Png {
  uint32_t w = 0, h = 0, ch = 1;
  std::vector<uint8_t> idat;                  // concatenated zlib stream
};

// Parse chunks of an 8-bit, non-interlaced PNG (compression 0, filter 0) whose colour type is in
// `types` (bit t set = colour type t accepted); png.ch = samples per pixel.
int parse_types(const std::vector<uint8_t>& b, Png& png, bool want_data, uint32_t types) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
  if (b.size() < 8 + 25 || memcmp(b.data(), sig, 8) != 0) return kInvalid;
  size_t o = 8;
  bool have_hdr = false, have_end = false;
  while (o + 12 <= b.size()) {
    const uint32_t len = be32(&b[o]);
    if (len > b.size() - o - 12) return kInvalid;
    const uint8_t* type = &b[o + 4];
    const uint8_t* data = &b[o + 8];
    const uint32_t crc = be32(&b[o + 8 + len]);
    const bool critical = !(type[0] & 0x20);
    if (critical && chunk_crc(type, size_t(len) + 4) != crc) return kInvalid;
    if (!memcmp(type, "IHDR", 4)) {
      if (len != 13) return kInvalid;
      png.w = be32(data);
      png.h = be32(data + 4);
      const uint8_t ct = data[9];
      if (data[8] != 8 || ct > 6 || !((types >> ct) & 1u) || data[10] != 0 || data[11] != 0 || data[12] != 0)
        return kUnsupported;
      png.ch = ct == 0 ? 1 : ct == 2 ? 3 : ct == 4 ? 2 : 4;
      if (png.w == 0 || png.h == 0 || png.w > (1u << 16) || png.h > (1u << 16)) return kUnsupported;
      have_hdr = true;
      if (!want_data) return kOk;
    } else if (!memcmp(type, "IDAT", 4)) {
      if (!have_hdr) return kInvalid;
      png.idat.insert(png.idat.end(), data, data + len);
    } else if (!memcmp(type, "IEND", 4)) {
      have_end = true;
      break;
    } else if (critical) {
      return kUnsupported;                     // PLTE etc.: not a capture this path decodes
    }
    o += 12 + size_t(len);
  }
  return have_hdr && have_end && !png.idat.empty() ? kOk : kInvalid;
}

// Only 8-bit grayscale (colour type 0).
int parse(const std::vector<uint8_t>& b, Png& png, bool want_data) { return parse_types(b, png, want_data, 1u); }

// libdeflate (optional): the three entry points of its stable public API.
using ld_alloc_t = void* (*)();
using ld_free_t = void (*)(void*);
using ld_zlib_t = int (*)(void*, const void*, size_t, void*, size_t, size_t*);
using ld_crc_t = uint32_t (*)(uint32_t, const void*, size_t);
struct Deflate {
  ld_alloc_t alloc = nullptr;
  ld_free_t free = nullptr;
  ld_zlib_t zlib = nullptr;
  ld_crc_t crc = nullptr;                      // carry-less-multiply CRC-32 (~10x zlib 1.2.11's)
};

const Deflate& deflate_lib() {
  static Deflate d;
  static std::once_flag once;
  std::call_once(once, [] {
    if (getenv("SLG_PNG_ZLIB")) return;      // A/B switch: force zlib
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    d.alloc = reinterpret_cast<ld_alloc_t>(dlsym(h, "libdeflate_alloc_decompressor"));
    d.free = reinterpret_cast<ld_free_t>(dlsym(h, "libdeflate_free_decompressor"));
    d.zlib = reinterpret_cast<ld_zlib_t>(dlsym(h, "libdeflate_zlib_decompress"));
    d.crc = reinterpret_cast<ld_crc_t>(dlsym(h, "libdeflate_crc32"));
    if (!d.alloc || !d.free || !d.zlib || !d.crc) d = Deflate{};
  });
  return d;
}

uint32_t chunk_crc(const uint8_t* p, size_t n) {
  const Deflate& d = deflate_lib();
  if (d.crc) return d.crc(0, p, n);
  return uint32_t(crc32(crc32(0L, Z_NULL, 0), p, uInt(n)));
}

bool inflate_all(const std::vector<uint8_t>& in, uint8_t* out, size_t n_out) {
  const Deflate& d = deflate_lib();
  if (d.zlib) {
    thread_local struct Dec {
      void* p = nullptr;
      ~Dec() { if (p) deflate_lib().free(p); }
    } dec;
    if (!dec.p) dec.p = d.alloc();
    if (dec.p) {
      size_t got = 0;
      // LIBDEFLATE_SUCCESS == 0; the stream must fill the buffer exactly
      return d.zlib(dec.p, in.data(), in.size(), out, n_out, &got) == 0 && got == n_out;
    }
  }
  z_stream s{};
  if (inflateInit(&s) != Z_OK) return false;
  s.next_in = const_cast<Bytef*>(in.data());
  s.avail_in = uInt(in.size());
  s.next_out = out;
  s.avail_out = uInt(n_out);
  const int rc = inflate(&s, Z_FINISH);
  const bool ok = rc == Z_STREAM_END && s.avail_out == 0;
  inflateEnd(&s);
  return ok;
}

inline int iabs(int x) { const int m = x >> 31; return (x ^ m) - m; }

inline int paeth(int a, int b, int c) {       // PNG spec §9.4, without branches: p - a = b - c,
  const int db = b - c, da = a - c;           // p - b = a - c, p - c = (b - c) + (a - c)
  const int pa = iabs(db), pb = iabs(da), pc = iabs(db + da);
  const int m_bc = -int(pb <= pc), m_a = -int((pa <= pb) & (pa <= pc));   // masks, not branches:
  const int bc = (b & m_bc) | (c & ~m_bc);                                 // the choice is data-
  return (a & m_a) | (bc & ~m_a);                                          // random per pixel
}

// Sub filter of one row: out[x] = s[x] + out[x - 1] (mod 256), a byte-wise prefix sum -- 16
// bytes per step (log-step shifts within the vector, then the carry of the previous block).
void unfilter_sub(const uint8_t* __restrict s, uint8_t* __restrict d, uint32_t w) {
  uint32_t x = 0;
  __m128i carry = _mm_setzero_si128();
  for (; x + 16 <= w; x += 16) {
    __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + x));
    v = _mm_add_epi8(v, _mm_slli_si128(v, 1));
    v = _mm_add_epi8(v, _mm_slli_si128(v, 2));
    v = _mm_add_epi8(v, _mm_slli_si128(v, 4));
    v = _mm_add_epi8(v, _mm_slli_si128(v, 8));
    v = _mm_add_epi8(v, carry);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(d + x), v);
    carry = _mm_set1_epi8(char(d[x + 15]));
  }
  uint8_t a = x ? d[x - 1] : 0;
  for (; x < w; ++x) d[x] = a = uint8_t(s[x] + a);
}

// Undo the row filters (1 byte per pixel) from raw [h][1 + w] into out [h][w].
bool unfilter(const uint8_t* raw, uint8_t* out, uint32_t w, uint32_t h) {
  for (uint32_t y = 0; y < h; ++y) {
    const uint8_t* __restrict s = raw + size_t(y) * (w + 1);
    uint8_t* __restrict d = out + size_t(y) * w;
    const uint8_t* __restrict up = y ? d - w : nullptr;
    const uint8_t f = s[0];
    ++s;
    switch (f) {
      case 0: memcpy(d, s, w); break;
      case 1: unfilter_sub(s, d, w); break;
      case 2:
        if (up) for (uint32_t x = 0; x < w; ++x) d[x] = uint8_t(s[x] + up[x]);
        else memcpy(d, s, w);
        break;
      case 3: {
        int a = 0;
        for (uint32_t x = 0; x < w; ++x) {
          const int b = up ? up[x] : 0;
          d[x] = uint8_t(s[x] + ((a + b) >> 1));
          a = d[x];
        }
        break;
      }
      case 4: {
        if (!up) { unfilter_sub(s, d, w); break; }     // no prior row: Paeth predicts a (= Sub)
        int a = 0, c = 0;
        for (uint32_t x = 0; x < w; ++x) {
          const int b = up[x];
          d[x] = uint8_t(s[x] + paeth(a, b, c));
          a = d[x];
          c = b;
        }
        break;
      }
      default: return false;
    }
  }
  return true;
}

}  // namespace

extern "C" {

// Size of an 8-bit grayscale, non-interlaced PNG: 0 and (*width, *height), else non-zero
// (not such a PNG or unreadable: decode it the general way).
int32_t slg_png_gray8_size(const char* path, int32_t* width, int32_t* height) {
  if (!path || !width || !height) return kInvalid;
  std::vector<uint8_t> b;
  if (!read_file(path, b)) return kInvalid;
  Png png;
  const int rc = parse(b, png, false);
  if (rc) return rc;
  *width = int32_t(png.w);
  *height = int32_t(png.h);
  return kOk;
}

// Decode it into out[height][width] (capacity `cap` bytes): 0 on success, else non-zero and
// `out` unspecified.  Thread-safe; meant to run on a host decode pool (ctypes drops the GIL).
int32_t slg_png_gray8_decode(const char* path, uint8_t* out, int64_t cap, int32_t width, int32_t height) {
  if (!path || !out) return kInvalid;
  // the file, its zlib stream and the filtered rows in buffers the decode thread keeps: a frame
  // is ~1 MB + 1 MB + 2 MB, and fresh ones per frame cost page faults and a 2 MB zero fill
  thread_local std::vector<uint8_t> b, raw;
  thread_local Png png;
  if (!read_file(path, b)) return kInvalid;
  png.idat.clear();
  int rc = parse(b, png, true);
  if (rc) return rc;
  if (int32_t(png.w) != width || int32_t(png.h) != height || cap < int64_t(png.w) * png.h) return kInvalid;
  if (raw.size() < size_t(png.h) * (png.w + 1)) raw.resize(size_t(png.h) * (png.w + 1));
  if (!inflate_all(png.idat, raw.data(), size_t(png.h) * (png.w + 1))) return kInvalid;
  return unfilter(raw.data(), out, png.w, png.h) ? kOk : kInvalid;
}

// The zlib stream of an 8-bit gray / gray+alpha / RGB / RGBA PNG for the device decoder
// (include/slgpu.h): the concatenated IDAT payload, 8 zero bytes of read-ahead padding after it.
int32_t slg_png_zstream(const char* path, uint8_t* buf, int64_t cap, int32_t* info) {
  if (!path || !buf || !info) return kInvalid;
  std::vector<uint8_t> b;
  if (!read_file(path, b)) return kInvalid;
  Png png;
  const int rc = parse_types(b, png, true, (1u << 0) | (1u << 2) | (1u << 4) | (1u << 6));
  if (rc) return rc;
  const int64_t n = int64_t(png.idat.size());
  if (cap < n + 8) return kInvalid;
  memcpy(buf, png.idat.data(), size_t(n));
  memset(buf + n, 0, 8);
  info[0] = int32_t(png.w);
  info[1] = int32_t(png.h);
  info[2] = int32_t(png.ch);
  info[3] = int32_t(n);
  return kOk;
}

}  // extern "C"
