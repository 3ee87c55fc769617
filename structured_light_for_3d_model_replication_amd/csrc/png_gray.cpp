// Host-side PNG decode for the frame ingest of the hot path (server/processing.py:59-60,98-99,124:
// cv2.imread(f, 0) of every used frame, cv2.imread(files[0]) for the texture).
//
// * slg_png_gray8_*: the fast path for 8-bit grayscale, non-interlaced captures (what the
//   reference's scanner writes), where cv2.imread(f, 0) is the identity on the stored samples:
//   inflate + the five row filters.
// * slg_png_read: every other PNG, decoded to what OpenCV's PNG decoder returns for it.  OpenCV
//   (modules/imgcodecs/src/grfmt_png.cpp, PngDecoder::readData, 4.x) hands the file to libpng
//   with png_set_strip_16, png_set_strip_alpha, png_set_palette_to_rgb,
//   png_set_expand_gray_1_2_4_to_8 and then png_set_bgr (colour read), png_set_gray_to_rgb
//   (gray file, colour read) or png_set_rgb_to_gray(png, 1, 0.299, 0.587) (colour file, gray
//   read).  Those libpng 1.6.37 transformations are restated here (png.c / pngrtran.c:
//   png_set_rgb_to_gray_fixed's 15-bit coefficients 9797 / 19234 / 3737, png_do_rgb_to_gray's
//   truncating 8-bit and rounding 16-bit sums, and -- when the file's gAMA / sRGB gamma is
//   significant -- png_build_gamma_table's 8-bit tables and its 16-bit tables at gamma_shift
//   max(16 - sBIT, 5)) and pinned byte for byte to the system libpng driven with OpenCV's calls
//   (tests/png_ref.py, tests/test_png_color.py).  Files whose colour handling libpng decides from
//   data not restated here -- an iCCP profile (libpng recognises some sRGB profiles by checksum),
//   duplicate or invalid gAMA / sRGB chunks, a gAMA that disagrees with sRGB -- are decoded by
//   the system libpng itself (dlopen, the same calls), when it is there.
//
// Inflate uses libdeflate when the image has it (dlopen, ~2-3x zlib's speed), else zlib.
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include <emmintrin.h>
#include <math.h>
#include <setjmp.h>

#include <algorithm>
#include <type_traits>

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
  bool color_chunks = false;                  // gAMA / sRGB / iCCP before the image data
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
    } else if (!memcmp(type, "gAMA", 4) || !memcmp(type, "sRGB", 4) || !memcmp(type, "iCCP", 4)) {
      png.color_chunks = png.color_chunks || png.idat.empty();
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

// ------------------------------------------------------------------ slg_png_read: any PNG
// Chunks and layout of any PNG (PNG 1.2 / ISO 15948) with what libpng's colour handling depends
// on: the gAMA / sRGB / iCCP / sBIT chunks that come before PLTE and IDAT (libpng ignores them
// afterwards, png_handle_gAMA & co.).
struct PngMeta {
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = 0, interlace = 0, ch = 1;
  std::vector<uint8_t> plte;                 // palette RGB triples (colour type 3)
  std::vector<uint8_t> idat;
  int n_gama = 0, n_srgb = 0, n_iccp = 0;
  bool gama_bad = false, srgb_bad = false;   // a chunk libpng rejects (length, range, intent)
  uint32_t gama = 0;
  bool sbit_ok = false;
  uint8_t sbit[4] = {0, 0, 0, 0};
  bool odd = false;                          // anything else this decoder leaves to libpng
};

int parse_meta(const std::vector<uint8_t>& b, PngMeta& m) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
  if (b.size() < 8 + 25 || memcmp(b.data(), sig, 8) != 0) return kInvalid;
  size_t o = 8;
  bool have_hdr = false, have_end = false, seen_plte = false;
  while (o + 12 <= b.size()) {
    const uint32_t len = be32(&b[o]);
    if (len > b.size() - o - 12) return kInvalid;
    const uint8_t* type = &b[o + 4];
    const uint8_t* data = &b[o + 8];
    const uint32_t crc = be32(&b[o + 8 + len]);
    const bool critical = !(type[0] & 0x20);
    const bool crc_ok = chunk_crc(type, size_t(len) + 4) == crc;
    o += 12 + size_t(len);
    if (!crc_ok) {
      if (critical) return kInvalid;
      m.odd = true;                          // libpng warns and drops it
      continue;
    }
    const bool early = have_hdr && !seen_plte && m.idat.empty();
    if (!memcmp(type, "IHDR", 4)) {
      if (len != 13 || have_hdr) return kInvalid;
      m.w = be32(data);
      m.h = be32(data + 4);
      m.depth = data[8];
      m.ctype = data[9];
      m.interlace = data[12];
      const int d = m.depth, c = m.ctype;
      const bool ok_depth = (c == 0 && (d == 1 || d == 2 || d == 4 || d == 8 || d == 16)) ||
                            (c == 3 && (d == 1 || d == 2 || d == 4 || d == 8)) ||
                            ((c == 2 || c == 4 || c == 6) && (d == 8 || d == 16));
      if (!ok_depth || data[10] != 0 || data[11] != 0 || m.interlace > 1) return kUnsupported;
      m.ch = c == 0 ? 1 : c == 2 ? 3 : c == 3 ? 1 : c == 4 ? 2 : 4;
      if (m.w == 0 || m.h == 0 || m.w > 65535 || m.h > 65535) return kUnsupported;
      have_hdr = true;
    } else if (!have_hdr) {
      return kInvalid;
    } else if (!memcmp(type, "PLTE", 4)) {
      if (seen_plte || !m.idat.empty() || len % 3 || len == 0 || len > 768) {
        if (m.ctype == 3) return kInvalid;
        m.odd = true;
      } else if (m.ctype == 3) {
        m.plte.assign(data, data + len);
      }
      seen_plte = true;
    } else if (!memcmp(type, "IDAT", 4)) {
      m.idat.insert(m.idat.end(), data, data + len);
    } else if (!memcmp(type, "IEND", 4)) {
      have_end = true;
      break;
    } else if (!memcmp(type, "gAMA", 4)) {
      if (!early) continue;
      ++m.n_gama;
      if (len != 4) { m.gama_bad = true; continue; }
      m.gama = be32(data);
      if (m.gama < 16 || m.gama > 625000000u) m.gama_bad = true;
    } else if (!memcmp(type, "sRGB", 4)) {
      if (!early) continue;
      ++m.n_srgb;
      if (len != 1 || data[0] > 3) m.srgb_bad = true;
    } else if (!memcmp(type, "iCCP", 4)) {
      if (early) ++m.n_iccp;
    } else if (!memcmp(type, "sBIT", 4)) {
      if (!early) continue;
      const int n = m.ctype == 3 ? 3 : m.ctype == 0 ? 1 : m.ctype == 4 ? 2 : m.ctype == 2 ? 3 : 4;
      const int sd = m.ctype == 3 ? 8 : m.depth;
      bool ok = int(len) == n && !m.sbit_ok;
      for (int i = 0; ok && i < n; ++i) ok = data[i] >= 1 && data[i] <= sd;
      if (ok) { m.sbit_ok = true; memcpy(m.sbit, data, size_t(n)); }
      else m.odd = true;
    } else if (critical) {
      return kUnsupported;
    }
  }
  if (!have_hdr || !have_end || m.idat.empty()) return kInvalid;
  if (m.ctype == 3 && m.plte.empty()) return kInvalid;
  return kOk;
}

// ---- libpng 1.6.37's gamma arithmetic (png.c), floating-point build, restated
constexpr int32_t kFp1 = 100000;
bool gamma_significant(int64_t g) { return g < kFp1 - 5000 || g > kFp1 + 5000; }   // PNG_GAMMA_THRESHOLD_FIXED
int32_t fp_reciprocal(int64_t a) {                                                    // png_reciprocal
  const double r = floor(1E10 / double(a) + .5);
  return (r <= 2147483647. && r >= -2147483648.) ? int32_t(r) : 0;
}
int32_t fp_reciprocal2(int64_t a, int64_t b) {                                        // png_reciprocal2
  double r = 1E15 / double(a);
  r /= double(b);
  r = floor(r + .5);
  return (r <= 2147483647. && r >= -2147483648.) ? int32_t(r) : 0;
}
int32_t fp_product2(int64_t a, int64_t b) {                                           // png_product2
  double r = double(a) * 1E-5;
  r *= double(b);
  r = floor(r + .5);
  return (r <= 2147483647. && r >= -2147483648.) ? int32_t(r) : 0;
}
uint8_t gamma_8bit_correct(unsigned v, int32_t g) {
  if (v > 0 && v < 255) return uint8_t(floor(255 * pow(int(v) / 255., g * .00001) + .5));
  return uint8_t(v);
}
uint16_t gamma_16bit_correct(unsigned v, int32_t g) {
  if (v > 0 && v < 65535) return uint16_t(floor(65535 * pow(int32_t(v) / 65535., g * .00001) + .5));
  return uint16_t(v);
}
void build_8bit_table(uint8_t* t, int32_t g) {                                        // png_build_8bit_table
  for (unsigned i = 0; i < 256; ++i) t[i] = gamma_significant(g) ? gamma_8bit_correct(i, g) : uint8_t(i);
}
// [i][j] flattened as t[i * 256 + j], i < 1 << (8 - shift): png_build_16bit_table
void build_16bit_table(std::vector<uint16_t>& t, unsigned shift, int32_t g) {
  const unsigned num = 1u << (8u - shift), max = (1u << (16u - shift)) - 1u, max_by_2 = 1u << (15u - shift);
  const double fmax = 1.0 / double((int32_t(1) << (16u - shift)) - 1);
  t.assign(size_t(num) * 256, 0);
  for (unsigned i = 0; i < num; ++i)
    for (unsigned j = 0; j < 256; ++j) {
      const uint32_t ig = (j << (8 - shift)) + i;
      t[i * 256 + j] = gamma_significant(g) ? uint16_t(floor(65535. * pow(ig * fmax, g * .00001) + .5))
                                            : uint16_t((shift ? (ig * 65535u + max_by_2) / max : ig));
    }
}
void build_16to8_table(std::vector<uint16_t>& t, unsigned shift, int32_t g) {        // png_build_16to8_table
  const unsigned num = 1u << (8u - shift), max = (1u << (16u - shift)) - 1u;
  t.assign(size_t(num) * 256, 0);
  uint32_t last = 0;
  for (unsigned i = 0; i < 255; ++i) {
    const uint16_t out = uint16_t(i * 257u);
    uint32_t bound = gamma_16bit_correct(out + 128u, g);
    bound = (bound * max + 32768u) / 65535u + 1u;
    while (last < bound) {
      t[(last & (0xffu >> shift)) * 256 + (last >> (8u - shift))] = out;
      ++last;
    }
  }
  while (last < (num << 8)) {
    t[(last & (0xffu >> shift)) * 256 + (last >> (8u - shift))] = 65535u;
    ++last;
  }
}

// png_set_rgb_to_gray_fixed(png, 1, png_fixed(0.299), png_fixed(0.587)): 15-bit coefficients
constexpr uint32_t kRc = uint32_t((uint32_t(29900) * 32768u) / 100000u);   // 9797
constexpr uint32_t kGc = uint32_t((uint32_t(58700) * 32768u) / 100000u);   // 19234
constexpr uint32_t kBc = 32768u - kRc - kGc;                               // 3737

// The colour-to-gray conversion of one file (png_init_read_transformations + png_do_rgb_to_gray)
struct GrayConv {
  bool tables = false;                       // the gamma path (png_build_gamma_table ran)
  uint8_t g8[256], to1[256], from1[256];     // gamma_table, gamma_to_1, gamma_from_1
  unsigned shift = 0;                        // gamma_shift (16-bit files)
  std::vector<uint16_t> g16, to1_16, from1_16;

  void init(const PngMeta& m, int32_t file_gamma) {
    // png_init_read_transformations: an unset file gamma is 1.0 and the screen gamma its inverse
    tables = false;
    if (file_gamma == 0) return;
    const int32_t screen = fp_reciprocal(file_gamma);
    if (!gamma_significant(file_gamma) && !gamma_significant(screen)) return;
    tables = true;
    if (m.depth <= 8) {
      build_8bit_table(g8, screen > 0 ? fp_reciprocal2(file_gamma, screen) : kFp1);
      build_8bit_table(to1, fp_reciprocal(file_gamma));
      build_8bit_table(from1, screen > 0 ? fp_reciprocal(screen) : file_gamma);
    } else {
      unsigned sig = 0;
      if (m.sbit_ok) sig = m.ctype & 2 ? std::max(m.sbit[0], std::max(m.sbit[1], m.sbit[2])) : m.sbit[0];
      shift = (sig > 0 && sig < 16u) ? 16u - sig : 0u;
      if (shift < 16u - 11u) shift = 16u - 11u;          // PNG_16_TO_8 (png_set_strip_16): PNG_MAX_GAMMA_8 = 11
      if (shift > 8u) shift = 8u;
      build_16to8_table(g16, shift, screen > 0 ? fp_product2(file_gamma, screen) : kFp1);
      build_16bit_table(to1_16, shift, fp_reciprocal(file_gamma));
      build_16bit_table(from1_16, shift, screen > 0 ? fp_reciprocal(screen) : file_gamma);
    }
  }
  uint8_t gray8(uint32_t r, uint32_t g, uint32_t b) const {
    if (r == g && r == b) return tables ? g8[r] : uint8_t(r);
    if (!tables) return uint8_t((kRc * r + kGc * g + kBc * b) >> 15);          // truncates (libpng)
    return from1[(kRc * to1[r] + kGc * to1[g] + kBc * to1[b] + 16384u) >> 15];
  }
  uint16_t lk(const std::vector<uint16_t>& t, uint32_t v) const { return t[((v & 0xffu) >> shift) * 256 + (v >> 8)]; }
  uint8_t gray16(uint32_t r, uint32_t g, uint32_t b) const {                    // then png_do_chop
    uint32_t w;
    if (r == g && r == b) {
      w = tables ? lk(g16, r) : r;
    } else if (!tables) {
      w = (kRc * r + kGc * g + kBc * b + 16384u) >> 15;
    } else {
      const uint32_t g1 = (kRc * lk(to1_16, r) + kGc * lk(to1_16, g) + kBc * lk(to1_16, b) + 16384u) >> 15;
      w = lk(from1_16, g1);
    }
    return uint8_t(w >> 8);
  }
};

// Whether this decoder restates libpng's colour handling for the file, and the file gamma it
// uses (0: none).  A gray file's colour chunks never matter (no colour transform runs).
bool restated_gamma(const PngMeta& m, int32_t* gamma) {
  *gamma = 0;
  if (!(m.ctype & 2)) return !m.odd;
  if (m.odd || m.n_iccp || m.gama_bad || m.srgb_bad || m.n_gama > 1 || m.n_srgb > 1) return false;
  if (m.n_srgb == 1) {
    *gamma = 45455;                                   // PNG_GAMMA_sRGB_INVERSE
    if (m.n_gama == 1) {                              // png_colorspace_check_gamma: they must agree
      const double a = floor(45455.0 * kFp1 / double(m.gama) + .5), b = floor(double(m.gama) * kFp1 / 45455.0 + .5);
      if (gamma_significant(int64_t(a)) || gamma_significant(int64_t(b))) return false;
    }
  } else if (m.n_gama == 1) {
    *gamma = int32_t(m.gama);
  }
  return true;
}

size_t row_bytes(uint32_t w, int ch, int depth) { return (size_t(w) * ch * depth + 7) / 8; }

// Generic PNG row un-filter, bpp bytes per complete pixel (>= 1).
bool unfilter_row(uint8_t f, const uint8_t* s, const uint8_t* up, uint8_t* d, size_t n, size_t bpp) {
  switch (f) {
    case 0: memcpy(d, s, n); return true;
    case 1:
      for (size_t x = 0; x < n; ++x) d[x] = uint8_t(s[x] + (x >= bpp ? d[x - bpp] : 0));
      return true;
    case 2:
      for (size_t x = 0; x < n; ++x) d[x] = uint8_t(s[x] + (up ? up[x] : 0));
      return true;
    case 3:
      for (size_t x = 0; x < n; ++x) d[x] = uint8_t(s[x] + (((x >= bpp ? d[x - bpp] : 0) + (up ? up[x] : 0)) >> 1));
      return true;
    case 4:
      for (size_t x = 0; x < n; ++x) {
        const int a = x >= bpp ? d[x - bpp] : 0, b = up ? up[x] : 0, c = (up && x >= bpp) ? up[x - bpp] : 0;
        d[x] = uint8_t(s[x] + paeth(a, b, c));
      }
      return true;
    default: return false;
  }
}

// Stored row of pw pixels -> canonical samples: 16-bit files keep their big-endian pairs, gray
// below 8 bits is expanded (png_set_expand_gray_1_2_4_to_8: x 255 / 85 / 17), palette indices
// become the PLTE colours (png_set_palette_to_rgb; an index past the palette reads 0, libpng's
// zero-filled 256-entry palette), everything else stays as stored.
void canon_row(const PngMeta& m, const uint8_t* src, uint32_t pw, uint8_t* dst) {
  if (m.depth >= 8 && m.ctype != 3) {
    memcpy(dst, src, size_t(pw) * m.ch * (m.depth / 8));
    return;
  }
  const int d = m.depth;
  const unsigned mask = (1u << d) - 1u, per = 8u / unsigned(d);
  for (uint32_t x = 0; x < pw; ++x) {
    const unsigned v = d == 8 ? src[x] : (src[x / per] >> (8 - d * (x % per + 1))) & mask;
    if (m.ctype == 3) {
      const size_t k = size_t(v) * 3;
      const bool in = k + 2 < m.plte.size();
      dst[3 * x] = in ? m.plte[k] : 0;
      dst[3 * x + 1] = in ? m.plte[k + 1] : 0;
      dst[3 * x + 2] = in ? m.plte[k + 2] : 0;
    } else {
      dst[x] = uint8_t(v * (255u / mask));
    }
  }
}

// Canonical row -> OpenCV's outputs (gray [w] and / or bgr [w][3]).
void out_row(const PngMeta& m, const GrayConv& gc, const uint8_t* c, uint32_t w, uint8_t* gray, uint8_t* bgr) {
  const bool color = m.ctype & 2;
  const int cch = m.ctype == 3 ? 3 : m.ch;                 // canonical channels
  if (m.depth == 16) {
    for (uint32_t x = 0; x < w; ++x) {
      const uint8_t* p = c + size_t(x) * cch * 2;
      if (color) {
        const uint32_t r = (uint32_t(p[0]) << 8) | p[1], g = (uint32_t(p[2]) << 8) | p[3], b = (uint32_t(p[4]) << 8) | p[5];
        if (gray) gray[x] = gc.gray16(r, g, b);
        if (bgr) { bgr[3 * x] = p[4]; bgr[3 * x + 1] = p[2]; bgr[3 * x + 2] = p[0]; }
      } else {
        if (gray) gray[x] = p[0];
        if (bgr) bgr[3 * x] = bgr[3 * x + 1] = bgr[3 * x + 2] = p[0];
      }
    }
    return;
  }
  for (uint32_t x = 0; x < w; ++x) {
    const uint8_t* p = c + size_t(x) * cch;
    if (color) {
      if (gray) gray[x] = gc.gray8(p[0], p[1], p[2]);
      if (bgr) { bgr[3 * x] = p[2]; bgr[3 * x + 1] = p[1]; bgr[3 * x + 2] = p[0]; }
    } else {
      if (gray) gray[x] = p[0];
      if (bgr) bgr[3 * x] = bgr[3 * x + 1] = bgr[3 * x + 2] = p[0];
    }
  }
}

// Inflate + un-filter (Adam7 passes when interlaced) into canonical rows, then the outputs.
int decode_general(const PngMeta& m, const GrayConv& gc, uint8_t* gray, uint8_t* bgr) {
  static const int kAdam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                   {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
  const int passes = m.interlace ? 7 : 1;
  const size_t bpp = std::max<size_t>(1, size_t(m.ch) * m.depth / 8);
  const int cch = m.ctype == 3 ? 3 : m.ch;
  const size_t canon_px = size_t(cch) * (m.depth == 16 ? 2 : 1);
  size_t total = 0;
  for (int p = 0; p < passes; ++p) {
    const uint32_t x0 = m.interlace ? kAdam7[p][0] : 0, y0 = m.interlace ? kAdam7[p][1] : 0;
    const uint32_t dx = m.interlace ? kAdam7[p][2] : 1, dy = m.interlace ? kAdam7[p][3] : 1;
    const uint32_t pw = m.w > x0 ? (m.w - x0 + dx - 1) / dx : 0, ph = m.h > y0 ? (m.h - y0 + dy - 1) / dy : 0;
    if (pw && ph) total += size_t(ph) * (1 + row_bytes(pw, m.ch, m.depth));
  }
  thread_local std::vector<uint8_t> raw, rows, canon, full;
  if (raw.size() < total) raw.resize(total);
  if (!inflate_all(m.idat, raw.data(), total)) return kInvalid;
  const size_t rb_max = row_bytes(m.w, m.ch, m.depth);
  if (rows.size() < 2 * rb_max) rows.resize(2 * rb_max);
  if (canon.size() < size_t(m.w) * canon_px) canon.resize(size_t(m.w) * canon_px);
  if (m.interlace && full.size() < size_t(m.h) * m.w * canon_px) full.resize(size_t(m.h) * m.w * canon_px);
  size_t at = 0;
  for (int p = 0; p < passes; ++p) {
    const uint32_t x0 = m.interlace ? kAdam7[p][0] : 0, y0 = m.interlace ? kAdam7[p][1] : 0;
    const uint32_t dx = m.interlace ? kAdam7[p][2] : 1, dy = m.interlace ? kAdam7[p][3] : 1;
    const uint32_t pw = m.w > x0 ? (m.w - x0 + dx - 1) / dx : 0, ph = m.h > y0 ? (m.h - y0 + dy - 1) / dy : 0;
    if (!pw || !ph) continue;
    const size_t rb = row_bytes(pw, m.ch, m.depth);
    uint8_t* cur = rows.data();
    uint8_t* prev = rows.data() + rb_max;
    for (uint32_t r = 0; r < ph; ++r) {
      const uint8_t* s = raw.data() + at;
      at += 1 + rb;
      if (!unfilter_row(s[0], s + 1, r ? prev : nullptr, cur, rb, bpp)) return kInvalid;
      const uint32_t y = y0 + r * dy;
      if (!m.interlace) {
        canon_row(m, cur, pw, canon.data());
        out_row(m, gc, canon.data(), m.w, gray ? gray + size_t(y) * m.w : nullptr,
                bgr ? bgr + size_t(y) * m.w * 3 : nullptr);
      } else {
        canon_row(m, cur, pw, canon.data());
        uint8_t* fr = full.data() + size_t(y) * m.w * canon_px;
        for (uint32_t k = 0; k < pw; ++k)
          memcpy(fr + size_t(x0 + k * dx) * canon_px, canon.data() + size_t(k) * canon_px, canon_px);
      }
      std::swap(cur, prev);
    }
  }
  if (m.interlace)
    for (uint32_t y = 0; y < m.h; ++y)
      out_row(m, gc, full.data() + size_t(y) * m.w * canon_px, m.w, gray ? gray + size_t(y) * m.w : nullptr,
              bgr ? bgr + size_t(y) * m.w * 3 : nullptr);
  return kOk;
}

// ---- the system libpng, for the files the restatement leaves to it (dlopen; OpenCV's calls)
struct LibPng {
  void* h = nullptr;
  typedef void (*err_fn)(void*, const char*);
  const char* (*get_libpng_ver)(void*) = nullptr;
  void* (*create_read_struct)(const char*, void*, err_fn, err_fn) = nullptr;
  void* (*create_info_struct)(void*) = nullptr;
  void (*destroy_read_struct)(void**, void**, void**) = nullptr;
  void* (*set_longjmp_fn)(void*, void (*)(jmp_buf, int), size_t) = nullptr;
  void (*set_read_fn)(void*, void*, void (*)(void*, uint8_t*, size_t)) = nullptr;
  void* (*get_io_ptr)(void*) = nullptr;
  void (*read_info)(void*, void*) = nullptr;
  uint32_t (*get_IHDR)(void*, void*, uint32_t*, uint32_t*, int*, int*, int*, int*, int*) = nullptr;
  void (*set_strip_16)(void*) = nullptr;
  void (*set_strip_alpha)(void*) = nullptr;
  void (*set_palette_to_rgb)(void*) = nullptr;
  void (*set_expand_gray_1_2_4_to_8)(void*) = nullptr;
  void (*set_bgr)(void*) = nullptr;
  void (*set_gray_to_rgb)(void*) = nullptr;
  void (*set_rgb_to_gray)(void*, int, double, double) = nullptr;
  int (*set_interlace_handling)(void*) = nullptr;
  void (*read_update_info)(void*, void*) = nullptr;
  size_t (*get_rowbytes)(void*, void*) = nullptr;
  void (*read_image)(void*, uint8_t**) = nullptr;
  void (*read_end)(void*, void*) = nullptr;
};

const LibPng* libpng() {
  static LibPng L;
  static bool ok = false;
  static std::once_flag once;
  std::call_once(once, [] {
    if (getenv("SLG_NO_LIBPNG")) return;                 // (tests: the restatement alone)
    void* h = dlopen("libpng16.so.16", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    bool all = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      all = all && f;
    };
    sym(L.get_libpng_ver, "png_get_libpng_ver");
    sym(L.create_read_struct, "png_create_read_struct");
    sym(L.create_info_struct, "png_create_info_struct");
    sym(L.destroy_read_struct, "png_destroy_read_struct");
    sym(L.set_longjmp_fn, "png_set_longjmp_fn");
    sym(L.set_read_fn, "png_set_read_fn");
    sym(L.get_io_ptr, "png_get_io_ptr");
    sym(L.read_info, "png_read_info");
    sym(L.get_IHDR, "png_get_IHDR");
    sym(L.set_strip_16, "png_set_strip_16");
    sym(L.set_strip_alpha, "png_set_strip_alpha");
    sym(L.set_palette_to_rgb, "png_set_palette_to_rgb");
    sym(L.set_expand_gray_1_2_4_to_8, "png_set_expand_gray_1_2_4_to_8");
    sym(L.set_bgr, "png_set_bgr");
    sym(L.set_gray_to_rgb, "png_set_gray_to_rgb");
    sym(L.set_rgb_to_gray, "png_set_rgb_to_gray");
    sym(L.set_interlace_handling, "png_set_interlace_handling");
    sym(L.read_update_info, "png_read_update_info");
    sym(L.get_rowbytes, "png_get_rowbytes");
    sym(L.read_image, "png_read_image");
    sym(L.read_end, "png_read_end");
    if (!all) return;
    L.h = h;
    ok = true;
  });
  return ok ? &L : nullptr;
}

struct MemReader {
  const std::vector<uint8_t>* b;
  size_t at;
};
void mem_read(void* png, uint8_t* out, size_t n);
void silent_warning(void*, const char*) {}

// cv2.imread(f, color ? IMREAD_COLOR : IMREAD_GRAYSCALE) through libpng itself; out [h][w][1|3].
int libpng_read(const LibPng& L, const std::vector<uint8_t>& file, bool color, uint8_t* out, uint32_t w,
                uint32_t h) {
  void* png = L.create_read_struct(L.get_libpng_ver(nullptr), nullptr, nullptr, silent_warning);
  if (!png) return kInvalid;
  void* info = L.create_info_struct(png);
  MemReader rd{&file, 0};
  std::vector<uint8_t*> rows(h);
  jmp_buf* jb = static_cast<jmp_buf*>(L.set_longjmp_fn(png, longjmp, sizeof(jmp_buf)));
  if (!info || !jb || setjmp(*jb)) {                     // libpng errors land here
    L.destroy_read_struct(&png, info ? &info : nullptr, nullptr);
    return kInvalid;
  }
  L.set_read_fn(png, &rd, mem_read);
  L.read_info(png, info);
  uint32_t fw = 0, fh = 0;
  int depth = 0, ctype = 0, inter = 0, comp = 0, filt = 0;
  L.get_IHDR(png, info, &fw, &fh, &depth, &ctype, &inter, &comp, &filt);
  if (fw != w || fh != h) {
    L.destroy_read_struct(&png, &info, nullptr);
    return kInvalid;
  }
  const bool is_color = ctype & 2;
  if (depth == 16) L.set_strip_16(png);
  L.set_strip_alpha(png);
  if (ctype == 3) L.set_palette_to_rgb(png);
  if (!is_color && depth < 8) L.set_expand_gray_1_2_4_to_8(png);
  if (is_color && color) L.set_bgr(png);
  else if (!is_color && color) L.set_gray_to_rgb(png);
  else if (is_color && !color) L.set_rgb_to_gray(png, 1, 0.299, 0.587);
  L.set_interlace_handling(png);
  L.read_update_info(png, info);
  if (L.get_rowbytes(png, info) != size_t(w) * (color ? 3 : 1)) {
    L.destroy_read_struct(&png, &info, nullptr);
    return kUnsupported;
  }
  for (uint32_t y = 0; y < h; ++y) rows[y] = out + size_t(y) * w * (color ? 3 : 1);
  L.read_image(png, rows.data());
  L.read_end(png, nullptr);
  L.destroy_read_struct(&png, &info, nullptr);
  return kOk;
}

void mem_read(void* png, uint8_t* out, size_t n) {
  MemReader* r = static_cast<MemReader*>(libpng()->get_io_ptr(png));   // (loaded: libpng_read runs)
  if (r->at + n > r->b->size()) {                        // png_error would longjmp: fill zeros, let
    memset(out, 0, n);                                   // libpng's own CRC / zlib checks fail
    r->at = r->b->size();
    return;
  }
  memcpy(out, r->b->data() + r->at, n);
  r->at += n;
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
  // a colour file's gray conversion under a gamma / ICC chunk is the host's (slg_png_read): the
  // device converts with the untagged file's integer formula only
  if (png.ch >= 3 && png.color_chunks) return kUnsupported;
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


// Layout of any PNG: info[0] width, [1] height, [2] colour type, [3] bit depth, [4] interlace,
// [5] 1 when the colour handling is restated here, 0 when the system libpng decodes it.
int32_t slg_png_info(const char* path, int32_t* info) {
  if (!path || !info) return kInvalid;
  std::vector<uint8_t> b;
  if (!read_file(path, b)) return kInvalid;
  PngMeta m;
  const int rc = parse_meta(b, m);
  if (rc) return rc;
  int32_t g = 0;
  info[0] = int32_t(m.w); info[1] = int32_t(m.h); info[2] = m.ctype; info[3] = m.depth; info[4] = m.interlace;
  info[5] = restated_gamma(m, &g) ? 1 : 0;
  return kOk;
}

// cv2.imread(path, 0) into gray [h][w] and / or cv2.imread(path) into bgr [h][w][3] (either may
// be NULL; caps in bytes).  info as slg_png_info, plus info[6] = 1 when the system libpng
// decoded it.  Thread-safe (per-thread buffers); non-zero on an unreadable, corrupt or
// unsupported file (cv2.imread returns None for those).
int32_t slg_png_read(const char* path, uint8_t* gray, int64_t gray_cap, uint8_t* bgr, int64_t bgr_cap, int32_t* info) {
  if (!path || !info || (!gray && !bgr)) return kInvalid;
  thread_local std::vector<uint8_t> b;
  if (!read_file(path, b)) return kInvalid;
  PngMeta m;
  int rc = parse_meta(b, m);
  if (rc) return rc;
  const int64_t n = int64_t(m.w) * m.h;
  if ((gray && gray_cap < n) || (bgr && bgr_cap < 3 * n)) return kInvalid;
  int32_t g = 0;
  const bool restated = restated_gamma(m, &g);
  info[0] = int32_t(m.w); info[1] = int32_t(m.h); info[2] = m.ctype; info[3] = m.depth; info[4] = m.interlace;
  info[5] = restated ? 1 : 0;
  info[6] = 0;
  const LibPng* L = libpng();
  if (!restated && L) {
    info[6] = 1;
    if (gray && (rc = libpng_read(*L, b, false, gray, m.w, m.h)) != kOk) return rc;
    if (bgr && (rc = libpng_read(*L, b, true, bgr, m.w, m.h)) != kOk) return rc;
    return kOk;
  }
  GrayConv gc;
  gc.init(m, g);                              // (no libpng: the gAMA / sRGB rule alone)
  rc = decode_general(m, gc, gray, bgr);
  if (rc != kOk && L) {                       // a stream libpng may still read (its call)
    info[6] = 1;
    if (gray && (rc = libpng_read(*L, b, false, gray, m.w, m.h)) != kOk) return rc;
    if (bgr && (rc = libpng_read(*L, b, true, bgr, m.w, m.h)) != kOk) return rc;
  }
  return rc;
}

}  // extern "C"
