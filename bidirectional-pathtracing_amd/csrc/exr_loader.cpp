// exr_loader.cpp — host OpenEXR reader for the environment map (-e), the product's replacement of
// the reference's load_exr (src/application/main.cpp:40-77, which drives the vendored tinyexr).
//
// Scope: single-part scanline files, compression NONE (0), RLE (1), ZIPS (2), ZIP (3); HALF and
// FLOAT channels (load_exr requests FLOAT for HALF channels, main.cpp:53-57). Tiled, multi-part,
// deep and PIZ/PXR24/B44/DWA files are rejected with BDPT_E_UNSUPPORTED. Like load_exr, channel k
// of the output pixel is the file's channel 2 - k in channel-list (alphabetical) order, so an RGB
// file maps R, G, B -> r, g, b (an RGBA file gets the reference's channel shift, main.cpp:66-74).
// Rows are returned top (y = dataWindow.yMin) first: HDRImageBuffer data[x + y * w].

#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "bdpt/bdpt.h"
#include "bdpt_err.h"

namespace {

using bdpt::g_err;

struct Chan {
  std::string name;
  int type;   // 0 UINT, 1 HALF, 2 FLOAT
  int xs, ys;
};

uint32_t rd32(const unsigned char* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
uint64_t rd64(const unsigned char* p) { return (uint64_t)rd32(p) | (uint64_t)rd32(p + 4) << 32; }

// IEEE half -> float, exact (every half is a float).
float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h >> 15) << 31;
  const uint32_t e = (h >> 10) & 31u, m = h & 1023u;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) {
      bits = s;
    } else {   // subnormal: normalise
      int ee = -1;
      uint32_t mm = m;
      do { ee++; mm <<= 1; } while (!(mm & 1024u));
      bits = s | (uint32_t)(127 - 15 - ee) << 23 | (mm & 1023u) << 13;
    }
  } else if (e == 31) {
    bits = s | 0x7f800000u | m << 13;
  } else {
    bits = s | (e - 15 + 127) << 23 | m << 13;
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

// ZIP / RLE post-processing (OpenEXR ImfZip / ImfRle): undo the byte predictor, then de-interleave
// the two half-streams.
void unpredict_deinterleave(std::vector<unsigned char>& t, std::vector<unsigned char>& out) {
  for (size_t i = 1; i < t.size(); i++) t[i] = (unsigned char)(t[i - 1] + t[i] - 128);
  out.resize(t.size());
  const size_t half = (t.size() + 1) / 2;
  size_t a = 0, b = half, k = 0;
  while (k < out.size()) {
    out[k++] = t[a++];
    if (k < out.size()) out[k++] = t[b++];
  }
}

bool rle_decode(const unsigned char* in, size_t n, std::vector<unsigned char>& out, size_t want) {
  out.clear();
  size_t i = 0;
  while (i < n) {
    int c = (signed char)in[i++];
    if (c < 0) {
      size_t k = (size_t)(-c);
      if (i + k > n) return false;
      out.insert(out.end(), in + i, in + i + k);
      i += k;
    } else {
      if (i >= n) return false;
      out.insert(out.end(), (size_t)c + 1, in[i++]);
    }
    if (out.size() > want) return false;
  }
  return out.size() == want;
}

int fail(int code, const std::string& msg) {
  g_err = "exr: " + msg;
  return code;
}

}  // namespace

extern "C" int bdpt_exr_load(const char* path, int32_t* width, int32_t* height, float** rgb_out) {
  if (!path || !width || !height || !rgb_out) return fail(BDPT_E_INVALID, "null argument");
  *rgb_out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) return fail(BDPT_E_INVALID, std::string("cannot open ") + path);
  std::vector<unsigned char> buf;
  {
    unsigned char tmp[1 << 16];
    size_t r;
    while ((r = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    fclose(f);
  }
  const size_t N = buf.size();
  const unsigned char* b = buf.data();
  if (N < 8 || rd32(b) != 20000630u) return fail(BDPT_E_INVALID, "not an OpenEXR file");
  const uint32_t ver = rd32(b + 4);
  if ((ver & 0xffu) != 2) return fail(BDPT_E_UNSUPPORTED, "unsupported OpenEXR version");
  if (ver & 0x200u) return fail(BDPT_E_UNSUPPORTED, "tiled files are not supported");
  if (ver & 0x1800u) return fail(BDPT_E_UNSUPPORTED, "multi-part / deep files are not supported");
  size_t p = 8;
  std::vector<Chan> chans;
  int comp = -1;
  int32_t dw[4] = {0, 0, -1, -1};
  bool have_dw = false;
  auto cstr = [&](std::string& s) {
    size_t e = p;
    while (e < N && b[e]) e++;
    if (e >= N) return false;
    s.assign((const char*)b + p, e - p);
    p = e + 1;
    return true;
  };
  for (;;) {
    if (p >= N) return fail(BDPT_E_INVALID, "truncated header");
    if (b[p] == 0) { p++; break; }
    std::string name, type;
    if (!cstr(name) || !cstr(type) || p + 4 > N) return fail(BDPT_E_INVALID, "bad attribute");
    const uint32_t sz = rd32(b + p);
    p += 4;
    if (p + sz > N) return fail(BDPT_E_INVALID, "truncated attribute " + name);
    const unsigned char* v = b + p;
    if (name == "channels") {
      size_t q = 0;
      while (q < sz && v[q]) {
        size_t e = q;
        while (e < sz && v[e]) e++;
        if (e + 17 > sz) return fail(BDPT_E_INVALID, "bad channel list");
        Chan c;
        c.name.assign((const char*)v + q, e - q);
        c.type = (int)rd32(v + e + 1);
        c.xs = (int)rd32(v + e + 9);
        c.ys = (int)rd32(v + e + 13);
        chans.push_back(c);
        q = e + 17;
      }
    } else if (name == "compression") {
      comp = sz ? v[0] : -1;
    } else if (name == "dataWindow" && sz >= 16) {
      for (int k = 0; k < 4; k++) dw[k] = (int32_t)rd32(v + 4 * k);
      have_dw = true;
    }
    p += sz;
  }
  if (!have_dw || chans.empty()) return fail(BDPT_E_INVALID, "missing channels / dataWindow");
  if (chans.size() < 3) return fail(BDPT_E_UNSUPPORTED, "need at least 3 channels (load_exr reads channels 0..2)");
  for (const Chan& c : chans) {
    if (c.type != 1 && c.type != 2) return fail(BDPT_E_UNSUPPORTED, "only HALF / FLOAT channels are supported");
    if (c.xs != 1 || c.ys != 1) return fail(BDPT_E_UNSUPPORTED, "subsampled channels are not supported");
  }
  int lines;
  switch (comp) {
    case 0: case 1: case 2: lines = 1; break;
    case 3: lines = 16; break;
    default: return fail(BDPT_E_UNSUPPORTED, "compression " + std::to_string(comp) + " not supported (NONE/RLE/ZIPS/ZIP)");
  }
  const long long W = (long long)dw[2] - dw[0] + 1, H = (long long)dw[3] - dw[1] + 1;
  if (W <= 0 || H <= 0 || W * H > (1LL << 28)) return fail(BDPT_E_INVALID, "bad dataWindow");
  size_t px_bytes = 0;
  for (const Chan& c : chans) px_bytes += c.type == 1 ? 2 : 4;
  const long long nchunks = (H + lines - 1) / lines;
  if (p + 8 * (size_t)nchunks > N) return fail(BDPT_E_INVALID, "truncated offset table");
  std::vector<float> planes(chans.size() * (size_t)(W * H));
  std::vector<unsigned char> raw, tmp;
  for (long long ci = 0; ci < nchunks; ci++) {
    const uint64_t off = rd64(b + p + 8 * ci);
    if (off + 8 > N) return fail(BDPT_E_INVALID, "bad chunk offset");
    const int32_t y0 = (int32_t)rd32(b + off);
    const uint32_t len = rd32(b + off + 4);
    if (off + 8 + len > N) return fail(BDPT_E_INVALID, "truncated chunk");
    const long long row0 = (long long)y0 - dw[1];
    if (row0 < 0 || row0 >= H) return fail(BDPT_E_INVALID, "chunk y out of range");
    const long long nrows = std::min<long long>(lines, H - row0);
    const size_t want = (size_t)(nrows * W) * px_bytes;
    const unsigned char* data = b + off + 8;
    if (comp == 0 || len == want) {   // stored (a compressor falls back to raw when it cannot shrink)
      if (len != want) return fail(BDPT_E_INVALID, "chunk size mismatch");
      raw.assign(data, data + len);
    } else if (comp == 1) {
      if (!rle_decode(data, len, tmp, want)) return fail(BDPT_E_INVALID, "bad RLE chunk");
      unpredict_deinterleave(tmp, raw);
    } else {
      tmp.resize(want);
      uLongf out_len = (uLongf)want;
      if (uncompress(tmp.data(), &out_len, data, len) != Z_OK || out_len != want)
        return fail(BDPT_E_INVALID, "bad ZIP chunk");
      unpredict_deinterleave(tmp, raw);
    }
    // per scanline: each channel's W values in channel-list order
    size_t q = 0;
    for (long long r = 0; r < nrows; r++) {
      const size_t rowbase = (size_t)((row0 + r) * W);
      for (size_t c = 0; c < chans.size(); c++) {
        float* dst = planes.data() + c * (size_t)(W * H) + rowbase;
        if (chans[c].type == 1) {
          for (long long x = 0; x < W; x++, q += 2) dst[x] = half_to_float((uint16_t)(raw[q] | raw[q + 1] << 8));
        } else {
          for (long long x = 0; x < W; x++, q += 4) {
            uint32_t u = rd32(raw.data() + q);
            std::memcpy(dst + x, &u, 4);
          }
        }
      }
    }
  }
  float* out = new (std::nothrow) float[(size_t)(W * H) * 3];
  if (!out) return fail(BDPT_E_NOMEM, "out of host memory");
  const size_t np = (size_t)(W * H);
  for (size_t i = 0; i < np; i++) {   // load_exr: r = images[2], g = images[1], b = images[0]
    out[3 * i + 0] = planes[2 * np + i];
    out[3 * i + 1] = planes[1 * np + i];
    out[3 * i + 2] = planes[0 * np + i];
  }
  *width = (int32_t)W;
  *height = (int32_t)H;
  *rgb_out = out;
  return BDPT_OK;
}

extern "C" void bdpt_exr_free(float* rgb) { delete[] rgb; }
