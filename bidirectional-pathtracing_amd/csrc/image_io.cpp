// image_io.cpp — see image_io.h.
#include "image_io.h"

#include <algorithm>
#include <cmath>
#include <cstdio>

namespace bdpt {

namespace {

uint32_t pack_color(float r, float g, float b) {   // ImageBuffer::update_pixel(Color)
  auto c = [](float v) { return std::min(std::max(v, 0.f), 1.f); };
  uint32_t p = 0;
  p |= ((uint32_t)(c(b) * 255)) << 16;
  p |= ((uint32_t)(c(g) * 255)) << 8;
  p |= ((uint32_t)(c(r) * 255));
  p |= 0xFF000000u;
  return p;
}

uint32_t crc_table[256];
void crc_init() {
  for (uint32_t n = 0; n < 256; n++) {
    uint32_t c = n;
    for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_table[n] = c;
  }
}
uint32_t crc32(const unsigned char* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  for (size_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}
void put32(std::vector<unsigned char>& o, uint32_t v) {
  o.push_back((unsigned char)(v >> 24));
  o.push_back((unsigned char)(v >> 16));
  o.push_back((unsigned char)(v >> 8));
  o.push_back((unsigned char)v);
}
void chunk(FILE* f, const char* type, const std::vector<unsigned char>& data) {
  std::vector<unsigned char> o;
  put32(o, (uint32_t)data.size());
  o.insert(o.end(), type, type + 4);
  o.insert(o.end(), data.begin(), data.end());
  const uint32_t c = crc32(o.data() + 4, o.size() - 4) ^ 0xFFFFFFFFu;
  put32(o, c);
  fwrite(o.data(), 1, o.size(), f);
}

}  // namespace

std::vector<uint32_t> tonemap(const double* rgb, int w, int h) {
  const float gamma = 2.2f, level = 1.0f;
  const float one_over_gamma = 1.0f / gamma;
  const float exposure = (float)std::sqrt(std::pow(2, level));
  std::vector<uint32_t> out((size_t)w * h);
  for (size_t i = 0; i < out.size(); i++) {
    const double s[3] = {rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]};
    float c[3];
    for (int k = 0; k < 3; k++) c[k] = (float)std::max(0.0, std::min(std::pow(s[k] * exposure, (double)one_over_gamma), 1.0));
    out[i] = pack_color(c[0], c[1], c[2]);
  }
  return out;
}

bool write_png(const std::string& path, const std::vector<uint32_t>& rgba, int w, int h) {
  static bool init = false;
  if (!init) { crc_init(); init = true; }
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return false;
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  fwrite(sig, 1, 8, f);
  std::vector<unsigned char> ihdr;
  put32(ihdr, (uint32_t)w);
  put32(ihdr, (uint32_t)h);
  ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});   // 8-bit RGBA, deflate, filter 0, no interlace
  chunk(f, "IHDR", ihdr);
  // raw scanlines (filter byte 0), top row first
  std::vector<unsigned char> raw;
  raw.reserve((size_t)h * (4 * (size_t)w + 1));
  for (int i = 0; i < h; i++) {
    raw.push_back(0);
    const uint32_t* row = &rgba[(size_t)(h - 1 - i) * w];
    for (int x = 0; x < w; x++) {
      const uint32_t p = row[x] | 0xFF000000u;
      raw.push_back((unsigned char)(p & 0xFF));
      raw.push_back((unsigned char)((p >> 8) & 0xFF));
      raw.push_back((unsigned char)((p >> 16) & 0xFF));
      raw.push_back((unsigned char)(p >> 24));
    }
  }
  // zlib stream of stored deflate blocks + Adler-32
  std::vector<unsigned char> z = {0x78, 0x01};
  size_t pos = 0;
  do {
    const size_t n = std::min<size_t>(65535, raw.size() - pos);
    const bool last = pos + n == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((unsigned char)(n & 0xFF));
    z.push_back((unsigned char)(n >> 8));
    z.push_back((unsigned char)(~n & 0xFF));
    z.push_back((unsigned char)((~n >> 8) & 0xFF));
    z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
    pos += n;
  } while (pos < raw.size());
  uint32_t a = 1, b = 0;
  for (unsigned char c : raw) {
    a = (a + c) % 65521u;
    b = (b + a) % 65521u;
  }
  put32(z, (b << 16) | a);
  chunk(f, "IDAT", z);
  chunk(f, "IEND", {});
  const bool ok = ferror(f) == 0;
  fclose(f);
  return ok;
}

bool write_rate_png(const std::string& png_path, const std::vector<float>& rate, int w, int h) {
  std::vector<uint32_t> buf((size_t)w * h);
  for (int x = 0; x < w; x++)
    for (int y = 0; y < h; y++) {
      const float s = rate[(size_t)y * w + x];
      float cr, cg, cb;
      if (s <= 0.5) {
        const float r = (0.5 - s) / 0.5;
        cr = 0.0f * r + 0.0f * (1.0 - r);
        cg = 0.0f * r + 1.0f * (1.0 - r);
        cb = 1.0f * r + 0.0f * (1.0 - r);
      } else {
        const float r = (1.0 - s) / 0.5;
        cr = 0.0f * r + 1.0f * (1.0 - r);
        cg = 1.0f * r + 0.0f * (1.0 - r);
        cb = 0.0f * r + 0.0f * (1.0 - r);
      }
      buf[x + (size_t)(h - 1 - y) * w] = pack_color(cr, cg, cb);
    }
  // save_sampling_rate_image writes outputBuffer rows as they are (no flip)
  std::vector<uint32_t> flipped((size_t)w * h);
  for (int i = 0; i < h; i++)
    std::copy(&buf[(size_t)i * w], &buf[(size_t)i * w] + w, &flipped[(size_t)(h - 1 - i) * w]);
  const std::string rp = png_path.size() > 4 ? png_path.substr(0, png_path.size() - 4) + "_rate.png" : png_path + "_rate.png";
  return write_png(rp, flipped, w, h);
}

}  // namespace bdpt
