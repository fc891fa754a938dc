// image_io.h — the reference's output stage for the `pathtracer` CLI.
//
// HDRImageBuffer::toColor (src/util/image.h:194-209: exposure sqrt(2^1), gamma 2.2, clamp),
// ImageBuffer::update_pixel (image.h:53-62: RGBA8 by truncation of clamp(c) * 255), the vertical
// flip + opaque alpha of RaytracedRenderer::save_image (raytraced_renderer.cpp:690-728) and the
// sampling-rate image of save_sampling_rate_image (:730-761). PNG encoding is our own (zlib
// stored blocks): the decoded pixels equal the reference's, the compressed bytes do not.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace bdpt {

// rgb: W*H*3 values, row 0 = bottom (as HDRImageBuffer). Returns W*H RGBA8 words, row 0 = bottom.
std::vector<uint32_t> tonemap(const double* rgb, int w, int h);

// Writes RGBA8 words (row 0 = bottom) flipped to top-first, alpha forced to 0xFF, as PNG.
bool write_png(const std::string& path, const std::vector<uint32_t>& rgba, int w, int h);

// save_sampling_rate_image: per-pixel samples / ns_aa as a blue-green-red ramp, "<name>_rate.png".
bool write_rate_png(const std::string& png_path, const std::vector<float>& rate, int w, int h);

}  // namespace bdpt
