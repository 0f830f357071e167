// tiff.hpp -- uncompressed grayscale TIFF I/O (see tiff.cpp).
#pragma once
#include <cstdint>
#include <string>

#include "dataset.hpp"

namespace fpmhost {
bool read_tiff(const std::string &path, Frame *out, std::string *err);
bool write_tiff16(const std::string &path, int width, int height, const uint16_t *px, std::string *err);
}  // namespace fpmhost
