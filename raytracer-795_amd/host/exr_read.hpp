// exr_read.hpp — OpenEXR texture decoding for the native host (what the reference's
// Texture::ReadExr -> ExrLibrary::ReadExr -> LoadEXR gives the texture code,
// src/Texture.cpp:185-189, src/Helper.cpp:346-359).
#pragma once
#include <string>
#include <vector>

namespace rtgh {

// Decode a single-part OpenEXR file into RGBA floats, row 0 = the data window's first line.
// Supported: scanline and one-level tiled images; NONE, RLE, ZIPS, ZIP and PIZ compression;
// HALF, FLOAT and UINT channels.  Channel selection follows LoadEXR: names are taken after
// their last '.', the first four (file order) are searched for R, G, B, A; a one-channel
// image is replicated into all four; without A, alpha is 1.  Returns false with `err` set.
bool read_exr_rgba(const std::string& path, std::vector<float>& rgba, int& w, int& h, std::string& err);

}  // namespace rtgh
