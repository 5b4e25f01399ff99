// quant_amd C++ API -- binary PPM images (reference: include/RGBImage.hpp, src/RGBImage.cpp).
// The raster keeps the file's pixel order; xSize is the header's first number (width) and
// ySize the second, and the block tiling reads pixel x*ySize + y, as the reference does.
#pragma once
#include <array>
#include <cstddef>
#include <string>
#include <vector>

const static int MAX_COL_BITS = 8;
const static int MAX_COL = 1 << MAX_COL_BITS;

typedef std::array<char, 3> RGB;
typedef std::array<double, 3> RGBDouble;

class RGBImage {
public:
    RGBImage() = default;
    explicit RGBImage(const std::string &path);   // throws std::runtime_error on a bad file
    void saveToFile(const std::string &path);
    size_t sizeInBytes() const;
    std::vector<RGB> img;
    int xSize = 0, ySize = 0;
};
