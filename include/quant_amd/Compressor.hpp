// quant_amd C++ API -- block VQ codec (reference: include/Compressor.hpp, src/Compressor.cpp).
//
// compress() tiles the raster and trains the codebook on the MI355X engine (qvq_set_images
// + qvq_lbg: the blocks are tiled on the device, the 8-byte-per-component fp64 training set
// of the reference is never built); the other functions are host code.  .quant files:
//   "<bits> <colorSpace> <count> <xSize> <ySize> <bw> <bh>\n", 2^bits codebook entries of
//   bw*bh*3 bytes, then count indices of ceil(bits/8) little-endian bytes.
// Errors throw std::runtime_error (the engine's message).
#pragma once
#include <chrono>
#include <cstddef>
#include <ostream>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "ColorSpace.hpp"
#include "Quantizer.hpp"
#include "VectorOperations.hpp"

class CompressionRaport {
public:
    VectorType distortion;
    float bitsPerPixel;
    size_t uncompressedSize;
    size_t compressedSize;
    std::chrono::duration<double> compressionTime;
    friend std::ostream &operator<<(std::ostream &stream, const CompressionRaport &raport);
};

class CompressedImage {
public:
    CompressedImage() = default;
    void saveToFile(const std::string &path);
    void loadFromFile(const std::string &path);
    size_t sizeInBits();

    static std::pair<CompressedImage, CompressionRaport> compress(const RGBImage &image, Quantizers quantizer,
                                                                  ColorSpaces colorSpace, int blockWidth,
                                                                  int blockHeight, VectorType eps, int N);
    static RGBImage decompress(const CompressedImage &);

    std::vector<CharVector> codeVectors;
    std::vector<size_t> assignedCodeVector;
    size_t xSize = 0, ySize = 0;
    size_t blockWidth = 0, blockHeight = 0;
    ColorSpaces colorSpace = ColorSpaces::SCALED;
    Quantizers quantizer = Quantizers::LBG;
};

std::vector<CharVector> vectorsToCharVectorsColorSpaced(const std::vector<Vector> &vectors,
                                                        const ColorSpacePtr &cs);
std::vector<Vector> getBlocksAsVectorsFromImage(const RGBImage &image, int w, int h, const ColorSpacePtr &);
RGBImage getImageFromVectors(const std::vector<CharVector> &blocks, int xSize, int ySize, int w, int h);
