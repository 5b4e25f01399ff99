// Block VQ codec on top of the engine; see include/quant_amd/Compressor.hpp.
// Semantics follow src/Compressor.cpp (file:line cited per function).
#include "quant_amd/Compressor.hpp"

#include <cmath>
#include <cstdint>
#include <fstream>
#include <functional>
#include <iomanip>
#include <sstream>
#include <stdexcept>

#include "engine_handle.hpp"

using quant_amd::EngineHandle;

// src/Compressor.cpp:12-29: each code vector back to bytes through the colour space.
std::vector<CharVector> vectorsToCharVectorsColorSpaced(const std::vector<Vector> &vectors, const ColorSpacePtr &cs) {
    std::vector<CharVector> out;
    out.reserve(vectors.size());
    for (const Vector &v : vectors) {
        CharVector bytes(v.size());
        for (size_t i = 0; i + 2 < v.size(); i += 3) {
            const RGB px = cs->colorSpaceToRGB({v[i], v[i + 1], v[i + 2]});
            bytes[i] = px[0];
            bytes[i + 1] = px[1];
            bytes[i + 2] = px[2];
        }
        out.push_back(std::move(bytes));
    }
    return out;
}

// src/Compressor.cpp:31-62: block (i, j) of w x h pixels, block index i * hBlocks + j;
// pixel (x, y) is raster entry x * ySize + y (columns past ySize run into the next row),
// entries past the raster are zero.  Component order: ((x - iw) * h + (y - jh)) * 3 + c.
std::vector<Vector> getBlocksAsVectorsFromImage(const RGBImage &image, int w, int h, const ColorSpacePtr &cs) {
    const size_t xs = (size_t)image.xSize, ys = (size_t)image.ySize;
    const size_t wB = (xs + w - 1) / w, hB = (ys + h - 1) / h, total = image.img.size();
    std::vector<Vector> blocks(wB * hB, Vector((size_t)3 * w * h, 0.0));
    for (size_t i = 0; i < wB; i++)
        for (size_t j = 0; j < hB; j++) {
            Vector &b = blocks[i * hB + j];
            for (size_t dx = 0; dx < (size_t)w; dx++)
                for (size_t dy = 0; dy < (size_t)h; dy++) {
                    const size_t src = (i * w + dx) * ys + (j * h + dy);
                    if (src >= total) continue;
                    const RGBDouble v = cs->RGBtoColorSpace(image.img[src]);
                    const size_t o = (dx * h + dy) * 3;
                    b[o] = v[0];
                    b[o + 1] = v[1];
                    b[o + 2] = v[2];
                }
        }
    return blocks;
}

// src/Compressor.cpp:64-92: the inverse placement; entries past the raster are dropped.
RGBImage getImageFromVectors(const std::vector<CharVector> &blocks, int xSize, int ySize, int w, int h) {
    const size_t xs = (size_t)xSize, ys = (size_t)ySize;
    const size_t wB = (xs + w - 1) / w, hB = (ys + h - 1) / h;
    RGBImage img;
    img.xSize = xSize;
    img.ySize = ySize;
    img.img.assign(xs * ys, RGB{0, 0, 0});
    for (size_t i = 0; i < wB; i++)
        for (size_t j = 0; j < hB; j++) {
            const CharVector &b = blocks.at(i * hB + j);
            for (size_t dx = 0; dx < (size_t)w; dx++)
                for (size_t dy = 0; dy < (size_t)h; dy++) {
                    const size_t dst = (i * w + dx) * ys + (j * h + dy);
                    if (dst >= img.img.size()) continue;
                    const size_t o = (dx * h + dy) * 3;
                    img.img[dst] = RGB{b.at(o), b.at(o + 1), b.at(o + 2)};
                }
        }
    return img;
}

namespace {

size_t floor_log2(size_t n) {   // smallestPow2, src/Compressor.cpp:167-172
    size_t p = 0;
    while (n /= 2) p++;
    return p;
}

bool engine_sums_exactly(ColorSpaces cs) { return cs == ColorSpaces::NORMAL || cs == ColorSpaces::SCALED; }

// The SCALED byte of one centroid component (ScaledColor::colorSpaceToRGB, src/ColorSpace.cpp:23-28).
int scaled_byte(double c) { return (int)std::round((c - 128.0) * 255); }

// True when some component c has another byte within FLIP_ULPS ulps: the exact-sum and Kahan
// centroids of a cell differ by at most a few ulps (both sums of nonnegative values: the exact
// one is rounded once, Kahan's error is <= 2u of the sum plus O(n u^2) of it), so outside that
// window both give the same byte.
bool codebook_near_byte_flip(const std::vector<double> &C) {
    constexpr double FLIP_ULPS = 16;
    for (double c : C) {
        const double w = FLIP_ULPS * (std::nextafter(std::fabs(c), INFINITY) - std::fabs(c));
        if (scaled_byte(c - w) != scaled_byte(c + w)) return true;
    }
    return false;
}

// The image's blocks trained on the engine straight from the raster (device tiling).
std::tuple<std::vector<Vector>, std::vector<size_t>, VectorType> quantize_raster(const RGBImage &image,
                                                                                 ColorSpaces cs, int bw, int bh,
                                                                                 VectorType eps, int n) {
    qvq_ctx *ctx = EngineHandle::get();
    EngineHandle::check(qvq_set_images(ctx, reinterpret_cast<const uint8_t *>(image.img.data()), 1,
                                       (uint32_t)image.xSize, (uint32_t)image.ySize, (uint32_t)bw, (uint32_t)bh,
                                       (int)cs),
                        "qvq_set_images");
    const size_t N = qvq_num_vectors(ctx), D = qvq_dim(ctx), K = (size_t)1 << n;
    std::vector<double> C(K * D);
    std::vector<uint32_t> A(N);
    double distortion = 0;
    EngineHandle::check(qvq_lbg(ctx, (uint32_t)n, eps, C.data(), A.data(), &distortion), "qvq_lbg");
    // qvq_lbg returns exact-sum centroids; the reference's are Kahan sums (src/Quantizer.cpp:59-87),
    // at most a few ulps away.  Only a component within a few ulps of a point where
    // round((c - 128) * 255) changes can turn into another byte (src/ColorSpace.cpp:23-28), so the
    // reference's bits are fetched when any component sits that close (SCALED only: NORMAL values
    // are integers, whose Kahan sums are exact).
    if (cs == ColorSpaces::SCALED && codebook_near_byte_flip(C)) {
        EngineHandle::check(qvq_update_kahan(ctx, A.data(), (uint32_t)K, C.data()), "qvq_update_kahan");
    }
    std::vector<Vector> codebook(K, Vector(D));
    for (size_t k = 0; k < K; k++) std::copy(C.begin() + k * D, C.begin() + (k + 1) * D, codebook[k].begin());
    return std::make_tuple(std::move(codebook), std::vector<size_t>(A.begin(), A.end()), distortion);
}

// Codebook bytes [K][bw*bh*3] (short entries zero-filled) and u32 indices for qvq_decode.
void flatten_for_decode(const CompressedImage &c, std::vector<uint8_t> &cb, std::vector<uint32_t> &idx) {
    const size_t D = c.blockWidth * c.blockHeight * 3, K = c.codeVectors.size();
    if (K == 0 || K > 0xFFFFFFFFull) throw std::runtime_error("decompress: bad codebook size");
    cb.assign(K * D, 0);
    for (size_t k = 0; k < K; k++) {
        const CharVector &v = c.codeVectors[k];
        std::copy(v.begin(), v.begin() + std::min(v.size(), D), reinterpret_cast<char *>(cb.data()) + k * D);
    }
    idx.resize(c.assignedCodeVector.size());
    for (size_t i = 0; i < idx.size(); i++) {
        if (c.assignedCodeVector[i] >= K) throw std::runtime_error("decompress: code-vector index out of range");
        idx[i] = (uint32_t)c.assignedCodeVector[i];
    }
}

std::string pretty_bytes(size_t bytes) {   // src/Compressor.cpp:270-287, remainder quirk kept
    std::ostringstream s;
    if (bytes < 1024) {
        s << bytes << "b";
    } else if (bytes < 1024 * 1024) {
        s << bytes / 1024 << "," << bytes % 1024 << "Kb";
    } else {
        s << bytes / (1024 * 1024) << "," << bytes % (1024 * 1024) << "Mb";
    }
    return s.str();
}

}  // namespace

// src/Compressor.cpp:107-154.  The timed region is tiling + quantize, as in the reference.
std::pair<CompressedImage, CompressionRaport> CompressedImage::compress(const RGBImage &image, Quantizers quantizer,
                                                                        ColorSpaces colorSpace, int blockWidth,
                                                                        int blockHeight, VectorType eps, int N) {
    if (blockWidth <= 0 || blockHeight <= 0 || N < 0) throw std::invalid_argument("compress: bad block size or bits");
    ColorSpacePtr cs = getColorSpace(colorSpace);
    std::vector<Vector> codebook;
    std::vector<size_t> assigned;
    VectorType distortion = 0;
    const auto t0 = std::chrono::system_clock::now();
    if (quantizer == Quantizers::LBG && engine_sums_exactly(colorSpace)) {
        std::tie(codebook, assigned, distortion) = quantize_raster(image, colorSpace, blockWidth, blockHeight, eps, N);
    } else {
        QuantizerPtr q = getQuantizer(quantizer);
        if (!q) throw std::runtime_error("compress: quantizer not implemented");
        std::tie(codebook, assigned, distortion) =
            q->quantize(getBlocksAsVectorsFromImage(image, blockWidth, blockHeight, cs), (size_t)N, eps);
    }
    const std::chrono::duration<double> elapsed = std::chrono::system_clock::now() - t0;

    CompressedImage out;
    out.codeVectors = vectorsToCharVectorsColorSpaced(codebook, cs);
    out.assignedCodeVector = std::move(assigned);
    out.xSize = (size_t)image.xSize;
    out.ySize = (size_t)image.ySize;
    out.blockWidth = (size_t)blockWidth;
    out.blockHeight = (size_t)blockHeight;
    out.colorSpace = colorSpace;
    out.quantizer = quantizer;

    // distortion of the decoded image in signed byte units (src/Compressor.cpp:133-146), from
    // one device decode pass that also sums the squared differences (qvq_decode_mse)
    double mse = 0;
    {
        std::vector<uint8_t> cb;
        std::vector<uint32_t> idx;
        flatten_for_decode(out, cb, idx);
        EngineHandle::check(qvq_decode_mse(EngineHandle::get(), cb.data(), (uint32_t)out.codeVectors.size(), idx.data(),
                                           idx.size(), (uint32_t)out.xSize, (uint32_t)out.ySize,
                                           (uint32_t)out.blockWidth, (uint32_t)out.blockHeight, nullptr,
                                           reinterpret_cast<const uint8_t *>(image.img.data()), &mse),
                            "qvq_decode_mse");
    }
    CompressionRaport r;
    r.distortion = mse;
    r.bitsPerPixel = (float)out.sizeInBits() / (float)(image.xSize * image.ySize);
    r.uncompressedSize = image.sizeInBytes();
    r.compressedSize = out.sizeInBits() / 8;
    r.compressionTime = elapsed;
    return std::make_pair(std::move(out), r);
}

// src/Compressor.cpp:156-165 (+ getImageFromVectors, :64-92): one device gather (qvq_decode).
RGBImage CompressedImage::decompress(const CompressedImage &c) {
    std::vector<uint8_t> cb;
    std::vector<uint32_t> idx;
    flatten_for_decode(c, cb, idx);
    RGBImage img;
    img.xSize = (int)c.xSize;
    img.ySize = (int)c.ySize;
    img.img.assign(c.xSize * c.ySize, RGB{0, 0, 0});
    EngineHandle::check(qvq_decode(EngineHandle::get(), cb.data(), (uint32_t)c.codeVectors.size(), idx.data(), idx.size(),
                                   (uint32_t)c.xSize, (uint32_t)c.ySize, (uint32_t)c.blockWidth,
                                   (uint32_t)c.blockHeight, reinterpret_cast<uint8_t *>(img.img.data())),
                        "qvq_decode");
    return img;
}

// src/Compressor.cpp:174-183
size_t CompressedImage::sizeInBits() {
    const size_t bits = floor_log2(codeVectors.size()) * assignedCodeVector.size() +
                        blockWidth * blockHeight * codeVectors.size() * 8 * 3;
    return (bits + 7) / 8 * 8;
}

// src/Compressor.cpp:191-224
void CompressedImage::saveToFile(const std::string &path) {
    const size_t bits = floor_log2(codeVectors.size());
    if (bits > 24 || ((size_t)1 << bits) != codeVectors.size())
        throw std::runtime_error("saveToFile: codebook size must be a power of two <= 2^24");
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("cannot write " + path);
    f << bits << ' ' << (int)colorSpace << ' ' << assignedCodeVector.size() << ' ' << xSize << ' ' << ySize << ' '
      << blockWidth << ' ' << blockHeight << '\n';
    const size_t D = blockWidth * blockHeight * 3;
    std::vector<char> row(D, 0);
    for (const CharVector &cv : codeVectors) {
        std::fill(row.begin(), row.end(), 0);
        std::copy(cv.begin(), cv.begin() + std::min(cv.size(), D), row.begin());
        f.write(row.data(), (std::streamsize)D);
    }
    const size_t nb = (bits + 7) / 8;
    std::vector<char> idx(assignedCodeVector.size() * nb);
    for (size_t i = 0; i < assignedCodeVector.size(); i++)
        for (size_t b = 0; b < nb; b++) idx[i * nb + b] = (char)((assignedCodeVector[i] >> (8 * b)) & 0xFF);
    f.write(idx.data(), (std::streamsize)idx.size());
    if (!f) throw std::runtime_error("write failed: " + path);
}

// src/Compressor.cpp:226-267
void CompressedImage::loadFromFile(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    size_t bits = 0, count = 0;
    int cs = 0;
    f >> bits >> cs >> count >> xSize >> ySize >> blockWidth >> blockHeight;
    if (!f || bits > 24) throw std::runtime_error(path + ": bad .quant header");
    f.get();
    colorSpace = (ColorSpaces)cs;
    const size_t D = blockWidth * blockHeight * 3;
    codeVectors.assign((size_t)1 << bits, CharVector(D));
    for (CharVector &cv : codeVectors) f.read(cv.data(), (std::streamsize)D);
    const size_t nb = (bits + 7) / 8;
    std::vector<unsigned char> idx(count * nb);
    f.read(reinterpret_cast<char *>(idx.data()), (std::streamsize)idx.size());
    if (!f) throw std::runtime_error(path + ": truncated .quant file");
    assignedCodeVector.assign(count, 0);
    for (size_t i = 0; i < count; i++)
        for (size_t b = 0; b < nb; b++) assignedCodeVector[i] |= (size_t)idx[i * nb + b] << (8 * b);
}

// src/Compressor.cpp:289-305 (same text, for scripts that grep it)
std::ostream &operator<<(std::ostream &s, const CompressionRaport &r) {
    s << "Compression raport: " << std::endl;
    s << "Distortion        = " << std::fixed << std::setprecision(10) << r.distortion << std::endl;
    s << "Bits per pixel    = " << r.bitsPerPixel << std::endl;
    s << "Uncompressed size = " << pretty_bytes(r.uncompressedSize) << std::endl;
    s << "Compressed size   = " << pretty_bytes(r.compressedSize) << std::endl;
    s << "Compression ratio = " << std::fixed << std::setprecision(3)
      << (double)r.compressedSize / (double)r.uncompressedSize << std::endl;
    s << "Compression time  = " << r.compressionTime.count() << "s" << std::endl;
    return s;
}
