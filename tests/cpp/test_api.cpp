// Tests of the C++ API (include/quant_amd/*.hpp, libquant_amd.so), driven by
// tests/test_cpp_api.py.  Modes:
//   host                         : no GPU -- tiling round trips (the reference's own
//                                  src/test.cpp cases), .quant and PPM round trips, colour
//                                  maps, report text, getQuantizer
//   compress IN.ppm OUT.quant OUT.ppm bits bw bh cs
//                                : CompressedImage::compress on the GPU, then saveToFile
//                                  and decompress+saveToFile; prints the raport
//   quantize X.f64 N D bits C.f64 A.u32
//                                : getQuantizer(LBG)->quantize on a flat training set
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

#include "quant_amd/Compressor.hpp"

static int g_fail = 0;
#define CHECK(cond)                                                                     \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            g_fail++;                                                                   \
        }                                                                               \
    } while (0)

static RGBImage letters_4x4() {
    RGBImage img;
    const char *px[4] = {"abc", "def", "ghi", "jkl"};
    for (int r = 0; r < 4; r++)
        for (int i = 0; i < 4; i++) img.img.push_back(RGB{px[i][0], px[i][1], px[i][2]});
    img.xSize = 4;
    img.ySize = 4;
    return img;
}

static void test_tiling_round_trip() {
    // the reference's only test (src/test.cpp:5-62): blocks -> bytes -> image, NORMAL
    const RGBImage img = letters_4x4();
    ColorSpacePtr cs = getColorSpace(ColorSpaces::NORMAL);
    const int shapes[][2] = {{1, 1}, {2, 2}, {1, 3}, {2, 4}, {3, 3}};
    for (auto &s : shapes) {
        auto blocks = getBlocksAsVectorsFromImage(img, s[0], s[1], cs);
        auto bytes = vectorsToCharVectorsColorSpaced(blocks, cs);
        auto back = getImageFromVectors(bytes, img.xSize, img.ySize, s[0], s[1]);
        CHECK(back.img == img.img);
    }
    // odd sizes: wrap into the next row and zero pad past the end
    RGBImage odd;
    odd.xSize = 3;
    odd.ySize = 5;
    for (int i = 0; i < 15; i++) odd.img.push_back(RGB{(char)i, (char)(i * 7), (char)(-i)});
    auto blocks = getBlocksAsVectorsFromImage(odd, 2, 2, cs);
    CHECK(blocks.size() == 2 * 3);
    // block (1, 2) = pixels x in {2,3}, y in {4,5}: (2,4) -> 14, (2,5) -> 15 past end, (3,*) past end
    CHECK(blocks[1 * 3 + 2][0] == 14.0);
    CHECK(blocks[1 * 3 + 2][3] == 0.0 && blocks[1 * 3 + 2][6] == 0.0);
    // block (0, 2) = x in {0,1}, y in {4,5}: (0,5) wraps to raster entry 5
    CHECK(blocks[0 * 3 + 2][3] == 5.0);
    auto back = getImageFromVectors(vectorsToCharVectorsColorSpaced(blocks, cs), 3, 5, 2, 2);
    CHECK(back.img == odd.img);
}

static void test_colour_maps() {
    ColorSpacePtr sc = getColorSpace(ColorSpaces::SCALED);
    for (int b = -128; b < 128; b++) {
        const RGB px{(char)b, (char)b, (char)b};
        const RGBDouble v = sc->RGBtoColorSpace(px);
        CHECK(v[0] == ((double)b + 128.0) / 255);
    }
    // (c - 128) * 255 rounded, low byte: c = 0.5 -> -32512.5 -> -32513 -> 0xFF
    CHECK((unsigned char)sc->colorSpaceToRGB({0.5, 0.0, 1.0})[0] == (unsigned char)((-32513) & 0xFF));
    CHECK((unsigned char)sc->colorSpaceToRGB({0.5, 0.0, 1.0})[1] == (unsigned char)((-32640) & 0xFF));
    ColorSpacePtr n = getColorSpace(ColorSpaces::NORMAL);
    CHECK(n->colorSpaceToRGB({-3.5, 2.49, 127.0})[0] == (char)-4);
    CHECK(n->colorSpaceToRGB({-3.5, 2.49, 127.0})[1] == (char)2);
}

static void test_quant_file_round_trip(const std::string &dir) {
    CompressedImage c;
    c.xSize = 5;
    c.ySize = 3;
    c.blockWidth = 2;
    c.blockHeight = 1;
    c.colorSpace = ColorSpaces::SCALED;
    for (int k = 0; k < 512; k++) {   // 9 bits -> 2-byte indices
        CharVector cv(6);
        for (int i = 0; i < 6; i++) cv[i] = (char)(k * 3 + i);
        c.codeVectors.push_back(cv);
    }
    for (int i = 0; i < 9; i++) c.assignedCodeVector.push_back((size_t)(i * 61) % 512);
    const std::string path = dir + "/rt.quant";
    c.saveToFile(path);
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string bytes = ss.str();
    CHECK(bytes.rfind("9 1 9 5 3 2 1\n", 0) == 0);
    CHECK(bytes.size() == std::strlen("9 1 9 5 3 2 1\n") + 512 * 6 + 9 * 2);
    CompressedImage d;
    d.loadFromFile(path);
    CHECK(d.codeVectors == c.codeVectors);
    CHECK(d.assignedCodeVector == c.assignedCodeVector);
    CHECK(d.xSize == 5 && d.ySize == 3 && d.blockWidth == 2 && d.blockHeight == 1);
    CHECK(d.colorSpace == ColorSpaces::SCALED);
    // sizeInBits: floor(log2 K) * count + bw*bh*K*8*3, aligned to 8
    CHECK(c.sizeInBits() == ((9 * 9 + 2 * 1 * 512 * 8 * 3) + 7) / 8 * 8);
}

static void test_ppm_and_raport(const std::string &dir) {
    RGBImage img = letters_4x4();
    img.xSize = 8;
    img.ySize = 2;
    img.saveToFile(dir + "/t.ppm");
    RGBImage back(dir + "/t.ppm");
    CHECK(back.xSize == 8 && back.ySize == 2 && back.img == img.img);
    bool threw = false;
    try {
        RGBImage bad(dir + "/does-not-exist.ppm");
    } catch (const std::runtime_error &) {
        threw = true;
    }
    CHECK(threw);
    CompressionRaport r{1.25, 2.5f, 3000000, 1500, std::chrono::duration<double>(0.5)};
    std::ostringstream s;
    s << r;
    CHECK(s.str().find("Distortion        = 1.2500000000\n") != std::string::npos);
    CHECK(s.str().find("Compressed size   = 1,476Kb\n") != std::string::npos);
    CHECK(s.str().find("Uncompressed size = 2,902848Mb\n") != std::string::npos);
    CHECK(getQuantizer(Quantizers::MEDIAN_CUT) == nullptr);
    CHECK(getQuantizer(Quantizers::LBG) != nullptr);
}

static std::vector<char> slurp(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string mode = argv[1];
    try {
        if (mode == "host") {
            const std::string dir = argc > 2 ? argv[2] : ".";
            test_tiling_round_trip();
            test_colour_maps();
            test_quant_file_round_trip(dir);
            test_ppm_and_raport(dir);
        } else if (mode == "compress" && argc == 9) {
            RGBImage img(argv[2]);
            auto res = CompressedImage::compress(img, Quantizers::LBG, (ColorSpaces)std::atoi(argv[8]),
                                                 std::atoi(argv[6]), std::atoi(argv[7]), 1e-6, std::atoi(argv[5]));
            res.first.saveToFile(argv[3]);
            CompressedImage::decompress(res.first).saveToFile(argv[4]);
            std::cout << res.second;
        } else if (mode == "quantize" && argc == 8) {
            const size_t N = std::stoul(argv[3]), D = std::stoul(argv[4]), bits = std::stoul(argv[5]);
            std::vector<char> raw = slurp(argv[2]);
            if (raw.size() != N * D * 8) return 3;
            std::vector<Vector> X(N, Vector(D));
            for (size_t i = 0; i < N; i++) std::memcpy(X[i].data(), raw.data() + i * D * 8, D * 8);
            auto [C, A, dist] = getQuantizer(Quantizers::LBG)->quantize(X, bits, 1e-6);
            std::ofstream fc(argv[6], std::ios::binary), fa(argv[7], std::ios::binary);
            for (auto &c : C) fc.write(reinterpret_cast<const char *>(c.data()), (std::streamsize)(c.size() * 8));
            for (size_t a : A) {
                const uint32_t v = (uint32_t)a;
                fa.write(reinterpret_cast<const char *>(&v), 4);
            }
            std::printf("distortion %.17g\n", dist);
        } else {
            return 2;
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 4;
    }
    if (g_fail) std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return g_fail ? 1 : 0;
}
