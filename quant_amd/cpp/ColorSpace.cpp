// Colour spaces; see include/quant_amd/ColorSpace.hpp.
#include "quant_amd/ColorSpace.hpp"

#include <cmath>
#include <cstdint>

namespace {

// The reference converts the rounded double straight to char; on its x86 builds that keeps
// the low byte of the integer, which is what SCALED's (c - 128) * 255 relies on.
inline char low_byte(double rounded) { return (char)(uint8_t)((int64_t)rounded & 0xFF); }

class ScaledSpace : public ColorSpace {
public:
    RGBDouble RGBtoColorSpace(const RGB &c) override {
        RGBDouble r;
        for (int i = 0; i < 3; i++) r[i] = ((double)c[i] + 128.0) / 255;
        return r;
    }
    RGB colorSpaceToRGB(const RGBDouble &c) override {
        RGB r;
        for (int i = 0; i < 3; i++) r[i] = low_byte(std::round((c[i] - 128.0) * 255));
        return r;
    }
};

class Cie1931Space : public ColorSpace {
public:
    RGBDouble RGBtoColorSpace(const RGB &c) override {
        const double r = c[0], g = c[1], b = c[2], n = 0.17697;
        return {(r * 0.490 + g * 0.310 + b * 0.200) / n, (r * 0.17697 + g * 0.81240 + b * 0.01063) / n,
                (r * 0 + g * 0.01 + b * 0.99) / n};
    }
    RGB colorSpaceToRGB(const RGBDouble &c) override {
        const double r = c[0] * 0.418 + c[1] * (-0.15866) + c[2] * (-0.082835);
        const double g = c[0] * (-0.091169) + c[1] * 0.25243 + c[2] * 0.015708;
        const double b = c[0] * 0.0009209 + c[1] * (-0.0025498) + c[2] * 0.17860;
        return {low_byte(std::round(r)), low_byte(std::round(g)), low_byte(std::round(b))};
    }
};

}  // namespace

RGBDouble ColorSpace::RGBtoColorSpace(const RGB &c) { return {(double)c[0], (double)c[1], (double)c[2]}; }

RGB ColorSpace::colorSpaceToRGB(const RGBDouble &c) {
    return {low_byte(std::round(c[0])), low_byte(std::round(c[1])), low_byte(std::round(c[2]))};
}

ColorSpacePtr getColorSpace(ColorSpaces cs) {
    switch (cs) {
    case ColorSpaces::NORMAL: return ColorSpacePtr(new ColorSpace());
    case ColorSpaces::SCALED: return ColorSpacePtr(new ScaledSpace());
    case ColorSpaces::CIE1931: return ColorSpacePtr(new Cie1931Space());
    }
    return nullptr;
}
