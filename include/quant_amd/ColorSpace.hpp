// quant_amd C++ API -- colour spaces (reference: include/ColorSpace.hpp, src/ColorSpace.cpp).
// NORMAL: the signed byte as a double.  SCALED: (byte + 128) / 255.  CIE1931: the
// reference's linear maps (host conversions; the engine sums NORMAL/SCALED byte images exactly,
// and CIE1931 training sets go through its exact mode, the reference's Kahan arithmetic).
#pragma once
#include <memory>

#include "RGBImage.hpp"

enum class ColorSpaces { NORMAL, SCALED, CIE1931 };

class ColorSpace {
public:
    virtual RGBDouble RGBtoColorSpace(const RGB &);
    virtual RGB colorSpaceToRGB(const RGBDouble &);
    virtual ~ColorSpace() = default;
};

typedef std::unique_ptr<ColorSpace> ColorSpacePtr;

ColorSpacePtr getColorSpace(ColorSpaces);
