// quant_amd C++ API -- the quantizer plugin interface (reference: include/Quantizer.hpp:8-20,
// src/Quantizer.cpp:119-155), with LBG running on the MI355X engine (include/qvq.h).
#pragma once
#include <cstddef>
#include <memory>
#include <tuple>
#include <vector>

#include "VectorOperations.hpp"

enum class Quantizers { LBG, MEDIAN_CUT, LBG_MEDIAN_CUT, ABC };

class AbstractQuantizer {
public:
    // (codebook 2^n x D, assigned code vector per training vector, distortion)
    virtual std::tuple<std::vector<Vector>, std::vector<size_t>, VectorType> quantize(
        const std::vector<Vector> &trainingSet, size_t n, VectorType eps) = 0;
    virtual ~AbstractQuantizer() = default;
};

typedef std::unique_ptr<AbstractQuantizer> QuantizerPtr;

// LBG -> the engine's split-LBG on HIP device QVQ_DEVICE (default 0); the other
// enumerators have no implementation, as in the reference, and give nullptr.
QuantizerPtr getQuantizer(Quantizers);
