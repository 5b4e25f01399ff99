// quant_amd C++ API -- value types of the reference's interface
// (include/VectorOperations.hpp:10-12 there: VectorType = double, Vector and CharVector
// are boost small_vectors; std::vector carries the same values here).
#pragma once
#include <vector>

using VectorType = double;
using Vector = std::vector<VectorType>;
using CharVector = std::vector<char>;
