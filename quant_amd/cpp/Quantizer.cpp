// getQuantizer / the LBG quantizer on the engine; see include/quant_amd/Quantizer.hpp.
#include "quant_amd/Quantizer.hpp"

#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>

#include "engine_handle.hpp"

namespace quant_amd {

namespace {
struct CtxDeleter {
    void operator()(qvq_ctx *c) const { qvq_destroy(c); }
};
thread_local std::unique_ptr<qvq_ctx, CtxDeleter> t_ctx;
}  // namespace

qvq_ctx *EngineHandle::get() {
    if (!t_ctx) {
        const char *dev = std::getenv("QVQ_DEVICE");
        qvq_ctx *c = nullptr;
        const qvq_status st = qvq_create(dev ? std::atoi(dev) : 0, &c);
        if (st != QVQ_OK) throw std::runtime_error(std::string("qvq_create: ") + qvq_last_error(nullptr));
        t_ctx.reset(c);
    }
    return t_ctx.get();
}

void EngineHandle::check(qvq_status st, const char *what) {
    if (st == QVQ_OK) return;
    const char *msg = qvq_last_error(t_ctx.get());
    throw std::runtime_error(std::string(what) + " failed (status " + std::to_string((int)st) + "): " +
                             (msg ? msg : ""));
}

}  // namespace quant_amd

namespace {

// LBGQuantizer::quantize (src/Quantizer.cpp:119-144) on the engine.  The training set is
// copied into one flat fp64 array.  Byte images of the NORMAL or SCALED colour space take the
// byte engine; any other finite data (CIE1931 values, arbitrary doubles) the engine's exact
// mode, the reference's arithmetic; non-finite values: std::runtime_error.
class HipLBGQuantizer : public AbstractQuantizer {
public:
    std::tuple<std::vector<Vector>, std::vector<size_t>, VectorType> quantize(const std::vector<Vector> &trainingSet,
                                                                              size_t n, VectorType eps) override {
        using quant_amd::EngineHandle;
        if (trainingSet.empty()) throw std::runtime_error("LBG quantize: empty training set");
        const size_t N = trainingSet.size(), D = trainingSet[0].size();
        std::vector<double> flat(N * D);
        for (size_t i = 0; i < N; i++) {
            if (trainingSet[i].size() != D) throw std::runtime_error("LBG quantize: vectors of different sizes");
            std::copy(trainingSet[i].begin(), trainingSet[i].end(), flat.begin() + i * D);
        }
        qvq_ctx *ctx = EngineHandle::get();
        EngineHandle::check(qvq_set_vectors(ctx, flat.data(), N, (uint32_t)D), "qvq_set_vectors");
        const size_t K = (size_t)1 << n;
        std::vector<double> C(K * D);
        std::vector<uint32_t> A(N);
        double distortion = 0;
        EngineHandle::check(qvq_lbg(ctx, (uint32_t)n, eps, C.data(), A.data(), &distortion), "qvq_lbg");
        std::vector<Vector> codebook(K, Vector(D));
        for (size_t k = 0; k < K; k++) std::copy(C.begin() + k * D, C.begin() + (k + 1) * D, codebook[k].begin());
        return std::make_tuple(std::move(codebook), std::vector<size_t>(A.begin(), A.end()), distortion);
    }
};

}  // namespace

QuantizerPtr getQuantizer(Quantizers q) {
    if (q == Quantizers::LBG) return QuantizerPtr(new HipLBGQuantizer());
    return nullptr;
}
