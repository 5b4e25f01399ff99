// Host-side sanitizer test ("-fsanitize=address on host tests").
// Built by tests/cpp/Makefile (target `sanitize`) with -fsanitize=address,undefined over the
// product's host C++ -- the reference kd-tree (quant_amd/csrc/kdtree.cpp), the bounded-wait
// policy (wait.hpp), the codec's host code (quant_amd/cpp/*.cpp: .quant writer/reader, PPM IO,
// colour spaces, tiling) -- and run on the CPU by tests/test_host_sanitize.py.  No GPU: the
// engine calls in quant_amd/cpp are linked (libqvq.so) but never reached.  The kd-tree is
// checked against the oracle's restatement (oracle/lbg_oracle.c, test infrastructure).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "kdtree.hpp"
#include "quant_amd/ColorSpace.hpp"
#include "quant_amd/Compressor.hpp"
#include "quant_amd/RGBImage.hpp"
#include "wait.hpp"

#include <cmath>
#include <functional>
#include <thread>

extern "C" void orc_kdtree_nn(const double *C, size_t K, int D, const double *Q, size_t nq, uint32_t *out);

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                                       \
        }                                                                     \
    } while (0)

// RefKDTree (nanoflann rules) against the oracle's kd-tree, on codebooks with duplicate
// points, equal coordinates and exact ties; the flattened device image filled too.
static void test_kdtree() {
    std::mt19937_64 rng(7);
    for (int D : {1, 3, 12, 48}) {
        for (size_t K : {1, 2, 5, 11, 64, 300, 1024, 4096}) {   // (>= 1024: the forked build)
            std::vector<double> C(K * D), Q;
            std::uniform_int_distribution<int> q8(0, 7);
            for (size_t i = 0; i < K; i++)
                for (int d = 0; d < D; d++) C[i * D + d] = (i % 3 == 2 && i > 0) ? C[(i - 1) * D + d] : q8(rng) * 0.125;
            for (size_t i = 0; i < 400; i++)
                for (int d = 0; d < D; d++) Q.push_back(q8(rng) * 0.125 + (i % 2 ? 0.0625 : 0.0));
            for (size_t i = 0; i < K; i++) Q.insert(Q.end(), C.begin() + i * D, C.begin() + (i + 1) * D);
            const size_t nq = Q.size() / D;
            std::vector<uint32_t> want(nq);
            orc_kdtree_nn(C.data(), K, D, Q.data(), nq, want.data());
            qvq::RefKDTree t(C.data(), K, D);
            for (size_t i = 0; i < nq; i++) CHECK(t.nearest(Q.data() + i * D) == want[i]);
            std::vector<qvq::KdNodeDev> nodes(t.num_nodes());
            std::vector<uint32_t> vind(K);
            std::vector<double> lo(D), hi(D);
            t.flatten(nodes.data(), vind.data(), lo.data(), hi.data());
            std::vector<int> seen(K, 0);
            for (uint32_t v : vind) CHECK(v < K && !seen[v]++);
            // the device build's image of this tree (breadth-first ids) imported back: node for
            // node the same tree (RefKDTree's image constructor renumbers depth first)
            std::vector<uint8_t> img(qvq::kdb_host_layout((uint32_t)K, (uint32_t)D).total);
            t.to_device_image(img.data());
            qvq::RefKDTree u(C.data(), K, D, img.data());
            std::string why;
            CHECK(t.same_as(u, &why));
            if (!why.empty()) std::fprintf(stderr, "import K=%zu D=%d: %s\n", K, D, why.c_str());
            for (size_t i = 0; i < nq; i += 7) CHECK(u.nearest(Q.data() + i * D) == want[i]);
        }
    }
}

// The tie certificate's host state (kdtree.cpp: recycled 64-byte aligned scratch, the
// aggregates built on one thread or split over threads by dimension, node-split replays,
// collecting replays, cert_update): the same answers either way, for trees built one after
// another (buffers passed from tree to tree), under the sanitizers.
static void test_certificate() {
    std::mt19937_64 rng(11);
    const double delta = std::ldexp(1.0, -49);
    auto threads = [](unsigned n, const std::function<void(unsigned)> &fn) {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < n; t++) th.emplace_back(fn, t);
        fn(0);
        for (auto &x : th) x.join();
    };
    for (int D : {12, 48}) {
        for (size_t K : {64, 512, 2048}) {
            std::vector<double> C(K * D);
            std::uniform_int_distribution<int> q8(0, 7);
            for (size_t i = 0; i < K; i++)
                for (int d = 0; d < D; d++) C[i * D + d] = (i % 5 == 4) ? 0.0 : q8(rng) * 0.1 + 0.05;
            std::vector<uint8_t> known0(K * D);
            for (size_t i = 0; i < K * D; i++) known0[i] = C[i] == 0.0 || (rng() % 4 == 0);
            std::vector<double> Q;
            for (int i = 0; i < 24; i++)
                for (int d = 0; d < D; d++) Q.push_back(q8(rng) * 0.1);
            int64_t first[24];
            for (int pass = 0; pass < 2; pass++) {
                std::vector<uint8_t> known(known0);   // (each pass from the same known split)
                qvq::RefKDTree t(C.data(), K, D);
                t.cert_clear();
                if (pass == 0) t.cert_warm(delta, C.data(), known.data());
                else t.cert_warm(delta, C.data(), known.data(), 3, threads);
                if (K <= 512) t.cert_prepare(delta, C.data(), known.data());
                std::vector<uint32_t> blame;
                for (int i = 0; i < 24; i++) {
                    const int64_t a = t.certified_search(Q.data() + (size_t)i * D, delta, C.data(), known.data());
                    CHECK(a >= -1 && a < (int64_t)K);
                    if (pass == 0) first[i] = a;
                    else CHECK(a == first[i]);
                    if (a < 0) t.certify_blame(Q.data() + (size_t)i * D, delta, C.data(), known.data(), blame);
                }
                for (uint32_t p : blame) {
                    CHECK(p < K);
                    std::fill(known.begin() + (size_t)p * D, known.begin() + (size_t)(p + 1) * D, 1);
                }
                t.cert_update(blame.data(), blame.size());
                for (int i = 0; i < 24; i++) {
                    const int64_t a = t.certified_search(Q.data() + (size_t)i * D, delta, C.data(), known.data());
                    CHECK(a >= -1 && a < (int64_t)K);
                }
            }
        }
    }
}

// wait_until (wait.hpp) under scripted probes: publish, timeout, peer failure, stream failure,
// drained stream.
static void test_wait() {
    using qvq::CommState;
    using qvq::StreamState;
    std::string err;
    int n = 0;
    CHECK(qvq::wait_until([&] { return ++n > 1000; }, [](std::string &) { return StreamState::Running; },
                          [](std::string &) { return CommState::None; }, 5.0, err) == QVQ_OK);
    CHECK(qvq::wait_until([] { return false; }, [](std::string &) { return StreamState::Running; },
                          [](std::string &) { return CommState::None; }, 0.05, err) == QVQ_EDEVICE);
    CHECK(qvq::wait_until([] { return false; }, [](std::string &) { return StreamState::Running; },
                          [](std::string &) { return CommState::Healthy; }, 0.05, err) == QVQ_ECOMM);
    CHECK(qvq::wait_until([] { return false; }, [](std::string &) { return StreamState::Running; },
                          [](std::string &m) { m = "peer"; return CommState::Failed; }, 5.0, err) == QVQ_ECOMM);
    CHECK(qvq::wait_until([] { return false; }, [](std::string &m) { m = "fault"; return StreamState::Failed; },
                          [](std::string &) { return CommState::None; }, 5.0, err) == QVQ_EDEVICE);
    CHECK(qvq::wait_until([] { return false; }, [](std::string &) { return StreamState::Drained; },
                          [](std::string &) { return CommState::None; }, 5.0, err) == QVQ_EDEVICE);
}

// The codec's host code: tiling <-> untiling round trips (src/test.cpp's cases and ragged
// sizes), colour spaces, .quant save/load (incl. a truncated file), PPM write/read.
static void test_codec(const std::string &tmp) {
    std::mt19937 rng(3);
    for (auto wh : std::vector<std::pair<int, int>>{{1, 1}, {2, 2}, {1, 3}, {2, 4}, {4, 4}, {3, 5}}) {
        for (auto xy : std::vector<std::pair<int, int>>{{4, 4}, {7, 5}, {16, 9}}) {
            RGBImage img;
            img.xSize = xy.first;
            img.ySize = xy.second;
            img.img.resize((size_t)img.xSize * img.ySize);
            for (auto &px : img.img)
                for (auto &c : px) c = (char)(rng() & 0xFF);
            for (ColorSpaces csn : {ColorSpaces::NORMAL, ColorSpaces::SCALED}) {
                const ColorSpacePtr cs = getColorSpace(csn);
                const auto blocks = getBlocksAsVectorsFromImage(img, wh.first, wh.second, cs);
                const auto bytes = vectorsToCharVectorsColorSpaced(blocks, cs);
                const RGBImage back = getImageFromVectors(bytes, img.xSize, img.ySize, wh.first, wh.second);
                CHECK(back.img.size() == img.img.size());
            }
        }
    }
    for (size_t bits : {1, 4, 8, 9, 12}) {
        CompressedImage c;
        c.xSize = 37;
        c.ySize = 21;
        c.blockWidth = 2;
        c.blockHeight = 3;
        const size_t D = c.blockWidth * c.blockHeight * 3, nb = ((c.xSize + 1) / 2) * ((c.ySize + 2) / 3);
        c.codeVectors.assign((size_t)1 << bits, CharVector(D));
        for (auto &cv : c.codeVectors)
            for (auto &b : cv) b = (char)(rng() & 0xFF);
        for (size_t i = 0; i < nb; i++) c.assignedCodeVector.push_back(rng() % ((size_t)1 << bits));
        const std::string path = tmp + "/rt.quant";
        c.saveToFile(path);
        CompressedImage d;
        d.loadFromFile(path);
        CHECK(d.codeVectors.size() == c.codeVectors.size() && d.assignedCodeVector == c.assignedCodeVector);
        for (size_t k = 0; k < c.codeVectors.size(); k++)
            CHECK(std::memcmp(d.codeVectors[k].data(), c.codeVectors[k].data(), D) == 0);
        CHECK(d.sizeInBits() == c.sizeInBits());
        {   // truncated: an exception, no out-of-bounds access
            std::ifstream in(path, std::ios::binary);
            std::string all((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
            std::ofstream out(tmp + "/trunc.quant", std::ios::binary);
            out.write(all.data(), (std::streamsize)(all.size() / 2));
        }
        bool threw = false;
        try {
            CompressedImage e;
            e.loadFromFile(tmp + "/trunc.quant");
        } catch (const std::runtime_error &) {
            threw = true;
        }
        CHECK(threw);
    }
    RGBImage img;
    img.xSize = 5;
    img.ySize = 3;
    img.img.resize(15);
    for (auto &px : img.img)
        for (auto &c : px) c = (char)(rng() & 0xFF);
    img.saveToFile(tmp + "/t.ppm");
    RGBImage back(tmp + "/t.ppm");
    CHECK(back.xSize == 5 && back.ySize == 3 && back.img == img.img);
}

int main(int argc, char **argv) {
    const std::string tmp = argc > 1 ? argv[1] : ".";
    test_kdtree();
    test_certificate();
    test_wait();
    test_codec(tmp);
    std::printf("host sanitize test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
