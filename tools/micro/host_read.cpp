// CPU read speed of hipHostMalloc(Mapped|Coherent) memory vs malloc (host-side diagnostics).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

int main() {
    const size_t n = 4096 * 48;
    double *h = nullptr;
    if (hipHostMalloc((void **)&h, n * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    for (size_t i = 0; i < n; i++) h[i] = (double)i;
    std::vector<double> local(n), dst(n);
    for (size_t i = 0; i < n; i++) local[i] = (double)i;
    for (int rep = 0; rep < 3; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        std::memcpy(dst.data(), h, n * 8);
        auto t1 = std::chrono::steady_clock::now();
        std::memcpy(dst.data(), local.data(), n * 8);
        auto t2 = std::chrono::steady_clock::now();
        double s = 0;
        for (size_t i = 0; i < n; i += 48 * 7 % n) s += h[(i * 48) % n];
        auto t3 = std::chrono::steady_clock::now();
        std::vector<double> fresh(n);
        for (size_t i = 0; i < n; i++) fresh[i] = 1.0;
        auto t4 = std::chrono::steady_clock::now();
        printf("mapped memcpy %.3f ms, local memcpy %.3f ms, mapped strided %.3f ms, fresh alloc+fill %.3f ms (%g)\n",
               std::chrono::duration<double, std::milli>(t1 - t0).count(),
               std::chrono::duration<double, std::milli>(t2 - t1).count(),
               std::chrono::duration<double, std::milli>(t3 - t2).count(),
               std::chrono::duration<double, std::milli>(t4 - t3).count(), s + fresh[5]);
    }
    return 0;
}
