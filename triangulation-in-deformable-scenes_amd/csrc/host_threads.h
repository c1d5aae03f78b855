// Host-side data-parallel loops of the plan build and the upload.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace deftri {

// [0, n) in contiguous chunks on up to 16 host threads (DEFTRI_HOST_THREADS); f(chunk, lo, hi).
// Callers write disjoint ranges or per-chunk counters merged in chunk order, so their results do not
// depend on the split
template <class F>
int chunked(int64_t n, int64_t min_chunk, F f) {
    static const int env_t = std::getenv("DEFTRI_HOST_THREADS") ? std::atoi(std::getenv("DEFTRI_HOST_THREADS")) : 0;
    const int hw = env_t > 0 ? env_t : (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)hw, 16, n / std::max<int64_t>(min_chunk, 1)}));
    if (nt <= 1) { f(0, (int64_t)0, n); return 1; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) {
        const int64_t b = n * t / nt, e = n * (t + 1) / nt;
        th.emplace_back([=, &f] { f(t, b, e); });
    }
    for (auto &x : th) x.join();
    return nt;
}

}  // namespace deftri
