// host_par.hpp -- host loops over large problems (a global BA's 1.5 M edges) on up to 16 threads,
// in contiguous ranges; small problems (a local BA) stay on the calling thread.
#pragma once
#include <algorithm>
#include <thread>
#include <vector>

namespace orbgpu {

// f(a, b) over [0, n): T ranges of ceil(n / T), the first one on the calling thread
template <class F>
void host_parallel(int n, F f, int minN = 1 << 18) {
    const int hw = (int)std::thread::hardware_concurrency();
    const int T = n >= minN ? std::max(1, std::min(16, hw)) : 1;
    if (T <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    const int chunk = (n + T - 1) / T;
    for (int t = 1; t < T; t++) {
        const int a = t * chunk, b = std::min(n, a + chunk);
        if (a < b) th.emplace_back([&f, a, b] { f(a, b); });
    }
    f(0, std::min(n, chunk));
    for (auto& x : th) x.join();
}

}  // namespace orbgpu
