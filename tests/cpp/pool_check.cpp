// Host pool (csrc/host/pool.hpp) behaviour the library relies on: every index runs exactly once,
// back-to-back loops, a loop started from inside a job runs serially instead of deadlocking, an
// exception thrown by any part reaches the caller after the workers finished, and the pool is
// usable again afterwards. Prints one JSON line.
#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "../../verkle-kzg_amd/csrc/host/pool.hpp"

int main() {
    vk::HostPool& P = vk::host_pool();
    int fails = 0;
    // 1. coverage: pool_for over ragged ranges, many loops in a row
    for (size_t n : {0u, 1u, 7u, 16u, 17u, 1000u, 4097u}) {
        for (int rep = 0; rep < 50; rep++) {
            std::vector<std::atomic<int>> hit(n);
            for (auto& h : hit) h = 0;
            vk::pool_for(0, n, 1, [&](size_t i) { hit[i]++; });
            for (auto& h : hit) fails += h != 1;
        }
    }
    // 2. nested: a job that starts a loop (serial on its thread)
    std::atomic<int> inner{0};
    P.run([&](unsigned) { vk::pool_for(0, 64, 1, [&](size_t) { inner++; }); });
    fails += inner != (int)(64 * P.size());
    // 3. exceptions from a worker and from the caller's own part
    for (unsigned thrower : {P.size() - 1, 0u}) {
        std::atomic<int> ran{0};
        bool caught = false;
        try {
            P.run([&](unsigned k) {
                ran++;
                if (k == thrower) throw std::runtime_error("part failed");
            });
        } catch (const std::runtime_error&) {
            caught = true;
        }
        fails += !caught;
        fails += ran != (int)P.size();  // every part ran before the rethrow
    }
    // 4. still usable
    std::atomic<long> sum{0};
    vk::pool_for(0, 100000, 1, [&](size_t i) { sum += (long)i; });
    fails += sum != 4999950000L;
    printf("{\"threads\": %u, \"fails\": %d}\n", P.size(), fails);
    return fails != 0;
}
