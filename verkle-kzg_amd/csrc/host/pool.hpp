// Persistent host worker pool for the library's parallel host loops (verkle node walks and row
// building, per-proof IPA rounds, multiproof transcript records). Spawning and joining 16 threads
// per loop cost ~0.3-0.8 ms; the pool's threads wait on a condition variable between loops and
// are never joined (the pool lives until process exit). Header-only: one pool per process.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace vk {

class HostPool {
public:
    explicit HostPool(unsigned n) : n_(n) {
        for (unsigned k = 1; k < n; k++) th_.emplace_back([this, k] { loop(k); });
    }
    unsigned size() const { return n_; }
    // f(k) for every k < size(), k == 0 on the calling thread; one loop at a time. A loop
    // started from inside a job (a worker, or the caller's own f(0)) runs serially on that thread
    // instead of waiting for the pool it occupies. The first exception thrown by any f(k) is
    // rethrown here once every worker has finished its part.
    void run(const std::function<void(unsigned)>& f) {
        if (n_ == 1 || in_job()) {
            for (unsigned k = 0; k < n_; k++) f(k);
            return;
        }
        std::lock_guard<std::mutex> one(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            pending_ = n_ - 1;
            err_ = nullptr;
            gen_++;
        }
        cv_.notify_all();
        call(f, 0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
        if (err_) std::rethrow_exception(std::exchange(err_, nullptr));
    }

private:
    static bool& in_job() {
        static thread_local bool flag = false;
        return flag;
    }
    void call(const std::function<void(unsigned)>& f, unsigned k) {
        in_job() = true;
        try {
            f(k);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu_);
            if (!err_) err_ = std::current_exception();
        }
        in_job() = false;
    }
    void loop(unsigned k) {
        unsigned seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                f = job_;
            }
            call(*f, k);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    unsigned n_;
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    std::exception_ptr err_;
    unsigned pending_ = 0, gen_ = 0;
};
inline HostPool& host_pool() {
    static HostPool* p = new HostPool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    return *p;
}

// std::vector whose resize leaves new elements uninitialised (value-init only when asked): the
// host staging of big batched calls (verkle rows, outputs) is written in full right after, and
// zero-filling 8-16 MB per level on one thread cost ~1 ms per level
template <class T>
struct default_init_alloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = default_init_alloc<U>;
    };
    using std::allocator<T>::allocator;
    template <class U, class... Args>
    void construct(U* p, Args&&... args) {
        if constexpr (sizeof...(Args) == 0) ::new (static_cast<void*>(p)) U;
        else ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
    }
};
template <class T>
using uvec = std::vector<T, default_init_alloc<T>>;

// fn(i) for i in [lo, hi) on the pool in contiguous ranges, or serially below `min_par` items
template <class Fn>
inline void pool_for(size_t lo, size_t hi, size_t min_par, Fn&& fn) {
    HostPool& P = host_pool();
    const size_t count = hi - lo;
    if (count < min_par || P.size() == 1) {
        for (size_t i = lo; i < hi; i++) fn(i);
        return;
    }
    const unsigned T = P.size();
    P.run([&](unsigned k) {
        for (size_t i = lo + count * k / T; i < lo + count * (k + 1) / T; i++) fn(i);
    });
}

}  // namespace vk
