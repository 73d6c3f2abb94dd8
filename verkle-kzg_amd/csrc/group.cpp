// One process, several GPUs (include/vc_group.h): one vc_ctx and one host worker per member; every
// call runs the members' shares concurrently and combines them in host memory. The reference's
// callers are single-process (vector-commit/src/lib.rs:70-174, multiproof.rs:119-144 with rayon),
// so this is the shape a stateless `impl VectorCommitment` needs to use a whole node without
// becoming SPMD itself (the vc_comm.h entry points remain for one-process-per-GPU deployments).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/vc_group.h"
#include "comm.hpp"
#include "ctx.hpp"

namespace {

// G workers; run(f) calls f(k) for every member k concurrently (k = 0 on the caller's thread) and
// returns when all have finished. Threads live as long as the group. An exception out of f(k)
// (std::bad_alloc from a vc_* call's host vectors) is caught on whichever thread ran it and
// reported through failed(k) after every member has finished: the caller's f outlives every
// worker that still runs it.
class Team {
public:
    explicit Team(int n) : n_(n), failed_(n, 0) {
        for (int k = 1; k < n; k++) th_.emplace_back([this, k] { loop(k); });
    }
    ~Team() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::function<void(int)>& f) {
        for (auto& x : failed_) x = 0;
        if (n_ == 1) {
            guarded(f, 0);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            pending_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        guarded(f, 0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    // member k's share threw in the last run (its status slot may not have been written)
    bool failed(int k) const { return failed_[k] != 0; }

private:
    void guarded(const std::function<void(int)>& f, int k) {
        try {
            f(k);
        } catch (...) {
            failed_[k] = 1;
        }
    }

private:
    void loop(int k) {
        unsigned seen = 0;
        for (;;) {
            const std::function<void(int)>* f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (quit_) return;
                f = job_;
            }
            guarded(*f, k);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<char> failed_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int pending_ = 0;
    unsigned gen_ = 0;
    bool quit_ = false;
};

// grow-only device buffer on one device (the member's input staging)
struct MemBuf {
    int dev = 0;
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return VC_OK;
        VK_CHECK_HIP(hipSetDevice(dev));
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        VK_CHECK_HIP(hipMalloc(&p, bytes ? bytes : 16));
        cap = bytes ? bytes : 16;
        return VC_OK;
    }
    ~MemBuf() {
        if (p) {
            (void)hipSetDevice(dev);
            (void)hipFree(p);
        }
    }
};

// the first failing member's status
int first_error(const std::vector<int>& st) {
    for (int s : st)
        if (s != VC_OK) return s;
    return VC_OK;
}

}  // namespace

struct vc_group {
    int curve = 0;
    std::vector<vc_ctx*> ctx;
    std::vector<std::vector<int>> tables;  // [group table id][member] -> member table id
    std::vector<MemBuf> data, sums;        // per member: input staging, multiproof sums
    std::vector<int> peer;                 // [from * G + to]: VC_GROUP_PEER_* (vc_group_peer_path)
    int split = VC_GROUP_SPLIT_AUTO;
    std::mutex mu;  // one group call at a time
    Team* team = nullptr;
    int size() const { return (int)ctx.size(); }
    bool table_ok(int id) const { return id >= 0 && id < (int)tables.size(); }
    // f(k) on every member; a share that threw reports VC_E_OOM in st[k]. Returns the first error.
    int run(std::vector<int>& st, const std::function<void(int)>& f) {
        team->run(f);
        for (int k = 0; k < size(); k++)
            if (team->failed(k)) st[k] = VC_E_OOM;
        return first_error(st);
    }
};

extern "C" {

int vc_group_create(int curve, int ndev, const int* devices, vc_group** out) {
    if (!out || ndev < 1 || ndev > 64) return VC_E_INVALID;
    *out = nullptr;
    vc_group* g = new vc_group();
    g->curve = curve;
    for (int k = 0; k < ndev; k++) {
        vc_ctx* c = nullptr;
        const int st = vc_ctx_create(curve, devices ? devices[k] : k, &c);
        if (st != VC_OK) {
            for (auto* x : g->ctx) vc_ctx_destroy(x);
            delete g;
            return st;
        }
        g->ctx.push_back(c);
    }
    g->data.resize(ndev);
    g->sums.resize(ndev);
    for (int k = 0; k < ndev; k++) g->data[k].dev = g->sums[k].dev = g->ctx[k]->device;
    // direct peer access (xGMI) for every member pair whose devices allow it; otherwise the
    // device-to-device copies (multiproof sums to member 0) are staged through host memory by HIP
    g->peer.assign((size_t)ndev * ndev, VC_GROUP_PEER_SAME);
    for (int a = 0; a < ndev; a++)
        for (int b = 0; b < ndev; b++) {
            const int da = g->ctx[a]->device, db = g->ctx[b]->device;
            if (da == db) continue;
            int can = 0;
            int path = VC_GROUP_PEER_STAGED;
            if (hipDeviceCanAccessPeer(&can, da, db) == hipSuccess && can) {
                (void)hipSetDevice(da);
                const hipError_t e = hipDeviceEnablePeerAccess(db, 0);
                if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) path = VC_GROUP_PEER_DIRECT;
                (void)hipGetLastError();  // an already-enabled pair is not an error for later calls
            }
            g->peer[(size_t)a * ndev + b] = path;
        }
    g->team = new Team(ndev);
    *out = g;
    return VC_OK;
}

void vc_group_destroy(vc_group* g) {
    if (!g) return;
    delete g->team;
    g->data.clear();
    g->sums.clear();
    for (auto* c : g->ctx) vc_ctx_destroy(c);
    delete g;
}

int vc_group_size(const vc_group* g) { return g ? g->size() : VC_E_INVALID; }

int vc_group_peer_path(const vc_group* g, int from, int to) {
    if (!g || from < 0 || to < 0 || from >= g->size() || to >= g->size()) return VC_E_INVALID;
    return g->peer[(size_t)from * g->size() + to];
}

vc_ctx* vc_group_member(vc_group* g, int k) { return (g && k >= 0 && k < g->size()) ? g->ctx[k] : nullptr; }

int vc_group_member_table(const vc_group* g, int id, int member, int* member_table) {
    if (!g || !member_table || member < 0 || member >= g->size()) return VC_E_INVALID;
    if (!g->table_ok(id)) return VC_E_TABLE;
    *member_table = g->tables[id][member];
    return VC_OK;
}

int vc_group_set_msm_split(vc_group* g, int split) {
    if (!g || split < VC_GROUP_SPLIT_AUTO || split > VC_GROUP_SPLIT_POINTS) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    g->split = split;
    return VC_OK;
}

}  // extern "C"

namespace {

// a new group table from per-member creators
int new_table(vc_group* g, const std::function<int(int k, int* id)>& make, int* table_id) {
    const int G = g->size();
    std::vector<int> ids(G, -1), st(G, VC_OK);
    VK_TRY(g->run(st, [&](int k) { st[k] = make(k, &ids[k]); }));
    g->tables.push_back(ids);
    *table_id = (int)g->tables.size() - 1;
    return VC_OK;
}

}  // namespace

extern "C" {

int vc_group_bases_upload(vc_group* g, const uint64_t* xy, const uint8_t* inf, size_t n, int* table_id) {
    if (!g || !table_id || (n && !xy)) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    return new_table(g, [&](int k, int* id) { return vc_bases_upload(g->ctx[k], xy, inf, n, id); }, table_id);
}

int vc_group_bases_random(vc_group* g, uint64_t seed, size_t n, int* table_id) {
    if (!g || !table_id) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    return new_table(g, [&](int k, int* id) { return vc_bases_random(g->ctx[k], seed, n, id); }, table_id);
}

int vc_group_kzg_setup(vc_group* g, size_t max_items, const uint64_t* secret_fr, int* table_id, size_t* size) {
    if (!g || !table_id || !size || !secret_fr) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    std::vector<size_t> sz(g->size(), 0);
    VK_TRY(new_table(g, [&](int k, int* id) { return vc_kzg_setup(g->ctx[k], max_items, secret_fr, id, &sz[k]); },
                     table_id));
    *size = sz[0];
    return VC_OK;
}

int vc_group_fixed_base_precompute(vc_group* g, int id, int window_bits, int windows) {
    if (!g) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    std::vector<int> st(g->size(), VC_OK);
    return g->run(st, [&](int k) {
        st[k] = vc_fixed_base_precompute_windows(g->ctx[k], g->tables[id][k], window_bits, windows);
    });
}

int vc_group_msm(vc_group* g, int id, size_t offset, const uint64_t* scalars, size_t n, int mont, uint64_t* out_xy,
                 uint8_t* out_inf) {
    if (!g || !out_xy || !out_inf || (n && !scalars)) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    const int G = g->size();
    if (G == 1) return vc_msm(g->ctx[0], g->tables[id][0], offset, scalars, n, mont, out_xy, out_inf);
    const bool windows = g->split == VC_GROUP_SPLIT_WINDOWS;
    if (n < (size_t)G) return vc_msm(g->ctx[0], g->tables[id][0], offset, scalars, n, mont, out_xy, out_inf);
    const int words = vc_point_words(g->curve);
    std::vector<uint32_t> accs((size_t)words * G, 0);
    std::vector<int> st(G, VC_OK);
    VK_TRY(g->run(st, [&](int k) {
        auto share = [&]() -> int {
            uint32_t* acc = accs.data() + (size_t)k * words;
            if (!windows) {  // its own scalars only, copied in chunks under its own MSM (vc_msm_partial)
                size_t lo, hi;
                vk::shard_range(n, k, G, &lo, &hi);  // n >= G: no empty share
                return vc_msm_partial(g->ctx[k], g->tables[id][k], offset + lo, scalars + lo * 4, hi - lo, mont, acc);
            }
            VK_TRY(g->data[k].ensure(n * 32));
            VK_CHECK_HIP(hipSetDevice(g->ctx[k]->device));
            VK_CHECK_HIP(hipMemcpy(g->data[k].p, scalars, n * 32, hipMemcpyHostToDevice));
            return vc_msm_device_window_part(g->ctx[k], g->tables[id][k], offset, g->data[k].p, n, mont, k, G, acc);
        };
        st[k] = share();
    }));
    return vc_partials_sum(g->curve, accs.data(), G, out_xy, out_inf);
}

int vc_group_msm_batch(vc_group* g, int id, size_t width, const uint64_t* scalars, size_t batch, int mont,
                       uint64_t* out_xy, uint8_t* out_inf) {
    if (!g || width == 0 || (batch && (!scalars || !out_xy || !out_inf))) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    const int G = g->size();
    const size_t W2 = 2 * (size_t)vk::aff_limbs64(g->curve);
    std::vector<int> st(G, VC_OK);
    return g->run(st, [&](int k) {
        size_t lo, hi;
        vk::shard_range(batch, k, G, &lo, &hi);
        if (hi > lo)
            st[k] = vc_msm_batch(g->ctx[k], g->tables[id][k], width, scalars + lo * width * 4, hi - lo, mont,
                                 out_xy + lo * W2, out_inf + lo);
    });
}

int vc_group_kzg_prove(vc_group* g, int id, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                       uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y) {
    if (!g || !point || !proof_xy || !proof_inf || !y || (max && !evals) || max > size) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    const int G = g->size();
    if (G == 1) return vc_kzg_prove(g->ctx[0], g->tables[id][0], size, evals, max, point, proof_xy, proof_inf, y);
    const int words = vc_point_words(g->curve);
    std::vector<uint32_t> accs((size_t)words * G, 0);
    std::vector<uint64_t> ys((size_t)4 * G, 0);
    std::vector<int> st(G, VC_OK);
    if (g->split == VC_GROUP_SPLIT_WINDOWS) {  // every member the whole quotient, a window slice of the MSM
        VK_TRY(g->run(st, [&](int k) {
            auto share = [&]() -> int {
                VK_TRY(g->data[k].ensure(max * 32));
                VK_CHECK_HIP(hipSetDevice(g->ctx[k]->device));
                if (max) VK_CHECK_HIP(hipMemcpy(g->data[k].p, evals, max * 32, hipMemcpyHostToDevice));
                return vc_kzg_prove_device_part(g->ctx[k], g->tables[id][k], size, g->data[k].p, max, point, k, G,
                                                accs.data() + (size_t)k * words, &ys[(size_t)4 * k]);
            };
            st[k] = share();
        }));
        memcpy(y, ys.data(), 32);
        return vc_partials_sum(g->curve, accs.data(), G, proof_xy, proof_inf);
    }
    // index ranges: member k uploads f on its 1/G of the domain, computes q there
    // and the MSM over SRS points [lo, hi); the in-domain q_m (or the out-of-domain y) needs one
    // exchange of G field partials between the two phases
    std::vector<vk::KzgShare*> sh(G, nullptr);
    std::vector<uint64_t> parts((size_t)4 * G, 0);
    struct Free {
        std::vector<vk::KzgShare*>& s;
        ~Free() {
            for (auto* x : s) vk::kzg_share_free(x);
        }
    } free_shares{sh};
    VK_TRY(g->run(st, [&](int k) {
        size_t lo, hi;
        vk::shard_range(size, k, G, &lo, &hi);
        st[k] = vk::kzg_share_begin(g->ctx[k], g->tables[id][k], size, evals, max, point, lo, hi, &sh[k],
                                    &parts[(size_t)4 * k]);
    }));
    uint64_t total[4];
    VK_TRY(vk::kzg_share_sum(g->curve, parts.data(), G, total));
    VK_TRY(g->run(st, [&](int k) {
        st[k] = vk::kzg_share_finish(sh[k], total, accs.data() + (size_t)k * words, &ys[(size_t)4 * k]);
    }));
    memcpy(y, ys.data(), 32);
    return vc_partials_sum(g->curve, accs.data(), G, proof_xy, proof_inf);
}

int vc_group_multiproof_prove(vc_group* g, int scheme, int id, size_t N, size_t Q, const uint64_t* data,
                              const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                              uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proof, uint64_t* kzg_proof_xy,
                              uint8_t* kzg_proof_inf, uint64_t* kzg_y) {
    if (!g || !data || !com_xy || !com_inf || !z || !y || !d_xy || !d_inf || Q == 0) return VC_E_INVALID;
    if (scheme != 0 && scheme != 1) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    const int G = g->size();
    if (G == 1)
        return vc_multiproof_prove(g->ctx[0], scheme, g->tables[id][0], N, Q, data, com_xy, com_inf, z, y, d_xy, d_inf,
                                   ipa_proof, kzg_proof_xy, kzg_proof_inf, kzg_y);
    // phase 1 once (the serial transcript over all queries, multiproof.rs:106-115) on a helper
    // thread while the members upload their slices of the evaluations: the transcript needs none
    // of them, and the accumulate needs its challenge r
    size_t rows = 0;
    VK_TRY(vc_multiproof_rows(N, Q, z, &rows));
    const size_t sbytes = rows * N * 32;
    vc_transcript* tr = nullptr;
    uint64_t r[4];
    size_t rows_b = 0;
    int st_b = VC_E_INVALID;
    auto begin = [&] {
        try {
            st_b = vc_multiproof_begin(N, Q, com_xy, com_inf, z, y, &tr, r, &rows_b);
        } catch (...) {  // nothing may leave a thread function
            st_b = VC_E_OOM;
        }
    };
    std::thread th;
    try {
        th = std::thread(begin);
    } catch (const std::system_error&) {
        begin();  // no thread: the transcript first
    }
    // member 0 holds every member's sums contiguously (vc_multiproof_finish adds G parts)
    int st0 = g->sums[0].ensure(sbytes * G);
    std::vector<int> st(G, st0);
    if (st0 == VC_OK)
        g->run(st, [&](int k) {
            auto upload = [&]() -> int {
                size_t lo, hi;
                vk::shard_range(Q, k, G, &lo, &hi);
                if (hi == lo) return VC_OK;
                VK_CHECK_HIP(hipSetDevice(g->ctx[k]->device));
                VK_TRY(g->data[k].ensure((hi - lo) * N * 32));
                VK_CHECK_HIP(hipMemcpy(g->data[k].p, data + lo * N * 4, (hi - lo) * N * 32, hipMemcpyHostToDevice));
                if (k != 0) VK_TRY(g->sums[k].ensure(sbytes));
                return VC_OK;
            };
            st[k] = upload();
        });
    if (th.joinable()) th.join();
    if (st_b != VC_OK) {
        if (tr) vc_transcript_free(tr);
        return st_b;
    }
    if (first_error(st) == VC_OK)
        g->run(st, [&](int k) {
            auto share = [&]() -> int {
                size_t lo, hi;
                vk::shard_range(Q, k, G, &lo, &hi);
                uint8_t* dst0 = static_cast<uint8_t*>(g->sums[0].p) + (size_t)k * sbytes;
                if (hi == lo) {  // an empty slice (Q < G) contributes zero sums, cleared on the stream
                    // vc_multiproof_finish reads them on
                    VK_CHECK_HIP(hipSetDevice(g->ctx[0]->device));
                    VK_CHECK_HIP(hipMemsetAsync(dst0, 0, sbytes, g->ctx[0]->stream));
                    VK_CHECK_HIP(hipStreamSynchronize(g->ctx[0]->stream));
                    return VC_OK;
                }
                VK_CHECK_HIP(hipSetDevice(g->ctx[k]->device));
                void* dS = k != 0 ? g->sums[k].p : static_cast<void*>(dst0);
                VK_TRY(vc_multiproof_accumulate(g->ctx[k], N, Q, z, lo, hi - lo, g->data[k].p, r, dS));
                if (k != 0)
                    VK_CHECK_HIP(hipMemcpyPeer(dst0, g->ctx[0]->device, dS, g->ctx[k]->device, sbytes));
                return VC_OK;
            };
            st[k] = share();
        });
    int s = first_error(st);
    if (s == VC_OK)
        s = vc_multiproof_finish(g->ctx[0], scheme, g->tables[id][0], N, Q, z, g->sums[0].p, G, tr, d_xy, d_inf,
                                 ipa_proof, kzg_proof_xy, kzg_proof_inf, kzg_y);
    vc_transcript_free(tr);
    return s;
}

int vc_group_multiproof_prove_many(vc_group* g, int scheme, int id, size_t N, size_t Q, size_t P,
                                   const uint64_t* data, const uint64_t* com_xy, const uint8_t* com_inf,
                                   const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                                   vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y) {
    if (!g || (P && (!data || !com_xy || !com_inf || !z || !y || !d_xy || !d_inf))) return VC_E_INVALID;
    if ((scheme != 0 && scheme != 1) || (P && scheme == 0 && !ipa_proofs) ||
        (P && scheme == 1 && (!kzg_xy || !kzg_inf || !kzg_y)))
        return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    const int G = g->size();
    std::vector<int> st(G, VC_OK);
    // each member's proofs in ONE upload and one vc_multiproof_prove_many (its proofs' transcripts
    // and GPU phases pipelined inside). Round 6 measured the alternative -- sub-batches over two
    // device buffers, the next one's data crossing PCIe on an uploader thread while the current one
    // is proven -- and it was slower (G = 1 / 2 on one card, 4 proofs of 2^14 x 256: 13.9-15.0 /
    // 13.0-13.3 ms against 12.6 / 11.8-12.1, profiles/r06/group/): a proof's own latency (its
    // transcript, ~3 ms) exceeds one proof's upload (128 MB in ~2.5 ms), so splitting the call
    // costs the pipelining across proofs more than the overlap gives back
    return g->run(st, [&](int k) {
        auto share = [&]() -> int {
            size_t lo, hi;
            vk::shard_range(P, k, G, &lo, &hi);
            if (hi == lo) return VC_OK;
            const size_t bytes = (hi - lo) * Q * N * 32;
            VK_TRY(g->data[k].ensure(bytes));
            VK_CHECK_HIP(hipSetDevice(g->ctx[k]->device));
            VK_CHECK_HIP(hipMemcpy(g->data[k].p, data + lo * Q * N * 4, bytes, hipMemcpyHostToDevice));
            return vc_multiproof_prove_many(g->ctx[k], scheme, g->tables[id][k], N, Q, hi - lo, g->data[k].p,
                                            com_xy + lo * Q * 8, com_inf + lo * Q, z + lo * Q, y + lo * Q * 4,
                                            d_xy + lo * 8, d_inf + lo, scheme == 0 ? ipa_proofs + lo : nullptr,
                                            scheme == 1 ? kzg_xy + lo * 8 : nullptr,
                                            scheme == 1 ? kzg_inf + lo : nullptr, scheme == 1 ? kzg_y + lo * 4 : nullptr);
        };
        st[k] = share();
    });
}

int vc_group_verkle_commitment(vc_group* g, int id, vc_verkle* tree, uint64_t* out_xy, uint8_t* out_inf) {
    if (!g || !tree || !out_xy || !out_inf) return VC_E_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->table_ok(id)) return VC_E_TABLE;
    vk::Multi mu;
    mu.ctx = g->ctx;
    mu.table = g->tables[id];
    // a member share that threw fails the level: rethrown here, after every member has finished
    mu.run = [&](const std::function<void(int)>& f) {
        std::vector<int> st(g->size(), VC_OK);
        if (g->run(st, f) != VC_OK) throw std::bad_alloc();
    };
    try {
        return vk::verkle_commitment(g->ctx[0], g->tables[id][0], tree, out_xy, out_inf, nullptr, &mu);
    } catch (const std::bad_alloc&) {
        return VC_E_OOM;
    }
}

}  // extern "C"
