// Verkle tree (reference verkle-tree/src/{lib,node}.rs) with level-batched commitments on the
// GPU engine. Host data structure + orchestration; all commitments go through
// vc_msm_batch_sparse (CSR rows of non-zeros against the fixed-base tables) and
// vc_to_data_item_batch. See include/vc_verkle.h.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <array>
#include <cstring>
#include <map>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../../include/vc_scheme.h"
#include "../../include/vc_verkle.h"
#include "ctx.hpp"
#include "comm.hpp"
#include "host/pool.hpp"
#include "host/fr.hpp"
#include "scheme_internal.hpp"

namespace {

using vk::Fr;

// a sorted run of entries whose first one lives inside the owner (an extension node of random
// keys holds one leaf: its rows are built from the node's own cache lines, no second miss into
// the heap); std::vector's API subset FlatMap uses
template <class T>
struct InlineVec {
    uint32_t n = 0;
    T inl[1];
    std::vector<T> heap;  // n >= 2: every entry here
    T* begin() { return n <= 1 ? inl : heap.data(); }
    T* end() { return begin() + n; }
    const T* begin() const { return n <= 1 ? inl : heap.data(); }
    const T* end() const { return begin() + n; }
    T* data() { return begin(); }
    const T* data() const { return begin(); }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    T* insert(T* it, const T& v) {
        const size_t k = (size_t)(it - begin());
        if (n == 0) {
            inl[0] = v;
            n = 1;
            return inl;
        }
        if (n == 1) heap.assign(inl, inl + 1);
        heap.insert(heap.begin() + (std::ptrdiff_t)k, v);
        n++;
        return heap.data() + k;
    }
};

// unit -> V, sorted by unit in one vector: the std::map API subset the tree uses, without a heap
// node per entry (pointer chasing made the commitment's node walks ~150 ns per node)
template <class V, class Vec = std::vector<std::pair<uint8_t, V>>>
struct FlatMap {
    Vec v;
    using iterator = decltype(v.begin());
    using const_iterator = decltype(static_cast<const Vec&>(v).begin());
    iterator begin() { return v.begin(); }
    iterator end() { return v.end(); }
    const_iterator begin() const { return v.begin(); }
    const_iterator end() const { return v.end(); }
    iterator lower(uint8_t k) {
        return std::lower_bound(v.begin(), v.end(), k, [](const std::pair<uint8_t, V>& a, uint8_t b) { return a.first < b; });
    }
    const_iterator lower(uint8_t k) const {
        return std::lower_bound(v.begin(), v.end(), k, [](const std::pair<uint8_t, V>& a, uint8_t b) { return a.first < b; });
    }
    iterator find(uint8_t k) {
        auto it = lower(k);
        return (it != v.end() && it->first == k) ? it : v.end();
    }
    const_iterator find(uint8_t k) const {
        auto it = lower(k);
        return (it != v.end() && it->first == k) ? it : v.end();
    }
    V& operator[](uint8_t k) {
        auto it = lower(k);
        if (it == v.end() || it->first != k) it = v.insert(it, {k, V{}});
        return it->second;
    }
};

// two cache lines (the row builders prefetch both); the commitment state is in vc_verkle's arrays
struct alignas(64) VNode {
    bool ext = false;
    int level = 0;                                           // internal: depth below the root
    std::array<uint8_t, 32> stem{};                          // extension: the full key (node.rs:45)
    using Leaf = std::pair<uint8_t, std::array<uint8_t, 32>>;
    FlatMap<std::array<uint8_t, 32>, InlineVec<Leaf>> leaves;  // extension: unit -> value
    FlatMap<int> children;                                   // internal: unit -> node
};

// LE bytes -> canonical Fr words (from_le_bytes_mod_order): < 31 bytes is already < r; 32
// bytes (< 2^256 < 6r) by at most five subtractions of r; longer inputs by the generic path
static void item_of_bytes(const uint8_t* b, size_t len, uint64_t out[4]) {
    if (len <= 32) {
        uint8_t w[32] = {0};
        memcpy(w, b, len);
        memcpy(out, w, 32);
        static const uint64_t R[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                                      0x30644e72e131a029ULL};  // BN254 r
        // v mod r with one quotient estimate: q = floor(v_3 / r_3) (<= 5) is floor(v / r) or one
        // more (r_3 ~ 2^61.6 dwarfs the lower limbs' share), so v - q r lies in [-r, r): one
        // conditional add (the compare-and-subtract loop it replaces mispredicted ~48 ns per stem)
        const uint64_t q = out[3] / R[3];
        typedef unsigned __int128 u128;
        u128 mc = 0, br = 0;
        for (int i = 0; i < 4; i++) {
            mc += (u128)q * R[i];
            const u128 d = (u128)out[i] - (uint64_t)mc - (uint64_t)br;
            out[i] = (uint64_t)d;
            br = (d >> 64) & 1;
            mc >>= 64;
        }
        if ((uint64_t)mc + (uint64_t)br) {  // negative: add r back
            u128 c = 0;
            for (int i = 0; i < 4; i++) {
                c += (u128)out[i] + R[i];
                out[i] = (uint64_t)c;
                c >>= 64;
            }
        }
        return;
    }
    vk::mont_to_canon<vk::BN254Fr>(vk::fe_from_le_bytes_mod<vk::BN254Fr>(b, len), out);
}

}  // namespace

// Device mirror of the tree's per-node results (one context's device): commitments, flags and
// to_data_item values indexed by node id, so a level's rows gather their children's items on the
// device and nothing travels back between levels (verkle_commitment_dev)
struct VerkleDev {
    uint64_t ctx_uid = 0;  // the context whose device holds it (0: none)
    int dev = -1;
    void* item = nullptr;  // [cap] x 4 u64 (the start of the one allocation)
    void* cxy = nullptr;   // [cap] x 8 u64
    void* inf = nullptr;   // [cap] u8
    size_t cap = 0, blk_bytes = 0;
    // the block comes from the context's pool and goes back to it (a fresh tree's mirror then
    // costs no hipMalloc: ~0.4 ms of a 4-ms full commitment)
    void release() {
        vk::pool_return_uid(ctx_uid, dev, item, blk_bytes);  // one block: item, then cxy, then inf
        item = cxy = inf = nullptr;
        cap = blk_bytes = 0;
        ctx_uid = 0;
        dev = -1;
    }
    ~VerkleDev() { release(); }
};

struct vc_verkle {
    int N = 3;
    std::vector<VNode> nodes;  // nodes[0] = root (internal)
    // per-node results (node id order): canonical affine commitment, identity flag, to_data_item
    std::vector<uint64_t> cxy;
    std::vector<uint8_t> cinf;
    std::vector<uint64_t> item;
    // per-node flags (compact: the commitment's bookkeeping touches no node lines)
    std::vector<uint8_t> has_commit, queued;
    // dirty nodes, kept at insert time: every extension, and the internal nodes by level (an insert
    // clears the commitments on its path; new nodes start dirty)
    std::vector<int> dirty_ext;
    std::vector<std::vector<int>> dirty_int;
    VerkleDev dev;
    bool host_valid = true;  // false: the device mirror holds newer results than cxy / cinf / item
    // delta updates (verkle_commitment_dev): base[id] = the node's stored commitment is its last
    // successful one, and every change of its slots since is in slog as (parent, slot, the child the
    // slot held then: -1 = empty) -- logged at insert time for base parents only
    struct SlotLog {
        int parent, old;
        uint8_t slot;
    };
    std::vector<uint8_t> base;
    std::vector<SlotLog> slog;
    // scratch of the commitment's delta plan, per node id (-1 outside a call): the node's plan /
    // its snapshot index (persistent arrays: no hash maps per call)
    std::vector<int32_t> plan_slot, snap_slot;
    void log_slot(int parent, uint8_t slot, int old) {
        if (base[parent]) slog.push_back({parent, old, slot});
    }
    int add(VNode&& n) {
        nodes.push_back(std::move(n));
        cxy.resize(cxy.size() + 8, 0);
        cinf.push_back(1);
        item.resize(item.size() + 4, 0);
        has_commit.push_back(0);
        queued.push_back(0);
        base.push_back(0);
        plan_slot.push_back(-1);
        snap_slot.push_back(-1);
        return (int)nodes.size() - 1;
    }
    void mark(int id) {  // commitment cleared (node.rs:150-152 commitment = None)
        has_commit[id] = 0;
        if (queued[id]) return;
        queued[id] = 1;
        const VNode& n = nodes[id];
        if (n.ext) {
            dirty_ext.push_back(id);
        } else {
            if ((int)dirty_int.size() <= n.level) dirty_int.resize(n.level + 1);
            dirty_int[n.level].push_back(id);
        }
    }
    size_t dirty_count() const {
        size_t c = dirty_ext.size();
        for (auto& lv : dirty_int) c += lv.size();
        return c;
    }
    void clear_dirty() {  // after a commitment: every listed node is committed
        for (int id : dirty_ext) has_commit[id] = 1, queued[id] = 0, base[id] = 1;
        for (auto& lv : dirty_int)
            for (int id : lv) has_commit[id] = 1, queued[id] = 0, base[id] = 1;
        dirty_ext.clear();
        dirty_int.clear();
        slog.clear();
    }
    // a failed commitment may have stored some dirty nodes' new results already: their stored
    // commitments are no delta bases any more (the retry recommits them in full)
    void drop_delta() {
        for (int id : dirty_ext) base[id] = 0;
        for (auto& lv : dirty_int)
            for (int id : lv) base[id] = 0;
        slog.clear();
    }
};

namespace {
// drop_delta unless the commitment reached its end (ok = true)
struct DeltaGuard {
    vc_verkle* t;
    bool ok = false;
    ~DeltaGuard() {
        if (!ok) t->drop_delta();
    }
};
}  // namespace

namespace {

int new_ext(vc_verkle* t, const uint8_t* stem, uint8_t unit, const uint8_t* value) {
    VNode n;
    n.ext = true;
    memcpy(n.stem.data(), stem, t->N);
    std::array<uint8_t, 32> v;
    memcpy(v.data(), value, 32);
    n.leaves[unit] = v;
    const int id = t->add(std::move(n));
    t->mark(id);
    return id;
}

// first d > cur with a[d] != b[d] (or N) -- KeyMethods::next_diff_depth (lib.rs:49-58)
int next_diff_depth(const uint8_t* a, const uint8_t* b, int cur, int N) {
    int d = cur + 1;
    while (d < N && a[d] == b[d]) d++;
    return d;
}

// get_stem (node.rs:74-95)
int find_stem(const vc_verkle* t, const uint8_t* stem) {
    int cur = 0, depth = 0;
    while (true) {
        const VNode& n = t->nodes[cur];
        if (n.ext) return memcmp(n.stem.data(), stem, t->N) == 0 ? cur : -1;
        if (depth >= t->N) return -1;
        auto it = n.children.find(stem[depth]);
        if (it == n.children.end()) return -1;
        cur = it->second;
        depth++;
    }
}

}  // namespace

extern "C" {

vc_verkle* vc_verkle_new(int key_len) {
    if (key_len < 2 || key_len > 32) return nullptr;
    vc_verkle* t = new vc_verkle();
    t->N = key_len;
    t->mark(t->add(VNode()));  // root: Node::new_internal(vec![]), level 0
    return t;
}

void vc_verkle_free(vc_verkle* t) { delete t; }

// Node::insert (node.rs:133-204), iteratively. The walk is checked before anything changes,
// so the reference's panic case leaves the tree untouched.
int vc_verkle_insert(vc_verkle* t, const uint8_t* key, const uint8_t* value) {
    if (!t || !key || !value) return VC_E_INVALID;
    const int N = t->N;
    const uint8_t* stem = key;       // split(): the stem keeps every unit (lib.rs:61-67)
    const uint8_t unit = key[N - 1];
    // dry run: find where the walk ends and reject the panic case first
    std::vector<int> path;
    int cur = 0, depth = 0;
    enum { INTO_EXT, NEW_EXT, SPLIT } action;
    int parent_k = -1;
    while (true) {
        path.push_back(cur);
        VNode& n = t->nodes[cur];
        if (n.ext) {
            if (memcmp(n.stem.data(), stem, N) != 0) return VC_E_INVALID;  // reference panics here
            action = INTO_EXT;
            break;
        }
        if (depth >= N) return VC_E_INVALID;
        const uint8_t k = stem[depth];
        auto it = n.children.find(k);
        if (it == n.children.end()) {
            action = NEW_EXT;
            parent_k = k;
            break;
        }
        VNode& c = t->nodes[it->second];
        if (c.ext && !(memcmp(c.stem.data(), stem, N) == 0 || depth == N - 2)) {
            // the reference indexes stem[d] out of bounds (panics) when no unit after `depth`
            // differs -- reachable only through its level-skipping splits
            if (next_diff_depth(c.stem.data(), stem, depth, N) >= N) return VC_E_INVALID;
            action = SPLIT;
            parent_k = k;
            break;
        }
        cur = it->second;
        depth++;
    }
    for (int p : path) t->mark(p);  // clear the commitments on the path
    // the path's slots (their children's items change) -- internal path[i] sits at depth i
    for (size_t i = 0; i + 1 < path.size(); i++) t->log_slot(path[i], stem[i], path[i + 1]);
    VNode* n = &t->nodes[cur];
    if (action == INTO_EXT) {
        std::array<uint8_t, 32> v;
        memcpy(v.data(), value, 32);
        n->leaves[unit] = v;
        return VC_OK;
    }
    if (action == NEW_EXT) {
        t->log_slot(cur, (uint8_t)parent_k, -1);
        int e = new_ext(t, stem, unit, value);
        t->nodes[cur].children[(uint8_t)parent_k] = e;
        return VC_OK;
    }
    // SPLIT: new internal keyed by the first differing unit d (which may skip levels, as in
    // the reference: node.rs:176-185)
    const int old = t->nodes[cur].children[(uint8_t)parent_k];
    t->log_slot(cur, (uint8_t)parent_k, old);
    const std::array<uint8_t, 32> old_stem = t->nodes[old].stem;
    const int d = next_diff_depth(old_stem.data(), stem, depth, N);
    int e = new_ext(t, stem, unit, value);
    VNode in;
    in.level = depth + 1;  // a child of `cur` (whose level is the walk depth)
    in.children[stem[d]] = e;
    in.children[old_stem[d]] = old;
    const int id = t->add(std::move(in));
    t->mark(id);
    t->nodes[cur].children[(uint8_t)parent_k] = id;
    return VC_OK;
}

int vc_verkle_get(const vc_verkle* t, const uint8_t* key, uint8_t* value, int* found) {
    if (!t || !key || !value || !found) return VC_E_INVALID;
    *found = 0;
    int e = find_stem(t, key);
    if (e < 0) return VC_OK;
    auto it = t->nodes[e].leaves.find(key[t->N - 1]);
    if (it == t->nodes[e].leaves.end()) return VC_OK;
    memcpy(value, it->second.data(), 32);
    *found = 1;
    return VC_OK;
}

// path_to_stem (node.rs:97-120): (prefix, unit) for every internal node down to the
// extension; the prefix is key[0..=depth], so only the units are returned.
int vc_verkle_path(const vc_verkle* t, const uint8_t* key, size_t max_len, uint8_t* units, size_t* len) {
    if (!t || !key || !len) return VC_E_INVALID;
    size_t n = 0;
    int cur = 0;
    while (!t->nodes[cur].ext) {
        if ((int)n >= t->N) return VC_E_INVALID;
        auto it = t->nodes[cur].children.find(key[n]);
        if (it == t->nodes[cur].children.end()) return VC_E_INVALID;  // VerkleError::InvalidPath
        if (units && n < max_len) units[n] = key[n];
        n++;
        cur = it->second;
    }
    *len = n;
    return VC_OK;
}

// diagnostics (tools/verkle_nodes.py): per node id, type (0 internal, 1 extension), level and the
// committed item (the device mirror's values brought to the host first)
int vc_verkle_debug_nodes(vc_verkle* t, size_t max, uint8_t* type, int32_t* level, uint64_t* items, size_t* n) {
    if (!t || !n) return VC_E_INVALID;
    VK_TRY(vk::verkle_pull_host(t));
    const size_t m = std::min(max, t->nodes.size());
    for (size_t i = 0; i < m; i++) {
        if (type) type[i] = t->nodes[i].ext ? 1 : 0;
        if (level) level[i] = t->nodes[i].level;
        if (items) memcpy(items + 4 * i, &t->item[4 * i], 32);
    }
    *n = t->nodes.size();
    return VC_OK;
}

// diagnostics (tools/verkle_host_probe.py, no GPU): the device path's extension host stage (rows
// built and merged into a plain buffer) over every extension node, `reps` times; *us = the median
int vc_verkle_debug_ext_stage(vc_verkle* t, int reps, double* us) {
    if (!t || !us || reps < 1) return VC_E_INVALID;
    return vk::verkle_debug_ext_stage(t, reps, us);
}

int vc_verkle_stats(const vc_verkle* t, size_t* internal, size_t* extension, size_t* dirty) {
    if (!t) return VC_E_INVALID;
    size_t a = 0, b = 0, c = 0;
    for (size_t i = 0; i < t->nodes.size(); i++) {
        (t->nodes[i].ext ? b : a)++;
        if (!t->has_commit[i]) c++;
    }
    if (internal) *internal = a;
    if (extension) *extension = b;
    if (dirty) *dirty = c;
    return VC_OK;
}

// gen_commitment (node.rs:205-277), level-batched. sh != nullptr: this rank's slices of every
// level, one all-gather of the per-node records per level (vc_verkle_commitment_sharded).
int vc_verkle_commitment(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf) {
    // the device-resident levels; VKZG_VERKLE_DEV=0 (read per call, A/B probe) takes the host path
    const char* env = getenv("VKZG_VERKLE_DEV");
    if (env && atoi(env) == 0) return vk::verkle_commitment(ctx, table, t, out_xy, out_inf, nullptr);
    return vk::verkle_commitment_dev(ctx, table, t, out_xy, out_inf);
}

}  // extern "C"

namespace vk {

// batched sparse commits (vc_msm_batch_sparse): rows of (column, value) non-zeros
struct Rows {
    uvec<uint64_t> ptr{0};
    uvec<uint32_t> cols;
    uvec<uint64_t> vals;
    void reserve(size_t rows, size_t nnz) {
        ptr.reserve(rows + 1);
        cols.reserve(nnz);
        vals.reserve(4 * nnz);
    }
    void add(uint32_t col, const uint64_t* v) {
        if (!(v[0] | v[1] | v[2] | v[3])) return;  // zero scalars contribute nothing
        cols.push_back(col);
        vals.insert(vals.end(), v, v + 4);
    }
    void end_row() { ptr.push_back(cols.size()); }
    size_t n() const { return ptr.size() - 1; }
};
// rows of items [lo, hi) built by fn(i, Rows&) on the host pool, in item order (the node walks
// are pointer-chasing code: ~100-200 ns per node on one thread); every worker builds the rows of
// its item range, then copies them into place in parallel. pf(i, stage): software prefetch of item
// i's node data ahead of the walk (stage 0 at 16 items ahead: the node; stage 1 at 8 ahead: what
// the node points to, its line now cached) -- the walks are chains of dependent DRAM misses
// (~360 ns per extension node on 16 threads)
// the per-worker parts of build_rows (one part when the range is small)
// reuse (optional): parts of an earlier call, cleared and refilled -- their storage stays
// allocated (a fresh 65,536-extension level's part vectors cost ~0.1 ms of page faults per worker)
template <class R, class Fn, class Pf>
std::vector<R> build_parts(HostPool& pool, size_t lo, size_t hi, size_t nnz_per, Fn fn, Pf pf,
                           std::vector<R>* reuse = nullptr) {
    const size_t count = hi - lo;
    auto walk_range = [&](size_t a, size_t b, R& r) {
        for (size_t i = a; i < std::min(b, a + 16); i++) pf(i, 0);
        for (size_t i = a; i < std::min(b, a + 8); i++) pf(i, 1);
        for (size_t i = a; i < b; i++) {
            if (i + 16 < b) pf(i + 16, 0);
            if (i + 8 < b) pf(i + 8, 1);
            fn(i, r);
        }
    };
    const unsigned T = (count >= 64 && count * nnz_per >= 16384)
                           ? (unsigned)std::min<size_t>(pool.size(), std::max<size_t>(1, count / 16))
                           : 1;
    std::vector<R> part;
    if (reuse) part.swap(*reuse);
    part.resize(T);
    auto run = [&](unsigned k) {
        if (k >= T) return;
        const size_t a = lo + count * k / T, b = lo + count * (k + 1) / T;
        // filled in a local object: the parts' vector headers share cache lines, and every
        // push_back updates its header (false sharing made 8 threads 1.6x one)
        R local = std::move(part[k]);
        local.clear();
        local.reserve(b - a, (b - a) * std::min<size_t>(nnz_per, 4));
        walk_range(a, b, local);
        part[k] = std::move(local);
    };
    if (T == 1) run(0);
    else pool.run(run);
    return part;
}

template <class R = Rows, class Fn, class Pf>
R build_rows(HostPool& pool, size_t lo, size_t hi, size_t nnz_per, Fn fn, Pf pf) {
    R out;
    const size_t count = hi - lo;
    auto walk_range = [&](size_t a, size_t b, R& r) {
        for (size_t i = a; i < std::min(b, a + 16); i++) pf(i, 0);
        for (size_t i = a; i < std::min(b, a + 8); i++) pf(i, 1);
        for (size_t i = a; i < b; i++) {
            if (i + 16 < b) pf(i + 16, 0);
            if (i + 8 < b) pf(i + 8, 1);
            fn(i, r);
        }
    };
    // by work, not rows: the 256 depth-1 nodes of a 65,536-key tree hold ~41K children (a
    // serial walk of their maps took 0.84 ms: profiles/r04/verkle/laps_before.txt)
    const unsigned T = (count >= 64 && count * nnz_per >= 16384)
                           ? (unsigned)std::min<size_t>(pool.size(), std::max<size_t>(1, count / 16))
                           : 1;
    if (T == 1) {
        out.reserve(count, count * nnz_per);
        walk_range(lo, hi, out);
        return out;
    }
    std::vector<R> part(T);
    pool.run([&](unsigned k) {  // the pool runs k < pool.size(): workers past T have no part
        if (k >= T) return;
        const size_t a = lo + count * k / T, b = lo + count * (k + 1) / T;
        R local;  // (a local object: no false sharing on the parts' vector headers)
        local.reserve(b - a, (b - a) * nnz_per);
        walk_range(a, b, local);
        part[k] = std::move(local);
    });
    std::vector<size_t> roff(T + 1, 0), noff(T + 1, 0);
    for (unsigned k = 0; k < T; k++) {
        roff[k + 1] = roff[k] + part[k].n();
        noff[k + 1] = noff[k] + part[k].cols.size();
        if constexpr (!std::is_same<R, Rows>::value) out.maxlen = std::max(out.maxlen, part[k].maxlen);
    }
    out.ptr.resize(roff[T] + 1);
    out.ptr[0] = 0;
    constexpr size_t VW = std::is_same<R, Rows>::value ? 4 : 2;  // u64 words per value
    out.cols.resize(noff[T]);
    out.vals.resize(VW * noff[T]);
    pool.run([&](unsigned k) {
        if (k >= T) return;
        const R& r = part[k];
        for (size_t i = 1; i < r.ptr.size(); i++) out.ptr[roff[k] + i] = noff[k] + r.ptr[i];
        if (!r.cols.empty()) {
            memcpy(&out.cols[noff[k]], r.cols.data(), r.cols.size() * 4);
            memcpy(&out.vals[VW * noff[k]], r.vals.data(), r.vals.size() * 8);
        }
    });
    return out;
}

// the c1 / c2 rows of extension node `id` (node.rs:216-244): every leaf's 16-byte halves as
// items at positions (2 index) % N, (2 index + 1) % N of c1 (index < N / 2) or c2; a later
// write to the same position overwrites, as c1_values[index] = ... does
static void ext_rows(const vc_verkle* t, int id, Rows& r) {
    const int N = t->N;
    struct PV {
        uint32_t pos;
        uint64_t v[4];
    };
    PV half[2][32];  // positions < N <= 32: fixed slots, no allocation
    int cnt[2] = {0, 0};
    auto put = [&](int h, uint32_t pos, const uint64_t* v) {
        for (int k = 0; k < cnt[h]; k++)
            if (half[h][k].pos == pos) {
                memcpy(half[h][k].v, v, 32);
                return;
            }
        half[h][cnt[h]].pos = pos;
        memcpy(half[h][cnt[h]].v, v, 32);
        cnt[h]++;
    };
    const VNode& n = t->nodes[id];
    for (auto& kv : n.leaves) {
        const size_t index = kv.first;
        uint64_t vlo[4], vhi[4];
        item_of_bytes(kv.second.data(), 16, vlo);
        item_of_bytes(kv.second.data() + 16, 16, vhi);
        const int h = index < (size_t)(N / 2) ? 0 : 1;
        put(h, (uint32_t)((2 * index) % N), vlo);
        put(h, (uint32_t)((2 * index + 1) % N), vhi);
    }
    for (int h = 0; h < 2; h++) {
        for (int k = 0; k < cnt[h]; k++) r.add(half[h][k].pos, half[h][k].v);
        r.end_row();
    }
}
// the device path's extension rows: c1 / c2 as ext_rows, but with 16-byte values (a leaf half is
// below 2^128: the device widens them) and the node's raw stem bytes (the device reduces them mod r);
// stem[] is indexed by the row pair
struct ExtRows16 {
    uvec<uint64_t> ptr{0};
    uvec<uint32_t> cols;
    uvec<uint64_t> vals;  // 2 u64 per non-zero
    uvec<uint64_t> stem;  // 4 u64 per extension node (its raw stem bytes, LE)
    uint32_t maxlen = 0;  // longest row (<= 4: the sparse commit's chunks are the rows)
    void clear() {  // (capacity kept)
        ptr.assign(1, 0);
        cols.clear();
        vals.clear();
        stem.clear();
        maxlen = 0;
    }
    void reserve(size_t rows, size_t nnz) {
        ptr.reserve(2 * rows + 1);
        cols.reserve(nnz);
        vals.reserve(2 * nnz);
        stem.reserve(4 * rows);
    }
    size_t n() const { return ptr.size() - 1; }
};
static void ext_rows16(const vc_verkle* t, int id, ExtRows16& r) {
    const int N = t->N;
    struct PV {
        uint32_t pos;
        uint64_t v[2];
    };
    PV half[2][32];
    int cnt[2] = {0, 0};
    auto put = [&](int h, uint32_t pos, const uint8_t* b16) {
        uint64_t v[2];
        memcpy(v, b16, 16);
        for (int k = 0; k < cnt[h]; k++)
            if (half[h][k].pos == pos) {
                half[h][k].v[0] = v[0];
                half[h][k].v[1] = v[1];
                return;
            }
        half[h][cnt[h]].pos = pos;
        half[h][cnt[h]].v[0] = v[0];
        half[h][cnt[h]].v[1] = v[1];
        cnt[h]++;
    };
    const VNode& n = t->nodes[id];
    for (auto& kv : n.leaves) {
        const size_t index = kv.first;
        const int h = index < (size_t)(N / 2) ? 0 : 1;
        put(h, (uint32_t)((2 * index) % N), kv.second.data());
        put(h, (uint32_t)((2 * index + 1) % N), kv.second.data() + 16);
    }
    for (int h = 0; h < 2; h++) {
        for (int k = 0; k < cnt[h]; k++) {
            if (!(half[h][k].v[0] | half[h][k].v[1])) continue;  // zero scalars contribute nothing
            r.cols.push_back(half[h][k].pos);
            r.vals.push_back(half[h][k].v[0]);
            r.vals.push_back(half[h][k].v[1]);
        }
        r.maxlen = std::max<uint32_t>(r.maxlen, (uint32_t)(r.cols.size() - r.ptr.back()));
        r.ptr.push_back(r.cols.size());
    }
    // the stem's raw LE bytes (zero beyond N): k_vk_ext_rows4 reduces them mod r on the device
    // (bytes_to_item(stem.to_bytes()), node.rs:248-250 -> lagrange_basis.rs:175-176) -- the host's
    // one-quotient reduction was ~35 % of this stage's single-thread time (profiles/r05/verkle/)
    r.stem.resize(r.stem.size() + 4);
    memcpy(r.stem.data() + r.stem.size() - 4, n.stem.data(), 32);
}

static void ext_prefetch(const vc_verkle* t, int id, int stage) {
    const VNode& n = t->nodes[id];
    if (stage == 0) {
        __builtin_prefetch(&n);
        __builtin_prefetch(reinterpret_cast<const char*>(&n) + 64);
    } else if (!n.leaves.v.empty()) {
        __builtin_prefetch(n.leaves.v.data());
    }
}

// The extension level's host stage (verkle_commitment_dev): c1 / c2 rows built in per-worker parts
// (with each node's raw stem bytes, reduced on the device), then merged in parallel straight into one
// buffer (page-locked in the commitment: the upload is plain DMA) laid out as row_ptr (2E + 1 u64) |
// stems (E x 32 B) |
// values (nnz x 2 u64) | node ids (E u32) | cols (nnz u32) -- everything after row_ptr goes up in one
// copy. `cache`: part storage kept between calls (no page faults on fresh vectors).
struct ExtStage {
    size_t nnz = 0, o_stem = 0, o_vals = 0, o_ids = 0, o_cols = 0, o_end = 0;
    uint32_t maxlen = 0;
    uint8_t* base = nullptr;
};
// rp_out (optional): the row pointers go there instead, each plus nnz_base (one piece of a level
// built in pieces: its rows' pointers in the level's array)
static int ext_stage(const vc_verkle* t, const std::vector<int>& exts, HostPool& pool, std::vector<ExtRows16>& cache,
                     const std::function<uint8_t*(size_t)>& buffer, ExtStage* out, double* t_build = nullptr,
                     uint64_t* rp_out = nullptr, uint64_t nnz_base = 0) {
    const size_t E = exts.size();
    const auto tb0 = std::chrono::steady_clock::now();
    std::vector<ExtRows16> parts = build_parts<ExtRows16>(
        pool, 0, E, (size_t)t->N, [&](size_t e, ExtRows16& r) { ext_rows16(t, exts[e], r); },
        [&](size_t e, int stage) { ext_prefetch(t, exts[e], stage); }, &cache);
    struct KeepParts {
        std::vector<ExtRows16>& p;
        std::vector<ExtRows16>& cache;
        ~KeepParts() { cache.swap(p); }
    } keep_parts{parts, cache};
    if (t_build) *t_build = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tb0).count();
    const size_t T = parts.size();
    std::vector<size_t> roff(T + 1, 0), noff(T + 1, 0), eoff(T + 1, 0);
    uint32_t maxlen = 0;
    for (size_t k = 0; k < T; k++) {
        roff[k + 1] = roff[k] + parts[k].n();
        noff[k + 1] = noff[k] + parts[k].cols.size();
        eoff[k + 1] = eoff[k] + parts[k].stem.size() / 4;
        maxlen = std::max(maxlen, parts[k].maxlen);
    }
    const size_t nnz = noff[T];
    ExtStage& X = *out;
    X.nnz = nnz;
    X.maxlen = maxlen;
    X.o_stem = (2 * E + 1) * 8;
    X.o_vals = X.o_stem + E * 32;
    X.o_ids = X.o_vals + nnz * 16;
    X.o_cols = X.o_ids + E * 4;
    X.o_end = X.o_cols + nnz * 4;
    uint8_t* pin = buffer(X.o_end);
    if (!pin) return VC_E_OOM;
    X.base = pin;
    uint64_t* rp = rp_out ? rp_out : reinterpret_cast<uint64_t*>(pin);
    uint32_t* ids = reinterpret_cast<uint32_t*>(pin + X.o_ids);
    rp[0] = nnz_base;
    auto merge = [&](unsigned k) {  // part k holds extensions [eoff[k], eoff[k + 1]) in order
        if (k >= T) return;
        const ExtRows16& r = parts[k];
        for (size_t i = 1; i < r.ptr.size(); i++) rp[roff[k] + i] = nnz_base + noff[k] + r.ptr[i];
        memcpy(pin + X.o_stem + eoff[k] * 32, r.stem.data(), r.stem.size() * 8);
        if (!r.cols.empty()) {
            memcpy(pin + X.o_vals + noff[k] * 16, r.vals.data(), r.vals.size() * 8);
            memcpy(pin + X.o_cols + noff[k] * 4, r.cols.data(), r.cols.size() * 4);
        }
        for (size_t e = eoff[k]; e < eoff[k + 1]; e++) ids[e] = (uint32_t)exts[e];
    };
    if (T == 1) merge(0);
    else pool.run(merge);
    return VC_OK;
}

int verkle_debug_ext_stage(vc_verkle* t, int reps, double* us) {
    std::vector<int> exts;
    for (size_t i = 0; i < t->nodes.size(); i++)
        if (t->nodes[i].ext) exts.push_back((int)i);
    std::vector<ExtRows16> cache;
    std::vector<uint8_t> buf;
    std::vector<double> ts, tbs;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        ExtStage X;
        double tb = 0;
        VK_TRY(ext_stage(t, exts, host_pool(), cache,
                         [&](size_t bytes) -> uint8_t* {
                             if (buf.size() < bytes) buf.resize(bytes);
                             return buf.data();
                         },
                         &X, &tb));
        ts.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        tbs.push_back(tb);
    }
    if (getenv("VKZG_VERBOSE")) {  // one thread over the whole level, and the stem items alone
        ExtRows16 r;
        r.reserve(exts.size(), exts.size() * 4);
        auto c0 = std::chrono::steady_clock::now();
        for (size_t e = 0; e < exts.size(); e++) ext_rows16(t, exts[e], r);
        auto c1 = std::chrono::steady_clock::now();
        uint64_t acc = 0, w[4];
        for (size_t e = 0; e < exts.size(); e++) {
            item_of_bytes(t->nodes[exts[e]].stem.data(), t->N, w);
            acc ^= w[0];
        }
        auto c2 = std::chrono::steady_clock::now();
        fprintf(stderr, "[ext stage] one thread: rows %.1f us, stem items alone %.1f us (%llu), sizeof(VNode) %zu\n",
                std::chrono::duration<double, std::micro>(c1 - c0).count(),
                std::chrono::duration<double, std::micro>(c2 - c1).count(), (unsigned long long)(acc & 1), sizeof(VNode));
    }
    std::sort(ts.begin(), ts.end());
    std::sort(tbs.begin(), tbs.end());
    *us = ts[ts.size() / 2];
    if (getenv("VKZG_VERBOSE"))
        fprintf(stderr, "[ext stage] %zu extensions, %u threads: build %.1f us, total %.1f us (medians)\n", exts.size(),
                host_pool().size(), tbs[tbs.size() / 2], *us);
    return VC_OK;
}

// vc_msm_batch_sparse + vc_to_data_item_batch in one call (capi.cpp vc_msm_batch_sparse_items)
static int sparse_items(vc_ctx* ctx, int table, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                        const uint64_t* vals, uint64_t* xy, uint8_t* inf, uint64_t* items) {
    return msm_batch_sparse_items_guarded(ctx, table, batch, row_ptr, cols, vals, xy, inf, items);
}

// ---- device mirror (VerkleDev) management
// the mirror's results -> the host arrays (before a host-path commitment or a move to another
// context's device)
static int mirror_pull(vc_verkle* t) {
    VerkleDev& D = t->dev;
    if (t->host_valid) return VC_OK;
    const size_t n = std::min(t->nodes.size(), D.cap);
    if (D.ctx_uid && n) {
        DeviceScope on(D.dev);  // the mirror's device, the caller's restored on return (a move to
                                // another context allocates the new mirror on that one's device)
        VK_CHECK_HIP(hipMemcpy(t->item.data(), D.item, n * 32, hipMemcpyDeviceToHost));
        VK_CHECK_HIP(hipMemcpy(t->cxy.data(), D.cxy, n * 64, hipMemcpyDeviceToHost));
        VK_CHECK_HIP(hipMemcpy(t->cinf.data(), D.inf, n, hipMemcpyDeviceToHost));
    }
    t->host_valid = true;
    return VC_OK;
}
int verkle_pull_host(vc_verkle* t) { return mirror_pull(t); }
// a mirror on ctx's device holding every committed node's results, with room for every node
static int mirror_prepare(vc_ctx* ctx, vc_verkle* t) {
    VerkleDev& D = t->dev;
    const size_t n = t->nodes.size();
    if (D.ctx_uid != ctx->uid) {  // first use, or another context: rebuild from the host arrays
        VK_TRY(mirror_pull(t));
        D.release();
        VK_CHECK_HIP(hipSetDevice(ctx->device));  // (both restore it; allocations below are ctx's)
    }
    const bool fresh = D.ctx_uid == 0;
    if (D.cap < n) {  // (with room: a tree that grows by an update's splits keeps its buffers)
        const size_t cap = std::max<size_t>({n + n / 4, 2 * D.cap, 1024});
        void* blk = nullptr;  // one allocation: items, commitments, flags
        size_t blk_bytes = 0;
        VK_TRY(pool_take(ctx, cap * (32 + 64 + 1), &blk, &blk_bytes));
        void* p[3] = {blk, static_cast<uint8_t*>(blk) + cap * 32, static_cast<uint8_t*>(blk) + cap * 96};
        if (!fresh && D.cap) {  // keep the committed results (every id < the old capacity)
            VK_CHECK_HIP(hipMemcpyAsync(p[0], D.item, D.cap * 32, hipMemcpyDeviceToDevice, ctx->stream));
            VK_CHECK_HIP(hipMemcpyAsync(p[1], D.cxy, D.cap * 64, hipMemcpyDeviceToDevice, ctx->stream));
            VK_CHECK_HIP(hipMemcpyAsync(p[2], D.inf, D.cap, hipMemcpyDeviceToDevice, ctx->stream));
            VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        }
        if (D.item) pool_put(ctx, D.item, D.blk_bytes);  // (the block's start; this context's, copied above)
        D.item = p[0];
        D.cxy = p[1];
        D.inf = p[2];
        D.cap = cap;
        D.blk_bytes = blk_bytes;
    }
    if (fresh) {  // the host arrays are current (mirror_pull above): upload them -- unless no node
        // has a commitment yet (a fresh tree: every value is written by this commitment)
        if (t->dirty_count() < n) {
            VK_CHECK_HIP(hipMemcpyAsync(D.item, t->item.data(), n * 32, hipMemcpyHostToDevice, ctx->stream));
            VK_CHECK_HIP(hipMemcpyAsync(D.cxy, t->cxy.data(), n * 64, hipMemcpyHostToDevice, ctx->stream));
            VK_CHECK_HIP(hipMemcpyAsync(D.inf, t->cinf.data(), n, hipMemcpyHostToDevice, ctx->stream));
        }
        D.ctx_uid = ctx->uid;
        D.dev = ctx->device;
    }
    return VC_OK;
}

int verkle_commitment(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf, const Shard* sh,
                      const Multi* mu) {
    if (!ctx || !t || !out_xy || !out_inf || (sh && mu)) return VC_E_INVALID;
    // the host path reads and writes the host arrays: bring them up to date, and drop the device
    // mirror afterwards (it would miss this call's results)
    VK_TRY(mirror_pull(t));
    struct DropMirror {
        vc_verkle* t;
        ~DropMirror() { t->dev.release(); }
    } drop{t};
    DeltaGuard delta_guard{t};
    const int N = t->N;
    static const bool verbose = getenv("VKZG_VERBOSE") != nullptr;
    auto tic = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!verbose) return;
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[verkle] %s %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tic).count());
        tic = now;
    };
    // dirty nodes reachable from the root, with depth (clean subtrees are skipped: an insert
    // clears every commitment on its path, so a clean node has clean descendants). Every rank
    // holds the same tree, so every rank walks it to the same lists in the same order.
    // The walk of the root's subtrees is split over the host pool (contiguous ranges of the
    // root's children; the per-worker lists are concatenated in worker order, so the lists --
    // and a sharded run's slices -- are the same on every rank).
    std::vector<int> exts;
    std::vector<std::vector<int>> internals;  // by depth
    auto walk = [&](int root, int depth0, std::vector<int>& ex, std::vector<std::vector<int>>& in) {
        std::vector<std::pair<int, int>> stack{{root, depth0}};
        while (!stack.empty()) {
            auto [id, depth] = stack.back();
            stack.pop_back();
            const VNode& n = t->nodes[id];
            if (t->has_commit[id]) continue;
            if (n.ext) {
                ex.push_back(id);
                continue;
            }
            if ((int)in.size() <= depth) in.resize(depth + 1);
            in[depth].push_back(id);
            for (auto& kv : n.children) {  // (popped in reverse: fetch their lines meanwhile)
                __builtin_prefetch(&t->nodes[kv.second]);
                stack.push_back({kv.second, depth + 1});
            }
        }
    };
    {
        const VNode& root = t->nodes[0];
        HostPool& P = host_pool();
        // (the branch depends only on the tree, never on this host's core count: ranks of a
        // sharded run with different pool sizes must produce the same lists; a one-thread pool
        // runs the same per-child walk serially)
        if (t->has_commit[0] || root.ext || root.children.v.size() < 2 || t->nodes.size() < 4096) {
            walk(0, 0, exts, internals);
        } else {
            internals.resize(1);
            internals[0].push_back(0);
            const auto& ch = root.children.v;
            const unsigned T = P.size();
            std::vector<std::vector<int>> ex(T);
            std::vector<std::vector<std::vector<int>>> in(T);
            auto part = [&](unsigned k) {
                for (size_t c = ch.size() * k / T; c < ch.size() * (k + 1) / T; c++) walk(ch[c].second, 1, ex[k], in[k]);
            };
            if (T == 1) part(0);
            else P.run(part);
            for (unsigned k = 0; k < T; k++) {
                exts.insert(exts.end(), ex[k].begin(), ex[k].end());
                if (internals.size() < in[k].size()) internals.resize(in[k].size());
                for (size_t d = 0; d < in[k].size(); d++)
                    internals[d].insert(internals[d].end(), in[k][d].begin(), in[k][d].end());
            }
        }
    }
    HostPool& pool = host_pool();
    auto build_rows = [&](size_t lo, size_t hi, size_t nnz_per, auto fn, auto pf) {
        return vk::build_rows(pool, lo, hi, nnz_per, fn, pf);
    };
    // fn(i) for i in [0, count) on the pool (independent per-item writes)
    auto for_each = [&](size_t count, auto fn) {
        const unsigned T = count >= 4096 ? pool.size() : 1;
        if (T == 1) {
            for (size_t i = 0; i < count; i++) fn(i);
            return;
        }
        pool.run([&](unsigned k) {
            for (size_t i = count * k / T; i < count * (k + 1) / T; i++) fn(i);
        });
    };
    lap("collect dirty");
    // outputs are written in full by the two calls (uninitialised staging, host/pool.hpp uvec)
    // dense rows (vc_msm_batch: the fixed-base batched commit over the first `width` bases) for
    // levels of <= 64 rows (its latency path: the root's one commit 0.44 -> 0.11 ms) -- the sparse
    // path's ~10 latency-bound launches and host round trips cost ~0.35 ms even for one row;
    // larger levels stay sparse (dense measured slower at 65 rows, equal at 65,536 x 4:
    // profiles/r04/verkle/). VKZG_VERKLE_DENSE (read per call) forces one path:
    // 0 = sparse, 1 = dense
    const char* dense_env = getenv("VKZG_VERKLE_DENSE");
    const int dense_mode = dense_env ? atoi(dense_env) : -1;
    uvec<uint64_t> dense;
    auto commit_rows = [&](const Rows& r, size_t width, uvec<uint64_t>& xy, uvec<uint8_t>& inf,
                           uvec<uint64_t>& items) -> int {
        const size_t B = r.n();
        xy.resize(B * 8);
        inf.resize(B);
        items.resize(B * 4);
        if (B == 0) return VC_OK;
        lap("build rows");
        const bool use_dense = !mu && (dense_mode == 1 || (dense_mode != 0 && B <= 64 && B * width <= 16384));
        if (use_dense) {
            dense.resize(B * width * 4);
            for_each(B, [&](size_t b) {
                uint64_t* row = &dense[b * width * 4];
                memset(row, 0, width * 32);
                for (uint64_t e = r.ptr[b]; e < r.ptr[b + 1]; e++) memcpy(row + 4 * (size_t)r.cols[e], &r.vals[4 * e], 32);
            });
            VK_TRY(vc_msm_batch(ctx, table, width, dense.data(), B, 0, xy.data(), inf.data()));
            // <= 64 points: to_data_item on the host (compress + mod r, no inversion: already affine)
            for (size_t b = 0; b < B; b++) {
                const Fr it = to_data_item_host(&xy[8 * b], inf[b] != 0);
                mont_to_canon<BN254Fr>(it, &items[4 * b]);
            }
            lap("dense commit + to_data_item");
            return VC_OK;
        }
        if (mu) {  // member k commits rows [B k / G, B (k + 1) / G) of the level on its own device
            const int G = (int)mu->ctx.size();
            std::vector<int> st(G, VC_OK);
            mu->run([&](int k) {
                size_t a, e;
                shard_range(B, k, G, &a, &e);
                if (a == e) return;
                std::vector<uint64_t> rp(e - a + 1);
                const uint64_t base = r.ptr[a];
                for (size_t i = 0; i <= e - a; i++) rp[i] = r.ptr[a + i] - base;
                const uint32_t* cols = r.cols.size() ? r.cols.data() + base : nullptr;
                const uint64_t* vals = r.vals.size() ? r.vals.data() + 4 * base : nullptr;
                st[k] = sparse_items(mu->ctx[k], mu->table[k], e - a, rp.data(), cols, vals, xy.data() + 8 * a,
                                     inf.data() + a, items.data() + 4 * a);
            });
            for (int s : st)
                if (s != VC_OK) return s;
            lap("sparse commit + to_data_item (members)");
            return VC_OK;
        }
        // the rows' commitments and their to_data_item values in one call (items computed on the
        // device from the normalised points: no second upload / read-back per level)
        VK_TRY(sparse_items(ctx, table, B, r.ptr.data(), r.cols.data(), r.vals.data(), xy.data(), inf.data(),
                            items.data()));
        lap("sparse commit + to_data_item");
        return VC_OK;
    };
    // the nodes nodes[lo, hi) of a level got (xy, inf, items) here: store them; with a shard,
    // first all-gather every rank's slice (records of 8 + 4 + 1 u64: xy, item, inf), so every
    // rank stores the whole level
    // st: this rank's status for the level -- a failed share still enters the exchange with it
    // (include/vc_comm.h), so every rank stops at the same level with an error
    auto store_level = [&](const std::vector<int>& ids, size_t lo, size_t hi, const uvec<uint64_t>& xy,
                           const uvec<uint8_t>& inf, const uvec<uint64_t>& items, int st) -> int {
        auto put = [&](size_t i, const uint64_t* rxy, uint8_t rinf, const uint64_t* ritem) {
            const size_t id = (size_t)ids[i];
            memcpy(&t->cxy[8 * id], rxy, 64);
            t->cinf[id] = rinf;
            memcpy(&t->item[4 * id], ritem, 32);
            t->has_commit[id] = 1;
        };
        if (!sh) {
            if (st != VC_OK) return st;
            for_each(hi - lo, [&](size_t b) { put(lo + b, &xy[b * 8], inf[b], &items[b * 4]); });
            return VC_OK;
        }
        constexpr size_t REC = 13;  // u64 words per record
        const size_t B = ids.size(), bmax = (B + sh->world - 1) / sh->world, slot = 1 + bmax * REC;
        std::vector<uint64_t> send(slot, 0), recv(slot * sh->world);
        send[0] = (uint64_t)(uint32_t)st;
        for (size_t b = 0; st == VC_OK && b < hi - lo; b++) {
            memcpy(&send[1 + b * REC], &xy[b * 8], 64);
            memcpy(&send[1 + b * REC + 8], &items[b * 4], 32);
            send[1 + b * REC + 12] = inf[b];
        }
        VK_TRY(sh->allgather(send.data(), send.size() * 8, recv.data()));
        if (st != VC_OK) return st;
        for (int k = 0; k < sh->world; k++)
            if ((int32_t)(uint32_t)recv[(size_t)k * slot] != VC_OK) return VC_E_PEER;
        for (int k = 0; k < sh->world; k++) {
            const size_t a = B * k / sh->world, e = B * (k + 1) / sh->world;
            const uint64_t* src = &recv[(size_t)k * slot + 1];
            for_each(e - a, [&](size_t b) {
                const uint64_t* rec = src + b * REC;
                put(a + b, rec, (uint8_t)rec[12], rec + 8);
            });
        }
        return VC_OK;
    };
    auto slice = [&](size_t B, size_t* lo, size_t* hi) {
        *lo = sh ? B * sh->rank / sh->world : 0;
        *hi = sh ? B * (sh->rank + 1) / sh->world : B;
    };
    uvec<uint64_t> xy, items, xy2, items2;
    uvec<uint8_t> inf, inf2;
    // extension nodes: c1, c2 (width N), then [1, stem, c1, c2] (width 4) -- both steps only need
    // the node's own values, so a rank runs both on its slice and exchanges once
    if (!exts.empty()) {
        const size_t E = exts.size();
        size_t lo, hi;
        slice(E, &lo, &hi);
        // (position, value) writes of c1 / c2 in leaf order; a later write to the same
        // position overwrites, as c1_values[index] = ... does (node.rs:226-239)
        Rows r12 = build_rows(lo, hi, (size_t)N, [&](size_t e, Rows& r) { ext_rows(t, exts[e], r); },
                              [&](size_t e, int stage) { ext_prefetch(t, exts[e], stage); });
        int st = commit_rows(r12, (size_t)N, xy, inf, items);
        Rows rx;
        if (st == VC_OK) rx = build_rows(lo, hi, 4, [&](size_t e, Rows& r) {
            const VNode& n = t->nodes[exts[e]];
            uint64_t one[4] = {1, 0, 0, 0}, stem_item[4];
            item_of_bytes(n.stem.data(), N, stem_item);  // bytes_to_item(stem.to_bytes())
            r.add(0, one);
            r.add(1, stem_item);
            r.add(2, &items[(2 * (e - lo)) * 4]);
            r.add(3, &items[(2 * (e - lo) + 1) * 4]);
            r.end_row();
        }, [&](size_t e, int stage) {
            if (stage == 0) __builtin_prefetch(t->nodes[exts[e]].stem.data());
        });
        if (st == VC_OK) st = commit_rows(rx, 4, xy2, inf2, items2);
        VK_TRY(store_level(exts, lo, hi, xy2, inf2, items2, st));
    }
    // internal nodes, deepest level first (HACK in the reference: width hard-coded 256); a
    // parent needs its children's items, so every depth is one exchange
    for (int depth = (int)internals.size() - 1; depth >= 0; depth--) {
        const std::vector<int>& lv = internals[depth];
        size_t lo, hi;
        slice(lv.size(), &lo, &hi);
        size_t kids = 0;  // children of the slice (the rows' non-zero bound)
        for (size_t b = lo; b < hi; b++) kids += t->nodes[lv[b]].children.v.size();
        Rows ri = build_rows(lo, hi, hi > lo ? (kids + hi - lo - 1) / (hi - lo) : 1, [&](size_t b, Rows& r) {
            for (auto& kv : t->nodes[lv[b]].children) r.add(kv.first, &t->item[4 * (size_t)kv.second]);
            r.end_row();
        }, [&](size_t b, int stage) {
            const VNode& n = t->nodes[lv[b]];
            if (stage == 0) {
                __builtin_prefetch(&n);
                __builtin_prefetch(reinterpret_cast<const char*>(&n) + 64);
            } else if (!n.children.v.empty()) {
                __builtin_prefetch(n.children.v.data());
            }
        });
        const int st = commit_rows(ri, 256, xy, inf, items);
        VK_TRY(store_level(lv, lo, hi, xy, inf, items, st));
    }
    memcpy(out_xy, &t->cxy[0], 64);
    *out_inf = t->cinf[0];
    t->clear_dirty();
    delta_guard.ok = true;
    return VC_OK;
}

// ---- the device-resident commitment (one context): every level's rows are built, committed and
// turned into items on the device, the items stored into the mirror by node id, so the next level
// gathers its children's items there -- no per-level read-back or host row values for internal
// levels. The host builds only the extension leaf rows (values it alone holds) and each internal
// level's (column, child id) lists.
__global__ void k_vk_gather(const uint64_t* __restrict__ item, const uint32_t* __restrict__ ids, size_t n,
                            uint64_t* __restrict__ out) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t* s = item + 4 * (size_t)ids[j];
    uint64_t* o = out + 4 * j;
    o[0] = s[0];
    o[1] = s[1];
    o[2] = s[2];
    o[3] = s[3];
}
// a level's row values: item(child) - (sidx < 0 ? 0 : snap[sidx]) mod r (canonical Fr words) --
// a full row's entries have no old value, a delta row's the child's item at the last commitment
__global__ void k_vk_delta(const uint64_t* __restrict__ item, const uint32_t* __restrict__ child,
                           const int32_t* __restrict__ sidx, const uint64_t* __restrict__ snap, size_t n,
                           uint64_t* __restrict__ out) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    fe<BN254Fr> a, b = fe_zero<BN254Fr>();
    memcpy(a.v, item + 4 * (size_t)child[j], 32);
    const int32_t k = sidx[j];
    if (k >= 0) memcpy(b.v, snap + 4 * (size_t)k, 32);
    const fe<BN254Fr> d = fe_sub<BN254Fr>(a, b);  // (canonical in, canonical out)
    memcpy(out + 4 * j, d.v, 32);
}
// 16-byte leaf halves -> 4-word scalars
__global__ void k_vk_widen16(const uint64_t* __restrict__ in, size_t n, uint64_t* __restrict__ out) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    out[4 * j] = in[2 * j];
    out[4 * j + 1] = in[2 * j + 1];
    out[4 * j + 2] = 0;
    out[4 * j + 3] = 0;
}
// extension commitment rows [1, stem item, c1 item, c2 item] (node.rs:245-256), columns 0..3; the
// stem arrives as its raw 32 LE bytes and is reduced mod r here (from_le_bytes_mod_order of a value
// below 2^256 < 6 r: at most five subtractions)
__global__ void k_vk_ext_rows4(const uint64_t* __restrict__ stem, const uint64_t* __restrict__ it12, size_t E,
                               uint32_t* __restrict__ cols, uint64_t* __restrict__ vals) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // entry 4 k + c
    if (j >= 4 * E) return;
    const size_t k = j >> 2;
    const uint32_t c = (uint32_t)(j & 3);
    cols[j] = c;
    const uint64_t one[4] = {1, 0, 0, 0};
    const uint64_t* v = c == 0 ? one : c == 1 ? stem + 4 * k : it12 + 4 * (2 * k + (c - 2));
    uint64_t w[4] = {v[0], v[1], v[2], v[3]};
    if (c == 1) {
        constexpr uint64_t R[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                                   0x30644e72e131a029ULL};  // BN254 r
        for (int it = 0; it < 5; it++) {
            uint64_t d[4], br = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint64_t a = w[i], b = R[i];
                d[i] = a - b - br;
                br = (a < b || (a == b && br)) ? 1 : 0;
            }
            if (br) break;  // w < r
#pragma unroll
            for (int i = 0; i < 4; i++) w[i] = d[i];
        }
    }
    uint64_t* o = vals + 4 * j;
    o[0] = w[0];
    o[1] = w[1];
    o[2] = w[2];
    o[3] = w[3];
}
// row pointers of E rows of 4: rp[k] = 4 k, k <= E
__global__ void k_vk_rp4(uint64_t* __restrict__ rp, size_t E) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= E) rp[k] = 4 * (uint64_t)k;
}
// rows' results -> the mirror at their node ids
__global__ void k_vk_scatter(const uint32_t* __restrict__ ids, size_t n, const uint64_t* __restrict__ xy,
                             const uint8_t* __restrict__ inf, const uint64_t* __restrict__ it,
                             uint64_t* __restrict__ m_cxy, uint8_t* __restrict__ m_inf, uint64_t* __restrict__ m_item) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const size_t id = ids[j];
#pragma unroll
    for (int k = 0; k < 8; k++) m_cxy[8 * id + k] = xy[8 * j + k];
#pragma unroll
    for (int k = 0; k < 4; k++) m_item[4 * id + k] = it[4 * j + k];
    m_inf[id] = inf[j];
}
// dense width-`width` rows of a small level: dense[b][col] = item[child] (zeroed before)
__global__ void k_vk_dense(const uint32_t* __restrict__ row, const uint32_t* __restrict__ cols,
                           const uint32_t* __restrict__ child, size_t nnz, const uint64_t* __restrict__ item,
                           uint32_t width, uint64_t* __restrict__ dense) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    const uint64_t* s = item + 4 * (size_t)child[j];
    uint64_t* o = dense + 4 * ((size_t)row[j] * width + cols[j]);
    o[0] = s[0];
    o[1] = s[1];
    o[2] = s[2];
    o[3] = s[3];
}

int verkle_commitment_dev(vc_ctx* ctx, int table, vc_verkle* t, uint64_t* out_xy, uint8_t* out_inf) {
    if (!ctx || !t || !out_xy || !out_inf) return VC_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    VK_CHECK_HIP(hipSetDevice(ctx->device));
    struct Collect {  // the per-kernel timers (vc_ctx_enable_timing), as the C ABI's Guard does
        vc_ctx* c;
        ~Collect() {
            if (c->timing) c->collect_timers();
        }
    } collect{ctx};
    Table* tab = ctx->table(table);
    if (!tab) return VC_E_TABLE;
    if (tab->curve != VC_CURVE_BN254) return VC_E_INVALID;
    static const bool verbose = getenv("VKZG_VERBOSE") != nullptr;
    // VKZG_VERKLE_STAMPS=1: the host's time at each lap without synchronising (printed at the end)
    static const bool stamps = getenv("VKZG_VERKLE_STAMPS") != nullptr;
    auto tic = std::chrono::steady_clock::now();
    const auto t_entry = tic;
    std::vector<std::pair<const char*, double>> marks;
    auto lap = [&](const char* what) {
        if (stamps) {
            marks.emplace_back(what, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_entry).count());
            return;
        }
        if (!verbose) return;
        (void)hipStreamSynchronize(ctx->stream);
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[verkle-dev] %s %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tic).count());
        tic = now;
    };
    struct PrintMarks {
        const std::vector<std::pair<const char*, double>>& m;
        ~PrintMarks() {
            if (m.empty()) return;
            std::string line = "[verkle-stamps]";
            char buf[96];
            for (auto& x : m) {
                snprintf(buf, sizeof buf, " %s@%.0f", x.first, x.second);
                line += buf;
            }
            fprintf(stderr, "%s\n", line.c_str());
        }
    } print_marks{marks};
    DeltaGuard delta_guard{t};
    VK_TRY(mirror_prepare(ctx, t));
    VerkleDev& D = t->dev;
    uint64_t* m_item = static_cast<uint64_t*>(D.item);
    uint64_t* m_cxy = static_cast<uint64_t*>(D.cxy);
    uint8_t* m_inf = static_cast<uint8_t*>(D.inf);
    hipStream_t st = ctx->stream;
    HostPool& pool = host_pool();
    const int N = t->N;
    auto grid = [](size_t n) { return (unsigned)((n + 255) / 256); };
    lap("mirror");
    // results of one level's B rows (device) -> the mirror at the nodes' ids
    auto scatter = [&](const uint32_t* d_ids, size_t B, const void* d_xy, const uint8_t* d_inf, const void* d_it) -> int {
        VK_LAUNCH(ctx, "verkle_scatter", k_vk_scatter, grid(B), 256, 0, d_ids, B, static_cast<const uint64_t*>(d_xy),
                  d_inf, static_cast<const uint64_t*>(d_it), m_cxy, m_inf, m_item);
        return VC_OK;
    };
    // levels of at most this many (non-zero, window) pairs take the sparse commits' latency path
    // (a wave per 64 pairs, msm.hip k_fb_sparse_small) instead of the sort-based one: an update's
    // levels; VKZG_SPARSE_SMALL_MAX (pairs, read per call; 0 = never) is the A/B knob
    const char* small_env = getenv("VKZG_SPARSE_SMALL_MAX");
    const size_t small_max = small_env ? (size_t)atoll(small_env) : (size_t)1 << 18;
    auto small_ok = [&](size_t nnz) { return sparse_small_pairs(tab, nnz) <= small_max; };
    // delta rows: an updated internal node whose last commitment is in the mirror (base) is
    // C_old + sum over its changed slots of (item(child now) - item(child then)) L_slot, instead of
    // its full row (~160 children per level-1 node of a 65,536-key tree, ~2 of them changed by a
    // 1 % update). The changed slots are the insert-time slot log's (first entry per slot: the child
    // at the last commitment); their old items are snapshotted here, before this call's scatters
    // overwrite them. VKZG_VERKLE_DELTA=0 (read per call, A/B probe) recommits every row in full.
    const char* delta_env = getenv("VKZG_VERKLE_DELTA");
    const bool use_delta = !(delta_env && atoi(delta_env) == 0);
    struct DPlan {
        uint64_t seen[4];
        uint32_t start, cnt;  // its entries in plan_e: (slot, snapshot index; -1: the slot was empty)
    };
    std::vector<DPlan> plans;
    std::vector<std::pair<uint8_t, int32_t>> plan_e;
    std::vector<uint32_t> snap_ids;
    std::vector<int> plan_nodes;  // nodes whose plan_slot is set (reset on exit)
    struct PlanReset {
        vc_verkle* t;
        const std::vector<int>& pn;
        const std::vector<uint32_t>& sn;
        ~PlanReset() {
            for (int id : pn) t->plan_slot[id] = -1;
            for (uint32_t id : sn) t->snap_slot[id] = -1;
        }
    } plan_reset{t, plan_nodes, snap_ids};
    if (use_delta && !t->slog.empty()) {
        // pass 1: a plan per logged parent, the first entry per (parent, slot) kept; snapshot slots
        std::vector<int32_t> kept(t->slog.size(), -1);  // its plan, or -1 for a repeated slot
        for (size_t i = 0; i < t->slog.size(); i++) {
            const auto& L = t->slog[i];
            int32_t p = t->plan_slot[L.parent];
            if (p < 0) {
                p = (int32_t)plans.size();
                plans.push_back(DPlan{{0, 0, 0, 0}, 0, 0});
                t->plan_slot[L.parent] = p;
                plan_nodes.push_back(L.parent);
            }
            DPlan& P = plans[p];
            if ((P.seen[L.slot >> 6] >> (L.slot & 63)) & 1) continue;
            P.seen[L.slot >> 6] |= 1ull << (L.slot & 63);
            P.cnt++;
            kept[i] = p;
            if (L.old >= 0 && t->snap_slot[L.old] < 0) {
                t->snap_slot[L.old] = (int32_t)snap_ids.size();
                snap_ids.push_back((uint32_t)L.old);
            }
        }
        // pass 2: the entries grouped by plan
        uint32_t run = 0;
        for (auto& P : plans) {
            P.start = run;
            run += P.cnt;
            P.cnt = 0;
        }
        plan_e.resize(run);
        for (size_t i = 0; i < t->slog.size(); i++) {
            if (kept[i] < 0) continue;
            const auto& L = t->slog[i];
            DPlan& P = plans[kept[i]];
            plan_e[P.start + P.cnt++] = {L.slot, L.old >= 0 ? t->snap_slot[L.old] : -1};
        }
    }
    DevBuf d_snap(ctx), d_snap_ids(ctx);
    if (!snap_ids.empty()) {
        const size_t S = snap_ids.size();
        VK_TRY(d_snap_ids.ensure(S * 4));
        VK_TRY(d_snap.ensure(S * 32));
        VK_CHECK_HIP(hipMemcpyAsync(d_snap_ids.p, snap_ids.data(), S * 4, hipMemcpyHostToDevice, st));
        VK_LAUNCH(ctx, "verkle_gather", k_vk_gather, grid(S), 256, 0, m_item, d_snap_ids.as<uint32_t>(), S,
                  d_snap.as<uint64_t>());
    }
    lap("delta plan");
    // one internal level's lists (column, child id[, snapshot index] per non-zero, node ids[, the
    // delta rows' add ids]) in page-locked memory for one upload: ints only, the values are the
    // children's items in the mirror (minus the snapshot for a delta row)
    struct LevelLists {
        int level = -1, status = VC_OK;
        size_t B = 0, nnz = 0, o_child = 0, o_ids = 0, o_sidx = 0, o_add = 0, o_end = 0;
        bool any_delta = false, dense = false;
        uvec<uint64_t> ptr;
        uint8_t* pin = nullptr;
    };
    const char* dense_env = getenv("VKZG_VERKLE_DENSE");
    const int dense_mode = dense_env ? atoi(dense_env) : -1;
    auto build_level = [&](int level, LevelLists& L, PinBuf& pinbuf) {
        const std::vector<int>& lv = t->dirty_int[level];
        const size_t B = lv.size();
        L.level = level;
        L.B = B;
        std::vector<const DPlan*> rplan(B, nullptr);
        bool any_delta = false;
        // the fixed-base latency path with host results for <= 64 full rows (the root: 0.44 -> 0.11
        // ms); VKZG_VERKLE_DENSE=0 / 1 (read per call, as the host path) forces sparse /
        // dense levels. A level of <= 64 rows commits full rows (delta rows would not shorten the
        // latency path's dependent adds).
        L.dense = dense_mode == 1 || (dense_mode != 0 && B <= 64);
        if (!plans.empty() && !L.dense)
            for (size_t b = 0; b < B; b++) {
                if (!t->base[lv[b]]) continue;
                const int32_t pi = t->plan_slot[lv[b]];
                if (pi < 0) continue;
                rplan[b] = &plans[pi];
                any_delta = true;
            }
        L.any_delta = any_delta;
        L.ptr.resize(B + 1);
        uvec<uint64_t>& ptr = L.ptr;
        ptr[0] = 0;
        for (size_t b = 0; b < B; b++)
            ptr[b + 1] = ptr[b] + (rplan[b] ? rplan[b]->cnt : t->nodes[lv[b]].children.v.size());
        const size_t nnz = ptr[B], nz1 = std::max<size_t>(nnz, 1);
        L.nnz = nnz;
        // layout: cols | child | ids | (delta) sidx | add_ids
        L.o_child = nz1 * 4;
        L.o_ids = L.o_child + nz1 * 4;
        L.o_sidx = L.o_ids + B * 4;
        L.o_add = L.o_sidx + (any_delta ? nz1 * 4 : 0);
        L.o_end = L.o_add + (any_delta ? B * 4 : 0);
        L.status = pinbuf.ensure(L.o_end);
        if (L.status != VC_OK) return;
        uint8_t* pin = pinbuf.as<uint8_t>();
        L.pin = pin;
        uint32_t* cols = reinterpret_cast<uint32_t*>(pin);
        uint32_t* child = reinterpret_cast<uint32_t*>(pin + L.o_child);
        uint32_t* ids = reinterpret_cast<uint32_t*>(pin + L.o_ids);
        int32_t* sidx = reinterpret_cast<int32_t*>(pin + L.o_sidx);
        uint32_t* add_ids = reinterpret_cast<uint32_t*>(pin + L.o_add);
        pool_for(0, B, 256, [&](size_t b) {
            size_t j = ptr[b];
            const VNode& n = t->nodes[lv[b]];
            ids[b] = (uint32_t)lv[b];
            if (rplan[b]) {
                for (uint32_t q = 0; q < rplan[b]->cnt; q++) {
                    const auto& e = plan_e[rplan[b]->start + q];
                    cols[j] = e.first;
                    child[j] = (uint32_t)n.children.find(e.first)->second;
                    sidx[j] = e.second;
                    j++;
                }
            } else {
                for (auto& kv : n.children.v) {
                    cols[j] = kv.first;
                    child[j] = (uint32_t)kv.second;
                    if (any_delta) sidx[j] = -1;
                    j++;
                }
            }
            if (any_delta) add_ids[b] = rplan[b] ? (uint32_t)lv[b] : 0xffffffffu;
        });
    };
    // internal nodes, deepest level first (width 256: the reference's hard-coded HACK). A level's
    // lists depend on the tree alone, so the next level's are built (into the other page-locked
    // buffer) while the current level's kernels run -- in the wait of its normalisation
    std::vector<int> order;
    for (int level = (int)t->dirty_int.size() - 1; level >= 0; level--)
        if (!t->dirty_int[level].empty()) order.push_back(level);
    LevelLists lists[2];
    size_t next_built = 0;  // levels of `order` whose lists are built
    // level cur's lists are in use: the other buffer takes order[cur + 1] (before the first level,
    // cur = 0 and both buffers are free: order[0] and order[1] may be built during the extension
    // commits' kernels)
    size_t cur = 0;
    auto build_next = [&]() {
        if (next_built < order.size() && next_built <= cur + 1) {
            build_level(order[next_built], lists[next_built & 1], ctx->pin_verkle_lv[next_built & 1]);
            next_built++;
        }
    };
    const std::function<void()> build_next_fn = build_next;
    // extension nodes: c1 / c2 rows (host: the leaves), then the width-4 rows on the device
    const std::vector<int>& exts = t->dirty_ext;
    const size_t E = exts.size();
    if (E) {
        static thread_local std::vector<ExtRows16> parts_cache[2];  // storage kept between calls
        // the rows in pieces (VKZG_VERKLE_EXT_PIECES, read per call; A/B knob, default 1): piece p
        // is built into page-locked buffer p & 1 while piece p - 1 crosses PCIe, each section of a
        // piece copied to its place in the level's device arrays (vals / cols at the non-zeros
        // before it: the device region holds the E 2 N upper bound). Measured slower at 65,536 keys
        // (full commitment 2.17-2.23 ms in one piece, 2.33-2.40 in 2, 2.49-2.53 in 4, 3 alternating
        // rounds, profiles/r06/verkle/pieces/): every piece pays the host pool's fork / join and
        // merge, more than the ~0.05-0.08 ms of upload it hides. One piece: the level's one buffer
        // in one copy.
        const char* pe = getenv("VKZG_VERKLE_EXT_PIECES");
        size_t NP = pe ? (size_t)std::max(1, atoi(pe)) : 1;
        const size_t cap = E * 2 * (size_t)N;  // non-zeros: at most 2 N per extension
        if (E < 4096 * NP || cap * 20 > ((size_t)256 << 20)) NP = 1;
        DevBuf d_up(ctx), d_vals(ctx), d_xy(ctx), d_inf(ctx), d_it(ctx);
        const uint64_t* d_stem = nullptr;
        const uint64_t* d_v16 = nullptr;
        const uint32_t* d_ids = nullptr;
        const uint32_t* d_cols = nullptr;
        const uint64_t* rp = nullptr;
        const uint64_t* d_rp_dev = nullptr;  // the row pointers on the device, when uploaded with the rows
        size_t nnz = 0;
        uint32_t maxlen = 0;
        static thread_local uvec<uint64_t> rp_all;
        if (NP == 1) {
            ExtStage X;
            VK_TRY(ext_stage(t, exts, pool, parts_cache[0],
                             [&](size_t bytes) -> uint8_t* {
                                 return ctx->pin_verkle.ensure(bytes) == VC_OK ? ctx->pin_verkle.as<uint8_t>() : nullptr;
                             },
                             &X));
            nnz = X.nnz;
            maxlen = X.maxlen;
            uint8_t* pin = X.base;
            rp = reinterpret_cast<const uint64_t*>(pin);
            lap("ext rows (host)");
            // the row pointers travel in the same copy: the sort-based commit reads them there
            // instead of uploading them again (one 1-MB copy and its gap less, profiles/r06/verkle/)
            VK_TRY(d_up.ensure(X.o_end));
            VK_CHECK_HIP(hipMemcpyAsync(d_up.p, pin, X.o_end, hipMemcpyHostToDevice, st));
            d_rp_dev = reinterpret_cast<const uint64_t*>(d_up.as<uint8_t>());
            d_stem = reinterpret_cast<const uint64_t*>(d_up.as<uint8_t>() + X.o_stem);
            d_v16 = reinterpret_cast<const uint64_t*>(d_up.as<uint8_t>() + X.o_vals);
            d_ids = reinterpret_cast<const uint32_t*>(d_up.as<uint8_t>() + X.o_ids);
            d_cols = reinterpret_cast<const uint32_t*>(d_up.as<uint8_t>() + X.o_cols);
        } else {
            // device: stems [E] x 32 B | ids [E] x 4 B | vals [cap] x 16 B | cols [cap] x 4 B
            const size_t o_ids = E * 32, o_vals = o_ids + E * 4, o_cols = o_vals + cap * 16;
            VK_TRY(d_up.ensure(o_cols + cap * 4));
            uint8_t* du = d_up.as<uint8_t>();
            rp_all.resize(2 * E + 1);
            hipEvent_t ev[2] = {nullptr, nullptr};
            struct Events {  // back to the pool on every exit, after the copies reading them finished
                vc_ctx* c;
                hipEvent_t* e;
                ~Events() {
                    for (int i = 0; i < 2; i++)
                        if (e[i]) {
                            (void)hipEventSynchronize(e[i]);
                            c->event_pool.push_back(e[i]);
                        }
                }
            } events{ctx, ev};
            std::vector<int> sub;
            for (size_t p = 0; p < NP; p++) {
                const size_t e0 = E * p / NP, e1 = E * (p + 1) / NP;
                sub.assign(exts.begin() + e0, exts.begin() + e1);
                PinBuf& pb = (p & 1) ? ctx->pin_verkle2 : ctx->pin_verkle;
                if (ev[p & 1]) VK_CHECK_HIP(hipEventSynchronize(ev[p & 1]));  // piece p - 2's copies are done
                ExtStage X;
                VK_TRY(ext_stage(t, sub, pool, parts_cache[p & 1],
                                 [&](size_t bytes) -> uint8_t* { return pb.ensure(bytes) == VC_OK ? pb.as<uint8_t>() : nullptr; },
                                 &X, nullptr, rp_all.data() + 2 * e0, nnz));
                const size_t ep = e1 - e0;
                uint8_t* pin = X.base;
                VK_CHECK_HIP(hipMemcpyAsync(du + e0 * 32, pin + X.o_stem, ep * 32, hipMemcpyHostToDevice, st));
                VK_CHECK_HIP(hipMemcpyAsync(du + o_ids + e0 * 4, pin + X.o_ids, ep * 4, hipMemcpyHostToDevice, st));
                if (X.nnz) {
                    VK_CHECK_HIP(hipMemcpyAsync(du + o_vals + nnz * 16, pin + X.o_vals, X.nnz * 16, hipMemcpyHostToDevice, st));
                    VK_CHECK_HIP(hipMemcpyAsync(du + o_cols + nnz * 4, pin + X.o_cols, X.nnz * 4, hipMemcpyHostToDevice, st));
                }
                if (!ev[p & 1]) ev[p & 1] = ctx->get_event();
                VK_CHECK_HIP(hipEventRecord(ev[p & 1], st));
                nnz += X.nnz;
                maxlen = std::max(maxlen, X.maxlen);
            }
            rp = rp_all.data();
            lap("ext rows (host, in pieces)");
            d_stem = reinterpret_cast<const uint64_t*>(du);
            d_ids = reinterpret_cast<const uint32_t*>(du + o_ids);
            d_v16 = reinterpret_cast<const uint64_t*>(du + o_vals);
            d_cols = reinterpret_cast<const uint32_t*>(du + o_cols);
        }
        VK_TRY(d_xy.ensure(2 * E * 64));
        VK_TRY(d_inf.ensure(2 * E));
        VK_TRY(d_it.ensure(2 * E * 32));
        if (small_ok(nnz)) {  // the 16-byte values read as they are
            SmallRows in;
            in.batch = 2 * E;
            in.row_ptr = rp;
            in.mode = 1;
            in.d_cols = d_cols;
            in.d_vals = d_v16;
            in.d_out_xy = d_xy.as<uint64_t>();
            in.d_out_inf = d_inf.as<uint8_t>();
            in.d_out_item = d_it.as<uint64_t>();
            VK_TRY(sparse_small_items_dev(ctx, tab, in));
        } else {
            VK_TRY(d_vals.ensure(std::max<size_t>(nnz, 1) * 32));
            if (nnz)
                VK_LAUNCH(ctx, "verkle_widen", k_vk_widen16, grid(nnz), 256, 0, d_v16, nnz, d_vals.as<uint64_t>());
            // rows of <= 4 non-zeros (random keys: one leaf per extension) are the sparse commit's
            // chunks as they are (an empty row is an empty chunk: the identity), no chunk lists
            VK_TRY(sparse_commit_items_dev(ctx, tab, 2 * E, rp, maxlen <= 4, d_cols, d_vals.p, d_xy.p,
                                           d_inf.as<uint8_t>(), d_it.p, nullptr, nullptr, nullptr, nullptr,
                                           order.empty() ? nullptr : &build_next_fn, d_rp_dev));
        }
        lap("ext c1 / c2 commits");
        // the width-4 rows use bases 0..3 only: their own table with 20-bit windows (13 instead of
        // 16 window adds per scalar, 3.5 GB; VKZG_VERKLE_LEAD_C: the window bits, 0 = the SRS's table)
        Table* tab4 = tab;
        {
            const char* lc = getenv("VKZG_VERKLE_LEAD_C");
            const int c4 = lc ? atoi(lc) : 20;
            if (c4 > 0 && tab->n >= 4 && c4 > tab->fb_c) {
                Table* lt = nullptr;
                VK_TRY(lead_table(ctx, tab, 4, c4, &lt));
                if (lt) tab4 = lt;
            }
        }
        DevBuf d_c4(ctx), d_v4(ctx);
        VK_TRY(d_c4.ensure(4 * E * 4));
        VK_TRY(d_v4.ensure(4 * E * 32));
        VK_LAUNCH(ctx, "verkle_ext_rows4", k_vk_ext_rows4, grid(4 * E), 256, 0, d_stem, d_it.as<uint64_t>(), E,
                  d_c4.as<uint32_t>(), d_v4.as<uint64_t>());
        // rows of 4: row_ptr[k] = 4 k, kept between calls (a fresh 0.5 MB vector's page faults and
        // fill were ~30 us of idle GPU before the width-4 commits)
        static thread_local uvec<uint64_t> rp4;
        if (rp4.size() < E + 1) {
            rp4.resize(E + 1);
            for (size_t k = 0; k <= E; k++) rp4[k] = 4 * k;
        }
        if (small_ok(4 * E)) {  // results straight into the mirror
            SmallRows in;
            in.batch = E;
            in.row_ptr = rp4.data();
            in.mode = 0;
            in.d_cols = d_c4.as<uint32_t>();
            in.d_vals = d_v4.as<uint64_t>();
            in.d_dst = d_ids;
            in.d_out_xy = m_cxy;
            in.d_out_inf = m_inf;
            in.d_out_item = m_item;
            VK_TRY(sparse_small_items_dev(ctx, tab4, in, order.empty() ? nullptr : &build_next_fn));
        } else {  // results straight into the mirror as well; row_ptr[k] = 4 k made on the device
            DevBuf d_rp4(ctx);
            VK_TRY(d_rp4.ensure((E + 1) * 8));
            VK_LAUNCH(ctx, "verkle_rp4", k_vk_rp4, grid(E + 1), 256, 0, d_rp4.as<uint64_t>(), E);
            VK_TRY(sparse_commit_items_dev(ctx, tab4, E, rp4.data(), true, d_c4.as<uint32_t>(), d_v4.p, m_cxy, m_inf,
                                           m_item, nullptr, nullptr, nullptr, d_ids,
                                           order.empty() ? nullptr : &build_next_fn, d_rp4.as<uint64_t>()));
        }
        lap("ext commits");
    }
    // the dense (host-result) levels' staging stays alive until the one sync at the end, and the
    // root's point is taken from them when the root was on such a level (no read-back)
    std::vector<std::vector<uint64_t>> keep64;
    std::vector<std::vector<uint8_t>> keep8;
    std::vector<uvec<uint32_t>> keep32;
    uint64_t root_xy[8];
    uint8_t root_inf = 1;
    bool root_known = false;
    for (size_t oi = 0; oi < order.size(); oi++) {
        cur = oi;
        if (next_built <= oi) build_next();
        LevelLists& L = lists[oi & 1];
        if (L.status != VC_OK) return L.status;
        const size_t B = L.B, nnz = L.nnz, nz1 = std::max<size_t>(nnz, 1);
        const uvec<uint64_t>& ptr = L.ptr;
        DevBuf d_up(ctx);
        VK_TRY(d_up.ensure(L.o_end));
        VK_CHECK_HIP(hipMemcpyAsync(d_up.p, L.pin, L.o_end, hipMemcpyHostToDevice, st));
        const uint32_t* d_cols = d_up.as<uint32_t>();
        const uint32_t* d_child = reinterpret_cast<const uint32_t*>(d_up.as<uint8_t>() + L.o_child);
        const uint32_t* d_ids = reinterpret_cast<const uint32_t*>(d_up.as<uint8_t>() + L.o_ids);
        const int32_t* d_sidx = L.any_delta ? reinterpret_cast<const int32_t*>(d_up.as<uint8_t>() + L.o_sidx) : nullptr;
        const uint32_t* d_add = L.any_delta ? reinterpret_cast<const uint32_t*>(d_up.as<uint8_t>() + L.o_add) : nullptr;
        // the next level's lists go into the other buffer while this level runs
        const std::function<void()>* ov = next_built < order.size() ? &build_next_fn : nullptr;
        if (L.dense) {
            // dense rows gathered on the device, committed on the latency path (host results), the
            // <= 64 items on the host, results uploaded into the mirror
            uvec<uint32_t> row(nz1);
            for (size_t b = 0; b < B; b++)
                for (uint64_t j = ptr[b]; j < ptr[b + 1]; j++) row[j] = (uint32_t)b;
            DevBuf d_row(ctx), d_dense(ctx), d_xy(ctx), d_inf(ctx), d_it(ctx);
            VK_TRY(d_row.ensure(nz1 * 4));
            VK_TRY(d_dense.ensure(B * 256 * 32));
            VK_TRY(d_xy.ensure(B * 64));
            VK_TRY(d_inf.ensure(B));
            VK_TRY(d_it.ensure(B * 32));
            VK_CHECK_HIP(hipMemsetAsync(d_dense.p, 0, B * 256 * 32, st));
            if (nnz) {
                VK_CHECK_HIP(hipMemcpyAsync(d_row.p, row.data(), nnz * 4, hipMemcpyHostToDevice, st));
                VK_LAUNCH(ctx, "verkle_dense", k_vk_dense, grid(nnz), 256, 0, d_row.as<uint32_t>(), d_cols, d_child,
                          nnz, m_item, 256u, d_dense.as<uint64_t>());
            }
            std::vector<uint64_t> hxy(B * 8), hit(B * 4);
            std::vector<uint8_t> hinf(B);
            bool on_host = false;
            VK_TRY(msm_batch_run(ctx, tab, 256, d_dense.p, B, 0, d_xy.p, d_inf.as<uint8_t>(), hxy.data(), hinf.data(),
                                 &on_host, nullptr, ov));
            if (!on_host) {
                VK_CHECK_HIP(hipMemcpyAsync(hxy.data(), d_xy.p, B * 64, hipMemcpyDeviceToHost, st));
                VK_CHECK_HIP(hipMemcpyAsync(hinf.data(), d_inf.p, B, hipMemcpyDeviceToHost, st));
                VK_CHECK_HIP(hipStreamSynchronize(st));
            }
            for (size_t b = 0; b < B; b++) mont_to_canon<BN254Fr>(to_data_item_host(&hxy[8 * b], hinf[b] != 0), &hit[4 * b]);
            VK_CHECK_HIP(hipMemcpyAsync(d_xy.p, hxy.data(), B * 64, hipMemcpyHostToDevice, st));
            VK_CHECK_HIP(hipMemcpyAsync(d_inf.p, hinf.data(), B, hipMemcpyHostToDevice, st));
            VK_CHECK_HIP(hipMemcpyAsync(d_it.p, hit.data(), B * 32, hipMemcpyHostToDevice, st));
            VK_TRY(scatter(d_ids, B, d_xy.p, d_inf.as<uint8_t>(), d_it.p));
            const uint32_t* h_ids = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(L.pin) + L.o_ids);
            for (size_t b = 0; b < B; b++)
                if (h_ids[b] == 0) {  // the root (node id 0)
                    memcpy(root_xy, &hxy[8 * b], 64);
                    root_inf = hinf[b];
                    root_known = true;
                }
            // the uploads above read these host vectors: kept (not synchronised) until the end
            keep64.push_back(std::move(hxy));
            keep64.push_back(std::move(hit));
            keep8.push_back(std::move(hinf));
            keep32.push_back(std::move(row));
            lap("internal level (dense)");
            continue;
        }
        if (small_ok(nnz)) {  // children's items gathered in the kernel; results into the mirror
            SmallRows in;
            in.batch = B;
            in.row_ptr = ptr.data();
            in.mode = 2;
            in.d_cols = d_cols;
            in.d_item = m_item;
            in.d_child = d_child;
            in.d_sidx = d_sidx;
            in.d_snap = d_snap.as<uint64_t>();
            in.d_add_ids = d_add;
            in.d_add_xy = m_cxy;
            in.d_add_inf = m_inf;
            in.d_dst = d_ids;
            in.d_out_xy = m_cxy;
            in.d_out_inf = m_inf;
            in.d_out_item = m_item;
            VK_TRY(sparse_small_items_dev(ctx, tab, in, ov));
            lap(L.any_delta ? "internal level (small, delta rows)" : "internal level (small)");
            continue;
        }
        DevBuf d_vals(ctx);
        VK_TRY(d_vals.ensure(nz1 * 32));
        if (L.any_delta) {
            if (nnz)
                VK_LAUNCH(ctx, "verkle_delta", k_vk_delta, grid(nnz), 256, 0, m_item, d_child, d_sidx,
                          d_snap.as<uint64_t>(), nnz, d_vals.as<uint64_t>());
        } else if (nnz) {
            VK_LAUNCH(ctx, "verkle_gather", k_vk_gather, grid(nnz), 256, 0, m_item, d_child, nnz, d_vals.as<uint64_t>());
        }
        // results straight into the mirror (a delta row's old commitment is read there by the first
        // normalisation kernel, its new one written by the second); the next level's lists are built
        // once this level's kernels are queued
        VK_TRY(sparse_commit_items_dev(ctx, tab, B, ptr.data(), false, d_cols, d_vals.p, m_cxy, m_inf, m_item, d_add,
                                       m_cxy, m_inf, d_ids, ov));
        lap(L.any_delta ? "internal level (sparse, delta rows)" : "internal level (sparse)");
    }
    // the root's commitment from the mirror (the rest stays there: host_valid = false)
    uint64_t rxy[8];
    uint8_t rinf = 1;
    if (root_known) {  // the root's level ran on the host-result path
        memcpy(rxy, root_xy, 64);
        rinf = root_inf;
    } else {
        VK_CHECK_HIP(hipMemcpyAsync(rxy, m_cxy, 64, hipMemcpyDeviceToHost, st));
        VK_CHECK_HIP(hipMemcpyAsync(&rinf, m_inf, 1, hipMemcpyDeviceToHost, st));
    }
    VK_CHECK_HIP(hipStreamSynchronize(st));  // also: every staging vector above may die now
    lap(root_known ? "final sync (root from the dense level)" : "root read-back");
    memcpy(out_xy, rxy, 64);
    *out_inf = rinf;
    t->clear_dirty();
    t->host_valid = false;
    delta_guard.ok = true;
    lap("dirty lists cleared");
    return VC_OK;
}

}  // namespace vk
