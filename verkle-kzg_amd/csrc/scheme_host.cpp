// Host-side protocol pieces (serial by nature): Fiat-Shamir transcript, hash_to_field,
// arkworks compressed encoding, IPA CRS generation. Exported through include/vc_scheme.h.
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/vc_scheme.h"
#include "host/fr.hpp"
#include "host/pool.hpp"
#include "host/sha256.hpp"
#include "scheme_internal.hpp"

namespace vk {

// ---------------------------------------------------------------- hash_to_field
// ark-ff 0.4 DefaultFieldHasher<Sha256, 128>: len_per_elem = ceil((254 + 128) / 8) = 48;
// ExpanderXmd { block_size: 48 } (z_pad of 48 zero bytes); output bytes read
// big-endian and reduced mod r.
static const size_t kLenPerElem = 48;

// the message reaches the hash through `feed` (a contiguous buffer, or records made chunk by chunk)
template <class Feed>
static void expand_message_xmd_feed(Feed&& feed, const uint8_t* dst, size_t dlen, size_t out_len, uint8_t* out) {
    Sha256 h;
    std::vector<uint8_t> dst_prime(dst, dst + dlen);
    dst_prime.push_back((uint8_t)dlen);  // DST <= 255 bytes here (labels)
    uint8_t zpad[kLenPerElem] = {0};
    uint8_t lib[2] = {(uint8_t)(out_len >> 8), (uint8_t)out_len};
    uint8_t zero = 0;
    h.update(zpad, sizeof zpad);
    feed(h);
    h.update(lib, 2);
    h.update(&zero, 1);
    h.update(dst_prime.data(), dst_prime.size());
    uint8_t b0[32], bi[32];
    h.final(b0);
    uint8_t one = 1;
    h.update(b0, 32);
    h.update(&one, 1);
    h.update(dst_prime.data(), dst_prime.size());
    h.final(bi);
    size_t ell = (out_len + 31) / 32;
    std::vector<uint8_t> u(bi, bi + 32);
    for (size_t i = 2; i <= ell; i++) {
        uint8_t x[32];
        for (int k = 0; k < 32; k++) x[k] = b0[k] ^ bi[k];
        uint8_t ib = (uint8_t)i;
        h.update(x, 32);
        h.update(&ib, 1);
        h.update(dst_prime.data(), dst_prime.size());
        h.final(bi);
        u.insert(u.end(), bi, bi + 32);
    }
    memcpy(out, u.data(), out_len);
}

void expand_message_xmd(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dlen, size_t out_len,
                        uint8_t* out) {
    expand_message_xmd_feed([&](Sha256& h) { h.update(msg, n); }, dst, dlen, out_len, out);
}

Fr hash_to_fr(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dlen) {
    uint8_t u[kLenPerElem];
    expand_message_xmd(msg, n, dst, dlen, kLenPerElem, u);
    return fe_from_be_bytes_mod<BN254Fr>(u, kLenPerElem);
}

// ---------------------------------------------------------------- compressed encoding
// SWFlags: byte[31] |= 0x80 if y > -y (YIsNegative), 0x40 for infinity (x = 0)
void compress_g1(const uint64_t* xy, bool inf, uint8_t out[32]) {
    memset(out, 0, 32);
    if (inf) {
        out[31] |= 0x40;
        return;
    }
    memcpy(out, xy, 32);
    Fq y = from_words<BN254Fq>(xy + 4);
    Fq ny = fe_sub<BN254Fq>(fe_zero<BN254Fq>(), y);  // canonical p - y (y != 0 on BN254 G1)
    if (canon_cmp<BN254Fq>(y, ny) > 0) out[31] |= 0x80;
}

Fr to_data_item_host(const uint64_t* xy, bool inf) {
    if (inf) return fe_zero<BN254Fr>();
    uint8_t b[32];
    compress_g1(xy, false, b);
    return fe_from_le_bytes_mod<BN254Fr>(b, 32);
}

// ---------------------------------------------------------------- from_random_bytes (A.6)
static bool from_random_bytes(const uint8_t b[32], uint64_t out[8], bool* inf) {
    uint8_t flags = b[31] & 0xC0;
    uint8_t xb[32];
    memcpy(xb, b, 32);
    xb[31] &= 0x3F;
    Fq x;
    memcpy(x.v, xb, 32);
    if (!fe_eq<BN254Fq>(fe_reduce_once<BN254Fq>(x), x)) return false;  // x >= p
    bool sign = flags & 0x80, infb = flags & 0x40;
    if (sign && infb) return false;
    if (infb) {
        if (!fe_is_zero<BN254Fq>(x)) return false;
        *inf = true;
        memset(out, 0, 64);
        return true;
    }
    Fq xm = fe_to_mont<BN254Fq>(x);
    Fq rhs = fe_add<BN254Fq>(fe_mul<BN254Fq>(fe_sqr<BN254Fq>(xm), xm), mont_from_u64<BN254Fq>(3));
    // p = 3 mod 4: sqrt = rhs^((p+1)/4)
    Fq e;
    for (int i = 0; i < 8; i++) e.v[i] = BN254Fq::p(i);
    // (p + 1) / 4
    uint64_t c = 1;
    for (int i = 0; i < 8; i++) {
        uint64_t s = (uint64_t)e.v[i] + c;
        e.v[i] = (uint32_t)s;
        c = s >> 32;
    }
    for (int k = 0; k < 2; k++) {
        for (int i = 0; i < 7; i++) e.v[i] = (e.v[i] >> 1) | (e.v[i + 1] << 31);
        e.v[7] >>= 1;
    }
    Fq y = fe_pow_fe<BN254Fq, BN254Fq>(rhs, e);
    if (!fe_eq<BN254Fq>(fe_sqr<BN254Fq>(y), rhs)) return false;  // non-residue
    Fq yc = fe_from_mont<BN254Fq>(y);
    Fq nyc = fe_sub<BN254Fq>(fe_zero<BN254Fq>(), yc);
    bool y_is_smaller = canon_cmp<BN254Fq>(yc, nyc) <= 0;
    Fq smaller = y_is_smaller ? yc : nyc, larger = y_is_smaller ? nyc : yc;
    bool greatest = !sign;  // YIsPositive -> get_point_from_x_unchecked(x, true) -> larger
    Fq yy = greatest ? larger : smaller;
    memcpy(out, x.v, 32);
    memcpy(out + 4, yy.v, 32);
    *inf = false;
    return true;
}

}  // namespace vk

using namespace vk;

struct vc_transcript {
    std::vector<uint8_t> state;
    std::string dst;
};

extern "C" {

int vc_host_sha256_path(void) { return vk::sha256_have_shani() ? 1 : 0; }

vc_transcript* vc_transcript_new(const char* label) {
    vc_transcript* t = new vc_transcript();
    t->dst = label ? label : "";
    return t;
}
vc_transcript* vc_transcript_clone(const vc_transcript* t) { return t ? new vc_transcript(*t) : nullptr; }
void vc_transcript_free(vc_transcript* t) { delete t; }
void vc_transcript_reserve(vc_transcript* t, size_t bytes) {
    if (t) t->state.reserve(bytes);
}

int vc_transcript_append_bytes(vc_transcript* t, const uint8_t* b, size_t n, const char* label) {
    if (!t || (n && !b)) return VC_E_INVALID;
    if (label) t->state.insert(t->state.end(), label, label + strlen(label));
    t->state.insert(t->state.end(), b, b + n);
    return VC_OK;
}
int vc_transcript_append_point(vc_transcript* t, const uint64_t* xy, uint8_t inf, const char* label) {
    if (!t || (!xy && !inf)) return VC_E_INVALID;
    uint8_t c[32];
    uint64_t zero[8] = {0};
    compress_g1(inf ? zero : xy, inf != 0, c);
    return vc_transcript_append_bytes(t, c, 32, label);
}
int vc_transcript_append_fr(vc_transcript* t, const uint64_t* fr, const char* label) {
    if (!t || !fr) return VC_E_INVALID;
    return vc_transcript_append_bytes(t, reinterpret_cast<const uint8_t*>(fr), 32, label);
}
int vc_transcript_append_u64(vc_transcript* t, uint64_t v, const char* label) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (8 * i));
    return vc_transcript_append_bytes(t, b, 8, label);
}
int vc_transcript_digest(vc_transcript* t, const char* label, uint64_t* out) {
    if (!t || !out) return VC_E_INVALID;
    Fr r = transcript_digest(t, label);
    mont_to_canon<BN254Fr>(r, out);
    return VC_OK;
}
int vc_hash_to_field(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dlen, uint64_t* out) {
    if ((n && !msg) || !out || (dlen && !dst) || dlen > 255) return VC_E_INVALID;
    mont_to_canon<BN254Fr>(hash_to_fr(msg, n, dst, dlen), out);
    return VC_OK;
}
int vc_point_compress(const uint64_t* xy, uint8_t inf, uint8_t* out32) {
    if (!out32 || (!xy && !inf)) return VC_E_INVALID;
    uint64_t zero[8] = {0};
    compress_g1(inf ? zero : xy, inf != 0, out32);
    return VC_OK;
}
int vc_ipa_crs(const uint8_t* seed, size_t seed_len, size_t max, size_t num, uint64_t* out_xy) {
    if ((seed_len && !seed) || (num && !out_xy)) return VC_E_INVALID;
    if (num > max) return VC_E_RANGE;  // PointGeneratorError::OutOfBounds
    size_t got = 0;
    for (uint64_t i = 0; got < num; i++) {
        Sha256 h;
        uint8_t le[8];
        for (int k = 0; k < 8; k++) le[k] = (uint8_t)(i >> (8 * k));
        h.update(seed, seed_len);
        h.update(le, 8);
        uint8_t d[32];
        h.final(d);
        bool inf = false;
        if (from_random_bytes(d, out_xy + 8 * got, &inf)) {
            if (inf) continue;  // identity cannot be a base in the affine table (prob. ~2^-256)
            got++;
        }
    }
    return VC_OK;
}

}  // extern "C"

namespace vk {
Fr transcript_digest(vc_transcript* t, const char* label) {
    if (label) t->state.insert(t->state.end(), label, label + strlen(label));
    Fr r = hash_to_fr(t->state.data(), t->state.size(), reinterpret_cast<const uint8_t*>(t->dst.data()),
                      t->dst.size());
    uint64_t w[4];
    mont_to_canon<BN254Fr>(r, w);
    t->state.assign(reinterpret_cast<uint8_t*>(w), reinterpret_cast<uint8_t*>(w) + 32);
    if (label) t->state.insert(t->state.end(), label, label + strlen(label));
    return r;
}
// transcript_digest of state || records || label without storing the records: `fill(lo, hi, out)`
// writes records [lo, hi) (rec bytes each) into out; the hash takes them chunk by chunk. With a
// pool, worker 0 hashes chunk k while the others make chunk k + 1, so the digest costs about the
// SHA-256 of the records alone -- the state of a 2^16-query multiproof is 4.9 MB, and building it
// first (allocation, zero fill, page faults, then the hash) took ~1.5-2x as long on this host.
// Same r and the same post-digest state as transcript_extend + fill + transcript_digest.
Fr transcript_digest_records(vc_transcript* t, size_t nrec, size_t rec, const RecordFill& fill, const char* label,
                             bool pool_ok) {
    constexpr size_t CH = 4096;  // records per chunk (~300 KB)
    HostPool& P = host_pool();
    // pool_ok: the shared host pool fills the next chunk while its worker 0 hashes; otherwise a
    // filler thread of the call's own does (concurrent transcripts -- a stream of multiproofs,
    // mp_prove_many's workers -- then run side by side instead of queueing on the one pool)
    const unsigned T = pool_ok ? P.size() : 1;
    const bool helper_ok = !pool_ok;
    std::vector<uint8_t> buf[2];
    buf[0].resize(std::min(nrec, CH) * rec);
    buf[1].resize(std::min(nrec, CH) * rec);
    const size_t nch = (nrec + CH - 1) / CH;
    auto chunk_fill = [&](size_t k, unsigned part, unsigned parts) {
        const size_t lo = k * CH, hi = std::min(nrec, lo + CH), n = hi - lo;
        const size_t a = lo + n * part / parts, b = lo + n * (part + 1) / parts;
        if (b > a) fill(a, b, buf[k & 1].data() + (a - lo) * rec);
    };
    auto feed = [&](Sha256& h) {
        h.update(t->state.data(), t->state.size());
        auto serial = [&] {
            for (size_t k = 0; k < nch; k++) {
                chunk_fill(k, 0, 1);
                h.update(buf[k & 1].data(), (std::min(nrec, (k + 1) * CH) - k * CH) * rec);
            }
        };
        if (nch > 0) {
            if (T == 1 && nch >= 2 && helper_ok) {
                // one filler thread of this call's own, a chunk ahead of the hash (double buffer;
                // both sides block rather than spin: spinning threads ate the CPU quota the host
                // pool's workers needed beside them)
                std::mutex mu;
                std::condition_variable cv;
                size_t filled = 0, hashed = 0;  // under mu; filled = nch + 1: the filler failed
                std::exception_ptr err;
                std::thread filler;
                bool threaded = true;
                try {
                    filler = std::thread([&] {
                        try {
                            for (size_t k = 0; k < nch; k++) {
                                {
                                    std::unique_lock<std::mutex> lk(mu);
                                    cv.wait(lk, [&] { return k < hashed + 2; });
                                }
                                chunk_fill(k, 0, 1);
                                std::lock_guard<std::mutex> lk(mu);
                                filled = k + 1;
                                cv.notify_all();
                            }
                        } catch (...) {
                            std::lock_guard<std::mutex> lk(mu);
                            err = std::current_exception();
                            filled = nch + 1;
                            cv.notify_all();
                        }
                    });
                } catch (const std::system_error&) {  // no thread to be had: fill in line
                    threaded = false;
                    serial();
                }
                for (size_t k = 0; threaded && k < nch; k++) {
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return filled > k; });
                        if (filled > nch) break;  // the filler failed
                    }
                    h.update(buf[k & 1].data(), (std::min(nrec, (k + 1) * CH) - k * CH) * rec);
                    std::lock_guard<std::mutex> lk(mu);
                    hashed = k + 1;
                    cv.notify_all();
                }
                if (threaded) filler.join();
                if (err) std::rethrow_exception(err);
            } else if (T == 1) {
                serial();
            } else {
                P.run([&](unsigned w) { chunk_fill(0, w, T); });
                for (size_t k = 0; k < nch; k++) {
                    const size_t bytes = (std::min(nrec, (k + 1) * CH) - k * CH) * rec;
                    P.run([&](unsigned w) {
                        if (w == 0) h.update(buf[k & 1].data(), bytes);
                        else if (k + 1 < nch) chunk_fill(k + 1, w - 1, T - 1);
                    });
                }
            }
        }
        if (label) h.update(label, strlen(label));
    };
    uint8_t u[kLenPerElem];
    expand_message_xmd_feed(feed, reinterpret_cast<const uint8_t*>(t->dst.data()), t->dst.size(), kLenPerElem, u);
    const Fr r = fe_from_be_bytes_mod<BN254Fr>(u, kLenPerElem);
    uint64_t w[4];
    mont_to_canon<BN254Fr>(r, w);
    t->state.assign(reinterpret_cast<uint8_t*>(w), reinterpret_cast<uint8_t*>(w) + 32);
    if (label) t->state.insert(t->state.end(), label, label + strlen(label));
    return r;
}

uint8_t* transcript_extend(vc_transcript* t, size_t n) {
    const size_t at = t->state.size();
    t->state.resize(at + n);
    return t->state.data() + at;
}
void transcript_append_point(vc_transcript* t, const uint64_t* xy, bool inf, const char* label) {
    vc_transcript_append_point(t, xy, inf ? 1 : 0, label);
}
void transcript_append_fr(vc_transcript* t, const Fr& mont, const char* label) {
    uint64_t w[4];
    mont_to_canon<BN254Fr>(mont, w);
    vc_transcript_append_fr(t, w, label);
}
}  // namespace vk
