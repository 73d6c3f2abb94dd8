// Declarations of the scalar-field device routines (poly.hip) used by the protocol layer.
#pragma once
#include "ctx.hpp"
#include "ec.hpp"

namespace vk {
template <class F>
int domain_powers(vc_ctx* ctx, const fe<F>& w, size_t n, fe<F>* d_out);
template <class F>
int batch_inverse(vc_ctx* ctx, const fe<F>* d_in, fe<F>* d_out, size_t n);
// per-ctx cached domain tables of size n (w = the n-th root of unity): pw[i] = w^i,
// pwi[i] = w^-i, inv1[k] = 1/(w^k - 1) (k > 0; inv1[0] unused)
template <class F>
int domain_tables(vc_ctx* ctx, const fe<F>& w, size_t n, const fe<F>** pw, const fe<F>** pwi, const fe<F>** inv1);
template <class F>
int kzg_quotient_dev(vc_ctx* ctx, size_t n, const fe<F>* d_f, size_t max, const fe<F>& point, const fe<F>& omega,
                     fe<F>* d_q, fe<F>* y_out, DevBuf& pw, DevBuf& tmp, DevBuf& part);
// index-range shards of the quotient (vc_group_kzg_prove): phase 1 writes q (in domain) or the
// slice's inverses (outside) and returns this share's partial of the global sum; phase 2 takes
// the members' total (poly.hip)
template <class F>
int kzg_range_part(vc_ctx* ctx, size_t n, const fe<F>* d_f, size_t nvalid, size_t lo, size_t L, const fe<F>& point,
                   const fe<F>& omega, bool in_domain, size_t m, const fe<F>& fm, fe<F>* d_q, fe<F>* d_inv,
                   DevBuf& part, fe<F>* partial);
template <class F>
int kzg_range_finish(vc_ctx* ctx, size_t n, const fe<F>* d_f, size_t nvalid, size_t lo, size_t L, const fe<F>& point,
                     const fe<F>& omega, bool in_domain, size_t m, const fe<F>& total, fe<F>* d_q, const fe<F>* d_inv,
                     fe<F>* y_mont);
template <class F>
int canon_to_mont_dev(vc_ctx* ctx, const void* d_in, size_t n, size_t n_valid, fe<F>* d_out);
template <class F>
int mont_to_canon_dev(vc_ctx* ctx, const fe<F>* d_in, size_t n, void* d_out);
template <class C, class Fr>
int kzg_srs_dev(vc_ctx* ctx, size_t max_items, size_t n, const fe<Fr>& s_mont, const fe<Fr>& omega,
                const typename C::Aff& g, typename C::Acc* d_out);
}  // namespace vk
