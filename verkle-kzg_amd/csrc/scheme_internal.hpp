// Internal declarations shared by the protocol-layer translation units.
#pragma once
#include <stdint.h>

#include <functional>

#include "../../include/vc_scheme.h"
#include "host/fr.hpp"

namespace vk {

Fr transcript_digest(vc_transcript* t, const char* label);
void transcript_append_point(vc_transcript* t, const uint64_t* xy, bool inf, const char* label);
void transcript_append_fr(vc_transcript* t, const Fr& mont, const char* label);
Fr hash_to_fr(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dlen);
void compress_g1(const uint64_t* xy, bool inf, uint8_t out[32]);
// grow the transcript state by n bytes and return the start of the new region (callers that
// serialise many records on several threads)
uint8_t* transcript_extend(vc_transcript* t, size_t n);
// transcript_digest of the state followed by nrec records of rec bytes (made by fill(lo, hi, out)
// chunk by chunk, never stored whole) and the label; pool_ok: make them on the host pool
using RecordFill = std::function<void(size_t lo, size_t hi, uint8_t* out)>;
Fr transcript_digest_records(vc_transcript* t, size_t nrec, size_t rec, const RecordFill& fill, const char* label,
                             bool pool_ok);
Fr to_data_item_host(const uint64_t* xy, bool inf);
// vc_multiproof_begin + vc_multiproof_accumulate of the query shard [first, first + Qs), the host
// transcript on a helper thread while this thread plans the shard (scheme.hip); r_out canonical
// the number of distinct z (rows of the per-point sums); VC_E_DOMAIN for z >= N
int mp_rows(size_t N, size_t Q, const uint64_t* z, size_t* rows);
int mp_begin_accumulate(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                        const uint64_t* z, const uint64_t* y, size_t first, size_t Qs, const void* d_data, void* d_S,
                        vc_transcript** tr_out, uint64_t* r_out);

}  // namespace vk
