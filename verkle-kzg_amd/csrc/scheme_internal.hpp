// Internal declarations shared by the protocol-layer translation units.
#pragma once
#include <stdint.h>

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
Fr to_data_item_host(const uint64_t* xy, bool inf);

}  // namespace vk
