// jr_host.cpp — host-side (CPU) helpers of libjr: CRC32C for the TFRecord
// container the reference reads through tf.data.TFRecordDataset
// (lib/dataset.py:5-8).  A TFRecord is
//   uint64 length | uint32 masked_crc32c(length) | bytes | uint32 masked_crc32c(bytes)
// with mask(c) = ((c >> 15) | (c << 17)) + 0xa282ead8  [TF-3P record format].
// Uses the SSE4.2 crc32 instruction (CRC32C / Castagnoli polynomial).
#include <nmmintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "jr_common.h"

__attribute__((target("sse4.2"))) static uint32_t crc32c_sse(const uint8_t* p, size_t n, uint32_t crc) {
  crc = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    crc = (uint32_t)_mm_crc32_u64(crc, v);
    p += 8;
    n -= 8;
  }
  while (n--) crc = _mm_crc32_u8(crc, *p++);
  return ~crc;
}

JR_API uint32_t jr_crc32c(const uint8_t* data, size_t n, uint32_t crc) { return crc32c_sse(data, n, crc); }

JR_API uint32_t jr_masked_crc32c(const uint8_t* data, size_t n) {
  const uint32_t c = crc32c_sse(data, n, 0);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}
