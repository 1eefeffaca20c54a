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

#include "jr_error.h"

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

// ---------------------------------------------------------------------------
// TFRecord file index and tf.train.Example parsing for the lib/dataset.py
// input pipeline (§8 f1).  The Python reader walked every record and every
// protobuf level in the interpreter (≈230 µs per 77 KiB record on the main
// thread); here a whole file image (mmap'd by the caller) is indexed in one
// call and the five FixedLenFeatures of lib/dataset.py:12-16 are located in
// one call per batch of records, so the host loop touches only offsets.
// ---------------------------------------------------------------------------

static uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// Records are indexed up to the first damaged one: *n_records is the number of
// good records in front of it and the status says what was wrong, so the
// caller yields those records and raises where tf.data would (DataLossError on
// reaching the bad record).  offsets == nullptr only counts.
JR_API int jr_tfrecord_index(const uint8_t* buf, size_t len, int verify, uint64_t* offsets, uint64_t* lengths,
                             size_t cap, size_t* n_records) {
  if (!n_records || (len && !buf) || (offsets && !lengths)) {
    jr::set_error("jr_tfrecord_index: null argument");
    return JR_ERR_INVALID;
  }
  size_t pos = 0, n = 0;
  int st = JR_OK;
  while (pos < len) {
    if (len - pos < 12) {
      jr::set_error("truncated record header at byte " + std::to_string(pos));
      st = JR_ERR_INVALID;
      break;
    }
    uint64_t rl;
    uint32_t lc;
    memcpy(&rl, buf + pos, 8);
    memcpy(&lc, buf + pos + 8, 4);
    if (verify && masked(crc32c_sse(buf + pos, 8, 0)) != lc) {
      jr::set_error("corrupted record length at byte " + std::to_string(pos));
      st = JR_ERR_INVALID;
      break;
    }
    if (rl > len - pos - 12 || len - pos - 12 - rl < 4) {
      jr::set_error("truncated record at byte " + std::to_string(pos));
      st = JR_ERR_INVALID;
      break;
    }
    const uint8_t* data = buf + pos + 12;
    uint32_t dc;
    memcpy(&dc, data + rl, 4);
    if (verify && masked(crc32c_sse(data, rl, 0)) != dc) {
      jr::set_error("corrupted record data at byte " + std::to_string(pos));
      st = JR_ERR_INVALID;
      break;
    }
    if (offsets) {
      if (n >= cap) {
        jr::set_error("jr_tfrecord_index: more records than capacity");
        *n_records = n;
        return JR_ERR_INVALID;
      }
      offsets[n] = pos + 12;
      lengths[n] = rl;
    }
    ++n;
    pos += 12 + rl + 4;
  }
  *n_records = n;
  return st;
}

namespace {

// Bounded protobuf reader over [p, end).
struct Pb {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  bool varint(uint64_t* v) {
    uint64_t r = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= end) return ok = false;
      const uint8_t b = *p++;
      r |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) {
        *v = r;
        return true;
      }
    }
    return ok = false;
  }
  // Length-delimited payload -> [*q, *qe).
  bool bytes(const uint8_t** q, const uint8_t** qe) {
    uint64_t n;
    if (!varint(&n) || n > (uint64_t)(end - p)) return ok = false;
    *q = p;
    *qe = p + n;
    p += n;
    return true;
  }
  bool skip(int wire) {
    uint64_t v;
    const uint8_t *q, *qe;
    switch (wire) {
      case 0: return varint(&v);
      case 1: if (end - p < 8) return ok = false; p += 8; return true;
      case 2: return bytes(&q, &qe);
      case 5: if (end - p < 4) return ok = false; p += 4; return true;
      default: return ok = false;
    }
  }
};

// The five keys of lib/dataset.py:12-16 and the list kind each must carry
// (Feature.kind: 1 bytes_list, 2 float_list, 3 int64_list).
constexpr int kKeys = 5;
const char* const kKeyName[kKeys] = {"image/encoded", "image/format", "image/class/label", "image/height",
                                     "image/width"};
const int kKeyKind[kKeys] = {1, 1, 3, 3, 3};

struct Slot {
  int kind = 0;     // last Feature.kind seen (oneof: last wins)
  int64_t count = 0;
  const uint8_t* b = nullptr;  // first bytes value
  uint64_t blen = 0;
  int64_t i = 0;    // first int64 value
};

// Feature message -> slot (kind, value count, first value).
bool parse_feature(const uint8_t* q, const uint8_t* qe, Slot* s) {
  Pb f{q, qe};
  while (f.p < f.end) {
    uint64_t key;
    if (!f.varint(&key)) return false;
    const int num = (int)(key >> 3), wire = (int)(key & 7);
    if (wire != 2 || num < 1 || num > 3) {
      if (!f.skip(wire)) return false;
      continue;
    }
    const uint8_t *l, *le;
    if (!f.bytes(&l, &le)) return false;
    *s = Slot();
    s->kind = num;
    Pb v{l, le};
    while (v.p < v.end) {
      uint64_t k2;
      if (!v.varint(&k2)) return false;
      if ((k2 >> 3) != 1) return false;  // only field 1 ("value") in a list
      const int w2 = (int)(k2 & 7);
      if (num == 1) {
        const uint8_t *b, *be;
        if (w2 != 2 || !v.bytes(&b, &be)) return false;
        if (s->count++ == 0) {
          s->b = b;
          s->blen = (uint64_t)(be - b);
        }
      } else if (num == 2) {
        if (w2 == 2) {
          const uint8_t *b, *be;
          if (!v.bytes(&b, &be) || (be - b) % 4) return false;
          s->count += (be - b) / 4;
        } else if (w2 == 5) {
          if (!v.skip(5)) return false;
          s->count++;
        } else {
          return false;
        }
      } else {
        if (w2 == 2) {
          const uint8_t *b, *be;
          if (!v.bytes(&b, &be)) return false;
          Pb pk{b, be};
          while (pk.p < pk.end) {
            uint64_t x;
            if (!pk.varint(&x)) return false;
            if (s->count++ == 0) s->i = (int64_t)x;
          }
        } else if (w2 == 0) {
          uint64_t x;
          if (!v.varint(&x)) return false;
          if (s->count++ == 0) s->i = (int64_t)x;
        } else {
          return false;
        }
      }
    }
  }
  return f.ok;
}

// Example bytes -> the five slots.  Returns false on malformed protobuf.
bool parse_example(const uint8_t* p, const uint8_t* end, Slot* slots) {
  Pb ex{p, end};
  while (ex.p < ex.end) {
    uint64_t key;
    if (!ex.varint(&key)) return false;
    if (key != ((1u << 3) | 2)) {  // Example.features (field 1, LEN)
      if (!ex.skip((int)(key & 7))) return false;
      continue;
    }
    const uint8_t *q, *qe;
    if (!ex.bytes(&q, &qe)) return false;
    Pb fs{q, qe};
    while (fs.p < fs.end) {
      uint64_t k1;
      if (!fs.varint(&k1)) return false;
      if (k1 != ((1u << 3) | 2)) {  // Features.feature map entry
        if (!fs.skip((int)(k1 & 7))) return false;
        continue;
      }
      const uint8_t *e, *ee;
      if (!fs.bytes(&e, &ee)) return false;
      Pb en{e, ee};
      const uint8_t *name = nullptr, *name_e = nullptr, *val = nullptr, *val_e = nullptr;
      while (en.p < en.end) {
        uint64_t k2;
        if (!en.varint(&k2)) return false;
        const int num = (int)(k2 >> 3), wire = (int)(k2 & 7);
        if (wire == 2 && num == 1) {
          if (!en.bytes(&name, &name_e)) return false;
        } else if (wire == 2 && num == 2) {
          if (!en.bytes(&val, &val_e)) return false;
        } else if (!en.skip(wire)) {
          return false;
        }
      }
      if (!name) continue;
      const size_t nl = (size_t)(name_e - name);
      for (int k = 0; k < kKeys; ++k) {
        if (strlen(kKeyName[k]) == nl && memcmp(kKeyName[k], name, nl) == 0) {
          slots[k] = Slot();  // map entry: last one wins
          if (val && !parse_feature(val, val_e, &slots[k])) return false;
          break;
        }
      }
    }
  }
  return ex.ok;
}

}  // namespace

// status[i]: 0 = all five features present with exactly one value of the
// declared type; > 0 = bitmask of the offending keys in kKeyName order
// (1 encoded, 2 format, 4 label, 8 height, 16 width); -1 = not a valid
// serialized Example.  enc_off is relative to base.
JR_API int jr_example_parse_image(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                                  uint64_t* enc_off, uint64_t* enc_len, int64_t* label, int64_t* height,
                                  int64_t* width, int32_t* status) {
  if (n && (!base || !offsets || !lengths || !enc_off || !enc_len || !label || !height || !width || !status)) {
    jr::set_error("jr_example_parse_image: null argument");
    return JR_ERR_INVALID;
  }
  for (size_t r = 0; r < n; ++r) {
    Slot s[kKeys];
    const uint8_t* p = base + offsets[r];
    enc_off[r] = enc_len[r] = 0;
    label[r] = height[r] = width[r] = 0;
    if (!parse_example(p, p + lengths[r], s)) {
      status[r] = -1;
      continue;
    }
    int32_t bad = 0;
    for (int k = 0; k < kKeys; ++k)
      if (s[k].kind != kKeyKind[k] || s[k].count != 1) bad |= 1 << k;
    status[r] = bad;
    if (s[0].kind == 1 && s[0].count >= 1) {
      enc_off[r] = (uint64_t)(s[0].b - base);
      enc_len[r] = s[0].blen;
    }
    label[r] = s[2].i;
    height[r] = s[3].i;
    width[r] = s[4].i;
  }
  return JR_OK;
}
