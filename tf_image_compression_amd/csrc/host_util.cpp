// host_util.cpp — host-only helpers of libtic.so (no device code).
//
// tic_crc32c: CRC-32C (Castagnoli, reflected polynomial 0x82F63B78), the checksum of
// TensorFlow's table blocks and tensor-bundle entries, used by the checkpoint reader
// (tf_image_compression_amd/tf_checkpoint.py) that stands in for tf.train.Saver.restore
// (utils/utils.py:84-93).  Slice-by-8 tables, built once.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/tic.h"

namespace {

struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};

const Crc32cTables& tables() {
  static const Crc32cTables tb;
  return tb;
}

}  // namespace

extern "C" uint32_t tic_crc32c(const void* data, size_t n, uint32_t crc) {
  const Crc32cTables& tb = tables();
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = tb.t[7][lo & 0xff] ^ tb.t[6][(lo >> 8) & 0xff] ^ tb.t[5][(lo >> 16) & 0xff] ^ tb.t[4][lo >> 24] ^
        tb.t[3][hi & 0xff] ^ tb.t[2][(hi >> 8) & 0xff] ^ tb.t[1][(hi >> 16) & 0xff] ^ tb.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = tb.t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return ~c;
}
