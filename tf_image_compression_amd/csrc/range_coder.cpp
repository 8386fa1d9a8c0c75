// range_coder.cpp — static-model range coder behind the C-ABI (include/tic.h, tic_rc_*).
//
// Replaces the third-party `range_coder` extension the reference imports
// (encode.py:9,76-97; decode.py:9,79-101): RangeEncoder(path).encode(symbols, cum_freq),
// RangeDecoder(path).decode(n, cum_freq), with the same argument contract and error
// classes as its test-suite pins (other/test_range_coder.py:13-136).  The package itself
// is not vendored, so its byte format is not reproduced bit for bit.
//
// Coder: 32-bit range with exact arithmetic — `range` starts at 2^32 (held in 64 bits),
// so power-of-two totals subdivide it without rounding; `low` is kept in 64 bits and a
// carry is resolved with a cached byte + a count of pending 0xFF bytes.  A byte leaves
// the coder whenever range < 2^24.  close() flushes the FEWEST bytes k (0..4) whose
// zero-extension lies in [low, low + range), so a stream of b information bits costs
// ceil(b/8) bytes when the model is dyadic: the KAT input (cum_freq [0,4,6,8],
// [0,0,0,0,1,2] x 17 = 136 bits) encodes to exactly 17 bytes of 0x0b.
// The decoder reads zeros past the end of the file.  Several encode() calls (each with
// its own table) append to one stream and are decoded by matching decode() calls.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tic.h"

namespace {
thread_local std::string g_rc_err;
int rc_fail(int code, const std::string& m) {
  g_rc_err = m;
  return code;
}

constexpr uint64_t kTop = 1ull << 24;
constexpr uint64_t kFull = 1ull << 32;
constexpr int64_t kMaxTotal = 1ll << 24;  // range >= 2^24 after normalisation

// Validate a cumulative frequency table (the reference's ValueError / OverflowError
// contract: other/test_range_coder.py:13-34,70-88,122-128).
int check_table(const int64_t* cum, size_t ncum, int64_t* total) {
  if (!cum || ncum < 2) return rc_fail(TIC_EINVAL, "invalid frequency table (needs >= 2 entries)");
  for (size_t i = 0; i < ncum; ++i)
    if (cum[i] < 0 || cum[i] >= (int64_t)kFull)
      return rc_fail(TIC_EOVERFLOW, "cumulative frequencies must fit in an unsigned 32-bit integer");
  if (cum[0] != 0) return rc_fail(TIC_EINVAL, "cumulative frequency table must start at 0");
  for (size_t i = 1; i < ncum; ++i)
    if (cum[i] < cum[i - 1]) return rc_fail(TIC_EINVAL, "cumulative frequencies must be non-decreasing");
  if (cum[ncum - 1] <= 0) return rc_fail(TIC_EINVAL, "invalid frequency table (zero total)");
  if (cum[ncum - 1] > kMaxTotal) return rc_fail(TIC_EINVAL, "total frequency must be <= 2^24");
  *total = cum[ncum - 1];
  return TIC_OK;
}
}  // namespace

struct tic_rc_encoder {
  FILE* f = nullptr;
  uint64_t low = 0, range = kFull;
  int cache = -1;          // byte waiting for a possible carry (-1: none yet)
  uint64_t pending = 0;    // 0xFF bytes after the cache
  bool closed = false;

  bool put(int b) { return fputc(b, f) != EOF; }
  bool emit_top() {  // move the top byte of the 32-bit window (bits 24..31) out of low
    if (low < 0xFF000000ull || low >= kFull) {
      const int carry = low >= kFull ? 1 : 0;
      if (cache >= 0 && !put((cache + carry) & 0xFF)) return false;
      for (; pending; --pending)
        if (!put((0xFF + carry) & 0xFF)) return false;
      cache = (int)((low >> 24) & 0xFF);
    } else {
      ++pending;  // top byte is 0xFF and a carry may still arrive
    }
    low = (low << 8) & (kFull - 1);
    return true;
  }
};

struct tic_rc_decoder {
  FILE* f = nullptr;
  uint64_t code = 0, range = kFull;
  bool closed = false;
  int get() {
    const int c = fgetc(f);
    return c == EOF ? 0 : c;
  }
};

extern "C" {

const char* tic_rc_last_error(void) { return g_rc_err.c_str(); }

int tic_rc_encoder_open(const char* path, tic_rc_encoder** out) {
  if (!path || !out) return rc_fail(TIC_EINVAL, "null argument");
  FILE* f = fopen(path, "wb");
  if (!f) return rc_fail(TIC_EIO, std::string("cannot open ") + path + ": " + strerror(errno));
  *out = new tic_rc_encoder();
  (*out)->f = f;
  return TIC_OK;
}

int tic_rc_encode(tic_rc_encoder* e, const int64_t* data, size_t n, const int64_t* cum, size_t ncum) {
  if (!e) return rc_fail(TIC_EINVAL, "null encoder");
  if (e->closed) return rc_fail(TIC_ESTATE, "encoder is closed");
  int64_t total = 0;
  int rc = check_table(cum, ncum, &total);
  if (rc) return rc;
  const int64_t nsym = (int64_t)ncum - 1;
  for (size_t i = 0; i < n; ++i) {
    const int64_t s = data[i];
    if (s < 0 || s >= nsym) return rc_fail(TIC_EINVAL, "symbol " + std::to_string(s) + " outside the table (cumFreq too short)");
    const uint64_t start = (uint64_t)cum[s], freq = (uint64_t)(cum[s + 1] - cum[s]);
    if (freq == 0) return rc_fail(TIC_EINVAL, "symbols with zero probability cannot be encoded");
    const uint64_t r = e->range / (uint64_t)total;
    e->low += start * r;
    e->range = (cum[s + 1] == total) ? e->range - start * r : freq * r;
    while (e->range < kTop) {
      e->range <<= 8;
      if (!e->emit_top()) return rc_fail(TIC_EIO, "write failed");
    }
  }
  return TIC_OK;
}

int tic_rc_encoder_close(tic_rc_encoder* e) {
  if (!e) return rc_fail(TIC_EINVAL, "null encoder");
  if (e->closed) return TIC_OK;
  e->closed = true;
  // fewest top bytes k of a value v in [low, low + range) whose remaining bytes are zero
  int k = 0;
  uint64_t v = e->low;
  for (; k <= 4; ++k) {
    const int shift = 32 - 8 * k;
    const uint64_t unit = shift >= 64 ? 0 : (1ull << shift);
    v = k == 4 ? e->low : ((e->low + unit - 1) / unit) * unit;
    if (v < e->low + e->range) break;
  }
  bool ok = true;
  e->low = v;
  for (int i = 0; i < k && ok; ++i) ok = e->emit_top();
  if (ok && k > 0) {  // drain cache + pending (with the carry already folded in)
    if (e->cache >= 0) ok = e->put(e->cache);
    for (; ok && e->pending; --e->pending) ok = e->put(0xFF);
  } else if (ok && e->cache >= 0) {
    const int carry = v >= kFull ? 1 : 0;
    ok = e->put((e->cache + carry) & 0xFF);
    for (; ok && e->pending; --e->pending) ok = e->put((0xFF + carry) & 0xFF);
  }
  if (fclose(e->f) != 0) ok = false;
  e->f = nullptr;
  return ok ? TIC_OK : rc_fail(TIC_EIO, "write failed");
}

void tic_rc_encoder_free(tic_rc_encoder* e) {
  if (!e) return;
  if (e->f) fclose(e->f);
  delete e;
}

int tic_rc_decoder_open(const char* path, tic_rc_decoder** out) {
  if (!path || !out) return rc_fail(TIC_EINVAL, "null argument");
  FILE* f = fopen(path, "rb");
  if (!f) return rc_fail(TIC_EIO, std::string("cannot open ") + path + ": " + strerror(errno));
  tic_rc_decoder* d = new tic_rc_decoder();
  d->f = f;
  for (int i = 0; i < 4; ++i) d->code = (d->code << 8) | (uint64_t)d->get();
  *out = d;
  return TIC_OK;
}

int tic_rc_decode(tic_rc_decoder* d, size_t n, const int64_t* cum, size_t ncum, int64_t* out) {
  if (!d) return rc_fail(TIC_EINVAL, "null decoder");
  if (d->closed) return rc_fail(TIC_ESTATE, "decoder is closed");
  int64_t total = 0;
  int rc = check_table(cum, ncum, &total);
  if (rc) return rc;
  const int64_t nsym = (int64_t)ncum - 1;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t r = d->range / (uint64_t)total;
    uint64_t val = d->code / r;
    if (val >= (uint64_t)total) val = (uint64_t)total - 1;
    // last s with cum[s] <= val (and freq > 0)
    int64_t lo = 0, hi = nsym - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) / 2;
      if ((uint64_t)cum[mid] <= val) lo = mid;
      else hi = mid - 1;
    }
    const uint64_t start = (uint64_t)cum[lo];
    d->code -= start * r;
    d->range = (cum[lo + 1] == total) ? d->range - start * r : (uint64_t)(cum[lo + 1] - cum[lo]) * r;
    out[i] = lo;
    while (d->range < kTop) {
      d->range <<= 8;
      d->code = ((d->code << 8) | (uint64_t)d->get()) & (kFull - 1);
    }
  }
  return TIC_OK;
}

int tic_rc_decoder_close(tic_rc_decoder* d) {
  if (!d) return rc_fail(TIC_EINVAL, "null decoder");
  if (!d->closed && d->f) fclose(d->f);
  d->f = nullptr;
  d->closed = true;
  return TIC_OK;
}

void tic_rc_decoder_free(tic_rc_decoder* d) {
  if (!d) return;
  if (d->f) fclose(d->f);
  delete d;
}

}  // extern "C"
