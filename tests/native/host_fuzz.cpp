// host_fuzz.cpp — sanitizer harness for the host-only C++ of libtic.so (range_coder.cpp,
// host_util.cpp), built by `make asan` with -fsanitize=address,undefined and run by
// tests/test_host_asan.py on the CPU.  These are the two native pieces that parse input a
// user hands in (.encoded streams, checkpoint bytes through tic_crc32c).
//
// Cases: the reference's known-answer stream (other/test_range_coder.py:37-68); random
// tables and symbol strings round-tripped through several encode() calls; decoding of
// random, truncated, bit-flipped and empty files with random tables (must not fault and
// must return in-range symbols); the error contract (bad tables, symbols outside the
// table, use after close); CRC-32C against a bitwise reference on unaligned slices.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "tic.h"

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

static std::vector<int64_t> random_table(std::mt19937_64& g, int nsym, int64_t max_total) {
  std::vector<int64_t> cum(nsym + 1, 0);
  for (int i = 0; i < nsym; ++i) cum[i + 1] = cum[i] + (int64_t)(g() % 50) + (g() % 4 == 0 ? 0 : 1);
  if (cum[nsym] == 0) cum[nsym] = 1;
  if (cum[nsym] > max_total) {  // rescale, keeping monotone
    for (auto& v : cum) v = v * max_total / cum[nsym];
  }
  return cum;
}

static std::string tmp_path(const char* dir, const char* name, int i) {
  return std::string(dir) + "/" + name + std::to_string(i);
}

static void write_file(const std::string& p, const std::vector<uint8_t>& b) {
  FILE* f = fopen(p.c_str(), "wb");
  if (!b.empty()) fwrite(b.data(), 1, b.size(), f);
  fclose(f);
}

static std::vector<uint8_t> read_file(const std::string& p) {
  std::vector<uint8_t> b;
  FILE* f = fopen(p.c_str(), "rb");
  int c;
  while ((c = fgetc(f)) != EOF) b.push_back((uint8_t)c);
  fclose(f);
  return b;
}

static uint32_t crc_ref(const uint8_t* p, size_t n, uint32_t crc) {
  uint32_t c = ~crc;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
  }
  return ~c;
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  std::mt19937_64 g(20261016);

  {  // known-answer stream
    const std::string p = tmp_path(dir, "kat", 0);
    tic_rc_encoder* e = nullptr;
    CHECK(tic_rc_encoder_open(p.c_str(), &e) == TIC_OK);
    std::vector<int64_t> data;
    for (int r = 0; r < 17; ++r)
      for (int64_t s : {0, 0, 0, 0, 1, 2}) data.push_back(s);
    const int64_t cum[4] = {0, 4, 6, 8};
    CHECK(tic_rc_encode(e, data.data(), data.size(), cum, 4) == TIC_OK);
    CHECK(tic_rc_encoder_close(e) == TIC_OK);
    CHECK(tic_rc_encode(e, data.data(), 1, cum, 4) == TIC_ESTATE);  // after close
    const int64_t bad1[3] = {1, 2, 3}, bad2[4] = {0, 8, 8, 8}, bad3[2] = {-1, 1};
    CHECK(tic_rc_encode(e, data.data(), 1, bad1, 3) != TIC_OK);
    tic_rc_encoder_free(e);
    const auto b = read_file(p);
    CHECK(b.size() == 17);
    for (size_t i = 4; i < b.size(); ++i) CHECK(b[i] == 0x0b);
    tic_rc_decoder* d = nullptr;
    CHECK(tic_rc_decoder_open(p.c_str(), &d) == TIC_OK);
    std::vector<int64_t> out(data.size());
    CHECK(tic_rc_decode(d, out.size(), cum, 4, out.data()) == TIC_OK);
    CHECK(out == data);
    CHECK(tic_rc_encode(nullptr, data.data(), 1, bad2, 4) == TIC_EINVAL);
    CHECK(tic_rc_decode(d, 1, bad3, 2, out.data()) != TIC_OK);
    CHECK(tic_rc_decode(d, 1, cum, 1, out.data()) != TIC_OK);
    tic_rc_decoder_close(d);
    CHECK(tic_rc_decode(d, 1, cum, 4, out.data()) == TIC_ESTATE);
    tic_rc_decoder_free(d);
  }

  for (int it = 0; it < 200; ++it) {  // random round trips, several tables per stream
    const std::string p = tmp_path(dir, "rt", it);
    tic_rc_encoder* e = nullptr;
    CHECK(tic_rc_encoder_open(p.c_str(), &e) == TIC_OK);
    const int parts = 1 + (int)(g() % 3);
    std::vector<std::vector<int64_t>> tables, datas;
    for (int k = 0; k < parts; ++k) {
      auto cum = random_table(g, 1 + (int)(g() % 300), it % 2 ? (1 << 24) : 4096);
      std::vector<int64_t> valid;
      for (size_t s = 0; s + 1 < cum.size(); ++s)
        if (cum[s + 1] > cum[s]) valid.push_back((int64_t)s);
      std::vector<int64_t> data;
      if (!valid.empty())
        for (int n = (int)(g() % 3000); n > 0; --n) data.push_back(valid[g() % valid.size()]);
      int64_t bogus = (int64_t)cum.size() + 3;
      CHECK(tic_rc_encode(e, &bogus, 1, cum.data(), cum.size()) == TIC_EINVAL);  // outside the table
      CHECK(tic_rc_encode(e, data.data(), data.size(), cum.data(), cum.size()) == TIC_OK);
      tables.push_back(cum);
      datas.push_back(data);
    }
    CHECK(tic_rc_encoder_close(e) == TIC_OK);
    tic_rc_encoder_free(e);
    tic_rc_decoder* d = nullptr;
    CHECK(tic_rc_decoder_open(p.c_str(), &d) == TIC_OK);
    for (int k = 0; k < parts; ++k) {
      std::vector<int64_t> out(datas[k].size() + 1);
      CHECK(tic_rc_decode(d, datas[k].size(), tables[k].data(), tables[k].size(), out.data()) == TIC_OK);
      out.pop_back();
      CHECK(out == datas[k]);
    }
    tic_rc_decoder_free(d);
    remove(p.c_str());
  }

  for (int it = 0; it < 300; ++it) {  // hostile streams: random, truncated, flipped, empty
    const std::string p = tmp_path(dir, "bad", it);
    std::vector<uint8_t> b;
    const int mode = it % 4;
    if (mode == 0) {
      b.resize(g() % 200);
      for (auto& x : b) x = (uint8_t)g();
    } else if (mode == 1 || mode == 2) {
      tic_rc_encoder* e = nullptr;
      CHECK(tic_rc_encoder_open(p.c_str(), &e) == TIC_OK);
      auto cum = random_table(g, 2 + (int)(g() % 10), 4096);
      std::vector<int64_t> data;
      for (int n = 500; n > 0; --n) {
        const int64_t s = (int64_t)(g() % (cum.size() - 1));
        if (cum[s + 1] > cum[s]) data.push_back(s);
      }
      CHECK(tic_rc_encode(e, data.data(), data.size(), cum.data(), cum.size()) == TIC_OK);
      tic_rc_encoder_close(e);
      tic_rc_encoder_free(e);
      b = read_file(p);
      if (mode == 1) b.resize(b.size() / 2);
      else if (!b.empty()) b[g() % b.size()] ^= (uint8_t)(1u << (g() % 8));
    }  // mode 3: empty file
    write_file(p, b);
    tic_rc_decoder* d = nullptr;
    CHECK(tic_rc_decoder_open(p.c_str(), &d) == TIC_OK);
    auto cum = random_table(g, 1 + (int)(g() % 40), it % 3 ? 4096 : (1 << 24));
    std::vector<int64_t> out(2000, -1);
    CHECK(tic_rc_decode(d, out.size(), cum.data(), cum.size(), out.data()) == TIC_OK);
    for (int64_t s : out) CHECK(s >= 0 && s + 1 < (int64_t)cum.size());
    tic_rc_decoder_free(d);
    remove(p.c_str());
  }

  {  // open errors
    tic_rc_decoder* d = nullptr;
    CHECK(tic_rc_decoder_open((std::string(dir) + "/does/not/exist").c_str(), &d) == TIC_EIO);
    CHECK(tic_rc_decoder_open(nullptr, &d) == TIC_EINVAL);
  }

  {  // CRC-32C on unaligned slices of every length up to 300
    std::vector<uint8_t> buf(400);
    for (auto& x : buf) x = (uint8_t)g();
    for (size_t off = 0; off < 9; ++off)
      for (size_t n = 0; n <= 300; ++n)
        CHECK(tic_crc32c(buf.data() + off, n, 0) == crc_ref(buf.data() + off, n, 0));
    CHECK(tic_crc32c("123456789", 9, 0) == 0xE3069283u);  // CRC-32C check value
    const uint32_t a = tic_crc32c(buf.data(), 100, 0);
    CHECK(tic_crc32c(buf.data() + 100, 50, a) == tic_crc32c(buf.data(), 150, 0));
  }

  if (g_fail) {
    fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  printf("host_fuzz ok\n");
  return 0;
}
