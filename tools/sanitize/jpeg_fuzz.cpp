// AddressSanitizer + UBSan harness for the host half of the JPEG codec (spotter_amd/csrc/jpeg_host.h): the
// marker / Huffman parser that reads bytes fetched from arbitrary URLs (serve.py:74-77, 96). Built and run on
// the CPU by tests/test_jpeg_corpus.py over a corpus of corrupted files:
//
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
//       tools/sanitize/jpeg_fuzz.cpp -o <out>
//   <out> corpus.bin        (corpus.bin: a sequence of [uint32 little-endian length][bytes] records)
//
// Prints one line per record: "<index> <rc> <width> <height> <total_blocks>". A record whose layout asks
// for more than kMaxCoefs coefficients is not decoded (rc printed as "big"): the product path never gets
// there, Pillow's decompression-bomb check runs first (spotter_amd/jpeg.py).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../spotter_amd/csrc/jpeg_host.h"

namespace sp {
static char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace sp

static int decode(const uint8_t* data, int64_t len, sp_jpeg_layout* lay, int16_t* coefs) {
  sp::jpeg_host::Decoder d{data, len, lay, coefs};
  return d.run(coefs != nullptr);
}

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s corpus.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> all;
  uint8_t tmp[65536];
  size_t n;
  while ((n = fread(tmp, 1, sizeof(tmp), f)) > 0) all.insert(all.end(), tmp, tmp + n);
  fclose(f);
  constexpr int64_t kMaxCoefs = int64_t(1) << 26;
  size_t pos = 0;
  int idx = 0;
  while (pos + 4 <= all.size()) {
    const uint32_t len = all[pos] | (all[pos + 1] << 8) | (all[pos + 2] << 16) | ((uint32_t)all[pos + 3] << 24);
    pos += 4;
    if (pos + len > all.size()) return 3;
    // each record in its own exact-size heap block, so ASan sees any read past its end
    std::vector<uint8_t> rec(all.begin() + pos, all.begin() + pos + len);
    pos += len;
    sp_jpeg_layout lay;
    memset(&lay, 0, sizeof(lay));
    int rc = rec.empty() ? -1 : decode(rec.data(), (int64_t)rec.size(), &lay, nullptr);
    const bool big = rc == 0 && lay.total_blocks * 64 > kMaxCoefs;
    if (rc == 0 && !big) {
      std::vector<int16_t> coefs((size_t)lay.total_blocks * 64);
      rc = decode(rec.data(), (int64_t)rec.size(), &lay, coefs.data());
    }
    if (big)
      printf("%d big %d %d %lld\n", idx, lay.width, lay.height, (long long)lay.total_blocks);
    else
      printf("%d %d %d %d %lld\n", idx, rc, lay.width, lay.height, (long long)lay.total_blocks);
    ++idx;
  }
  return 0;
}
