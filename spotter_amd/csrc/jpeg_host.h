// Host side of the JPEG codec (serve.py:96-97 decode, serve.py:139-142 encode): the parts that are a serial bit
// stream or a few header bytes and therefore stay on the CPU. Plain C++ with no HIP dependency, so the same
// source is linked into libspotter_hip.so (through jpeg.hip) and into the AddressSanitizer / UBSan harness
// (tools/sanitize/jpeg_fuzz.cpp) that runs the corrupt-input corpus on the CPU.
//
// Policy on malformed input: the GPU path takes well-formed files only. Anything libjpeg would warn about or
// reject (a bad Huffman code, data past the end of a segment, extraneous bytes before a marker, a bogus
// progression, an impossible table) returns SP_JPEG_UNSUPPORTED, and the caller hands the bytes to Pillow,
// i.e. to the reference's own decoder and its own error or warning.
#pragma once

#include <climits>
#include <cstdint>
#include <cstring>

#include "../../include/spotter_hip.h"

// libjpeg(-turbo)'s JPEG_MAX_DIMENSION (jmorecfg.h): larger frames raise JERR_IMAGE_TOO_BIG on load and save
#define SP_JPEG_MAX_DIMENSION 65500

namespace sp {

void set_error(const char* fmt, ...);

namespace jpeg_host {

// jpeg_natural_order: zig-zag index → natural (row-major) index; 16 extra entries absorb the k overshoot
// of corrupt run lengths exactly as libjpeg's table does.
constexpr int kNatural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int kLook = 11;  // Huffman lookahead bits (code + magnitude bits of most AC symbols fit)

struct Huff {
  bool set = false;
  uint16_t look[1 << kLook];  // (code length << 8) | symbol; length 0: longer than kLook bits
  // AC tables: (run, size) symbols whose code and magnitude bits fit the lookahead together, fully decoded
  // — (value << 16) | (run << 8) | total bits; 0 = take the general path (stb-style fast AC)
  int32_t fast_ac[1 << kLook];
  int32_t maxcode[18];
  int32_t valoff[18];
  uint8_t vals[256];
};

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes from the 16 code-length counts. A DC table whose symbols
// exceed 15 is rejected as there (JERR_BAD_HUFF_TABLE): a DC symbol is a magnitude bit count.
inline bool build_huff(Huff& h, const uint8_t* bits, const uint8_t* vals, int nvals, bool is_dc) {
  int huffsize[257], huffcode[257];
  int p = 0;
  for (int l = 1; l <= 16; ++l)
    for (int i = 0; i < bits[l - 1]; ++i) {
      if (p >= 256) return false;
      huffsize[p++] = l;
    }
  huffsize[p] = 0;
  const int n = p;
  if (n != nvals || n == 0) return false;
  if (is_dc)
    for (int i = 0; i < n; ++i)
      if (vals[i] > 15) return false;
  int code = 0, si = huffsize[0];
  p = 0;
  while (huffsize[p]) {
    while (huffsize[p] == si) huffcode[p++] = code++;
    if (code >= (1 << si)) return false;  // bad table
    code <<= 1;
    ++si;
  }
  p = 0;
  for (int l = 1; l <= 16; ++l) {
    if (bits[l - 1]) {
      h.valoff[l] = p - huffcode[p];
      p += bits[l - 1];
      h.maxcode[l] = huffcode[p - 1];
    } else {
      h.maxcode[l] = -1;
    }
  }
  h.maxcode[17] = 0x7fffffff;
  for (int i = 0; i < n; ++i) h.vals[i] = vals[i];
  memset(h.look, 0, sizeof(h.look));
  memset(h.fast_ac, 0, sizeof(h.fast_ac));
  for (int i = 0; i < n; ++i) {
    const int l = huffsize[i];
    if (l > kLook) continue;
    const int lo = huffcode[i] << (kLook - l), cnt = 1 << (kLook - l);
    for (int j = 0; j < cnt; ++j) h.look[lo + j] = (uint16_t)((l << 8) | vals[i]);
    const int run = vals[i] >> 4, sz = vals[i] & 15;
    if (sz && l + sz <= kLook) {
      for (int j = 0; j < cnt; ++j) {
        const int mag = (j >> (kLook - l - sz)) & ((1 << sz) - 1);
        const int val = mag < (1 << (sz - 1)) ? mag - (1 << sz) + 1 : mag;
        h.fast_ac[lo + j] = (int32_t)((uint32_t)val << 16) | (run << 8) | (l + sz);
      }
    }
  }
  h.set = true;
  return true;
}

// Entropy-coded segment reader: 64-bit MSB-first buffer; 0xFF00 stuffing removed; at a marker it stops
// consuming and supplies zero bits (libjpeg's behaviour on truncated / corrupt data).
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int cnt = 0;
  bool at_marker = false;
  int fake = 0;  // zero bits appended past the data; fake > cnt: a decode used bits that do not exist
  bool corrupt = false;  // a condition libjpeg warns about (bad Huffman code, coefficient index past 63)

  __attribute__((noinline)) void fill_slow() {
    while (cnt <= 56) {
      uint64_t b = 0;
      bool real = false;
      if (!at_marker && p < end) {
        b = *p;
        if (b == 0xFF) {
          const int nb = p + 1 < end ? p[1] : 0xD9;
          if (nb == 0x00) {
            p += 2;
            real = true;
          } else {
            at_marker = true;
            b = 0;
          }
        } else {
          ++p;
          real = true;
        }
      }
      if (!real) fake += 8;
      buf |= b << (56 - cnt);
      cnt += 8;
    }
  }
  // fast path: the next whole bytes that fit hold no 0xFF (no stuffing, no marker): one 8-byte load
  __attribute__((always_inline)) void fill() {
    if (!at_marker && end - p >= 8) {
      uint64_t w;
      memcpy(&w, p, 8);
      w = __builtin_bswap64(w);
      const int nb = (64 - cnt) >> 3;  // whole bytes that fit (cnt <= 56 → >= 1)
      const uint64_t top = nb >= 8 ? ~0ull : ~(~0ull >> (8 * nb));
      const uint64_t x = ~w | ~top;  // a 0xFF byte in the top nb bytes becomes a zero byte
      if (!((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull)) {
        buf |= (w & top) >> cnt;
        cnt += 8 * nb;
        p += nb;
        return;
      }
    }
    fill_slow();
  }
  // n <= 16 on every call path (DC symbols <= 15 by build_huff, AC sizes and EOB runs are 4-bit fields)
  __attribute__((always_inline)) uint32_t get(int n) {
    if (n <= 0 || n > 16) return 0;
    if (cnt < n) fill();
    const uint32_t v = (uint32_t)(buf >> (64 - n));
    buf <<= n;
    cnt -= n;
    return v;
  }
  // restart: drop the buffered bits and consume the RSTn marker. A well-formed segment ends exactly at
  // RST(expect) (0xFF fill bytes allowed before it); skipped data or another marker number is what libjpeg
  // resynchronises with a warning (jdmarker.c read_restart_marker), so the file is flagged corrupt.
  void restart(int expect) {
    buf = 0;
    cnt = 0;
    fake = 0;
    at_marker = false;
    const uint8_t* q = p;
    while (q + 1 < end && q[0] == 0xFF && q[1] == 0xFF) ++q;
    if (!(q + 1 < end && q[0] == 0xFF && q[1] == 0xD0 + (expect & 7))) corrupt = true;
    while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < end) p += 2;
  }
};

__attribute__((always_inline)) inline int huff_decode(Bits& b, const Huff& h) {
  if (b.cnt < 16) b.fill();
  const uint16_t e = h.look[b.buf >> (64 - kLook)];
  if (e >> 8) {
    const int l = e >> 8;
    b.buf <<= l;
    b.cnt -= l;
    return e & 0xFF;
  }
  const uint32_t code = (uint32_t)(b.buf >> 48);
  int l = kLook + 1;
  while (l <= 16 && (int32_t)(code >> (16 - l)) > h.maxcode[l]) ++l;
  if (l > 16) {  // corrupt: libjpeg warns (JWRN_HUFF_BAD_CODE) and returns 0; the file is left to Pillow
    b.buf <<= 16;
    b.cnt -= 16;
    b.corrupt = true;
    return 0;
  }
  b.buf <<= l;
  b.cnt -= l;
  const int idx = (int)(code >> (16 - l)) + h.valoff[l];
  if (idx < 0 || idx >= 256) {
    b.corrupt = true;
    return 0;
  }
  return h.vals[idx];
}

inline int extend(uint32_t v, int s) {  // HUFF_EXTEND
  return s == 0 ? 0 : ((int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v);
}

enum { kBase, kDcFirst, kDcRefine, kAcFirst, kAcRefine };

// One block of one scan kind: jdhuff.c decode_mcu (baseline) and jdphuff.c decode_mcu_DC_first / DC_refine /
// AC_first / AC_refine (progressive), same control flow and bit consumption.
template <int KIND>
__attribute__((always_inline)) inline void decode_blk(Bits& b, int16_t* blk, const Huff& dct, const Huff& act,
                                                      int& pred, int& eobrun, int Ss, int Se, int Al) {
  if (KIND == kBase || KIND == kDcFirst) {
    const int s = huff_decode(b, dct);
    const int diff = extend(b.get(s), s);
    // jdhuff.c: a DC prediction that would overflow int is JERR_BAD_DCT_COEF
    if ((pred >= 0 && diff > INT_MAX - pred) || (pred < 0 && diff < INT_MIN - pred)) {
      b.corrupt = true;
      return;
    }
    pred += diff;
    blk[0] = (int16_t)(KIND == kBase ? pred : (int)((uint32_t)pred << Al));
    if (KIND == kDcFirst) return;
  }
  if (KIND == kDcRefine) {
    if (b.get(1)) blk[0] = (int16_t)(blk[0] | (1 << Al));
    return;
  }
  if (KIND == kBase || KIND == kAcFirst) {
    if (KIND == kAcFirst && eobrun > 0) {
      --eobrun;
      return;
    }
    const int k0 = KIND == kBase ? 1 : Ss, k1 = KIND == kBase ? 63 : Se;
    const int sh = KIND == kBase ? 0 : Al;
    for (int k = k0; k <= k1; ++k) {
      if (b.cnt < 16) b.fill();
      const int32_t f = act.fast_ac[b.buf >> (64 - kLook)];
      if (f) {  // code + magnitude bits in one lookup
        b.buf <<= (f & 31);
        b.cnt -= (f & 31);
        k += (f >> 8) & 15;
        if (k > 63) b.corrupt = true;
        blk[kNatural[k]] = (int16_t)((uint32_t)(f >> 16) << sh);
        continue;
      }
      const int rs = huff_decode(b, act);
      const int r = rs >> 4, sz = rs & 15;
      if (sz) {
        k += r;
        if (k > 63) b.corrupt = true;
        blk[kNatural[k]] = (int16_t)((uint32_t)extend(b.get(sz), sz) << sh);
      } else if (r == 15) {
        k += 15;
      } else {
        if (KIND == kAcFirst) {
          eobrun = 1 << r;
          if (r) eobrun += (int)b.get(r);
          --eobrun;
        }
        break;
      }
    }
    return;
  }
  // kAcRefine
  const int p1 = 1 << Al, m1 = -(1 << Al);
  int k = Ss;
  if (eobrun == 0) {
    for (; k <= Se; ++k) {
      const int rs = huff_decode(b, act);
      int r = rs >> 4;
      int s = rs & 15;
      if (s) {
        if (s != 1) b.corrupt = true;  // jdphuff.c: JWRN_HUFF_BAD_CODE
        s = b.get(1) ? p1 : m1;
      } else if (r != 15) {
        eobrun = 1 << r;
        if (r) eobrun += (int)b.get(r);
        break;
      }
      do {
        int16_t* tc = blk + kNatural[k];
        if (*tc != 0) {
          if (b.get(1) && (*tc & p1) == 0) *tc = (int16_t)(*tc >= 0 ? *tc + p1 : *tc + m1);
        } else if (--r < 0) {
          break;
        }
        ++k;
      } while (k <= Se);
      if (s) {
        if (k > Se) b.corrupt = true;
        blk[kNatural[k]] = (int16_t)s;
      }
    }
  }
  if (eobrun > 0) {
    for (; k <= Se; ++k) {
      int16_t* tc = blk + kNatural[k];
      if (*tc != 0 && b.get(1) && (*tc & p1) == 0) *tc = (int16_t)(*tc >= 0 ? *tc + p1 : *tc + m1);
    }
    --eobrun;
  }
}

struct Comp {
  int id = 0, h = 1, v = 1, tq = 0;
  int wb = 0, hb = 0;  // blocks holding image data (non-interleaved scan extent)
  bool latched = false;
};

struct Decoder {
  const uint8_t* data;
  int64_t len;
  sp_jpeg_layout* lay;
  int16_t* coefs;
  Comp comp[3];
  int nc = 0;
  uint16_t qt[4][64];
  bool qset[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  int restart_interval = 0;
  bool jfif = false;
  int adobe = -1;
  bool frame = false;
  int mcux = 0, mcuy = 0;
  bool dry_seen = false;  // some scan ran out of entropy-coded data (truncated / corrupt file)
  bool corrupt = false;   // a condition libjpeg warns about or resynchronises from (see the header comment)
  int coef_bits[3][64];   // jdphuff.c coef_bits: successive-approximation state per coefficient (-1 = none)
  int scans_seen[3] = {0, 0, 0};

  int fail(int code, const char* msg) {
    set_error("sp_jpeg_decode_coefs: %s", msg);
    return code;
  }
  // malformed input: the file is left to the host decoder (Pillow / libjpeg), whatever it then does
  int bad(const char* msg) { return fail(SP_JPEG_UNSUPPORTED, msg); }

  int16_t* block(int c, int by, int bx) {
    return coefs + (lay->block_off[c] + (int64_t)by * lay->bw[c] + bx) * 64;
  }

  struct ScanCtx {
    int ns, ci[3], td[3], ta[3], Ss, Se, Ah, Al;
  };

  // One scan's MCU walk with the block decoder of its kind inlined and the bit state in registers (a local
  // copy of the reader, written back at the end).
  template <int KIND>
  void scan_blocks(const ScanCtx& S, Bits& bref) {
    Bits b = bref;
    int pred[3] = {0, 0, 0};
    int eobrun = 0;
    int togo = restart_interval;
    int next_rst = 0;
    bool first = true;
    // jdhuff.c / jdphuff.c insufficient_data: once a block has used bits past the end of the segment's data
    // (decoded as zeros), the remaining MCUs of the segment are left zero, not decoded
    bool dry = false;
    auto mcu_start = [&]() {
      if (restart_interval) {
        if (!first && togo == 0) {  // jdhuff.c process_restart
          b.restart(next_rst++);
          pred[0] = pred[1] = pred[2] = 0;
          eobrun = 0;
          togo = restart_interval;
          dry = false;
        }
        --togo;
      }
      first = false;
      if (b.fake > b.cnt) dry = dry_seen = true;
      return !dry;
    };
    if (S.ns == 1) {  // non-interleaved: one block per MCU over the component's own block extent
      const int c = S.ci[0];
      const Huff& dct = dc[S.td[0]];
      const Huff& act = ac[S.ta[0]];
      for (int by = 0; by < comp[c].hb; ++by) {
        int16_t* blk = block(c, by, 0);
        for (int bx = 0; bx < comp[c].wb; ++bx, blk += 64)
          if (mcu_start()) decode_blk<KIND>(b, blk, dct, act, pred[c], eobrun, S.Ss, S.Se, S.Al);
      }
    } else {
      for (int my = 0; my < mcuy; ++my)
        for (int mx = 0; mx < mcux; ++mx) {
          if (!mcu_start()) continue;
          for (int si = 0; si < S.ns; ++si) {
            const int c = S.ci[si];
            const Huff& dct = dc[S.td[si]];
            const Huff& act = ac[S.ta[si]];
            for (int v = 0; v < comp[c].v; ++v)
              for (int h = 0; h < comp[c].h; ++h)
                decode_blk<KIND>(b, block(c, my * comp[c].v + v, mx * comp[c].h + h), dct, act, pred[c], eobrun,
                                 S.Ss, S.Se, S.Al);
          }
        }
    }
    if (b.fake > b.cnt) dry_seen = true;
    if (b.corrupt) corrupt = true;
    bref = b;
  }

  int parse_sof(const uint8_t* q, int L, int type) {
    if (frame) return bad("second frame header");
    if (type != 0xC0 && type != 0xC1 && type != 0xC2) return bad("lossless / arithmetic-coded / hierarchical JPEG");
    if (L < 6 || q[0] != 8) return bad("not 8-bit samples");
    const int H = (q[1] << 8) | q[2], W = (q[3] << 8) | q[4];
    nc = q[5];
    if (H <= 0 || W <= 0) return bad("zero image size (DNL) or bad header");
    // libjpeg's JPEG_MAX_DIMENSION (jmorecfg.h): jdinput.c initial_setup raises JERR_IMAGE_TOO_BIG above it
    if (H > SP_JPEG_MAX_DIMENSION || W > SP_JPEG_MAX_DIMENSION) return bad("image wider or higher than 65500");
    if (nc != 1 && nc != 3) return bad("component count other than 1 or 3");
    if (L != 6 + 3 * nc) return bad("SOF length does not match its component count");  // JERR_BAD_LENGTH
    int maxh = 1, maxv = 1;
    for (int i = 0; i < nc; ++i) {
      comp[i].id = q[6 + 3 * i];
      comp[i].h = q[7 + 3 * i] >> 4;
      comp[i].v = q[7 + 3 * i] & 15;
      comp[i].tq = q[8 + 3 * i];
      if (comp[i].h < 1 || comp[i].h > 4 || comp[i].v < 1 || comp[i].v > 4) return bad("bad sampling factor");
      if (comp[i].tq > 3) return bad("quantisation table id above 3");  // JERR_NO_QUANT_TABLE at latch time
      for (int k = 0; k < i; ++k)
        if (comp[k].id == comp[i].id) return bad("duplicate component id");
      maxh = comp[i].h > maxh ? comp[i].h : maxh;
      maxv = comp[i].v > maxv ? comp[i].v : maxv;
    }
    if (nc == 1) comp[0].h = comp[0].v = maxh = maxv = 1;  // a lone component is never subsampled (jdinput.c)
    // supported sampling: component 0 at the maxima, the others 1x or 2x below them
    if (comp[0].h != maxh || comp[0].v != maxv) return bad("luma below the maximum sampling");
    for (int i = 1; i < nc; ++i) {
      const int rh = maxh / comp[i].h, rv = maxv / comp[i].v;
      if (maxh % comp[i].h || maxv % comp[i].v || rh > 2 || rv > 2)
        return bad("chroma sampling ratio other than 1 or 2");
    }
    mcux = (W + 8 * maxh - 1) / (8 * maxh);
    mcuy = (H + 8 * maxv - 1) / (8 * maxv);
    memset(lay, 0, sizeof(*lay));
    lay->width = W;
    lay->height = H;
    lay->ncomp = nc;
    lay->progressive = type == 0xC2;
    lay->max_h = maxh;
    lay->max_v = maxv;
    int64_t off = 0, poff = 0;
    for (int i = 0; i < nc; ++i) {
      lay->h[i] = comp[i].h;
      lay->v[i] = comp[i].v;
      lay->bw[i] = mcux * comp[i].h;
      lay->bh[i] = mcuy * comp[i].v;
      lay->block_off[i] = off;
      off += (int64_t)lay->bw[i] * lay->bh[i];
      lay->plane_off[i] = poff;
      poff += (int64_t)lay->bw[i] * lay->bh[i] * 64;
      // jdinput.c: width_in_blocks = ceil(W * h / (maxh * 8))
      comp[i].wb = (int)(((int64_t)W * comp[i].h + 8 * maxh - 1) / (8 * maxh));
      comp[i].hb = (int)(((int64_t)H * comp[i].v + 8 * maxv - 1) / (8 * maxv));
      for (int k = 0; k < 64; ++k) coef_bits[i][k] = -1;
    }
    lay->total_blocks = off;
    lay->plane_bytes = poff;
    frame = true;
    return 0;
  }

  int parse_dqt(const uint8_t* q, int L) {
    int i = 0;
    while (i < L) {
      const int pq = q[i] >> 4, tq = q[i] & 15;
      if (tq > 3) return bad("bad DQT table id");
      if (pq > 1) return bad("bad DQT precision");
      ++i;
      const int need = pq ? 128 : 64;
      if (i + need > L) return bad("short DQT");
      for (int k = 0; k < 64; ++k) qt[tq][kNatural[k]] = pq ? (uint16_t)((q[i + 2 * k] << 8) | q[i + 2 * k + 1]) : q[i + k];
      qset[tq] = true;
      i += need;
    }
    return 0;
  }

  int parse_dht(const uint8_t* q, int L) {
    int i = 0;
    while (i < L) {
      if (i + 17 > L) return bad("short DHT");
      const int tc = q[i] >> 4, th = q[i] & 15;
      if (tc > 1 || th > 3) return bad("bad DHT table id");
      const uint8_t* bits = q + i + 1;
      int n = 0;
      for (int l = 0; l < 16; ++l) n += bits[l];
      if (n > 256 || i + 17 + n > L) return bad("bad DHT counts");
      if (!build_huff(tc ? ac[th] : dc[th], bits, q + i + 17, n, tc == 0)) return bad("bad Huffman table");
      i += 17 + n;
    }
    return 0;
  }

  // jdphuff.c start_pass_phuff_decoder: the scan must continue each coefficient's successive-approximation
  // sequence (JWRN_BOGUS_PROGRESSION otherwise; the file is then left to the host decoder)
  bool progression_ok(int ns, const int* ci, int Ss, int Se, int Ah, int Al) {
    for (int i = 0; i < ns; ++i) {
      int* cb = coef_bits[ci[i]];
      if (Ss != 0 && cb[0] < 0) return false;  // AC scan before the component's DC scan
      for (int k = Ss; k <= Se; ++k) {
        const int expected = cb[k] < 0 ? 0 : cb[k];
        if (Ah != expected) return false;
        cb[k] = Al;
      }
    }
    return true;
  }

  // One scan (SOS header at q, entropy-coded data from `after`); returns the position after its data.
  int scan(const uint8_t* q, int L, const uint8_t* after, const uint8_t** next) {
    if (!frame) return bad("SOS before SOF");
    if (L < 1) return bad("bad SOS");
    const int ns = q[0];
    if (ns < 1 || ns > nc || L != 1 + 2 * ns + 3) return bad("bad SOS");  // JERR_BAD_LENGTH
    int ci[3], td[3], ta[3];
    for (int i = 0; i < ns; ++i) {
      const int id = q[1 + 2 * i];
      int c = -1;
      for (int k = 0; k < nc; ++k)
        if (comp[k].id == id) c = k;
      if (c < 0) return bad("SOS names an unknown component");
      for (int k = 0; k < i; ++k)
        if (ci[k] == c) return bad("SOS names a component twice");
      ci[i] = c;
      td[i] = q[2 + 2 * i] >> 4;
      ta[i] = q[2 + 2 * i] & 15;
      if (td[i] > 3 || ta[i] > 3) return bad("bad table selector");
      if (!comp[c].latched) {  // jdinput.c latch_quant_tables: the table as of the component's first scan
        if (!qset[comp[c].tq]) return bad("quantisation table missing");
        memcpy(lay->quant[c], qt[comp[c].tq], sizeof(lay->quant[c]));
        comp[c].latched = true;
      }
    }
    const int Ss = q[1 + 2 * ns], Se = q[2 + 2 * ns], Ah = q[3 + 2 * ns] >> 4, Al = q[3 + 2 * ns] & 15;
    const bool prog = lay->progressive != 0;
    if (prog) {
      // jdphuff.c: JERR_BAD_PROGRESSION conditions, then the coefficient-bit bookkeeping
      if (Ss > Se || Se > 63 || Al > 13 || (Ss == 0 && Se != 0) || (Ss > 0 && ns != 1) || (Ah != 0 && Al != Ah - 1))
        return bad("bad progressive scan parameters");
      if (!progression_ok(ns, ci, Ss, Se, Ah, Al)) return bad("bogus progression");
    } else {
      if (Ss != 0 || Se != 63 || Ah != 0 || Al != 0) return bad("bad sequential scan parameters");
      for (int i = 0; i < ns; ++i)
        if (scans_seen[ci[i]]) return bad("sequential component scanned twice");
    }
    for (int i = 0; i < ns; ++i) {
      ++scans_seen[ci[i]];
      const bool need_dc = Ss == 0 && Ah == 0, need_ac = Se > 0;
      if ((need_dc && !dc[td[i]].set) || (need_ac && !ac[ta[i]].set)) return bad("Huffman table missing");
    }
    Bits b{after, data + len};
    ScanCtx S{ns, {ci[0], ci[1], ci[2]}, {td[0], td[1], td[2]}, {ta[0], ta[1], ta[2]}, Ss, Se, Ah, Al};
    if (!prog) scan_blocks<kBase>(S, b);
    else if (Ss == 0 && Ah == 0) scan_blocks<kDcFirst>(S, b);
    else if (Ss == 0) scan_blocks<kDcRefine>(S, b);
    else if (Ah == 0) scan_blocks<kAcFirst>(S, b);
    else scan_blocks<kAcRefine>(S, b);
    // resume marker parsing at the first marker (not an RSTn) at or after the reader's position; anything
    // but 0xFF fill bytes between the end of the data and that marker is extraneous data
    const uint8_t* r = b.p;
    while (r + 1 < data + len && !(r[0] == 0xFF && r[1] != 0x00 && r[1] != 0xFF && !(r[1] >= 0xD0 && r[1] <= 0xD7))) {
      if (r[0] != 0xFF) corrupt = true;
      ++r;
    }
    *next = r;
    return 0;
  }

  int run(bool decode) {
    if (len < 4 || data[0] != 0xFF || data[1] != 0xD8) return bad("not a JPEG (no SOI)");
    const uint8_t* p = data + 2;
    const uint8_t* end = data + len;
    bool zeroed = false;
    bool saw_eoi = false;
    while (p + 2 <= end) {
      if (p[0] != 0xFF) {  // garbage between markers: libjpeg warns and resyncs (JWRN_EXTRANEOUS_DATA)
        corrupt = true;
        ++p;
        continue;
      }
      const int m = p[1];
      if (m == 0xFF) {  // fill byte
        ++p;
        continue;
      }
      if (m == 0xD9) {  // EOI
        saw_eoi = true;
        break;
      }
      // markers a well-formed file does not hold here: TEM / reserved codes (Pillow: "no marker found"),
      // a second SOI, RSTn outside a scan, DNL, DHP, EXP, the JPGn extensions
      if (m < 0xC0 || m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0xDC || m == 0xDE || m == 0xDF ||
          m == 0xC8 || (m >= 0xF0 && m <= 0xFD))
        return bad("unexpected marker");
      if (p + 4 > end) break;
      const int L = (p[2] << 8) | p[3];
      if (L < 2 || p + 2 + L > end) return bad("truncated marker segment: left to the host decoder");
      const uint8_t* q = p + 4;
      const int n = L - 2;
      int rc = 0;
      if (m == 0xC4) {
        rc = parse_dht(q, n);
      } else if (m == 0xDB) {
        rc = parse_dqt(q, n);
      } else if (m == 0xDD) {
        if (n != 2) return bad("bad DRI length");
        restart_interval = (q[0] << 8) | q[1];
      } else if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xCC) {
        rc = parse_sof(q, n, m);
        if (rc == 0 && !decode) {  // headers up to SOF give the layout; the colour rules below need APPn too
          p += 2 + L;
          continue;
        }
      } else if (m == 0xCC) {
        return bad("arithmetic coding");
      } else if (m == 0xE0) {
        if (n >= 5 && memcmp(q, "JFIF\0", 5) == 0) jfif = true;
      } else if (m == 0xEE) {
        if (n >= 12 && memcmp(q, "Adobe", 5) == 0) adobe = q[11];
      } else if (m == 0xDA) {
        if (!decode) break;
        if (!zeroed) {
          if (!frame) return bad("SOS before SOF");
          memset(coefs, 0, (size_t)lay->total_blocks * 64 * sizeof(int16_t));
          zeroed = true;
        }
        const uint8_t* nx = nullptr;
        rc = scan(q, n, p + 2 + L, &nx);
        if (rc) return rc;
        p = nx;
        continue;
      }
      if (rc) return rc;
      p += 2 + L;
    }
    if (!frame) return bad("no frame header");
    // jdapimin.c default_decompress_parms: the colour space of a 3-component frame
    if (nc == 1) {
      lay->color = 0;
    } else if (jfif) {
      lay->color = 1;
    } else if (adobe >= 0) {
      lay->color = adobe == 0 ? 2 : 1;
    } else if (comp[0].id == 82 && comp[1].id == 71 && comp[2].id == 66) {
      lay->color = 2;
    } else {
      lay->color = 1;
    }
    if (adobe >= 2) return bad("Adobe YCCK / unknown transform");
    if (!decode) return 0;
    if (!zeroed) return bad("no scan");
    for (int c = 0; c < nc; ++c)
      if (!scans_seen[c] || (lay->progressive && coef_bits[c][0] < 0)) return bad("a component was never scanned");
    // Pillow raises on a truncated file ("image file is truncated") unless told otherwise, and libjpeg only
    // warns on corrupt data: either way those files keep the reference's own decoder, whose behaviour on them
    // is Pillow's policy, not libjpeg arithmetic
    if (dry_seen || !saw_eoi || corrupt)
      return bad("truncated or corrupt entropy-coded data: left to the host decoder");
    return 0;
  }
};


// ============================================================================================ encoder, host half
// jcparam.c: the Annex K example tables (natural order) and the Annex K.3 Huffman tables (std_huff_tables).
constexpr uint8_t kStdLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                  14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                  18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                  49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
constexpr uint8_t kStdChrQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                  24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                  99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                  99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
constexpr uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
constexpr uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
constexpr uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
constexpr uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
constexpr uint8_t kAcLumVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71, 0x14,
    0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09,
    0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a,
    0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65,
    0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88,
    0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9,
    0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
constexpr uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
constexpr uint8_t kAcChrVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22, 0x32,
    0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16,
    0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39,
    0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86,
    0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8,
    0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9,
    0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

// jchuff.c jpeg_make_c_derived_tbl: symbol → (code, length); constexpr so the device tables are built at compile
// time from the same arrays the DHT markers are written from.
struct EncHuff {
  uint16_t code[256];
  uint8_t size[256];
};
constexpr EncHuff derive_enc(const uint8_t (&bits)[16], const uint8_t* vals) {
  EncHuff h{};
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    for (int i = 0; i < bits[l - 1]; ++i, ++k, ++code) {
      h.code[vals[k]] = (uint16_t)code;
      h.size[vals[k]] = (uint8_t)l;
    }
    code <<= 1;
  }
  return h;
}

// worst case per block: DC code (<= 11 bits) + 11 magnitude bits, 63 AC codes (<= 16) + 10 magnitude bits, EOB
constexpr int64_t kMaxBitsPerBlock = 22 + 63 * 26 + 16;

inline int enc_plan(int32_t W, int32_t H, int32_t quality, int32_t subsampling, sp_jpeg_enc_layout* L) {
  // jcinit / jcmaster.c initial_setup: JERR_IMAGE_TOO_BIG above JPEG_MAX_DIMENSION; the caller falls back to Pillow
  if (W <= 0 || H <= 0 || W > SP_JPEG_MAX_DIMENSION || H > SP_JPEG_MAX_DIMENSION) return -1;
  if (quality != -1 && (quality < 1 || quality > 100)) return -1;
  int h0, v0;
  switch (subsampling) {  // Pillow's codes (JpegEncode.c): -1 keeps libjpeg's default 2x2
    case -1:
    case 2: h0 = 2; v0 = 2; break;
    case 1: h0 = 2; v0 = 1; break;
    case 0: h0 = 1; v0 = 1; break;
    default: return -1;
  }
  memset(L, 0, sizeof(*L));
  L->width = W;
  L->height = H;
  L->quality = quality == -1 ? 75 : quality;
  L->h0 = h0;
  L->v0 = v0;
  L->mcux = (W + 8 * h0 - 1) / (8 * h0);
  L->mcuy = (H + 8 * v0 - 1) / (8 * v0);
  L->bpm = h0 * v0 + 2;
  L->wb0 = (W + 7) / 8;
  L->hb0 = (H + 7) / 8;
  L->total_blocks = (int64_t)L->mcux * L->mcuy * L->bpm;
  // jcparam.c jpeg_quality_scaling + jpeg_add_quant_table(force_baseline = TRUE)
  const int q = L->quality;
  const int scale = q < 50 ? 5000 / q : 200 - q * 2;
  for (int t = 0; t < 2; ++t)
    for (int i = 0; i < 64; ++i) {
      long v = ((long)(t ? kStdChrQ : kStdLumQ)[i] * scale + 50L) / 100L;
      v = v <= 0 ? 1 : (v > 255 ? 255 : v);
      L->quant[t][i] = (uint16_t)v;
      // jcdctmgr.c compute_reciprocal(quantval << 3) with 16-bit DCTELEM (libjpeg-turbo's SIMD build)
      const uint32_t d = (uint32_t)v << 3;
      uint32_t b = 0;
      while ((d >> (b + 1)) != 0) ++b;  // flss(d) - 1
      uint32_t r = 16 + b;
      uint32_t fq = (1u << r) / d, fr = (1u << r) % d, c = d / 2;
      if (fr == 0) {
        fq >>= 1;
        --r;
      } else if (fr <= d / 2) {
        ++c;
      } else {
        ++fq;
      }
      L->recip[t][i] = (uint16_t)fq;
      L->corr[t][i] = (uint16_t)c;
      L->shift[t][i] = (int16_t)(r - 16);
    }
  const int64_t nmcu = (int64_t)L->mcux * L->mcuy;
  // device workspace: [total bits int64][per-MCU offsets int64][per-MCU bits int32][coefficients int16, 256-B aligned]
  const int64_t coef_off = ((8 + 8 * nmcu + 4 * nmcu) + 255) / 256 * 256;
  L->work_bytes = coef_off + L->total_blocks * 64 * 2;
  L->bits_cap = (L->total_blocks * kMaxBitsPerBlock + 7) / 8 + 16;
  return 0;
}
inline int64_t enc_coef_offset(const sp_jpeg_enc_layout& L) {
  const int64_t nmcu = (int64_t)L.mcux * L.mcuy;
  return ((8 + 8 * nmcu + 4 * nmcu) + 255) / 256 * 256;
}

inline int64_t enc_max_bytes(const sp_jpeg_enc_layout& L, int64_t nbits, int64_t clen) {
  return 20 + (clen > 0 ? clen + 4 : 0) + 2 * 69 + 19 + 4 * (5 + 16) + 2 * 12 + 2 * 162 + 14 + 2 * ((nbits + 7) / 8) + 2;
}

// jcmarker.c write_file_header / write_frame_header / write_scan_header for the configuration above, Pillow's
// COM (jpeg_write_marker after jpeg_start_compress) between them; then jchuff.c's emit_byte stuffing and
// flush_bits padding on the segment, and EOI.
inline int enc_finish(const sp_jpeg_enc_layout& L, const uint8_t* bits, int64_t nbits, const uint8_t* comment,
                      int64_t clen, uint8_t* out, int64_t cap, int64_t* out_len) {
  if (nbits < 0 || clen < 0 || clen > 65533 || cap < enc_max_bytes(L, nbits, clen)) return -1;
  uint8_t* o = out;
  auto b1 = [&](int v) { *o++ = (uint8_t)v; };
  auto b2 = [&](int v) {
    *o++ = (uint8_t)(v >> 8);
    *o++ = (uint8_t)v;
  };
  b1(0xFF), b1(0xD8);
  static const uint8_t jfif[18] = {0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
  memcpy(o, jfif, 18);
  o += 18;
  if (clen > 0) {
    b1(0xFF), b1(0xFE), b2((int)clen + 2);
    memcpy(o, comment, (size_t)clen);
    o += clen;
  }
  for (int t = 0; t < 2; ++t) {
    b1(0xFF), b1(0xDB), b2(67), b1(t);
    for (int k = 0; k < 64; ++k) b1(L.quant[t][kNatural[k]]);
  }
  b1(0xFF), b1(0xC0), b2(17), b1(8), b2(L.height), b2(L.width), b1(3);
  b1(1), b1((L.h0 << 4) | L.v0), b1(0);
  b1(2), b1(0x11), b1(1);
  b1(3), b1(0x11), b1(1);
  struct T {
    int idx;
    const uint8_t* bits;
    const uint8_t* vals;
  } tabs[4] = {{0x00, kDcLumBits, kDcVals}, {0x10, kAcLumBits, kAcLumVals}, {0x01, kDcChrBits, kDcVals},
               {0x11, kAcChrBits, kAcChrVals}};
  for (const T& t : tabs) {
    int n = 0;
    for (int l = 0; l < 16; ++l) n += t.bits[l];
    b1(0xFF), b1(0xC4), b2(n + 19), b1(t.idx);
    memcpy(o, t.bits, 16);
    o += 16;
    memcpy(o, t.vals, (size_t)n);
    o += n;
  }
  static const uint8_t sos[14] = {0xFF, 0xDA, 0x00, 0x0C, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0x00, 0x3F, 0x00};
  memcpy(o, sos, 14);
  o += 14;
  // the segment: whole bytes, then the last partial byte padded with 1s; every 0xFF byte followed by 0x00
  const int64_t whole = nbits >> 3;
  const int rest = (int)(nbits & 7);
  const uint8_t* p = bits;
  const uint8_t* end = bits + whole;
  while (p < end) {
    const uint8_t* ff = static_cast<const uint8_t*>(memchr(p, 0xFF, (size_t)(end - p)));
    const uint8_t* stop = ff ? ff + 1 : end;
    memcpy(o, p, (size_t)(stop - p));
    o += stop - p;
    if (ff) *o++ = 0x00;
    p = stop;
  }
  if (rest) {
    const uint8_t last = (uint8_t)((bits[whole] & (0xFF00 >> rest)) | (0xFF >> rest));
    *o++ = last;
    if (last == 0xFF) *o++ = 0x00;
  }
  b1(0xFF), b1(0xD9);
  *out_len = o - out;
  return 0;
}

}  // namespace jpeg_host
}  // namespace sp
