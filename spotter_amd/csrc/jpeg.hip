// JPEG decode in front of A1 (serve.py:96-97: Image.open(BytesIO(..)).convert("RGB"), which Pillow runs
// through libjpeg-turbo). The entropy decode is a serial bit stream and stays on the host (C++ below); the
// per-pixel work runs on the GPU: dequantisation + the ISLOW integer IDCT per 8x8 block (jidctint.c), then
// "fancy" triangle upsampling of the chroma planes (jdsample.c h2v1 / h2v2 / h1v2_fancy_upsample) with the
// edge-row replication of the main controller's context rows (jdmainct.c), then the integer YCbCr→RGB
// tables (jdcolor.c) — the same integer arithmetic, so the pixels are Pillow's, bit for bit.
// libjpeg-turbo is a dependency of Pillow (absent from /root/reference); its published algorithms are
// restated here and in oracle/jpeg_np.py, and tests/test_jpeg.py pins both against Pillow's own decode.
#include <cstdint>
#include <vector>

#include "common.h"

namespace sp {
namespace {

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

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes from the 16 code-length counts.
bool build_huff(Huff& h, const uint8_t* bits, const uint8_t* vals, int nvals) {
  int huffsize[257], huffcode[257];
  int p = 0;
  for (int l = 1; l <= 16; ++l)
    for (int i = 0; i < bits[l - 1]; ++i) {
      if (p >= 256) return false;
      huffsize[p++] = l;
    }
  huffsize[p] = 0;
  const int n = p;
  if (n != nvals) return false;
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
  __attribute__((always_inline)) uint32_t get(int n) {
    if (n == 0) return 0;
    if (cnt < n) fill();
    const uint32_t v = (uint32_t)(buf >> (64 - n));
    buf <<= n;
    cnt -= n;
    return v;
  }
  // restart: drop the buffered bits, consume the RSTn marker (scanning forward to it if data is missing)
  void restart() {
    buf = 0;
    cnt = 0;
    fake = 0;
    at_marker = false;
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
  if (l > 16) {  // corrupt: libjpeg warns and returns 0
    b.buf <<= 16;
    b.cnt -= 16;
    return 0;
  }
  b.buf <<= l;
  b.cnt -= l;
  const int idx = (int)(code >> (16 - l)) + h.valoff[l];
  return (idx >= 0 && idx < 256) ? h.vals[idx] : 0;
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
    pred += extend(b.get(s), s);
    blk[0] = (int16_t)(KIND == kBase ? pred : pred * (1 << Al));
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
        blk[kNatural[k]] = (int16_t)((f >> 16) * (1 << sh));
        continue;
      }
      const int rs = huff_decode(b, act);
      const int r = rs >> 4, sz = rs & 15;
      if (sz) {
        k += r;
        blk[kNatural[k]] = (int16_t)(extend(b.get(sz), sz) * (1 << sh));
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
      if (s) blk[kNatural[k]] = (int16_t)s;
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

  int fail(int code, const char* msg) {
    set_error("sp_jpeg_decode_coefs: %s", msg);
    return code;
  }

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
    bool first = true;
    // jdhuff.c / jdphuff.c insufficient_data: once a block has used bits past the end of the segment's data
    // (decoded as zeros), the remaining MCUs of the segment are left zero, not decoded
    bool dry = false;
    auto mcu_start = [&]() {
      if (restart_interval) {
        if (!first && togo == 0) {  // jdhuff.c process_restart
          b.restart();
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
    bref = b;
  }

  int parse_sof(const uint8_t* q, int L, int type) {
    if (frame) return fail(-1, "second frame header");
    if (type != 0xC0 && type != 0xC1 && type != 0xC2)
      return fail(SP_JPEG_UNSUPPORTED, "lossless / arithmetic-coded / hierarchical JPEG");
    if (L < 6 || q[0] != 8) return fail(SP_JPEG_UNSUPPORTED, "not 8-bit samples");
    const int H = (q[1] << 8) | q[2], W = (q[3] << 8) | q[4];
    nc = q[5];
    if (H <= 0 || W <= 0) return fail(SP_JPEG_UNSUPPORTED, "zero image size (DNL) or bad header");
    if (nc != 1 && nc != 3) return fail(SP_JPEG_UNSUPPORTED, "component count other than 1 or 3");
    if (L < 6 + 3 * nc) return fail(-1, "short SOF");
    int maxh = 1, maxv = 1;
    for (int i = 0; i < nc; ++i) {
      comp[i].id = q[6 + 3 * i];
      comp[i].h = q[7 + 3 * i] >> 4;
      comp[i].v = q[7 + 3 * i] & 15;
      comp[i].tq = q[8 + 3 * i] & 3;
      if (comp[i].h < 1 || comp[i].h > 4 || comp[i].v < 1 || comp[i].v > 4) return fail(-1, "bad sampling factor");
      maxh = comp[i].h > maxh ? comp[i].h : maxh;
      maxv = comp[i].v > maxv ? comp[i].v : maxv;
    }
    if (nc == 1) comp[0].h = comp[0].v = maxh = maxv = 1;  // a lone component is never subsampled (jdinput.c)
    // supported sampling: component 0 at the maxima, the others 1x or 2x below them
    if (comp[0].h != maxh || comp[0].v != maxv) return fail(SP_JPEG_UNSUPPORTED, "luma below the maximum sampling");
    for (int i = 1; i < nc; ++i) {
      const int rh = maxh / comp[i].h, rv = maxv / comp[i].v;
      if (maxh % comp[i].h || maxv % comp[i].v || rh > 2 || rv > 2)
        return fail(SP_JPEG_UNSUPPORTED, "chroma sampling ratio other than 1 or 2");
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
      if (tq > 3) return fail(-1, "bad DQT table id");
      ++i;
      const int need = pq ? 128 : 64;
      if (i + need > L) return fail(-1, "short DQT");
      for (int k = 0; k < 64; ++k) qt[tq][kNatural[k]] = pq ? (uint16_t)((q[i + 2 * k] << 8) | q[i + 2 * k + 1]) : q[i + k];
      qset[tq] = true;
      i += need;
    }
    return 0;
  }

  int parse_dht(const uint8_t* q, int L) {
    int i = 0;
    while (i < L) {
      if (i + 17 > L) return fail(-1, "short DHT");
      const int tc = q[i] >> 4, th = q[i] & 15;
      if (tc > 1 || th > 3) return fail(-1, "bad DHT table id");
      const uint8_t* bits = q + i + 1;
      int n = 0;
      for (int l = 0; l < 16; ++l) n += bits[l];
      if (n > 256 || i + 17 + n > L) return fail(-1, "bad DHT counts");
      if (!build_huff(tc ? ac[th] : dc[th], bits, q + i + 17, n)) return fail(-1, "bad Huffman table");
      i += 17 + n;
    }
    return 0;
  }

  // One scan (SOS header at q, entropy-coded data from `after`); returns the position after its data.
  int scan(const uint8_t* q, int L, const uint8_t* after, const uint8_t** next) {
    if (!frame) return fail(-1, "SOS before SOF");
    const int ns = q[0];
    if (ns < 1 || ns > nc || L < 1 + 2 * ns + 3) return fail(-1, "bad SOS");
    int ci[3], td[3], ta[3];
    for (int i = 0; i < ns; ++i) {
      const int id = q[1 + 2 * i];
      int c = -1;
      for (int k = 0; k < nc; ++k)
        if (comp[k].id == id) c = k;
      if (c < 0) return fail(-1, "SOS names an unknown component");
      ci[i] = c;
      td[i] = q[2 + 2 * i] >> 4;
      ta[i] = q[2 + 2 * i] & 15;
      if (td[i] > 3 || ta[i] > 3) return fail(-1, "bad table selector");
      if (!comp[c].latched) {  // jdinput.c latch_quant_tables: the table as of the component's first scan
        if (!qset[comp[c].tq]) return fail(-1, "quantisation table missing");
        memcpy(lay->quant[c], qt[comp[c].tq], sizeof(lay->quant[c]));
        comp[c].latched = true;
      }
    }
    const int Ss = q[1 + 2 * ns], Se = q[2 + 2 * ns], Ah = q[3 + 2 * ns] >> 4, Al = q[3 + 2 * ns] & 15;
    const bool prog = lay->progressive != 0;
    if (prog) {
      if (Ss > Se || Se > 63 || Al > 13 || (Ss == 0 && Se != 0) || (Ss > 0 && ns != 1))
        return fail(-1, "bad progressive scan parameters");
    } else if (Ss != 0 || Se != 63 || Ah != 0 || Al != 0) {
      return fail(-1, "bad sequential scan parameters");
    }
    for (int i = 0; i < ns; ++i) {
      const bool need_dc = Ss == 0 && Ah == 0, need_ac = Se > 0;
      if ((need_dc && !dc[td[i]].set) || (need_ac && !ac[ta[i]].set)) return fail(-1, "Huffman table missing");
    }
    Bits b{after, data + len};
    ScanCtx S{ns, {ci[0], ci[1], ci[2]}, {td[0], td[1], td[2]}, {ta[0], ta[1], ta[2]}, Ss, Se, Ah, Al};
    if (!prog) scan_blocks<kBase>(S, b);
    else if (Ss == 0 && Ah == 0) scan_blocks<kDcFirst>(S, b);
    else if (Ss == 0) scan_blocks<kDcRefine>(S, b);
    else if (Ah == 0) scan_blocks<kAcFirst>(S, b);
    else scan_blocks<kAcRefine>(S, b);
    // resume marker parsing at the first marker (not an RSTn) at or after the reader's position
    const uint8_t* r = b.p;
    while (r + 1 < data + len && !(r[0] == 0xFF && r[1] != 0x00 && r[1] != 0xFF && !(r[1] >= 0xD0 && r[1] <= 0xD7)))
      ++r;
    *next = r;
    return 0;
  }

  int run(bool decode) {
    if (len < 4 || data[0] != 0xFF || data[1] != 0xD8) return fail(SP_JPEG_UNSUPPORTED, "not a JPEG (no SOI)");
    const uint8_t* p = data + 2;
    const uint8_t* end = data + len;
    bool zeroed = false;
    bool saw_eoi = false;
    while (p + 2 <= end) {
      if (p[0] != 0xFF) {  // garbage between markers: skip to the next 0xFF (libjpeg warns and resyncs)
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
      if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {
        p += 2;
        continue;
      }
      if (p + 4 > end) break;
      const int L = (p[2] << 8) | p[3];
      if (L < 2 || p + 2 + L > end)
        return fail(SP_JPEG_UNSUPPORTED, "truncated marker segment: left to the host decoder");
      const uint8_t* q = p + 4;
      const int n = L - 2;
      int rc = 0;
      if (m == 0xC4) {
        rc = parse_dht(q, n);
      } else if (m == 0xDB) {
        rc = parse_dqt(q, n);
      } else if (m == 0xDD) {
        if (n < 2) return fail(-1, "short DRI");
        restart_interval = (q[0] << 8) | q[1];
      } else if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
        rc = parse_sof(q, n, m);
        if (rc == 0 && !decode) {  // headers up to SOF give the layout; the colour rules below need APPn too
          p += 2 + L;
          continue;
        }
      } else if (m == 0xCC) {
        return fail(SP_JPEG_UNSUPPORTED, "arithmetic coding");
      } else if (m == 0xE0) {
        if (n >= 5 && memcmp(q, "JFIF\0", 5) == 0) jfif = true;
      } else if (m == 0xEE) {
        if (n >= 12 && memcmp(q, "Adobe", 5) == 0) adobe = q[11];
      } else if (m == 0xDA) {
        if (!decode) break;
        if (!zeroed) {
          if (!frame) return fail(-1, "SOS before SOF");
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
    if (!frame) return fail(SP_JPEG_UNSUPPORTED, "no frame header");
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
    if (adobe >= 2) return fail(SP_JPEG_UNSUPPORTED, "Adobe YCCK / unknown transform");
    if (decode && !zeroed) return fail(SP_JPEG_UNSUPPORTED, "no scan");
    // Pillow raises on a truncated file ("image file is truncated") unless told otherwise, and libjpeg only
    // warns on corrupt data: either way those files keep the reference's own decoder, whose behaviour on them
    // is Pillow's policy, not libjpeg arithmetic
    if (decode && (dry_seen || !saw_eoi))
      return fail(SP_JPEG_UNSUPPORTED, "truncated or corrupt entropy-coded data: left to the host decoder");
    return 0;
  }
};

// ------------------------------------------------------------------------------------------------ device
// jidctint.c jpeg_idct_islow constants (CONST_BITS 13, PASS1_BITS 2)
constexpr int kCB = 13, kP1 = 2;
constexpr int F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
              F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;

// The 1-D ISLOW butterfly on 8 values in (pass 1: dequantised coefficients; pass 2: the workspace row),
// out[i] = (value + rounding) >> shift, exactly the jidctint.c sequence of products and sums.
__device__ __forceinline__ void islow_1d(const int64_t (&in)[8], int shift, int64_t (&out)[8]) {
  int64_t z2 = in[2], z3 = in[6];
  int64_t z1 = (z2 + z3) * F0_541;
  const int64_t tmp2 = z1 + z3 * -F1_847;
  const int64_t tmp3 = z1 + z2 * F0_765;
  z2 = in[0];
  z3 = in[4];
  const int64_t t0 = (z2 + z3) * (1 << kCB);
  const int64_t t1 = (z2 - z3) * (1 << kCB);
  const int64_t tmp10 = t0 + tmp3, tmp13 = t0 - tmp3, tmp11 = t1 + tmp2, tmp12 = t1 - tmp2;
  int64_t o0 = in[7], o1 = in[5], o2 = in[3], o3 = in[1];
  z1 = o0 + o3;
  z2 = o1 + o2;
  z3 = o0 + o2;
  int64_t z4 = o1 + o3;
  const int64_t z5 = (z3 + z4) * F1_175;
  o0 *= F0_298;
  o1 *= F2_053;
  o2 *= F3_072;
  o3 *= F1_501;
  z1 *= -F0_899;
  z2 *= -F2_562;
  z3 *= -F1_961;
  z4 *= -F0_390;
  z3 += z5;
  z4 += z5;
  o0 += z1 + z3;
  o1 += z2 + z4;
  o2 += z2 + z3;
  o3 += z1 + z4;
  const int64_t rnd = (int64_t)1 << (shift - 1);
  out[0] = (tmp10 + o3 + rnd) >> shift;
  out[7] = (tmp10 - o3 + rnd) >> shift;
  out[1] = (tmp11 + o2 + rnd) >> shift;
  out[6] = (tmp11 - o2 + rnd) >> shift;
  out[2] = (tmp12 + o1 + rnd) >> shift;
  out[5] = (tmp12 - o1 + rnd) >> shift;
  out[3] = (tmp13 + o0 + rnd) >> shift;
  out[4] = (tmp13 - o0 + rnd) >> shift;
}

// IDCT_range_limit: the & RANGE_MASK (1023) wrap, then clamp of value + 128 to [0, 255] (jdmaster.c
// prepare_range_limit_table)
__device__ __forceinline__ uint8_t idct_limit(int64_t x) {
  int v = (int)(x & 1023);
  v = v >= 512 ? v - 1024 : v;
  v += 128;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// 8 threads per 8x8 block (thread = column in pass 1, row in pass 2), 32 blocks per workgroup.
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coefs, const sp_jpeg_layout L,
                                                        uint8_t* __restrict__ work) {
  __shared__ int32_t ws[32][8][9];
  const int lb = threadIdx.x >> 3, t = threadIdx.x & 7;
  const int64_t blk = (int64_t)blockIdx.x * 32 + lb;
  const bool live = blk < L.total_blocks;
  int c = 0;
  if (L.ncomp > 1 && blk >= L.block_off[1]) c = 1;
  if (L.ncomp > 2 && blk >= L.block_off[2]) c = 2;
  if (live) {
    const int16_t* in = coefs + blk * 64;
    int64_t col[8], out[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) col[r] = (int64_t)in[r * 8 + t] * L.quant[c][r * 8 + t];
    islow_1d(col, kCB - kP1, out);
#pragma unroll
    for (int r = 0; r < 8; ++r) ws[lb][r][t] = (int32_t)out[r];
  }
  __syncthreads();
  if (!live) return;
  int64_t row[8], out[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) row[i] = ws[lb][t][i];
  islow_1d(row, kCB + kP1 + 3, out);
  const int64_t local = blk - L.block_off[c];
  const int by = (int)(local / L.bw[c]), bx = (int)(local - (int64_t)by * L.bw[c]);
  const int64_t stride = (int64_t)L.bw[c] * 8;
  uint8_t* dst = work + L.plane_off[c] + ((int64_t)by * 8 + t) * stride + (int64_t)bx * 8;
  uint32_t w0 = 0, w1 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w0 |= (uint32_t)idct_limit(out[i]) << (8 * i);
    w1 |= (uint32_t)idct_limit(out[i + 4]) << (8 * i);
  }
  *reinterpret_cast<uint2*>(dst) = make_uint2(w0, w1);
}

// One chroma sample at output (x, y): jdsample.c fancy upsampling (triangle filter 3/4 nearer + 1/4 further
// in each upsampled direction), rows past the component's edge replicating its first / last row as the
// main controller's context rows do; box replication where libjpeg-turbo picks it (downsampled width <= 2
// for the horizontal-doubling forms).
__device__ __forceinline__ int chroma_at(const uint8_t* pl, int64_t stride, int rh, int rv, int dw, int dh, int x,
                                         int y) {
  if (rh == 1 && rv == 1) return pl[(int64_t)y * stride + x];
  const int xc = rh == 2 ? x >> 1 : x, yc = rv == 2 ? y >> 1 : y;
  if (rh == 2 && dw <= 2) return pl[(int64_t)yc * stride + xc];  // h2v1_upsample / h2v2_upsample
  if (rh == 2 && rv == 1) {  // h2v1_fancy_upsample
    const uint8_t* r = pl + (int64_t)yc * stride;
    const int in = r[xc];
    if ((x & 1) == 0) return xc == 0 ? in : (in * 3 + r[xc - 1] + 1) >> 2;
    return xc == dw - 1 ? in : (in * 3 + r[xc + 1] + 2) >> 2;
  }
  // vertical doubling: the nearer row yc and the further row above (even y) or below (odd y)
  const int yn = (y & 1) ? (yc + 1 < dh ? yc + 1 : dh - 1) : (yc > 0 ? yc - 1 : 0);
  const uint8_t* r0 = pl + (int64_t)yc * stride;
  const uint8_t* r1 = pl + (int64_t)yn * stride;
  if (rh == 1) return (r0[x] * 3 + r1[x] + ((y & 1) ? 2 : 1)) >> 2;  // h1v2_fancy_upsample
  // h2v2_fancy_upsample: column sums 3·nearer row + further row, then 3/4 · 1/4 across columns
  const int cs = r0[xc] * 3 + r1[xc];
  if ((x & 1) == 0) {
    if (xc == 0) return (cs * 4 + 8) >> 4;
    return (cs * 3 + r0[xc - 1] * 3 + r1[xc - 1] + 8) >> 4;
  }
  if (xc == dw - 1) return (cs * 4 + 7) >> 4;
  return (cs * 3 + r0[xc + 1] * 3 + r1[xc + 1] + 7) >> 4;
}

__device__ __forceinline__ uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// One thread per output pixel: luma from its plane, chroma upsampled, jdcolor.c ycc_rgb_convert (SCALEBITS 16
// fixed point: Cr→R 1.40200, Cb→B 1.77200, G = y + ((−0.34414·Cb + ½ − 0.71414·Cr) >> 16)).
__global__ __launch_bounds__(256) void jpeg_color_kernel(const sp_jpeg_layout L, const uint8_t* __restrict__ work,
                                                         uint8_t* __restrict__ rgb, int64_t rgb_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)L.width * L.height) return;
  const int y = (int)(i / L.width), x = (int)(i - (int64_t)y * L.width);
  uint8_t* o = rgb + (int64_t)y * rgb_stride + (int64_t)x * 3;
  const int yy = work[L.plane_off[0] + (int64_t)y * L.bw[0] * 8 + x];
  if (L.ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)yy;
    return;
  }
  int cc[2];
#pragma unroll
  for (int k = 1; k < 3; ++k) {
    const int rh = L.max_h / L.h[k], rv = L.max_v / L.v[k];
    const int dw = (int)(((int64_t)L.width * L.h[k] + L.max_h - 1) / L.max_h);
    const int dh = (int)(((int64_t)L.height * L.v[k] + L.max_v - 1) / L.max_v);
    cc[k - 1] = chroma_at(work + L.plane_off[k], (int64_t)L.bw[k] * 8, rh, rv, dw, dh, x, y);
  }
  if (L.color == 2) {  // RGB components: no conversion
    o[0] = (uint8_t)yy;
    o[1] = (uint8_t)cc[0];
    o[2] = (uint8_t)cc[1];
    return;
  }
  const int cb = cc[0] - 128, cr = cc[1] - 128;
  const int r_off = (91881 * cr + 32768) >> 16;
  const int b_off = (116130 * cb + 32768) >> 16;
  const int g_off = (-22554 * cb + 32768 + -46802 * cr) >> 16;
  o[0] = clamp8(yy + r_off);
  o[1] = clamp8(yy + g_off);
  o[2] = clamp8(yy + b_off);
}

}  // namespace
}  // namespace sp

extern "C" int sp_jpeg_decode_coefs(const uint8_t* data, int64_t len, sp_jpeg_layout* lay, int16_t* coefs,
                                    int64_t coef_elems) {
  using namespace sp;
  SP_ARG_CHECK(data && lay && len > 0, "sp_jpeg_decode_coefs: null args");
  Decoder d{data, len, lay, coefs};
  const int rc = d.run(false);
  if (rc || !coefs) return rc;
  SP_ARG_CHECK(coef_elems >= lay->total_blocks * 64, "sp_jpeg_decode_coefs: coefficient buffer holds %lld < %lld",
               (long long)coef_elems, (long long)(lay->total_blocks * 64));
  Decoder d2{data, len, lay, coefs};
  return d2.run(true);
}

extern "C" int sp_jpeg_to_rgb(const int16_t* coefs, const sp_jpeg_layout* lay, uint8_t* work, int64_t work_bytes,
                              uint8_t* rgb, int64_t rgb_stride, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(coefs && lay && work && rgb, "sp_jpeg_to_rgb: null args");
  SP_ARG_CHECK(lay->ncomp == 1 || lay->ncomp == 3, "sp_jpeg_to_rgb: ncomp %d", lay->ncomp);
  SP_ARG_CHECK(work_bytes >= lay->plane_bytes, "sp_jpeg_to_rgb: work %lld < %lld bytes", (long long)work_bytes,
               (long long)lay->plane_bytes);
  SP_ARG_CHECK(rgb_stride >= 3LL * lay->width, "sp_jpeg_to_rgb: rgb_stride");
  for (int c = 0; c < lay->ncomp; ++c)
    SP_ARG_CHECK((int64_t)lay->bw[c] * 8 >= ((int64_t)lay->width * lay->h[c] + lay->max_h - 1) / lay->max_h &&
                     (int64_t)lay->bh[c] * 8 >= ((int64_t)lay->height * lay->v[c] + lay->max_v - 1) / lay->max_v &&
                     (reinterpret_cast<uintptr_t>(work + lay->plane_off[c]) & 7) == 0,
                 "sp_jpeg_to_rgb: inconsistent layout");
  hipStream_t s = as_stream(stream);
  const int64_t g1 = (lay->total_blocks + 31) / 32;
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)g1), dim3(256), 0, s, coefs, *lay, work);
  int rc = check_launch("sp_jpeg_to_rgb(idct)");
  if (rc) return rc;
  const int64_t px = (int64_t)lay->width * lay->height;
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((px + 255) / 256)), dim3(256), 0, s, *lay, work, rgb,
                     rgb_stride);
  return check_launch("sp_jpeg_to_rgb(color)");
}
