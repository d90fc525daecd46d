// JPEG encode behind serve.py:139-142 (`image.save(buffer, format="JPEG")`, Pillow → libjpeg-turbo), on the GPU:
//
//   jpeg_fdct_kernel    one wave per MCU: RGB → YCbCr (jccolor.c fixed point), 2x2 / 2x1 chroma averaging with
//                       libjpeg's alternating bias (jcsample.c) over the edge-replicated image (jcprepct.c),
//                       ISLOW forward DCT (jfdctint.c, rows then columns through LDS), quantisation by the
//                       reciprocal / correction / shift of jcdctmgr.c, dummy blocks past the image edge
//                       (jccoefct.c); quantised coefficients stored in scan order, zig-zag order per block.
//   jpeg_mcu_bits_kernel  one thread per MCU: the Huffman-coded length of the MCU (DC differences against the
//                       previous block of each component, AC run lengths, ZRL, EOB; jchuff.c encode_one_block).
//   jpeg_scan_kernel    one workgroup: exclusive prefix sum of the MCU lengths → each MCU's bit offset; the
//                       total; zeroes the words the segment will occupy.
//   jpeg_emit_kernel    one thread per MCU: the same walk again, writing its codes at its offset (32-bit
//                       atomic ORs; only the first and last word of an MCU are shared with its neighbours).
//
// The host (jpeg_host.h enc_finish) adds the markers, the 0xFF byte stuffing and the final 1-bit padding. The
// Huffman tables are the Annex K.3 ones libjpeg uses without optimize_coding, derived at compile time from the
// same arrays the DHT markers are written from. oracle/jpeg_enc_np.py restates the whole path and pins it
// against Pillow's own output; tests/test_gpu_jpeg.py checks this file's bytes against both.
#include "common.h"
#include "jpeg_host.h"

namespace sp {
namespace {
using namespace jpeg_host;

__constant__ EncHuff kEncTab[4] = {derive_enc(kDcLumBits, kDcVals), derive_enc(kAcLumBits, kAcLumVals),
                                   derive_enc(kDcChrBits, kDcVals), derive_enc(kAcChrBits, kAcChrVals)};
// natural (row-major) index → zig-zag position
__constant__ uint8_t kZigzag[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                    3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                    10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// jccolor.c rgb_ycc_start: FIX(x) = x * 2^16 rounded; Cb / Cr carry CBCR_OFFSET + ONE_HALF - 1
constexpr int kFR_Y = 19595, kFG_Y = 38470, kFB_Y = 7471;
constexpr int kFR_CB = 11059, kFG_CB = 21709, kF_HALF = 32768, kFG_CR = 27439, kFB_CR = 5329;

__device__ __forceinline__ int rgb_y(const uint8_t* p) {
  return (kFR_Y * p[0] + kFG_Y * p[1] + kFB_Y * p[2] + 32768) >> 16;
}
__device__ __forceinline__ int rgb_cb(const uint8_t* p) {
  return (-kFR_CB * p[0] - kFG_CB * p[1] + kF_HALF * p[2] + (128 << 16) + 32767) >> 16;
}
__device__ __forceinline__ int rgb_cr(const uint8_t* p) {
  return (kF_HALF * p[0] - kFG_CR * p[1] - kFB_CR * p[2] + (128 << 16) + 32767) >> 16;
}

// jfdctint.c jpeg_fdct_islow, one 1-D pass over 8 values: pass 1 (rows) leaves the even DC terms scaled up by
// PASS1_BITS and DESCALEs the rest by CONST_BITS - PASS1_BITS; pass 2 (columns) DESCALEs by PASS1_BITS and
// CONST_BITS + PASS1_BITS (output scaled by 8, which the quantiser's divisors quantval << 3 absorb).
template <bool PASS2>
__device__ __forceinline__ void fdct_1d(const int (&d)[8], int (&o)[8]) {
  constexpr int CB = 13, P1 = 2, SH = PASS2 ? CB + P1 : CB - P1;
  const int tmp0 = d[0] + d[7], tmp7 = d[0] - d[7], tmp1 = d[1] + d[6], tmp6 = d[1] - d[6];
  const int tmp2 = d[2] + d[5], tmp5 = d[2] - d[5], tmp3 = d[3] + d[4], tmp4 = d[3] - d[4];
  const int tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  auto ds = [](int v, int n) { return (v + (1 << (n - 1))) >> n; };
  if (PASS2) {
    o[0] = ds(tmp10 + tmp11, P1);
    o[4] = ds(tmp10 - tmp11, P1);
  } else {
    o[0] = (tmp10 + tmp11) * (1 << P1);
    o[4] = (tmp10 - tmp11) * (1 << P1);
  }
  const int z1 = (tmp12 + tmp13) * 4433;
  o[2] = ds(z1 + tmp13 * 6270, SH);
  o[6] = ds(z1 + tmp12 * -15137, SH);
  const int z5 = (tmp4 + tmp6 + tmp5 + tmp7) * 9633;
  const int a1 = (tmp4 + tmp7) * -7373, a2 = (tmp5 + tmp6) * -20995;
  const int a3 = (tmp4 + tmp6) * -16069 + z5, a4 = (tmp5 + tmp7) * -3196 + z5;
  o[7] = ds(tmp4 * 2446 + a1 + a3, SH);
  o[5] = ds(tmp5 * 16819 + a2 + a4, SH);
  o[3] = ds(tmp6 * 25172 + a2 + a3, SH);
  o[1] = ds(tmp7 * 12299 + a1 + a4, SH);
}

constexpr int kMcuPerWg = 4;  // one wave per MCU

__global__ __launch_bounds__(256) void jpeg_fdct_kernel(const uint8_t* __restrict__ rgb, int64_t stride, int pb,
                                                        const sp_jpeg_enc_layout L, int16_t* __restrict__ coefs) {
  __shared__ int ws[kMcuPerWg][6][8][9];
  __shared__ int qv[kMcuPerWg][6][64];
  __shared__ uint8_t nat_of_zz[64];
  if (threadIdx.x < 64) nat_of_zz[kZigzag[threadIdx.x]] = (uint8_t)threadIdx.x;  // read after the barriers below
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t mcu = (int64_t)blockIdx.x * kMcuPerWg + w;
  const int64_t nmcu = (int64_t)L.mcux * L.mcuy;
  const int j = lane >> 3, r = lane & 7;  // block within the MCU, row (pass 1) / column (pass 2)
  const int ny = L.h0 * L.v0;
  const bool live = mcu < nmcu && j < L.bpm;
  const int my = live ? (int)(mcu / L.mcux) : 0, mx = live ? (int)(mcu - (int64_t)my * L.mcux) : 0;
  const int W = L.width, H = L.height;
  const int comp = j < ny ? 0 : j - ny + 1;
  const int bx = comp == 0 ? mx * L.h0 + (j % L.h0) : mx, by = comp == 0 ? my * L.v0 + (j / L.h0) : my;
  const bool dummy = comp == 0 && (bx >= L.wb0 || by >= L.hb0);
  if (live && !dummy) {
    int s[8];
    if (comp == 0) {  // luma: the edge-replicated plane (columns and rows past the image repeat the last one)
      const int y = min(by * 8 + r, H - 1);
      SP_BCHECK(y, H);
      SP_BCHECK(bx * 8, (int64_t)L.wb0 * 8);
      const uint8_t* row = rgb + (int64_t)y * stride;
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = rgb_y(row + (int64_t)min(bx * 8 + i, W - 1) * pb) - 128;
    } else {
      // chroma at 1x1 against luma (h0, v0): rows of the downsampled plane past ceil(H / v0) repeat its last
      // row (jcprepct.c pads the iMCU after downsampling); the full-resolution rows and columns feeding a
      // sample are clamped to the image (expand_right_edge, the row-group padding)
      const int cy = min(by * 8 + r, (H + L.v0 - 1) / L.v0 - 1);
      const int y0 = min(cy * L.v0, H - 1), y1 = min(cy * L.v0 + L.v0 - 1, H - 1);
      SP_BCHECK(y0, H);
      SP_BCHECK(y1, H);
      const uint8_t* r0 = rgb + (int64_t)y0 * stride;
      const uint8_t* r1 = rgb + (int64_t)y1 * stride;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int cx = bx * 8 + i;
        int v;
        if (L.h0 == 1) {
          const uint8_t* p = r0 + (int64_t)min(cx, W - 1) * pb;
          v = comp == 1 ? rgb_cb(p) : rgb_cr(p);
        } else {
          const uint8_t* p0 = r0 + (int64_t)min(2 * cx, W - 1) * pb;
          const uint8_t* p1 = r0 + (int64_t)min(2 * cx + 1, W - 1) * pb;
          if (L.v0 == 2) {  // h2v2_downsample: bias 1, 2, 1, 2, ...
            const uint8_t* p2 = r1 + (int64_t)min(2 * cx, W - 1) * pb;
            const uint8_t* p3 = r1 + (int64_t)min(2 * cx + 1, W - 1) * pb;
            const int sum = comp == 1 ? rgb_cb(p0) + rgb_cb(p1) + rgb_cb(p2) + rgb_cb(p3)
                                      : rgb_cr(p0) + rgb_cr(p1) + rgb_cr(p2) + rgb_cr(p3);
            v = (sum + 1 + (cx & 1)) >> 2;
          } else {  // h2v1_downsample: bias 0, 1, 0, 1, ...
            const int sum = comp == 1 ? rgb_cb(p0) + rgb_cb(p1) : rgb_cr(p0) + rgb_cr(p1);
            v = (sum + (cx & 1)) >> 1;
          }
        }
        s[i] = v - 128;
      }
    }
    int o[8];
    fdct_1d<false>(s, o);
#pragma unroll
    for (int i = 0; i < 8; ++i) ws[w][j][r][i] = o[i];
  }
  __syncthreads();
  if (live && !dummy) {
    int col[8], o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) col[i] = ws[w][j][i][r];
    fdct_1d<true>(col, o);
    const int t = comp == 0 ? 0 : 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // jcdctmgr.c quantize, 16-bit DCTELEM form
      const int n = i * 8 + r;
      const int x = o[i];
      const uint32_t a = (uint32_t)(x < 0 ? -x : x);
      const uint32_t q = ((a + L.corr[t][n]) * (uint32_t)L.recip[t][n]) >> (16 + L.shift[t][n]);
      qv[w][j][n] = x < 0 ? -(int)q : (int)q;
    }
  }
  __syncthreads();
  if (!live) return;
  // store: lane (j, r) writes zig-zag positions 8r .. 8r+7 of block j as one 16-byte piece
  SP_BCHECK(mcu * L.bpm + j, (int64_t)L.mcux * L.mcuy * L.bpm);
  int16_t* dst = coefs + (mcu * L.bpm + j) * 64;
  int16_t v[8];
  if (!dummy) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (int16_t)qv[w][j][nat_of_zz[8 * r + i]];
  } else {
    // jccoefct.c compress_data: zero AC; a right-edge dummy takes the DC of the block to its left, a dummy row
    // below the image the DC of the last block of the row above (itself a right-edge dummy → its left one)
    int src;
    if (by < L.hb0) {
      src = j - 1;
    } else {
      const int row_above = (j / L.h0) - 1;
      src = row_above * L.h0 + (L.h0 - 1);
      if (mx * L.h0 + (L.h0 - 1) >= L.wb0) src -= 1;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0;
    SP_BCHECK(src, L.bpm);
    if (r == 0) v[0] = (int16_t)qv[w][src][0];
  }
  int4 pk;
  pk.x = (int)((uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16));
  pk.y = (int)((uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16));
  pk.z = (int)((uint16_t)v[4] | ((uint32_t)(uint16_t)v[5] << 16));
  pk.w = (int)((uint16_t)v[6] | ((uint32_t)(uint16_t)v[7] << 16));
  *reinterpret_cast<int4*>(dst + 8 * r) = pk;
}

__device__ __forceinline__ int nbits_of(int a) { return a ? 32 - __clz(a) : 0; }

// Walks one MCU's blocks in scan order and hands every (code, length) / (magnitude bits, count) to `put`:
// jchuff.c encode_one_block.
template <typename Put>
__device__ __forceinline__ void walk_mcu(const int16_t* __restrict__ coefs, const sp_jpeg_enc_layout& L, int64_t mcu,
                                         Put&& put) {
  const int ny = L.h0 * L.v0;
  const int16_t* blk = coefs + mcu * L.bpm * 64;
  const int16_t* prev_mcu = mcu > 0 ? blk - L.bpm * 64 : nullptr;
  for (int j = 0; j < L.bpm; ++j, blk += 64) {
    const int comp = j < ny ? 0 : j - ny + 1;
    const EncHuff& dc = kEncTab[comp == 0 ? 0 : 2];
    const EncHuff& ac = kEncTab[comp == 0 ? 1 : 3];
    int last;
    if (comp == 0)
      last = j > 0 ? blk[-64] : (prev_mcu ? prev_mcu[(ny - 1) * 64] : 0);
    else
      last = prev_mcu ? prev_mcu[j * 64] : 0;
    int diff = blk[0] - last;
    int a = diff < 0 ? -diff : diff;
    int nb = nbits_of(a);
    put(dc.code[nb], dc.size[nb]);
    if (nb) put((uint32_t)(diff < 0 ? diff - 1 : diff) & ((1u << nb) - 1), nb);
    int run = 0;
    const int4* q = reinterpret_cast<const int4*>(blk);
#pragma unroll 1
    for (int c8 = 0; c8 < 8; ++c8) {
      const int4 pk = q[c8];
      const uint32_t w4[4] = {(uint32_t)pk.x, (uint32_t)pk.y, (uint32_t)pk.z, (uint32_t)pk.w};
      if ((w4[0] | w4[1] | w4[2] | w4[3]) == 0 && c8 > 0) {  // 8 zero coefficients
        run += 8;
        continue;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (c8 == 0 && e == 0) continue;  // DC
        const int x = (int16_t)(w4[e >> 1] >> (16 * (e & 1)));
        if (x == 0) {
          ++run;
          continue;
        }
        while (run > 15) {
          put(ac.code[0xF0], ac.size[0xF0]);
          run -= 16;
        }
        a = x < 0 ? -x : x;
        nb = nbits_of(a);
        const int sym = (run << 4) + nb;
        put(ac.code[sym], ac.size[sym]);
        put((uint32_t)(x < 0 ? x - 1 : x) & ((1u << nb) - 1), nb);
        run = 0;
      }
    }
    if (run > 0) put(ac.code[0], ac.size[0]);
  }
}

__global__ __launch_bounds__(256) void jpeg_mcu_bits_kernel(const int16_t* __restrict__ coefs,
                                                            const sp_jpeg_enc_layout L, int32_t* __restrict__ bits) {
  const int64_t mcu = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (mcu >= (int64_t)L.mcux * L.mcuy) return;
  int n = 0;
  walk_mcu(coefs, L, mcu, [&](uint32_t, int len) { n += len; });
  bits[mcu] = n;
}

// exclusive prefix sum of the per-MCU bit counts (one workgroup, each thread a contiguous chunk), the total at
// total[0], then the words [0, ceil(total / 32)] of the bit buffer zeroed for the atomic ORs of the emit pass
__global__ __launch_bounds__(1024) void jpeg_scan_kernel(const int32_t* __restrict__ bits, int64_t n,
                                                         int64_t* __restrict__ off, int64_t* __restrict__ total,
                                                         uint32_t* __restrict__ words, int64_t words_cap) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t lo = min(n, t * chunk), hi = min(n, lo + chunk);
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += bits[i];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan of the chunk sums
    const int64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int64_t i = lo; i < hi; ++i) {
    off[i] = run;
    run += bits[i];
  }
  const int64_t tot = part[1023];
  if (t == 0) total[0] = tot;
  const int64_t nw = (tot + 31) / 32 + 1;
  for (int64_t i = t; i < nw; i += 1024) SP_BCHECK(i, words_cap);
  for (int64_t i = t; i < nw; i += 1024) words[i] = 0;
}

__global__ __launch_bounds__(256) void jpeg_emit_kernel(const int16_t* __restrict__ coefs, const sp_jpeg_enc_layout L,
                                                        const int64_t* __restrict__ off, uint32_t* __restrict__ words) {
  const int64_t mcu = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (mcu >= (int64_t)L.mcux * L.mcuy) return;
  const int64_t o = off[mcu];
  int64_t wi = o >> 5;
  uint64_t acc = 0;  // pending bits, left-aligned; the first (o & 31) belong to the previous MCU's word
  int nacc = (int)(o & 31);
  walk_mcu(coefs, L, mcu, [&](uint32_t code, int len) {
    acc |= (uint64_t)code << (64 - nacc - len);
    nacc += len;
    if (nacc >= 32) {
      SP_BCHECK(wi, L.bits_cap / 4);  // the MCU's bits stay inside the layout's bit buffer bound
      atomicOr(words + wi, __builtin_bswap32((uint32_t)(acc >> 32)));
      acc <<= 32;
      nacc -= 32;
      ++wi;
    }
  });
  if (nacc > 0) SP_BCHECK(wi, L.bits_cap / 4);
  if (nacc > 0) atomicOr(words + wi, __builtin_bswap32((uint32_t)(acc >> 32)));
}

}  // namespace
}  // namespace sp

extern "C" int sp_jpeg_enc_plan(int32_t width, int32_t height, int32_t quality, int32_t subsampling,
                                sp_jpeg_enc_layout* lay) {
  SP_ARG_CHECK(lay, "sp_jpeg_enc_plan: null layout");
  SP_ARG_CHECK(sp::jpeg_host::enc_plan(width, height, quality, subsampling, lay) == 0,
               "sp_jpeg_enc_plan: unsupported %dx%d quality %d subsampling %d", width, height, quality, subsampling);
  return 0;
}

extern "C" int sp_jpeg_enc_rgb(const uint8_t* rgb, int64_t row_stride, int32_t pixel_bytes,
                               const sp_jpeg_enc_layout* lay, uint8_t* work, int64_t work_bytes, uint8_t* bits,
                               int64_t bits_cap, int64_t* nbits, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(rgb && lay && work && bits && nbits, "sp_jpeg_enc_rgb: null args");
  SP_ARG_CHECK(pixel_bytes == 3 || pixel_bytes == 4, "sp_jpeg_enc_rgb: pixel_bytes %d", pixel_bytes);
  SP_ARG_CHECK(row_stride >= (int64_t)pixel_bytes * lay->width, "sp_jpeg_enc_rgb: row_stride");
  sp_jpeg_enc_layout chk;
  SP_ARG_CHECK(jpeg_host::enc_plan(lay->width, lay->height, lay->quality, lay->h0 == 1 ? 0 : (lay->v0 == 1 ? 1 : 2),
                                   &chk) == 0 &&
                   memcmp(&chk, lay, sizeof(chk)) == 0,
               "sp_jpeg_enc_rgb: layout is not sp_jpeg_enc_plan's");
  SP_ARG_CHECK(work_bytes >= lay->work_bytes && bits_cap >= lay->bits_cap, "sp_jpeg_enc_rgb: buffers too small");
  SP_ARG_CHECK((reinterpret_cast<uintptr_t>(work) & 255) == 0 && (reinterpret_cast<uintptr_t>(bits) & 3) == 0,
               "sp_jpeg_enc_rgb: work must be 256-byte and bits 4-byte aligned");
  hipStream_t s = as_stream(stream);
  const int64_t nmcu = (int64_t)lay->mcux * lay->mcuy;
  int64_t* total = reinterpret_cast<int64_t*>(work);
  int64_t* off = total + 1;
  int32_t* mbits = reinterpret_cast<int32_t*>(off + nmcu);
  int16_t* coefs = reinterpret_cast<int16_t*>(work + jpeg_host::enc_coef_offset(*lay));
  hipLaunchKernelGGL(jpeg_fdct_kernel, dim3((unsigned)((nmcu + kMcuPerWg - 1) / kMcuPerWg)), dim3(256), 0, s, rgb,
                     row_stride, (int)pixel_bytes, *lay, coefs);
  int rc = check_launch("sp_jpeg_enc_rgb(fdct)");
  if (rc) return rc;
  const unsigned g = (unsigned)((nmcu + 255) / 256);
  hipLaunchKernelGGL(jpeg_mcu_bits_kernel, dim3(g), dim3(256), 0, s, coefs, *lay, mbits);
  if ((rc = check_launch("sp_jpeg_enc_rgb(bits)"))) return rc;
  hipLaunchKernelGGL(jpeg_scan_kernel, dim3(1), dim3(1024), 0, s, mbits, nmcu, off, total,
                     reinterpret_cast<uint32_t*>(bits), bits_cap / 4);
  if ((rc = check_launch("sp_jpeg_enc_rgb(scan)"))) return rc;
  hipLaunchKernelGGL(jpeg_emit_kernel, dim3(g), dim3(256), 0, s, coefs, *lay, off, reinterpret_cast<uint32_t*>(bits));
  if ((rc = check_launch("sp_jpeg_enc_rgb(emit)"))) return rc;
  if (hipMemcpyAsync(nbits, total, sizeof(int64_t), hipMemcpyDeviceToDevice, s) != hipSuccess) {
    set_error("sp_jpeg_enc_rgb: copy of the bit count failed");
    return -1;
  }
  return 0;
}

extern "C" int64_t sp_jpeg_enc_max_bytes(const sp_jpeg_enc_layout* lay, int64_t nbits, int64_t comment_len) {
  return lay ? sp::jpeg_host::enc_max_bytes(*lay, nbits, comment_len) : -1;
}

extern "C" int sp_jpeg_enc_finish(const sp_jpeg_enc_layout* lay, const uint8_t* bits, int64_t nbits,
                                  const uint8_t* comment, int64_t comment_len, uint8_t* out, int64_t out_cap,
                                  int64_t* out_len) {
  SP_ARG_CHECK(lay && (bits || nbits == 0) && out && out_len && (comment || comment_len == 0),
               "sp_jpeg_enc_finish: null args");
  SP_ARG_CHECK(nbits <= lay->bits_cap * 8, "sp_jpeg_enc_finish: %lld bits exceed the layout's bound",
               (long long)nbits);
  SP_ARG_CHECK(sp::jpeg_host::enc_finish(*lay, bits, nbits, comment, comment_len, out, out_cap, out_len) == 0,
               "sp_jpeg_enc_finish: output buffer of %lld bytes too small (or comment too long)", (long long)out_cap);
  return 0;
}
