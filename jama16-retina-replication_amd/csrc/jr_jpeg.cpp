// jr_jpeg.cpp — native JPEG decode for the input pipeline (libjr_jpeg.so,
// host only; include/jr_jpeg.h).
//
// Replaces the decode half of tf.image.decode_jpeg at lib/dataset.py:20
// (channels=0: the file's own channel count).  TF decodes with libjpeg-turbo,
// dct_method "" = JDCT_IFAST, fancy upsampling on [TF-3P]; here the DCT
// method is selectable (JR_JPEG_IFAST, the TF default, or JR_JPEG_ISLOW, what
// Pillow uses).  The library linked is IJG libjpeg 9 (the only libjpeg with
// headers in this image, /opt/conda).  Its IDCTs are the same integer
// algorithms, but for subsampled chroma it scales the chroma IDCT up instead
// of upsampling (and its colour conversion differs in detail), up to 65 LSB
// away from libjpeg-turbo on 4:2:0 files.  So libjpeg 9 only runs the entropy
// decode and the IDCT (raw_data_out: every component at its own resolution)
// and this file does what libjpeg-turbo's decompressor does after that:
// "fancy" triangle-filter upsampling of h2v1 / h2v2 chroma (jdsample.c:
// 3/4 nearer + 1/4 further sample per dimension, the same rounding biases),
// with edge rows / columns replicated as jdmainct.c provides them, and the
// fixed-point YCbCr -> RGB tables of jdcolor.c (16 fraction bits).  Other
// sampling layouts fall back to libjpeg 9's own output path.
//
// One call decodes one image straight into the caller's HWC uint8 buffer,
// with no interpreter involvement: the pipeline's worker threads (ctypes
// releases the GIL) decode in parallel.
#include <algorithm>
#include <csetjmp>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
#include <jpeglib.h>
}

#include "../../include/jr_jpeg.h"

#define JR_JPEG_API extern "C" __attribute__((visibility("default")))

namespace {

thread_local std::string g_err;

struct ErrMgr {
  jpeg_error_mgr pub;
  jmp_buf jump;
};

void on_error(j_common_ptr cinfo) {
  ErrMgr* e = reinterpret_cast<ErrMgr*>(cinfo->err);
  char buf[JMSG_LENGTH_MAX];
  (*cinfo->err->format_message)(cinfo, buf);
  g_err = buf;
  std::longjmp(e->jump, 1);
}

void on_message(j_common_ptr) {}   // corrupt-data warnings: libjpeg recovers; TF does the same

// jdcolor.c build_ycc_rgb_table (SCALEBITS 16): the tables hold
//   Cr_r[cr] = (FIX(1.40200) * x + HALF) >> 16,  Cb_b[cb] = (FIX(1.77200) * x + HALF) >> 16,
//   Cr_g[cr] = -FIX(0.71414) * x,                Cb_g[cb] = -FIX(0.34414) * x + HALF
// (x = sample - 128), and R = y + Cr_r, G = y + ((Cb_g + Cr_g) >> 16),
// B = y + Cb_b, clamped.  Computed inline (the same int32 values, arithmetic
// shifts) so the row loop vectorises.
constexpr int kFixCrR = 91881, kFixCbB = 116130, kFixCrG = 46802, kFixCbG = 22554, kHalf = 1 << 15;
static_assert(kFixCrR == (int)(1.40200 * 65536 + 0.5) && kFixCbB == (int)(1.77200 * 65536 + 0.5) &&
                  kFixCrG == (int)(0.71414 * 65536 + 0.5) && kFixCbG == (int)(0.34414 * 65536 + 0.5),
              "jdcolor.c FIX() constants");

inline int clamp255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// one output row; planar R/G/B first (three vectorisable loops), then interleaved
void ycc_row(const uint8_t* __restrict Y, const uint8_t* __restrict cb, const uint8_t* __restrict cr, int w,
             uint8_t* __restrict rgb, uint8_t* __restrict tmp) {
  uint8_t* __restrict R = tmp;
  uint8_t* __restrict G = tmp + w;
  uint8_t* __restrict B = tmp + 2 * w;
  for (int x = 0; x < w; ++x) R[x] = (uint8_t)clamp255(Y[x] + ((kFixCrR * (cr[x] - 128) + kHalf) >> 16));
  for (int x = 0; x < w; ++x)
    G[x] = (uint8_t)clamp255(Y[x] + ((-kFixCbG * (cb[x] - 128) + kHalf - kFixCrG * (cr[x] - 128)) >> 16));
  for (int x = 0; x < w; ++x) B[x] = (uint8_t)clamp255(Y[x] + ((kFixCbB * (cb[x] - 128) + kHalf) >> 16));
  for (int x = 0; x < w; ++x) {
    rgb[3 * x] = R[x];
    rgb[3 * x + 1] = G[x];
    rgb[3 * x + 2] = B[x];
  }
}

// jdsample.c h2v1_fancy_upsample: one row, out has 2 * w samples
void up_h2(const uint8_t* in, int w, uint8_t* out) {
  if (w == 1) { out[0] = out[1] = in[0]; return; }
  int v = in[0];
  out[0] = (uint8_t)v;
  out[1] = (uint8_t)((v * 3 + in[1] + 2) >> 2);
  for (int c = 1; c < w - 1; ++c) {
    v = in[c] * 3;
    out[2 * c] = (uint8_t)((v + in[c - 1] + 1) >> 2);
    out[2 * c + 1] = (uint8_t)((v + in[c + 1] + 2) >> 2);
  }
  v = in[w - 1];
  out[2 * w - 2] = (uint8_t)((v * 3 + in[w - 2] + 1) >> 2);
  out[2 * w - 1] = (uint8_t)v;
}

// jdsample.c h2v2_fancy_upsample: one output row from the nearest input row
// (near) and the next nearest (far: the row above for the upper output row
// of a pair, below for the lower one).  Column sums s[c] = 3 near + far, then
// out[2c] = (3 s[c] + s[c-1] + 8) >> 4, out[2c+1] = (3 s[c] + s[c+1] + 7) >> 4,
// with s[-1] -> s[0] and s[w] -> s[w-1] at the edges (turbo writes those two
// as (4 s + 8) >> 4 and (4 s + 7) >> 4: the same values).
void up_h2v2_row(const uint8_t* __restrict near, const uint8_t* __restrict far, int w, uint8_t* __restrict out,
                 int16_t* __restrict s) {
  for (int c = 0; c < w; ++c) s[c + 1] = (int16_t)(near[c] * 3 + far[c]);
  s[0] = s[1];
  s[w + 1] = s[w];
  for (int c = 0; c < w; ++c) {
    const int t = s[c + 1] * 3;
    out[2 * c] = (uint8_t)((t + s[c] + 8) >> 4);
    out[2 * c + 1] = (uint8_t)((t + s[c + 2] + 7) >> 4);
  }
}

// jdsample.c h1v2_fancy_upsample (libjpeg-turbo; 4:4:0 files, e.g. losslessly
// transposed 4:2:2): out[c] = (3 near[c] + far[c] + bias) >> 2, bias 1 for the
// upper output row of a pair (far = the row above), 2 for the lower one
void up_v2_row(const uint8_t* __restrict near, const uint8_t* __restrict far, int w, int bias,
               uint8_t* __restrict out) {
  for (int c = 0; c < w; ++c) out[c] = (uint8_t)((near[c] * 3 + far[c] + bias) >> 2);
}

}  // namespace

JR_JPEG_API const char* jr_jpeg_last_error(void) { return g_err.c_str(); }

JR_JPEG_API int jr_jpeg_header(const uint8_t* data, size_t len, int32_t* height, int32_t* width, int32_t* channels) {
  if (!data || !height || !width || !channels) {
    g_err = "jr_jpeg_header: null argument";
    return -1;
  }
  jpeg_decompress_struct cinfo;
  ErrMgr err;
  cinfo.err = jpeg_std_error(&err.pub);
  err.pub.error_exit = on_error;
  err.pub.output_message = on_message;
  if (setjmp(err.jump)) {
    jpeg_destroy_decompress(&cinfo);
    return -1;
  }
  jpeg_create_decompress(&cinfo);
  jpeg_mem_src(&cinfo, const_cast<uint8_t*>(data), (unsigned long)len);
  jpeg_read_header(&cinfo, TRUE);
  *height = (int32_t)cinfo.image_height;
  *width = (int32_t)cinfo.image_width;
  *channels = cinfo.num_components == 1 ? 1 : 3;
  jpeg_destroy_decompress(&cinfo);
  return 0;
}

namespace {

// Every buffer of one decode.  It lives in jr_jpeg_decode's frame, OUTSIDE
// the function that calls setjmp: libjpeg reports errors by longjmp, which
// must not jump over the construction of objects with destructors (C++
// [csetjmp]); decode_into only resizes these through a reference.
struct DecodeBufs {
  std::vector<uint8_t> plane[3];
  std::vector<JSAMPROW> ptrs[3];
  std::vector<uint8_t> up_cb, up_cr, tmp;
  std::vector<int16_t> colsum;
};

int decode_into(DecodeBufs& bufs, const uint8_t* data, size_t len, uint8_t* out, int32_t height, int32_t width,
                int32_t channels, int32_t dct_method) {
  jpeg_decompress_struct cinfo;
  ErrMgr err;
  cinfo.err = jpeg_std_error(&err.pub);
  err.pub.error_exit = on_error;
  err.pub.output_message = on_message;
  if (setjmp(err.jump)) {
    jpeg_destroy_decompress(&cinfo);
    return -1;
  }
  jpeg_create_decompress(&cinfo);
  jpeg_mem_src(&cinfo, const_cast<uint8_t*>(data), (unsigned long)len);
  jpeg_read_header(&cinfo, TRUE);
  cinfo.dct_method = dct_method == JR_JPEG_IFAST ? JDCT_IFAST : JDCT_ISLOW;
  if ((int)cinfo.image_height != height || (int)cinfo.image_width != width ||
      (cinfo.num_components == 1 ? 1 : 3) != channels) {
    g_err = "jr_jpeg_decode: image is " + std::to_string(cinfo.image_height) + "x" +
            std::to_string(cinfo.image_width) + "x" + std::to_string(cinfo.num_components == 1 ? 1 : 3) +
            ", buffer " + std::to_string(height) + "x" + std::to_string(width) + "x" + std::to_string(channels);
    jpeg_destroy_decompress(&cinfo);
    return -1;
  }
  // the turbo-equivalent output path: YCbCr files whose chroma is full
  // (h1v1), h2v1, h1v2 (4:4:0) or h2v2 subsampled; anything else (4:1:1,
  // ...) takes libjpeg 9's own output path below
  bool own = cinfo.jpeg_color_space == JCS_YCbCr && cinfo.num_components == 3;
  if (own) {
    const jpeg_component_info* cp = cinfo.comp_info;
    const int H = cinfo.max_h_samp_factor, V = cinfo.max_v_samp_factor;
    own = cp[0].h_samp_factor == H && cp[0].v_samp_factor == V &&
          (H == 1 || H == 2) && (V == 1 || V == 2);
    for (int k = 1; k < 3 && own; ++k) own = cp[k].h_samp_factor == 1 && cp[k].v_samp_factor == 1;
  }
  if (own) {
    cinfo.raw_data_out = TRUE;
    jpeg_start_decompress(&cinfo);
    const int H = cinfo.max_h_samp_factor, V = cinfo.max_v_samp_factor;
    const int lw = (int)cinfo.comp_info[0].width_in_blocks * DCTSIZE;
    const int cw = (int)cinfo.comp_info[1].width_in_blocks * DCTSIZE;
    const int lh = (int)cinfo.comp_info[0].height_in_blocks * DCTSIZE;
    const int ch = (int)cinfo.comp_info[1].height_in_blocks * DCTSIZE;
    const int rows_per_call = V * DCTSIZE;
    // whole planes at component resolution (+ one iMCU row of slack)
    std::vector<uint8_t>* plane = bufs.plane;
    plane[0].resize((size_t)(lh + rows_per_call) * lw);
    plane[1].resize((size_t)(ch + DCTSIZE) * cw);
    plane[2].resize((size_t)(ch + DCTSIZE) * cw);
    std::vector<JSAMPROW>* ptrs = bufs.ptrs;
    ptrs[0].resize(rows_per_call);
    ptrs[1].resize(DCTSIZE);
    ptrs[2].resize(DCTSIZE);
    int y0 = 0, c0 = 0;
    while (cinfo.output_scanline < cinfo.output_height) {
      for (int r = 0; r < rows_per_call; ++r) ptrs[0][r] = plane[0].data() + (size_t)(y0 + r) * lw;
      for (int k = 1; k < 3; ++k)
        for (int r = 0; r < DCTSIZE; ++r) ptrs[k][r] = plane[k].data() + (size_t)(c0 + r) * cw;
      JSAMPARRAY arr[3] = {ptrs[0].data(), ptrs[1].data(), ptrs[2].data()};
      if (jpeg_read_raw_data(&cinfo, arr, rows_per_call) == 0) break;
      y0 += rows_per_call;
      c0 += DCTSIZE;
    }
    // downsampled (valid) chroma geometry, as jdmaster.c computes it
    const int dw = (width * 1 + H - 1) / H, dh = (height * 1 + V - 1) / V;
    std::vector<uint8_t>& up_cb = bufs.up_cb;
    std::vector<uint8_t>& up_cr = bufs.up_cr;
    std::vector<uint8_t>& tmp = bufs.tmp;
    std::vector<int16_t>& colsum = bufs.colsum;
    up_cb.resize((size_t)2 * dw + 2);
    up_cr.resize((size_t)2 * dw + 2);
    tmp.resize((size_t)3 * width);
    colsum.resize((size_t)dw + 2);
    for (int y = 0; y < height; ++y) {
      const uint8_t* Y = plane[0].data() + (size_t)y * lw;
      const uint8_t *cb, *cr;
      if (H == 1 && V == 1) {
        cb = plane[1].data() + (size_t)y * cw;
        cr = plane[2].data() + (size_t)y * cw;
      } else if (V == 1) {   // h2v1
        up_h2(plane[1].data() + (size_t)y * cw, dw, up_cb.data());
        up_h2(plane[2].data() + (size_t)y * cw, dw, up_cr.data());
        cb = up_cb.data();
        cr = up_cr.data();
      } else if (H == 1) {   // h1v2 (4:4:0): vertical triangle filter only
        const int cy = y >> 1;
        const int far = (y & 1) ? std::min(cy + 1, dh - 1) : std::max(cy - 1, 0);   // replicated edge rows
        for (int k = 1; k < 3; ++k)
          up_v2_row(plane[k].data() + (size_t)cy * cw, plane[k].data() + (size_t)far * cw, dw, (y & 1) ? 2 : 1,
                    (k == 1 ? up_cb : up_cr).data());
        cb = up_cb.data();
        cr = up_cr.data();
      } else {               // h2v2: row pair of chroma row cy
        const int cy = y >> 1;
        const int far = (y & 1) ? std::min(cy + 1, dh - 1) : std::max(cy - 1, 0);   // replicated edge rows
        for (int k = 1; k < 3; ++k) {
          const uint8_t* n = plane[k].data() + (size_t)cy * cw;
          const uint8_t* f = plane[k].data() + (size_t)far * cw;
          up_h2v2_row(n, f, dw, (k == 1 ? up_cb : up_cr).data(), colsum.data());
        }
        cb = up_cb.data();
        cr = up_cr.data();
      }
      ycc_row(Y, cb, cr, width, out + (size_t)y * width * 3, tmp.data());
    }
    jpeg_finish_decompress(&cinfo);
    jpeg_destroy_decompress(&cinfo);
    return 0;
  }
  cinfo.out_color_space = channels == 1 ? JCS_GRAYSCALE : JCS_RGB;
  cinfo.do_fancy_upsampling = TRUE;
  jpeg_start_decompress(&cinfo);
  if ((int)cinfo.output_height != height || (int)cinfo.output_width != width ||
      (int)cinfo.output_components != channels) {
    g_err = "jr_jpeg_decode: image is " + std::to_string(cinfo.output_height) + "x" +
            std::to_string(cinfo.output_width) + "x" + std::to_string(cinfo.output_components) + ", buffer " +
            std::to_string(height) + "x" + std::to_string(width) + "x" + std::to_string(channels);
    jpeg_destroy_decompress(&cinfo);
    return -1;
  }
  const size_t row = (size_t)width * channels;
  while (cinfo.output_scanline < cinfo.output_height) {
    JSAMPROW r = out + (size_t)cinfo.output_scanline * row;
    jpeg_read_scanlines(&cinfo, &r, 1);
  }
  jpeg_finish_decompress(&cinfo);
  jpeg_destroy_decompress(&cinfo);
  return 0;
}

}  // namespace

JR_JPEG_API int jr_jpeg_decode(const uint8_t* data, size_t len, uint8_t* out, int32_t height, int32_t width,
                               int32_t channels, int32_t dct_method) {
  if (!data || !out || height <= 0 || width <= 0 || (channels != 1 && channels != 3)) {
    g_err = "jr_jpeg_decode: bad arguments";
    return -1;
  }
  if (dct_method != JR_JPEG_IFAST && dct_method != JR_JPEG_ISLOW) {
    g_err = "jr_jpeg_decode: dct_method must be JR_JPEG_IFAST or JR_JPEG_ISLOW";
    return -1;
  }
  DecodeBufs bufs;
  return decode_into(bufs, data, len, out, height, width, channels, dct_method);
}
