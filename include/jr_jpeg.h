/*
 * jr_jpeg.h — C-ABI of libjr_jpeg.so, the native JPEG decoder of the input
 * pipeline (host only; replaces the decode of tf.image.decode_jpeg at
 * lib/dataset.py:20, channels=0).  Kept out of libjr.so so the compute
 * library does not depend on the image's libjpeg.
 *
 * Functions return 0 on success, -1 on failure (message: jr_jpeg_last_error,
 * thread-local).  dct_method selects the IDCT: JR_JPEG_IFAST is TF's default
 * (dct_method ""), JR_JPEG_ISLOW what Pillow uses.
 */
#ifndef JR_JPEG_H_
#define JR_JPEG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { JR_JPEG_IFAST = 0, JR_JPEG_ISLOW = 1 };

const char* jr_jpeg_last_error(void);
/* image geometry; channels = 1 (grayscale) or 3 (every colour file is RGB) */
int jr_jpeg_header(const uint8_t* data, size_t len, int32_t* height, int32_t* width, int32_t* channels);
/* decode into out [height][width][channels] uint8; the geometry must match */
int jr_jpeg_decode(const uint8_t* data, size_t len, uint8_t* out, int32_t height, int32_t width, int32_t channels,
                   int32_t dct_method);

#ifdef __cplusplus
}
#endif
#endif /* JR_JPEG_H_ */
