/* jdenc.h — deterministic baseline JPEG encoder for bench / test inputs (see jdenc.c). */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { JDENC_EINVAL = -1, JDENC_ENOMEM = -2, JDENC_ESPACE = -3 };

/* Encodes width x height pixels (ncomp 3: RGB interleaved; 1: grayscale) as a baseline JPEG.
 * hs x vs = luma sampling factors (chroma 1x1), restart = MCUs per restart interval (0: none).
 * Returns the file length, or a negative JDENC_* code (JDENC_ESPACE: cap too small). */
long jdenc_encode(const uint8_t* px, int width, int height, int ncomp, int quality, int hs, int vs, int restart,
                  uint8_t* out, size_t cap);

/* An output capacity that always suffices. */
size_t jdenc_bound(int width, int height);

#ifdef __cplusplus
}
#endif
