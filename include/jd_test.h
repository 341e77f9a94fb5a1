/*
 * jd_test.h — known-answer test hooks of libjdamd.so.
 *
 * They run exactly the device arithmetic of the decode path's stage 3 (jd_kernels.hip) on
 * caller-provided data so tests can check the integer IDCT (reference cpp-decoder/src/idct.cpp:
 * 34-133) and the colour conversion (utils/color.cpp:8-19) exhaustively.  All pointers are
 * device pointers (jd_device_alloc); the calls are synchronous.
 */
#ifndef JD_TEST_H
#define JD_TEST_H

#include "jd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* in: nblocks x 64 dequantised coefficients in zig-zag order; out: nblocks x 64 natural order */
jd_status jd_test_idct(jd_ctx* ctx, const int32_t* in_dev, int32_t* out_dev, int nblocks);
/* ycc: n x (Y, Cb, Cr) IDCT outputs in [-256,255]; rgb: n x 3 bytes */
jd_status jd_test_color(jd_ctx* ctx, const int32_t* ycc_dev, uint8_t* rgb_dev, int n);

#ifdef __cplusplus
}
#endif
#endif
