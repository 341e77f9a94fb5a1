/*
 * jdoracle.h — CPU restatement of the reference decoder's decode(file) -> RGB path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gpu-jpeg-decoder_amd/) links, loads or calls
 * this code.  It is imported solely by tests/, __graft_entry__.smoke() (as the checker) and the
 * cpu_baseline leg of bench.py.
 *
 * Parity pinning: the 4:4:4 / no-restart subset is pinned bit-exactly against the reference's own
 * ground truth (/root/reference/testing/ground_truth/NAME.array, digests in tests/golden/) and against
 * the reference C++ decoder compiled from its sources by oracle/Makefile (oracle/_ref/decoder).
 * The extension to other sampling factors and restart intervals is NOT covered by the reference
 * (it decodes those to garbage); its semantics are defined in DESIGN.md §3 and are
 * pinned by the invariance tests in tests/test_oracle.py.
 */
#ifndef JDORACLE_H
#define JDORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: numerically identical to include/jd.h so tests can compare them directly. */
enum {
    JDO_OK = 0,
    JDO_ERR_INVALID_ARG = 1,
    JDO_ERR_CORRUPT = 2,
    JDO_ERR_UNSUPPORTED = 3,
    JDO_ERR_TRUNCATED = 4,
};

typedef struct {
    int width, height, ncomp;
    int hmax, vmax, mcux, mcuy, blocks_per_mcu;
    int restart_interval;
    int h[4], v[4], tq[4];
    size_t ecs_offset;
} jdo_info;

/* Parse headers only. */
int jdo_parse(const uint8_t* jpeg, size_t len, jdo_info* info);

/* Full decode to interleaved uint8 RGB (H*W*3).  rgb may be NULL (decode + status only). */
int jdo_decode(const uint8_t* jpeg, size_t len, uint8_t* rgb, int* width, int* height);

/* As jdo_decode; flags: JDO_FANCY_UPSAMPLING = libjpeg's triangular chroma filter for 2x1, 2x2
 * and 1x2 sampling ratios instead of replication (numerically equal to jd.h's flag). */
#define JDO_FANCY_UPSAMPLING 8u
int jdo_decode_ex(const uint8_t* jpeg, size_t len, uint8_t* rgb, int* width, int* height, unsigned flags);

/* Entropy-decode only: quantised coefficients of every block, 64 int32 per block in zig-zag order
 * with the DC already un-predicted (absolute).  Blocks are in scan order: mcu * blocks_per_mcu + b.
 * coef must hold mcux*mcuy*blocks_per_mcu*64 ints. */
int jdo_decode_coefs(const uint8_t* jpeg, size_t len, int32_t* coef);

/* Arithmetic kernels exposed for known-answer tests. */
void jdo_idct_ref(const int32_t in_zigzag_dequant[64], int32_t out_natural[64]);
void jdo_color_ref(int y, int cb, int cr, uint8_t rgb[3]);

/* Batch timing helper for the CPU baseline: decodes n files, `threads` worker threads.
 * Returns wall seconds; statuses written to status[i] when non-NULL. */
double jdo_decode_many(const uint8_t* const* jpegs, const size_t* lens, int n, uint8_t* const* rgbs,
                       int threads, int* status);
/* "fast" CPU mode (LUT Huffman): the same pixels and status as jdo_decode, a CPU
 * baseline only.  jdo_decode_many_ex(..., fast = 1) times it. */
int jdo_decode_fast(const uint8_t* jpeg, size_t len, uint8_t* rgb, int* width, int* height);
/* Mismatches of the fast mode's integer colour against jdo_color_ref over all of [-256, 255]^3. */
long jdo_check_color_fast(void);
double jdo_decode_many_ex(const uint8_t* const* jpegs, const size_t* lens, int n, uint8_t* const* rgbs,
                          int threads, int* status, int fast);

#ifdef __cplusplus
}
#endif
#endif
