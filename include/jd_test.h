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
/* jd_test_idct runs the decode path's choice per block: the fast 24-bit-multiply form when every
 * input is within +-2^16, else the exact form (the reference's formulas with its DC-only
 * shortcuts, any int32 input).  jd_test_idct_exact forces the exact form. */
jd_status jd_test_idct_exact(jd_ctx* ctx, const int32_t* in_dev, int32_t* out_dev, int nblocks);
/* ycc: n x (Y, Cb, Cr) IDCT outputs in [-256,255]; rgb: n x 3 bytes */
jd_status jd_test_color(jd_ctx* ctx, const int32_t* ycc_dev, uint8_t* rgb_dev, int n);

/* HBM copy peak: copies `bytes` (a multiple of 16) from src_dev to dst_dev `reps` times with a
 * 16-byte-per-lane kernel and returns the read + write rate in GB/s (hipEvents on the context
 * stream; the roofline reference of bench.py). */
jd_status jd_test_copy_peak(jd_ctx* ctx, const void* src_dev, void* dst_dev, size_t bytes, int reps, double* gbs);

/* Copies an internal array of the most recent batch to the host (debugging / white-box tests).
 * what: 0 blocks (8 B each), 1 seg_cstart, 2 seg_cend, 3 seg_sub_base, 4 seg_nsub (u32 each),
 *       5 piece_bit, 6 piece_end, 7 piece_nmcu, 8 piece_nent, 9 sub_seg (u32 per piece slot),
 *       10 status (u32 per image), 11 entries (u32), 12 piece_mcu0, 13 piece_ent0 (u32 per piece
 *       slot), 14 piece_cp (9 x 16 B per piece slot: 8 scan checkpoints {bit, MCUs, entries,
 *       error} and the totals {end, MCUs, entries, error | checkpoints << 8}), 15 stamps,
 *       16 piece_emcu, 17 piece_amcu, 18 piece_join (u32 per piece slot), 19 seg_ent (u32 per
 *       segment), 20 entry_base (u64 per image: first 32-bit word of its AC-entry region),
 *       21 rw_div (u32 per image: walk bits per piece-region word, jd_internal.hpp region_words).
 *       22 rw_slack (u32 per image: region words per piece beyond plen / rw_div, region_words).
 *       *nbytes receives the array size; at most cap bytes are copied. */
jd_status jd_debug_fetch(jd_ctx* ctx, int what, void* host_dst, size_t cap, size_t* nbytes);

#ifdef __cplusplus
}
#endif
#endif
