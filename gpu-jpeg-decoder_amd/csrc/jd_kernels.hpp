// jd_kernels.hpp — host-callable launchers for the gfx950 kernels in jd_kernels.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include "jd_internal.hpp"

namespace jd {

// The decode pipeline, kernel by kernel (jd_kernel_name(k) names them; DESIGN.md §4 describes
// each):  0 k_scan, 1 k_index, 2 k_compact (un-stuffing), 3 k_pieceplan + k_subplan, 4 k_piece,
// 5 k_redo, 6 k_chain + k_chain_fix, 7 k_gather (Huffman), 8 k_dc_sum + k_dc_scan,
// 9 k_idct_color (+ k_idct_color_exact), 10 k_colour_fancy.
hipError_t launch_kernel(int k, const BatchDev& b, hipStream_t s);
size_t huffman_lds_bytes(uint32_t max_slots);
// Piece lanes k_piece keeps resident on the device at this dynamic LDS (workgroups per CU x CUs x
// workgroup size); k_pieceplan fits the batch's pieces to whole rounds of them.
uint32_t piece_lanes_resident(size_t lds);

// Known-answer hooks: run exactly the device arithmetic of stage 3 on caller data.
hipError_t launch_test_idct(const int32_t* in_zz, int32_t* out, int nblocks, int exact_only, hipStream_t s);
hipError_t launch_test_color(const int32_t* ycc, uint8_t* rgb, int n, hipStream_t s);
// 16-byte-per-lane device copy (bytes a multiple of 16): the in-run HBM peak (jd_test_copy_peak).
hipError_t launch_copy16(const void* src, void* dst, size_t bytes, hipStream_t s);

}  // namespace jd
