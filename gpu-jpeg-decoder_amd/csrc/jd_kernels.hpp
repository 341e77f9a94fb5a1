// jd_kernels.hpp — host-callable launchers for the gfx950 kernels in jd_kernels.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include "jd_internal.hpp"

namespace jd {

// Stage 0: find RSTn markers of every restart-interval image (HBM-bound byte scan).
hipError_t launch_rst_scan(const BatchDev& b, hipStream_t s);
// Stage 1: order the markers into per-segment start offsets (one wave per image).
hipError_t launch_rst_index(const BatchDev& b, hipStream_t s);
// Stage 2: Huffman entropy decode, one lane per restart interval (or per image without DRI).
hipError_t launch_huffman(const BatchDev& b, hipStream_t s);
// Stage 3: dequantise + 8x8 integer IDCT + chroma upsample + YCbCr->RGB, uint8 HWC out.
hipError_t launch_idct_color(const BatchDev& b, hipStream_t s);

// Known-answer hooks: run exactly the device arithmetic of stage 3 on caller data.
hipError_t launch_test_idct(const int32_t* in_zz, int32_t* out, int nblocks, hipStream_t s);
hipError_t launch_test_color(const int32_t* ycc, uint8_t* rgb, int n, hipStream_t s);

}  // namespace jd
