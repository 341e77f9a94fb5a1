// jd_kernels.hpp — host-callable launchers for the gfx950 kernels in jd_kernels.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include "jd_internal.hpp"

namespace jd {

// Stage 0: scan every image's ECS for stuffed zeros and RSTn / terminating markers (HBM-bound).
hipError_t launch_scan(const BatchDev& b, hipStream_t s);
// Stage 1: per image (one wave): un-stuffed chunk offsets and restart-interval boundaries.
hipError_t launch_index(const BatchDev& b, hipStream_t s);
// Stage 2: un-stuff (drop the 00 after every FF) into one contiguous stream per image.
hipError_t launch_compact(const BatchDev& b, hipStream_t s);
// Stage 3: Huffman entropy decode, one lane per restart interval (or per image without DRI).
hipError_t launch_huffman(const BatchDev& b, hipStream_t s);
size_t huffman_lds_bytes(uint32_t max_slots);
// Stage 4: dequantise + 8x8 integer IDCT + chroma upsample + YCbCr->RGB, uint8 HWC out.
hipError_t launch_idct_color(const BatchDev& b, hipStream_t s);

// Known-answer hooks: run exactly the device arithmetic of stage 3 on caller data.
hipError_t launch_test_idct(const int32_t* in_zz, int32_t* out, int nblocks, hipStream_t s);
hipError_t launch_test_color(const int32_t* ycc, uint8_t* rgb, int n, hipStream_t s);

}  // namespace jd
