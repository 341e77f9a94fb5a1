// jd_plan.hpp — the host plan's pure functions (no HIP): geometry of a parsed image, its
// AC-entry reservation and its device descriptor.  jd_runtime.cpp's build_plan calls them; the
// sanitizer harness (tools/jd_fuzz_host.cpp, ASan + UBSan) drives them on mutated files.
#pragma once

#include <stdint.h>

#include <algorithm>

#include "jd.h"
#include "jd_internal.hpp"
#include "jd_parse.hpp"

namespace jd {

// Sampling layout of an image for k_idct_color's specialised instances (jd_kernels.hip TMode):
// 1 = 4:2:0 (Y 2x2), 2 = 4:2:2 (Y 2x1), 3 = 4:4:4, each with one Cb and one Cr block per MCU in
// frame order; 0 = anything else (generic instance).
uint32_t image_mode(const ImgDesc& d);

// AC-entry region words of one image: its pieces' regions (jd_internal.hpp
// region_words: at most ECS bits / 2 + kRegionSlack + 8 per piece slot) and spare regions for the
// re-walks of pieces whose speculative start was wrong (~0.6 % of full-size pieces; with short
// pieces, up to every piece).
inline uint64_t piece_slots(uint64_t ecs_bytes, uint32_t nseg, uint32_t piece_bits) {
    return (ecs_bytes * 8 + piece_bits - 1) / piece_bits + nseg;
}
inline uint64_t entry_words(uint64_t ecs_bytes, uint32_t nseg, uint32_t piece_bits, int64_t spare_pieces = -1,
                            uint32_t div = 2u, uint32_t slack = kRegionSlack) {
    const uint64_t bits = ecs_bytes * 8, slots = piece_slots(ecs_bytes, nseg, piece_bits);
    uint64_t spare = (piece_bits >= bits) ? 0 : (piece_bits >= 4096 ? slots / 16 + 8 : slots);
    if (spare_pieces >= 0) spare = uint64_t(spare_pieces);  // JD_SPARE_PIECES (tests: in-place re-walks)
    return bits / div + 4 + slots * (slack + 8) +
           spare * region_words(uint32_t(std::min<uint64_t>(piece_bits, bits)), div, slack);
}
// Fewest walk bits per region word any block or entry of the image can take, from its Huffman
// tables (in [2, 8]; 2 holds for any tables): the divisor of its piece regions (region_words).
uint32_t region_divisor(const ParsedJpeg& pj);
// The divisor and slack an image's regions are planned with: the worst case (region_divisor,
// kRegionSlack: no valid stream can fill them), or the optimistic default (kOptRegionDiv and the
// image's largest MCU: a denser stream overflows, is flagged and is decoded again with the worst case).
struct RegionSizing {
    uint32_t div, slack;
};
inline RegionSizing region_sizing(const ParsedJpeg& pj, bool worst) {
    if (worst) return {region_divisor(pj), kRegionSlack};
    return {std::max(region_divisor(pj), kOptRegionDiv), opt_region_slack(uint32_t(pj.hdr.blocks_per_mcu))};
}
inline uint32_t image_segments(const jd_header& h) {
    const uint64_t nmcu = uint64_t(h.mcux) * h.mcuy;
    return h.restart_interval ? uint32_t((nmcu + h.restart_interval - 1) / h.restart_interval) : 1u;
}

// Piece size of a batch of ecs_bits entropy-coded bits (jd_runtime.cpp build_plan): kPieceBits,
// halved (down to kMinPieceBits) while the batch would have fewer than kPieceTarget pieces.  It
// grows with the batch, so an image's own bits give a lower bound for any batch holding it.
inline uint32_t adaptive_piece_bits(uint64_t ecs_bits, uint32_t pmin = kMinPieceBits) {
    uint32_t p = kPieceBits;
    while (p > pmin && ecs_bits / p < kPieceTarget) p >>= 1;
    return p;
}

// An image's AC-entry offsets are image-relative 32-bit values in 16-bit slot units
// (BlockInfo::entry_start, k_gather's running offset): its reservation must stay below 2^31
// words, else the plan rejects it with JD_ERR_CAPACITY.  The reservation is made at the batch's
// piece size, which lies between the shortest pieces any batch holding the image can get
// (pmin: adaptive_piece_bits of its own bits) and pmax (kPieceBits; a forced size gives pmin =
// pmax), always a power-of-two multiple of pmin.  entry_words is not monotonic in the piece size
// (the spare regions grow with it, the per-piece slack shrinks), so every candidate is checked.
// div: the image's region divisor.
constexpr uint64_t kMaxImageEntryWords = 0x7FFFFF00ull;
inline bool image_fits(uint64_t ecs_bytes, const jd_header& h, uint32_t pmin, uint32_t pmax, int64_t spare_pieces = -1,
                       uint32_t div = 2u, uint32_t slack = kRegionSlack) {
    for (uint64_t p = pmin;; p *= 2) {
        if (entry_words(ecs_bytes, image_segments(h), uint32_t(p), spare_pieces, div, slack) > kMaxImageEntryWords) return false;
        if (p >= pmax) return true;
    }
}

// Per image of the plan: what the sequential pass decides (table set, quant slots, bases).
struct PlanImg {
    int item, ts;
    uint16_t qslot[3];
    uint64_t block_base, entry_base, comp;
    uint32_t seg_base, nseg, chunk_base, nchunks;
};

// Fills d (everything but the piece ranges) for item it; pure function of the header + bases
// (worst: worst-case region sizing, region_sizing).
void fill_desc(const ParsedJpeg& pj, const jd_item& item, uint64_t dev_addr, uint64_t out_addr, const PlanImg& pi,
               ImgDesc& d, bool worst);

}  // namespace jd
