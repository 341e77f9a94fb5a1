// jd_plan.cpp — the host plan's pure functions (jd_plan.hpp).
#include "jd_plan.hpp"

#include <string.h>

namespace jd {

// Sampling layout of an image for k_idct_color's specialised instances (jd_kernels.hip TMode):
// 1 = 4:2:0 (Y 2x2), 2 = 4:2:2 (Y 2x1), 3 = 4:4:4, each with one Cb and one Cr block per MCU in
// frame order; 0 = anything else (generic instance).
uint32_t image_mode(const ImgDesc& d) {
    if (d.ncomp != 3 || d.h[1] != 1 || d.v[1] != 1 || d.h[2] != 1 || d.v[2] != 1) return 0;
    if (d.h[0] == 2 && d.v[0] == 2) return 1;
    if (d.h[0] == 2 && d.v[0] == 1) return 2;
    if (d.h[0] == 1 && d.v[0] == 1) return 3;
    return 0;
}

// Fills d (everything but the piece ranges) for item it; pure function of the header + bases.
void fill_desc(const ParsedJpeg& pj, const jd_item& item, uint64_t dev_addr, uint64_t out_addr, const PlanImg& pi,
               ImgDesc& d) {
    const jd_header& h = pj.hdr;
    memset(&d, 0, sizeof(d));
    d.jpeg = dev_addr;
    d.rgb = out_addr;
    d.len = uint32_t(item.len);
    d.ecs_off = uint32_t(h.ecs_offset);
    d.width = uint32_t(h.width);
    d.height = uint32_t(h.height);
    d.mcux = uint32_t(h.mcux);
    d.mcuy = uint32_t(h.mcuy);
    d.ncomp = uint32_t(h.ncomp);
    d.hmax = uint32_t(h.hmax);
    d.vmax = uint32_t(h.vmax);
    d.bpm = uint32_t(h.blocks_per_mcu);
    uint32_t pat = 0, b = 0;
    for (int c = 0; c < h.ncomp; c++) {
        d.h[c] = uint8_t(h.h[c]);
        d.v[c] = uint8_t(h.v[c]);
        d.comp_block0[c] = uint8_t(b);
        for (int j = 0; j < h.h[c] * h.v[c]; j++, b++) pat |= uint32_t(c) << (2 * b);
        d.qslot[c] = pi.qslot[c];
    }
    {  // k_idct_color's fast-IDCT range test: |c| <= 2^(k-1) keeps |c * step| < 2^15 (int16)
        uint32_t qmax = 1;
        for (int c = 0; c < h.ncomp; c++)
            for (int k = 0; k < 64; k++) qmax = std::max<uint32_t>(qmax, pj.q[h.tq[c]][k]);
        uint32_t k = 1;
        while (k < 16 && (uint64_t(1) << k) * qmax < 32768) k++;  // largest k: 2^(k-1) * qmax < 2^15
        const uint32_t lo = (0xFFFFu << k) & 0xFFFFu;
        d.qmask = lo | (lo << 16);
    }
    d.block_pattern = pat;
    d.restart_interval = uint32_t(h.restart_interval);
    d.nseg = pi.nseg;
    d.seg_base = pi.seg_base;
    d.block_base = pi.block_base;
    d.tableset = uint32_t(pi.ts);
    {  // IDCT/colour tiles: one wave, one lane per block: the most blocks <= 64 over 1 or 2 MCU rows
        uint32_t lw = 0, lh = 0;
        while ((8u << lw) < 8u * d.hmax) lw++;
        while ((8u << lh) < 8u * d.vmax) lh++;
        d.lg_mw = 3 + lw;
        d.lg_mh = 3 + lh;
        // a run of consecutive MCUs of one MCU row (k_idct_color's DC prediction scans it in order)
        d.tile_mcus = std::max(1u, uint32_t(kTileMaxBlocks) / d.bpm);
        d.tile_mrows = 1;
        d.tiles_x = (d.mcux + d.tile_mcus - 1) / d.tile_mcus;
        d.tiles_y = (d.mcuy + d.tile_mrows - 1) / d.tile_mrows;
        for (int c = 0; c < h.ncomp; c++) {
            uint32_t sx = 0, sy = 0;
            while ((uint32_t(h.h[c]) << sx) < d.hmax) sx++;
            while ((uint32_t(h.v[c]) << sy) < d.vmax) sy++;
            d.shx[c] = uint8_t(sx);
            d.shy[c] = uint8_t(sy);
        }
    }
    d.nchunks = pi.nchunks;  // scan chunks over [align16(file + ecs_off), file + len)
    d.chunk_base = pi.chunk_base;
    d.comp = pi.comp;  // offset for now; rebased onto the pool in launch_batch
}


}  // namespace jd
