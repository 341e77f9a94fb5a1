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

// Region words per walk bit, bounded from the image's Huffman tables (any table may meet any block
// in a speculative walk, so minima run over every component's tables).  A block is one record word
// plus half a word per emitted entry.  It takes its DC symbol (>= min_dc bits: code + magnitude) and
// either ends with an EOB (>= min_eob) after E entries (>= mbe bits each: code + >= 1 magnitude bit),
// or reaches coefficient 63 without one, which takes >= 4 AC symbols (a symbol advances the index
// by at most 16): E entries and 4 - E other symbols (ZRL and other size-0 codes, >= min_ne).  The
// words-per-bit ratio of a block shape, (2 + E) / (2 bits), is monotonic in E, so its maximum is at
// E = 0, at E = 4 or at E -> infinity (1 / (2 mbe)); the divisor is the largest d in [2, 8] with
// d x ratio <= 1 for all of them (2 holds for any tables: every item takes >= 2 bits).
uint32_t region_divisor(const ParsedJpeg& pj) {
#ifdef JD_RW_DIV_FORCE
    return JD_RW_DIV_FORCE;  // experiment builds: the table-free bound (2) for A/B
#endif
    const jd_header& h = pj.hdr;
    constexpr uint32_t kInf = 1u << 20;
    uint32_t min_dc = kInf, min_eob = kInf, mbe = kInf, min_ne = kInf;
    for (int c = 0; c < h.ncomp; c++) {
        const HuffSpec& dc = pj.dc[pj.td[c]];
        const HuffSpec& ac = pj.ac[pj.ta[c]];
        for (int l = 1, k = 0; l <= 16; l++)
            for (int i = 0; i < dc.counts[l] && k < dc.nvals; i++, k++) min_dc = std::min<uint32_t>(min_dc, uint32_t(l) + dc.vals[k]);
        for (int l = 1, k = 0; l <= 16; l++)
            for (int i = 0; i < ac.counts[l] && k < ac.nvals; i++, k++) {
                const uint32_t sym = ac.vals[k], sz = sym & 15u;
                if (sym == 0) min_eob = std::min<uint32_t>(min_eob, uint32_t(l));
                else if (sz) mbe = std::min<uint32_t>(mbe, uint32_t(l) + sz);
                else min_ne = std::min<uint32_t>(min_ne, uint32_t(l));
            }
    }
    if (min_dc == kInf) return 2u;
    // candidate block shapes as words-per-bit fractions num / den
    uint64_t num[8], den[8];
    int n = 0;
    if (min_eob < kInf) num[n] = 1, den[n++] = uint64_t(min_dc) + min_eob;
    if (mbe < kInf) num[n] = 1, den[n++] = 2ull * mbe;
    for (uint32_t e = 0; e <= 4; e++) {  // no EOB: e entries and 4 - e other symbols
        if ((e > 0 && mbe == kInf) || (e < 4 && min_ne == kInf)) continue;
        num[n] = 2 + e;
        den[n++] = 2ull * (uint64_t(min_dc) + uint64_t(e) * (e ? mbe : 0u) + uint64_t(4 - e) * (e < 4 ? min_ne : 0u));
    }
    uint32_t d = 8;
    for (int i = 0; i < n; i++)
        while (d > 2 && uint64_t(d) * num[i] > den[i]) d--;
    return d;
}

// Fills d (everything but the piece ranges) for item it; pure function of the header + bases.
void fill_desc(const ParsedJpeg& pj, const jd_item& item, uint64_t dev_addr, uint64_t out_addr, const PlanImg& pi,
               ImgDesc& d, bool worst) {
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
    const RegionSizing rs = region_sizing(pj, worst);
    d.rw_div = rs.div;
    d.rw_slack = rs.slack;
}


}  // namespace jd
