// jd_fuzz_host.cpp — host-side sanitizer harness (the reference's only memory
// checking is a valgrind log; here the parser and the host plan run under ASan + UBSan).
//
// Built by `make -C gpu-jpeg-decoder_amd fuzz_host_asan` (-fsanitize=address,undefined, no HIP).
// Input: a file of records [u32 little-endian length][bytes]; every record is copied into an
// exactly-sized heap buffer, so a read past the file's end is an ASan report.  Per record it runs
// what the runtime's host side runs on a batch item before any kernel:
//   parse_jpeg (marker walk, jd_parse.cpp), hash_huff + build_lut of every component's tables
//   (the LUT cache, jd_runtime.cpp lut_id), image_fits / entry_words / piece_slots (the AC-entry
//   reservation) and fill_desc + image_mode (the device descriptor, jd_plan.cpp),
// and prints one line: parse status, then (status 0) width height ncomp mcux mcuy blocks_per_mcu
// restart_interval ecs_offset plan mode tiles_x tiles_y rw_div.  `plan` is 0, or JD_ERR_CORRUPT for a table
// the LUT builder rejects, or JD_ERR_CAPACITY for an image beyond the 32-bit entry offsets.
// Any sanitizer finding aborts the process with a non-zero status (-fno-sanitize-recover=all).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "jd_parse.hpp"
#include "jd_plan.hpp"

using namespace jd;

static int plan_one(const uint8_t* buf, size_t len, const ParsedJpeg& pj, ImgDesc& d) {
    const jd_header& h = pj.hdr;
    HuffLut* lut = new HuffLut;
    bool ok = true;
    for (int c = 0; c < h.ncomp && ok; c++) {
        (void)hash_huff(pj.dc[pj.td[c]], true);
        (void)hash_huff(pj.ac[pj.ta[c]], false);
        ok = build_lut(pj.dc[pj.td[c]], true, lut) && build_lut(pj.ac[pj.ta[c]], false, lut);
    }
    delete lut;
    if (!ok) return JD_ERR_CORRUPT;
    const uint64_t ecs = len - h.ecs_offset;
    const RegionSizing opt = region_sizing(pj, false), worst = region_sizing(pj, true);
    if (!image_fits(ecs, h, adaptive_piece_bits(ecs * 8), kPieceBits, -1, worst.div, worst.slack)) return JD_ERR_CAPACITY;
    (void)image_fits(ecs, h, adaptive_piece_bits(ecs * 8), kPieceBits, -1, opt.div, opt.slack);
    PlanImg pi{};
    pi.nseg = image_segments(h);
    pi.nchunks = uint32_t((len - (h.ecs_offset & ~uint64_t(15)) + kScanChunk - 1) / kScanChunk);
    (void)piece_slots(ecs, pi.nseg, kPieceBits);
    (void)entry_words(ecs, pi.nseg, kPieceBits, -1, opt.div, opt.slack);
    jd_item item{buf, nullptr, len, nullptr};
    fill_desc(pj, item, 0x100000000ull, 0x200000000ull, pi, d, false);  // the default (optimistic) plan
    fill_desc(pj, item, 0x100000000ull, 0x200000000ull, pi, d, true);   // the retry's: reported (rw_div)
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s records.bin\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> all;
    uint8_t tmp[1 << 16];
    size_t got;
    while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) all.insert(all.end(), tmp, tmp + got);
    fclose(f);
    size_t off = 0;
    while (off + 4 <= all.size()) {
        const uint32_t len = uint32_t(all[off]) | uint32_t(all[off + 1]) << 8 | uint32_t(all[off + 2]) << 16 |
                             uint32_t(all[off + 3]) << 24;
        off += 4;
        if (off + len > all.size()) return 3;
        uint8_t* buf = static_cast<uint8_t*>(malloc(len ? len : 1));  // exactly sized: over-reads are reported
        if (len) memcpy(buf, all.data() + off, len);
        off += len;
        ParsedJpeg* pj = new ParsedJpeg();
        const jd_status st = parse_jpeg(buf, len, pj);
        if (st != JD_OK) {
            printf("%d\n", int(st));
        } else {
            const jd_header& h = pj->hdr;
            ImgDesc d;
            memset(&d, 0, sizeof(d));
            const int plan = plan_one(buf, len, *pj, d);
            printf("0 %d %d %d %d %d %d %d %llu %d %u %u %u %u\n", h.width, h.height, h.ncomp, h.mcux, h.mcuy,
                   h.blocks_per_mcu, h.restart_interval, (unsigned long long)h.ecs_offset, plan,
                   plan ? 0u : image_mode(d), d.tiles_x, d.tiles_y, plan ? 0u : d.rw_div);
        }
        delete pj;
        free(buf);
    }
    return 0;
}
