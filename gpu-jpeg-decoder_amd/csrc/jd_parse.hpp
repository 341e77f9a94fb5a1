// jd_parse.hpp — host-side marker parser and Huffman-table builder.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "jd_internal.hpp"

namespace jd {

struct HuffSpec {
    bool present = false;
    uint8_t counts[17] = {};  // counts[l] = codes of length l, l = 1..16
    uint8_t vals[256] = {};
    int nvals = 0;
};

struct ParsedJpeg {
    jd_header hdr{};
    int cid[4] = {};
    int td[4] = {}, ta[4] = {};  // DC / AC table selectors per (scan == frame) component
    HuffSpec dc[4], ac[4];
    uint16_t q[4][64] = {};      // zig-zag order, as stored in DQT
    bool qp[4] = {};
    uint64_t hdc[4] = {}, hac[4] = {};  // hash_huff of each component's DC / AC table (parse workers)
};

// Walks SOI .. SOS.  Replaces the reference's extract() marker loop
// (cpp-decoder/src/parser.cpp:24-103, cuda-decoder/src/parser.cu:360-471), generalised to
// multi-table DQT/DHT segments, SOF/SOS table selectors, DRI and any integral Hi/Vi sampling.
jd_status parse_jpeg(const uint8_t* d, size_t n, ParsedJpeg* out);

// Canonical code assignment (the reference's leftmost-first tree insertion,
// cpp-decoder/src/huffmanTree.cpp:20-68) flattened into a LUT + canonical limits.
// Returns false for an over-subscribed table.
// AC entries carry the following symbol when both fit the index (jd_internal.hpp, HuffLut).
bool build_lut(const HuffSpec& h, bool is_dc, HuffLut* lut);

// Content hash of a table (for de-duplication across a batch / across calls).
uint64_t hash_huff(const HuffSpec& h, bool is_dc);

}  // namespace jd
