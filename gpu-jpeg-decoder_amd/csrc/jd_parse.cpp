// jd_parse.cpp — host-side marker parser and Huffman LUT builder.
//
// The reference walks a fixed marker sequence (APP0, DQT, DQT, SOF0, 4x DHT, SOS:
// cpp-decoder/src/parser.cpp:31-101) and maps "first DQT -> Y, second -> chroma" and DHT ids
// 0x00/0x01/0x10/0x11 positionally.  For the files the reference accepts that is the same as
// honouring the SOF Tq and SOS Td/Ta selectors, which is what this parser does; it also accepts
// any marker order, multi-table segments, DRI, fill bytes and 1-component frames, and rejects
// what the GPU path does not implement with JD_ERR_UNSUPPORTED instead of decoding garbage.
#include "jd_parse.hpp"

#include <algorithm>

#include <string.h>

namespace jd {

static inline uint32_t be16(const uint8_t* p) { return (uint32_t(p[0]) << 8) | p[1]; }

jd_status parse_jpeg(const uint8_t* d, size_t n, ParsedJpeg* out) {
    *out = ParsedJpeg();
    if (!d || n < 4) return JD_ERR_INVALID_ARG;
    if (d[0] != 0xFF || d[1] != 0xD8) return JD_ERR_CORRUPT;
    jd_header& h = out->hdr;
    size_t p = 2;
    bool have_sof = false;
    for (;;) {
        if (p + 2 > n) return JD_ERR_TRUNCATED;
        if (d[p] != 0xFF) return JD_ERR_CORRUPT;
        while (p + 1 < n && d[p + 1] == 0xFF) p++;
        if (p + 2 > n) return JD_ERR_TRUNCATED;
        const uint8_t m = d[p + 1];
        p += 2;
        if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // standalone markers
        if (m == 0xD9) return JD_ERR_CORRUPT;                               // EOI before SOS
        if (p + 2 > n) return JD_ERR_TRUNCATED;
        const size_t L = be16(d + p);
        if (L < 2 || p + L > n) return JD_ERR_TRUNCATED;
        const uint8_t* s = d + p + 2;
        const size_t sl = L - 2;
        switch (m) {
            case 0xC0:
            case 0xC1: {  // baseline / extended sequential, Huffman
                if (sl < 6) return JD_ERR_CORRUPT;
                if (s[0] != 8) return JD_ERR_UNSUPPORTED;  // 12-bit samples
                h.height = int(be16(s + 1));
                h.width = int(be16(s + 3));
                const int nc = s[5];
                if (nc != 1 && nc != 3) return JD_ERR_UNSUPPORTED;  // CMYK / 2-component
                if (sl < 6 + 3 * size_t(nc)) return JD_ERR_CORRUPT;
                if (h.width == 0 || h.height == 0) return JD_ERR_UNSUPPORTED;  // DNL
                h.ncomp = nc;
                for (int c = 0; c < nc; c++) {
                    out->cid[c] = s[6 + 3 * c];
                    h.h[c] = s[7 + 3 * c] >> 4;
                    h.v[c] = s[7 + 3 * c] & 15;
                    h.tq[c] = s[8 + 3 * c];
                    if (h.h[c] < 1 || h.h[c] > 4 || h.v[c] < 1 || h.v[c] > 4 || h.tq[c] > 3)
                        return JD_ERR_CORRUPT;
                }
                have_sof = true;
                break;
            }
            case 0xC4: {  // DHT
                size_t q = 0;
                while (q < sl) {
                    if (q + 17 > sl) return JD_ERR_CORRUPT;
                    const int tc = s[q] >> 4, th = s[q] & 15;
                    if (tc > 1 || th > 3) return JD_ERR_CORRUPT;
                    HuffSpec& t = tc ? out->ac[th] : out->dc[th];
                    t = HuffSpec();
                    int tot = 0;
                    for (int l = 1; l <= 16; l++) tot += (t.counts[l] = s[q + l]);
                    if (tot > 256 || q + 17 + tot > sl) return JD_ERR_CORRUPT;
                    memcpy(t.vals, s + q + 17, size_t(tot));
                    t.nvals = tot;
                    t.present = true;
                    q += 17 + size_t(tot);
                }
                break;
            }
            case 0xDB: {  // DQT
                size_t q = 0;
                while (q < sl) {
                    const int pq = s[q] >> 4, tq = s[q] & 15;
                    if (pq > 1 || tq > 3) return JD_ERR_CORRUPT;
                    if (q + 1 + 64 * size_t(pq + 1) > sl) return JD_ERR_CORRUPT;
                    for (int k = 0; k < 64; k++)
                        out->q[tq][k] = uint16_t(pq ? be16(s + q + 1 + 2 * k) : s[q + 1 + k]);
                    out->qp[tq] = true;
                    q += 1 + 64 * size_t(pq + 1);
                }
                break;
            }
            case 0xDD:  // DRI
                if (sl < 2) return JD_ERR_CORRUPT;
                h.restart_interval = int(be16(s));
                break;
            case 0xDA: {  // SOS
                if (!have_sof || sl < 1) return JD_ERR_CORRUPT;
                const int ns = s[0];
                if (sl < 4 + 2 * size_t(ns)) return JD_ERR_CORRUPT;
                if (ns != h.ncomp) return JD_ERR_UNSUPPORTED;  // multi-scan sequential
                for (int i = 0; i < ns; i++) {
                    if (s[1 + 2 * i] != out->cid[i]) return JD_ERR_UNSUPPORTED;
                    out->td[i] = s[2 + 2 * i] >> 4;
                    out->ta[i] = s[2 + 2 * i] & 15;
                    if (out->td[i] > 3 || out->ta[i] > 3) return JD_ERR_CORRUPT;
                    if (!out->dc[out->td[i]].present || !out->ac[out->ta[i]].present)
                        return JD_ERR_CORRUPT;
                    if (!out->qp[h.tq[i]]) return JD_ERR_CORRUPT;
                }
                if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0)
                    return JD_ERR_UNSUPPORTED;  // spectral selection / approximation
                h.ecs_offset = p + L;
                goto done;
            }
            default:
                if (m >= 0xC2 && m <= 0xCF && m != 0xC8 && m != 0xCC)
                    return JD_ERR_UNSUPPORTED;  // progressive, lossless, arithmetic
                break;                          // APPn, COM, DNL, ...: skipped by length
        }
        p += L;
    }
done:
    if (h.ncomp == 1) {
        h.h[0] = h.v[0] = 1;  // non-interleaved scan: MCU = one block
        h.hmax = h.vmax = 1;
    } else {
        h.hmax = h.vmax = 1;
        for (int c = 0; c < h.ncomp; c++) {
            if (h.h[c] > h.hmax) h.hmax = h.h[c];
            if (h.v[c] > h.vmax) h.vmax = h.v[c];
        }
        for (int c = 0; c < h.ncomp; c++)
            if (h.h[c] == 3 || h.v[c] == 3 || h.hmax % h.h[c] || h.vmax % h.v[c]) return JD_ERR_UNSUPPORTED;
    }
    h.mcux = (h.width + 8 * h.hmax - 1) / (8 * h.hmax);
    h.mcuy = (h.height + 8 * h.vmax - 1) / (8 * h.vmax);
    h.blocks_per_mcu = 0;
    for (int c = 0; c < h.ncomp; c++) h.blocks_per_mcu += h.h[c] * h.v[c];
    if (h.blocks_per_mcu > 10) return JD_ERR_UNSUPPORTED;
    if (h.ncomp == 1) {
        h.subsampling = JD_SS_GRAY;
    } else if (h.h[1] == h.h[2] && h.v[1] == h.v[2] && h.h[1] == 1 && h.v[1] == 1) {
        if (h.hmax == 1 && h.vmax == 1) h.subsampling = JD_SS_444;
        else if (h.hmax == 2 && h.vmax == 1) h.subsampling = JD_SS_422;
        else if (h.hmax == 2 && h.vmax == 2) h.subsampling = JD_SS_420;
        else if (h.hmax == 1 && h.vmax == 2) h.subsampling = JD_SS_440;
        else h.subsampling = JD_SS_OTHER;
    } else {
        h.subsampling = JD_SS_OTHER;
    }
    return JD_OK;
}


bool build_lut(const HuffSpec& h, bool is_dc, HuffLut* lut) {
    memset(lut, 0, sizeof(*lut));
    int code = 0, k = 0;
    int codes[256];
    int lens[256];
    for (int l = 1; l <= 16; l++) {
        lut->base[l] = k - code;  // valptr[l] - mincode[l]
        for (int i = 0; i < h.counts[l]; i++) {
            if (k >= 256) return false;
            codes[k] = code++;
            lens[k] = l;
            k++;
        }
        if (code > (1 << l)) return false;  // over-subscribed
        lut->lim[l] = uint32_t(code) << (16 - l);
        code <<= 1;
    }
    lut->lim[17] = 0xFFFFFFFFu;  // sentinel: unmatched 16-bit prefix -> corrupt
    lut->lim[19] = is_dc ? 1u : 0u;
    for (int i = 0; i < h.nvals; i++) lut->vals[i] = h.vals[i];
    // code length and symbol of every index whose top bits are a code of <= kLutBits bits
    uint8_t len_of[kLutSize] = {}, sym_of[kLutSize] = {};
    for (int i = 0; i < k; i++) {
        const int l = lens[i];
        if (l > kLutBits) continue;
        const int shift = kLutBits - l;
        const int first = codes[i] << shift, last = ((codes[i] + 1) << shift) - 1;
        for (int idx = first; idx <= last; idx++) {
            len_of[idx] = uint8_t(l);
            sym_of[idx] = h.vals[i];
        }
    }
    // EXTEND (utils/stream.cpp:44-52) of the sz bits of idx that follow its first `at` bits
    auto value_at = [](uint32_t idx, uint32_t at, uint32_t sz) {
        const uint32_t mag = (idx >> (uint32_t(kLutBits) - at - sz)) & ((1u << sz) - 1u);
        return sz == 0 ? 0 : (mag >> (sz - 1)) ? int(mag) : int(mag) - int((1u << sz) - 1u);
    };
    for (uint32_t idx = 0; idx < uint32_t(kLutSize); idx++) {
        uint32_t& lo = lut->fast[2 * idx];
        uint32_t& hi = lut->fast[2 * idx + 1];
        const uint32_t l1 = len_of[idx], sym1 = sym_of[idx];
        const uint32_t e1 = l1 ? lut_entry(l1, sym1, is_dc) : 0u;  // 0: longer code (or unrepresentable)
        const uint32_t sz1 = is_dc ? sym1 : (sym1 & 15u);
        if (e1 == 0 || (is_dc ? sz1 > 11u : sz1 >= 10u)) {  // rare: the walks' generic branch
            // hi bits 0..11 (the width w1 and the first symbol's advance) are clear, so the common
            // path reads width 0 and advance 0 (a no-op).  The pair fields (adv2 12..18, L12
            // 19..22, v2 23..31) do hold the rare entry's bits; they are inert because lo carries
            // neither kLoPair nor kLoE2, which gate every use of them in the walks.
            lo = kLoRare;
            hi = e1 << kRareShift;
            static_assert((kLoRare & (kLoPair | kLoE2)) == 0u, "a rare lo word never gates the pair fields");
            continue;
        }
        const uint32_t L1 = l1 + sz1, adv1 = (e1 >> 8) & 127u;
        uint32_t w1 = 0;
        int32_t m1;
        if (L1 <= uint32_t(kLutBits)) {
            m1 = -value_at(idx, l1, sz1);
        } else {
            w1 = sz1;
            m1 = int32_t((1u << sz1) - 1u);
        }
        lo = ((32u - L1) & 31u) | (L1 << kLoL1Shift) | (is_dc ? kLoDc : 0u) | ((!is_dc && sz1) ? kLoE1 : 0u) |
             (uint32_t(m1) << 16);
        hi = w1 | (adv1 << 5);
        // pair: the following AC symbol, when the first is not EOB and both lie within the index
        if (is_dc || adv1 == 64u || L1 >= uint32_t(kLutBits)) continue;
        const uint32_t idx2 = (idx << L1) & (kLutSize - 1), l2 = len_of[idx2], sym2 = sym_of[idx2];
        if (l2 == 0) continue;
        const uint32_t sz2 = sym2 & 15u, L2 = l2 + sz2;
        if (L2 > uint32_t(kLutBits) - L1) continue;  // needs bits beyond the index
        const uint32_t adv2 = sym2 == 0u ? 64u : (sym2 >> 4) + 1u;
        const int v2 = value_at(idx, L1 + l2, sz2);
        lo |= kLoPair | (sz2 ? kLoE2 : 0u);
        hi |= (adv2 << 12) | ((L1 + L2) << 19) | ((uint32_t(v2) & 511u) << 23);  // the pair's length
    }
    return true;
}

uint64_t hash_huff(const HuffSpec& h, bool is_dc) {
    // 8 bytes per round (tables are hashed per image per call: this runs in the parse workers)
    uint64_t x = 0x9e3779b97f4a7c15ull ^ (is_dc ? 1u : 2u) ^ (uint64_t(h.nvals) << 8);
    auto mix = [&](uint64_t w) {
        x ^= w;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 32;
    };
    uint64_t w[2];
    memcpy(w, h.counts + 1, 16);
    mix(w[0]);
    mix(w[1]);
    const int n = h.nvals;
    for (int i = 0; i < n; i += 8) {
        uint64_t v = 0;
        memcpy(&v, h.vals + i, size_t(std::min(8, n - i)));
        mix(v);
    }
    return x;
}

}  // namespace jd
