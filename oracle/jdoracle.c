/*
 * jdoracle.c — CPU restatement of the reference decoder (TEST INFRASTRUCTURE ONLY).
 *
 * This is the checker for the GPU decode path, never part of it: the product library
 * (gpu-jpeg-decoder_amd/) does not link or call anything here.  Only tests/, the smoke() checker in
 * __graft_entry__.py and bench.py's cpu_baseline leg load liboracle.so.
 *
 * It restates, function by function, the reference's CPU decoder (/root/reference/cpp-decoder):
 *   bit reader / EXTEND        utils/stream.cpp:8-52
 *   marker walk                src/parser.cpp:24-103
 *   Huffman code assignment    src/huffmanTree.cpp:4-110 (tree walk == canonical decode, F.2.2.3)
 *   block decode + dequant     src/parser.cpp:105-142
 *   zig-zag + integer IDCT     src/idct.cpp:7-133, src/idct.h:3-9
 *   MCU raster + crop          src/parser.cpp:144-195
 *   YCbCr -> RGB               utils/color.cpp:4-19
 * and extends it (semantics in DESIGN.md §3, not pinned by the reference) to: any Hi/Vi sampling
 * with replicate chroma upsampling, DRI/RSTn restart intervals (byte-align, predictor reset,
 * marker skip), SOS/SOF table selectors, multi-table DQT/DHT segments and 1-component frames.
 */
#define _POSIX_C_SOURCE 200809L
#include "jdoracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------------------------ */
/* tables                                                                                      */
/* ------------------------------------------------------------------------------------------ */

/* natural (row-major) position -> zig-zag index; src/idct.cpp:8-16 */
static const int kZigzagOfNatural[64] = {
    0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42, 3,  8,  12, 17, 25, 30,
    41, 43, 9,  11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38,
    46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

typedef struct {
    int present;
    uint8_t counts[17]; /* counts[l]: number of codes of length l, l = 1..16 */
    uint8_t vals[256];
    int nvals;
    int32_t mincode[17], maxcode[18], valptr[17];
} huff_t;

typedef struct {
    jdo_info info;
    int cid[4];
    int td[4], ta[4];
    int32_t q[4][64]; /* zig-zag order as stored in DQT */
    int qpresent[4];
    huff_t dc[4], ac[4];
} img_t;

static uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

/* Canonical code assignment.  The reference inserts leaves leftmost-first in order of increasing
 * length (huffmanTree.cpp:20-68), which is exactly the canonical assignment of JPEG Annex C. */
static int huff_build(huff_t* h) {
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        h->valptr[l] = k;
        h->mincode[l] = code;
        code += h->counts[l];
        k += h->counts[l];
        h->maxcode[l] = h->counts[l] ? code - 1 : -1;
        if (code > (1 << l)) return JDO_ERR_CORRUPT; /* over-subscribed */
        code <<= 1;
    }
    h->maxcode[17] = 0x7fffffff;
    h->present = 1;
    return JDO_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* marker walk (restates parser.cpp:24-103, generalised)                                       */
/* ------------------------------------------------------------------------------------------ */

static int parse(const uint8_t* d, size_t n, img_t* im) {
    memset(im, 0, sizeof(*im));
    if (!d || n < 4) return JDO_ERR_INVALID_ARG;
    if (d[0] != 0xFF || d[1] != 0xD8) return JDO_ERR_CORRUPT;
    size_t p = 2;
    int have_sof = 0;
    for (;;) {
        if (p + 2 > n) return JDO_ERR_TRUNCATED;
        if (d[p] != 0xFF) return JDO_ERR_CORRUPT;
        while (p + 1 < n && d[p + 1] == 0xFF) p++; /* fill bytes */
        if (p + 2 > n) return JDO_ERR_TRUNCATED;
        uint8_t m = d[p + 1];
        p += 2;
        if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
        if (m == 0xD9) return JDO_ERR_CORRUPT; /* EOI before SOS */
        if (p + 2 > n) return JDO_ERR_TRUNCATED;
        size_t L = be16(d + p);
        if (L < 2 || p + L > n) return JDO_ERR_TRUNCATED;
        const uint8_t* s = d + p + 2;
        size_t sl = L - 2;
        if (m == 0xC0 || m == 0xC1) { /* SOF0 / SOF1: Huffman sequential */
            if (sl < 6) return JDO_ERR_CORRUPT;
            if (s[0] != 8) return JDO_ERR_UNSUPPORTED;
            im->info.height = be16(s + 1);
            im->info.width = be16(s + 3);
            int nc = s[5];
            if (nc != 1 && nc != 3) return JDO_ERR_UNSUPPORTED;
            if (sl < 6 + 3 * (size_t)nc) return JDO_ERR_CORRUPT;
            if (im->info.width == 0 || im->info.height == 0) return JDO_ERR_UNSUPPORTED;
            im->info.ncomp = nc;
            for (int c = 0; c < nc; c++) {
                im->cid[c] = s[6 + 3 * c];
                im->info.h[c] = s[7 + 3 * c] >> 4;
                im->info.v[c] = s[7 + 3 * c] & 15;
                im->info.tq[c] = s[8 + 3 * c];
                if (im->info.h[c] < 1 || im->info.h[c] > 4 || im->info.v[c] < 1 ||
                    im->info.v[c] > 4 || im->info.tq[c] > 3)
                    return JDO_ERR_CORRUPT;
            }
            have_sof = 1;
        } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return JDO_ERR_UNSUPPORTED; /* progressive, lossless, arithmetic */
        } else if (m == 0xC4) { /* DHT, possibly several tables */
            size_t q = 0;
            while (q < sl) {
                if (q + 17 > sl) return JDO_ERR_CORRUPT;
                int tc = s[q] >> 4, th = s[q] & 15;
                if (tc > 1 || th > 3) return JDO_ERR_CORRUPT;
                huff_t* h = tc ? &im->ac[th] : &im->dc[th];
                memset(h, 0, sizeof(*h));
                int tot = 0;
                for (int l = 1; l <= 16; l++) {
                    h->counts[l] = s[q + l];
                    tot += s[q + l];
                }
                if (tot > 256 || q + 17 + tot > sl) return JDO_ERR_CORRUPT;
                memcpy(h->vals, s + q + 17, tot);
                h->nvals = tot;
                if (huff_build(h)) return JDO_ERR_CORRUPT;
                q += 17 + tot;
            }
        } else if (m == 0xDB) { /* DQT, possibly several tables */
            size_t q = 0;
            while (q < sl) {
                int pq = s[q] >> 4, tq = s[q] & 15;
                if (pq > 1 || tq > 3) return JDO_ERR_CORRUPT;
                if (q + 1 + 64 * (pq + 1) > sl) return JDO_ERR_CORRUPT;
                for (int k = 0; k < 64; k++)
                    im->q[tq][k] = pq ? be16(s + q + 1 + 2 * k) : s[q + 1 + k];
                im->qpresent[tq] = 1;
                q += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) { /* DRI */
            if (sl < 2) return JDO_ERR_CORRUPT;
            im->info.restart_interval = be16(s);
        } else if (m == 0xDA) { /* SOS */
            if (!have_sof) return JDO_ERR_CORRUPT;
            if (sl < 1) return JDO_ERR_CORRUPT;
            int ns = s[0];
            if (sl < 4 + 2 * (size_t)ns) return JDO_ERR_CORRUPT;
            if (ns != im->info.ncomp) return JDO_ERR_UNSUPPORTED; /* multi-scan sequential */
            for (int i = 0; i < ns; i++) {
                int cs = s[1 + 2 * i];
                if (cs != im->cid[i]) return JDO_ERR_UNSUPPORTED; /* scan order != frame order */
                im->td[i] = s[2 + 2 * i] >> 4;
                im->ta[i] = s[2 + 2 * i] & 15;
                if (im->td[i] > 3 || im->ta[i] > 3) return JDO_ERR_CORRUPT;
                if (!im->dc[im->td[i]].present || !im->ac[im->ta[i]].present)
                    return JDO_ERR_CORRUPT;
                if (!im->qpresent[im->info.tq[i]]) return JDO_ERR_CORRUPT;
            }
            int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahal = s[3 + 2 * ns];
            if (ss != 0 || se != 63 || ahal != 0) return JDO_ERR_UNSUPPORTED;
            im->info.ecs_offset = p + L;
            break;
        }
        /* APPn, COM, DNL, anything else: skipped by length */
        p += L;
    }
    jdo_info* f = &im->info;
    if (f->ncomp == 1) {
        f->h[0] = f->v[0] = 1; /* non-interleaved: MCU = one block */
        f->hmax = f->vmax = 1;
    } else {
        f->hmax = f->vmax = 1;
        for (int c = 0; c < f->ncomp; c++) {
            if (f->h[c] > f->hmax) f->hmax = f->h[c];
            if (f->v[c] > f->vmax) f->vmax = f->v[c];
        }
        /* sampling factors of 3 are rejected (the GPU path indexes samples with shifts) */
        for (int c = 0; c < f->ncomp; c++)
            if (f->h[c] == 3 || f->v[c] == 3 || f->hmax % f->h[c] || f->vmax % f->v[c])
                return JDO_ERR_UNSUPPORTED;
    }
    f->mcux = (f->width + 8 * f->hmax - 1) / (8 * f->hmax);
    f->mcuy = (f->height + 8 * f->vmax - 1) / (8 * f->vmax);
    f->blocks_per_mcu = 0;
    for (int c = 0; c < f->ncomp; c++) f->blocks_per_mcu += f->h[c] * f->v[c];
    if (f->blocks_per_mcu > 10) return JDO_ERR_UNSUPPORTED;
    return JDO_OK;
}

int jdo_parse(const uint8_t* jpeg, size_t len, jdo_info* info) {
    img_t im;
    int st = parse(jpeg, len, &im);
    if (info) *info = im.info;
    return st;
}

/* ------------------------------------------------------------------------------------------ */
/* bit reader (restates stream.cpp:8-52 plus byte un-stuffing from parser.cpp:84-98)           */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    const uint8_t* d;
    size_t n, pos;
    int acc, nacc, acc_fill;
    int at_marker; /* reader stopped in front of a marker (FF xx, xx != 00) */
    int overrun;   /* consumed a bit that lies beyond the segment's data */
} br_t;

/* next un-stuffed data byte, or a 0xFF fill byte once a marker / the end is reached */
static int br_fetch(br_t* b, int* is_fill) {
    if (!b->at_marker && b->pos < b->n) {
        uint8_t c = b->d[b->pos];
        if (c != 0xFF) {
            b->pos++;
            *is_fill = 0;
            return c;
        }
        if (b->pos + 1 < b->n && b->d[b->pos + 1] == 0x00) {
            b->pos += 2;
            *is_fill = 0;
            return 0xFF;
        }
        b->at_marker = 1; /* leave the marker in place */
    }
    *is_fill = 1;
    return 0xFF;
}

static inline int br_bit(br_t* b) {
    if (b->nacc == 0) {
        b->acc = br_fetch(b, &b->acc_fill);
        b->nacc = 8;
    }
    if (b->acc_fill) b->overrun = 1;
    b->nacc--;
    return (b->acc >> b->nacc) & 1;
}

static inline int br_bits(br_t* b, int n) { /* stream.cpp:15-22 */
    int v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | br_bit(b);
    return v;
}

/* EXTEND; stream.cpp:44-52 (s == 0 -> 0, the value the reference computes for ZRL/size-0) */
static inline int extend(int v, int s) {
    if (s == 0) return 0;
    int l = 1 << (s - 1);
    return v >= l ? v : v - ((l << 1) - 1);
}

/* huffmanTree.cpp:85-110 bit-by-bit walk, as the canonical DECODE procedure (F.2.2.3) */
static inline int huff_decode(br_t* b, const huff_t* h, int* bad) {
    int code = 0;
    for (int l = 1; l <= 16; l++) {
        code = (code << 1) | br_bit(b);
        if (code <= h->maxcode[l]) return h->vals[h->valptr[l] + code - h->mincode[l]];
    }
    *bad = 1;
    return 0;
}

/* restart: byte-align, expect RST(k mod 8), skip it; resync on the next RSTn when missing */
static int br_restart(br_t* b, int k) {
    b->nacc = 0;
    b->acc_fill = 0;
    b->at_marker = 0;
    size_t p = b->pos;
    while (p + 1 < b->n && b->d[p] == 0xFF && b->d[p + 1] == 0xFF) p++;
    if (p + 1 < b->n && b->d[p] == 0xFF && b->d[p + 1] == (0xD0 | (k & 7))) {
        b->pos = p + 2;
        return 1;
    }
    for (; p + 1 < b->n; p++) {
        if (b->d[p] == 0xFF && b->d[p + 1] >= 0xD0 && b->d[p + 1] <= 0xD7) {
            b->pos = p + 2;
            return 0;
        }
    }
    b->pos = b->n;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* integer IDCT (restates idct.cpp:20-133, shortcuts included) and colour (color.cpp:4-19)     */
/* ------------------------------------------------------------------------------------------ */

enum { C1 = 2841, C2 = 2676, C3 = 2408, C5 = 1609, C6 = 1108, C7 = 565 };

static inline int clip256(int v) { return v < -256 ? -256 : (v > 255 ? 255 : v); }

static void idct_row(int* blk) {
    int x0, x1, x2, x3, x4, x5, x6, x7, x8;
    if (!((x1 = blk[4] << 11) | (x2 = blk[6]) | (x3 = blk[2]) | (x4 = blk[1]) | (x5 = blk[7]) |
          (x6 = blk[5]) | (x7 = blk[3]))) {
        int v = blk[0] << 3;
        for (int i = 0; i < 8; i++) blk[i] = v;
        return;
    }
    x0 = (blk[0] << 11) + 128;
    x8 = C7 * (x4 + x5);
    x4 = x8 + (C1 - C7) * x4;
    x5 = x8 - (C1 + C7) * x5;
    x8 = C3 * (x6 + x7);
    x6 = x8 - (C3 - C5) * x6;
    x7 = x8 - (C3 + C5) * x7;
    x8 = x0 + x1;
    x0 -= x1;
    x1 = C6 * (x3 + x2);
    x2 = x1 - (C2 + C6) * x2;
    x3 = x1 + (C2 - C6) * x3;
    x1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = x0 + x2;
    x0 -= x2;
    x2 = (181 * (x4 + x5) + 128) >> 8;
    x4 = (181 * (x4 - x5) + 128) >> 8;
    blk[0] = (x7 + x1) >> 8;
    blk[1] = (x3 + x2) >> 8;
    blk[2] = (x0 + x4) >> 8;
    blk[3] = (x8 + x6) >> 8;
    blk[4] = (x8 - x6) >> 8;
    blk[5] = (x0 - x4) >> 8;
    blk[6] = (x3 - x2) >> 8;
    blk[7] = (x7 - x1) >> 8;
}

static void idct_col(int* blk) {
    int x0, x1, x2, x3, x4, x5, x6, x7, x8;
    if (!((x1 = (blk[8 * 4] << 8)) | (x2 = blk[8 * 6]) | (x3 = blk[8 * 2]) | (x4 = blk[8 * 1]) |
          (x5 = blk[8 * 7]) | (x6 = blk[8 * 5]) | (x7 = blk[8 * 3]))) {
        int v = clip256((blk[0] + 32) >> 6);
        for (int i = 0; i < 8; i++) blk[8 * i] = v;
        return;
    }
    x0 = (blk[8 * 0] << 8) + 8192;
    x8 = C7 * (x4 + x5) + 4;
    x4 = (x8 + (C1 - C7) * x4) >> 3;
    x5 = (x8 - (C1 + C7) * x5) >> 3;
    x8 = C3 * (x6 + x7) + 4;
    x6 = (x8 - (C3 - C5) * x6) >> 3;
    x7 = (x8 - (C3 + C5) * x7) >> 3;
    x8 = x0 + x1;
    x0 -= x1;
    x1 = C6 * (x3 + x2) + 4;
    x2 = (x1 - (C2 + C6) * x2) >> 3;
    x3 = (x1 + (C2 - C6) * x3) >> 3;
    x1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = x0 + x2;
    x0 -= x2;
    x2 = (181 * (x4 + x5) + 128) >> 8;
    x4 = (181 * (x4 - x5) + 128) >> 8;
    blk[8 * 0] = clip256((x7 + x1) >> 14);
    blk[8 * 1] = clip256((x3 + x2) >> 14);
    blk[8 * 2] = clip256((x0 + x4) >> 14);
    blk[8 * 3] = clip256((x8 + x6) >> 14);
    blk[8 * 4] = clip256((x8 - x6) >> 14);
    blk[8 * 5] = clip256((x0 - x4) >> 14);
    blk[8 * 6] = clip256((x3 - x2) >> 14);
    blk[8 * 7] = clip256((x7 - x1) >> 14);
}

void jdo_idct_ref(const int32_t in_zz[64], int32_t out[64]) {
    int blk[64];
    for (int i = 0; i < 64; i++) blk[i] = in_zz[kZigzagOfNatural[i]]; /* idct.cpp:24-32 */
    for (int r = 0; r < 8; r++) idct_row(blk + 8 * r);
    for (int c = 0; c < 8; c++) idct_col(blk + c);
    for (int i = 0; i < 64; i++) out[i] = blk[i];
}

static inline int clamp255(int v) { return v > 255 ? 255 : (v < 0 ? 0 : v); }

void jdo_color_ref(int y, int cb, int cr, uint8_t rgb[3]) {
    /* color.cpp:11-17: products and sums in double, stored to float, +128 in float, truncation */
    float r = cr * (2 - 2 * 0.299) + y;
    float b = cb * (2 - 2 * 0.114) + y;
    float g = (y - 0.114 * b - 0.299 * r) / 0.587;
    rgb[0] = (uint8_t)clamp255((int)(r + 128));
    rgb[1] = (uint8_t)clamp255((int)(g + 128));
    rgb[2] = (uint8_t)clamp255((int)(b + 128));
}

/* ------------------------------------------------------------------------------------------ */
/* scan decode                                                                                 */
/* ------------------------------------------------------------------------------------------ */

/* One block: parser.cpp:105-142.  zz[] receives quantised values (zig-zag order, DC absolute). */
static void decode_block(br_t* b, const huff_t* dc, const huff_t* ac, int* pred, int32_t zz[64],
                         int* bad) {
    memset(zz, 0, 64 * sizeof(int32_t));
    int s = huff_decode(b, dc, bad);
    if (s > 16) {
        *bad = 1;
        s = 16;
    }
    int diff = extend(br_bits(b, s), s);
    *pred += diff;
    zz[0] = *pred;
    int k = 1;
    while (k < 64) {
        int rs = huff_decode(b, ac, bad);
        if (rs == 0) break; /* EOB */
        k += rs >> 4;       /* run (ZRL: 15 zeros + the explicit zero below) */
        int sz = rs & 15;
        int bits = br_bits(b, sz);
        if (k < 64) {
            zz[k] = extend(bits, sz);
            k++;
        }
    }
}

typedef struct {
    int32_t* plane[4];
    int stride[4]; /* samples per plane row */
} planes_t;

/* Decodes the whole scan.  Either stores IDCT output into planes (pl != NULL) or quantised
 * coefficients into coef (coef != NULL). */
static int decode_scan(const img_t* im, const uint8_t* d, size_t n, planes_t* pl, int32_t* coef) {
    const jdo_info* f = &im->info;
    br_t b;
    memset(&b, 0, sizeof(b));
    b.d = d + f->ecs_offset;
    b.n = n - f->ecs_offset;
    int pred[4] = {0, 0, 0, 0};
    int bad = 0, rst = 0;
    const int nmcu = f->mcux * f->mcuy;
    const int ri = f->restart_interval;
    int32_t zz[64], deq[64], out[64];
    for (int m = 0; m < nmcu; m++) {
        if (ri && m > 0 && m % ri == 0) {
            if (b.overrun) bad = 1;
            if (!br_restart(&b, rst)) bad = 1;
            rst++;
            b.overrun = 0;
            for (int c = 0; c < 4; c++) pred[c] = 0;
        }
        const int my = m / f->mcux, mx = m % f->mcux;
        int blk = 0;
        for (int c = 0; c < f->ncomp; c++) {
            const huff_t* dc = &im->dc[im->td[c]];
            const huff_t* ac = &im->ac[im->ta[c]];
            const int32_t* q = im->q[f->tq[c]];
            for (int by = 0; by < f->v[c]; by++)
                for (int bx = 0; bx < f->h[c]; bx++, blk++) {
                    decode_block(&b, dc, ac, &pred[c], zz, &bad);
                    if (coef) {
                        memcpy(coef + ((size_t)m * f->blocks_per_mcu + blk) * 64, zz, sizeof(zz));
                        continue;
                    }
                    for (int k = 0; k < 64; k++) deq[k] = zz[k] * q[k]; /* parser.cpp:111,130 */
                    jdo_idct_ref(deq, out);
                    int32_t* dst = pl->plane[c] + (size_t)((my * f->v[c] + by) * 8) * pl->stride[c] +
                                   (mx * f->h[c] + bx) * 8;
                    for (int r = 0; r < 8; r++)
                        memcpy(dst + (size_t)r * pl->stride[c], out + 8 * r, 8 * sizeof(int32_t));
                }
        }
    }
    if (b.overrun) bad = 1;
    return bad ? JDO_ERR_CORRUPT : JDO_OK;
}

int jdo_decode_coefs(const uint8_t* jpeg, size_t len, int32_t* coef) {
    img_t* im = (img_t*)malloc(sizeof(img_t));
    if (!im) return JDO_ERR_INVALID_ARG;
    int st = parse(jpeg, len, im);
    if (st == JDO_OK) st = decode_scan(im, jpeg, len, NULL, coef);
    free(im);
    return st;
}

/* Fancy (triangular) chroma upsampling, an OPTION beyond the reference (which has no chroma
 * subsampling at all): the published libjpeg / libjpeg-turbo filters (jdsample.c
 * h2v1_fancy_upsample, h2v2_fancy_upsample, h1v2_fancy_upsample) restated on the reference's
 * un-shifted samples.  The level shift commutes with the filters exactly (+128 on every input
 * adds 4 * 128 or 16 * 128 before the >> 2 / >> 4), so this equals libjpeg's filter on shifted
 * samples minus 128.  Neighbours outside the component's real samples (ceil(W * h / hmax) x
 * ceil(H * v / vmax)) are replaced by the edge sample, as libjpeg's edge cases and context rows do.
 * Ratios other than 2x1, 2x2 and 1x2 keep replicate upsampling. */
static int fancy_sample(const planes_t* pl, const jdo_info* f, int c, int x, int y) {
    const int rx = f->hmax / f->h[c], ry = f->vmax / f->v[c];
    const int cw = (f->width * f->h[c] + f->hmax - 1) / f->hmax;
    const int ch = (f->height * f->v[c] + f->vmax - 1) / f->vmax;
    const int32_t* P = pl->plane[c];
    const size_t st = (size_t)pl->stride[c];
#define S(xx, yy) P[(size_t)(yy) * st + (xx)]
    if (rx == 2 && ry == 1) {
        const int i = x >> 1;
        if (x & 1) return i >= cw - 1 ? S(i, y) : (3 * S(i, y) + S(i + 1, y) + 2) >> 2;
        return i == 0 ? S(0, y) : (3 * S(i, y) + S(i - 1, y) + 1) >> 2;
    }
    if (ry == 2 && (rx == 1 || rx == 2)) {
        const int r = y >> 1;
        int far = (y & 1) ? r + 1 : r - 1;
        far = far < 0 ? 0 : (far > ch - 1 ? ch - 1 : far);
        if (rx == 1) return (3 * S(x, r) + S(x, far) + ((y & 1) ? 2 : 1)) >> 2;
        const int i = x >> 1;
        const int cs = 3 * S(i, r) + S(i, far);
        if (x & 1) {
            if (i >= cw - 1) return (4 * cs + 7) >> 4;
            return (3 * cs + 3 * S(i + 1, r) + S(i + 1, far) + 7) >> 4;
        }
        if (i == 0) return (4 * cs + 8) >> 4;
        return (3 * cs + 3 * S(i - 1, r) + S(i - 1, far) + 8) >> 4;
    }
#undef S
    return P[(size_t)(y * f->v[c] / f->vmax) * st + (size_t)(x * f->h[c] / f->hmax)];
}

int jdo_decode(const uint8_t* jpeg, size_t len, uint8_t* rgb, int* width, int* height) {
    return jdo_decode_ex(jpeg, len, rgb, width, height, 0);
}

int jdo_decode_ex(const uint8_t* jpeg, size_t len, uint8_t* rgb, int* width, int* height, unsigned flags) {
    img_t* im = (img_t*)malloc(sizeof(img_t));
    if (!im) return JDO_ERR_INVALID_ARG;
    int st = parse(jpeg, len, im);
    if (st != JDO_OK) {
        free(im);
        return st;
    }
    const jdo_info* f = &im->info;
    if (width) *width = f->width;
    if (height) *height = f->height;
    planes_t pl;
    memset(&pl, 0, sizeof(pl));
    int ok = 1;
    for (int c = 0; c < f->ncomp; c++) {
        pl.stride[c] = f->mcux * f->h[c] * 8;
        pl.plane[c] = (int32_t*)malloc(sizeof(int32_t) * pl.stride[c] * f->mcuy * f->v[c] * 8);
        if (!pl.plane[c]) ok = 0;
    }
    if (!ok) {
        for (int c = 0; c < 4; c++) free(pl.plane[c]);
        free(im);
        return JDO_ERR_INVALID_ARG;
    }
    st = decode_scan(im, jpeg, len, &pl, NULL);
    if (rgb) {
        /* crop + colour: parser.cpp:169-193 with replicate upsampling for Hi < Hmax / Vi < Vmax */
        for (int y = 0; y < f->height; y++)
            for (int x = 0; x < f->width; x++) {
                int s[3] = {0, 0, 0};
                for (int c = 0; c < f->ncomp; c++) {
                    if (flags & JDO_FANCY_UPSAMPLING) {
                        s[c] = fancy_sample(&pl, f, c, x, y);
                        continue;
                    }
                    int sx = x * f->h[c] / f->hmax, sy = y * f->v[c] / f->vmax;
                    s[c] = pl.plane[c][(size_t)sy * pl.stride[c] + sx];
                }
                jdo_color_ref(s[0], s[1], s[2], rgb + ((size_t)y * f->width + x) * 3);
            }
    }
    for (int c = 0; c < 4; c++) free(pl.plane[c]);
    free(im);
    return st;
}

/* ------------------------------------------------------------------------------------------ */
/* "fast" CPU mode (a CPU baseline only, never the product): the same decode with  */
/* a 9-bit Huffman lookup table, a 64-bit bit buffer, the reference IDCT unchanged and integer     */
/* colour terms per chroma sample (the reference's double G near integers, as the GPU does).       */
/* Bit-exact with jdo_decode, status included (tests/test_oracle.py).                              */
/* ------------------------------------------------------------------------------------------ */

enum { kFastBits = 9 };
typedef struct {
    uint16_t e[1 << kFastBits]; /* len << 8 | symbol; 0: code longer than kFastBits */
} hfast_t;

static void hfast_build(const huff_t* h, hfast_t* t) {
    memset(t, 0, sizeof(*t));
    int code = 0, k = 0;
    for (int l = 1; l <= kFastBits; l++) {
        for (int i = 0; i < h->counts[l]; i++, k++, code++) {
            const int sh = kFastBits - l;
            for (int x = code << sh; x < ((code + 1) << sh) && x < (1 << kFastBits); x++)
                t->e[x] = (uint16_t)((l << 8) | h->vals[k]);
        }
        code <<= 1;
    }
}

typedef struct {
    const uint8_t* d;
    size_t n, pos;
    uint64_t buf;  /* bits left-aligned */
    int nbits;     /* bits in buf */
    int nreal;     /* of which real data (the rest are 1-bit fill past a marker / the end) */
    int at_marker;
    int overrun;
} fbr_t;

static inline void fbr_fill(fbr_t* b) {
    while (b->nbits <= 56) {
        int c = 0xFF, real = 0;
        if (!b->at_marker && b->pos < b->n) {
            const uint8_t x = b->d[b->pos];
            if (x != 0xFF) {
                c = x;
                real = 1;
                b->pos++;
            } else if (b->pos + 1 < b->n && b->d[b->pos + 1] == 0x00) {
                c = 0xFF;
                real = 1;
                b->pos += 2;
            } else {
                b->at_marker = 1;
            }
        }
        b->buf |= (uint64_t)c << (56 - b->nbits);
        b->nbits += 8;
        if (real && b->nreal == b->nbits - 8) b->nreal += 8;
    }
}

static inline void fbr_skip(fbr_t* b, int n) {
    if (n > b->nreal) b->overrun = 1;
    b->buf <<= n;
    b->nbits -= n;
    b->nreal = b->nreal > n ? b->nreal - n : 0;
}

static inline int fbr_bits(fbr_t* b, int n) {
    if (n == 0) return 0;
    fbr_fill(b);
    const int v = (int)(b->buf >> (64 - n));
    fbr_skip(b, n);
    return v;
}

static inline int fhuff(fbr_t* b, const huff_t* h, const hfast_t* t, int* bad) {
    fbr_fill(b);
    const uint16_t e = t->e[b->buf >> (64 - kFastBits)];
    if (e) {
        fbr_skip(b, e >> 8);
        return e & 0xFF;
    }
    const uint32_t p16 = (uint32_t)(b->buf >> 48);
    for (int l = kFastBits + 1; l <= 16; l++) {
        const int code = (int)(p16 >> (16 - l));
        if (code <= h->maxcode[l]) {
            fbr_skip(b, l);
            return h->vals[h->valptr[l] + code - h->mincode[l]];
        }
    }
    fbr_skip(b, 16);
    *bad = 1;
    return 0;
}

static int fbr_restart(fbr_t* b, int k) {
    /* br_restart from where the bit-serial reader would stand: after the last byte any of whose
     * bits were consumed.  The whole unconsumed data bytes still buffered were the last ones
     * fetched; give their file bytes back (a data 0xFF took two: FF 00). */
    size_t pos = b->pos;
    for (int u = b->nreal / 8; u > 0 && pos > 0; u--)
        pos -= (pos >= 2 && b->d[pos - 1] == 0x00 && b->d[pos - 2] == 0xFF) ? 2 : 1;
    br_t r;
    memset(&r, 0, sizeof(r));
    r.d = b->d;
    r.n = b->n;
    r.pos = pos;
    const int ok = br_restart(&r, k);
    b->pos = r.pos;
    b->buf = 0;
    b->nbits = b->nreal = 0;
    b->at_marker = 0;
    return ok;
}

static int decode_scan_fast(const img_t* im, const uint8_t* d, size_t n, planes_t* pl) {
    const jdo_info* f = &im->info;
    hfast_t* ft = (hfast_t*)malloc(sizeof(hfast_t) * 8);
    if (!ft) return JDO_ERR_INVALID_ARG;
    for (int c = 0; c < f->ncomp; c++) {
        hfast_build(&im->dc[im->td[c]], &ft[2 * c]);
        hfast_build(&im->ac[im->ta[c]], &ft[2 * c + 1]);
    }
    fbr_t b;
    memset(&b, 0, sizeof(b));
    b.d = d + f->ecs_offset;
    b.n = n - f->ecs_offset;
    int pred[4] = {0, 0, 0, 0};
    int bad = 0, rst = 0;
    const int nmcu = f->mcux * f->mcuy;
    const int ri = f->restart_interval;
    int32_t deq[64], out[64];
    for (int m = 0; m < nmcu; m++) {
        if (ri && m > 0 && m % ri == 0) {
            if (b.overrun) bad = 1;
            if (!fbr_restart(&b, rst)) bad = 1;
            rst++;
            b.overrun = 0;
            for (int c = 0; c < 4; c++) pred[c] = 0;
        }
        const int my = m / f->mcux, mx = m % f->mcux;
        for (int c = 0; c < f->ncomp; c++) {
            const huff_t* dc = &im->dc[im->td[c]];
            const huff_t* ac = &im->ac[im->ta[c]];
            const int32_t* q = im->q[f->tq[c]];
            for (int by = 0; by < f->v[c]; by++)
                for (int bx = 0; bx < f->h[c]; bx++) {
                    memset(deq, 0, sizeof(deq));
                    int s = fhuff(&b, dc, &ft[2 * c], &bad);
                    if (s > 16) {
                        bad = 1;
                        s = 16;
                    }
                    pred[c] += extend(fbr_bits(&b, s), s);
                    deq[0] = pred[c] * q[0];
                    for (int k = 1; k < 64;) {
                        const int rs = fhuff(&b, ac, &ft[2 * c + 1], &bad);
                        if (rs == 0) break;
                        k += rs >> 4;
                        const int sz = rs & 15;
                        const int bits = fbr_bits(&b, sz);
                        if (k < 64) {
                            deq[k] = extend(bits, sz) * q[k];
                            k++;
                        }
                    }
                    jdo_idct_ref(deq, out);
                    int32_t* dst = pl->plane[c] + (size_t)((my * f->v[c] + by) * 8) * pl->stride[c] +
                                   (mx * f->h[c] + bx) * 8;
                    for (int r = 0; r < 8; r++) memcpy(dst + (size_t)r * pl->stride[c], out + 8 * r, 8 * sizeof(int32_t));
                }
        }
    }
    if (b.overrun) bad = 1;
    free(ft);
    return bad ? JDO_ERR_CORRUPT : JDO_OK;
}

/* Integer colour of one pixel from precomputed terms (tests/test_oracle.py::test_color_fast_path_exhaustive). */
static inline void color_fast(int y, int cb, int cr, uint8_t rgb[3]) {
    /* n' = n + 271 * 587000 in [0, 2^29): floor(n' / 587000) by one multiply-high (the GPU's
     * chroma_terms), the remainder exact; R and B by the GPU's 24-bit multiply-add forms */
    const uint32_t np = (uint32_t)(202008 * cb + 419198 * cr + 271 * 587000);
    const uint32_t qp = (uint32_t)(((uint64_t)np * 3836115526u) >> 51);
    const int rem = (int)(np - qp * 587000u);
    if (np != 271u * 587000u && (rem < 64 || rem > 587000 - 64)) {
        jdo_color_ref(y, cb, cr, rgb);
        return;
    }
    rgb[0] = (uint8_t)clamp255(y + ((91881 * cr + (128 << 16)) >> 16));
    rgb[1] = (uint8_t)clamp255(np == 271u * 587000u ? y + 128 : y + 127 + 271 - (int)qp);
    rgb[2] = (uint8_t)clamp255(y + ((58065 * cb + (128 << 15) + 32) >> 15));
}

/* Mismatches of color_fast against jdo_color_ref over every (y, cb, cr) in [-256, 255]^3. */
long jdo_check_color_fast(void) {
    long bad = 0;
    for (int cb = -256; cb < 256; cb++)
        for (int cr = -256; cr < 256; cr++)
            for (int y = -256; y < 256; y++) {
                uint8_t a[3], b[3];
                jdo_color_ref(y, cb, cr, a);
                color_fast(y, cb, cr, b);
                bad += a[0] != b[0] || a[1] != b[1] || a[2] != b[2];
            }
    return bad;
}

int jdo_decode_fast(const uint8_t* jpeg, size_t len, uint8_t* rgb, int* width, int* height) {
    img_t* im = (img_t*)malloc(sizeof(img_t));
    if (!im) return JDO_ERR_INVALID_ARG;
    int st = parse(jpeg, len, im);
    if (st != JDO_OK) {
        free(im);
        return st;
    }
    const jdo_info* f = &im->info;
    if (width) *width = f->width;
    if (height) *height = f->height;
    planes_t pl;
    memset(&pl, 0, sizeof(pl));
    int ok = 1;
    for (int c = 0; c < f->ncomp; c++) {
        pl.stride[c] = f->mcux * f->h[c] * 8;
        pl.plane[c] = (int32_t*)malloc(sizeof(int32_t) * pl.stride[c] * f->mcuy * f->v[c] * 8);
        if (!pl.plane[c]) ok = 0;
    }
    if (ok) st = decode_scan_fast(im, jpeg, len, &pl);
    int* sx = ok && rgb ? (int*)malloc(sizeof(int) * 3 * (size_t)f->width) : NULL;
    if (ok && rgb && sx) {
        for (int c = 0; c < f->ncomp && c < 3; c++)
            for (int x = 0; x < f->width; x++) sx[c * f->width + x] = x * f->h[c] / f->hmax;
        for (int y = 0; y < f->height; y++) {
            const int32_t* row[3] = {NULL, NULL, NULL};
            for (int c = 0; c < f->ncomp && c < 3; c++) row[c] = pl.plane[c] + (size_t)(y * f->v[c] / f->vmax) * pl.stride[c];
            uint8_t* o = rgb + (size_t)y * f->width * 3;
            if (f->ncomp == 1) {
                for (int x = 0; x < f->width; x++) color_fast(row[0][x], 0, 0, o + 3 * x);
            } else {
                const int *s1 = sx + f->width, *s2 = sx + 2 * f->width;
                for (int x = 0; x < f->width; x++) color_fast(row[0][sx[x]], row[1][s1[x]], row[2][s2[x]], o + 3 * x);
            }
        }
    } else if (ok && rgb) {
        ok = 0;
    }
    free(sx);
    for (int c = 0; c < 4; c++) free(pl.plane[c]);
    free(im);
    return ok ? st : JDO_ERR_INVALID_ARG;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline helper                                                                         */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    const uint8_t* const* jpegs;
    const size_t* lens;
    uint8_t* const* rgbs;
    int* status;
    int n;
    int next;
    int fast;
} work_t;

static void* worker(void* arg) {
    work_t* w = (work_t*)arg;
    for (;;) {
        int i = __sync_fetch_and_add(&w->next, 1);
        if (i >= w->n) break;
        int st = w->fast ? jdo_decode_fast(w->jpegs[i], w->lens[i], w->rgbs ? w->rgbs[i] : NULL, NULL, NULL)
                         : jdo_decode(w->jpegs[i], w->lens[i], w->rgbs ? w->rgbs[i] : NULL, NULL, NULL);
        if (w->status) w->status[i] = st;
    }
    return NULL;
}

double jdo_decode_many(const uint8_t* const* jpegs, const size_t* lens, int n, uint8_t* const* rgbs,
                       int threads, int* status) {
    return jdo_decode_many_ex(jpegs, lens, n, rgbs, threads, status, 0);
}

double jdo_decode_many_ex(const uint8_t* const* jpegs, const size_t* lens, int n, uint8_t* const* rgbs,
                          int threads, int* status, int fast) {
    work_t w = {jpegs, lens, rgbs, status, n, 0, fast};
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (threads == 1) {
        worker(&w);
    } else {
        for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &w);
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
