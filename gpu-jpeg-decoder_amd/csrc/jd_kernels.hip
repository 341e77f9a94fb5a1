// jd_kernels.hip — gfx950 (CDNA4, wave64) kernels of the batched JPEG decode path.
//
//   k_rst_scan    byte scan for RSTn / terminating markers, 16 KiB of ECS per workgroup
//   k_rst_index   one wave per image: ordered RSTn positions -> per-interval start offsets
//   k_huffman     one lane per restart interval: Huffman + DPCM/RLE -> sparse coefficients
//   k_idct_color  one workgroup per MCU-row slice: dequant + integer IDCT (LDS tile) +
//                 replicate chroma upsample + YCbCr->RGB -> uint8 HWC
//
// Arithmetic follows the reference CPU decoder bit for bit (cpp-decoder/src/idct.cpp,
// utils/color.cpp); the restatement used as checker lives in oracle/ (tests only).
#include <hip/hip_runtime.h>

#include "jd_kernels.hpp"

#pragma clang fp contract(off)

namespace jd {

// zig-zag index -> natural (row-major) position: inverse of src/idct.cpp:8-16.
__constant__ uint8_t kNatOfZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18,
                                     11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                                     13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43,
                                     36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                                     38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ------------------------------------------------------------------------------------------
// wave helpers (wave64)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// ------------------------------------------------------------------------------------------
// Stage 0: RSTn marker scan.  A marker is FF Dx (x = 0..7); FF 00 is a stuffed data byte and
// FF FF a fill byte, so "FF followed by D0..D7" is unambiguous.  Any other FF xx ends the ECS.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kScanThreads) void k_rst_scan(BatchDev b) {
    const uint32_t r = blockIdx.y;
    if (r >= b.nrst) return;
    const uint32_t ii = b.rst_imgs[r];
    const ImgDesc& im = b.imgs[ii];
    const uint32_t c = blockIdx.x;
    if (c >= im.nchunks) return;
    const uint8_t* file = reinterpret_cast<const uint8_t*>(im.jpeg);
    const uintptr_t lo = reinterpret_cast<uintptr_t>(file) + im.ecs_off;
    const uintptr_t fend = reinterpret_cast<uintptr_t>(file) + im.len;
    const uintptr_t a0 = lo & ~uintptr_t(15);
    const uintptr_t t0 = a0 + uintptr_t(c) * kScanChunk + uintptr_t(threadIdx.x) * kScanBytesPerThread;

    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uintptr_t a = t0 + 16 * q;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (a < fend) v = *reinterpret_cast<const uint4*>(a);  // 16B-aligned: never crosses a page
        w[4 * q + 0] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
    const uint32_t nextb = (t0 + 64 < fend) ? *reinterpret_cast<const uint8_t*>(t0 + 64) : 0u;

    uint32_t count = 0, term = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint32_t by = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        const uint32_t nb = (i < 63) ? ((w[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xFFu) : nextb;
        const uintptr_t a = t0 + i;
        if (by == 0xFFu && a >= lo && a + 1 < fend) {
            if ((nb & 0xF8u) == 0xD0u) count++;
            else if (nb != 0x00u && nb != 0xFFu) term = min(term, uint32_t(a - reinterpret_cast<uintptr_t>(file)));
        }
    }

    __shared__ uint32_t s_wsum[kScanThreads / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(count);
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t off = incl - count, total = 0;
#pragma unroll
    for (int j = 0; j < kScanThreads / 64; j++) {
        if (j < wv) off += s_wsum[j];
        total += s_wsum[j];
    }
    if (count) {
        uint32_t* out = b.chunk_pos + size_t(im.chunk_base + c) * kScanCap;
#pragma unroll
        for (int i = 0; i < 64; i++) {
            const uint32_t by = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            const uint32_t nb = (i < 63) ? ((w[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xFFu) : nextb;
            const uintptr_t a = t0 + i;
            if (by == 0xFFu && a >= lo && a + 1 < fend && (nb & 0xF8u) == 0xD0u)
                out[off++] = uint32_t(a - reinterpret_cast<uintptr_t>(file));
        }
    }
    if (threadIdx.x == 0) b.chunk_cnt[im.chunk_base + c] = total;
    if (term != 0xFFFFFFFFu) atomicMin(&b.ecs_end[ii], term);
}

// ------------------------------------------------------------------------------------------
// Stage 1: per image, the k-th marker (in stream order) starts interval k+1.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_rst_index(BatchDev b) {
    const uint32_t ii = b.rst_imgs[blockIdx.x];
    const ImgDesc& im = b.imgs[ii];
    const uint8_t* file = reinterpret_cast<const uint8_t*>(im.jpeg);
    const uint32_t term = b.ecs_end[ii];
    const uint32_t need = im.nseg - 1;
    const int lane = threadIdx.x;
    uint32_t running = 0, valid = 0;
    bool order_bad = false;
    for (uint32_t c0 = 0; c0 < im.nchunks; c0 += 64) {
        const uint32_t c = c0 + lane;
        const uint32_t cnt = (c < im.nchunks) ? b.chunk_cnt[im.chunk_base + c] : 0u;
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t excl = incl - cnt;
        const uint32_t tot = __shfl(incl, 63, 64);
        const uint32_t* pos = b.chunk_pos + size_t(im.chunk_base + c) * kScanCap;
        for (uint32_t j = 0; j < cnt; j++) {
            const uint32_t p = pos[j];
            const uint32_t idx = running + excl + j;
            if (p < term) {
                valid++;
                if (idx < need) {
                    b.seg_start[im.seg_base + 1 + idx] = p + 2;
                    if ((file[p + 1] & 7u) != (idx & 7u)) order_bad = true;
                }
            }
        }
        running += tot;
    }
    // wave-reduce the number of markers in front of the terminator
    uint32_t v = valid;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (v < need) {
        for (uint32_t idx = v + lane; idx < need; idx += 64) b.seg_start[im.seg_base + 1 + idx] = term + 2;
        if (lane == 0) atomicOr(&b.status[ii], kStRstMissing);
    }
    if (__any(order_bad) && lane == 0) atomicOr(&b.status[ii], kStRstOrder);
}

// ------------------------------------------------------------------------------------------
// Stage 2: Huffman decode.  One lane owns one restart interval (segment) and walks it symbol by
// symbol in a single flattened loop (DC and AC steps share one body, so lanes of a wave never
// wait for each other's blocks).
//
// Memory discipline (the whole point of the structure): the decode steps contain NO global loads.
// gfx950 counts stores and loads on one vmcnt, so any wait for a bitstream load inside the
// divergent step would also wait for every coefficient store in flight — and with 64 lanes some
// lane needs new bytes almost every step.  Instead each lane's raw ECS bytes live in a 256-byte
// LDS ring (layout [word][lane]: a lane always hits bank lane%32, conflict-free), refilled in a
// wave-uniform service phase every kRound steps.  A service writes the 64 bytes loaded by the
// previous service into the ring and issues the next 64-byte load, so every load has a full
// round to land.  Un-stuffing (FF 00 -> FF) happens when bytes move from the ring to the bit
// buffer.
// ------------------------------------------------------------------------------------------
constexpr int kRingWords = 64;  // per-lane ring: 256 raw bytes (+1 mirror word for wrap reads)
constexpr int kRingBytes = kRingWords * 4;
constexpr int kFillBytes = 64;  // raw bytes fetched per lane per service
constexpr int kRound = 8;       // decode steps between services (<= 64 raw bytes consumed)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

// Unconditional load (no phi with a fill value, so hipcc does not wait at issue); the address is
// clamped to the file's last 16-byte chunk, which is always mapped.  Bytes past the segment end
// are never consumed as data, so what a clamped load returns there is irrelevant.
__device__ __forceinline__ u32x4 load16(uintptr_t a, uintptr_t last) {
    return *reinterpret_cast<gu32x4*>(a < last ? a : last);
}

__device__ __forceinline__ int extend(uint32_t v, int s) {  // utils/stream.cpp:44-52
    if (s == 0) return 0;
    const int l = 1 << (s - 1);
    return int(v) >= l ? int(v) : int(v) - ((l << 1) - 1);
}

struct Lane {
    uint64_t buf;  // bit buffer, MSB-aligned
    int nb;        // valid bits in buf
    int p;         // next raw byte (relative to the lane's 16-byte aligned base)
    int end_p;     // first raw byte past the segment
    int wr;        // ring holds raw bytes [p, wr)
    int req;       // loads issued up to base + req
    bool pending;  // q0..q3 hold bytes [wr, wr + 64) in flight
    bool ended;    // reached a marker / the segment end: only 1-bit fill follows
    uint32_t data_bits, used_bits;
};

__device__ __forceinline__ uint32_t ring_byte(const uint32_t* ring, int x) {
    return (ring[((x >> 2) & (kRingWords - 1)) * kHuffThreads] >> ((x & 3) * 8)) & 0xFFu;
}

// Moves 32 bits from the ring into the bit buffer when it holds <= 32.  Returns false when the
// ring does not hold the 8 raw bytes a refill may need (the lane then idles until the next service).
__device__ __forceinline__ bool refill(Lane& L, const uint32_t* ring) {
    if (L.nb > 32) return true;
    if (L.wr - L.p < 8) return false;
    const int w = (L.p >> 2) & (kRingWords - 1);
    const uint32_t w0 = ring[w * kHuffThreads], w1 = ring[(w + 1) * kHuffThreads];
    const uint32_t t = __builtin_amdgcn_alignbyte(w1, w0, uint32_t(L.p & 3));
    const bool has_ff = (((~t) - 0x01010101u) & t & 0x80808080u) != 0u;
    uint32_t w32;
    if (!L.ended && L.end_p - L.p >= 4 && !has_ff) {
        w32 = __builtin_bswap32(t);
        L.p += 4;
        L.data_bits += 32;
    } else {
        w32 = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t by = 0xFFu;
            if (!L.ended && L.p < L.end_p) {
                const uint32_t c = ring_byte(ring, L.p);
                if (c != 0xFFu) {
                    by = c;
                    L.p += 1;
                    L.data_bits += 8;
                } else if (L.p + 1 < L.end_p && ring_byte(ring, L.p + 1) == 0u) {
                    L.p += 2;  // stuffed FF 00
                    L.data_bits += 8;
                } else {
                    L.ended = true;  // marker
                }
            } else {
                L.ended = true;
            }
            w32 = (w32 << 8) | by;
        }
    }
    L.buf |= uint64_t(w32) << (32 - L.nb);
    L.nb += 32;
    return true;
}

__device__ __forceinline__ void skip_bits(Lane& L, int n) {
    L.buf <<= n;
    L.nb -= n;
    L.used_bits += uint32_t(n);
}

// Wave-uniform service: commit last service's load to the ring, issue the next one.
__device__ __forceinline__ void service(Lane& L, uint32_t* ring, u32x4& q0, u32x4& q1, u32x4& q2, u32x4& q3,
                                        uintptr_t base, uintptr_t last, bool active) {
    if (L.pending) {
        const int w = (L.wr >> 2) & (kRingWords - 1);  // wr is a multiple of 64: no wrap inside
        uint32_t* r = ring + w * kHuffThreads;
        r[0 * kHuffThreads] = q0.x;
        r[1 * kHuffThreads] = q0.y;
        r[2 * kHuffThreads] = q0.z;
        r[3 * kHuffThreads] = q0.w;
        r[4 * kHuffThreads] = q1.x;
        r[5 * kHuffThreads] = q1.y;
        r[6 * kHuffThreads] = q1.z;
        r[7 * kHuffThreads] = q1.w;
        r[8 * kHuffThreads] = q2.x;
        r[9 * kHuffThreads] = q2.y;
        r[10 * kHuffThreads] = q2.z;
        r[11 * kHuffThreads] = q2.w;
        r[12 * kHuffThreads] = q3.x;
        r[13 * kHuffThreads] = q3.y;
        r[14 * kHuffThreads] = q3.z;
        r[15 * kHuffThreads] = q3.w;
        if (w == 0) ring[kRingWords * kHuffThreads] = q0.x;  // mirror word for wrap reads
        L.wr += kFillBytes;
    }
    // the bytes requested now land in the ring at the next service, over [req-256, req-192)
    L.pending = active && (L.req - L.p <= kRingBytes - kFillBytes);
    const uintptr_t a = base + uintptr_t(L.req);
    q0 = load16(a, last);
    q1 = load16(a + 16, last);
    q2 = load16(a + 32, last);
    q3 = load16(a + 48, last);
    if (L.pending) L.req += kFillBytes;
}

// One Huffman symbol (+ magnitude bits): symbol and EXTENDed value.
__device__ __forceinline__ void decode_sym(Lane& L, const HuffLut* t, bool is_dc, int& sym, int& val, bool& bad) {
    const uint32_t e = t->fast[uint32_t(L.buf >> (64 - kLutBits))];
    int len;
    bool complete;
    if (e & 31u) {
        len = int(e & 31u);
        complete = (e & kLutFlagComplete) != 0u;
        sym = int((e >> 8) & 255u);
        val = int32_t(e) >> 16;
    } else {  // code longer than kLutBits (or invalid): canonical limits, F.2.2.3
        const uint32_t v16 = uint32_t(L.buf >> 48);
        int l = kLutBits + 1;
        while (l <= 16 && v16 >= t->lim[l]) l++;
        if (l > 16) {
            bad = true;
            l = 16;
            sym = 0;
        } else {
            sym = t->vals[(t->base[l] + int(v16 >> (16 - l))) & 255];
        }
        len = l;
        complete = false;
        val = 0;
    }
    skip_bits(L, len);
    if (!complete) {
        int s = is_dc ? sym : (sym & 15);
        if (s > 16) {
            bad = true;
            s = 16;
        }
        const uint32_t bits = s ? uint32_t(L.buf >> (64 - s)) : 0u;
        skip_bits(L, s);
        val = extend(bits, s);
    }
}

__global__ __launch_bounds__(kHuffThreads) void k_huffman(BatchDev b) {
    __shared__ HuffLut s_lut[kSlotsPerSet];
    __shared__ uint32_t s_ring[(kRingWords + 1) * kHuffThreads];
    const TableSet& ts = b.tablesets[b.wg_tableset[blockIdx.x]];
    for (int slot = 0; slot < kSlotsPerSet; slot++) {
        const int id = ts.lut[slot];
        if (id < 0) continue;
        const uint4* src = reinterpret_cast<const uint4*>(b.luts + id);
        uint4* dst = reinterpret_cast<uint4*>(s_lut + slot);
        for (int i = threadIdx.x; i < int(sizeof(HuffLut) / 16); i += kHuffThreads) dst[i] = src[i];
    }
    __syncthreads();

    const uint32_t g = blockIdx.x * kHuffThreads + threadIdx.x;
    const uint32_t ii = (g < b.nseg) ? b.seg_img[g] : kInvalidImage;
    if (__all(ii == kInvalidImage)) return;  // whole wave is padding
    const bool valid = ii != kInvalidImage;
    const ImgDesc& im = b.imgs[valid ? ii : 0u];
    uint32_t* ring = s_ring + threadIdx.x;

    uint64_t gblk = 0, gend = 0;
    uint32_t start = 0, end = 0;
    if (valid) {
        const uint32_t k_seg = g - im.seg_base;
        const uint32_t nmcu = im.mcux * im.mcuy;
        const uint32_t ri = im.restart_interval;
        const uint32_t mcu0 = ri ? k_seg * ri : 0u;
        const uint32_t mcu1 = ri ? min(mcu0 + ri, nmcu) : nmcu;
        start = b.seg_start[g];
        end = (k_seg + 1 < im.nseg) ? b.seg_start[g + 1] - 2u : b.ecs_end[ii];
        gblk = im.block_base + uint64_t(mcu0) * im.bpm;
        gend = im.block_base + uint64_t(mcu1) * im.bpm;
    }
    const uintptr_t file = valid ? uintptr_t(im.jpeg) : uintptr_t(b.imgs);
    const uintptr_t last = valid ? ((file + im.len - 1) & ~uintptr_t(15)) : (uintptr_t(b.imgs) & ~uintptr_t(15));
    const uintptr_t base = (file + start) & ~uintptr_t(15);

    Lane L;
    L.buf = 0;
    L.nb = 0;
    L.p = int((file + start) & 15);
    L.end_p = L.p + (end > start ? int(end - start) : 0);
    L.wr = 0;
    L.req = 0;
    L.pending = false;
    L.ended = false;
    L.data_bits = 0;
    L.used_bits = 0;
    u32x4 q0, q1, q2, q3;
    service(L, ring, q0, q1, q2, q3, base, last, valid);
    service(L, ring, q0, q1, q2, q3, base, last, valid);

    const int d0 = ts.dc_slot[0], d1 = ts.dc_slot[1], d2 = ts.dc_slot[2];
    const int a0 = ts.ac_slot[0], a1 = ts.ac_slot[1], a2 = ts.ac_slot[2];
    const uint32_t pattern = im.block_pattern, bpm = im.bpm;
    uint32_t bi = 0;
    int comp = int(pattern & 3u);
    int k = 0, p0 = 0, p1 = 0, p2 = 0, dc = 0;
    const uint32_t ent_first = valid ? b.seg_entry[g] : 0u;
    uint32_t ent = ent_first, ent0 = ent_first;
    bool bad = false;

    for (;;) {
        const bool active = gblk < gend;
        if (!__any(active)) break;
        service(L, ring, q0, q1, q2, q3, base, last, active);
        for (int it = 0; it < kRound; it++) {
            if (gblk < gend && refill(L, ring)) {
                const bool is_dc = (k == 0);
                const int slot = is_dc ? (comp == 0 ? d0 : (comp == 1 ? d1 : d2))
                                       : (comp == 0 ? a0 : (comp == 1 ? a1 : a2));
                int sym, val;
                decode_sym(L, &s_lut[slot], is_dc, sym, val, bad);
                if (is_dc) {  // parser.cpp:106-111: DPCM
                    const int pr = (comp == 0 ? p0 : (comp == 1 ? p1 : p2)) + val;
                    if (comp == 0) p0 = pr;
                    else if (comp == 1) p1 = pr;
                    else p2 = pr;
                    if (pr < -32768 || pr > 32767) bad = true;
                    dc = pr;
                    ent0 = ent;
                    k = 1;
                } else if (sym == 0) {  // EOB: parser.cpp:117-119
                    k = 64;
                } else {  // run/size: parser.cpp:122-133
                    k += sym >> 4;
                    if (k < 64) {
                        if (sym & 15) b.entries[ent++] = (uint32_t(val) << 16) | uint32_t(k);
                        k++;
                    }
                }
                if (k >= 64) {
                    b.blocks[gblk] = BlockInfo{ent0, ((ent - ent0) << 16) | (uint32_t(dc) & 0xFFFFu)};
                    gblk++;
                    bi = (bi + 1 == bpm) ? 0u : bi + 1;
                    comp = int((pattern >> (2 * bi)) & 3u);
                    k = 0;
                }
            }
        }
    }
    if (!valid) return;
    if (L.used_bits > L.data_bits) bad = true;
    if (bad) atomicOr(&b.status[ii], kStCorrupt);
    atomicAdd(&b.counters[0], (unsigned long long)(ent - ent_first));
}

// ------------------------------------------------------------------------------------------
// Stage 3: dequantise + IDCT + upsample + colour.
// ------------------------------------------------------------------------------------------
enum { kC1 = 2841, kC2 = 2676, kC3 = 2408, kC5 = 1609, kC6 = 1108, kC7 = 565 };

__device__ __forceinline__ int clip256(int v) { return min(max(v, -256), 255); }

// idct.cpp:34-77 without the DC shortcut (identical results: SURVEY.md App. B P7, and
// tests/test_gpu.py::test_idct_kat).
__device__ __forceinline__ void idct_row(int* blk) {
    int x0, x1, x2, x3, x4, x5, x6, x7, x8;
    x1 = blk[4] << 11;
    x2 = blk[6];
    x3 = blk[2];
    x4 = blk[1];
    x5 = blk[7];
    x6 = blk[5];
    x7 = blk[3];
    x0 = (blk[0] << 11) + 128;
    x8 = kC7 * (x4 + x5);
    x4 = x8 + (kC1 - kC7) * x4;
    x5 = x8 - (kC1 + kC7) * x5;
    x8 = kC3 * (x6 + x7);
    x6 = x8 - (kC3 - kC5) * x6;
    x7 = x8 - (kC3 + kC5) * x7;
    x8 = x0 + x1;
    x0 -= x1;
    x1 = kC6 * (x3 + x2);
    x2 = x1 - (kC2 + kC6) * x2;
    x3 = x1 + (kC2 - kC6) * x3;
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

// idct.cpp:79-122 without the DC shortcut.
__device__ __forceinline__ void idct_col(int* blk) {
    int x0, x1, x2, x3, x4, x5, x6, x7, x8;
    x1 = blk[8 * 4] << 8;
    x2 = blk[8 * 6];
    x3 = blk[8 * 2];
    x4 = blk[8 * 1];
    x5 = blk[8 * 7];
    x6 = blk[8 * 5];
    x7 = blk[8 * 3];
    x0 = (blk[0] << 8) + 8192;
    x8 = kC7 * (x4 + x5) + 4;
    x4 = (x8 + (kC1 - kC7) * x4) >> 3;
    x5 = (x8 - (kC1 + kC7) * x5) >> 3;
    x8 = kC3 * (x6 + x7) + 4;
    x6 = (x8 - (kC3 - kC5) * x6) >> 3;
    x7 = (x8 - (kC3 + kC5) * x7) >> 3;
    x8 = x0 + x1;
    x0 -= x1;
    x1 = kC6 * (x3 + x2) + 4;
    x2 = (x1 - (kC2 + kC6) * x2) >> 3;
    x3 = (x1 + (kC2 - kC6) * x3) >> 3;
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

__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }

// utils/color.cpp:11-17 verbatim in double/float; taken only for the rare G inputs below.
__device__ __attribute__((noinline)) int color_g_exact(int y, int cb, int cr) {
    const float r = float(double(cr) * (2 - 2 * 0.299) + double(y));
    const float b = float(double(cb) * (2 - 2 * 0.114) + double(y));
    const float g = float((double(y) - 0.114 * double(b) - 0.299 * double(r)) / 0.587);
    return clamp255(int(g + 128.0f));
}

// Exact restatement of utils/color.cpp:8-19 (verified exhaustively over [-256,255]^3:
// tests/test_gpu.py::test_color_exhaustive):
//   R, B: one fp32 FMA; the true value is >= 0.002 away from an integer unless it is one, so the
//         fp32 result truncates like the reference's double->float result.
//   G   : g = y - N/587000 with N = 202008*cb + 419198*cr exactly; away from integers (rem not
//         within 64/587000 of 0) trunc(g + 128) = y + 127 - floor(N/587000); else exact path.
__device__ __forceinline__ void color_px(int y, int cb, int cr, uint32_t& R, uint32_t& G, uint32_t& B) {
    const float r = __builtin_fmaf(float(cr), 1.402f, float(y));
    const float bb = __builtin_fmaf(float(cb), 1.772f, float(y));
    R = uint32_t(clamp255(int(r + 128.0f)));
    B = uint32_t(clamp255(int(bb + 128.0f)));
    const int n = 202008 * cb + 419198 * cr;
    const int nq = n + 587000 * 512;  // > 0 for |cb|,|cr| <= 256
    const int q = int(uint32_t(nq) / 587000u) - 512;
    const int rem = n - q * 587000;
    if (rem < 64 || rem > 587000 - 64) G = uint32_t(color_g_exact(y, cb, cr));
    else G = uint32_t(clamp255(y + 127 - q));
}

__global__ __launch_bounds__(kIdctThreads) void k_idct_color(BatchDev b) {
    __shared__ int s_coef[kTileMaxBlocks * 64];
    __shared__ int s_q[4][64];
    const uint32_t ii = blockIdx.y;
    const ImgDesc& im = b.imgs[ii];
    const uint32_t tile = blockIdx.x;
    const uint32_t tiles_x = im.tiles_x;
    if (tile >= tiles_x * im.mcuy) return;
    const uint32_t tr = tile / tiles_x, tc = tile - tr * tiles_x;
    const uint32_t T = im.tile_mcus;
    const uint32_t m0 = tc * T;
    const uint32_t nm = min(T, im.mcux - m0);
    const uint32_t bpm = im.bpm, nblk = nm * bpm;
    const int tid = threadIdx.x;

    for (uint32_t i = tid; i < nblk * 16; i += kIdctThreads)
        reinterpret_cast<int4*>(s_coef)[i] = make_int4(0, 0, 0, 0);
    if (tid < int(im.ncomp) * 64) {
        const int c = tid >> 6, z = tid & 63;
        s_q[c][z] = int(b.qtabs[size_t(im.qslot[c]) * 64 + z]);
    }
    __syncthreads();

    {  // sparse -> dense, dequantised in zig-zag order (parser.cpp:111,130), natural placement
        const uint32_t j = uint32_t(tid) >> 2, sub = uint32_t(tid) & 3;
        if (j < nblk) {
            const uint32_t mi = j / bpm, bb = j - mi * bpm;
            const uint32_t comp = (im.block_pattern >> (2 * bb)) & 3u;
            const uint64_t gb = im.block_base + uint64_t(tr * im.mcux + m0 + mi) * bpm + bb;
            const BlockInfo bi = b.blocks[gb];
            const int cnt = int(bi.cnt_dc >> 16);
            int* blk = s_coef + j * 64;
            if (sub == 0) blk[0] = int(int16_t(bi.cnt_dc & 0xFFFFu)) * s_q[comp][0];
            for (int i = int(sub); i < cnt; i += 4) {
                const uint32_t e = b.entries[bi.entry_start + i];
                const int z = int(e & 63u);
                blk[kNatOfZz[z]] = (int32_t(e) >> 16) * s_q[comp][z];
            }
        }
    }
    __syncthreads();
    for (uint32_t r = tid; r < nblk * 8; r += kIdctThreads) idct_row(s_coef + r * 8);
    __syncthreads();
    for (uint32_t c = tid; c < nblk * 8; c += kIdctThreads) idct_col(s_coef + (c >> 3) * 64 + (c & 7));
    __syncthreads();

    const uint32_t mw = 8 * im.hmax, mh = 8 * im.vmax;
    const uint32_t PW = nm * mw, PH = mh;
    const uint32_t x0 = m0 * mw, y0 = tr * mh;
    uint8_t* out = reinterpret_cast<uint8_t*>(im.rgb);
    const uint32_t W = im.width, H = im.height, nc = im.ncomp;
    for (uint32_t p = tid; p < PW * PH; p += kIdctThreads) {
        const uint32_t py = p / PW, px = p - py * PW;
        const uint32_t x = x0 + px, y = y0 + py;
        if (x >= W || y >= H) continue;
        const uint32_t mi = px / mw, ux = px - mi * mw;
        int s[3] = {0, 0, 0};
#pragma unroll
        for (int c = 0; c < 3; c++) {
            if (uint32_t(c) < nc) {
                const uint32_t sx = ux * im.h[c] / im.hmax, sy = py * im.v[c] / im.vmax;
                const uint32_t bc = im.comp_block0[c] + (sy >> 3) * im.h[c] + (sx >> 3);
                s[c] = s_coef[(mi * bpm + bc) * 64 + (sy & 7) * 8 + (sx & 7)];
            }
        }
        uint32_t R, G, B;
        color_px(s[0], s[1], s[2], R, G, B);
        const size_t o = (size_t(y) * W + x) * 3;
        out[o] = uint8_t(R);
        out[o + 1] = uint8_t(G);
        out[o + 2] = uint8_t(B);
    }
}

// ------------------------------------------------------------------------------------------
// Known-answer hooks
// ------------------------------------------------------------------------------------------
__global__ void k_test_idct(const int32_t* in_zz, int32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int blk[64];
    for (int z = 0; z < 64; z++) blk[kNatOfZz[z]] = in_zz[size_t(i) * 64 + z];
    for (int r = 0; r < 8; r++) idct_row(blk + 8 * r);
    for (int c = 0; c < 8; c++) idct_col(blk + c);
    for (int z = 0; z < 64; z++) out[size_t(i) * 64 + z] = blk[z];
}

__global__ void k_test_color(const int32_t* ycc, uint8_t* rgb, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t R, G, B;
    color_px(ycc[3 * i], ycc[3 * i + 1], ycc[3 * i + 2], R, G, B);
    rgb[3 * i] = uint8_t(R);
    rgb[3 * i + 1] = uint8_t(G);
    rgb[3 * i + 2] = uint8_t(B);
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_rst_scan(const BatchDev& b, hipStream_t s) {
    if (!b.nrst || !b.max_chunks) return hipSuccess;
    hipLaunchKernelGGL(k_rst_scan, dim3(b.max_chunks, b.nrst), dim3(kScanThreads), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_rst_index(const BatchDev& b, hipStream_t s) {
    if (!b.nrst) return hipSuccess;
    hipLaunchKernelGGL(k_rst_index, dim3(b.nrst), dim3(64), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_huffman(const BatchDev& b, hipStream_t s) {
    if (!b.nseg) return hipSuccess;
    hipLaunchKernelGGL(k_huffman, dim3(b.nseg / kHuffThreads), dim3(kHuffThreads), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_idct_color(const BatchDev& b, hipStream_t s) {
    if (!b.nimg || !b.max_tiles_x) return hipSuccess;
    hipLaunchKernelGGL(k_idct_color, dim3(b.max_tiles_x, b.nimg), dim3(kIdctThreads), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_test_idct(const int32_t* in_zz, int32_t* out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_test_idct, dim3((n + 63) / 64), dim3(64), 0, s, in_zz, out, n);
    return hipGetLastError();
}

hipError_t launch_test_color(const int32_t* ycc, uint8_t* rgb, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_test_color, dim3((n + 255) / 256), dim3(256), 0, s, ycc, rgb, n);
    return hipGetLastError();
}

}  // namespace jd
