// jd_kernels.hip — gfx950 (CDNA4, wave64) kernels of the batched JPEG decode path.
//
//   k_scan        16 KiB of ECS per workgroup: stuffed-zero counts, RSTn / terminator positions
//   k_index       one wave per image: chunk offsets in the un-stuffed stream, restart-interval
//                 (segment) boundaries, RSTn order / count checks
//   k_compact     16 KiB per workgroup: drops the stuffed 00 after every FF (byte compaction)
//   k_huffman     one lane per restart interval: Huffman + DPCM/RLE -> sparse coefficients
//   k_idct_color  one workgroup per 128-px tile: dequant + integer IDCT (LDS tile) + replicate
//                 chroma upsample + YCbCr->RGB -> uint8 HWC
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint8_t gu8;

// ------------------------------------------------------------------------------------------
// wave / block helpers (wave64)
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

// Exclusive scan over a 256-thread block; returns the exclusive prefix, *total the block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(x);
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t off = incl - x, tot = 0;
#pragma unroll
    for (int j = 0; j < kScanThreads / 64; j++) {
        if (j < wv) off += s_wsum[j];
        tot += s_wsum[j];
    }
    *total = tot;
    return off;
}

// 64 raw bytes of a thread (16B-aligned loads never cross a page; bytes at/after fend read 0).
__device__ __forceinline__ void load64(uintptr_t t0, uintptr_t fend, uint32_t (&w)[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uintptr_t a = t0 + 16 * q;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (a < fend) v = *reinterpret_cast<gu32x4*>(a);
        w[4 * q + 0] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[16], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; }

// ------------------------------------------------------------------------------------------
// Stage 0: scan.  In an ECS a data FF is always followed by a stuffed 00, so:
//   FF 00      -> the 00 is dropped by un-stuffing (the reference's loop, parser.cpp:84-96)
//   FF D0..D7  -> RSTn marker: the next restart interval starts after it
//   FF FF      -> fill byte (part of the break that follows)
//   FF other   -> terminating marker (EOI ...): the ECS ends
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kScanThreads) void k_scan(BatchDev b) {
    __shared__ uint32_t s_wsum[2][kScanThreads / 64];
    const ImgDesc& im = b.imgs[blockIdx.y];
    const uint32_t c = blockIdx.x;
    if (c >= im.nchunks) return;
    const uintptr_t file = uintptr_t(im.jpeg);
    const uintptr_t lo = file + im.ecs_off, fend = file + im.len;
    const uintptr_t t0 = (lo & ~uintptr_t(15)) + uintptr_t(c) * kScanChunk + uintptr_t(threadIdx.x) * kScanBytesPerThread;
    uint32_t w[16];
    load64(t0, fend, w);
    const uint32_t prevb = (t0 > lo && t0 - 1 < fend) ? uint32_t(*reinterpret_cast<gu8*>(t0 - 1)) : 0u;
    const uint32_t nextb = (t0 + 64 < fend) ? uint32_t(*reinterpret_cast<gu8*>(t0 + 64)) : 0u;

    uint32_t ndrop = 0, nbrk = 0;
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint32_t by = byte_of(w, i);
        const uint32_t pb = i ? byte_of(w, i - 1) : prevb;
        const uint32_t nb = i < 63 ? byte_of(w, i + 1) : nextb;
        const uintptr_t a = t0 + i;
        const bool inr = a >= lo && a < fend;
        ndrop += (inr && a > lo && by == 0x00u && pb == 0xFFu) ? 1u : 0u;
        nbrk += (inr && a + 1 < fend && by == 0xFFu && nb != 0x00u && nb != 0xFFu) ? 1u : 0u;
    }
    uint32_t tot_drop, tot_brk;
    const uint32_t drop_before = block_excl_scan(ndrop, s_wsum[0], &tot_drop);
    uint32_t off = block_excl_scan(nbrk, s_wsum[1], &tot_brk);
    if (nbrk) {
        Break* out = b.chunk_brk + size_t(im.chunk_base + c) * kScanCap;
        uint32_t d = drop_before;
#pragma unroll
        for (int i = 0; i < 64; i++) {
            const uint32_t by = byte_of(w, i);
            const uint32_t pb = i ? byte_of(w, i - 1) : prevb;
            const uint32_t nb = i < 63 ? byte_of(w, i + 1) : nextb;
            const uintptr_t a = t0 + i;
            const bool inr = a >= lo && a < fend;
            d += (inr && a > lo && by == 0x00u && pb == 0xFFu) ? 1u : 0u;
            if (inr && a + 1 < fend && by == 0xFFu && nb != 0x00u && nb != 0xFFu) {
                const uint32_t is_term = (nb & 0xF8u) == 0xD0u ? 0u : 1u;
                out[off++] = Break{uint32_t(a - file), (d << 1) | is_term};
            }
        }
    }
    if (threadIdx.x == 0) {
        b.chunk_nbrk[im.chunk_base + c] = tot_brk;
        b.chunk_drops[im.chunk_base + c] = tot_drop;
    }
}

// ------------------------------------------------------------------------------------------
// Stage 1: per image (one wave), in un-stuffed ("compacted") coordinates:
//   chunk_coff[c]        = offset of chunk c's first ECS byte
//   seg_cstart[k], [k+1] = interval k+1 starts after the k-th RSTn (in stream order)
//   seg_cend[k]          = interval k's data ends at the first fill byte / marker after it
// The first terminating marker ends the ECS; breaks after it are ignored.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fill_before(uintptr_t file, uint32_t lo, uint32_t pos) {
    uint32_t n = 0;
    while (pos > lo + n && *reinterpret_cast<gu8*>(file + pos - 1 - n) == 0xFFu) n++;
    return n;
}

__global__ __launch_bounds__(64) void k_index(BatchDev b) {
    const uint32_t ii = blockIdx.x;
    const ImgDesc& im = b.imgs[ii];
    const uintptr_t file = uintptr_t(im.jpeg);
    const uint32_t lo = im.ecs_off;
    const uint32_t a0 = uint32_t(((file + lo) & ~uintptr_t(15)) - file);
    const uint32_t cb = im.chunk_base, nch = im.nchunks, nseg = im.nseg, sb = im.seg_base;
    const int lane = threadIdx.x;

    // pass A: first terminating marker
    uint32_t term = 0xFFFFFFFFu;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
        const uint32_t c = c0 + lane;
        if (c < nch) {
            const uint32_t n = b.chunk_nbrk[cb + c];
            const Break* br = b.chunk_brk + size_t(cb + c) * kScanCap;
            for (uint32_t j = 0; j < n; j++)
                if (br[j].info & 1u) {
                    term = min(term, br[j].pos);
                    break;
                }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) term = min(term, uint32_t(__shfl_xor(int(term), d, 64)));

    // pass B: offsets and segment boundaries
    uint32_t drops_run = 0, marks_run = 0;
    uint32_t term_comp = 0xFFFFFFFFu;
    bool order_bad = false;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
        const uint32_t c = c0 + lane;
        const bool vc = c < nch;
        const uint32_t drops = vc ? b.chunk_drops[cb + c] : 0u;
        const uint32_t nbrk = vc ? b.chunk_nbrk[cb + c] : 0u;
        const Break* br = b.chunk_brk + size_t(cb + c) * kScanCap;
        uint32_t nmark = 0;
        for (uint32_t j = 0; j < nbrk; j++) nmark += (!(br[j].info & 1u) && br[j].pos < term) ? 1u : 0u;
        const uint32_t di = wave_incl_scan(drops), mi = wave_incl_scan(nmark);
        const uint32_t dprefix = drops_run + di - drops, mprefix = marks_run + mi - nmark;
        if (vc) {
            const uint32_t clo = max(lo, a0 + c * uint32_t(kScanChunk));
            b.chunk_coff[cb + c] = (clo - lo) - dprefix;
            uint32_t m = mprefix;
            for (uint32_t j = 0; j < nbrk; j++) {
                const Break k = br[j];
                const uint32_t cpos = (k.pos - lo) - (dprefix + (k.info >> 1));
                if (k.info & 1u) {
                    if (k.pos == term) term_comp = cpos - fill_before(file, lo, k.pos);
                    continue;
                }
                if (k.pos >= term) continue;
                if (m < nseg) b.seg_cend[sb + m] = cpos - fill_before(file, lo, k.pos);
                if (m + 1 < nseg) {
                    b.seg_cstart[sb + m + 1] = cpos + 2;
                    if ((*reinterpret_cast<gu8*>(file + k.pos + 1) & 7u) != (m & 7u)) order_bad = true;
                }
                m++;
            }
        }
        drops_run += __shfl(int(di), 63, 64);
        marks_run += __shfl(int(mi), 63, 64);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) term_comp = min(term_comp, uint32_t(__shfl_xor(int(term_comp), d, 64)));
    const uint32_t total = (im.len - lo) - drops_run;  // un-stuffed length of the whole ECS region
    const uint32_t end_all = term_comp != 0xFFFFFFFFu ? term_comp : total;
    if (lane == 0) {
        b.seg_cstart[sb] = 0;
        if (marks_run < nseg) b.seg_cend[sb + marks_run] = end_all;
        if (marks_run + 1 < nseg) atomicOr(&b.status[ii], kStRstMissing);
    }
    for (uint32_t k = marks_run + 1 + lane; k < nseg; k += 64) {
        b.seg_cstart[sb + k] = end_all;
        b.seg_cend[sb + k] = end_all;
    }
    if (__any(order_bad) && lane == 0) atomicOr(&b.status[ii], kStRstOrder);
}

// ------------------------------------------------------------------------------------------
// Stage 2: compaction (un-stuffing).  A chunk's kept bytes are staged in LDS, then written to
// the image's un-stuffed stream with byte stores at the unaligned head/tail and dword stores in
// between, so neighbouring chunks (other workgroups) never share a stored word.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kScanThreads) void k_compact(BatchDev b) {
    __shared__ uint32_t s_out[kScanChunk / 4 + 4];
    __shared__ uint32_t s_wsum[kScanThreads / 64];
    const ImgDesc& im = b.imgs[blockIdx.y];
    const uint32_t c = blockIdx.x;
    if (c >= im.nchunks) return;
    const uintptr_t file = uintptr_t(im.jpeg);
    const uintptr_t lo = file + im.ecs_off, fend = file + im.len;
    const uintptr_t t0 = (lo & ~uintptr_t(15)) + uintptr_t(c) * kScanChunk + uintptr_t(threadIdx.x) * kScanBytesPerThread;
    uint32_t w[16];
    load64(t0, fend, w);
    const uint32_t prevb = (t0 > lo && t0 - 1 < fend) ? uint32_t(*reinterpret_cast<gu8*>(t0 - 1)) : 0u;
    uint64_t keep = 0;
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint32_t by = byte_of(w, i);
        const uint32_t pb = i ? byte_of(w, i - 1) : prevb;
        const uintptr_t a = t0 + i;
        const bool inr = a >= lo && a < fend;
        const bool drop = a > lo && by == 0x00u && pb == 0xFFu;
        if (inr && !drop) keep |= 1ull << i;
    }
    uint32_t total;
    uint32_t off = block_excl_scan(uint32_t(__builtin_popcountll(keep)), s_wsum, &total);
    uint8_t* so = reinterpret_cast<uint8_t*>(s_out);
    if (keep == ~0ull && (off & 3u) == 0u) {  // common case: whole thread kept, aligned in LDS
#pragma unroll
        for (int q = 0; q < 16; q++) s_out[(off >> 2) + q] = w[q];
    } else {
#pragma unroll
        for (int i = 0; i < 64; i++)
            if ((keep >> i) & 1ull) so[off++] = uint8_t(byte_of(w, i));
    }
    __syncthreads();
    uint8_t* dst = reinterpret_cast<uint8_t*>(im.comp) + b.chunk_coff[im.chunk_base + c];
    const uint32_t head = min(total, uint32_t((4u - (reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u));
    if (threadIdx.x < head) dst[threadIdx.x] = so[threadIdx.x];
    const uint32_t nwords = (total - head) >> 2;
    uint32_t* dw = reinterpret_cast<uint32_t*>(dst + head);
    const uint32_t sh = head & 3u;
    for (uint32_t i = threadIdx.x; i < nwords; i += kScanThreads) {
        const uint32_t o = (head >> 2) + i;  // head < 4: word o and o+1 hold bytes head+4i..+3
        dw[i] = __builtin_amdgcn_alignbyte(s_out[o + 1], s_out[o], sh);
    }
    const uint32_t done = head + (nwords << 2);
    if (threadIdx.x < total - done) dst[done + threadIdx.x] = so[done + threadIdx.x];
}

// ------------------------------------------------------------------------------------------
// Stage 3: Huffman decode.  One lane owns one restart interval (segment) and walks it symbol by
// symbol in a single flattened loop (DC and AC steps share one body, so lanes of a wave never
// wait for each other's blocks).
//
// Memory discipline: the decode steps contain NO global loads.  gfx950 counts stores and loads
// on one vmcnt, so any wait for a bitstream load inside the divergent step would also wait for
// every coefficient store in flight — and with 64 lanes some lane needs new bytes almost every
// step.  Each lane's (already un-stuffed) bitstream lives in a 128-byte LDS ring (layout
// [word][lane]: a lane always hits bank lane%32, conflict-free), refilled in a wave-uniform
// service phase every kRound steps: a service commits the 64 bytes loaded by the previous service
// and issues the next load, so every load has a full round to land.  Ring words are stored
// byte-swapped (MSB-first), so a symbol's 32-bit window is two LDS reads and one funnel shift.
// ------------------------------------------------------------------------------------------
constexpr int kRingWords = 32;  // per-lane ring: 128 bytes (+1 mirror word for wrap reads)
constexpr int kRingBytes = kRingWords * 4;
constexpr int kFillBytes = 64;  // bytes fetched per lane per service
constexpr int kRound = 8;       // decode steps between services (<= 32 bytes consumed)

__device__ __forceinline__ u32x4 load16(uintptr_t a, uintptr_t last) {
    // Unconditional (no phi with a fill value, so hipcc does not wait at issue); clamped to the
    // image's last mapped 16-byte chunk.  Bytes past a segment's end are never consumed as data.
    return *reinterpret_cast<gu32x4*>(a < last ? a : last);
}

__device__ __forceinline__ int extend(uint32_t v, int s) {  // utils/stream.cpp:44-52
    if (s == 0) return 0;
    const int l = 1 << (s - 1);
    return int(v) >= l ? int(v) : int(v) - ((l << 1) - 1);
}

struct Lane {
    int bitpos;    // next bit (relative to the lane's 16-byte aligned base)
    int wr;        // ring holds bytes [.., wr)
    int req;       // loads issued up to base + req
    bool pending;  // q0..q3 hold bytes [wr, wr + 64) in flight
};

__device__ __forceinline__ void service(Lane& L, uint32_t* ring, u32x4& q0, u32x4& q1, u32x4& q2, u32x4& q3,
                                        uintptr_t base, uintptr_t last, bool active) {
    if (L.pending) {
        const int w = (L.wr >> 2) & (kRingWords - 1);  // wr is a multiple of 64: no wrap inside
        uint32_t* r = ring + w * kHuffThreads;
        r[0 * kHuffThreads] = __builtin_bswap32(q0.x);
        r[1 * kHuffThreads] = __builtin_bswap32(q0.y);
        r[2 * kHuffThreads] = __builtin_bswap32(q0.z);
        r[3 * kHuffThreads] = __builtin_bswap32(q0.w);
        r[4 * kHuffThreads] = __builtin_bswap32(q1.x);
        r[5 * kHuffThreads] = __builtin_bswap32(q1.y);
        r[6 * kHuffThreads] = __builtin_bswap32(q1.z);
        r[7 * kHuffThreads] = __builtin_bswap32(q1.w);
        r[8 * kHuffThreads] = __builtin_bswap32(q2.x);
        r[9 * kHuffThreads] = __builtin_bswap32(q2.y);
        r[10 * kHuffThreads] = __builtin_bswap32(q2.z);
        r[11 * kHuffThreads] = __builtin_bswap32(q2.w);
        r[12 * kHuffThreads] = __builtin_bswap32(q3.x);
        r[13 * kHuffThreads] = __builtin_bswap32(q3.y);
        r[14 * kHuffThreads] = __builtin_bswap32(q3.z);
        r[15 * kHuffThreads] = __builtin_bswap32(q3.w);
        if (w == 0) ring[kRingWords * kHuffThreads] = __builtin_bswap32(q0.x);  // mirror word
        L.wr += kFillBytes;
    }
    // the bytes requested now land at the next service over ring bytes [req-128, req-64)
    L.pending = active && (L.req - ((L.bitpos >> 5) << 2) <= kRingBytes - kFillBytes);
    const uintptr_t a = base + uintptr_t(L.req);
    q0 = load16(a, last);
    q1 = load16(a + 16, last);
    q2 = load16(a + 32, last);
    q3 = load16(a + 48, last);
    if (L.pending) L.req += kFillBytes;
}

// One Huffman symbol (+ magnitude bits) from the 32-bit window `peek`: symbol, EXTENDed value,
// bits consumed.
__device__ __forceinline__ int decode_sym(uint32_t peek, const HuffLut* t, bool is_dc, int& sym, int& val, bool& bad) {
    const uint32_t e = t->fast[peek >> (32 - kLutBits)];
    int len;
    if (e & 31u) {
        len = int(e & 31u);
        sym = int((e >> 8) & 255u);
        val = int32_t(e) >> 16;
        if (e & kLutFlagComplete) return len;
    } else {  // code longer than kLutBits (or invalid): canonical limits, F.2.2.3
        // lim[] is non-decreasing, so the code length is kLutBits+1 plus the number of limits
        // <= v16: independent LDS reads, no dependent search loop.
        const uint32_t v16 = peek >> 16;
        int l = kLutBits + 1;
#pragma unroll
        for (int j = kLutBits + 1; j <= 16; j++) l += (v16 >= t->lim[j]) ? 1 : 0;
        if (l > 16) {
            bad = true;
            l = 16;
            sym = 0;
        } else {
            sym = t->vals[(t->base[l] + int(v16 >> (16 - l))) & 255];
        }
        len = l;
    }
    int s = is_dc ? sym : (sym & 15);
    if (s > 16) {
        bad = true;
        s = 16;
    }
    const uint32_t bits = s ? ((peek << len) >> (32 - s)) : 0u;
    val = extend(bits, s);
    return len + s;
}

__global__ __launch_bounds__(kHuffThreads) void k_huffman(BatchDev b) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    HuffLut* s_lut = reinterpret_cast<HuffLut*>(s_dyn);
    uint32_t* s_ring = reinterpret_cast<uint32_t*>(s_dyn + size_t(b.max_slots) * sizeof(HuffLut));
    const TableSet& ts = b.tablesets[b.wg_tableset[blockIdx.x]];
    for (int slot = 0; slot < ts.nslots; slot++) {
        const uint4* src = reinterpret_cast<const uint4*>(b.luts + ts.lut[slot]);
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
    uint32_t cstart = 0, cend = 0;
    if (valid) {
        const uint32_t k_seg = g - im.seg_base;
        const uint32_t nmcu = im.mcux * im.mcuy;
        const uint32_t ri = im.restart_interval;
        const uint32_t mcu0 = ri ? k_seg * ri : 0u;
        const uint32_t mcu1 = ri ? min(mcu0 + ri, nmcu) : nmcu;
        cstart = b.seg_cstart[g];
        cend = max(cstart, b.seg_cend[g]);
        gblk = im.block_base + uint64_t(mcu0) * im.bpm;
        gend = im.block_base + uint64_t(mcu1) * im.bpm;
    }
    const uintptr_t comp = valid ? uintptr_t(im.comp) : uintptr_t(b.imgs);
    const uintptr_t last = valid ? ((comp + (im.len - im.ecs_off) + 63) & ~uintptr_t(15)) : (comp & ~uintptr_t(15));
    const uintptr_t base = (comp + cstart) & ~uintptr_t(15);
    const int bit0 = int((comp + cstart) & 15) * 8;
    const int bit_end = bit0 + int(cend - cstart) * 8;

    Lane L;
    L.bitpos = bit0;
    L.wr = 0;
    L.req = 0;
    L.pending = false;
    u32x4 q0, q1, q2, q3;
    service(L, ring, q0, q1, q2, q3, base, last, valid);
    service(L, ring, q0, q1, q2, q3, base, last, valid);

    const int d0 = ts.dc_slot[0], d1 = ts.dc_slot[1], d2 = ts.dc_slot[2];
    const int a0 = ts.ac_slot[0], a1 = ts.ac_slot[1], a2 = ts.ac_slot[2];
    const uint32_t pattern = im.block_pattern, bpm = im.bpm;
    uint32_t bi = 0;
    int comp_id = int(pattern & 3u);
    int k = 0, p0 = 0, p1 = 0, p2 = 0, dc = 0;
    const uint32_t ent_first = valid ? b.seg_entry[g] : 0u;
    uint32_t ent = ent_first, ent0 = ent_first;
    bool bad = false;

    for (;;) {
        const bool active = gblk < gend;
        if (!__any(active)) break;
        service(L, ring, q0, q1, q2, q3, base, last, active);
        for (int it = 0; it < kRound; it++) {
            if (gblk < gend && ((L.bitpos >> 5) << 2) + 8 <= L.wr) {
                const int w = (L.bitpos >> 5) & (kRingWords - 1);
                const uint32_t w0 = ring[w * kHuffThreads];
                const uint32_t w1 = ring[(w + 1) * kHuffThreads];
                const uint32_t sh = uint32_t(L.bitpos) & 31u;
                const uint32_t al = __builtin_amdgcn_alignbit(w0, w1, 32u - sh);
                const uint32_t peek = sh ? al : w0;
                const bool is_dc = (k == 0);
                const int slot = is_dc ? (comp_id == 0 ? d0 : (comp_id == 1 ? d1 : d2))
                                       : (comp_id == 0 ? a0 : (comp_id == 1 ? a1 : a2));
                int sym, val;
                L.bitpos += decode_sym(peek, &s_lut[slot], is_dc, sym, val, bad);
                if (is_dc) {  // parser.cpp:106-111: DPCM
                    const int pr = (comp_id == 0 ? p0 : (comp_id == 1 ? p1 : p2)) + val;
                    if (comp_id == 0) p0 = pr;
                    else if (comp_id == 1) p1 = pr;
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
                    comp_id = int((pattern >> (2 * bi)) & 3u);
                    k = 0;
                }
            }
        }
    }
    if (!valid) return;
    if (L.bitpos > bit_end) bad = true;  // consumed bits beyond the interval's data
    if (bad) atomicOr(&b.status[ii], kStCorrupt);
    atomicAdd(&b.counters[0], (unsigned long long)(ent - ent_first));
}

// ------------------------------------------------------------------------------------------
// Stage 4: dequantise + IDCT + upsample + colour.
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

// One workgroup per tile: 128 px wide x (16 px, or one MCU row when MCUs are 32 px tall).
// Phases: zero LDS tile -> sparse entries to dense dequantised blocks (4 lanes per block) -> row
// IDCT (one lane per block row) -> column IDCT -> colour, where each lane owns 8 consecutive
// pixels of one row and stores them as 24 contiguous bytes (3 x 8-byte stores when aligned).
__global__ __launch_bounds__(kIdctThreads) void k_idct_color(BatchDev b) {
    __shared__ int s_coef[kTileMaxBlocks * 64];
    __shared__ int s_q[3][64];
    const ImgDesc& im = b.imgs[blockIdx.y];
    const uint32_t tile = blockIdx.x;
    const uint32_t tiles_x = im.tiles_x;
    if (tile >= tiles_x * im.tiles_y) return;
    const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const uint32_t T = im.tile_mcus, R = im.tile_mrows;
    const uint32_t m0 = tx * T, r0 = ty * R;
    const uint32_t nm = min(T, im.mcux - m0), nr = min(R, im.mcuy - r0);
    const uint32_t bpm = im.bpm, nblk = T * R * bpm;
    const int tid = threadIdx.x;

    for (uint32_t i = tid; i < nblk * 16; i += kIdctThreads)
        reinterpret_cast<int4*>(s_coef)[i] = make_int4(0, 0, 0, 0);
    if (tid < int(im.ncomp) * 64) {
        const int c = tid >> 6, z = tid & 63;
        s_q[c][z] = int(b.qtabs[size_t(im.qslot[c]) * 64 + z]);
    }
    __syncthreads();

    // sparse -> dense, dequantised in zig-zag order (parser.cpp:111,130), natural placement
    for (uint32_t j = uint32_t(tid) >> 2; j < nblk; j += kIdctThreads / 4) {
        const uint32_t m = j / bpm, bb = j - m * bpm;
        const uint32_t mr = m / T, mi = m - mr * T;
        if (mi >= nm || mr >= nr) continue;
        const uint32_t sub = uint32_t(tid) & 3;
        const uint32_t comp = (im.block_pattern >> (2 * bb)) & 3u;
        const uint64_t gb = im.block_base + uint64_t((r0 + mr) * im.mcux + m0 + mi) * bpm + bb;
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
    __syncthreads();
    for (uint32_t r = tid; r < nblk * 8; r += kIdctThreads) idct_row(s_coef + r * 8);
    __syncthreads();
    for (uint32_t c = tid; c < nblk * 8; c += kIdctThreads) idct_col(s_coef + (c >> 3) * 64 + (c & 7));
    __syncthreads();

    const uint32_t lg_mw = im.lg_mw, lg_mh = im.lg_mh;
    const uint32_t rows = R << lg_mh;  // tile rows
    const uint32_t W = im.width, H = im.height, nc = im.ncomp;
    const uint32_t x_tile = m0 << lg_mw, y_tile = r0 << lg_mh;
    uint8_t* out = reinterpret_cast<uint8_t*>(im.rgb);
    for (uint32_t it = tid; it < rows * (kTileWidth / 8); it += kIdctThreads) {
        const uint32_t py = it >> 4, gx = (it & 15u) << 3;
        const uint32_t y = y_tile + py, x = x_tile + gx;
        if (y >= H || x >= W) continue;
        const uint32_t mr = py >> lg_mh, uy = py & ((1u << lg_mh) - 1);
        const uint32_t mi = gx >> lg_mw, ux0 = gx & ((1u << lg_mw) - 1);
        const uint32_t mcu_base = (mr * T + mi) * bpm;
        int sbase[3], ssh[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const uint32_t sy = uy >> im.shy[c];
            sbase[c] = int((mcu_base + im.comp_block0[c] + (sy >> 3) * im.h[c]) * 64 + (sy & 7) * 8);
            ssh[c] = im.shx[c];
        }
        uint32_t rgb[8][3];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            int s3[3];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const uint32_t sx = (ux0 + j) >> ssh[c];
                s3[c] = (uint32_t(c) < nc) ? s_coef[sbase[c] + int((sx >> 3) * 64 + (sx & 7))] : 0;
            }
            color_px(s3[0], s3[1], s3[2], rgb[j][0], rgb[j][1], rgb[j][2]);
        }
        uint8_t* dst = out + (size_t(y) * W + x) * 3;
        const uintptr_t ad = reinterpret_cast<uintptr_t>(dst);
        if (x + 8 <= W && (ad & 3) == 0) {
            uint32_t w[6];
#pragma unroll
            for (int q = 0; q < 6; q++) {
                uint32_t v = 0;
#pragma unroll
                for (int bb = 0; bb < 4; bb++) v |= rgb[(4 * q + bb) / 3][(4 * q + bb) % 3] << (8 * bb);
                w[q] = v;
            }
            if ((ad & 7) == 0) {
                uint2* d2 = reinterpret_cast<uint2*>(dst);
                d2[0] = make_uint2(w[0], w[1]);
                d2[1] = make_uint2(w[2], w[3]);
                d2[2] = make_uint2(w[4], w[5]);
            } else {
                uint32_t* d1 = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
                for (int q = 0; q < 6; q++) d1[q] = w[q];
            }
        } else {
            const uint32_t n = min(8u, W - x);
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (uint32_t(j) < n) {
                    dst[3 * j] = uint8_t(rgb[j][0]);
                    dst[3 * j + 1] = uint8_t(rgb[j][1]);
                    dst[3 * j + 2] = uint8_t(rgb[j][2]);
                }
        }
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
hipError_t launch_scan(const BatchDev& b, hipStream_t s) {
    if (!b.nimg || !b.max_chunks) return hipSuccess;
    hipLaunchKernelGGL(k_scan, dim3(b.max_chunks, b.nimg), dim3(kScanThreads), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_index(const BatchDev& b, hipStream_t s) {
    if (!b.nimg) return hipSuccess;
    hipLaunchKernelGGL(k_index, dim3(b.nimg), dim3(64), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_compact(const BatchDev& b, hipStream_t s) {
    if (!b.nimg || !b.max_chunks) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3(b.max_chunks, b.nimg), dim3(kScanThreads), 0, s, b);
    return hipGetLastError();
}

size_t huffman_lds_bytes(uint32_t max_slots) {
    return size_t(max_slots) * sizeof(HuffLut) + size_t(kRingWords + 1) * kHuffThreads * 4;
}

hipError_t launch_huffman(const BatchDev& b, hipStream_t s) {
    if (!b.nseg) return hipSuccess;
    hipLaunchKernelGGL(k_huffman, dim3(b.nseg / kHuffThreads), dim3(kHuffThreads), huffman_lds_bytes(b.max_slots), s, b);
    return hipGetLastError();
}

hipError_t launch_idct_color(const BatchDev& b, hipStream_t s) {
    if (!b.nimg || !b.max_tiles) return hipSuccess;
    hipLaunchKernelGGL(k_idct_color, dim3(b.max_tiles, b.nimg), dim3(kIdctThreads), 0, s, b);
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
