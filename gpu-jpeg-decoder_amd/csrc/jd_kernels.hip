// jd_kernels.hip — gfx950 (CDNA4, wave64) kernels of the batched JPEG decode path, in launch order
// (launch_kernel's slots; DESIGN.md §4.2 gives each one's work unit, bytes and bound):
//
//   k_scan         16 KiB of ECS per 256-thread workgroup: stuffed-zero counts, RSTn / terminator
//                  positions (SWAR byte masks)
//   k_index        one wave per image: chunk offsets in the un-stuffed stream, restart-interval
//                  (segment) boundaries, RSTn order / count checks
//   k_compact      16 KiB per workgroup: drops the stuffed 00 after every FF (byte compaction)
//   k_pieceplan    one workgroup: the piece size for the batch (whole rounds of resident lanes)
//   k_subplan      one wave per image: pieces (<= piece_bits un-stuffed bits) of every interval
//   k_piece        one lane per piece: a speculative, self-synchronising Huffman walk (warm-up
//                  from before the piece, then block records + sparse AC entries into the piece's
//                  own region, checkpoints); k_redo re-walks the pieces whose speculative start
//                  was wrong (joining the speculative walk at a checkpoint); k_chain / k_chain_fix
//                  verify the chain of pieces and prefix-sum each piece's first MCU
//   k_gather       64 pieces per wave (one row of 16 lanes per piece): block records -> BlockInfo
//                  (DC difference, entry range) at the blocks' global positions
//   k_dc_sum / k_dc_scan   DC predictors at every IDCT tile's first block
//   k_idct_color   one wave per tile (a run of <= 64 blocks of one MCU row): DC prediction,
//                  dequantisation, integer IDCT in registers, replicate chroma upsampling and
//                  YCbCr->RGB -> uint8 HWC; k_idct_color_exact takes the (never seen) tiles whose
//                  coefficients are beyond the fast IDCT form's range
//   k_colour_fancy (JD_FLAG_FANCY_UPSAMPLING only) libjpeg's triangular upsampling + colour
//
// Arithmetic follows the reference CPU decoder bit for bit (cpp-decoder/src/idct.cpp,
// utils/color.cpp); the restatement used as checker lives in oracle/ (tests only).
#include <hip/hip_runtime.h>
#include <mutex>
#include <type_traits>

#include "jd_kernels.hpp"

#pragma clang fp contract(off)

namespace jd {

// Wave priority of the latency-bound kernels.  Two batches are in flight: batch k's
// re-walks (k_redo: a few lanes with long serial walks) and short kernels share the CUs with batch
// k+1's k_piece or batch k-1's k_idct_color, whose 16-20 waves per CU would otherwise take most
// issue slots and stretch k_redo from 0.4 to 2.5 ms on the critical path.  s_setprio raises the
// issue priority of their waves over the two big kernels' waves on the same SIMD.
#ifndef JD_PRIO
#define JD_PRIO 1  // 0: off, 1: k_redo / k_chain / k_chain_fix, 2: every kernel but k_piece / k_idct_color
                   // (2 made k_dc_sum 40 % slower)
#endif
#define JD_PRIO_CRIT() do { if (JD_PRIO >= 1) __builtin_amdgcn_s_setprio(3); } while (0)
#define JD_PRIO_SHORT() do { if (JD_PRIO >= 2) __builtin_amdgcn_s_setprio(2); } while (0)


// zig-zag index -> natural (row-major) position: inverse of src/idct.cpp:8-16.
// constexpr: fully unrolled loops index it at compile time (register naming, no lookups)
constexpr uint8_t kNatOfZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18,
                                     11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                                     13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43,
                                     36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                                     38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint8_t gu8;
// Output pointers as global (not flat) addresses: a flat store also counts on lgkmcnt, so every
// LDS wait after it would wait for the store too.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

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

// The same inclusive scan in six DPP adds (no LDS traffic): Hillis-Steele within each row of 16
// lanes (row_shr 1, 2, 4, 8), then row_bcast 15 / 31 carry rows into the rows above.  Every lane
// of the wave must be active.
__device__ __forceinline__ int wave_scan_dpp(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15, rows 1 and 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31, rows 2 and 3
    return x;
}

// Exclusive scan over a 256-thread block; returns the exclusive prefix, *total the block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t incl = uint32_t(wave_scan_dpp(int(x)));  // (every thread of the block calls this)
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

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[16], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; }

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

// load64 again, as a fresh load (k_scan's edge threads: the count pass's words are not kept alive)
__device__ __forceinline__ void reload64(uintptr_t t0, uintptr_t fend, uint32_t (&w)[16]) {
    asm("" : "+v"(t0));
    load64(t0, fend, w);
}

// ------------------------------------------------------------------------------------------
// Stage 0: scan.  In an ECS a data FF is always followed by a stuffed 00, so:
//   FF 00      -> the 00 is dropped by un-stuffing (the reference's loop, parser.cpp:84-96)
//   FF D0..D7  -> RSTn marker: the next restart interval starts after it
//   FF FF      -> fill byte (part of the break that follows)
//   FF other   -> terminating marker (EOI ...): the ECS ends
// ------------------------------------------------------------------------------------------
// Per-byte masks of a word (high bit of each byte lane): returns byte == 0x00; ff: byte == 0xFF;
// nz: neither 00 nor FF.
__device__ __forceinline__ uint32_t scan_masks(uint32_t x, uint32_t& ff, uint32_t& nz) {
    const uint32_t t = ~x;
    ff = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    const uint32_t zero = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    nz = ~(zero | ff) & 0x80808080u;
    return zero;
}

__device__ void subplan_image(const BatchDev& b, uint32_t img, int lane);  // (below, with k_subplan)

__global__ __launch_bounds__(kScanThreads) void k_scan(BatchDev b) {
    JD_PRIO_SHORT();
    __shared__ uint32_t s_wsum[2][kScanThreads / 64];
    // every piece slot reads invalid until k_subplan (or k_compact's subplan) claims it for an
    // interval: the slots of per-image slack and padding stay so.  A slot per thread of the grid (a
    // memset launch cost a single-image decode ~5 us on its critical path)
    {
        const uint64_t g = (uint64_t(blockIdx.y) * gridDim.x + blockIdx.x) * kScanThreads + threadIdx.x;
        const uint64_t stride = uint64_t(gridDim.x) * gridDim.y * kScanThreads;  // (64-bit: never wraps)
        for (uint64_t u = g; u < b.nsub; u += stride) b.sub_seg[u] = kInvalidImage;
    }
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
    const bool interior = t0 >= lo && t0 + 64 < fend;
    // interior thread: exact per-byte masks (high bit of each byte lane), one word at a time with
    // the neighbours' masks carried
    //   drop : 00 preceded by FF       brk : FF followed by neither 00 nor FF, or FF 00 preceded
    //                                        by FF (a run of FFs that ends in 00 is no stuffing but a
    //                                        marker at its first FF: the oracle's reader stops there,
    //                                        jdoracle.c br_fetch; never in a valid stream)
    // Only which words hold a break (brkw) and the stuffed zeros before each word (cum, a byte per
    // word) are kept for the break walk below, which recomputes the masks of those words alone:
    // keeping both masks of all 16 words took 84 VGPRs, so only one workgroup per CU fitted beside
    // k_idct_color (112 VGPRs per SIMD left), and the next batch's scan ran one chunk per CU at a time
    // (computed in every thread, so that nothing needs a zero-initialised copy for the edge threads,
    // which count byte by byte below instead)
    uint32_t brkw = 0, cum[4];
    {
        uint32_t ff_prev = (prevb == 0xFFu) ? 0x80000000u : 0u;  // only its top byte is used
        uint32_t ff_cur, nz_cur;
        uint32_t zero_cur = scan_masks(w[0], ff_cur, nz_cur);
        const uint32_t nznext = (nextb != 0x00u && nextb != 0xFFu) ? 0x80u : 0u;  // byte after it
        const uint32_t znext = (nextb == 0x00u) ? 0x80u : 0u;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            uint32_t ff_nx = 0, nz_nx = nznext, zero_nx = znext;
            if (q < 15) zero_nx = scan_masks(w[q + 1], ff_nx, nz_nx);
            const uint32_t ffb = __builtin_amdgcn_alignbit(ff_cur, ff_prev, 24);  // byte before is FF: (ff_cur << 8) | (ff_prev >> 24)
            const uint32_t dm = zero_cur & ffb;
            const uint32_t bm = ff_cur & (__builtin_amdgcn_alignbit(nz_nx, nz_cur, 8) |  // (nz_cur >> 8) | (nz_nx << 24)
                                          (__builtin_amdgcn_alignbit(zero_nx, zero_cur, 8) & ffb));
            cum[q >> 2] = (q & 3) ? (cum[q >> 2] | (ndrop << (8 * (q & 3)))) : ndrop;
            ndrop += __builtin_popcount(dm);
            nbrk += __builtin_popcount(bm);
            brkw |= min(bm, 1u) << q;
            // (brkw and cum built here: left to itself the compiler sinks them past the block scan and
            // keeps every word's break mask and drop prefix alive until then: 71 VGPRs)
            asm volatile("" : "+v"(brkw), "+v"(cum[q >> 2]));
            ff_prev = ff_cur;
            ff_cur = ff_nx;
            nz_cur = nz_nx;
            zero_cur = zero_nx;
        }
    }
    if (!interior) {
        ndrop = nbrk = 0;
        reload64(t0, fend, w);
#pragma unroll 1
        for (int i = 0; i < 64; i++) {
            const uint32_t by = byte_of(w, i);
            const uint32_t pb = i ? byte_of(w, i - 1) : prevb;
            const uint32_t nb = i < 63 ? byte_of(w, i + 1) : nextb;
            const uintptr_t a = t0 + i;
            const bool inr = a >= lo && a < fend;
            ndrop += (inr && a > lo && by == 0x00u && pb == 0xFFu) ? 1u : 0u;
            nbrk += (inr && a + 1 < fend && by == 0xFFu &&
                     ((nb != 0x00u && nb != 0xFFu) || (nb == 0x00u && a > lo && pb == 0xFFu))) ? 1u : 0u;
        }
    }
    uint32_t tot_drop, tot_brk;
    const uint32_t drop_before = block_excl_scan(ndrop, s_wsum[0], &tot_drop);
    uint32_t off = block_excl_scan(nbrk, s_wsum[1], &tot_brk);
    if (nbrk && interior) {
        // walk the break bits only, in the words that hold one (a word without a break in any lane
        // of the wave costs two instructions); their masks recomputed as in the count pass
        Break* out = b.chunk_brk + size_t(im.chunk_base + c) * b.brk_cap;
        const uint32_t cap = b.brk_cap;  // (breaks past it are counted, not stored: k_index)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            if (__any((brkw >> q) & 1u)) {
                // (the words loaded again: the L1 / L2 still hold them, and keeping the count pass's
                // words or masks alive for this is what the recomputation is to avoid)
                uintptr_t aq = t0 + 4u * q;
                asm("" : "+v"(aq));  // (a fresh load, not the count pass's value kept alive)
                const uint32_t wc = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(aq);
                const uint32_t wp = q > 0 ? *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(aq - 4) : 0u;
                const uint32_t wn = q < 15 ? *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(aq + 4) : 0u;
                uint32_t ff, nz, ffp = (prevb == 0xFFu) ? 0x80000000u : 0u, nzp, ffn, nzn = (nextb != 0x00u && nextb != 0xFFu) ? 0x80u : 0u;
                uint32_t zn = (nextb == 0x00u) ? 0x80u : 0u;
                const uint32_t zero = scan_masks(wc, ff, nz);
                if (q > 0) (void)scan_masks(wp, ffp, nzp);
                if (q < 15) zn = scan_masks(wn, ffn, nzn);
                const uint32_t ffb = __builtin_amdgcn_alignbit(ff, ffp, 24);
                const uint32_t dm = zero & ffb;
                uint32_t bm = ff & (__builtin_amdgcn_alignbit(nzn, nz, 8) | (__builtin_amdgcn_alignbit(zn, zero, 8) & ffb));
                const uint32_t d = drop_before + ((cum[q >> 2] >> (8 * (q & 3))) & 0xFFu);
                while (bm) {
                    const uint32_t bit = __builtin_ctz(bm);  // 7, 15, 23 or 31: byte k = bit >> 3
                    const uint32_t k = bit >> 3;
                    const uint32_t nbv = k < 3u ? (wc >> (8u * (k + 1u))) & 0xFFu : (q < 15 ? wn & 0xFFu : nextb);
                    const uint32_t dd = d + __builtin_popcount(dm & ((1u << bit) - 1u));
                    const uint32_t is_term = (nbv & 0xF8u) == 0xD0u ? 0u : 1u;
                    if (off < cap) out[off] = brk_make(threadIdx.x * uint32_t(kScanBytesPerThread) + 4u * q + k, dd, is_term);
                    off++;
                    bm &= bm - 1u;
                }
            }
        }
    } else if (nbrk) {  // edge threads: byte by byte
        Break* out = b.chunk_brk + size_t(im.chunk_base + c) * b.brk_cap;
        uint32_t d = drop_before;
        reload64(t0, fend, w);
#pragma unroll 1
        for (int i = 0; i < 64; i++) {
            const uint32_t by = byte_of(w, i);
            const uint32_t pb = i ? byte_of(w, i - 1) : prevb;
            const uint32_t nb = i < 63 ? byte_of(w, i + 1) : nextb;
            const uintptr_t a = t0 + i;
            const bool inr = a >= lo && a < fend;
            d += (inr && a > lo && by == 0x00u && pb == 0xFFu) ? 1u : 0u;
            if (inr && a + 1 < fend && by == 0xFFu && ((nb != 0x00u && nb != 0xFFu) || (nb == 0x00u && a > lo && pb == 0xFFu))) {
                const uint32_t is_term = (nb & 0xF8u) == 0xD0u ? 0u : 1u;
                if (off < b.brk_cap) out[off] = brk_make(threadIdx.x * uint32_t(kScanBytesPerThread) + uint32_t(i), d, is_term);
                off++;
            }
        }
    }
    if (threadIdx.x == 0) {
        b.chunk_nbrk[im.chunk_base + c] = tot_brk;  // (all of them: k_index reads at most brk_cap)
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
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, uint32_t(__shfl_xor(int(x), o, 64)));
    return x;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, uint32_t(__shfl_xor(int(x), o, 64)));
    return x;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += uint32_t(__shfl_xor(int(x), o, 64));
    return x;
}

// Piece-size candidates of a large batch (k_pieceplan): P = piece_bits * (8 + c) / 8, c < kPlanCands.
constexpr int kPlanCands = 16;
__device__ __forceinline__ uint32_t plan_cand(uint32_t piece_bits, int c) { return piece_bits * uint32_t(8 + c) / 8u; }
// Pieces of an interval of `bits` bits at piece size p: ceil(bits / p), at least 1 (k_subplan's count).
__device__ __forceinline__ uint32_t pieces_of(uint32_t bits, uint32_t p) {
    const uint32_t q = bits / p;
    return max(1u, q + (q * p != bits ? 1u : 0u));
}
// The same from a float reciprocal of p: the estimate is within one of bits / p (q < 2^23), then
// corrected exactly.
__device__ __forceinline__ uint32_t pieces_of_rcp(uint32_t bits, uint32_t p, float inv) {
    int64_t q = int64_t(float(bits) * inv);
    const int64_t r = int64_t(bits) - q * int64_t(p);
    q += r < 0 ? -1 : (r >= int64_t(p) ? 1 : 0);
    return max(1u, uint32_t(q) + (uint64_t(q) * p != bits ? 1u : 0u));
}

__device__ __forceinline__ uint32_t fill_before(uintptr_t file, uint32_t lo, uint32_t pos) {
    uint32_t n = 0;
    while (pos > lo + n && *reinterpret_cast<gu8*>(file + pos - 1 - n) == 0xFFu) n++;
    return n;
}

__global__ __launch_bounds__(64) void k_index(BatchDev b) {
    JD_PRIO_SHORT();
    const uint32_t ii = blockIdx.x;

    const ImgDesc& im = b.imgs[ii];
    const uintptr_t file = uintptr_t(im.jpeg);
    const uint32_t lo = im.ecs_off;
    const uint32_t a0 = uint32_t(((file + lo) & ~uintptr_t(15)) - file);
    const uint32_t cb = im.chunk_base, nch = im.nchunks, nseg = im.nseg, sb = im.seg_base;
    const int lane = threadIdx.x;

    // pass A: first terminating marker.  A chunk may hold more breaks than its brk_cap slots (the
    // optimistic cap: the batch's most intervals + kBrkSlack); those past the cap were counted, not
    // stored, and they come after the stored ones in stream order.  They are harmless when the chunk
    // starts after the first terminator or stored one itself (every later break is ignored); else
    // the image is flagged kStOverflow and decoded again with kScanCap slots per chunk.
    const uint32_t cap = b.brk_cap;
    uint32_t term = 0xFFFFFFFFu, ovf_from = 0xFFFFFFFFu;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
        const uint32_t c = c0 + lane;
        if (c < nch) {
            const uint32_t nt = b.chunk_nbrk[cb + c], n = min(nt, cap);
            const Break* br = b.chunk_brk + size_t(cb + c) * cap;
            bool has_term = false;
            for (uint32_t j = 0; j < n; j++)
                if (brk_term(br[j])) {
                    term = min(term, a0 + c * uint32_t(kScanChunk) + brk_rel(br[j]));
                    has_term = true;
                    break;
                }
            if (nt > cap && !has_term) ovf_from = min(ovf_from, a0 + c * uint32_t(kScanChunk));
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        term = min(term, uint32_t(__shfl_xor(int(term), d, 64)));
        ovf_from = min(ovf_from, uint32_t(__shfl_xor(int(ovf_from), d, 64)));
    }
    if (ovf_from < term && lane == 0) atomicOr(&b.status[ii], kStOverflow);

    // pass B: offsets and segment boundaries
    uint32_t drops_run = 0, marks_run = 0;
    uint32_t term_comp = 0xFFFFFFFFu;
    bool order_bad = false;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
        const uint32_t c = c0 + lane;
        const bool vc = c < nch;
        const uint32_t drops = vc ? b.chunk_drops[cb + c] : 0u;
        const uint32_t nbrk = vc ? min(b.chunk_nbrk[cb + c], cap) : 0u;
        const Break* br = b.chunk_brk + size_t(cb + c) * cap;
        uint32_t nmark = 0;
        const uint32_t cpos0 = a0 + c * uint32_t(kScanChunk);  // file offset of the chunk's first byte
        for (uint32_t j = 0; j < nbrk; j++) nmark += (!brk_term(br[j]) && cpos0 + brk_rel(br[j]) < term) ? 1u : 0u;
        const uint32_t di = wave_incl_scan(drops), mi = wave_incl_scan(nmark);
        const uint32_t dprefix = drops_run + di - drops, mprefix = marks_run + mi - nmark;
        if (vc) {
            const uint32_t clo = max(lo, a0 + c * uint32_t(kScanChunk));
            b.chunk_coff[cb + c] = (clo - lo) - dprefix;
            uint32_t m = mprefix;
            for (uint32_t j = 0; j < nbrk; j++) {
                const Break k = br[j];
                const uint32_t kpos = cpos0 + brk_rel(k);  // file offset of the FF
                const uint32_t cpos = (kpos - lo) - (dprefix + brk_drops(k));
                if (brk_term(k)) {
                    if (kpos == term) term_comp = cpos - fill_before(file, lo, kpos);
                    continue;
                }
                if (kpos >= term) continue;
                if (m < nseg) b.seg_cend[sb + m] = cpos - fill_before(file, lo, kpos);
                if (m + 1 < nseg) {
                    b.seg_cstart[sb + m + 1] = cpos + 2;
                    if ((*reinterpret_cast<gu8*>(file + kpos + 1) & 7u) != (m & 7u)) order_bad = true;
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
    if (!b.piece_plan) return;
    // large batches: the image's pieces at each of k_pieceplan's candidate piece sizes (exact, as
    // k_subplan will count them), so that k_pieceplan only sums per image and k_subplan needs no
    // allocation atomic (1 024 images on one table set's cursor took ~60 us, serialised)
    // this wave's seg_cstart / seg_cend stores are read back by other lanes of the wave: wait until
    // the L2 has them (vmcnt(0); __threadfence's L2 write-back cost ~20 us here) and read past the L1
    // (the immediate is gfx9's vmcnt(0) encoding, where stores count on vmcnt too: ADVICE r05)
#if !defined(__HIP_DEVICE_COMPILE__) || defined(__GFX9__)
    __builtin_amdgcn_s_waitcnt(0x0F70);
#else
#error "k_index: the vmcnt(0) wait is written for gfx9 (gfx950)"
#endif
    // lane = candidate c (lane & 15) over every 4th interval (lane >> 4): few registers, so that
    // k_index still fits beside a walk (64 VGPRs per SIMD left)
    const uint32_t p = plan_cand(b.piece_bits, lane & 15);
    const float inv = 1.0f / float(p);
    uint32_t cnt = 0;
#pragma unroll 4
    for (uint32_t k = uint32_t(lane) >> 4; k < nseg; k += 4) {
        const uint32_t cs = __hip_atomic_load(b.seg_cstart + sb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t ce = max(cs, __hip_atomic_load(b.seg_cend + sb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        cnt += pieces_of_rcp((ce - cs) * 8, p, inv);
    }
    cnt += uint32_t(__shfl_xor(int(cnt), 16, 64));
    cnt += uint32_t(__shfl_xor(int(cnt), 32, 64));
    if (lane < kPlanCands) b.img_cand[size_t(ii) * kPlanCands + lane] = cnt;
}

// ------------------------------------------------------------------------------------------
// Stage 2: compaction (un-stuffing).  A chunk's kept bytes are staged in LDS, then written to
// the image's un-stuffed stream with byte stores at the unaligned head/tail and dword stores in
// between, so neighbouring chunks (other workgroups) never share a stored word.
// ------------------------------------------------------------------------------------------
// Bytes [0, n) of c (a thread's kept bytes, contiguous in the run), n >= 60, to LDS bytes
// [off, off + n): aligned dword stores for every word wholly inside the run, byte stores at its
// two ends (the neighbouring threads own the other bytes of those two words).
__device__ __forceinline__ void store_run(uint32_t* s_out, uint32_t off, const uint32_t (&c)[16], uint32_t n) {
    uint8_t* so = reinterpret_cast<uint8_t*>(s_out);
    const uint32_t a = (4u - (off & 3u)) & 3u;  // bytes before the first aligned word
    const uint32_t wb = (off + a) >> 2, nf = (n - a) >> 2, t = a + 4u * nf;
#pragma unroll
    for (int j = 0; j < 3; j++)
        if (uint32_t(j) < a) so[off + j] = uint8_t(c[0] >> (8 * j));
#pragma unroll
    for (int k = 0; k < 16; k++)  // run bytes [a + 4k, a + 4k + 4)
        if (uint32_t(k) < nf) s_out[wb + k] = __builtin_amdgcn_alignbyte(k < 15 ? c[k < 15 ? k + 1 : k] : 0u, c[k], a);
#pragma unroll
    for (int j = 56; j < 64; j++)  // the tail: at most 3 bytes, all at j >= n - 3 >= 57
        if (uint32_t(j) >= t && uint32_t(j) < n) so[off + j] = uint8_t(c[j >> 2] >> (8 * (j & 3)));
}

// Stuffed zeros per thread (64 bytes) removed in registers, one pass over the words each (a pass
// runs when any lane of the wave has that many); a thread with more takes the byte-wise path.
// Entropy-coded data has an FF (so a stuffed 00) in about 1 byte of 256: with 2, 13 % of the waves
// had a lane beyond it and ran the byte path (~860 VALU); with 4, 0.04 %.
constexpr int kFastDrops = 4;
__global__ __launch_bounds__(kScanThreads) void k_compact(BatchDev b) {
    JD_PRIO_SHORT();
    __shared__ uint32_t s_out[kScanChunk / 4 + 4];
    __shared__ uint32_t s_wsum[kScanThreads / 64];
    const ImgDesc& im = b.imgs[blockIdx.y];
    const uint32_t c = blockIdx.x;
    if (b.small_fold && c == 0 && threadIdx.x < 64) subplan_image(b, blockIdx.y, int(threadIdx.x));  // (k_index's output only)
    if (c >= im.nchunks) return;
    const uintptr_t file = uintptr_t(im.jpeg);
    const uintptr_t lo = file + im.ecs_off, fend = file + im.len;
    const uintptr_t t0 = (lo & ~uintptr_t(15)) + uintptr_t(c) * kScanChunk + uintptr_t(threadIdx.x) * kScanBytesPerThread;
    uint32_t w[16];
    load64(t0, fend, w);
    const uint32_t prevb = (t0 > lo && t0 - 1 < fend) ? uint32_t(*reinterpret_cast<gu8*>(t0 - 1)) : 0u;
    // interior threads (all 64 bytes in the ECS): stuffed zeros from the SWAR masks of k_scan,
    // their positions kept (the kFastDrops highest); others: a per-byte keep mask
    const bool interior = t0 >= lo && t0 + 64 <= fend;
    uint64_t keep = 0;
    uint32_t nd = 0, pd[kFastDrops] = {};  // stuffed zeros, the positions of the highest kFastDrops (pd[0] highest)
    if (interior) {
        uint32_t ff_prev = (prevb == 0xFFu) ? 0x80000000u : 0u;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            uint32_t ff, nz;
            const uint32_t zero = scan_masks(w[q], ff, nz);
            uint32_t dm = zero & ((ff << 8) | (ff_prev >> 24));
            if (q == 0 && t0 == lo) dm &= ~0x80u;  // the ECS's first byte is never dropped
            ff_prev = ff;
            if (__any(dm != 0u)) {  // (wave-uniform: a word without a stuffed zero in any lane is skipped)
                while (dm) {
#pragma unroll
                    for (int r = kFastDrops - 1; r > 0; r--) pd[r] = pd[r - 1];
                    pd[0] = 4u * q + (uint32_t(__builtin_ctz(dm)) >> 3);
                    nd++;
                    dm &= dm - 1u;
                }
            }
        }
    }
    if (!interior || nd > uint32_t(kFastDrops)) {
#pragma unroll
        for (int i = 0; i < 64; i++) {
            const uint32_t by = byte_of(w, i);
            const uint32_t pb = i ? byte_of(w, i - 1) : prevb;
            const uintptr_t a = t0 + i;
            const bool inr = a >= lo && a < fend;
            const bool drop = a > lo && by == 0x00u && pb == 0xFFu;
            if (inr && !drop) keep |= 1ull << i;
        }
    }
    const bool fast = interior && nd <= uint32_t(kFastDrops);
    const uint32_t nkeep = fast ? 64u - nd : uint32_t(__builtin_popcountll(keep));
    uint32_t total;
    uint32_t off = block_excl_scan(nkeep, s_wsum, &total);
    uint8_t* so = reinterpret_cast<uint8_t*>(s_out);
    if (fast) {
        // common case: at most kFastDrops stuffed zeros (a wave with one used to run a 64-byte
        // loop): remove them, highest first, by shifting the later bytes down one (a funnel shift and a
        // bit-field insert per word), then store the run
        uint32_t cw[16];
#pragma unroll
        for (int q = 0; q < 16; q++) cw[q] = w[q];
#pragma unroll
        for (int r = 0; r < kFastDrops; r++) {
            if (uint32_t(r) < nd) {
                const uint32_t p = pd[r];
                const uint32_t qp = p >> 2, lowm = (1u << (8u * (p & 3u))) - 1u;
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    const uint32_t sh = __builtin_amdgcn_alignbyte(q < 15 ? cw[q < 15 ? q + 1 : q] : 0u, cw[q], 1u);
                    const uint32_t m = uint32_t(q) < qp ? 0xFFFFFFFFu : (uint32_t(q) == qp ? lowm : 0u);
                    cw[q] = (cw[q] & m) | (sh & ~m);
                }
            }
        }
        store_run(s_out, off, cw, 64u - nd);
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
// Stage 3: Huffman decode.  Every restart interval (the whole scan when there is no DRI) is cut
// into pieces of piece_bits un-stuffed bits, one lane each — the reference's self-synchronising
// decode (parallelHuffManDecode, cuda-decoder/src/parser.cu:132-208) re-planned so that pieces
// start on MCU boundaries, every piece is decoded once, and nothing runs serially:
//   k_subplan      per image: pieces of every interval (interval lengths are only known on the
//                  GPU, after k_index) and their output regions
//   k_piece        lane per piece j of n = ceil(bits / piece_bits) equal shares L = ceil(bits / n):
//                  starts piece_overlap bits before j*L with a guessed state (Huffman codes
//                  self-synchronise; so does the MCU phase given a few thousand bits), takes the
//                  first MCU boundary at/after j*L as the piece start, and from there writes its
//                  blocks (a record per block, the AC entries) into its own region up to the first
//                  MCU boundary at/after (j+1)*L.  Piece 0 starts at bit 0 in the true state.
//   k_redo         lane per piece whose start is not its predecessor's end: re-walk from that end
//                  into a spare region until it meets one of the speculative walk's checkpoints
//   k_chain        wave per interval: piece j's end must be piece j+1's start (k_chain_fix walks
//                  the rare interval where it still is not serially, re-walking).  Prefix sums
//                  give each piece its first MCU.
//   k_gather       wave per piece: records -> BlockInfo (entry range, DC difference) in block order
//   k_dc_sum/scan  per tile, the DC predictors at its first block (parser.cpp:106-111); the tile's
//                  own wave in k_idct_color finishes the prediction
//
// A lane's bitstream streams through its own LDS row in windows of WIN bytes: a round issues
// the loads of the NEXT window into registers, decodes every symbol whose refill word lies in the
// current window, then commits the registers.  The only vmcnt wait per round is that commit
// (gfx950 counts stores and loads on one vmcnt, so a wait inside the symbol loop would stall on
// the coefficient stores).  The symbol loop keeps a 64-bit bit buffer in registers, refilled
// from a row word read one symbol ahead, so its only LDS latency is the table lookup.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ u32x4 load16(uintptr_t a, uintptr_t last) {
    // clamped to the image's last mapped 16-byte chunk; bytes past an interval's end are never
    // consumed as data, so what a clamped load returns there is irrelevant
    return *reinterpret_cast<gu32x4*>(a < last ? a : last);
}

// Codes longer than kLutBits: the canonical limits decide the length (kLutBits+1 plus the number
// of left-justified limits <= v16: F.2.2.3 restated, independent LDS reads), then the symbol.
// Returns the entry in the fast-table format.  Codes that match nothing and symbols the format
// cannot represent (corrupt streams/tables) give kEntryBad: 16 bits consumed (decoding always
// advances), the bad bit set.
constexpr uint32_t kEntryBad = 16u | kEntBad;
__device__ __forceinline__ uint32_t huff_slow(const uint32_t* lutw, uint32_t peek) {
    const HuffLut* t = reinterpret_cast<const HuffLut*>(lutw);
    const uint32_t v16 = peek >> 16;
    uint32_t l = kLutBits + 1;
#pragma unroll
    for (int j = kLutBits + 1; j <= 16; j++) l += (v16 >= t->lim[j]) ? 1u : 0u;
    uint32_t e = 0;
    if (l <= 16 && v16 >= t->lim[kLutBits]) {
        const uint32_t sym = t->vals[uint32_t(t->base[l] + int(v16 >> (16 - l))) & 255u];
        e = lut_entry(l, sym, t->lim[19] != 0);
    }
    return e ? e : kEntryBad;
}

// EXTEND (utils/stream.cpp:44-52) of the last sz bits of the L bits at the top of peek.
__device__ __forceinline__ int huff_value(uint32_t peek, uint32_t e) {
    const uint32_t L = e & 31u, sz = __builtin_amdgcn_ubfe(e, 16u, 4u) | ((e & kEntSz16) >> 1);
    const uint32_t mag = __builtin_amdgcn_ubfe(peek, 32u - L, sz);  // width 0 -> 0
    const uint32_t half = (1u << sz) >> 1;
    return int(mag) - (mag < half ? int(2 * half - 1) : 0);
}

// BlockInfo.cnt_dc (jd_internal.hpp): AC-entry slot count (7 bits) | escape flag | 24-bit DC difference.
__device__ __forceinline__ uint32_t pack_cnt_dc(uint32_t cnt, int dc, uint32_t esc) {
    return (min(cnt, 127u) << kCntShift) | (esc ? kCntEsc : 0u) | (uint32_t(dc) & kDcMask);
}
__device__ __forceinline__ int cnt_dc_dc(uint32_t cd) { return int32_t(cd << 8) >> 8; }

struct SegInfo {
    uint64_t blk0;     // first global block of the interval
    uint32_t nblk;     // blocks in the interval
    uint32_t bits;     // un-stuffed data bits of the interval
    uintptr_t data;    // address of the interval's first un-stuffed byte
    uintptr_t last;    // last mapped 16-byte chunk of the image's un-stuffed region
    uint32_t ent0;     // first region word of the interval's pieces (image-relative, k_subplan)
    uint32_t pattern, bpm;
    uint32_t rw_div;   // the image's region divisor and slack (region_words)
    uint32_t rw_slack;
    uint32_t* eimg;    // the image's AC entries (BatchDev::entries + ImgDesc::entry_base)
};

// The image's last interval: it ends at EOI, not at an RSTn.
__device__ __forceinline__ bool seg_is_final(const BatchDev& b, uint32_t s) {
    const ImgDesc& im = b.imgs[b.seg_img[s]];
    return s + 1 == im.seg_base + im.nseg;
}

__device__ __forceinline__ void seg_info(const BatchDev& b, uint32_t s, SegInfo& S) {
    const ImgDesc& im = b.imgs[b.seg_img[s]];
    const uint32_t k_seg = s - im.seg_base;
    const uint32_t nmcu = im.mcux * im.mcuy;
    const uint32_t ri = im.restart_interval;
    const uint32_t mcu0 = ri ? k_seg * ri : 0u;
    const uint32_t mcu1 = ri ? min(mcu0 + ri, nmcu) : nmcu;
    const uint32_t cstart = b.seg_cstart[s];
    const uint32_t cend = max(cstart, b.seg_cend[s]);
    S.blk0 = im.block_base + uint64_t(mcu0) * im.bpm;
    S.nblk = (mcu1 - mcu0) * im.bpm;
    S.bits = (cend - cstart) * 8;
    S.data = uintptr_t(im.comp) + cstart;
    S.last = (uintptr_t(im.comp) + (im.len - im.ecs_off) + 63) & ~uintptr_t(15);
    S.ent0 = b.seg_ent[s];
    S.eimg = b.entries + im.entry_base;
    S.pattern = im.block_pattern;
    S.bpm = im.bpm;
    S.rw_div = im.rw_div;
    S.rw_slack = im.rw_slack;
}

// Nominal piece length of an interval cut into npc pieces: equal shares of its bits (at most
// piece_bits), so the lanes of a wave walk about the same number of bits.
__device__ __forceinline__ uint32_t piece_len(const SegInfo& S, uint32_t npc) { return (S.bits + npc - 1u) / npc; }

__device__ __forceinline__ void seg_invalid(const BatchDev& b, SegInfo& S) {
    S.data = S.last = uintptr_t(b.imgs) & ~uintptr_t(15);
    S.bits = 0;
    S.nblk = 0;
    S.blk0 = 0;
    S.ent0 = 0;
    S.eimg = b.entries;
    S.pattern = 0;
    S.bpm = 1;
    S.rw_div = 2;
    S.rw_slack = kRegionSlack;
}

__device__ __forceinline__ void stage_luts(const BatchDev& b, const TableSet& ts, HuffLut* s_lut, int nthreads) {
    for (int slot = 0; slot < ts.nslots; slot++) {
        const uint4* src = reinterpret_cast<const uint4*>(b.luts + ts.lut[slot]);
        uint4* dst = reinterpret_cast<uint4*>(s_lut + slot);
        for (int i = threadIdx.x; i < int(sizeof(HuffLut) / 16); i += nthreads) dst[i] = src[i];
    }
}

// Piece size of a large batch (one workgroup, after k_index, before k_subplan): every interval of b
// bits is cut into ceil(b / P) pieces, a lane each, and a lane walks about P + overlap bits; k_piece
// keeps piece_plan lanes resident.  The candidates P = plan_cand(piece_bits, c) are scored by
// ceil(pieces / resident) x (P + overlap) -- a partial last round of lanes takes as long as a full
// one -- and the cheapest (the smallest P on ties) is written to counters[3] (pieces << 32 | P).
// The pieces per image and candidate come from k_index (img_cand, exact).  Then each image's first
// piece slot (img_base): its table set's range start plus the pieces of the images before it in
// the host's table-set order (img_order), so the batch's pieces are dense from each range's start
// without an allocation atomic in k_subplan.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x = max(x, y);
    }
    return x;
}
// One workgroup of kPlanThreads (JD_PLAN_THREADS): 1024 by default; 256 fit beside a walk or the
// colour stage (one wave per SIMD), which the 1024-lane form does not.
#ifndef JD_PLAN_THREADS
#define JD_PLAN_THREADS 1024
#endif
constexpr uint32_t kPlanThreads = JD_PLAN_THREADS, kPlanWaves = kPlanThreads / 64;
__global__ __launch_bounds__(kPlanThreads) void k_pieceplan(BatchDev b) {
    JD_PRIO_SHORT();
    __shared__ unsigned long long s_cnt[kPlanCands];
    __shared__ uint32_t s_ws[kPlanWaves], s_wm[kPlanWaves], s_choice;
    const uint32_t t = threadIdx.x;
    const int lane = int(t & 63u), wv = int(t >> 6);
    if (t < kPlanCands) s_cnt[t] = 0;
    __syncthreads();
    uint32_t cnt[kPlanCands] = {};
    for (uint32_t img = t; img < b.nimg; img += kPlanThreads) {
        const u32x4* src = reinterpret_cast<const u32x4*>(b.img_cand + size_t(img) * kPlanCands);
#pragma unroll
        for (int q = 0; q < kPlanCands / 4; q++) {
            const u32x4 v = src[q];
            cnt[4 * q] += v.x;
            cnt[4 * q + 1] += v.y;
            cnt[4 * q + 2] += v.z;
            cnt[4 * q + 3] += v.w;
        }
    }
#pragma unroll
    for (int c = 0; c < kPlanCands; c++) {
        const uint32_t w = wave_sum_u32(cnt[c]);
        if (lane == 0) atomicAdd(&s_cnt[c], (unsigned long long)w);
    }
    __syncthreads();
    if (t == 0) {
        double best = 1e300;
        uint32_t pb = b.piece_bits, bc = 0;
        unsigned long long np = s_cnt[0];
        for (int c = 0; c < kPlanCands; c++) {
            const uint32_t p = plan_cand(b.piece_bits, c);
            const double rounds = double((s_cnt[c] + b.piece_plan - 1) / b.piece_plan);
            const double cost = rounds * double(p + b.piece_overlap);
            if (cost < best) {
                best = cost;
                pb = p;
                bc = uint32_t(c);
                np = s_cnt[c];
            }
        }
        b.counters[3] = (np << 32) | pb;
        s_choice = bc;
    }
    __syncthreads();
    const uint32_t c = s_choice;
    uint32_t run = 0, mrun = 0;
    for (uint32_t i0 = 0; i0 < b.nimg; i0 += kPlanThreads) {
        const uint32_t i = i0 + t;
        const bool v = i < b.nimg;
        uint32_t img = 0, ts = 0, used = 0;
        bool first = false;
        if (v) {
            img = b.img_order[i];
            const ImgDesc& im = b.imgs[img];
            ts = im.tableset;
            used = min(b.img_cand[size_t(img) * kPlanCands + c], im.sub_cap);
            first = i == 0 || b.imgs[b.img_order[i - 1]].tableset != ts;
        }
        // exclusive sum of the pieces over the order
        const uint32_t incl = uint32_t(wave_scan_dpp(int(used)));
        if (lane == 63) s_ws[wv] = incl;
        __syncthreads();
        uint32_t excl = run + incl - used, tot = 0;
#pragma unroll
        for (int j = 0; j < int(kPlanWaves); j++) {
            if (j < wv) excl += s_ws[j];
            tot += s_ws[j];
        }
        // the sum at the first image of this image's table set: an inclusive max over the order of
        // (first ? sum : 0), the sums never decreasing
        const uint32_t mk = wave_incl_max(first ? excl : 0u);
        if (lane == 63) s_wm[wv] = mk;
        __syncthreads();
        uint32_t m = max(mrun, mk), mt = mrun;
#pragma unroll
        for (int j = 0; j < int(kPlanWaves); j++) {
            if (j < wv) m = max(m, s_wm[j]);
            mt = max(mt, s_wm[j]);
        }
        if (v) b.img_base[img] = b.ts_cursor[ts] + (excl - m);
        run += tot;
        mrun = mt;
        __syncthreads();  // (s_ws / s_wm are rewritten by the next round)
    }
}

// Per image (one wave): pieces of every interval, interval -> piece map, and each interval's
// first region word: piece j of an interval of n pieces owns region_words(plen) words from
// seg_ent + j * region_words(plen).  The image's spare words after them (img_pool) are handed
// out to re-walks (k_redo, k_chain_fix).  The image's slots are the next ones of its table set's
// range (every image's share fits: the range holds the sum of their caps), so the batch's pieces
// are dense from the range's start: k_pieceplan's img_base in a large batch, else an atomic on the
// table set's cursor.  One pass over the intervals, 64 at a time; the interval -> piece map of
// each 64 is written from registers (an earlier form re-read every interval's base and count
// after a fence: two dependent loads per interval, ~60 us per C2 batch with the atomic).
// (small batches: run by the first k_compact workgroup of each image, beside its compaction, which
// saves a launch on a small batch's critical path; in a large batch the per-image waves lengthen
// k_compact's tail by more than the launch costs: 0.24 -> 0.48 ms on C2, so k_subplan runs as a
// kernel of its own there)
__device__ void subplan_image(const BatchDev& b, uint32_t img, int lane) {
    const ImgDesc& im = b.imgs[img];
    const uint32_t piece_bits = b.piece_plan ? uint32_t(b.counters[3] & 0xFFFFFFFFull) : b.piece_bits;
    uint32_t base;
    if (b.piece_plan) {
        base = b.img_base[img];
    } else {
        uint32_t n = 0;
        for (uint32_t k = uint32_t(lane); k < im.nseg; k += 64) {
            const uint32_t s = im.seg_base + k;
            const uint32_t cs = b.seg_cstart[s], ce = max(cs, b.seg_cend[s]);
            n += pieces_of((ce - cs) * 8, piece_bits);
        }
        // run <= sub_cap by construction (host bound: ceil(ECS bits / piece_bits) + nseg pieces)
        const uint32_t used = min(wave_sum_u32(n), im.sub_cap);
        uint32_t bs = 0;
        if (lane == 0) bs = atomicAdd(&b.ts_cursor[im.tableset], used);
        base = uint32_t(__shfl(int(bs), 0, 64));
    }
    uint32_t run = 0, wrun = 0;
    for (uint32_t k0 = 0; k0 < im.nseg; k0 += 64) {
        const uint32_t k = k0 + uint32_t(lane);
        uint32_t n = 0, w = 0;
        if (k < im.nseg) {
            const uint32_t s = im.seg_base + k;
            const uint32_t cs = b.seg_cstart[s], ce = max(cs, b.seg_cend[s]);
            const uint32_t bits = (ce - cs) * 8;
            n = pieces_of(bits, piece_bits);
            w = n * region_words((bits + n - 1u) / n, im.rw_div, im.rw_slack);
        }
        const uint32_t incl = wave_incl_scan(n), wincl = wave_incl_scan(w);
        const uint32_t off = run + incl - n;
        if (k < im.nseg) {
            const uint32_t s = im.seg_base + k;
            b.seg_sub_base[s] = base + off;
            b.seg_nsub[s] = n;
            b.seg_ent[s] = wrun + wincl - w;
        }
        // (wrun <= entry_cap by construction: ECS bits / rw_div + rw_slack + 4 words per piece)
        const uint32_t m = min(64u, im.nseg - k0);
        for (uint32_t j = 0; j < m; j++) {
            const uint32_t oj = uint32_t(__builtin_amdgcn_readlane(int(off), int(j)));
            const uint32_t nj = uint32_t(__builtin_amdgcn_readlane(int(n), int(j)));
            const uint32_t sj = im.seg_base + k0 + j;
            const uint32_t lim = oj < im.sub_cap ? min(nj, im.sub_cap - oj) : 0u;  // (slots past the cap: none)
            uint32_t* const dst = b.sub_seg + base + oj;
            if (lim < 256u) {  // wave-uniform: the short intervals of DRI streams
                for (uint32_t u = uint32_t(lane); u < lim; u += 64) dst[u] = sj;
            } else {  // a long interval (an image without DRI): 16-byte stores (one wave wrote 68 K
                      // slots of a 2 000 x 2 000 image in 0.1 ms, 4 bytes a lane at a time)
                const uint32_t h = (4u - ((base + oj) & 3u)) & 3u;  // slots before the first aligned quad
                const uint32_t q4 = (lim - h) >> 2, tail = h + 4u * q4;
                if (uint32_t(lane) < h) dst[lane] = sj;
                u32x4* const dq = reinterpret_cast<u32x4*>(dst + h);
                const u32x4 v = {sj, sj, sj, sj};
#pragma unroll 4
                for (uint32_t q = uint32_t(lane); q < q4; q += 64) dq[q] = v;
                if (uint32_t(lane) < lim - tail) dst[tail + lane] = sj;
            }
        }
        run += uint32_t(__shfl(int(incl), 63, 64));
        wrun += uint32_t(__shfl(int(wincl), 63, 64));
    }
    if (lane == 0) b.img_pool[img] = wrun;  // (64-bit)
}
__global__ __launch_bounds__(64) void k_subplan(BatchDev b) {
    JD_PRIO_SHORT();
    subplan_image(b, blockIdx.x, int(threadIdx.x));
}

// Bytes a window round advances (the piece walks' LDS rows hold one window plus an 8-byte
// overlap per lane; 16-byte windows measured 3 % slower).
constexpr int kWin = 32;
// Bytes of the next window a row also holds: a round decodes the symbols whose refill word index
// is <= kWin / 4, and the last of them reads word kWin / 4 + 1, so 8 bytes suffice.
constexpr int kRowOverlap = 8;
constexpr int win_loads(int win) { return win / 16 + 1; }  // loads per window: win / 16 of 16 bytes + the overlap
constexpr int row_words(int win) { return 1 + (win + kRowOverlap) / 4; }  // odd pitch (last word unused)
static_assert(row_words(kWin) % 2 == 1, "row pitch must be odd");
constexpr uint32_t kNoPiece = 0xFFFFFFFFu;
// Walk iterations between two executions of the rare-entry branch (a power of two; 1: every
// iteration).  A rare entry is 0.45 % of lookups on the bench images, but with 64 lanes a quarter
// of the wave-iterations would take the ~40-instruction branch.
#ifndef JD_RARE_EVERY
#define JD_RARE_EVERY 4
#endif
constexpr uint32_t kRareEvery = JD_RARE_EVERY;
static_assert((kRareEvery & (kRareEvery - 1u)) == 0u, "kRareEvery: a power of two");
// items (entries + block records) one window round can add: every item takes >= 2 bits
constexpr uint32_t kRoundItems = (kWin * 8 + 31) / 2 + 4;
static_assert(kRegionSlack >= 640 + kRoundItems + 2, "region slack: straddling MCU + one round past the data");
static_assert(kRoundItems <= kRoundItemsMax, "opt_region_slack: one round past a region's fill");

constexpr int kRingWords = 8;  // per-lane ring of two entry quads (16-byte aligned)
// Block records staged four at a time in a per-lane LDS ring and stored as one 16-byte quad (a
// record at a time, 4 bytes, each store became its own write-back: 1.1 GB written for 0.2 GB of
// records on C2).  16 bytes per lane is what two 512-lane workgroups per CU leave with 4 tables.
constexpr int kRecRingWords = 4;
// walk_piece counts blocks in steps of 4 (the record ring's slot address rrb | (~blk & 12): one op)
constexpr uint32_t kBlkStep = 4u;
// k_redo: 64-lane workgroups with the tables in global memory, so that they fit beside the other
// batch's k_piece / k_idct_color waves instead of waiting for a whole CU's LDS.
constexpr int kRedoThreads = 64;
static_assert(kPieceThreads % kRedoThreads == 0, "a redo workgroup lies inside one piece workgroup");
constexpr size_t kRedoLds = size_t(kRedoThreads) * (row_words(kWin) + kRingWords + kRecRingWords) * 4;
// Large-batch re-walks (k_redo<false>, k_chain_fix) as direct walks (walk_piece DR: no LDS, <= 64
// VGPRs), for builds whose walk workgroup fills a CU (JD_PIECE_THREADS=1024 with 11-bit tables:
// the LDS rows would keep them from running beside it).  Off with the default 512-lane walk, where
// the LDS form measured 1-4 % faster per step.
#ifndef JD_REWALK_DIRECT
#define JD_REWALK_DIRECT (JD_PIECE_THREADS >= 1024)
#endif
constexpr bool kRewalkDirect = JD_REWALK_DIRECT;
constexpr size_t kRewalkLds = kRewalkDirect ? 0 : kRedoLds;
static_assert((kRedoThreads * row_words(kWin) * 4) % 32 == 0, "redo rings must start 32-byte aligned (ring_put)");
size_t piece_lds_bytes(uint32_t max_slots, int nt) {
    return size_t(max_slots) * sizeof(HuffLut) + size_t(nt) * (row_words(kWin) + kRingWords + kRecRingWords) * 4;
}
static_assert((kPieceThreads * row_words(kWin) * 4) % 32 == 0 && (64 * row_words(kWin) * 4) % 32 == 0 && sizeof(HuffLut) % 32 == 0 && kRingWords == 8,
              "rings must start 32-byte aligned (ring_put)");
static_assert((kPieceThreads * (row_words(kWin) + kRingWords) * 4) % 16 == 0 && (64 * (row_words(kWin) + kRingWords) * 4) % 16 == 0,
              "record rings must start 16-byte aligned");

typedef const __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) { return uint32_t(size_t((lds_u32*)p)); }

// Stream reader over a lane's LDS row of big-endian words.  A and B are the words under the read
// position and s = 32 - (bits of A consumed), 0..31 (s = 0: A is used up, the next symbol starts
// at B), so the next 32 stream bits are alignbit(A, B, s).  nextw is the word after B, read one
// symbol ahead from rp, its LDS byte address; wb places the row in the interval: bit of the next
// symbol = rp * 8 + wb - s.  A symbol advances the reader by at most 31 bits, so by at most one
// word.  skip() takes the word step from the sign of s - L alone: v_bfi selects with it as the
// mask and rp moves by -4 x it (one v_mad_i32_i24), no compare.
__device__ __forceinline__ uint32_t bfi_sel(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b, m = 0 / ~0
    uint32_t r = b;
    asm("v_bfi_b32 %0, %1, %2, %0" : "+v"(r) : "v"(m), "v"(a));
    return r;
}
struct BitRow {
    uint32_t A, B, nextw, rp, lim, wb;
    int s;
    __device__ __forceinline__ void init(const uint32_t* row, uint32_t off, uint32_t start) {
        const uint32_t w0 = off >> 5, o = off & 31u, base = lds_addr(row);
        A = o ? row[w0] : 0u;
        B = row[w0 + (o ? 1u : 0u)];
        const uint32_t r = w0 + (o ? 2u : 1u);
        nextw = row[r];
        rp = base + 4u * r;
        lim = base + uint32_t(kWin);  // the window's last refill word: kWin / 4
        s = int((32u - o) & 31u);
        wb = start - off - 32u - 8u * base;  // modulo 2^32
    }
    __device__ __forceinline__ uint32_t peek() const { return __builtin_amdgcn_alignbit(A, B, uint32_t(s)); }
    __device__ __forceinline__ void skip(uint32_t L) {
        s -= int(L);
        const int m = s >> 31;  // ~0: B becomes A (L <= 31)
        s &= 31;                // s + 32 when negative
        A = bfi_sel(uint32_t(m), B, A);
        B = bfi_sel(uint32_t(m), nextw, B);
        asm("v_mad_i32_i24 %0, %1, -4, %0" : "+v"(rp) : "v"(m));  // rp += 4 when m = ~0
        nextw = *(const __attribute__((address_space(3))) uint32_t*)size_t(rp);
    }
    __device__ __forceinline__ uint32_t bit() const { return rp * 8u + wb - uint32_t(s); }
    __device__ __forceinline__ bool in_window() const { return rp <= lim; }
    template <int WIN>
    __device__ __forceinline__ void next_window() {
        rp -= uint32_t(WIN);
        wb += uint32_t(WIN * 8);
    }
};

// The same reader straight over the un-stuffed stream in global memory, for the re-walks that run
// beside a walk which holds a CU's whole LDS (k_redo<false>, k_chain_fix: DR walks).  rp is a byte
// offset from `base`, the walk's first 16-byte aligned window, so the arithmetic (and the window
// rounds: lim moves instead of rp) is BitRow's; each word is a clamped dword load + byte swap.
struct BitStream {
    uint32_t A, B, nextw, rp, lim, wb;
    int s;
    uintptr_t base, lastw;
    __device__ __forceinline__ uint32_t word(uint32_t off) const {
        const uintptr_t a = base + off;
        return __builtin_bswap32(*reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(a < lastw ? a : lastw));
    }
    __device__ __forceinline__ void init(uintptr_t wa, uintptr_t last, uint32_t off, uint32_t start) {
        base = wa;
        lastw = last + 12u;  // the last mapped dword (last: the image's last mapped 16-byte chunk)
        const uint32_t w0 = off >> 5, o = off & 31u;
        A = o ? word(4u * w0) : 0u;
        B = word(4u * (w0 + (o ? 1u : 0u)));
        const uint32_t r = w0 + (o ? 2u : 1u);
        nextw = word(4u * r);
        rp = 4u * r;
        lim = uint32_t(kWin);
        s = int((32u - o) & 31u);
        wb = start - off - 32u;
    }
    __device__ __forceinline__ uint32_t peek() const { return __builtin_amdgcn_alignbit(A, B, uint32_t(s)); }
    __device__ __forceinline__ void skip(uint32_t L) {
        s -= int(L);
        const int m = s >> 31;
        s &= 31;
        A = bfi_sel(uint32_t(m), B, A);
        B = bfi_sel(uint32_t(m), nextw, B);
        asm("v_mad_i32_i24 %0, %1, -4, %0" : "+v"(rp) : "v"(m));
        nextw = word(rp);
    }
    __device__ __forceinline__ uint32_t bit() const { return rp * 8u + wb - uint32_t(s); }
    __device__ __forceinline__ bool in_window() const { return rp <= lim; }
    template <int WIN>
    __device__ __forceinline__ void next_window() { lim += uint32_t(WIN); }
};

// Load q of a window at a (the last one is the overlap: 8 or 16 bytes), and its row words.
__device__ __forceinline__ u32x4 win_load(uintptr_t a, int q, uintptr_t last) {
    if (q == win_loads(kWin) - 1 && kRowOverlap == 8) {
        const uintptr_t c = a + 16 * q;
        const u32x2 v = *reinterpret_cast<const __attribute__((address_space(1))) u32x2*>(c < last ? c : last);
        return u32x4{v.x, v.y, 0u, 0u};
    }
    return load16(a + 16 * q, last);
}
#define JD_ROW_FILL(row, v, q)                                              \
    do {                                                                    \
        (row)[4 * (q) + 0] = __builtin_bswap32(v.x);                 \
        (row)[4 * (q) + 1] = __builtin_bswap32(v.y);                 \
        if ((q) < win_loads(kWin) - 1 || kRowOverlap == 16) {               \
            (row)[4 * (q) + 2] = __builtin_bswap32(v.z);             \
            (row)[4 * (q) + 3] = __builtin_bswap32(v.w);             \
        }                                                                   \
    } while (0)

// The next G windows of a lane's stream (G * kWin bytes + the row overlap), loaded together once
// every G window rounds and copied into the LDS row one window per round.  A lane's 128-byte line
// is then fetched in one go instead of once per 32-byte round: with ~32 K lanes per XCD streaming
// their own pieces, a line read round by round is often evicted from L2 between two rounds.
constexpr int kWinGroup = 128 / kWin;  // 128 bytes of a lane's stream per group (two windows: 1 % slower)
static_assert(kWin % 16 == 0 && kRowOverlap == 8, "WinGroup: whole 16-byte loads per window, an 8-byte overlap");
template <int G>
struct WinGroup {
    static constexpr int L = kWin / 16;  // 16-byte loads per window
    u32x4 v[L * G + 1];
    __device__ __forceinline__ void load(uintptr_t a, uintptr_t last) {
#pragma unroll
        for (int q = 0; q < L * G; q++) v[q] = load16(a + 16 * q, last);
        const uintptr_t c = a + kWin * G;
        const u32x2 t = *reinterpret_cast<const __attribute__((address_space(1))) u32x2*>(c < last ? c : last);
        v[L * G] = u32x4{t.x, t.y, 0u, 0u};
    }
    // the group's next window into the row, then the rest moves down one window (constant register
    // indices throughout: a window index would put the group in scratch memory)
    __device__ __forceinline__ void fill_next(uint32_t* row) {
#pragma unroll
        for (int q = 0; q <= L; q++) JD_ROW_FILL(row, v[q], q);  // q == L: the overlap (first 8 bytes)
#pragma unroll
        for (int q = 0; q + L < L * G + 1; q++) v[q] = v[q + L];
    }
};

// Decoder state per symbol: z = coefficient index of the last symbol (DC: 0), b3 = 3 x block
// within the MCU, tab = LDS byte offset of the next symbol's table (DC table of the block after a
// block ends, else the block's AC table).
constexpr uint32_t kLutBytes = sizeof(HuffLut);
// tab is an LDS address: lut_fast is one v_lshl_add of the index onto it and the LDS read (the
// empty asm keeps the compiler from re-associating (peek >> 22) << 2 into a shift-and-mask).
__device__ __forceinline__ const uint32_t* lut_at(uint32_t tab) { return (const uint32_t*)(lds_u32*)size_t(tab); }
typedef const __attribute__((address_space(3))) u32x2 lds_u64;
__device__ __forceinline__ u32x2 lut_fast(uint32_t tab, uint32_t peek) {
    uint32_t idx = peek >> (32 - kLutBits);
    asm("" : "+v"(idx));
    return *reinterpret_cast<lds_u64*>(size_t((idx << 3) + tab));
}

// Where a walk's tables live: LDS (k_piece, k_chain_fix: tab is an LDS byte address) or global
// memory (k_redo: tab is the 64-bit address of the table in BatchDev::set_luts, so its workgroups
// need LDS only for the lanes' rows and rings).
template <bool GL>
struct TabSpace {
    typedef uint32_t T;
    static __device__ __forceinline__ T base(const uint32_t* p) { return lds_addr(p); }
    static __device__ __forceinline__ u32x2 fast(T tab, uint32_t peek) { return lut_fast(tab, peek); }
    static __device__ __forceinline__ const uint32_t* at(T tab) { return lut_at(tab); }
};
template <>
struct TabSpace<true> {
    typedef uint64_t T;
    static __device__ __forceinline__ T base(const uint32_t* p) { return uint64_t(reinterpret_cast<uintptr_t>(p)); }
    static __device__ __forceinline__ u32x2 fast(T tab, uint32_t peek) {
        const uint64_t idx = peek >> (32 - kLutBits);
        return *reinterpret_cast<const __attribute__((address_space(1))) u32x2*>((idx << 3) + tab);
    }
    static __device__ __forceinline__ const uint32_t* at(T tab) { return reinterpret_cast<const uint32_t*>(tab); }
};

// Block record in a piece's region: AC-entry slot count (<= 126) << 18 | escape flag << 17 | the
// DC difference, 17-bit two's complement (a DC size is <= 16 bits, jd_internal.hpp lut_entry: the
// difference lies within +-65535).  A block stores at most 63 coefficients (each at a zig-zag index
// < 64, strictly increasing), of at most two slots each, so the count fits its 7 bits.
// cnt2e = 2 x the slot count + the escape flag: the walks keep slot counts doubled (ent2, always
// even) and mark a block with an escaped value by making its start ent_blk2 odd and one lower
// (esc_mark), so that ent2 - ent_blk2 = 2 x count + 1 and its shift puts the flag at bit 17.
constexpr uint32_t kRecEsc = 1u << 17;
__device__ __forceinline__ uint32_t block_rec(uint32_t cnt2e, int dc) {
    // one v_bfi_b32 for the DC field (the compiler's and + or3 cost two; the mask in an SGPR:
    // VOP3 takes no literal on gfx9)
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x1FFFFu), "v"(dc), "v"(cnt2e << 17));
    return r;
}
// (idempotent: an already odd start stays as it is)
__device__ __forceinline__ uint32_t esc_mark(uint32_t ent_blk2) { return (ent_blk2 - 1u) | 1u; }
__device__ __forceinline__ uint32_t record_cnt(uint32_t r) { return r >> 18; }
__device__ __forceinline__ bool record_esc(uint32_t r) { return (r & kRecEsc) != 0; }
__device__ __forceinline__ int record_dc(uint32_t r) { return int32_t(r << 15) >> 15; }
// A 16-bit slot into a lane's ring of 16 (ringb 32-byte aligned, ent2 = 2 x the slot count).
__device__ __forceinline__ void ring_put(uint32_t ringb, uint32_t ent2, uint32_t v) {
    *(__attribute__((address_space(3))) uint16_t*)size_t(ringb | (ent2 & 30u)) = uint16_t(v);
}
// Whether x != 0 in every lane of the wave that is executing this: one v_cmp into an SGPR pair,
// compared with exec (a ballot of a bool re-derives the compare; asm keeps it one instruction).
__device__ __forceinline__ bool all_lanes_nz(uint32_t x) {
    uint64_t m;
    asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(m) : "v"(x));
    return m == __builtin_amdgcn_read_exec();
}
// A 16-bit AC entry: value << 6 | zig-zag index for |value| <= 511; else an escape (0x8000 | zz)
// followed by the value itself (jd_internal.hpp).
__device__ __forceinline__ bool entry_big(int v) { return uint32_t(v + 511) > 1022u; }
__device__ __forceinline__ uint32_t entry16(int v, uint32_t zz, bool big) {
    return big ? (0x8000u | zz) : ((uint32_t(v) << 6) | zz);
}

// One piece walk.
//   kSpec: the writing walk from `start`, an MCU boundary (piece 0: bit 0; piece j > 0: where its
//          warm-up, sync_piece, synchronised), with a checkpoint at the first MCU boundary after
//          every cp_bits bits.
//   kRedo: the writing walk from the true MCU boundary `start`; it stops at the first MCU
//          boundary that is one of the speculative walk's checkpoints (cpb) and joins it.
// The writing walk stores, per block, one record (count, DC difference) and the AC entries, into
// the region reg[0, rw), until the first MCU boundary at/after stop_at or the data end.  It
// counts MCUs and notes the number of MCUs before the first error (bad code, bits past the data).
// The chain decides which MCUs count (the last interval's trailing bytes are ignored, as the
// oracle ignores them).
struct PWalk {
    uint32_t start, stop_at;
    uint32_t* reg;
    uint32_t rw;
    uint32_t m_start, m_end, mcus, ents, emcu, ncp, join, tail;
    uint32_t ovf;               // the region guard stopped the walk (optimistic regions: kStOverflow)
    unsigned long long* stats;  // JD_PSTAT builds
};

__device__ __forceinline__ uint32_t piece_emcu_code(uint32_t emcu, uint32_t tail) {
    return emcu != kNoError ? emcu : kNoError - min(tail, kNoError - kTailErr);
}
constexpr int kSpec = 0, kRedo = 1;

// (non-temporal entry stores measured 3x slower: the lines are written back piecemeal anyway)
__device__ __forceinline__ void st_ent(uint4* p, const uint4& v) { *p = v; }

#ifndef JD_PSTAT
#define JD_PSTAT 0  // diagnostic builds: k_piece walk statistics summed into BatchDev::stamps[0..15]
#endif

// DR (direct): the stream read from global memory (BitStream) and every entry slot and block record
// stored straight into the region, so the walk needs no LDS at all (row, ring and rring unused):
// the re-walks that must fit beside a walk holding a CU's whole LDS (k_redo<false>, k_chain_fix).
template <int KIND, bool GL = false, bool DR = false>
__device__ __forceinline__ void walk_piece(const SegInfo& S, const uint32_t* s_lutw, uint32_t dcp, uint32_t acp,
                                           uint32_t* row, uint32_t* ring, uint32_t* rring, bool active_in, PWalk& W, CpRec* cp,
                                           uint32_t cp_bits, const uint32_t (&cpb)[kCpMax]) {
    const uintptr_t a_start = S.data + (W.start >> 3);
    uintptr_t wa = a_start & ~uintptr_t(15);
    typename std::conditional<DR, BitStream, BitRow>::type R;
    if constexpr (DR) {
        R.init(wa, S.last, uint32_t(a_start & 15) * 8 + (W.start & 7u), W.start);
    } else {
#pragma unroll
        for (int q = 0; q < win_loads(kWin); q++) {
            const u32x4 v = win_load(wa, q, S.last);
            JD_ROW_FILL(row, v, q);
        }
        R.init(row, uint32_t(a_start & 15) * 8 + (W.start & 7u), W.start);
    }
    const uint32_t sbits = S.bits;
    const uint32_t bpm3 = 3u * S.bpm;
    typedef TabSpace<GL> TS;
    typedef typename TS::T TabT;
    const TabT lbase = TS::base(s_lutw);
    const TabT tab_dc0 = lbase + (dcp & 7u) * kLutBytes;
    uint32_t* const reg = W.reg;
    uint32_t* const rec_top = W.reg + (W.rw - 1u);  // block record k at rec_top[-k]
    const uint32_t ringb = DR ? 0u : lds_addr(ring);  // 32-byte aligned: slot address = ringb | (ent2 & 30)
    uint16_t* const reg16 = reinterpret_cast<uint16_t*>(W.reg);  // (DR: slot i straight to reg16[i])
    // a 16-bit slot at 2 x slot index e2: into the lane's ring, or (DR) straight into the region
    auto put_slot = [&](uint32_t e2, uint32_t v) {
        if constexpr (DR) reg16[e2 >> 1] = uint16_t(v);
        else ring_put(ringb, e2, v);
    };
    uint32_t z = 0, b3 = 0;
    TabT tab = tab_dc0;
    bool active = active_in;
    uint32_t m_start = W.start, m_end = W.start;
    if (W.start >= sbits) active = false;  // starts at the data end: empty
    // No MCU begins in the piece's share (an MCU longer than a piece: 4:4:4 q95 MCUs take ~450 bits,
    // 256-bit pieces were tried in round 5): the piece is empty, its end its start, which is then the
    // next piece's start too.  (Walking one MCU regardless made every piece after such a share start
    // one MCU late against its successor, so nearly every start disagreed and the chain could only be
    // repaired piece by piece: the r05ac run that went silent, profiles/r06j_*.)
    if (W.start >= W.stop_at) active = false;
    uint32_t next_cp = W.start + cp_bits, ncp = 0, join = 0;
    // The last byte: an MCU end at/after end_thr leaves fewer than 8 bits, which are padding (1-bits
    // before RSTn / EOI) or, where an MCU can be that short (a grayscale block: DC "00" + EOB
    // "1010"), one more MCU.  From there every MCU end takes the slow branch, and m_end (unused until
    // the walk ends) holds where the current MCU began: m_end >= end_thr marks this tail.  If the MCU
    // fails (a bad code, or bits past the data) it was padding -- padding never completes an MCU, no
    // Huffman code being all 1-bits -- and the piece ends at m_end without an error (the oracle
    // decodes exactly the interval's MCUs and skips the padding).
    const uint32_t end_thr = sbits >= 8u ? sbits - 7u : 0u;
    // the next bit at which an MCU end needs the slow branch: the next of piece end, data end,
    // checkpoint (0 after an error)
    uint32_t nxt0 = next_cp;
    if (KIND == kRedo) {
        nxt0 = 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c < kCpMax; c++) nxt0 = (cpb[c] > W.start) ? min(nxt0, cpb[c]) : nxt0;
    }
    uint32_t thr = min(min(W.stop_at, end_thr), nxt0);
    // errs: bit 0, an error in the current MCU; bits 1..: MCUs completed that began in the last byte
    uint32_t mcus = 0, emcu = kNoError, errs = 0;
    // ent2 / ent_blk2: 2 x the slot counts (the ring's byte offsets; ent_blk2 odd: the block has an
    // escaped value, block_rec); blk: blocks x kBlkStep
    uint32_t ent2 = 0, ent_blk2 = 0, blk = 0;
    int dcd = 0;
    // AC entries are 16-bit slots (an escaped value takes two).  Stores are deferred and issued
    // every other loop iteration, so that one store instruction carries many lanes.  An iteration
    // emits at most two slots (a pair of AC symbols, or one escaped value: pairs never escape), and
    // a block takes at least two iterations (its DC symbol never pairs), so taking one quad (8
    // slots) every two iterations keeps fewer than 16 slots pending: one ring of two quads
    // suffices.  Slots go to the ring at slot ent & 15 (a symbol that emits nothing writes the next
    // free slot without advancing, so it is overwritten).  An even quad is copied from the ring
    // into registers when complete and stored together with the odd quad after it (32 bytes: one
    // HBM write granule); block records go four at a time through their own ring.
    uint32_t fq = 0;  // quads stored so far (regions start on a quad)
    uint32_t ovf = 0;
    uint32_t st_wit = 0, st_lit = 0, st_rare = 0, st_rare_w = 0, st_rounds = 0, st_mend_w = 0, st_sym = 0;
    // block record k goes to ring word 3 - (k & 3), so that the ring reads as the records' memory
    // order (descending from rec_top); group fr (records 4fr .. 4fr + 3) is stored when complete,
    // at most one group pending (a block takes >= 2 iterations, a flush comes every other one)
    const uint32_t rrb = DR ? 0u : lds_addr(rring);  // 16-byte aligned
    uint32_t fr = 0;  // record groups stored
    uint4* rgp = reinterpret_cast<uint4*>(rec_top - 3u);  // where group fr goes (a pointer stepped down)
    // an even quad is held in registers and stored with the odd one after it: 32 contiguous bytes
    uint4 hq = {0u, 0u, 0u, 0u};
#define JD_FLUSH_Q()                                                                                   \
    do {                                                                                               \
        if (fq < (ent2 >> 4)) {                                                                        \
            if (fq & 1u) { /* (each branch reads its ring quad at a fixed address) */                   \
                st_ent(reinterpret_cast<uint4*>(reg + 4u * fq - 4u), hq);                              \
                st_ent(reinterpret_cast<uint4*>(reg + 4u * fq), *reinterpret_cast<const uint4*>(ring + 4u)); \
            } else {                                                                                   \
                hq = *reinterpret_cast<const uint4*>(ring);                                            \
            }                                                                                          \
            fq++;                                                                                      \
        }                                                                                              \
    } while (0)
#define JD_FLUSH_B()                                                                                   \
    do {                                                                                               \
        if (fr < (blk >> 4)) {                                                                         \
            st_ent(rgp, *reinterpret_cast<const uint4*>(rring));                                       \
            rgp--;                                                                                     \
            fr++;                                                                                      \
        }                                                                                              \
    } while (0)
    uint32_t pos = W.start;  // == R.bit(): the stream bit of the next symbol
    // (re-walks are short and run few lanes: one window ahead keeps their registers down)
    constexpr int kGroup = KIND == kSpec ? kWinGroup : 1;
    WinGroup<kGroup> nx;
    uint32_t gi = 0;  // window round within the group, wave-uniform
    while (true) {
        if (!DR && gi == 0) nx.load(wa + kWin, S.last);
        uint32_t it = 0;  // equal in every lane still in the loop (lanes only leave it)
        while (active && R.in_window()) {
            it++;
            const uint32_t peek = R.peek();
            const u32x2 E = TS::fast(tab, peek);
            const uint32_t lo = E.x, hi = E.y;
            if (JD_PSTAT) {
                st_rare += (lo & kLoRare) ? 1u : 0u;
                st_rare_w += __any(lo & kLoRare) ? 1u : 0u;
                st_sym += ((lo & kLoRare) == 0 && (lo & kLoPair)) ? 2u : 1u;
            }
            // The table's entry (jd_internal.hpp HuffLut).  A rare entry (lo = kLoRare: no flags,
            // no pair) passes through this part without effect and is decoded below.
            // EXTEND with the table's constants: v = s - (M1 ^ (s >> 31)) for the magnitude bits s
            // sign-extended (none left to extract when the index resolves the value: v = -M1).
            const int s1 = __builtin_amdgcn_sbfe(int(peek), lo, hi);
            const int v1 = s1 - ((int(lo) >> 16) ^ (s1 >> 31));
            uint32_t zn = z + __builtin_amdgcn_ubfe(hi, 5u, 7u);
            uint32_t L = __builtin_amdgcn_ubfe(lo, kLoL1Shift, 5u);
            // a slot is written for every symbol; a stored coefficient (E1, zn < 64: bit 6 of
            // lo & ~zn) advances ent
            put_slot(ent2, (uint32_t(v1) << 6) | zn);
            uint32_t e1 = __builtin_amdgcn_ubfe(lo & ~zn, 6u, 1u);
            asm("" : "+v"(e1));  // keeps bfe + lshl_add (not lshr + and + add)
            ent2 += e1 << 1;
            {  // dcd = DC ? v1 : dcd as one bit-field select on the sign-extended DC flag (bit 5);
               // asm: the compiler turns it back into and + cmp + cndmask
                const int m = __builtin_amdgcn_sbfe(int(lo), 5u, 1u);
                asm("v_bfi_b32 %0, %1, %2, %0" : "+v"(dcd) : "v"(m), "v"(v1));
            }
            // the second symbol of a pair, when the first left the block open (its slot goes to
            // the next free position either way).  It stores a coefficient iff E2 (bit 7 of lo,
            // pairs only) and zn2 < 64: a first symbol that closed the block (zn >= 63, never EOB:
            // EOB does not pair) leaves zn2 >= 64, so the test needs no `pr`.  hi[19:22] is the
            // pair's total length L1 + L2.
            const bool pr = (lo & kLoPair) && zn < 63u;
            const uint32_t zn2 = zn + __builtin_amdgcn_ubfe(hi, 12u, 7u);
            put_slot(ent2, (uint32_t(int(hi) >> 23) << 6) | zn2);
            // E2 (bit 7 of lo) and zn2 < 64 (zn2 <= 127: bit 6 clear) as bit 7 of lo & ~(zn2 << 1)
            uint32_t zs = zn2 << 1;
            asm("" : "+v"(zs));  // (else not + shift + and instead of shift + one v_bitop3)
            uint32_t e2 = __builtin_amdgcn_ubfe(lo & ~zs, 7u, 1u);
            asm("" : "+v"(e2));  // keeps bfe + lshl_add
            ent2 += e2 << 1;
            L = pr ? __builtin_amdgcn_ubfe(hi, 19u, 4u) : L;
            zn = pr ? zn2 : zn;
            // A rare entry consumes nothing in the common path above (L = 0, no emit, no pair,
            // zn = z): it is resolved in this one-sided branch, taken only every kRareEvery-th
            // iteration, so the wave pays for the branch once for all the lanes that have met a
            // rare entry since (they stall in place meanwhile).
            // (also as soon as every lane still in this window round is stalled: the round would
            // otherwise idle until the period comes round)
            uint32_t rl = lo & kLoRare;
            asm("" : "+v"(rl));  // one v_and for both compares
            const bool rare = rl != 0;
            // (| of ints, not ||: the asm compare stays unconditional, in the loop's block)
            const bool rare_now = (int((it & (kRareEvery - 1u)) == kRareEvery - 1u) | int(all_lanes_nz(rl))) != 0;  // wave-uniform
            if (rare && rare_now) {  // codes longer than the index, escaped magnitudes, corrupt codes
                uint32_t e = hi >> kRareShift;
                if ((e & 31u) == 0) e = huff_slow(TS::at(tab), peek);
                const int val = huff_value(peek, e);
                // EOB / ZRL / run-size (parser.cpp:114-134)
                zn = z + __builtin_amdgcn_ubfe(e, 8u, 7u);
                L = e & 31u;
                const bool emit = (e & ~zn & 64u) != 0;  // kEntEmit is bit 6: zn < 64
                dcd = (e & kEntDc) ? val : dcd;
                // the escaped value goes to the next slot unconditionally (a free slot, overwritten
                // by the next entry unless the value needed it)
                const bool big = entry_big(val);
                put_slot(ent2, entry16(val, zn, big));
                put_slot(ent2 + 2u, uint32_t(val));
                ent_blk2 = (emit && big) ? esc_mark(ent_blk2) : ent_blk2;
                ent2 += emit ? (big ? 4u : 2u) : 0u;
                if (e & kEntBad) {  // the next MCU end takes the branch below
                    errs |= 1u;
                    thr = 0u;
                }
            }
            R.skip(L);
            pos += L;
            const bool fin = zn >= 63u;
            // the block's end: its record to the ring and the per-block counters, in the branch the
            // record store needs anyway (exec-masked increments instead of select + add outside it)
            if (fin) {
                if constexpr (DR) rec_top[-int(blk >> 2)] = block_rec(ent2 - ent_blk2, dcd);
                else *(__attribute__((address_space(3))) uint32_t*)size_t(rrb | (~blk & 12u)) = block_rec(ent2 - ent_blk2, dcd);
                blk += 4u;
                b3 += 3u;
                ent_blk2 = ent2;
            }
            if (!DR && (it & 1u) == 0u) {
                JD_FLUSH_Q();
                JD_FLUSH_B();
            }
            z = fin ? 0u : zn;
            // (a stalled rare lane keeps its table: its symbol, DC or AC, is still ahead)
            tab = (rare && !rare_now) ? tab : lbase + __builtin_amdgcn_ubfe(fin ? dcp : acp, b3, 3u) * kLutBytes;
            // MCU end: the common case only counts; the branch is taken at the next threshold
            // (piece end, data end, checkpoint) or after an error
            const bool mend = b3 == bpm3;
            b3 = mend ? 0u : b3;
            tab = mend ? tab_dc0 : tab;
            mcus += mend ? 1u : 0u;
            if (JD_PSTAT) st_mend_w += __any(mend && pos >= thr) ? 1u : 0u;
            if (mend && pos >= thr) {
                const uint32_t consumed = pos;
                const bool fail = (errs & 1u) || consumed > sbits;
                errs &= ~1u;
                uint32_t nxt = 0xFFFFFFFFu;
                if (fail && m_end >= end_thr) {  // an MCU begun in the last byte: padding, not an MCU
                    mcus--;
                    active = false;
                } else if (fail) {  // an error in this MCU
                    emcu = min(emcu, mcus - 1u);
                } else if (m_end >= end_thr) {  // an MCU begun in the last byte, complete
                    errs += 2u;
                }
                if (!active) {
                    // (rolled back)
                } else if (consumed >= W.stop_at || consumed >= sbits) {  // the piece ends here
                    m_end = consumed;
                    active = false;
                } else if (consumed >= end_thr) {  // the last byte (thr stays <= the next MCU end)
                    m_end = consumed;
                } else if (KIND == kSpec) {
                    if (consumed >= next_cp && ncp < uint32_t(kCpMax)) {
                        cp[ncp] = CpRec{consumed, mcus, ent2 >> 1, emcu};  // the segment before it
                        emcu = kNoError;
                        ncp++;
                        next_cp = (ncp < uint32_t(kCpMax)) ? consumed + cp_bits : 0xFFFFFFFFu;
                    }
                    nxt = next_cp;
                } else {
                    bool hit = false;
#pragma unroll
                    for (int c = 0; c < kCpMax; c++) {
                        hit = hit || cpb[c] == consumed;
                        if (cpb[c] == consumed) join = uint32_t(c + 1);
                        nxt = (cpb[c] > consumed) ? min(nxt, cpb[c]) : nxt;
                    }
                    if (hit) {  // in the speculative walk's state: join it
                        m_end = consumed;
                        active = false;
                    }
                }
                thr = min(min(W.stop_at, end_thr), nxt);
            }
        }
        if (!DR) {
            JD_FLUSH_Q();
            JD_FLUSH_B();
        }
        if (active && R.bit() > sbits) {  // past the data
            if (m_end < end_thr) {  // (else in an MCU begun in the last byte, at m_end: padding)
                m_end = R.bit();
                emcu = min(emcu, mcus);
            }
            active = false;
        }
        if (active && (ent2 + 2u) / 4u + blk / kBlkStep + kRoundItems > W.rw) {  // worst-case regions: never for a
                                                                                    // valid stream (region bound)
            m_end = R.bit();
            emcu = min(emcu, mcus);
            active = false;
            ovf = 1u;
        }
        if (JD_PSTAT) {
            st_wit += wave_max_u32(it);
            st_lit += it;
            st_rounds++;
        }
        if (__ballot(active) == 0) break;  // wave-uniform
        if (!DR) nx.fill_next(row);
        gi = __builtin_amdgcn_readfirstlane(gi + 1u == uint32_t(kGroup) ? 0u : gi + 1u);
        R.template next_window<kWin>();
        wa += kWin;
    }
#undef JD_FLUSH_Q
#undef JD_FLUSH_B
    if constexpr (!DR) {
        if (fq & 1u) st_ent(reinterpret_cast<uint4*>(reg + 4u * fq - 4u), hq);  // a held quad
        if (ent2 & 15u)  // the last, partial quad (every complete one is stored; the region has room for all of it)
            st_ent(reinterpret_cast<uint4*>(reg + 4u * fq), *reinterpret_cast<const uint4*>(ring + 4u * (fq & 1u)));
        // the last, partial record group (every complete one is stored: the window round's flush)
        for (uint32_t r = 0; r < ((blk >> 2) & 3u); r++) rec_top[-int(4u * fr + r)] = rring[3u - r];
    }
    W.m_start = m_start;
    W.m_end = m_end;
    W.mcus = mcus;
    W.ents = ent2 >> 1;
    W.emcu = emcu;
    W.ncp = ncp;
    W.join = join;
    W.tail = errs >> 1;
    W.ovf = ovf;
    if (JD_PSTAT && KIND == kSpec && W.stats) {
        const uint32_t v[10] = {st_wit, 0u, wave_sum_u32(st_lit), 0u, wave_sum_u32(st_rare),
                                wave_max_u32(st_rare_w), st_rounds, 1u, wave_max_u32(st_mend_w), wave_sum_u32(st_sym)};
        if ((threadIdx.x & 63u) == 0)
            for (int k = 0; k < 10; k++) atomicAdd(W.stats + k, (unsigned long long)v[k]);
    }
}

// Warm-up of a speculative piece (k_piece, before its writing walk): from `start` in the guessed
// state (first block of an MCU, its DC symbol next) follow the symbols only -- no entries,
// records, counts or errors -- to the first MCU boundary at/after warm_to, where the piece's
// writing walk (walk_piece) starts.  The loop is the writing walk's decode without its
// bookkeeping (about half its instructions); a lane that synchronises early idles until the
// wave's last one has (the separate loop measured 7 % faster than warming up inside the writing
// walk, a separate kernel for it slower: its boundary costs the two batches' overlap).
// Returns that boundary, or kNoPiece with `end` = the bit at which the walk ran past the data.
__device__ __forceinline__ uint32_t sync_piece(const SegInfo& S, const uint32_t* s_lutw, uint32_t dcp, uint32_t acp,
                                               uint32_t* row, uint32_t start, uint32_t warm_to, bool active,
                                               uint32_t& end) {
    const uintptr_t a_start = S.data + (start >> 3);
    uintptr_t wa = a_start & ~uintptr_t(15);
#pragma unroll
    for (int q = 0; q < win_loads(kWin); q++) {
        const u32x4 v = win_load(wa, q, S.last);
        JD_ROW_FILL(row, v, q);
    }
    BitRow R;
    R.init(row, uint32_t(a_start & 15) * 8 + (start & 7u), start);
    const uint32_t bpm3 = 3u * S.bpm;
    const uint32_t lbase = lds_addr(s_lutw);
    const uint32_t tab_dc0 = lbase + (dcp & 7u) * kLutBytes;
    uint32_t z = 0, b3 = 0, tab = tab_dc0, pos = start, res = kNoPiece;
    end = 0;
    WinGroup<kWinGroup> nx;
    uint32_t gi = 0;  // window round within the group, wave-uniform
    while (true) {
        if (gi == 0) nx.load(wa + kWin, S.last);
        uint32_t it = 0;
        while (active && R.in_window()) {
            it++;
            const uint32_t peek = R.peek();
            const u32x2 E = lut_fast(tab, peek);
            const uint32_t lo = E.x, hi = E.y;
            uint32_t zn = z + __builtin_amdgcn_ubfe(hi, 5u, 7u);
            uint32_t L = __builtin_amdgcn_ubfe(lo, kLoL1Shift, 5u);
            const bool pr = (lo & kLoPair) && zn < 63u;
            L = pr ? __builtin_amdgcn_ubfe(hi, 19u, 4u) : L;  // the pair's L1 + L2
            zn = pr ? zn + __builtin_amdgcn_ubfe(hi, 12u, 7u) : zn;
            // rare entries as in walk_piece: deferred to every kRareEvery-th iteration
            uint32_t rl = lo & kLoRare;
            asm("" : "+v"(rl));
            const bool rare = rl != 0;
            const bool rare_now = (int((it & (kRareEvery - 1u)) == kRareEvery - 1u) | int(all_lanes_nz(rl))) != 0;
            if (rare && rare_now) {
                uint32_t e = hi >> kRareShift;
                if ((e & 31u) == 0) e = huff_slow(lut_at(tab), peek);
                zn = z + __builtin_amdgcn_ubfe(e, 8u, 7u);
                L = e & 31u;
            }
            R.skip(L);
            pos += L;
            const bool fin = zn >= 63u;
            z = fin ? 0u : zn;
            b3 += fin ? 3u : 0u;
            tab = (rare && !rare_now) ? tab : lbase + __builtin_amdgcn_ubfe(fin ? dcp : acp, b3, 3u) * kLutBytes;
            const bool mend = b3 == bpm3;
            b3 = mend ? 0u : b3;
            tab = mend ? tab_dc0 : tab;
            if (mend && pos >= warm_to) {
                res = pos;
                active = false;
            }
        }
        if (active && R.bit() > S.bits) {  // past the data before a boundary
            end = R.bit();
            active = false;
        }
        if (__ballot(active) == 0) break;  // wave-uniform
        nx.fill_next(row);
        gi = __builtin_amdgcn_readfirstlane(gi + 1u == uint32_t(kWinGroup) ? 0u : gi + 1u);
        R.template next_window<kWin>();
        wa += kWin;
    }
    return res;
}

__device__ __forceinline__ void table_slots(const TableSet& ts, const SegInfo& S, uint32_t& dcp, uint32_t& acp) {
    dcp = acp = 0;  // 3-bit table slot per MCU block
    for (uint32_t q = 0; q < S.bpm && q < 10; q++) {
        const uint32_t c = (S.pattern >> (2 * q)) & 3u;
        dcp |= uint32_t(ts.dc_slot[c] & 7u) << (3 * q);
        acp |= uint32_t(ts.ac_slot[c] & 7u) << (3 * q);
    }
}

// Piece geometry of lane/slot u in interval s.
struct PieceGeo {
    uint32_t j, npc, plen, rw, own;  // own: first word of the piece's region (image-relative)
};
__device__ __forceinline__ PieceGeo piece_geo(const BatchDev& b, const SegInfo& S, uint32_t s, uint32_t u) {
    PieceGeo P;
    P.j = u - b.seg_sub_base[s];
    P.npc = b.seg_nsub[s];
    P.plen = piece_len(S, P.npc);
    P.rw = region_words(P.plen, S.rw_div, S.rw_slack);
    P.own = S.ent0 + P.j * P.rw;
    return P;
}
__device__ __forceinline__ uint32_t piece_stop(const PieceGeo& P) {
    return (P.j + 1 == P.npc) ? 0xFFFFFFFFu : uint32_t(min<uint64_t>(uint64_t(P.j + 1) * P.plen, 0xFFFFFFFEu));
}

// A piece's speculative walk (k_piece's lane, and k_redo's re-speculation with a longer warm-up):
// for piece j > 0 first the warm-up (sync_piece, every lane of the wave together) from `overlap`
// bits before its nominal start, then the writing walk into the piece's own region, with
// checkpoints.  Piece 0 of an interval starts at bit 0 in the true state.  luts: the table set in LDS.
__device__ __forceinline__ void spec_piece(const BatchDev& b, const SegInfo& S, const PieceGeo& P, uint32_t u, bool valid,
                                           const uint32_t* luts, uint32_t dcp, uint32_t acp, uint32_t* row, uint32_t* ring,
                                           uint32_t* rring, uint32_t overlap, unsigned long long* stats) {
    PWalk W;
    // piece j > 0 synchronises from piece_overlap bits before its nominal start (from bit 0,
    // exactly, when that is closer) to the first MCU boundary at/after it
    const uint64_t pstart = uint64_t(P.j) * P.plen;
    const uint32_t warm_to = (P.j == 0) ? 0u : uint32_t(min<uint64_t>(pstart, S.bits));
    W.start = (pstart <= overlap) ? 0u : min(uint32_t(pstart - overlap), warm_to);
    bool live = valid;
    uint32_t sync_end = 0;
    const bool spec = valid && P.j != 0;
    const uint32_t m = sync_piece(S, luts, dcp, acp, row, W.start, warm_to, spec, sync_end);
    if (spec) {
        live = m != kNoPiece;
        W.start = live ? m : 0u;
    }
    W.stop_at = piece_stop(P);
    W.reg = S.eimg + P.own;
    W.rw = P.rw;
    W.stats = stats;
    CpRec* const cp = b.piece_cp + size_t(u) * kCpRecords;
    const uint32_t none[kCpMax] = {};
    walk_piece<kSpec>(S, luts, dcp, acp, row, ring, rring, live, W, cp, max(1u, P.plen / kCpMax), none);
    if (!valid) return;
    if (W.ovf) atomicOr(&b.status[b.seg_img[b.sub_seg[u]]], kStOverflow);  // (the host decodes it again)
    if (!live) {  // as a warm-up that runs past the data: no piece, an error at its first MCU
        W.m_start = kNoPiece;
        W.m_end = sync_end;
        W.emcu = 0u;
    }
    b.piece_bit[u] = (P.j == 0) ? 0u : W.m_start;
    b.piece_end[u] = W.m_end;
    b.piece_nmcu[u] = W.mcus;
    b.piece_nent[u] = W.ents;
    // W.emcu: the first error after the last checkpoint; each checkpoint holds its segment's
    uint32_t emcu = W.emcu;
#pragma unroll
    for (int k = 0; k < kCpMax; k++)
        if (uint32_t(k) < W.ncp) emcu = min(emcu, cp[k].flags);
    b.piece_emcu[u] = piece_emcu_code(emcu, W.tail);
    b.piece_abase[u] = P.own;
    b.piece_amcu[u] = W.mcus;
    b.piece_join[u] = (min(W.tail, 255u) << 24) | (W.ncp << 16);
    cp[kCpMax] = CpRec{W.m_end, W.mcus, W.ents, W.emcu};
}

// Lane per piece slot: the speculative walk -- for a piece j > 0 first the warm-up (sync_piece,
// every lane of the wave together), then the writing walk into the piece's own region.  Piece 0 of an interval starts at bit 0 in the true state.
// NT = kPieceThreads, or 64 for batches with few pieces (one small image: a few 512-lane
// workgroups would leave all but a few CUs idle; 64-lane ones spread the same lanes over 8x as
// many CUs, each staging its own table copy).
template <int NT>
__global__ __launch_bounds__(NT) void k_piece(BatchDev b) {
    extern __shared__ __attribute__((aligned(32))) uint8_t s_dyn[];
    HuffLut* s_lut = reinterpret_cast<HuffLut*>(s_dyn);
    uint32_t* s_rows = reinterpret_cast<uint32_t*>(s_dyn + size_t(b.max_slots) * sizeof(HuffLut));
    const TableSet& ts = b.tablesets[b.wg_tableset[(blockIdx.x * NT) / kPieceThreads]];
    stage_luts(b, ts, s_lut, NT);
    __syncthreads();

    const uint32_t u = blockIdx.x * NT + threadIdx.x;
    const uint32_t s = (u < b.nsub) ? b.sub_seg[u] : kInvalidImage;
    const bool valid = s != kInvalidImage;
    SegInfo S;
    PieceGeo P{0u, 1u, 0u, 0u, 0u};
    if (valid) {
        seg_info(b, s, S);
        P = piece_geo(b, S, s, u);
    } else {
        seg_invalid(b, S);
    }
    uint32_t dcp, acp;
    table_slots(ts, S, dcp, acp);
    spec_piece(b, S, P, u, valid, reinterpret_cast<const uint32_t*>(s_lut), dcp, acp, s_rows + threadIdx.x * row_words(kWin),
               s_rows + NT * row_words(kWin) + threadIdx.x * kRingWords,
               s_rows + NT * (row_words(kWin) + kRingWords) + threadIdx.x * kRecRingWords, b.piece_overlap, b.stamps);
}

// Re-walk piece u of interval s from its true start `expect` (its predecessor's end): into a
// spare region of the image when one is left (joining the speculative walk at a checkpoint),
// else over its own region (no join: that overwrites what the checkpoints describe).
// Returns the piece's new end.
template <bool GL, bool DR = false>
__device__ uint32_t redo_piece(const BatchDev& b, const SegInfo& S, const PieceGeo& P, uint32_t s, uint32_t u,
                               uint32_t expect, const uint32_t* s_lutw, uint32_t dcp, uint32_t acp, uint32_t* row,
                               uint32_t* ring, uint32_t* rring, bool need) {
    CpRec* const cp = b.piece_cp + size_t(u) * kCpRecords;
    uint32_t ncp = 0, base = P.own, stail = 0;
    CpRec tot{0u, 0u, 0u, kNoError};
    uint32_t cpb[kCpMax];
    if (need) {
        const uint32_t pj = b.piece_join[u];  // k_piece's: tail << 24 | checkpoints << 16
        ncp = (pj >> 16) & 0xFFu;
        stail = pj >> 24;
        tot = cp[kCpMax];
        const uint32_t img = b.seg_img[s];
        // (a 64-bit cursor: many rounds of re-walks cannot wrap it into the image's own pieces)
        const unsigned long long a = b.no_pool ? 0ull : atomicAdd(&b.img_pool[img], (unsigned long long)P.rw);
        if (!b.no_pool && a + P.rw <= b.imgs[img].entry_cap) base = uint32_t(a);
        else ncp = 0;  // in place
    }
#pragma unroll
    for (int c = 0; c < kCpMax; c++) cpb[c] = (need && uint32_t(c) < ncp) ? cp[c].bit : 0xFFFFFFFFu;
    PWalk W;
    W.stats = nullptr;
    W.start = expect;
    W.stop_at = piece_stop(P);
    W.reg = S.eimg + base;
    W.rw = P.rw;
    walk_piece<kRedo, GL, DR>(S, s_lutw, dcp, acp, row, ring, rring, need, W, cp, 0xFFFFFFFFu, cpb);
    if (!need) return 0;
    if (W.ovf) atomicOr(&b.status[b.seg_img[s]], kStOverflow);
    uint32_t end = W.m_end, mcus = W.mcus, ents = W.ents, emcu = W.emcu, tail = W.tail;
    if (W.join) {  // (checkpoints lie before the last byte: the tail, if any, is the speculative walk's)
        const CpRec c = cp[W.join - 1];
        end = tot.bit;
        mcus += tot.mcus - c.mcus;
        ents += tot.ents - c.ents;
        tail = stail;
        // the speculative walk's first error after the joined checkpoint: in the segments of the
        // checkpoints after it (each holds the one before it), or after the last (the totals')
        uint32_t e = tot.flags;
#pragma unroll
        for (int k = 0; k < kCpMax; k++)
            if (uint32_t(k) >= W.join && uint32_t(k) < ncp) e = min(e, cp[k].flags);
        if (e != kNoError) emcu = min(emcu, W.mcus + (e - c.mcus));
    }
    b.piece_bit[u] = expect;
    b.piece_end[u] = end;
    b.piece_nmcu[u] = mcus;
    b.piece_nent[u] = ents;
    b.piece_emcu[u] = piece_emcu_code(emcu, tail);
    b.piece_abase[u] = base;
    b.piece_amcu[u] = W.mcus;
    b.piece_join[u] = (ncp << 16) | W.join;
    return end;
}

// Lane per piece: re-walk, all at once, every piece whose speculative start disagrees with its
// predecessor's end (about 0.6 % of 8192-bit pieces with a 4096-bit overlap on the bench images).
// Starting from that end is exact when the predecessor is right; a predecessor re-walked in the same
// round mostly joins its speculative walk and keeps its end, and otherwise the piece disagrees again.
// Small batches (LT: short pieces, where runs of failed starts are common) go on for up to
// kRedoRounds rounds, each only while some lane of the workgroup still has work, and from the second
// round re-walk only a piece whose predecessor now agrees with its own (re-walked from an end that
// is likely wrong, it would come out wrong again).  A lane's predecessor may belong to another
// workgroup, whose rounds run at the same time, so what is left, k_chain finds.
// LT: the table set staged in LDS (small batches, BatchDev::big_chain or small_fold: the re-walks'
// lookups are a serial chain, ~1 us each from global memory); else read from global memory, so the
// workgroups need little LDS and fit beside the other batch's big kernels.
constexpr uint32_t kRedoRoundsLT = 16;  // small batches: short pieces, runs of failed starts are common
constexpr uint32_t kRedoRoundsBig = 1;  // large batches: double failures are rare (k_chain finds them)
template <bool LT>
__global__ __launch_bounds__(kRedoThreads, (!LT && kRewalkDirect) ? 8 : 1) void k_redo(BatchDev b) {
    JD_PRIO_CRIT();
    constexpr uint32_t kRedoRounds = LT ? kRedoRoundsLT : kRedoRoundsBig;
    extern __shared__ __attribute__((aligned(32))) uint8_t s_dyn[];  // (LT) the tables, the lanes' rows and rings
    HuffLut* s_lut = reinterpret_cast<HuffLut*>(s_dyn);
    uint32_t* s_rows = reinterpret_cast<uint32_t*>(s_dyn + (LT ? size_t(b.max_slots) * sizeof(HuffLut) : 0));
    const uint32_t lane = threadIdx.x;
    const uint32_t u = blockIdx.x * kRedoThreads + lane;
    const uint32_t s = (u < b.nsub) ? b.sub_seg[u] : kInvalidImage;
    const uint32_t sb = s != kInvalidImage ? b.seg_sub_base[s] : 0u;
    const bool valid = s != kInvalidImage && u != sb;  // (piece 0 of an interval starts at bit 0)
    uint32_t expect = 0;
    bool dis = false;  // this piece's start disagrees with its predecessor's end
    if (valid) {
        expect = b.piece_end[u - 1];
        dis = b.piece_bit[u] != expect;
    }
    // the predecessor's own agreement: lane - 1's, or (lane 0) read from memory
    auto pred_dis = [&](bool agent) {
        const bool up = __shfl_up(int(dis), 1, 64) != 0;
        bool pd = lane > 0 && up;
        if (lane == 0 && valid && u - 1u != sb) {
            const uint32_t pb = agent ? __hip_atomic_load(b.piece_bit + u - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : b.piece_bit[u - 1];
            const uint32_t pe = agent ? __hip_atomic_load(b.piece_end + u - 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : b.piece_end[u - 2];
            pd = pb != pe;
        }
        return pd;
    };
    if (__ballot(dis) == 0) return;  // wave-uniform (one wave per workgroup)
    bool need = dis;  // the first round: every disagreeing start (most predecessors re-walked with it join their speculative walk and keep their end)
    uint64_t needm = __ballot(need);
    // the piece workgroup (kPieceThreads lanes, one table set) this one is part of
    const TableSet& ts = b.tablesets[b.wg_tableset[(blockIdx.x * kRedoThreads) / kPieceThreads]];
    if (LT) {
        stage_luts(b, ts, s_lut, kRedoThreads);
        __syncthreads();
    }
    SegInfo S;
    PieceGeo P{0u, 1u, 0u, 0u, 0u};
    if (kRedoRounds > 1 ? valid : need) {  // (one round: only the lanes with a re-walk)
        seg_info(b, s, S);
        P = piece_geo(b, S, s, u);
    } else {
        seg_invalid(b, S);
    }
    uint32_t dcp, acp;
    table_slots(ts, S, dcp, acp);
    const uint32_t* const luts = LT ? reinterpret_cast<const uint32_t*>(s_lut) : reinterpret_cast<const uint32_t*>(b.set_luts + ts.set_lut0);
    uint32_t rewalks = 0;
    for (uint32_t r = 0; needm != 0; r++) {  // (needm: wave-uniform)
        rewalks += uint32_t(__builtin_popcountll(needm));
        if constexpr (!LT && kRewalkDirect)  // no LDS at all: fits beside a walk that holds a CU's whole LDS
            redo_piece<true, true>(b, S, P, s, u, expect, luts, dcp, acp, nullptr, nullptr, nullptr, need);
        else
            redo_piece<!LT>(b, S, P, s, u, expect, luts, dcp, acp, s_rows + lane * row_words(kWin),
                            s_rows + kRedoThreads * row_words(kWin) + lane * kRingWords,
                            s_rows + kRedoThreads * (row_words(kWin) + kRingWords) + lane * kRecRingWords, need);
        if (r + 1 == kRedoRounds) break;
        // the next round, from the current starts and ends.  This round's stores are waited for
        // (vmcnt(0): they are in the L2), and the arrays are read past the L1; a predecessor in a
        // workgroup on another XCD may be seen late, which only leaves its disagreement to k_chain
        // (an agent-scope release would write the L2 back, ~20 us, as in k_index).
#if !defined(__HIP_DEVICE_COMPILE__) || defined(__GFX9__)
        __builtin_amdgcn_s_waitcnt(0x0F70);
#else
#error "k_redo: the vmcnt(0) wait is written for gfx9 (gfx950)"
#endif
        if (valid) {
            expect = __hip_atomic_load(b.piece_end + u - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            dis = __hip_atomic_load(b.piece_bit + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != expect;
        }
        need = dis && !pred_dis(true);
        needm = __ballot(need);
    }
    if (lane == 0) atomicAdd(&b.counters[kCtrRedo], (unsigned long long)rewalks);
}

// The MCUs piece j contributes, given its first MCU m0 (the interval has nmcu_seg): a piece before
// the last one that matters takes all it walked, error-free; the last takes the rest, which it must
// have walked error-free — exactly, unless the interval is the scan's last, whose trailing bytes
// are ignored (the oracle stops after the frame's MCUs).  The last piece of an interval that ends
// at an RSTn walks to the data end: an error anywhere in it, even after its last counted MCU,
// means bytes were left before the marker (the walk ran into them), which the oracle reports as
// a corrupt restart (br_restart finds no marker at the byte-aligned position).  Except for MCUs
// that began in the data's last byte (em's tail count, piece_emcu_code): where the interval's last
// MCU ends in that byte, its leftover bits -- not padding, in a corrupt stream -- may complete
// another short MCU, which the oracle, having decoded the interval's count, never reads; the count
// is then right if it lies between the MCUs before the tail and all of them.  (Only the interval's
// last piece can hold them, unless a piece boundary falls in that byte: such a piece's tail MCUs
// count in full.)
__device__ __forceinline__ uint32_t piece_take(uint32_t pm, uint32_t em, uint32_t m0, uint32_t nmcu_seg, bool last,
                                               bool final_seg, bool& bad) {
    const bool err = em < kTailErr;
    if (!last) {
        bad |= err;
        return pm;
    }
    const uint32_t take = nmcu_seg >= m0 ? nmcu_seg - m0 : 0u;
    const uint32_t tail = err ? 0u : kNoError - em;
    bad |= m0 > nmcu_seg || (final_seg ? pm < take || em < take : pm < take || pm - tail > take || err);
    return min(take, pm);
}

// One wave per interval, all pieces at once: verify that every piece starts where its predecessor
// ended, and give each piece its first MCU and its MCU count by prefix sums.  An interval where
// some start still disagrees after k_redo (a double failure, rare) is flagged for k_chain_fix,
// which walks it serially with re-walks.
// One wave per interval s of n pieces (k_chain), kPer consecutive pieces per lane: an interval
// without DRI can have a thousand pieces, and each wave-iteration is a round of dependent global
// loads (kPer = 4 there; 1 for the short intervals of DRI streams).
template <uint32_t kPer>
__device__ __forceinline__ void chain_interval(const BatchDev& b, uint32_t s, uint32_t lane, const SegInfo& S,
                                               uint32_t base, uint32_t n, uint32_t nmcu_seg, bool final_seg) {
    // The scan's last interval ends at EOI, and what follows its last MCU is ignored: the piece
    // whose MCUs reach the interval's count is the last one that matters, and the pieces after it
    // (decoding trailing bytes) are dropped.
    constexpr uint32_t kStep = 64 * kPer;
    uint32_t jl = n - 1;
    if (final_seg) {
        uint32_t run = 0;
        for (uint32_t j0 = 0; j0 < n; j0 += kStep) {
            const uint32_t jb = j0 + kPer * lane;
            uint32_t c[kPer];
#pragma unroll
            for (uint32_t t = 0; t < kPer; t++) c[t] = jb + t < n ? b.piece_nmcu[base + jb + t] : 0u;
#pragma unroll
            for (uint32_t t = 1; t < kPer; t++) c[t] += c[t - 1];  // inclusive within the lane
            const uint32_t before = run + uint32_t(wave_scan_dpp(int(c[kPer - 1]))) - c[kPer - 1];
            uint32_t tf = kPer;  // the lane's first piece whose running count reaches the interval's
#pragma unroll
            for (int t = kPer - 1; t >= 0; t--)
                if (jb + t < n && before + c[t] >= nmcu_seg) tf = uint32_t(t);
            const uint64_t hit = __ballot(tf < kPer);
            if (hit) {  // wave-uniform
                const int L = __builtin_ctzll(hit);
                jl = j0 + kPer * uint32_t(L) + uint32_t(__shfl(int(tf), L, 64));
                break;
            }
            run = uint32_t(__shfl(int(before + c[kPer - 1]), 63, 64));
        }
    }
    bool need = false;
    for (uint32_t j0 = 0; j0 <= jl; j0 += kStep) {
#pragma unroll
        for (uint32_t t = 0; t < kPer; t++) {
            const uint32_t j = j0 + kPer * lane + t;
            if (j <= jl) need |= b.piece_bit[base + j] != (j ? b.piece_end[base + j - 1] : 0u);
        }
    }
    if (__any(need)) {  // wave-uniform
        if (lane == 0) b.seg_fix[s] = 1u;
        return;
    }
    if (lane == 0) b.seg_fix[s] = 0u;
    uint32_t mcu_run = 0;
    bool bad = false;
    for (uint32_t j0 = 0; j0 < n; j0 += kStep) {
        const uint32_t jb = j0 + kPer * lane;
        uint32_t pm[kPer], pin[kPer], em[kPer], ex[kPer];
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t t = 0; t < kPer; t++) {
            const uint32_t j = jb + t;
            const bool in = j <= jl;  // pieces past jl: no MCUs
            pm[t] = in ? b.piece_nmcu[base + j] : 0u;
            em[t] = in ? b.piece_emcu[base + j] : kNoError;
            pin[t] = (in && j != jl) ? pm[t] : 0u;
            ex[t] = tot;  // exclusive within the lane
            tot += pin[t];
        }
        const uint32_t before = mcu_run + uint32_t(wave_scan_dpp(int(tot))) - tot;
#pragma unroll
        for (uint32_t t = 0; t < kPer; t++) {
            const uint32_t j = jb + t;
            const uint32_t m0 = before + ex[t];
            uint32_t take = 0;
            if (j <= jl) take = piece_take(pm[t], em[t], m0, nmcu_seg, j == jl, final_seg, bad);
            if (j < n) {
                b.piece_mcu0[base + j] = min(m0, nmcu_seg);
                b.piece_nmcu[base + j] = (m0 <= nmcu_seg) ? min(take, nmcu_seg - m0) : 0u;
            }
        }
        mcu_run = uint32_t(__shfl(int(before + tot), 63, 64));
    }
    if (__any(bad) && lane == 0) atomicOr(&b.status[b.seg_img[s]], kStCorrupt);
}

// Intervals of more than kBigInterval pieces are left to k_chain_big (launched instead of
// k_chain_fix when the host sees that an interval may have that many: BatchDev::big_chain).
__global__ __launch_bounds__(256) void k_chain(BatchDev b) {
    JD_PRIO_CRIT();
    const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (s >= b.nseg) return;  // wave-uniform
    SegInfo S;
    seg_info(b, s, S);
    const uint32_t base = b.seg_sub_base[s], n = b.seg_nsub[s];
    const uint32_t nmcu_seg = S.nblk / S.bpm;
    const bool final_seg = seg_is_final(b, s);
    if (b.big_chain && n > kBigInterval) {  // (one interval without DRI: a big image in short pieces) -> k_chain_big
        if (lane == 0) b.seg_fix[s] = 1u;
        return;
    }
    if (n > 64)
        chain_interval<4>(b, s, lane, S, base, n, nmcu_seg, final_seg);
    else
        chain_interval<1>(b, s, lane, S, base, n, nmcu_seg, final_seg);
}

// The intervals k_chain flagged: a start still disagreeing after k_redo (a double failure, rare),
// or (k_chain_big) an interval of more than kBigInterval pieces.
//  * k_chain_fix: one lane per interval (64-lane workgroups grouped by table set) walks its pieces
//    in order, re-walking every disagreeing one (chain_fix_serial).  64-lane workgroups with the
//    tables in global memory, as k_redo: almost every workgroup exits at once, and with the 73 KB
//    of LDS a piece workgroup takes, each of them had to wait for a CU's LDS under the other
//    batch's k_idct_color (1.1 ms instead of 0.02 in a kernel trace).
//  * k_chain_big: for batches whose intervals may have thousands of pieces (an image without DRI in
//    a small batch, in short pieces: one 2000 x 2000 4:4:4 q95 image has ~68 K pieces of 512 bits,
//    and the serial walk took 0.3 us per piece, 13 ms).  One 8-wave workgroup per entry of the chain
//    list (most exit at once: their interval is not flagged), on its flagged interval:
//      - rounds, each in two phases split by a workgroup barrier: (A) every piece of the chunks to
//        check whose start disagrees with its predecessor's end is flagged (piece_mcu0 = the round's
//        tag: that array is scratch until the counts), then (B) every flagged piece is re-walked
//        from its predecessor's end, and the lane goes on into the pieces after it for as long as
//        the new end still disagrees with the next start and that piece is not flagged itself (no
//        other lane touches it in this round).  The pieces before the first flagged one all agree,
//        so they are right: each round settles at least the first disagreement, and a run of
//        pieces whose speculative walks agree with each other in a wrong MCU phase is re-walked by
//        one lane in one round, not one round per piece;
//      - it stops when a round flags nothing, or when a piece before the first flagged one (so a
//        right one) has an error: the counts are then exact already (the error either lies in
//        the MCUs the interval counts, and the image is corrupt, or after them, in trailing bytes
//        of the final interval, and the pieces that matter all precede it).  No round limit is
//        needed (the first disagreement moves on every round), and no serial fallback;
//      - then the counts by prefix sums over per-wave slices (chain_counts_wg).
constexpr uint32_t kFixPer = 16;
// A piece's start and its predecessor's end, as this round sees them: loads that another lane of
// the wave may have stored in the previous round (a workgroup-scope fence orders the rounds).
__device__ __forceinline__ uint32_t ld_wg(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool GL, bool DR = false>
__device__ void chain_fix_serial(const BatchDev& b, uint32_t s, const SegInfo& S, const uint32_t* luts, uint32_t dcp,
                                 uint32_t acp, uint32_t* row, uint32_t* ring, uint32_t* rring) {
    const uint32_t base = b.seg_sub_base[s], n = b.seg_nsub[s];
    const uint32_t nmcu_seg = S.nblk / S.bpm;
    const bool final_seg = seg_is_final(b, s);  // trailing bytes after its last MCU are ignored
    bool bad = false, done = false;
    uint32_t expect = 0, mcu_run = 0, rewalks = 0;
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t u = base + j;
        if (done) {  // past the piece that completed the final interval: nothing to take
            b.piece_mcu0[u] = nmcu_seg;
            b.piece_nmcu[u] = 0u;
            continue;
        }
        uint32_t pend = ld_wg(b.piece_end + u);
        if (ld_wg(b.piece_bit + u) != expect) {  // the start had not synchronised: re-walk from the truth
            const PieceGeo P = piece_geo(b, S, s, u);
            pend = redo_piece<GL, DR>(b, S, P, s, u, expect, luts, dcp, acp, row, ring, rring, true);
            rewalks++;
        }
        const uint32_t pm = b.piece_nmcu[u], em = b.piece_emcu[u];
        const bool last = j + 1 == n || (final_seg && mcu_run + pm >= nmcu_seg);
        const uint32_t take = piece_take(pm, em, mcu_run, nmcu_seg, last, final_seg, bad);
        b.piece_mcu0[u] = min(mcu_run, nmcu_seg);
        b.piece_nmcu[u] = (mcu_run <= nmcu_seg) ? min(take, nmcu_seg - mcu_run) : 0u;
        mcu_run += take;
        done = last;
        expect = pend;
    }
    if (bad) atomicOr(&b.status[b.seg_img[s]], kStCorrupt);
    b.seg_fix[s] = 0u;
    atomicAdd(&b.counters[kCtrFixIntervals], 1ull);  // jd_stats (one serial pass: one round)
    atomicAdd(&b.counters[kCtrFixRounds], 1ull);
    if (rewalks) atomicAdd(&b.counters[kCtrFixRewalks], (unsigned long long)rewalks);
}

__global__ __launch_bounds__(kRedoThreads, kRewalkDirect ? 8 : 1) void k_chain_fix(BatchDev b) {
    JD_PRIO_CRIT();
    extern __shared__ __attribute__((aligned(32))) uint8_t s_dyn[];  // the lanes' rows and rings (none when direct)
    uint32_t* s_rows = reinterpret_cast<uint32_t*>(s_dyn);
    const uint32_t li = blockIdx.x * kRedoThreads + threadIdx.x;
    uint32_t s = (li < b.nchain) ? b.chain_seg[li] : kInvalidImage;
    if (s != kInvalidImage && !b.seg_fix[s]) s = kInvalidImage;
    const bool need = s != kInvalidImage;
    if (__ballot(need) == 0) return;  // wave-uniform (one wave per workgroup): the common case
    const TableSet& ts = b.tablesets[b.chain_wg_tableset[(blockIdx.x * kRedoThreads) / kPieceThreads]];
    if (!need) return;
    SegInfo S;
    seg_info(b, s, S);
    uint32_t dcp, acp;
    table_slots(ts, S, dcp, acp);
    const uint32_t* luts = reinterpret_cast<const uint32_t*>(b.set_luts + ts.set_lut0);
    if constexpr (kRewalkDirect)
        chain_fix_serial<true, true>(b, s, S, luts, dcp, acp, nullptr, nullptr, nullptr);
    else
        chain_fix_serial<true>(b, s, S, luts, dcp, acp, s_rows + threadIdx.x * row_words(kWin),
                               s_rows + kRedoThreads * row_words(kWin) + threadIdx.x * kRingWords,
                               s_rows + kRedoThreads * (row_words(kWin) + kRingWords) + threadIdx.x * kRecRingWords);
}

// k_chain_big's workgroup: 8 waves on one interval at a time (16 would leave 128 VGPRs a lane and
// spill).  One wave took 0.69 ms for the 68 K pieces of a single 2 000 x 2 000 4:4:4 q95 image:
// every round and the counts pass walked its 67 chunks of 1 024 pieces one after the other.
constexpr uint32_t kBigWaves = 8;
constexpr uint32_t kBigThreads = 64 * kBigWaves;
constexpr size_t kBigLds = size_t(kBigThreads) * (row_words(kWin) + kRingWords + kRecRingWords) * 4;

// chain_interval's counts for an interval whose starts all agree (k_chain_big), its pieces cut into
// one contiguous slice of whole chunks per wave: the slices' MCU sums, their prefix, the piece whose
// MCUs reach the final interval's count (jl, the last that matters: found by the wave whose slice
// holds it), then every wave hands out its slice's first MCUs from its prefix.  Pieces before jl
// take what they walked, jl the rest, the ones after it nothing; if no piece reaches the count, the
// interval is short of MCUs (corrupt), as chain_interval decides with jl = n - 1.  Within a chunk
// piece j0 + 64 t + lane: every load and store of the wave is contiguous, and the prefix runs as 16
// wave scans.  (Sixteen consecutive pieces per lane put 64 cache lines under every load: 0.1 ms
// for the 68 K pieces of a 2 000 x 2 000 image.)
__device__ void chain_counts_wg(const BatchDev& b, uint32_t s, uint32_t base, uint32_t n, uint32_t nmcu_seg,
                                bool final_seg, uint32_t* s_sum, uint32_t* s_jl) {
    constexpr uint32_t kPer = kFixPer, kStep = 64 * kPer;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t sl = (n + kBigWaves * kStep - 1u) / (kBigWaves * kStep) * kStep;  // pieces per slice
    const uint32_t lo = min(n, wv * sl), hi = min(n, lo + sl);
    const uint32_t* const nm = b.piece_nmcu + base;
    const uint32_t* const er = b.piece_emcu + base;
    // the slice's MCUs
    uint32_t sum = 0;
    for (uint32_t j0 = lo; j0 < hi; j0 += kStep) {
#pragma unroll
        for (uint32_t t = 0; t < kPer; t++) {
            const uint32_t j = j0 + 64u * t + lane;
            sum += j < hi ? nm[j] : 0u;
        }
    }
    sum = uint32_t(__builtin_amdgcn_readlane(wave_scan_dpp(int(sum)), 63));
    if (lane == 0) s_sum[wv] = sum;
    __syncthreads();
    uint32_t pre = 0, wj = kBigWaves;  // MCUs before the slice; the slice holding jl
    for (uint32_t v = 0, run = 0; v < kBigWaves; v++) {
        if (v == wv) pre = run;
        if (wj == kBigWaves && final_seg && run + s_sum[v] >= nmcu_seg) wj = v;
        run += s_sum[v];
    }
    if (final_seg && wv == wj) {  // find jl in this slice (it is there: the slice reaches the count)
        uint32_t run = pre;
        bool found = false;
        for (uint32_t j0 = lo; j0 < hi && !found; j0 += kStep) {
            uint32_t x[kPer];
#pragma unroll
            for (uint32_t t = 0; t < kPer; t++) {
                const uint32_t j = j0 + 64u * t + lane;
                x[t] = j < hi ? nm[j] : 0u;
            }
#pragma unroll
            for (uint32_t t = 0; t < kPer; t++) {
                if (found) continue;  // wave-uniform
                const uint32_t incl = run + uint32_t(wave_scan_dpp(int(x[t])));
                const uint64_t hit = __ballot(j0 + 64u * t + lane < hi && incl >= nmcu_seg);
                if (hit) {  // wave-uniform
                    const int L = __builtin_ctzll(hit);
                    const uint32_t run_jl = uint32_t(__builtin_amdgcn_readlane(int(incl - x[t]), L));  // MCUs before jl
                    if (lane == 0) {
                        s_jl[0] = j0 + 64u * t + uint32_t(L);
                        s_jl[1] = run_jl;
                    }
                    found = true;
                }
                run = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
            }
        }
    }
    if (threadIdx.x == 0 && (!final_seg || wj == kBigWaves)) {
        s_jl[0] = final_seg ? 0xFFFFFFFFu : n - 1u;  // (final and never reached: every piece before jl)
        s_jl[1] = 0u;
    }
    __syncthreads();
    const uint32_t jl = s_jl[0];
    // the MCUs before this slice that count: every piece before min(lo, jl)
    uint32_t run = (jl == 0xFFFFFFFFu || lo <= jl) ? pre : s_jl[1];
    bool bad = false;
    for (uint32_t j0 = lo; j0 < hi; j0 += kStep) {
        uint32_t pm[kPer], em[kPer];
#pragma unroll
        for (uint32_t t = 0; t < kPer; t++) {
            const uint32_t j = j0 + 64u * t + lane;
            pm[t] = j < hi ? nm[j] : 0u;
            em[t] = j < hi ? er[j] : kNoError;
        }
#pragma unroll
        for (uint32_t t = 0; t < kPer; t++) {
            const uint32_t j = j0 + 64u * t + lane;
            const uint32_t pin = (j < hi && j < jl) ? pm[t] : 0u;
            const uint32_t incl = run + uint32_t(wave_scan_dpp(int(pin)));
            const uint32_t m0 = incl - pin;
            uint32_t take = 0;
            if (j < hi && j <= jl) take = piece_take(pm[t], em[t], m0, nmcu_seg, j == jl, final_seg, bad);
            if (j < hi) {
                b.piece_mcu0[base + j] = min(m0, nmcu_seg);
                b.piece_nmcu[base + j] = (m0 <= nmcu_seg) ? min(take, nmcu_seg - m0) : 0u;
            }
            run = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
        }
    }
    bad |= jl == 0xFFFFFFFFu && wv == 0;  // no piece reached the final interval's count
    if (__any(bad) && lane == 0) atomicOr(&b.status[b.seg_img[s]], kStCorrupt);
    if (threadIdx.x == 0) b.seg_fix[s] = 0u;
}

__global__ __launch_bounds__(kBigThreads) void k_chain_big(BatchDev b) {
    JD_PRIO_CRIT();
    // (small batches only: the table set is staged in LDS, as in k_piece -- the re-walks of each
    // round are serial chains of lookups, ~1 us each from global memory)
    extern __shared__ __attribute__((aligned(32))) uint8_t s_dyn[];
    __shared__ unsigned long long s_mask[2];  // [0] this round's chunks to check (< 64), [1] the next round's
    __shared__ uint32_t s_state;              // bit 0: chunks >= 64 to check, 1: the next round's
    __shared__ uint32_t s_jmin, s_jerr;       // this round: first flagged piece; first piece seen with an error
    __shared__ uint32_t s_nflag;              // this round: pieces flagged (diagnostics: BatchDev::stamps)
    __shared__ uint32_t s_sum[kBigWaves], s_jl[2];
    HuffLut* s_lut = reinterpret_cast<HuffLut*>(s_dyn);
    uint32_t* s_rows = reinterpret_cast<uint32_t*>(s_dyn + size_t(b.max_slots) * sizeof(HuffLut));
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    // one entry of the chain list per workgroup, so that a small batch's big intervals (a few images
    // without DRI) are fixed side by side (64 entries per workgroup took them one after the other)
    const uint32_t s = (blockIdx.x < b.nchain) ? b.chain_seg[blockIdx.x] : kInvalidImage;
    if (s == kInvalidImage || b.seg_fix[s] == 0u) return;  // workgroup-uniform: the common case
    const TableSet& ts = b.tablesets[b.chain_wg_tableset[blockIdx.x / kPieceThreads]];
    stage_luts(b, ts, s_lut, int(kBigThreads));
    __syncthreads();
    const uint32_t* const luts = reinterpret_cast<const uint32_t*>(s_lut);
    uint32_t* const row = s_rows + tid * row_words(kWin);
    uint32_t* const ring = s_rows + kBigThreads * row_words(kWin) + tid * kRingWords;
    uint32_t* const rring = s_rows + kBigThreads * (row_words(kWin) + kRingWords) + tid * kRecRingWords;
    constexpr uint32_t kStep = 64 * kFixPer;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    SegInfo S;
    seg_info(b, s, S);
    uint32_t dcp, acp;
    table_slots(ts, S, dcp, acp);
    const uint32_t base = b.seg_sub_base[s], n = b.seg_nsub[s];
    uint32_t* const flag = b.piece_mcu0 + base;  // round tags (scratch until chain_counts_wg)
    // chunks of kStep pieces to check: every chunk in the first round, then only those holding a
    // piece the round before re-walked, and the chunk after each (its first piece follows the
    // re-walked chunk's last); chunk ci belongs to wave ci mod kBigWaves
    if (tid == 0) {
        s_mask[0] = ~0ull;
        s_mask[1] = 0ull;
        s_state = 1u;
    }
    uint32_t jerr_all = kNone;  // (tid 0) first piece seen with an error in any round, checked again before use
    uint32_t rewalks = 0, rounds = 0;
    bool early = false;
    for (uint32_t round = 0;; round++) {
        if (tid == 0) {
            s_jmin = kNone;
            s_jerr = kNone;
            s_nflag = 0;
        }
        __syncthreads();
        const uint64_t dirty = s_mask[0];
        const bool dirty_hi = (s_state & 1u) != 0u;
        const uint32_t tag = 0x80000000u | round;  // (an MCU index never has the top bit)
        auto look = [&](uint32_t ci) {
            return ci < 64 ? (((dirty >> ci) & 1u) || (ci > 0 && ((dirty >> (ci - 1)) & 1u)))
                           : (dirty_hi || (ci == 64 && (dirty >> 63)));
        };
        // (A) flag the disagreeing pieces of the chunks to check; piece j0 + 64 t + lane (every load
        // of the wave contiguous)
        uint32_t nfl = 0;
        for (uint32_t ci = wv, j0 = wv * kStep; j0 < n; ci += kBigWaves, j0 += kBigWaves * kStep) {
            if (!look(ci)) continue;  // wave-uniform
            uint32_t jm = kNone, je = kNone;
#pragma unroll 4
            for (uint32_t t = 0; t < kFixPer; t++) {
                const uint32_t j = j0 + 64u * t + lane;
                if (j >= n) continue;
                const uint32_t st = ld_wg(b.piece_bit + base + j);
                const uint32_t pe = j > 0 ? ld_wg(b.piece_end + base + j - 1u) : 0u;  // piece 0 starts at bit 0
                if (st != pe) {
                    flag[j] = tag;
                    jm = min(jm, j);
                    nfl++;
                }
                if (ld_wg(b.piece_emcu + base + j) < kTailErr) je = min(je, j);
            }
            jm = __builtin_amdgcn_readfirstlane(wave_min_u32(jm));
            je = __builtin_amdgcn_readfirstlane(wave_min_u32(je));
            if (lane == 0) {
                if (jm != kNone) atomicMin(&s_jmin, jm);
                if (je != kNone) atomicMin(&s_jerr, je);
            }
        }
        if (b.stamps) {  // diagnostics (JD_STAMPS): per round, the first flagged piece and how many
            const uint32_t w = uint32_t(__builtin_amdgcn_readlane(wave_scan_dpp(int(nfl)), 63));
            if (lane == 0 && w) atomicAdd(&s_nflag, w);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the flags before (B) reads them
        __syncthreads();
        const uint32_t jmin = s_jmin;
        if (b.stamps && tid == 0 && round < 4096u) b.stamps[round] = (uint64_t(jmin) << 32) | s_nflag;
        if (tid == 0) {
            jerr_all = min(jerr_all, s_jerr);
            // a right piece (before the first disagreement) with an error: the counts are exact now
            // (the piece may have been re-walked since its error was seen: checked again)
            if (jmin != kNone && jerr_all < jmin) {
                if (ld_wg(b.piece_emcu + base + jerr_all) < kTailErr) s_state |= 4u;
                else jerr_all = kNone;
            }
        }
        __syncthreads();
        rounds = round + 1u;
        early = (s_state & 4u) != 0u;
        if (jmin == kNone || early || round > n) break;  // workgroup-uniform (round > n: never, see above)
        if (b.fix_round_cap && round + 1u >= b.fix_round_cap) {  // diagnostics (JD_FIX_ROUND_CAP): give up
            rounds = n + 2u;
            break;
        }
        // (B) re-walk every flagged piece whose predecessor is not flagged (from that predecessor's
        // end: a flagged predecessor's end is likely wrong, and a piece re-walked from it would come
        // out wrong and poison the next one, as k_redo's rule); the re-walk of the first flagged
        // piece, whose start is right (the front), goes on into the pieces after it.
        for (uint32_t ci = wv, j0 = wv * kStep; j0 < n; ci += kBigWaves, j0 += kBigWaves * kStep) {
            if (!look(ci)) continue;  // wave-uniform
            for (uint32_t t = 0; t < kFixPer; t++) {
                const uint32_t j = j0 + 64u * t + lane;
                bool act = j < n && j > 0 && ld_wg(flag + j) == tag && (j == jmin || ld_wg(flag + j - 1u) != tag);
                if (!__any(act)) continue;  // wave-uniform
                const bool front = act && j == jmin;
                uint32_t cur = j, from = act ? ld_wg(b.piece_end + base + j - 1u) : 0u;
                while (__any(act)) {
                    PieceGeo P{0u, 1u, 0u, 0u, 0u};
                    if (act) P = piece_geo(b, S, s, base + cur);
                    const uint32_t e = redo_piece<false>(b, S, P, s, base + cur, from, luts, dcp, acp, row, ring, rring, act);
                    if (act) {
                        rewalks++;
                        const uint32_t c = cur / kStep;  // the next round checks this chunk and the one after
                        if (c < 64) atomicOr(&s_mask[1], 1ull << c);
                        else atomicOr(&s_state, 2u);
                        // the front goes on while the next start still disagrees: it stops at an
                        // error (corrupt data, or trailing bytes: the next round decides), where the
                        // next start agrees, and at a piece another lane re-walks (flagged, with an
                        // unflagged predecessor: only the front's own predecessor chain is its own)
                        const uint32_t nx = cur + 1u;
                        act = front && nx < n && ld_wg(b.piece_emcu + base + cur) >= kTailErr && ld_wg(b.piece_bit + base + nx) != e &&
                              !(ld_wg(flag + nx) == tag && ld_wg(flag + cur) != tag);
                        cur = nx;
                        from = e;
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // this round's ends before the next reads them
        __syncthreads();
        if (tid == 0) {
            s_mask[0] = s_mask[1];
            s_mask[1] = 0ull;
            s_state = (s_state >> 1) & 1u;
        }
    }
    {  // jd_stats: intervals fixed, rounds, pieces re-walked, early stops
        const uint32_t rw = uint32_t(__builtin_amdgcn_readlane(wave_scan_dpp(int(rewalks)), 63));
        if (lane == 0 && rw) atomicAdd(&b.counters[kCtrFixRewalks], (unsigned long long)rw);
        if (tid == 0) {
            atomicAdd(&b.counters[kCtrFixIntervals], 1ull);
            atomicAdd(&b.counters[kCtrFixRounds], (unsigned long long)rounds);
            if (early) atomicAdd(&b.counters[kCtrFixEarly], 1ull);
        }
    }
    if (rounds > n + 1u) {  // (unreachable: every round settles the first disagreement) corrupt, nothing counted
        for (uint32_t j = tid; j < n; j += kBigThreads) {
            b.piece_mcu0[base + j] = 0u;
            b.piece_nmcu[base + j] = 0u;
        }
        if (tid == 0) {
            atomicOr(&b.status[b.seg_img[s]], kStCorrupt);
            b.seg_fix[s] = 0u;
        }
        return;
    }
    chain_counts_wg(b, s, base, n, S.nblk / S.bpm, seg_is_final(b, s), s_sum, s_jl);
}

// k_gather: a piece's block records -> BlockInfo at the blocks' global positions, AC-entry offsets
// by a prefix sum of the records' counts.  Segment A (the piece's own region, or a re-walk's spare
// region) comes first, then segment B (the own region from the joined checkpoint on).
// A wave takes 64 consecutive pieces: their descriptors lane-parallel, then four pieces at a time,
// one per row of 16 lanes; lane t of a row handles records t, t + 16, ... of its piece, so every
// load (64 B per row) and store (128 B per row) is contiguous, with eight loads in flight per lane.
__device__ __forceinline__ int row_scan_dpp(int x) {  // inclusive, within each row of 16 lanes
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    return x;
}
constexpr int kGatherLoads = 8;
__device__ __forceinline__ uint32_t gather_rows(BlockInfo* out, const uint32_t* rec_top, uint32_t n, uint32_t ebase,
                                                uint32_t lane) {
    const uint32_t t = lane & 15u, last = lane | 15u;
    uint32_t run = ebase;
    for (uint32_t k0 = 0; __any(k0 < n); k0 += 16 * kGatherLoads) {  // wave-uniform trip count
        uint32_t r[kGatherLoads];
#pragma unroll
        for (int i = 0; i < kGatherLoads; i++) {
            const uint32_t k = k0 + t + 16u * i;
            r[i] = (k < n) ? rec_top[-int(k)] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kGatherLoads; i++) {
            const uint32_t k = k0 + t + 16u * i;
            const uint32_t cnt = record_cnt(r[i]);
            const uint32_t incl = uint32_t(row_scan_dpp(int(cnt)));
            if (k < n)
                out[k] = BlockInfo{run + incl - cnt, pack_cnt_dc(cnt, record_dc(r[i]), record_esc(r[i]))};
            run += uint32_t(__shfl(int(incl), int(last), 64));
        }
    }
    return run - ebase;
}
// Lane per piece (short pieces: a small batch's few-hundred-bit pieces hold a few dozen blocks at
// most): the piece's records in order, kGatherLoads loads in flight.  (Four pieces per step took
// 16 dependent steps per wave, ~22 us of a one-image decode whatever its size.)
__device__ __forceinline__ uint32_t gather_lane(BlockInfo* out, const uint32_t* rec_top, uint32_t n, uint32_t ebase) {
    uint32_t run = ebase;
    for (uint32_t k0 = 0; k0 < n; k0 += kGatherLoads) {
        uint32_t r[kGatherLoads];
#pragma unroll
        for (int i = 0; i < kGatherLoads; i++) r[i] = (k0 + uint32_t(i) < n) ? rec_top[-int(k0 + uint32_t(i))] : 0u;
#pragma unroll
        for (int i = 0; i < kGatherLoads; i++) {
            if (k0 + uint32_t(i) >= n) break;
            const uint32_t cnt = record_cnt(r[i]);
            out[k0 + uint32_t(i)] = BlockInfo{run, pack_cnt_dc(cnt, record_dc(r[i]), record_esc(r[i]))};
            run += cnt;
        }
    }
    return run - ebase;
}
constexpr uint32_t kGatherLanePieceBits = 2048;  // pieces this short: lane per piece

__global__ __launch_bounds__(256) void k_gather(BatchDev b) {
    JD_PRIO_SHORT();
    __shared__ uint32_t s_ents;
    if (threadIdx.x == 0) s_ents = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t u = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + lane;
    // 1. descriptors, lane = piece
    const uint32_t s = (u < b.nsub) ? b.sub_seg[u] : kInvalidImage;
    const uint32_t take = (s != kInvalidImage) ? b.piece_nmcu[u] : 0u;
    uint32_t nA = 0, nB = 0, topA = 0, eA = 0, topB = 0, eB = 0;
    uint64_t outi = 0, eimg = 0;
    if (take) {
        SegInfo S;
        seg_info(b, s, S);
        const PieceGeo P = piece_geo(b, S, s, u);
        const uint32_t m0 = b.piece_mcu0[u];
        if (uint64_t(m0) + take <= S.nblk / S.bpm) {  // else corrupt counts (the chain flagged them)
            outi = S.blk0 + uint64_t(m0) * S.bpm;
            eimg = uint64_t(reinterpret_cast<uintptr_t>(S.eimg));
            const uint32_t abase = b.piece_abase[u], amcu = b.piece_amcu[u], join = b.piece_join[u] & 0xFFFFu;
            const uint32_t na = min(take, amcu);
            nA = na * S.bpm;
            eA = 2u * abase;  // entry indices count 16-bit slots
            topA = abase + P.rw - 1u;
            if (take > na && join) {
                const CpRec c = b.piece_cp[size_t(u) * kCpRecords + join - 1];
                nB = (take - na) * S.bpm;
                eB = 2u * P.own + c.ents;
                topB = P.own + P.rw - 1u - c.mcus * S.bpm;
            }
        }
    }
    uint32_t ents = 0;
    if (b.piece_bits <= kGatherLanePieceBits) {  // 2. short pieces: lane per piece
        if (nA + nB) {
            const uint32_t* eptr = reinterpret_cast<const uint32_t*>(uintptr_t(eimg));
            BlockInfo* out = b.blocks + outi;
            ents = gather_lane(out, eptr + topA, nA, eA);
            if (nB) ents += gather_lane(out + nA, eptr + topB, nB, eB);
        }
    } else {  // 2. four pieces at a time, one per row
    const uint64_t busy = __ballot(nA + nB > 0);
    const uint32_t row = lane >> 4;
    for (uint32_t g = 0; g < 16; g++) {
        if (!((busy >> (4 * g)) & 0xFull)) continue;  // wave-uniform
        const int p = int(4 * g + row);
        const uint32_t pnA = __shfl(nA, p, 64), pnB = __shfl(nB, p, 64);
        const uint32_t ptA = __shfl(topA, p, 64), peA = __shfl(eA, p, 64);
        const uint32_t ptB = __shfl(topB, p, 64), peB = __shfl(eB, p, 64);
        const uint64_t po = (uint64_t(uint32_t(__shfl(uint32_t(outi >> 32), p, 64))) << 32) |
                            uint32_t(__shfl(uint32_t(outi), p, 64));
        const uint64_t pe = (uint64_t(uint32_t(__shfl(uint32_t(eimg >> 32), p, 64))) << 32) |
                            uint32_t(__shfl(uint32_t(eimg), p, 64));
        const uint32_t* eptr = reinterpret_cast<const uint32_t*>(uintptr_t(pe));
        BlockInfo* out = b.blocks + po;
        uint32_t e = gather_rows(out, eptr + ptA, pnA, peA, lane);
        if (__any(pnB > 0)) e += gather_rows(out + pnA, eptr + ptB, pnB, peB, lane);
        ents += (lane & 15u) == 0u ? e : 0u;
    }
    }
    const int tot = wave_scan_dpp(int(ents));
    if (lane == 63u && tot) atomicAdd(&s_ents, uint32_t(tot));
    __syncthreads();
    if (threadIdx.x == 0 && s_ents) atomicAdd(&b.counters[0], (unsigned long long)s_ents);
}

// DC prediction (parser.cpp:106-111: per component, the predictor restarts at 0 at every
// interval) is a segmented prefix sum of the DC differences the write pass stores.  It is folded
// into k_idct_color, whose tile is a run of consecutive MCUs of one MCU row (its lanes scan their
// own blocks); the two kernels below give every tile its predictors at entry.
//
// Lane = block of a tile (TR = 1: tile_mcus consecutive MCUs): DC difference, component, and
// whether the block starts an interval (first block of an MCU whose index is a multiple of DRI).
// floor(x / d) for x < 64 and 1 <= d <= 64 with magic = ceil(2^16 / d): one full-rate 24-bit
// multiply and a shift (the error x (magic - 2^16 / d) / 2^16 < 1/1024 never crosses an integer).
__device__ __forceinline__ uint32_t magic16(uint32_t d) { return (65536u + d - 1u) / d; }
__device__ __forceinline__ uint32_t div_small(uint32_t x, uint32_t magic) { return __umul24(x, magic) >> 16; }

// Tile geometry shared by k_dc_sum and k_idct_color (TR = 1: tile_mcus consecutive MCUs of one
// MCU row).  Interval starts among the tile's MCUs without a per-lane modulo: the first is ms
// MCUs in (g0 % DRI computed once per wave), the others every DRI MCUs after it.
struct TileGeo {
    uint32_t m0, nm, g0;  // first MCU column, MCUs in the tile, raster index of its first MCU
    uint32_t ty;          // MCU row of the tile
    uint32_t ri, ms;      // restart interval (0: none) and the first interval start (>= 64: none)
    uint32_t ri_magic;    // magic16(ri) when 0 < ri < tile_mcus (several starts), else 0
};

// Sampling layouts k_idct_color is specialised for (compile-time block pattern, tile width, plane
// geometry and colour mode); every other layout takes the generic instance, which reads them from
// the ImgDesc.  The host (jd_runtime.cpp image_mode) classifies each image the same way and its
// tile choice (tile_mcus = kTileMaxBlocks / bpm) matches tm below.
constexpr int kModeGen = 0, kMode420 = 1, kMode422 = 2, kMode444 = 3;
template <int M>
struct TMode {  // generic: from the image descriptor
    static constexpr bool kFixed = false;
    __device__ static uint32_t bpm(const ImgDesc& im) { return im.bpm; }
    __device__ static uint32_t tm(const ImgDesc& im) { return im.tile_mcus; }
    __device__ static uint32_t pattern(const ImgDesc& im) { return im.block_pattern; }
    __device__ static uint32_t ncomp(const ImgDesc& im) { return im.ncomp; }
    __device__ static uint32_t h(const ImgDesc& im, uint32_t c) { return im.h[c]; }
    __device__ static uint32_t v(const ImgDesc& im, uint32_t c) { return im.v[c]; }
    __device__ static uint32_t cb0(const ImgDesc& im, uint32_t c) { return im.comp_block0[c]; }
    __device__ static uint32_t shx(const ImgDesc& im, uint32_t c) { return im.shx[c]; }
    __device__ static uint32_t shy(const ImgDesc& im, uint32_t c) { return im.shy[c]; }
    __device__ static uint32_t lg_mw(const ImgDesc& im) { return im.lg_mw; }
    __device__ static uint32_t lg_mh(const ImgDesc& im) { return im.lg_mh; }
};
// H1 x V1 luma blocks, one Cb and one Cr block per MCU
template <uint32_t H1, uint32_t V1>
struct TModeYcc {
    static constexpr bool kFixed = true;
    static constexpr uint32_t kBpm = H1 * V1 + 2;
    __device__ static constexpr uint32_t bpm(const ImgDesc&) { return kBpm; }
    __device__ static constexpr uint32_t tm(const ImgDesc&) { return uint32_t(kTileMaxBlocks) / kBpm; }
    __device__ static constexpr uint32_t pattern(const ImgDesc&) { return (1u << (2 * H1 * V1)) | (2u << (2 * H1 * V1 + 2)); }
    __device__ static constexpr uint32_t ncomp(const ImgDesc&) { return 3; }
    __device__ static constexpr uint32_t h(const ImgDesc&, uint32_t c) { return c == 0 ? H1 : 1u; }
    __device__ static constexpr uint32_t v(const ImgDesc&, uint32_t c) { return c == 0 ? V1 : 1u; }
    __device__ static constexpr uint32_t cb0(const ImgDesc&, uint32_t c) { return c == 0 ? 0u : H1 * V1 + c - 1; }
    __device__ static constexpr uint32_t shx(const ImgDesc&, uint32_t c) { return c == 0 ? 0u : (H1 == 2 ? 1u : 0u); }
    __device__ static constexpr uint32_t shy(const ImgDesc&, uint32_t c) { return c == 0 ? 0u : (V1 == 2 ? 1u : 0u); }
    __device__ static constexpr uint32_t lg_mw(const ImgDesc&) { return H1 == 2 ? 4u : 3u; }
    __device__ static constexpr uint32_t lg_mh(const ImgDesc&) { return V1 == 2 ? 4u : 3u; }
};
template <> struct TMode<kMode420> : TModeYcc<2, 2> {};
template <> struct TMode<kMode422> : TModeYcc<2, 1> {};
template <> struct TMode<kMode444> : TModeYcc<1, 1> {};

template <int M = kModeGen>
__device__ __forceinline__ TileGeo tile_geo(const ImgDesc& im, uint32_t tile) {
    TileGeo G;
    const uint32_t TM = TMode<M>::tm(im);
    const uint32_t ty = tile / im.tiles_x, tx = tile - ty * im.tiles_x;
    G.ty = ty;
    G.m0 = tx * TM;
    G.nm = min(TM, im.mcux - G.m0);
    G.g0 = ty * im.mcux + G.m0;
    G.ri = im.restart_interval;
    if (G.ri) {
        const uint32_t r = G.g0 % G.ri;
        G.ms = r ? G.ri - r : 0u;
    } else {
        G.ms = G.g0 == 0 ? 0u : 64u;
    }
    G.ri_magic = (G.ri && G.ri < TM) ? magic16(G.ri) : 0u;
    return G;
}
// MCU m of the tile (m < 64) starts an interval
__device__ __forceinline__ bool tile_mcu_starts(const TileGeo& G, uint32_t m) {
    if (!G.ri_magic) return m == G.ms;  // wave-uniform: at most one start in the tile
    if (m < G.ms) return false;
    const uint32_t v = m - G.ms;
    return v - div_small(v, G.ri_magic) * G.ri == 0;
}

// Lane = block of a tile: DC difference, component, and whether the block starts an interval
// (first block of an MCU whose raster index is a multiple of DRI).
struct TileLane {
    int d;
    uint32_t comp;
    bool have, start;
};
__device__ __forceinline__ TileLane tile_lane(const BatchDev& b, const ImgDesc& im, const TileGeo& G, uint32_t lane) {
    const uint32_t m = div_small(lane, magic16(im.bpm)), bb = lane - m * im.bpm;
    TileLane t;
    t.have = m < G.nm;
    t.comp = (im.block_pattern >> (2 * bb)) & 3u;
    t.start = t.have && bb == 0 && tile_mcu_starts(G, m);
    t.d = 0;
    if (t.have) t.d = cnt_dc_dc(b.blocks[im.block_base + uint64_t(G.g0 + m) * im.bpm + bb].cnt_dc);
    return t;
}

// Wave per tile: the per-component sums of the differences after the tile's last interval start
// (all of them when it has none) and whether it has one.
constexpr uint32_t kDcTilesPerWave = 4;  // k_dc_sum: the tiles' BlockInfo loads are in flight together
__global__ __launch_bounds__(256) void k_dc_sum(BatchDev b) {
    JD_PRIO_SHORT();
    const ImgDesc& im = b.imgs[blockIdx.y];
    const uint32_t nt = im.tiles_x * im.tiles_y, lane = threadIdx.x & 63u;
    // (readfirstlane: the compiler cannot see that threadIdx.x >> 6 is wave-uniform, and would
    // divide in vector registers, ~30 VALU per division, four tiles x two divisions per wave)
    const uint32_t tile0 = __builtin_amdgcn_readfirstlane((blockIdx.x * 4 + (threadIdx.x >> 6)) * kDcTilesPerWave);
    if (tile0 >= nt) return;  // wave-uniform
    TileLane t[kDcTilesPerWave];
#pragma unroll
    for (uint32_t k = 0; k < kDcTilesPerWave; k++)
        t[k] = tile0 + k < nt ? tile_lane(b, im, tile_geo(im, tile0 + k), lane) : TileLane{0, 0u, false, false};
#pragma unroll
    for (uint32_t k = 0; k < kDcTilesPerWave; k++) {
        if (tile0 + k >= nt) break;  // wave-uniform
        const uint64_t mask = __ballot(t[k].start);
        const uint32_t last = mask ? 63u - uint32_t(__clzll(mask)) : 0u;
        const bool after = lane >= last;
        const int s0 = wave_scan_dpp(after && t[k].comp == 0 ? t[k].d : 0);
        const int s1 = wave_scan_dpp(after && t[k].comp == 1 ? t[k].d : 0);
        const int s2 = wave_scan_dpp(after && t[k].comp == 2 ? t[k].d : 0);
        if (lane == 63) b.tile_dc[im.tile_base + tile0 + k] = DcPred{s0, s1, s2, mask ? 1 : 0};
    }
}

// Wave per image: segmented exclusive scan over its tiles in raster order, in place: tile_dc
// becomes the predictor of each component at the tile's first block.  (f, v) o (g, w) = (f | g,
// g ? w : v + w).  Each lane takes a run of consecutive tiles: its aggregate, a scan of the 64
// aggregates, then the run again with the lane's carry.  (64 tiles per step with a carry from step
// to step took ~40 us for the 3 250 tiles of a 2 000 x 2 000 4:4:4 image: 51 steps of dependent
// loads and shuffles.)
__global__ __launch_bounds__(64) void k_dc_scan(BatchDev b) {
    JD_PRIO_SHORT();
    const ImgDesc& im = b.imgs[blockIdx.x];
    const uint32_t lane = threadIdx.x, nt = im.tiles_x * im.tiles_y;
    const uint32_t per = (nt + 63u) / 64u, t0 = min(nt, lane * per), t1 = min(nt, t0 + per);
    DcPred* const td = b.tile_dc + im.tile_base;
    int f = 0, v0 = 0, v1 = 0, v2 = 0;
#pragma unroll 8
    for (uint32_t t = t0; t < t1; t++) {
        const DcPred a = td[t];
        v0 = a.flag ? a.p0 : v0 + a.p0;
        v1 = a.flag ? a.p1 : v1 + a.p1;
        v2 = a.flag ? a.p2 : v2 + a.p2;
        f |= a.flag;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // inclusive over the lanes' runs
        const int n0 = __shfl_up(v0, d, 64), n1 = __shfl_up(v1, d, 64), n2 = __shfl_up(v2, d, 64);
        const int nf = __shfl_up(f, d, 64);
        if (int(lane) >= d && !f) {
            v0 += n0;
            v1 += n1;
            v2 += n2;
            f = nf;
        }
    }
    int r0 = __shfl_up(v0, 1, 64), r1 = __shfl_up(v1, 1, 64), r2 = __shfl_up(v2, 1, 64);  // exclusive
    if (lane == 0) r0 = r1 = r2 = 0;
#pragma unroll 8
    for (uint32_t t = t0; t < t1; t++) {
        const DcPred a = td[t];
        td[t] = DcPred{r0, r1, r2, 0};
        r0 = a.flag ? a.p0 : r0 + a.p0;
        r1 = a.flag ? a.p1 : r1 + a.p1;
        r2 = a.flag ? a.p2 : r2 + a.p2;
    }
}

// ------------------------------------------------------------------------------------------
// Stage 4: dequantise + IDCT + upsample + colour.
// ------------------------------------------------------------------------------------------
enum { kC1 = 2841, kC2 = 2676, kC3 = 2408, kC5 = 1609, kC6 = 1108, kC7 = 565 };

__device__ __forceinline__ int clip256(int v) { return min(max(v, -256), 255); }
// clip256(v >> 14) before the shift: v clamped to [-256 * 2^14, 255 * 2^14 + 2^14 - 1]
__device__ __forceinline__ int clip256_pre(int v) { return min(max(v, -256 * 16384), 255 * 16384 + 16383); }

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

// The IDCT the decode path runs (idct.cpp:34-122), in two forms:
//
//  * fast: every constant multiply on a single input (C7 (x4 + x5) + (C1 - C7) x4 = C1 x4 + C7 x5
//    and so on: equal in int32 arithmetic, which is arithmetic mod 2^32), each one full-rate
//    v_mul/v_mad_i32_i24 instead of a quarter-rate v_mul_lo_u32 on a sum.  Exact when every
//    multiplied input fits 24 signed bits: with all dequantised coefficients within +-2^16 the
//    row inputs do and the row outputs stay within +-6.7e6 < 2^23 (interval bound of the row
//    pass), so the column inputs do too.  Within that range the reference's DC-only shortcuts
//    (idct.cpp:38-41, 83-86) equal the general formulas (no shift overflows), so the fast form is
//    branch-free.
//  * exact: the general formulas plus the shortcuts, selected per row / column exactly as the
//    reference tests them (including a block[4] << 11 that wraps to 0): any int32 input.
//
// k_idct_color takes the fast form when every lane of the wave is in range (wave-uniform), which
// real images always are; tests/test_gpu.py::test_idct_kat covers both over int32 inputs.
// a * k + c as one v_mad_i32_i24 (k an inline constant or literal-free SGPR operand; |a| < 2^23)
__device__ __forceinline__ int mad24v(int a, int k, int c) {
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return r;
}
// blk[0] and blk[32] hold the column pass's x0 = (b0 << 8) + 8192 and x1 = b4 << 8 already: rows 0
// and 4 leave their outputs unshifted with the low byte cleared (idct_row_dot2<true>), because
// ((v >> 8) << 8) + 8192 = (v + 8192) & ~255 (8192 a multiple of 256; no overflow: |v| < 2^31 - 8192
// in the fast form's range), the 8192 riding in row 0's rounding constant.
__device__ __forceinline__ void idct_col_fast(const int* blk, int (&o)[8]) {
    const int x1 = blk[8 * 4], x0 = blk[0];
    const int b1 = blk[8 * 1], b2 = blk[8 * 2], b3 = blk[8 * 3], b5 = blk[8 * 5], b6 = blk[8 * 6], b7 = blk[8 * 7];
    // (the rounding 4 rides in the inner multiply-add: two v_mad_i32_i24 per term, forced through
    // asm: left to itself the compiler emitted two v_mul_i32_i24 and a v_add3 for a third of them)
    int c4;
    asm("v_mov_b32 %0, 4" : "=v"(c4));
    int x4 = mad24v(b1, kC1, mad24v(b7, kC7, c4)) >> 3;
    int x5 = mad24v(b1, kC7, mad24v(b7, -kC1, c4)) >> 3;
    int x6 = mad24v(b5, kC5, mad24v(b3, kC3, c4)) >> 3;
    int x7 = mad24v(b5, kC3, mad24v(b3, -kC5, c4)) >> 3;
    int x2 = mad24v(b2, kC6, mad24v(b6, -kC2, c4)) >> 3;
    int x3 = mad24v(b2, kC2, mad24v(b6, kC6, c4)) >> 3;
    int x8 = x0 + x1;
    int y0 = x0 - x1;
    const int y1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = y0 + x2;
    y0 -= x2;
    x2 = (181 * (x4 + x5) + 128) >> 8;
    x4 = (181 * (x4 - x5) + 128) >> 8;
    o[0] = clip256_pre(x7 + y1);
    o[1] = clip256_pre(x3 + x2);
    o[2] = clip256_pre(y0 + x4);
    o[3] = clip256_pre(x8 + x6);
    o[4] = clip256_pre(x8 - x6);
    o[5] = clip256_pre(y0 - x4);
    o[6] = clip256_pre(x3 - x2);
    o[7] = clip256_pre(x7 - y1);
}
// The column pass's outputs of columns 2p and 2p + 1 as one int16 pair: clip256(v >> 14) is
// clip256_pre(v) >> 14, and the second shift writes its low 16 bits straight into the pair's high
// half (SDWA destination), so no v_perm packs the pair (32 per block).
__device__ __forceinline__ uint32_t pair14(int lo, int hi) {
    uint32_t r = uint32_t(lo >> 14);
    asm("v_ashrrev_i32_sdwa %0, 14, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(r) : "v"(hi));
    return r;
}


__device__ __forceinline__ void idct_row_exact(int* blk) {
    const bool dc_only = ((blk[4] << 11) | blk[6] | blk[2] | blk[1] | blk[7] | blk[5] | blk[3]) == 0;
    const int s = blk[0] << 3;
    idct_row(blk);
#pragma unroll
    for (int k = 0; k < 8; k++) blk[k] = dc_only ? s : blk[k];
}

__device__ __forceinline__ void idct_col_exact(int* blk) {
    const bool dc_only = ((blk[8 * 4] << 8) | blk[8 * 6] | blk[8 * 2] | blk[8 * 1] | blk[8 * 7] | blk[8 * 5] | blk[8 * 3]) == 0;
    const int s = clip256((blk[0] + 32) >> 6);
    idct_col(blk);
#pragma unroll
    for (int k = 0; k < 8; k++) blk[8 * k] = dc_only ? s : blk[8 * k];
}

// The exact form on a block of dequantised coefficients in natural order (blk[0] = DC).
__device__ __forceinline__ void idct_block_exact(int (&blk)[64]) {
#pragma unroll
    for (int r = 0; r < 8; r++) idct_row_exact(blk + 8 * r);
#pragma unroll
    for (int c = 0; c < 8; c++) idct_col_exact(blk + c);
}

// The fast form when every dequantised coefficient fits int16 (k_idct_color's range test).  The
// row pass multiplies int16 pairs by constant pairs with v_dot2_i32_i16 (one instruction per pair
// of products: C1 b1 + C7 b7 = C7 (b1 + b7) + (C1 - C7) b1 and so on, equal in int32), its x0 +- x1
// terms included ((b0 << 11) + 128 +- (b4 << 11) = 2048 b0 +- 2048 b4 + 128); the inputs stay the
// zig-zag-ordered packed words the dequantisation produced (v_pk_mul_lo_u16), each natural pair
// picked by one v_perm_b32.  The column pass is the 24-bit one (row outputs stay within +-2^23).
struct ZzOfNat {  // zig-zag index of each natural position (inverse of kNatOfZz)
    uint8_t v[64];
    constexpr ZzOfNat() : v() {
        for (int z = 0; z < 64; z++) v[kNatOfZz[z]] = uint8_t(z);
    }
};
constexpr ZzOfNat kZzOfNat{};
constexpr uint32_t pk16(int lo, int hi) { return (uint32_t(lo) & 0xFFFFu) | (uint32_t(hi) << 16); }
// The same as one VOP3P v_dot2_i32_i16 with its own accumulator operand: the builtin compiles to the
// tied-accumulator v_dot2c form, which costs a v_mov per product to seed the accumulator (64 per
// block).  k: the constant pair, in an SGPR (the one scalar operand VOP3P allows); the accumulator
// is the inline constant 0 (dot2_0) or a VGPR (dot2_v).
__device__ __forceinline__ int dot2_0(uint32_t a, uint32_t k) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "s"(k));
    return r;
}
__device__ __forceinline__ int dot2_v(uint32_t a, uint32_t k, int c) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return r;
}
// (natural n_lo, natural n_hi) as one int16 pair from the zig-zag pair words dw
__device__ __forceinline__ uint32_t nat_pair(const uint32_t (&dw)[32], int n_lo, int n_hi) {
    const int zl = kZzOfNat.v[n_lo], zh = kZzOfNat.v[n_hi];
    const uint32_t sel = uint32_t(2 * (zl & 1)) | (uint32_t(2 * (zl & 1) + 1) << 8) | (uint32_t(4 + 2 * (zh & 1)) << 16) |
                         (uint32_t(5 + 2 * (zh & 1)) << 24);
    return __builtin_amdgcn_perm(dw[zh >> 1], dw[zl >> 1], sel);
}
// KEEP: the row feeds the column pass's x0 / x1 (rows 0 and 4): outputs v & ~255 instead of v >> 8
// (one full-rate v_and instead of a shift here and another in the column pass).
template <bool KEEP = false>
__device__ __forceinline__ void idct_row_dot2(const uint32_t (&dw)[32], int r, int* out, int c128) {
    const uint32_t P0 = nat_pair(dw, 8 * r + 0, 8 * r + 4), P1 = nat_pair(dw, 8 * r + 1, 8 * r + 7);
    const uint32_t P2 = nat_pair(dw, 8 * r + 5, 8 * r + 3), P3 = nat_pair(dw, 8 * r + 2, 8 * r + 6);
    int x8 = dot2_v(P0, pk16(2048, 2048), c128);
    int y0 = dot2_v(P0, pk16(2048, -2048), c128);
    int x4 = dot2_0(P1, pk16(kC1, kC7));
    int x5 = dot2_0(P1, pk16(kC7, -kC1));
    int x6 = dot2_0(P2, pk16(kC5, kC3));
    int x7 = dot2_0(P2, pk16(kC3, -kC5));
    int x2 = dot2_0(P3, pk16(kC6, -kC2));
    int x3 = dot2_0(P3, pk16(kC2, kC6));
    const int y1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = y0 + x2;
    y0 -= x2;
    x2 = (181 * (x4 + x5) + 128) >> 8;
    x4 = (181 * (x4 - x5) + 128) >> 8;
    const int v[8] = {x7 + y1, x3 + x2, y0 + x4, x8 + x6, x8 - x6, y0 - x4, x3 - x2, x7 - y1};
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = KEEP ? (v[k] & ~255) : (v[k] >> 8);
}
// NR: rows 0 .. NR - 1 may hold nonzero coefficients, the rest are zero in every lane of the wave
// (their row outputs are 0: (0 + 128) >> 8), so their row passes are skipped and the column pass's
// products with them fold away at compile time.
// skip7 (wave-uniform): row 7 is zero in every lane, its row pass is skipped at run time.
// pk[4 r + p]: row r's samples 2p, 2p + 1 as an int16 pair (the planes' layout).
template <int NR = 8>
__device__ __forceinline__ void idct_block_dot2(const uint32_t (&dw)[32], uint32_t (&pk)[32], bool skip7 = false) {
    int blk[64];  // the row pass's outputs
    int c128, c8320;
    asm("v_mov_b32 %0, 0x80" : "=v"(c128));  // one VGPR holding the row pass's rounding term
    asm("v_mov_b32 %0, 0x2080" : "=v"(c8320));  // row 0: + the column pass's 8192 (idct_col_fast)
#pragma unroll
    for (int r = 0; r < 8; r++) {
        if (r < NR && !(r == 7 && skip7)) {
            if (r == 0) idct_row_dot2<true>(dw, r, blk, c8320);
            else if (r == 4) idct_row_dot2<true>(dw, r, blk + 32, c128);
            else idct_row_dot2(dw, r, blk + 8 * r, c128);
        } else {  // (rows 1..7 only: NR >= 1)
#pragma unroll
            for (int k = 0; k < 8; k++) blk[8 * r + k] = 0;
        }
    }
#pragma unroll
    for (int c = 0; c < 8; c += 2) {
        int lo[8], hi[8];
        idct_col_fast(blk + c, lo);
        idct_col_fast(blk + c + 1, hi);
#pragma unroll
        for (int r = 0; r < 8; r++) pk[4 * r + (c >> 1)] = pair14(lo[r], hi[r]);
    }
}
// OR of the natural row r's eight zig-zag-ordered int16 coefficients held in the pair words dw.
template <int R>
__device__ __forceinline__ uint32_t row_bits(const uint32_t (&dw)[32]) {
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const int z = kZzOfNat.v[8 * R + c];
        acc |= dw[z >> 1] & ((z & 1) ? 0xFFFF0000u : 0x0000FFFFu);
    }
    return acc;
}

__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }

// utils/color.cpp:11-17 verbatim in double/float; taken only for the rare G inputs below.
__device__ __attribute__((noinline)) int color_g_exact(int y, int cb, int cr) {
    const float r = float(double(cr) * (2 - 2 * 0.299) + double(y));
    const float b = float(double(cb) * (2 - 2 * 0.114) + double(y));
    const float g = float((double(y) - 0.114 * double(b) - 0.299 * double(r)) / 0.587);
    return clamp255(int(g + 128.0f));
}

// Exact integer restatement of utils/color.cpp:8-19, split into per-chroma-sample terms and a
// per-pixel add + clamp (verified over all of [-256,255]^3: tests/test_oracle.py):
//   R = clamp(y + 128 + floor(1402 cr / 1000))       (1.402 cr is >= 0.002 from any integer
//   B = clamp(y + 128 + floor(1772 cb / 1000))        unless it is one: float rounding is harmless)
//   G = clamp(y + 127 - floor(N / 587000)), N = 202008 cb + 419198 cr; y + 128 when N == 0; the
//       reference's double/float path when N / 587000 is within 64/587000 of an integer (2e-4)
struct ChromaTerms {
    int r, b, g;
    bool exact;
};
// R and B as one 24-bit multiply-add and a shift each: floor(1402 cr / 1000) + 128 =
// (91881 cr + 128 * 2^16) >> 16 and floor(1772 cb / 1000) + 128 = (58065 cb + 128 * 2^15 + 32) >> 15
// for every cr, cb in [-256, 255] (magic constants found by exhaustive search; the products stay
// below 2^31).  G's quotient by a multiply-high on n offset to [0, 2^29) (below), its remainder
// exact in integers.  Equal to the integer definitions above for every (cb, cr) in [-256, 255]^2
// (tests/test_oracle.py::test_chroma_terms_exhaustive, and the GPU's all-2^27 test_color_exhaustive).
// a * k + c as one v_mad_i32_i24 whatever the compiler knows of a's range (k in an SGPR: the
// compiler otherwise falls back to v_mul_lo_u32 / v_mad_u64_u32 for values whose 24-bit range it
// lost across basic blocks, e.g. the filtered chroma of k_colour_fancy).  |a| < 2^23.
__device__ __forceinline__ int mad24(int a, int k, int c) {
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return r;
}
__device__ __forceinline__ ChromaTerms chroma_terms(int cb, int cr) {
    ChromaTerms t;
    t.r = mad24(cr, 91881, 128 << 16) >> 16;
    t.b = mad24(cb, 58065, (128 << 15) + 32) >> 15;
    // G = clamp(y + 128 - ceil(n / 587000)) (the N == 0 case of the definition above included):
    // m = 272 * 587000 - n is in [0, 2^29), and floor(m / 587000) = 272 - ceil(n / 587000) =
    // mulhi(m, M) >> 19 with M = ceil(2^51 / 587000) for every m of the domain (checked
    // exhaustively): the term is that quotient - 144, with no select for n == 0.  The remainder
    // of m is within 64 of 0 or 587000 exactly when n's is (n != 0: m != 272 * 587000).
    constexpr int kOff = 272 * 587000;
    const uint32_t m = uint32_t(mad24(cb, -202008, mad24(cr, -419198, kOff)));
    const uint32_t qm = __umulhi(m, 3836115526u) >> 19;
    const int rem = mad24(int(qm), -587000, int(m));
    t.exact = m != uint32_t(kOff) && (rem < 64 || rem > 587000 - 64);
    t.g = int(qm) - 144;
    return t;
}
__device__ __forceinline__ uint32_t clamp_u8(int v) { return uint32_t(min(max(v, 0), 255)); }  // v_med3_i32

__device__ __forceinline__ void colour_px(int y, int cb, int cr, const ChromaTerms& t, uint32_t& R, uint32_t& G,
                                          uint32_t& B) {
    R = clamp_u8(y + t.r);
    B = clamp_u8(y + t.b);
    G = t.exact ? uint32_t(color_g_exact(y, cb, cr)) : clamp_u8(y + t.g);
}

// The production per-pixel path in one call (known-answer hook, tests/test_gpu.py).
__device__ __forceinline__ void color_px(int y, int cb, int cr, uint32_t& R, uint32_t& G, uint32_t& B) {
    colour_px(y, cb, cr, chroma_terms(cb, cr), R, G, B);
}

// n = 8 >> SH consecutive int16 samples of a plane row (SH = log2 of the horizontal replication)
template <int SH>
__device__ __forceinline__ void load_plane(const int16_t* pl, uint32_t off, int (&v)[8]) {
    if (SH == 0) {
        const uint4 q = *reinterpret_cast<const uint4*>(pl + off);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            v[2 * i] = int(int16_t(w[i] & 0xFFFFu));
            v[2 * i + 1] = int32_t(w[i]) >> 16;
        }
    } else if (SH == 1) {
        const uint2 q = *reinterpret_cast<const uint2*>(pl + off);
        v[0] = int(int16_t(q.x & 0xFFFFu));
        v[1] = int32_t(q.x) >> 16;
        v[2] = int(int16_t(q.y & 0xFFFFu));
        v[3] = int32_t(q.y) >> 16;
    } else {
        const uint32_t q = *reinterpret_cast<const uint32_t*>(pl + off);
        v[0] = int(int16_t(q & 0xFFFFu));
        v[1] = int32_t(q) >> 16;
    }
}

// Colour of 8 pixels whose chroma samples repeat 2^SH times horizontally (both chroma planes);
// SH == 3: grayscale (cb = cr = 0).
template <int SH>
__device__ __forceinline__ void colour8(const int (&Yv)[8], const int16_t* s_pl, uint32_t cboff, uint32_t croff,
                                        uint32_t (&rgb)[8][3]) {
    if (SH == 3) {
#pragma unroll
        for (int j = 0; j < 8; j++) rgb[j][0] = rgb[j][1] = rgb[j][2] = clamp_u8(Yv[j] + 128);
        return;
    }
    constexpr int NU = 8 >> SH;
    int cb[8], cr[8];
    load_plane<SH>(s_pl, cboff, cb);
    load_plane<SH>(s_pl, croff, cr);
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const ChromaTerms t = chroma_terms(cb[u], cr[u]);
#pragma unroll
        for (int r = 0; r < (1 << SH); r++) {
            const int j = (u << SH) + r;
            colour_px(Yv[j], cb[u], cr[u], t, rgb[j][0], rgb[j][1], rgb[j][2]);
        }
    }
}

// 8 RGB pixels -> 24 bytes in 6 words (byte k of the group = word k / 4, bits 8 (k % 4)).
__device__ __forceinline__ void pack24(const uint32_t (&rgb)[8][3], uint32_t (&w)[6]) {
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const int k = 4 * q;
        w[q] = rgb[k / 3][k % 3] | (rgb[(k + 1) / 3][(k + 1) % 3] << 8) | (rgb[(k + 2) / 3][(k + 2) % 3] << 16) |
               (rgb[(k + 3) / 3][(k + 3) % 3] << 24);
    }
}

// Pixel (x, y) of an RGB image of row pitch W3 = 3 W bytes: one 32 x 32 -> 64-bit multiply-add for
// the row (the form (size_t(y) * W + x) * 3 costs three of them), x * 3 as a 24-bit multiply.
__device__ __forceinline__ uint8_t* rgb_at(uint8_t* out, uint32_t y, uint32_t W3, uint32_t x) {
    return out + size_t(y) * W3 + __umul24(x, 3u);
}
// n <= 8 pixels (24 bytes when n == 8) of a row: 8-byte stores when aligned, else words/bytes
__device__ __forceinline__ void store24(uint8_t* dst, const uint32_t (&w)[6], uint32_t n) {
    const uintptr_t ad = reinterpret_cast<uintptr_t>(dst);
    if (n == 8 && (ad & 3) == 0) {
        if ((ad & 7) == 0) {
            auto d2 = gptr(reinterpret_cast<u32x2*>(dst));
            d2[0] = u32x2{w[0], w[1]};
            d2[1] = u32x2{w[2], w[3]};
            d2[2] = u32x2{w[4], w[5]};
        } else {
            auto d1 = gptr(reinterpret_cast<uint32_t*>(dst));
#pragma unroll
            for (int q = 0; q < 6; q++) d1[q] = w[q];
        }
    } else {
        auto d = gptr(dst);
#pragma unroll
        for (int k = 0; k < 24; k++)
            if (uint32_t(k) < 3 * n) d[k] = uint8_t(w[k / 4] >> (8 * (k % 4)));
    }
}

// Two rows of 8 pixels sharing their chroma samples (vertically subsampled chroma): the chroma
// terms are computed once for both rows.
template <int SH>
__device__ __forceinline__ void colour16(const int (&Y0)[8], const int (&Y1)[8], const int16_t* s_pl, uint32_t cboff,
                                         uint32_t croff, uint32_t (&w0)[6], uint32_t (&w1)[6]) {
    constexpr int NU = 8 >> SH;
    int cb[8], cr[8];
    load_plane<SH>(s_pl, cboff, cb);
    load_plane<SH>(s_pl, croff, cr);
    uint32_t a[8][3], c[8][3];
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const ChromaTerms t = chroma_terms(cb[u], cr[u]);
#pragma unroll
        for (int r = 0; r < (1 << SH); r++) {
            const int j = (u << SH) + r;
            colour_px(Y0[j], cb[u], cr[u], t, a[j][0], a[j][1], a[j][2]);
            colour_px(Y1[j], cb[u], cr[u], t, c[j][0], c[j][1], c[j][2]);
        }
    }
    pack24(a, w0);
    pack24(c, w1);
}

// Packed colour (the common case): two pixels per 32-bit word as int16 halves, exactly the
// integer terms above: R = clamp(y + t.r), B = clamp(y + t.b), G = clamp(y + t.g) with
// v_pk_add_u16 + v_sat_pk_u8_i16 (2 VALU per two pixels and channel), then v_perm byte shuffles
// into RGB order.  Taken when no chroma sample of the wave's lane-step needs the reference's
// double-precision G (ChromaTerms::exact, about 2e-4 of the samples).
__device__ __forceinline__ uint32_t pair16(int lo, int hi) { return __builtin_amdgcn_perm(uint32_t(hi), uint32_t(lo), 0x05040100u); }
// The R and B terms of two chroma samples as one int16 pair, straight from their 32-bit multiply-add
// sums: bits 16..31 of each (one v_perm instead of two shifts and a v_perm; the terms fit int16).
// R: (91881 cr + 2^23) >> 16; B: (116130 cb + 2^23 + 64) >> 16 = (58065 cb + 2^22 + 32) >> 15
// (chroma_terms).
__device__ __forceinline__ uint32_t rb_pair(int c0, int c1, int k, int add) {
    const int x0 = mad24(c0, k, add), x1 = mad24(c1, k, add);
    return __builtin_amdgcn_perm(uint32_t(x1), uint32_t(x0), 0x07060302u);
}
__device__ __forceinline__ uint32_t r_pair(int cr0, int cr1) { return rb_pair(cr0, cr1, 91881, 128 << 16); }
__device__ __forceinline__ uint32_t b_pair(int cb0, int cb1) { return rb_pair(cb0, cb1, 116130, (128 << 16) + 64); }
// y + t of two int16 lanes; LO: t's low half serves both lanes (op_sel_hi), for the pixel pairs that
// share one chroma sample, so no duplicated pair is built
template <bool LO>
__device__ __forceinline__ uint32_t pk_add16(uint32_t y, uint32_t t) {
    uint32_t s;
    if (LO) asm("v_pk_add_u16 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(s) : "v"(y), "v"(t));
    else asm("v_pk_add_u16 %0, %1, %2" : "=v"(s) : "v"(y), "v"(t));
    return s;
}
// clamp(y + t, 0, 255) of the two lanes as bytes 0, 1 (bytes 2, 3 zero)
template <bool LO>
__device__ __forceinline__ uint32_t pk_sat_add(uint32_t y, uint32_t t) {
    uint32_t o;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(o) : "v"(pk_add16<LO>(y, t)));
    return o;
}
// the same as bytes 2, 3 of lo2, whose bytes 0, 1 are kept (SDWA destination: no v_perm to merge)
template <bool LO>
__device__ __forceinline__ uint32_t pk_sat_add_hi(uint32_t lo2, uint32_t y, uint32_t t) {
    asm("v_sat_pk_u8_i16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(lo2)
        : "v"(pk_add16<LO>(y, t)));
    return lo2;
}

// Terms of the 8 >> SH chroma samples under 8 pixels as per-word pairs (word u = pixels 2u, 2u+1).
// Returns the mask of samples (bit u) whose G needs the reference's double-precision path.
template <int SH>
__device__ __forceinline__ uint32_t terms_words(const int16_t* s_pl, uint32_t cboff, uint32_t croff, uint32_t (&TR)[4],
                                                uint32_t (&TG)[4], uint32_t (&TB)[4]) {
    constexpr int NU = 8 >> SH;
    int cb[8], cr[8];
    load_plane<SH>(s_pl, cboff, cb);
    load_plane<SH>(s_pl, croff, cr);
    ChromaTerms t[NU];
    uint32_t ex = 0;
#pragma unroll
    for (int u = 0; u < NU; u++) {
        t[u] = chroma_terms(cb[u], cr[u]);
        ex |= t[u].exact ? (1u << u) : 0u;
    }
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const int a = SH == 0 ? 2 * w : (SH == 1 ? w : w >> 1);  // sample of the word's pixels
        if (SH == 0) {
            TR[w] = r_pair(cr[a], cr[2 * w + 1]);
            TG[w] = pair16(t[a].g, t[2 * w + 1].g);
            TB[w] = b_pair(cb[a], cb[2 * w + 1]);
        } else {  // one sample under both pixels: the term in the low half (row_rgb_packed<true>)
            TR[w] = uint32_t(t[a].r);
            TG[w] = uint32_t(t[a].g);
            TB[w] = uint32_t(t[a].b);
        }
    }
    return ex;
}

// The rare fix-up of the packed path: the G byte of every pixel of this row whose chroma sample
// is in exmask, recomputed with the reference's double-precision formula (color.cpp:13-17).
template <int SH>
__device__ __forceinline__ void fix_g_exact(const uint4& Yq, const int16_t* s_pl, uint32_t cboff, uint32_t croff,
                                            uint32_t exmask, uint32_t (&w)[6]) {
    const uint32_t Y[4] = {Yq.x, Yq.y, Yq.z, Yq.w};
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int u = j >> SH;
        if ((exmask >> u) & 1u) {
            const int y = (j & 1) ? int32_t(Y[j >> 1]) >> 16 : int(int16_t(Y[j >> 1] & 0xFFFFu));
            const int g = color_g_exact(y, s_pl[cboff + u], s_pl[croff + u]);
            const int byte = 3 * j + 1;  // channel G of pixel j: byte 3j + 1 of the 24
            w[byte >> 2] = (w[byte >> 2] & ~(0xFFu << (8 * (byte & 3)))) | (uint32_t(g) << (8 * (byte & 3)));
        }
    }
}

// 8 pixels of one row: Y as 4 words of int16 pairs -> 24 RGB bytes in 6 words (pack24's order):
// per pixel pair and channel one packed add and one saturating pack to bytes (G's straight into
// the high half of R's word), then byte shuffles.  LO: terms in the words' low halves (a pixel
// pair on one chroma sample, terms_words<SH >= 1>), else one term per pixel (int16 pairs).
template <bool LO>
__device__ __forceinline__ void row_rgb_packed(const uint4& Yq, const uint32_t (&TR)[4], const uint32_t (&TG)[4],
                                               const uint32_t (&TB)[4], uint32_t (&w)[6]) {
    const uint32_t Y[4] = {Yq.x, Yq.y, Yq.z, Yq.w};
    uint32_t RG[4], B[4];  // RG: r0 r1 g0 g1; B: b0 b1 in the low half
#pragma unroll
    for (int u = 0; u < 4; u++) {
        RG[u] = pk_sat_add_hi<LO>(pk_sat_add<LO>(Y[u], TR[u]), Y[u], TG[u]);
        B[u] = pk_sat_add<LO>(Y[u], TB[u]);
    }
    // perm(hi, lo, sel): selector bytes 0-3 take lo's bytes, 4-7 hi's, 0x0c a zero byte
    w[0] = __builtin_amdgcn_perm(B[0], RG[0], 0x01040200u);                                            // r0 g0 b0 r1
    w[1] = __builtin_amdgcn_perm(RG[1], __builtin_amdgcn_perm(B[0], RG[0], 0x0c0c0503u), 0x06040100u);  // g1 b1 r2 g2
    w[2] = __builtin_amdgcn_perm(B[1], RG[1], 0x05030104u);                                            // b2 r3 g3 b3
    w[3] = __builtin_amdgcn_perm(B[2], RG[2], 0x01040200u);                                            // r4 g4 b4 r5
    w[4] = __builtin_amdgcn_perm(RG[3], __builtin_amdgcn_perm(B[2], RG[2], 0x0c0c0503u), 0x06040100u);  // g5 b5 r6 g6
    w[5] = __builtin_amdgcn_perm(B[3], RG[3], 0x05030104u);                                            // b6 r7 g7 b7
}

// The same 24 bytes with the channels interleaved by the adds themselves: pixels 2u, 2u + 1 are
// the int16 pairs (r0 g0) (b0 r1) (g1 b1), each y + t of its lanes with y taken from the pixel word's
// low or high half (op_sel), against the term words A = (tr0, tg0), B = (tb0, tr1), C = (tg1, tb1)
// (terms_il).  Output word k is pairs 2k and 2k + 1, saturated straight into its two halves: 12
// adds and 12 saturations per 8 pixels, no byte shuffles (row_rgb_packed: 12 + 12 + 8 v_perm).
__device__ __forceinline__ uint32_t pk_add_ll(uint32_t y, uint32_t t) {  // (y.lo + t.lo, y.lo + t.hi)
    uint32_t s;
    asm("v_pk_add_u16 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(s) : "v"(y), "v"(t));
    return s;
}
__device__ __forceinline__ uint32_t pk_add_hh(uint32_t y, uint32_t t) {  // (y.hi + t.lo, y.hi + t.hi)
    uint32_t s;
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(s) : "v"(y), "v"(t));
    return s;
}
__device__ __forceinline__ uint32_t sat_lo(uint32_t x) {  // bytes 0, 1 (2, 3 zero)
    uint32_t o;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(o) : "v"(x));
    return o;
}
__device__ __forceinline__ uint32_t sat_hi(uint32_t lo2, uint32_t x) {  // bytes 2, 3 of lo2
    asm("v_sat_pk_u8_i16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(lo2) : "v"(x));
    return lo2;
}
__device__ __forceinline__ void row_rgb_il(const uint4& Yq, const uint32_t (&A)[4], const uint32_t (&B)[4],
                                           const uint32_t (&C)[4], uint32_t (&w)[6]) {
    const uint32_t Y[4] = {Yq.x, Yq.y, Yq.z, Yq.w};
    uint32_t P[12];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        P[3 * u] = pk_add_ll(Y[u], A[u]);
        P[3 * u + 1] = pk_add16<false>(Y[u], B[u]);
        P[3 * u + 2] = pk_add_hh(Y[u], C[u]);
    }
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = sat_hi(sat_lo(P[2 * k]), P[2 * k + 1]);
}
// The term words of row_rgb_il for the 8 >> SH chroma samples under 8 pixels (word u = pixels 2u,
// 2u + 1): R and B straight from the high halves of their multiply-add sums (rb_pair), G's low half.
// Returns the mask of samples (bit u) whose G needs the reference's double-precision path.
template <int SH>
__device__ __forceinline__ uint32_t terms_il(const int16_t* s_pl, uint32_t cboff, uint32_t croff, uint32_t (&A)[4],
                                             uint32_t (&B)[4], uint32_t (&C)[4]) {
    constexpr int NU = 8 >> SH;
    int cb[8], cr[8];
    load_plane<SH>(s_pl, cboff, cb);
    load_plane<SH>(s_pl, croff, cr);
    uint32_t xr[NU], xb[NU], tg[NU];
    uint32_t ex = 0;
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const ChromaTerms t = chroma_terms(cb[u], cr[u]);
        ex |= t.exact ? (1u << u) : 0u;
        xr[u] = uint32_t(mad24(cr[u], 91881, 128 << 16));
        xb[u] = uint32_t(mad24(cb[u], 116130, (128 << 16) + 64));
        tg[u] = uint32_t(t.g);
    }
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const int a0 = SH == 0 ? 2 * w : (SH == 1 ? w : w >> 1), a1 = SH == 0 ? 2 * w + 1 : a0;  // samples of pixels 2w, 2w + 1
        A[w] = __builtin_amdgcn_perm(tg[a0], xr[a0], 0x05040302u);  // (tr0, tg0)
        B[w] = __builtin_amdgcn_perm(xr[a1], xb[a0], 0x07060302u);  // (tb0, tr1)
        C[w] = __builtin_amdgcn_perm(xb[a1], tg[a1], 0x07060100u);  // (tg1, tb1)
    }
    return ex;
}

// The 4:2:0 tail step: 4 pixels of two rows that share their two chroma samples (both chroma
// planes subsampled 2x2).  A 4:2:0 tile of 10 MCUs has 160 8-pixel row-pair groups, two and a half
// lane-steps: the last half step is done as 64 4-pixel halves, so no lane idles (k_idct_color).
// LO: terms in the low halves (both pixels of a word share their sample), else one term per pixel
template <bool LO = true>
__device__ __forceinline__ void rgb4_packed(const uint2& Yq, const uint32_t (&TR)[2], const uint32_t (&TG)[2],
                                            const uint32_t (&TB)[2], uint32_t (&w)[3]) {
    const uint32_t Y[2] = {Yq.x, Yq.y};
    uint32_t RG[2], B[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
        RG[u] = pk_sat_add_hi<LO>(pk_sat_add<LO>(Y[u], TR[u]), Y[u], TG[u]);
        B[u] = pk_sat_add<LO>(Y[u], TB[u]);
    }
    w[0] = __builtin_amdgcn_perm(B[0], RG[0], 0x01040200u);                                            // r0 g0 b0 r1
    w[1] = __builtin_amdgcn_perm(RG[1], __builtin_amdgcn_perm(B[0], RG[0], 0x0c0c0503u), 0x06040100u);  // g1 b1 r2 g2
    w[2] = __builtin_amdgcn_perm(B[1], RG[1], 0x05030104u);                                            // b2 r3 g3 b3
}
__device__ __forceinline__ void fix_g4_exact(const uint2& Yq, const int (&cb)[2], const int (&cr)[2], uint32_t exmask,
                                             uint32_t (&w)[3]) {
    const uint32_t Y[2] = {Yq.x, Yq.y};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int u = j >> 1;
        if ((exmask >> u) & 1u) {
            const int y = (j & 1) ? int32_t(Y[u]) >> 16 : int(int16_t(Y[u] & 0xFFFFu));
            const int g = color_g_exact(y, cb[u], cr[u]);
            const int byte = 3 * j + 1;
            w[byte >> 2] = (w[byte >> 2] & ~(0xFFu << (8 * (byte & 3)))) | (uint32_t(g) << (8 * (byte & 3)));
        }
    }
}
// n <= 4 pixels (12 bytes when n == 4) of a row
__device__ __forceinline__ void store12(uint8_t* dst, const uint32_t (&w)[3], uint32_t n) {
    if (n == 4 && (reinterpret_cast<uintptr_t>(dst) & 3) == 0) {
        auto d1 = gptr(reinterpret_cast<uint32_t*>(dst));
        d1[0] = w[0];
        d1[1] = w[1];
        d1[2] = w[2];
    } else {
        auto d = gptr(dst);
#pragma unroll
        for (int k = 0; k < 12; k++)
            if (uint32_t(k) < 3 * n) d[k] = uint8_t(w[k / 4] >> (8 * (k % 4)));
    }
}
// 4 pixels (2 words of Y) -> 12 bytes, row_rgb_il's form
__device__ __forceinline__ void rgb4_il(const uint2& Yq, const uint32_t (&A)[2], const uint32_t (&B)[2],
                                        const uint32_t (&C)[2], uint32_t (&w)[3]) {
    const uint32_t Y[2] = {Yq.x, Yq.y};
    uint32_t P[6];
#pragma unroll
    for (int u = 0; u < 2; u++) {
        P[3 * u] = pk_add_ll(Y[u], A[u]);
        P[3 * u + 1] = pk_add16<false>(Y[u], B[u]);
        P[3 * u + 2] = pk_add_hh(Y[u], C[u]);
    }
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] = sat_hi(sat_lo(P[2 * k]), P[2 * k + 1]);
}
// term words (terms_il) of pixels 2w, 2w + 1 on chroma samples a0, a1
__device__ __forceinline__ void term_words_of(const ChromaTerms& t0, int cb0, int cr0, const ChromaTerms& t1, int cb1,
                                              int cr1, uint32_t& A, uint32_t& B, uint32_t& C) {
    const uint32_t xr0 = uint32_t(mad24(cr0, 91881, 128 << 16)), xr1 = uint32_t(mad24(cr1, 91881, 128 << 16));
    const uint32_t xb0 = uint32_t(mad24(cb0, 116130, (128 << 16) + 64)), xb1 = uint32_t(mad24(cb1, 116130, (128 << 16) + 64));
    A = __builtin_amdgcn_perm(uint32_t(t0.g), xr0, 0x05040302u);
    B = __builtin_amdgcn_perm(xr1, xb0, 0x07060302u);
    C = __builtin_amdgcn_perm(xb1, uint32_t(t1.g), 0x07060100u);
}
__device__ __forceinline__ void colour4x2(const int16_t* s_pl, uint32_t yoff, uint32_t ypitch, uint32_t cboff,
                                          uint32_t croff, uint32_t (&w0)[3], uint32_t (&w1)[3]) {
    const uint32_t cbw = *reinterpret_cast<const uint32_t*>(s_pl + cboff);
    const uint32_t crw = *reinterpret_cast<const uint32_t*>(s_pl + croff);
    const int cb[2] = {int(int16_t(cbw & 0xFFFFu)), int32_t(cbw) >> 16};
    const int cr[2] = {int(int16_t(crw & 0xFFFFu)), int32_t(crw) >> 16};
    const ChromaTerms t0 = chroma_terms(cb[0], cr[0]), t1 = chroma_terms(cb[1], cr[1]);
    uint32_t A[2], B[2], C[2];  // word u = pixels 2u, 2u + 1 on sample u
    term_words_of(t0, cb[0], cr[0], t0, cb[0], cr[0], A[0], B[0], C[0]);
    term_words_of(t1, cb[1], cr[1], t1, cb[1], cr[1], A[1], B[1], C[1]);
    const uint32_t ex = (t0.exact ? 1u : 0u) | (t1.exact ? 2u : 0u);
    const uint2 Y0 = *reinterpret_cast<const uint2*>(s_pl + yoff), Y1 = *reinterpret_cast<const uint2*>(s_pl + yoff + ypitch);
    rgb4_il(Y0, A, B, C, w0);
    rgb4_il(Y1, A, B, C, w1);
    if (__any(ex != 0u)) {
        fix_g4_exact(Y0, cb, cr, ex, w0);
        fix_g4_exact(Y1, cb, cr, ex, w1);
    }
}

// The 4:4:4 tail step: 4 pixels of one row, one chroma sample each.  A 4:4:4 tile of 20 MCUs has
// 160 8-pixel groups, two and a half lane-steps: the last half step is done as 64 4-pixel halves.
__device__ __forceinline__ void colour4x1(const int16_t* s_pl, uint32_t yoff, uint32_t cboff, uint32_t croff,
                                          uint32_t (&w)[3]) {
    const uint2 cbq = *reinterpret_cast<const uint2*>(s_pl + cboff);
    const uint2 crq = *reinterpret_cast<const uint2*>(s_pl + croff);
    const int cb[4] = {int(int16_t(cbq.x & 0xFFFFu)), int32_t(cbq.x) >> 16, int(int16_t(cbq.y & 0xFFFFu)), int32_t(cbq.y) >> 16};
    const int cr[4] = {int(int16_t(crq.x & 0xFFFFu)), int32_t(crq.x) >> 16, int(int16_t(crq.y & 0xFFFFu)), int32_t(crq.y) >> 16};
    ChromaTerms t[4];
    uint32_t ex = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        t[u] = chroma_terms(cb[u], cr[u]);
        ex |= t[u].exact ? (1u << u) : 0u;
    }
    uint32_t A[2], B[2], C[2];  // word u = pixels 2u, 2u + 1 on samples 2u, 2u + 1
    term_words_of(t[0], cb[0], cr[0], t[1], cb[1], cr[1], A[0], B[0], C[0]);
    term_words_of(t[2], cb[2], cr[2], t[3], cb[3], cr[3], A[1], B[1], C[1]);
    const uint2 Y0 = *reinterpret_cast<const uint2*>(s_pl + yoff);
    rgb4_il(Y0, A, B, C, w);
    if (__any(ex != 0u)) {
        const uint32_t Y[2] = {Y0.x, Y0.y};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if ((ex >> j) & 1u) {
                const int y = (j & 1) ? int32_t(Y[j >> 1]) >> 16 : int(int16_t(Y[j >> 1] & 0xFFFFu));
                const int g = color_g_exact(y, cb[j], cr[j]);
                const int byte = 3 * j + 1;
                w[byte >> 2] = (w[byte >> 2] & ~(0xFFu << (8 * (byte & 3)))) | (uint32_t(g) << (8 * (byte & 3)));
            }
        }
    }
}

// One wave per tile of tile_mcus x tile_mrows MCUs (host-chosen, <= 64 blocks):
//  1. lane j owns block j: its LDS row (pitch 65 words) is filled with the block's DC and AC
//     entries, dequantised in zig-zag order (parser.cpp:111,130) and placed at natural positions
//  2. integer IDCT entirely in registers: rows, then columns (idct.cpp:34-122)
//  3. the clipped samples go to int16 component planes of the tile (16-byte LDS stores)
//  4. lane = 8 consecutive output pixels: replicate chroma upsampling from the planes, colour
//     (color.cpp:8-19), 24 contiguous output bytes per lane
// Every LDS access pattern is conflict-free or 16-byte-vectorised; no LDS traffic in the IDCT.

// 8 horizontally consecutive output samples of one plane row, replicate-upsampled by 2^shx:
// one aligned 16-byte LDS read, then register selects only (no dynamically indexed arrays).
__device__ __forceinline__ void load8_samples(const int16_t* pl, uint32_t off, uint32_t shx, int (&v)[8]) {
    const uint4 q = *reinterpret_cast<const uint4*>(pl + (off & ~7u));
    const uint32_t d2 = (off & 7u) >> 1;  // first dword holding the samples (shx >= 1: off even)
    const uint32_t a0 = d2 == 0 ? q.x : (d2 == 1 ? q.y : (d2 == 2 ? q.z : q.w));
    const uint32_t a1 = d2 == 0 ? q.y : (d2 == 1 ? q.z : q.w);
    const int x0 = int(int16_t(q.x & 0xFFFFu)), x1 = int32_t(q.x) >> 16;
    const int x2 = int(int16_t(q.y & 0xFFFFu)), x3 = int32_t(q.y) >> 16;
    const int x4 = int(int16_t(q.z & 0xFFFFu)), x5 = int32_t(q.z) >> 16;
    const int x6 = int(int16_t(q.w & 0xFFFFu)), x7 = int32_t(q.w) >> 16;
    const int l0 = int(int16_t(a0 & 0xFFFFu)), h0 = int32_t(a0) >> 16;
    const int l1 = int(int16_t(a1 & 0xFFFFu)), h1 = int32_t(a1) >> 16;
    const bool s0 = shx == 0, s1 = shx == 1;
    v[0] = s0 ? x0 : l0;
    v[1] = s0 ? x1 : l0;
    v[2] = s0 ? x2 : (s1 ? h0 : l0);
    v[3] = s0 ? x3 : (s1 ? h0 : l0);
    v[4] = s0 ? x4 : (s1 ? l1 : h0);
    v[5] = s0 ? x5 : (s1 ? l1 : h0);
    v[6] = s0 ? x6 : (s1 ? h1 : h0);
    v[7] = s0 ? x7 : (s1 ? h1 : h0);
}

// Fancy-upsampling planes in HBM: component c of an image at int16 offset fancy_plane_off, pitch
// mcux * h[c] * 8 samples, mcuy * v[c] * 8 rows (the padded MCU grid).
__device__ __forceinline__ size_t fancy_plane_off(const ImgDesc& im, uint32_t c) {
    size_t off = 0;
    for (uint32_t k = 0; k < c; k++) off += size_t(im.mcux * im.h[k] * 8) * (im.mcuy * im.v[k] * 8);
    return off;
}

// LDS of a tile (8112 B, so 20 waves fit a CU: 5 per SIMD, which the kernel's 96 VGPRs allow too):
//  * staging: kTileMaxBlocks rows of 64 int16 (128 B, zig-zag order), the 16-byte quads of lane l's
//    row XOR-swizzled by (l >> 1) & 7 so that a wave's ds_read_b128 of one quad index from every row
//    is bank-conflict free (the 16 lanes of each of its four lane groups hit 16 distinct quad slots)
//  * then, reusing the same words, the tile's component planes (int16, unpadded: exactly the tile's
//    kTileMaxBlocks * 64 samples)
//  * the quant steps of the image's components
constexpr int kIdctBufWords = kTileMaxBlocks * 32;
constexpr int kQzWords = 3 * 36;  // quant steps per component, zig-zag order, as u16 pairs (pitch 36
                                  // words: 16-byte rows; a wave reads at most 3 distinct rows)
static_assert(kIdctBufWords * 4 + kQzWords * 4 <= 8192, "k_idct_color must fit 20 waves per CU");
// Byte address (in s_buf) of quad q of lane l's staging row; base = staging_base(l).
__device__ __forceinline__ uint32_t staging_base(uint32_t l) { return l * 128u + (((l >> 1) & 7u) << 4); }
#ifndef JD_PRE_QUADS
#define JD_PRE_QUADS 4
#endif
constexpr int kPreQuads = JD_PRE_QUADS;  // entry quads per lane loaded before the DC prediction

// A tile's lane: lane j owns block j of the tile (MCU m, block bb within the MCU).
struct TileLaneGeo {
    uint32_t m, bb, comp;
    bool have;
};
template <int M = kModeGen>
__device__ __forceinline__ TileLaneGeo tile_lane_geo(const ImgDesc& im, const TileGeo& G, uint32_t lane) {
    TileLaneGeo L;
    const uint32_t bpm = TMode<M>::bpm(im);
    L.m = TMode<M>::kFixed ? lane / bpm : div_small(lane, magic16(bpm));
    L.bb = lane - L.m * bpm;
    L.have = L.m < G.nm;
    L.comp = (TMode<M>::pattern(im) >> (2 * L.bb)) & 3u;
    return L;
}

template <int M = kModeGen>
__device__ __forceinline__ BlockInfo load_block_info(const BatchDev& b, const ImgDesc& im, const TileGeo& G,
                                                     const TileLaneGeo& L) {
    return L.have ? b.blocks[im.block_base + uint64_t(G.g0 + L.m) * TMode<M>::bpm(im) + L.bb] : BlockInfo{0u, 0u};
}

// The lane's AC entries: 16-bit slots [first, first + cnt) of the image's entry array, read as
// 16-byte quads (8 slots) from the quad holding the first one (lead = its position in that quad).
// A block of a corrupt stream may never have been written: never index past the image's entries.
struct EntryRange {
    const uint16_t* ep;  // 16-byte aligned
    uint32_t lead;
    int cnt, n4;         // slots, quads (cnt == 0: no quad is touched)
    bool esc;            // the block has an escaped (wide) value
};
__device__ __forceinline__ EntryRange entry_range(const BatchDev& b, const ImgDesc& im, const BlockInfo& bi, bool have) {
    EntryRange r;
    r.cnt = have ? int(bi.cnt_dc >> kCntShift) : 0;
    if (uint64_t(bi.entry_start) + uint64_t(r.cnt) > 2ull * im.entry_cap) r.cnt = 0;
    r.esc = r.cnt > 0 && (bi.cnt_dc & kCntEsc) != 0;
    r.lead = bi.entry_start & 7u;
    r.ep = reinterpret_cast<const uint16_t*>(b.entries + im.entry_base) + (bi.entry_start - r.lead);
    r.n4 = r.cnt > 0 ? int(r.lead + uint32_t(r.cnt) + 7u) >> 3 : 0;
    return r;
}

// The first kPreQuads quads (the entry buffer is padded by 64 B past its last slot).
__device__ __forceinline__ void load_entry_quads(const EntryRange& r, uint4 (&E)[kPreQuads]) {
#pragma unroll
    for (int u = 0; u < kPreQuads; u++)
        E[u] = (u < r.n4) ? *reinterpret_cast<const uint4*>(r.ep + 8 * u) : make_uint4(0, 0, 0, 0);
}

// Slots of quad index qi (its 4 words in v) to the lane's staging row at their zig-zag positions:
// int16 zz of the row is at byte 2 zz, swizzled (staging_base): row base ^ (2 zz & 0x7E).
// value = slot >> 6 (arithmetic), zz = slot & 63 (blocks without escaped values).
// Per slot one compare against the quad's limit (slot q is the block's when q < lead + cnt - 8 qi,
// and, in quad 0, q >= lead); both values of a word by one packed arithmetic shift, the high one
// stored from the word's upper half (ds_write_b16_d16_hi).
#ifndef JD_ABL_PHASE
#define JD_ABL_PHASE 0  // diagnostic builds (wrong pixels): k_idct_color stops after the IDCT's plane
                        // stores (1) or after the entry scatter (2): SQ counters of the phases
#endif
#ifndef JD_ABL_SCATTER
#define JD_ABL_SCATTER 0  // diagnostic builds (wrong pixels): 1 = every slot to a fixed, bank-conflict-free
                          // position of its row; 2 = no scatter stores
#endif
__device__ __forceinline__ void scatter_quad(uint8_t* s_bytes, uint32_t base, const uint4& v, int qi,
                                             const EntryRange& r) {
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const int lim = int(r.lead) + r.cnt - 8 * qi;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const s16x2 val = __builtin_bit_cast(s16x2, w[d]) >> short(6);
        if (JD_ABL_SCATTER == 2) {
            if (2 * d < lim) __builtin_amdgcn_sched_barrier(0);
            continue;
        }
        if (JD_ABL_SCATTER == 1) {  // dword (l + d) mod 32 of the lane's row: bank (l + d) mod 32
            const uint32_t a = (base & ~127u) | (((threadIdx.x + uint32_t(d)) & 31u) << 2);
            if (2 * d < lim && (qi > 0 || 2 * d >= int(r.lead))) *reinterpret_cast<int16_t*>(s_bytes + a) = val.x;
            if (2 * d + 1 < lim && (qi > 0 || 2 * d + 1 >= int(r.lead))) *reinterpret_cast<int16_t*>(s_bytes + (a | 2u)) = val.y;
            continue;
        }
        if (2 * d < lim && (qi > 0 || 2 * d >= int(r.lead)))
            *reinterpret_cast<int16_t*>(s_bytes + (base ^ ((w[d] << 1) & 0x7Eu))) = val.x;
        if (2 * d + 1 < lim && (qi > 0 || 2 * d + 1 >= int(r.lead)))
            *reinterpret_cast<int16_t*>(s_bytes + (base ^ ((w[d] >> 15) & 0x7Eu))) = val.y;
    }
}

// Sparse -> dense for the lane's block: the prefetched quads, then the rest (blocks with more
// than 8 * kPreQuads - lead slots) four quads in flight at a time.  A block with an escaped value
// (|value| > 511: rare below quality 95) walks its slots one by one instead.
__device__ __forceinline__ void scatter_entries(uint32_t* s_buf, uint32_t base, const EntryRange& r,
                                                const uint4 (&E)[kPreQuads]) {
    uint8_t* row = reinterpret_cast<uint8_t*>(s_buf);
    if (__builtin_expect(r.esc, 0)) {
        for (int i = 0; i < r.cnt; i++) {
            const uint32_t h = r.ep[r.lead + i];
            int v = int(int16_t(uint16_t(h))) >> 6;
            if ((h & 0xFFC0u) == 0x8000u && i + 1 < r.cnt) v = int(int16_t(r.ep[r.lead + ++i]));
            *reinterpret_cast<int16_t*>(row + (base ^ ((h << 1) & 0x7Eu))) = int16_t(v);
        }
        return;
    }
    // quads no lane of the wave has are skipped (wave-uniform): their slots would all be masked
#pragma unroll
    for (int u = 0; u < kPreQuads; u++)
        if (u == 0 || __any(u < r.n4)) scatter_quad(row, base, E[u], u, r);
    for (int c = kPreQuads; c < r.n4; c += 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
            v[u] = (c + u < r.n4) ? *reinterpret_cast<const uint4*>(r.ep + 8 * (c + u)) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; u++) scatter_quad(row, base, v[u], c + u, r);
    }
}

// DC prediction (parser.cpp:106-111): segmented scan of the tile's DC differences onto its entry
// predictors (tile_dc, k_dc_scan); a block that starts an interval resets its component's
// predictor.  Exact int, as the reference's int predictor: the int16 staging is bypassed.
__device__ __forceinline__ int tile_dc_predict(const TileGeo& G, const TileLaneGeo& L, const BlockInfo& bi,
                                               const DcPred& cin, uint32_t lane) {
    const int d = L.have ? cnt_dc_dc(bi.cnt_dc) : 0;
    const bool start = L.have && L.bb == 0 && tile_mcu_starts(G, L.m);
    const uint64_t smask = __ballot(start);
    const uint32_t comp = L.comp;
    const int p0 = wave_scan_dpp(comp == 0 ? d : 0);
    const int p1 = wave_scan_dpp(comp == 1 ? d : 0);
    const int p2 = wave_scan_dpp(comp == 2 ? d : 0);
    int dc = comp == 0 ? p0 : (comp == 1 ? p1 : p2);
    const uint64_t upto = smask & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
    if (upto == 0) dc += comp == 0 ? cin.p0 : (comp == 1 ? cin.p1 : cin.p2);
    if (smask & ~1ull) {  // wave-uniform: an interval starts inside the tile
        const int ls = upto ? 63 - int(__clzll(upto)) : 0;  // my segment's first lane
        const int src = max(ls - 1, 0);
        const int q0 = __shfl(p0, src, 64), q1 = __shfl(p1, src, 64), q2 = __shfl(p2, src, 64);
        if (upto && ls > 0) dc -= comp == 0 ? q0 : (comp == 1 ? q1 : q2);
    }
    return dc;
}

// Quant steps of the image's components to LDS (lane = 4 steps of one component).
__device__ __forceinline__ void stage_quant(const BatchDev& b, const ImgDesc& im, int* s_qz, uint32_t lane) {
    if (lane < 16 * im.ncomp) {
        const uint32_t c = lane >> 4, q = lane & 15u;
        const uint2 v = *reinterpret_cast<const uint2*>(b.qtabs + size_t(im.qslot[c]) * 64 + 4 * q);
        *reinterpret_cast<uint2*>(s_qz + c * 36 + 2 * q) = v;
    }
}

// Each lane zeroes its own staging row, quad j at base ^ 16 j: no per-store bound test, and for one
// j the wave's 16-byte stores hit distinct bank groups (the row swizzle of staging_base).
__device__ __forceinline__ void zero_staging(uint32_t* s_buf, uint32_t lane) {
    if (lane < uint32_t(kTileMaxBlocks)) {
        uint8_t* const row = reinterpret_cast<uint8_t*>(s_buf);
        const uint32_t base = staging_base(lane);
        const uint4 zq = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) *reinterpret_cast<uint4*>(row + (base ^ (16u * j))) = zq;
    }
}

// The rest of a tile once its staging rows hold the quantised coefficients (zig-zag order) and
// dc_pred the lane's DC: dequantisation, IDCT, planes, upsample + colour + store.
//  * EXACT = false (k_idct_color): a wave with a coefficient beyond the fast IDCT's range (never
//    seen in real images) appends its tile to slow_tiles and returns false;
//  * EXACT = true (k_idct_color_exact) decodes those tiles with the exact IDCT form.
template <bool EXACT, int M, class Mid>
__device__ __forceinline__ bool idct_colour_tile(const BatchDev& b, const ImgDesc& im, uint32_t img, uint32_t tile,
                                                 const TileGeo& G, const TileLaneGeo& L, int dc_pred, bool esc,
                                                 uint32_t* s_buf, const int* s_qz, Mid&& mid) {
    const uint32_t lane = threadIdx.x;
    using TM_ = TMode<M>;
    const uint32_t TM = TM_::tm(im), nc = TM_::ncomp(im);
    const uint32_t m0 = G.m0, r0 = G.ty;
    const uint32_t mi = L.m, mr = 0, bb = L.bb, comp = L.comp;
    const bool have = L.have;
    // dequantise in zig-zag order (24-bit multiplies: |coef| < 2^15, q < 2^16) into natural
    // positions (a compile-time permutation of registers), then the IDCT in registers
    //    The fast IDCT form needs every dequantised coefficient within +-2^16: an AC coefficient
    //    c is when |c| <= 2^(k-1) with 2^(k-1) * (largest quant step) < 2^16 (host: im.qmask),
    //    i.e. when bits k-1..15 of c all equal its sign: c ^ (c << 1) has bits k..15 clear.
    // the lane's staging row as 8 quads (swizzled: quad q at base ^ 16 q); lanes without a block
    // read row 0 (their results are never used)
    const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_buf);
    const uint32_t sbase = staging_base(have ? lane : 0u);
    uint32_t rw[32];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const uint4 v = *reinterpret_cast<const uint4*>(s_bytes + (sbase ^ (16u * q)));
        rw[4 * q + 0] = v.x;
        rw[4 * q + 1] = v.y;
        rw[4 * q + 2] = v.z;
        rw[4 * q + 3] = v.w;
    }
    const uint4* qz4 = reinterpret_cast<const uint4*>(s_qz + comp * 36);
    const int dq0 = dc_pred * int(reinterpret_cast<const uint16_t*>(s_qz)[comp * 72]);
    if (!EXACT) {  // range test before dequantising: the branch then holds no 64-value block
        // When the quant steps are below 64 (qmask bit 9 clear: k >= 10), every value of a 16-bit
        // slot (|v| <= 511) passes, so only a wave with an escaped value tests its coefficients.
        bool in_range = !have || uint32_t(dq0 + 32768) <= 65535u;
        if ((im.qmask & 0x200u) || __any(have && esc)) {  // wave-uniform
            uint32_t acc = 0;
#pragma unroll
            for (int p = 0; p < 32; p++) {
                const uint32_t w = rw[p];
                acc |= w ^ (w << 1);
            }
            in_range = in_range && (!have || (acc & im.qmask) == 0);
        }
        if (!__all(in_range)) {  // wave-uniform
            if (lane == 0) {
                const uint32_t k = uint32_t(atomicAdd(&b.counters[1], 1ull));
                b.slow_tiles[k] = TileRef{img, tile};
            }
            mid();
            return false;
        }
    }
    uint32_t pk[32];  // row r's int16 pairs: pk[4 r] .. pk[4 r + 3]
    if (!EXACT) {
        // every dequantised coefficient fits int16: packed multiplies in zig-zag order, DC in place
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        uint32_t dw[32];
#pragma unroll
        for (int p4 = 0; p4 < 8; p4++) {
            const uint4 qv = qz4[p4];
            const uint32_t qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
            for (int k = 0; k < 4; k++)
                dw[4 * p4 + k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, rw[4 * p4 + k]) * __builtin_bit_cast(u16x2, qw[k]));
        }
        dw[0] = __builtin_amdgcn_perm(dw[0], uint32_t(dq0), 0x07060100u);
        // row 7 is zero across a whole C2 tile in 96 % of tiles: its row pass is skipped by a
        // wave-uniform branch (a second copy of the IDCT without it made the kernel spill)
        idct_block_dot2<8>(dw, pk, __all(!have || row_bits<7>(dw) == 0u));
    } else {
        int blk[64];
#pragma unroll
        for (int p4 = 0; p4 < 8; p4++) {
            const uint4 qv = qz4[p4];
            const uint32_t qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int p = 4 * p4 + k;
                const uint32_t w = rw[p];
                blk[kNatOfZz[2 * p]] = p == 0 ? dq0 : __mul24(int(int16_t(w & 0xFFFFu)), int(qw[k] & 0xFFFFu));
                blk[kNatOfZz[2 * p + 1]] = __mul24(int32_t(w) >> 16, int(qw[k] >> 16));
            }
        }
        idct_block_exact(blk);
#pragma unroll
        for (int q = 0; q < 32; q++) pk[q] = pair16(blk[2 * q], blk[2 * q + 1]);
    }
    mid();  // (k_idct_color: the next tile's entry loads, issued here so they are not live across the IDCT)
    if (b.fancy) {  // wave-uniform: component planes to HBM, k_colour_fancy takes it from there
        if (have) {
            const uint32_t hc = TM_::h(im, comp), vc = TM_::v(im, comp);
            const uint32_t t = bb - TM_::cb0(im, comp);
            const uint32_t tyb = t >> __builtin_ctz(hc), txb = t - tyb * hc;  // hc in {1, 2, 4}
            // (the plane pitch in a local: the stores below may alias the descriptor as far as the
            // compiler knows, and it would reload im.mcux after each of them)
            const uint32_t ppc = im.mcux * hc * 8;
            int16_t* dst = reinterpret_cast<int16_t*>(im.planes) + fancy_plane_off(im, comp) +
                           size_t(((r0 + mr) * vc + tyb) * 8) * ppc + ((m0 + mi) * hc + txb) * 8;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                *gptr(reinterpret_cast<u32x4*>(dst)) = u32x4{pk[4 * r], pk[4 * r + 1], pk[4 * r + 2], pk[4 * r + 3]};
                dst += ppc;
            }
        }
        return true;
    }
    __syncthreads();  // every row read back before the planes overwrite the staging area

    // component planes (int16), pitch = plane width
    int16_t* s_pl = reinterpret_cast<int16_t*>(s_buf);  // planes reuse the staging area
    uint32_t pbase[3] = {0u, 0u, 0u}, ppitch[3] = {8u, 8u, 8u};
    {
        uint32_t off = 0;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            if (uint32_t(c) < nc) {
                ppitch[c] = TM * TM_::h(im, c) * 8;
                pbase[c] = off;
                off += ppitch[c] * TM_::v(im, c) * 8;  // one MCU row
            }
        }
    }
    if (have) {
        const uint32_t hc = TM_::h(im, comp);
        const uint32_t t = bb - TM_::cb0(im, comp);
        const uint32_t tyb = t >> __builtin_ctz(hc), txb = t - tyb * hc;  // hc in {1, 2, 4}
        const uint32_t pitch = comp == 0 ? ppitch[0] : (comp == 1 ? ppitch[1] : ppitch[2]);
        const uint32_t base = comp == 0 ? pbase[0] : (comp == 1 ? pbase[1] : pbase[2]);
        int16_t* dst = s_pl + base + ((mr * TM_::v(im, comp) + tyb) * 8) * pitch + (mi * hc + txb) * 8;
#pragma unroll
        for (int r = 0; r < 8; r++)
            *reinterpret_cast<uint4*>(dst + r * pitch) = uint4{pk[4 * r], pk[4 * r + 1], pk[4 * r + 2], pk[4 * r + 3]};
    }
    __syncthreads();
    if (JD_ABL_PHASE == 1) return true;  // diagnostic builds: no colour stage (the planes are kept)

    // upsample + colour: 8 pixels of one row per lane-step, or of two rows when both chroma
    // planes are vertically subsampled (the two rows share their chroma samples and terms)
    const uint32_t lg_mw = TM_::lg_mw(im), lg_mh = TM_::lg_mh(im);
    const uint32_t gpr = (TM << lg_mw) >> 3;  // 8-pixel groups per tile row
    const uint32_t th = 1u << lg_mh;
    const uint32_t W = im.width, H = im.height, W3 = 3u * W;  // W3 < 2^18
    const uint32_t x_tile = m0 << lg_mw, y_tile = r0 << lg_mh;
    const uint32_t shx1 = TM_::shx(im, 1), shy1 = TM_::shy(im, 1), shx2 = TM_::shx(im, 2), shy2 = TM_::shy(im, 2);
    const uint32_t cmode = nc == 1 ? 3u : (shx1 == shx2 ? shx1 : 4u);
    const bool pair = cmode <= 2u && shy1 >= 1u && shy2 >= 1u;  // wave-uniform; th is even then
    const uint32_t rows = pair ? 2u : 1u, ngy = th / rows;
    uint8_t* out = reinterpret_cast<uint8_t*>(im.rgb);
    // lane -> (row group gy, column group gc), advanced by 64 groups per iteration
    const uint32_t step_y = kIdctThreads / gpr, step_c = kIdctThreads - step_y * gpr;
    uint32_t gy = gpr <= 64u ? div_small(lane, magic16(gpr)) : 0u, gc = lane - gy * gpr;
    // 4:2:0 (row pairs, chroma subsampled 2x horizontally): when the last lane-step would be at most
    // half full, it is done as 4-pixel halves of the remaining groups (colour4x2) instead
    const uint32_t ngroups = gpr * ngy, nfull = ngroups / kIdctThreads, nrem = ngroups - nfull * kIdctThreads;
    // 4:4:4 (per-pixel chroma, single rows) likewise, as 4-pixel halves of one row (colour4x1)
    const bool halves = nrem != 0u && 2u * nrem <= kIdctThreads &&
                        ((pair && cmode == 1u) || (!pair && cmode == 0u));  // wave-uniform
    const uint32_t nsteps = halves ? nfull : ~0u;
    for (uint32_t st = 0; gy < ngy && st < nsteps;
         st++, gy += step_y + (gc + step_c >= gpr ? 1u : 0u), gc = gc + step_c >= gpr ? gc + step_c - gpr : gc + step_c) {
        const uint32_t py = gy * rows, gx = gc << 3;
        const uint32_t y = y_tile + py, x = x_tile + gx;
        if (y >= H || x >= W) continue;
        const uint32_t yoff = pbase[0] + py * ppitch[0] + gx;
        const uint32_t cboff = pbase[1] + (py >> shy1) * ppitch[1] + (gx >> shx1);
        const uint32_t croff = pbase[2] + (py >> shy2) * ppitch[2] + (gx >> shx2);
        uint32_t w0[6], w1[6];
        if (cmode <= 2u) {  // wave-uniform: both chroma planes share one horizontal factor
            // packed integer colour for every pixel; G of the few pixels whose chroma sample needs
            // the reference's double-precision path is patched afterwards (about 5 % of the
            // lane-steps have one such sample in some lane)
            uint32_t TA[4], TB[4], TC[4], ex;
            switch (cmode) {
                case 0: ex = terms_il<0>(s_pl, cboff, croff, TA, TB, TC); break;
                case 1: ex = terms_il<1>(s_pl, cboff, croff, TA, TB, TC); break;
                default: ex = terms_il<2>(s_pl, cboff, croff, TA, TB, TC); break;
            }
            const uint4 Y0q = *reinterpret_cast<const uint4*>(s_pl + yoff);
            row_rgb_il(Y0q, TA, TB, TC, w0);
            uint4 Y1q = make_uint4(0, 0, 0, 0);
            if (pair) {
                Y1q = *reinterpret_cast<const uint4*>(s_pl + yoff + ppitch[0]);
                row_rgb_il(Y1q, TA, TB, TC, w1);  // (shares the term words: vertically subsampled chroma)
            }
            if (__any(ex != 0u)) {  // uniform over the lanes in this step
                switch (cmode) {
                    case 0: fix_g_exact<0>(Y0q, s_pl, cboff, croff, ex, w0); break;
                    case 1: fix_g_exact<1>(Y0q, s_pl, cboff, croff, ex, w0); break;
                    default: fix_g_exact<2>(Y0q, s_pl, cboff, croff, ex, w0); break;
                }
                if (pair) {
                    switch (cmode) {
                        case 0: fix_g_exact<0>(Y1q, s_pl, cboff, croff, ex, w1); break;
                        case 1: fix_g_exact<1>(Y1q, s_pl, cboff, croff, ex, w1); break;
                        default: fix_g_exact<2>(Y1q, s_pl, cboff, croff, ex, w1); break;
                    }
                }
            }
        } else {  // grayscale, or chroma planes with different horizontal factors: per pixel
            int Y0[8];
            load_plane<0>(s_pl, yoff, Y0);
            uint32_t rgb[8][3];
            if (cmode == 3u) {
                colour8<3>(Y0, s_pl, cboff, croff, rgb);
            } else {
                int Cb[8], Cr[8];
                load8_samples(s_pl, cboff, shx1, Cb);
                load8_samples(s_pl, croff, shx2, Cr);
#pragma unroll
                for (int j = 0; j < 8; j++)
                    colour_px(Y0[j], Cb[j], Cr[j], chroma_terms(Cb[j], Cr[j]), rgb[j][0], rgb[j][1], rgb[j][2]);
            }
            pack24(rgb, w0);
        }
        {
            uint8_t* const p0 = rgb_at(out, y, W3, x);
            store24(p0, w0, min(8u, W - x));
            if (pair && y + 1 < H) store24(p0 + W3, w1, min(8u, W - x));
        }
    }
    if (halves && !pair && lane < 2u * nrem) {  // 4:4:4
        const uint32_t g = nfull * kIdctThreads + (lane >> 1);
        const uint32_t py = div_small(g, magic16(gpr)), hc = g - py * gpr;
        const uint32_t gx = (hc << 3) + ((lane & 1u) << 2);
        const uint32_t y = y_tile + py, x = x_tile + gx;
        if (y < H && x < W) {
            uint32_t w0[3];
            colour4x1(s_pl, pbase[0] + py * ppitch[0] + gx, pbase[1] + py * ppitch[1] + gx, pbase[2] + py * ppitch[2] + gx, w0);
            store12(rgb_at(out, y, W3, x), w0, min(4u, W - x));
        }
    } else if (halves && lane < 2u * nrem) {
        const uint32_t g = nfull * kIdctThreads + (lane >> 1);
        const uint32_t hy = div_small(g, magic16(gpr)), hc = g - hy * gpr;
        const uint32_t py = hy * 2u, gx = (hc << 3) + ((lane & 1u) << 2);
        const uint32_t y = y_tile + py, x = x_tile + gx;
        if (y < H && x < W) {
            uint32_t w0[3], w1[3];
            colour4x2(s_pl, pbase[0] + py * ppitch[0] + gx, ppitch[0], pbase[1] + (py >> 1) * ppitch[1] + (gx >> 1),
                      pbase[2] + (py >> 1) * ppitch[2] + (gx >> 1), w0, w1);
            uint8_t* const p0 = rgb_at(out, y, W3, x);
            store12(p0, w0, min(4u, W - x));
            if (y + 1 < H) store12(p0 + W3, w1, min(4u, W - x));
        }
    }
    return true;
}

typedef __attribute__((address_space(4))) const DcPred const_dcpred;
__device__ __forceinline__ DcPred load_dcpred(const BatchDev& b, const ImgDesc& im, uint32_t tile) {
    const_dcpred* p = (const_dcpred*)(size_t)(b.tile_dc + im.tile_base + tile);  // uniform: a scalar load
    return DcPred{p->p0, p->p1, p->p2, p->flag};
}

#ifndef JD_IDCT_LB
#define JD_IDCT_LB 5  // 96 VGPRs: 5 waves per SIMD (LDS allows 20 per CU)
#endif
#ifndef JD_STAMP
#define JD_STAMP 0  // diagnostic builds: per-tile s_memtime stamps at the phase boundaries (BatchDev::stamps)
#endif
#define JD_STAMP_AT(k)                                                                                     \
    do {                                                                                                   \
        if (JD_STAMP && b.stamps && lane == 0) b.stamps[size_t(im.tile_base + tile) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

// One wave per tile; grid: tiles x the batch's images of sampling layout M (b.mode_imgs).  (Two
// tiles per wave, the second's BlockInfo loaded up front, took 3.7 instead of 2.9 ms: DESIGN.md §8.)
// JD_IDCT_PRIO (experiment builds): a wave issues its descriptor, BlockInfo and entry loads at
// raised priority, then drops to 0 for the DC prediction, IDCT and colour, so that a newly started
// wave's loads go out ahead of the older waves' arithmetic.
#ifndef JD_IDCT_PRIO
#define JD_IDCT_PRIO 0
#endif
#ifndef JD_IDCT_PRIO_LATE
#define JD_IDCT_PRIO_LATE 0  // (experiment builds) the reverse: priority raised once the loads are out
#endif
template <int M>
__global__ __launch_bounds__(kIdctThreads, JD_IDCT_LB) void k_idct_color(BatchDev b) {
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[kIdctBufWords];
    __shared__ __attribute__((aligned(16))) int s_qz[kQzWords];
    if (JD_IDCT_PRIO) __builtin_amdgcn_s_setprio(JD_IDCT_PRIO);
    const uint32_t lane = threadIdx.x, img = b.mode_imgs[b.mode_off[M] + blockIdx.y], tile = blockIdx.x;
    const ImgDesc& im = b.imgs[img];
    if (tile >= im.tiles_x * im.tiles_y) return;
    const TileGeo G = tile_geo<M>(im, tile);
    const TileLaneGeo L = tile_lane_geo<M>(im, G, lane);
    const BlockInfo bi = load_block_info<M>(b, im, G, L);
    const DcPred dcin = load_dcpred(b, im, tile);
    stage_quant(b, im, s_qz, lane);
    JD_STAMP_AT(0);
    zero_staging(s_buf, lane);
    const EntryRange R = entry_range(b, im, bi, L.have);
    uint4 E[kPreQuads];
    load_entry_quads(R, E);
    if (JD_IDCT_PRIO) __builtin_amdgcn_s_setprio(0);
    if (JD_IDCT_PRIO_LATE) __builtin_amdgcn_s_setprio(JD_IDCT_PRIO_LATE);
    const int dc_pred = tile_dc_predict(G, L, bi, dcin, lane);
    JD_STAMP_AT(1);
    __syncthreads();
    scatter_entries(s_buf, staging_base(lane), R, E);
    __syncthreads();
    if (JD_ABL_PHASE == 2) return;  // diagnostic builds: no IDCT and colour (the staging rows are kept)
    JD_STAMP_AT(2);
    idct_colour_tile<false, M>(b, im, img, tile, G, L, dc_pred, R.esc, s_buf, s_qz, [&] { JD_STAMP_AT(3); });
    JD_STAMP_AT(4);
}

// The tiles k_idct_color left (grid-stride over the list; empty in practice).
__global__ __launch_bounds__(kIdctThreads) void k_idct_color_exact(BatchDev b) {
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[kIdctBufWords];
    __shared__ __attribute__((aligned(16))) int s_qz[kQzWords];
    const uint32_t lane = threadIdx.x;
    const uint32_t n = uint32_t(min(b.counters[1], (unsigned long long)b.total_tiles));
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const TileRef tr = b.slow_tiles[i];
        const ImgDesc& im = b.imgs[tr.img];
        if (tr.tile >= im.tiles_x * im.tiles_y) continue;
        const TileGeo G = tile_geo(im, tr.tile);
        const TileLaneGeo L = tile_lane_geo(im, G, lane);
        __syncthreads();
        stage_quant(b, im, s_qz, lane);
        zero_staging(s_buf, lane);
        const BlockInfo bi = load_block_info(b, im, G, L);
        const int dc_pred = tile_dc_predict(G, L, bi, b.tile_dc[im.tile_base + tr.tile], lane);
        __syncthreads();
        const EntryRange R = entry_range(b, im, bi, L.have);
        uint4 E[kPreQuads];
        load_entry_quads(R, E);
        scatter_entries(s_buf, staging_base(lane), R, E);
        __syncthreads();
        idct_colour_tile<true, kModeGen>(b, im, tr.img, tr.tile, G, L, dc_pred, R.esc, s_buf, s_qz, [] {});
    }
}

// ------------------------------------------------------------------------------------------
// Fancy upsampling + colour (JD_FLAG_FANCY_UPSAMPLING), lane = 8 consecutive pixels of a row.
// The triangular filters of libjpeg (jdsample.c h2v1 / h2v2 / h1v2 fancy upsampling) on the
// reference's un-shifted samples, edges replicated at the component's real sample extent; the
// same definition as oracle/jdoracle.c fancy_sample().  Other ratios replicate.
// ------------------------------------------------------------------------------------------
// Fancy upsampling (libjpeg's h2v1 / h2v2 / h1v2 triangular filters, restated in
// oracle/jdoracle.c fancy_sample; other ratios replicate) + colour, from the int16 component
// planes k_idct_color wrote to HBM.  One 256-thread workgroup per 128 x 16-pixel band (four
// bands stacked per workgroup): every component's window of plane samples (the band's rows and
// columns plus the filter's one-sample halo, 16-byte aligned) is staged in LDS with coalesced
// 16-byte loads, then thread t colours 8 consecutive pixels of row t / 16 and stores their 24 bytes.
constexpr uint32_t kFancyThreads = 256;  // kFancyW x kFancyH bands (jd_internal.hpp)
constexpr uint32_t kFancyRows = kFancyH + 2, kFancyCols = kFancyW + 16;  // window bound per component
static_assert((kFancyW / 8) * kFancyH == kFancyThreads, "one 8-pixel group per thread");

struct FancyWin {
    const int16_t* s;       // LDS window: rows r0.., pitch kFancyCols samples, first column c0, ncols used
    int r0, c0, ncols;
    uint32_t rx, ry, cw, ch;
    __device__ __forceinline__ const int16_t* row(int y) const { return s + __mul24(y - r0, int(kFancyCols)); }
    __device__ __forceinline__ int at(int x, int y) const { return row(y)[x - c0]; }
};

__device__ __forceinline__ int fancy_win(const FancyWin& P, uint32_t x, uint32_t y) {
    if (P.rx == 2 && P.ry == 1) {  // h2v1_fancy_upsample
        const int i = int(x >> 1);
        if (x & 1) return uint32_t(i) + 1 >= P.cw ? P.at(i, y) : (3 * P.at(i, y) + P.at(i + 1, y) + 2) >> 2;
        return i == 0 ? P.at(0, y) : (3 * P.at(i, y) + P.at(i - 1, y) + 1) >> 2;
    }
    if (P.ry == 2 && (P.rx == 1 || P.rx == 2)) {  // h1v2 / h2v2_fancy_upsample
        const int r = int(y >> 1);
        const int far = (y & 1) ? min(r + 1, int(P.ch) - 1) : (r == 0 ? 0 : r - 1);
        if (P.rx == 1) return (3 * P.at(x, r) + P.at(x, far) + ((y & 1) ? 2 : 1)) >> 2;
        const int i = int(x >> 1);
        const int cs = 3 * P.at(i, r) + P.at(i, far);
        if (x & 1) {
            if (uint32_t(i) + 1 >= P.cw) return (4 * cs + 7) >> 4;
            return (3 * cs + 3 * P.at(i + 1, r) + P.at(i + 1, far) + 7) >> 4;
        }
        if (i == 0) return (4 * cs + 8) >> 4;
        return (3 * cs + 3 * P.at(i - 1, r) + P.at(i - 1, far) + 8) >> 4;
    }
    return P.at(int(x / P.rx), int(y / P.ry));  // replicate
}

// The 8 chroma values under output pixels gx .. gx + 7 (gx a multiple of 8) of row y, for the
// window's filter mode (both chroma planes share it): MODE 0 none (1x1), 1 h2v2, 2 h2v1, 3 h1v2.
// Vector LDS reads: a 2x-horizontal filter needs samples i0 - 1 .. i0 + 4 of its rows (i0 = gx / 2,
// a multiple of 4: one 8-byte read plus the two neighbours), a 1x one the 8 samples (16 bytes).
template <int MODE>
__device__ __forceinline__ void fancy_row8(const FancyWin& P, uint32_t gx, uint32_t y, int (&v)[8]) {
    auto s16 = [](uint32_t w, int hi) { return hi ? int32_t(w) >> 16 : int(int16_t(w & 0xFFFFu)); };
    if (MODE == 0 || MODE == 3) {
        const int rr = MODE == 0 ? int(y) : int(y >> 1);
        const uint4 q = *reinterpret_cast<const uint4*>(P.row(rr) + (int(gx) - P.c0));
        const uint32_t a[4] = {q.x, q.y, q.z, q.w};
        if (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = s16(a[j >> 1], j & 1);
            return;
        }
        const int far = (y & 1) ? min(rr + 1, int(P.ch) - 1) : max(rr - 1, 0);
        const uint4 f = *reinterpret_cast<const uint4*>(P.row(far) + (int(gx) - P.c0));
        const uint32_t b[4] = {f.x, f.y, f.z, f.w};
        const int rnd = (y & 1) ? 2 : 1;
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = (3 * s16(a[j >> 1], j & 1) + s16(b[j >> 1], j & 1) + rnd) >> 2;
        return;
    }
    const int i0 = int(gx >> 1);
    const int lo = max(i0 - 1, P.c0) - P.c0, hi = min(i0 + 4 - P.c0, P.ncols - 1);
    int C[6];  // columns i0 - 1 .. i0 + 4: 3 S(i, r) + S(i, far) (h2v2) or S(i, y) (h2v1)
    {
        const int rr = MODE == 1 ? int(y >> 1) : int(y);
        const int16_t* row = P.row(rr);
        const uint2 q = *reinterpret_cast<const uint2*>(row + (i0 - P.c0));
        C[0] = row[lo];
        C[1] = s16(q.x, 0);
        C[2] = s16(q.x, 1);
        C[3] = s16(q.y, 0);
        C[4] = s16(q.y, 1);
        C[5] = row[hi];
        if (MODE == 1) {
            const int far = (y & 1) ? min(rr + 1, int(P.ch) - 1) : max(rr - 1, 0);
            const int16_t* frow = P.row(far);
            const uint2 f = *reinterpret_cast<const uint2*>(frow + (i0 - P.c0));
            C[0] = mad24(C[0], 3, frow[lo]);
            C[1] = mad24(C[1], 3, s16(f.x, 0));
            C[2] = mad24(C[2], 3, s16(f.x, 1));
            C[3] = mad24(C[3], 3, s16(f.y, 0));
            C[4] = mad24(C[4], 3, s16(f.y, 1));
            C[5] = mad24(C[5], 3, frow[hi]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {  // pixels 2k (even: sample i0 + k and its left) and 2k + 1 (odd: its right)
        const int i = i0 + k, c = C[k + 1];
        const bool first = i == 0, last = uint32_t(i) + 1 >= P.cw;
        // the image's edge column is its own neighbour (libjpeg's edge cases: (4c + 8) >> 4 and
        // (4c + 7) >> 4 for h2v2; c itself for h2v1, where (3c + c + 1) >> 2 = c as well)
        const int left = first ? c : C[k], right = last ? c : C[k + 2];
        if (MODE == 1) {
            v[2 * k] = mad24(c, 3, left + 8) >> 4;
            v[2 * k + 1] = mad24(c, 3, right + 7) >> 4;
        } else {
            v[2 * k] = mad24(c, 3, left + 1) >> 2;
            v[2 * k + 1] = mad24(c, 3, right + 2) >> 2;
        }
    }
}

// 8 pixels: Y (1x1 window), filtered chroma, then the packed integer colour of k_idct_color (terms
// per pixel here) with the same double-precision G patch.
template <int MODE>
__device__ __forceinline__ void fancy_colour8(const FancyWin (&P)[3], uint32_t gx, uint32_t y, uint32_t (&w)[6]) {
    const uint4 Yq = *reinterpret_cast<const uint4*>(P[0].row(int(y)) + (int(gx) - P[0].c0));
    int cb[8], cr[8];
    fancy_row8<MODE>(P[1], gx, y, cb);
    fancy_row8<MODE>(P[2], gx, y, cr);
    uint32_t TR[4], TG[4], TB[4], ex = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const ChromaTerms t0 = chroma_terms(cb[2 * u], cr[2 * u]), t1 = chroma_terms(cb[2 * u + 1], cr[2 * u + 1]);
        ex |= (t0.exact ? 1u : 0u) << (2 * u);
        ex |= (t1.exact ? 1u : 0u) << (2 * u + 1);
        TR[u] = pair16(t0.r, t1.r);
        TG[u] = pair16(t0.g, t1.g);
        TB[u] = pair16(t0.b, t1.b);
    }
    row_rgb_packed<false>(Yq, TR, TG, TB, w);
    if (__any(ex != 0u)) {
        const uint32_t Y[4] = {Yq.x, Yq.y, Yq.z, Yq.w};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if ((ex >> j) & 1u) {
                const int yv = (j & 1) ? int32_t(Y[j >> 1]) >> 16 : int(int16_t(Y[j >> 1] & 0xFFFFu));
                const int g = color_g_exact(yv, cb[j], cr[j]);
                const int byte = 3 * j + 1;
                w[byte >> 2] = (w[byte >> 2] & ~(0xFFu << (8 * (byte & 3)))) | (uint32_t(g) << (8 * (byte & 3)));
            }
        }
    }
}

// Bands per workgroup (kFancyBands, stacked vertically): the next band's window is fetched into
// registers while the current band is coloured, so a workgroup waits on HBM latency once, not per band.
#ifndef JD_FANCY_LB
#define JD_FANCY_LB 1  // minimum waves per SIMD asked of the compiler (register budget)
#endif
constexpr int kFancyQuadsPerThread = 2;  // window quads per thread and component: 18 x 18 <= 512
static_assert((kFancyRows * (kFancyCols / 8) + kFancyThreads - 1) / kFancyThreads <= kFancyQuadsPerThread,
              "window quads per thread");

// One instance per sampling layout (the images of b.mode_imgs, as k_idct_color<M>): 4:2:0 is the
// h2v2 filter, 4:2:2 h2v1, 4:4:4 none (all vectorised, fancy_colour8, with the layout's ratios as
// compile-time constants); every other layout (h1v2, grayscale, other ratios) takes the per-pixel
// fancy_win path with ratios from the image descriptor.
template <int M>
__global__ __launch_bounds__(kFancyThreads, JD_FANCY_LB) void k_colour_fancy(BatchDev b) {
    __shared__ __attribute__((aligned(16))) int16_t s_win[3][kFancyRows * kFancyCols];
    constexpr bool kFixed = M != kModeGen;
    constexpr int kFilt = M == kMode420 ? 1 : M == kMode422 ? 2 : 0;
    constexpr uint32_t kLgRx = (M == kMode420 || M == kMode422) ? 1u : 0u, kLgRy = M == kMode420 ? 1u : 0u;
    const ImgDesc& im = b.imgs[b.mode_imgs[b.mode_off[M] + blockIdx.z]];
    const uint32_t W = im.width, H = im.height;
    const uint32_t x0 = blockIdx.x * kFancyW, yb = blockIdx.y * (kFancyH * kFancyBands);
    if (x0 >= W || yb >= H) return;  // workgroup-uniform (the grid covers the layout's largest image)
    const uint32_t t = threadIdx.x, nc = kFixed ? 3u : im.ncomp;
    FancyWin P[3];
    const int16_t* src[3];
    uint32_t pitch[3], prow[3], qpr[3], qmagic[3];
    {
        size_t off = 0;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const uint32_t cc = uint32_t(c) < nc ? uint32_t(c) : 0u;
            FancyWin& F = P[c];
            if (kFixed) {  // Y 1x1, chroma 2^kLgRx x 2^kLgRy
                const uint32_t lx = c ? kLgRx : 0u, ly = c ? kLgRy : 0u;
                F.rx = 1u << lx;
                F.ry = 1u << ly;
                F.cw = (W + F.rx - 1) >> lx;
                F.ch = (H + F.ry - 1) >> ly;
                pitch[c] = im.mcux * ((c ? 1u : 1u << kLgRx) * 8);
                prow[c] = im.mcuy * ((c ? 1u : 1u << kLgRy) * 8);
            } else {
                F.rx = im.hmax / im.h[cc];
                F.ry = im.vmax / im.v[cc];
                F.cw = (W * im.h[cc] + im.hmax - 1) / im.hmax;
                F.ch = (H * im.v[cc] + im.vmax - 1) / im.vmax;
                pitch[c] = im.mcux * im.h[cc] * 8;
                prow[c] = im.mcuy * im.v[cc] * 8;
            }
            const uint32_t xs = kFixed ? (x0 >> (c ? kLgRx : 0u)) : x0 / F.rx;
            const uint32_t xe = kFixed ? ((x0 + kFancyW - 1) >> (c ? kLgRx : 0u)) : (x0 + kFancyW - 1) / F.rx;
            const int c0 = max(0, (int(xs) - 1) & ~7);
            const int c1 = min(int(pitch[c]), int((xe + 9) & ~7u));
            F.s = s_win[c];
            F.c0 = c0;
            F.ncols = c1 - c0;
            qpr[c] = uint32_t(F.ncols) >> 3;
            qmagic[c] = (65536u + qpr[c] - 1u) / qpr[c];
            src[c] = reinterpret_cast<const int16_t*>(im.planes) + off + c0;
            if (uint32_t(c) < nc) off += size_t(pitch[c]) * prow[c];
        }
    }
    // window rows of a band: the band's sample rows plus the vertical filters' one-row halo
    auto rows_of = [&](int c, uint32_t y0, int& r0, int& r1) {
        const int vh = P[c].ry == 2 ? 1 : 0;
        const uint32_t ys = kFixed ? (y0 >> (c ? kLgRy : 0u)) : y0 / P[c].ry;
        const uint32_t ye = kFixed ? ((y0 + kFancyH - 1) >> (c ? kLgRy : 0u)) : (y0 + kFancyH - 1) / P[c].ry;
        r0 = max(0, int(ys) - vh);
        r1 = min(int(prow[c]) - 1, int(ye) + vh);
    };
    u32x4 pf[3][kFancyQuadsPerThread];
    uint32_t pdst[3][kFancyQuadsPerThread];  // LDS word offset of each fetched quad (~0u: none)
    auto fetch = [&](uint32_t y0) {  // this thread's quads of every component's window -> registers
#pragma unroll
        for (int c = 0; c < 3; c++) {
            int r0, r1;
            rows_of(c, y0, r0, r1);
            const uint32_t nq = uint32_t(c) < nc ? qpr[c] * uint32_t(r1 - r0 + 1) : 0u;
#pragma unroll
            for (int k = 0; k < kFancyQuadsPerThread; k++) {
                const uint32_t q = t + uint32_t(k) * kFancyThreads;
                pdst[c][k] = ~0u;
                if (q < nq) {
                    const uint32_t rr = __umul24(q, qmagic[c]) >> 16, cq = q - rr * qpr[c];
                    pf[c][k] = *gptr(reinterpret_cast<const u32x4*>(src[c] + size_t(uint32_t(r0) + rr) * pitch[c] + 8 * cq));
                    pdst[c][k] = __umul24(rr, kFancyCols) + 8 * cq;
                }
            }
        }
    };
    auto put = [&]() {  // registers -> the LDS windows
#pragma unroll
        for (int c = 0; c < 3; c++)
#pragma unroll
            for (int k = 0; k < kFancyQuadsPerThread; k++)
                if (pdst[c][k] != ~0u) *reinterpret_cast<u32x4*>(s_win[c] + pdst[c][k]) = pf[c][k];
    };
    fetch(yb);
    put();
    __syncthreads();
#pragma unroll 1
    for (uint32_t band = 0; band < kFancyBands; band++) {
        const uint32_t y0 = yb + band * kFancyH;
        const bool next = band + 1 < kFancyBands && y0 + kFancyH < H;  // workgroup-uniform
        if (next) fetch(y0 + kFancyH);  // in flight while this band is coloured
#pragma unroll
        for (int c = 0; c < 3; c++) {
            int r1;
            rows_of(c, y0, P[c].r0, r1);
        }
        const uint32_t y = y0 + (t >> 4), gx = x0 + ((t & 15u) << 3);
        if (y < H && gx < W) {
            uint32_t w[6];
            if (kFixed) {
                fancy_colour8<kFilt>(P, gx, y, w);
            } else {  // grayscale, h1v2, a subsampled Y, or chroma planes with different ratios: per pixel
                uint32_t rgb[8][3];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t x = min(gx + uint32_t(j), W - 1);
                    const int yv = fancy_win(P[0], x, y);
                    if (nc == 1) {
                        rgb[j][0] = rgb[j][1] = rgb[j][2] = clamp_u8(yv + 128);
                    } else {
                        const int cb = fancy_win(P[1], x, y), cr = fancy_win(P[2], x, y);
                        colour_px(yv, cb, cr, chroma_terms(cb, cr), rgb[j][0], rgb[j][1], rgb[j][2]);
                    }
                }
                pack24(rgb, w);
            }
            store24(rgb_at(reinterpret_cast<uint8_t*>(im.rgb), y, 3u * W, gx), w, min(8u, W - gx));
        }
        if (!next) break;
        __syncthreads();  // every read of this band's windows is done
        put();
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Known-answer hooks
// ------------------------------------------------------------------------------------------
// exact_only = 0: the decode path's choice per block (the int16 fast form when every input fits
// int16, else the exact form); 1: the exact form whatever the inputs.
__global__ void k_test_idct(const int32_t* in_zz, int32_t* out, int n, int exact_only) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int blk[64];
    bool in_range = !exact_only;
    uint32_t dw[32];
#pragma unroll
    for (int z = 0; z < 64; z++) {
        const int v = in_zz[size_t(i) * 64 + z];
        blk[kNatOfZz[z]] = v;
        in_range = in_range && uint32_t(v + 32768) <= 65535u;
        if (z & 1) dw[z >> 1] = pk16(blk[kNatOfZz[z - 1]], v);
    }
    if (in_range) {
        uint32_t pk[32];
        idct_block_dot2(dw, pk);
#pragma unroll
        for (int q = 0; q < 32; q++) {
            blk[2 * q] = int(int16_t(pk[q] & 0xFFFFu));
            blk[2 * q + 1] = int32_t(pk[q]) >> 16;
        }
    } else {
        idct_block_exact(blk);
    }
#pragma unroll
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

// HBM copy peak (bench.py's in-run roofline reference, MI355X_MICROARCH.md "float4 copy"): each
// lane moves four 16-byte vectors, all four loads issued before the stores, consecutive lanes on
// consecutive vectors (every wave instruction covers 1 KiB).
constexpr int kCopyThreads = 256, kCopyPer = 4;
typedef uint32_t copy_v4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(kCopyThreads) void k_copy16(const copy_v4* __restrict__ src, copy_v4* __restrict__ dst,
                                                         size_t n16) {
    const size_t base = size_t(blockIdx.x) * (kCopyThreads * kCopyPer) + threadIdx.x;
    copy_v4 v[kCopyPer];
    if (base + (kCopyPer - 1) * kCopyThreads < n16) {
#pragma unroll
        for (int k = 0; k < kCopyPer; k++) v[k] = src[base + k * kCopyThreads];
#pragma unroll
        for (int k = 0; k < kCopyPer; k++) dst[base + k * kCopyThreads] = v[k];
        return;
    }
    for (int k = 0; k < kCopyPer; k++)
        if (base + k * kCopyThreads < n16) dst[base + k * kCopyThreads] = src[base + k * kCopyThreads];
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
size_t huffman_lds_bytes(uint32_t max_slots) { return piece_lds_bytes(max_slots, kPieceThreads); }

uint32_t piece_lanes_resident(size_t lds) {
    // cached per device (a process may drive several GPUs, one context each)
    constexpr int kMaxDev = 64;
    static std::mutex m;
    static size_t cached_lds[kMaxDev] = {};
    static uint32_t cached[kMaxDev] = {};
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    std::lock_guard<std::mutex> l(m);
    if (dev < kMaxDev && lds == cached_lds[dev] && cached[dev]) return cached[dev];
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_piece<kPieceThreads>), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_piece<kPieceThreads>, kPieceThreads, lds) != hipSuccess || nb <= 0) return 0;
    const uint32_t lanes = uint32_t(nb) * uint32_t(cus) * uint32_t(kPieceThreads);
    if (dev < kMaxDev) {
        cached_lds[dev] = lds;
        cached[dev] = lanes;
    }
    return lanes;
}

// Dynamic LDS above 64 KiB (large piece workgroups) has to be allowed per kernel once.
static hipError_t allow_lds(size_t lds) {
    constexpr int kMaxDev = 64;  // per device, as piece_lanes_resident
    static std::mutex m;
    static size_t allowed[kMaxDev] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
    std::lock_guard<std::mutex> l(m);
    if (lds <= std::max<size_t>(65536, allowed[dev])) return hipSuccess;
    for (const void* f : {reinterpret_cast<const void*>(&k_piece<kPieceThreads>), reinterpret_cast<const void*>(&k_piece<64>)}) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    allowed[dev] = lds;
    return hipSuccess;
}

// The same for k_chain_big's 8-wave workgroups (their lanes' rows and rings beside the tables).
static hipError_t allow_lds_big(size_t lds) {
    constexpr int kMaxDev = 64;
    static std::mutex m;
    static size_t allowed[kMaxDev] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
    std::lock_guard<std::mutex> l(m);
    if (lds <= std::max<size_t>(65536, allowed[dev])) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_chain_big),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (e == hipSuccess) allowed[dev] = lds;
    return e;
}

hipError_t launch_kernel(int k, const BatchDev& b, hipStream_t s) {
    if (!b.nimg) return hipSuccess;
    const size_t lds = piece_lds_bytes(b.max_slots, kPieceThreads);
    if (k == 4 || k == 5 || k == 6) {
        const hipError_t e = allow_lds(lds);
        if (e != hipSuccess) return e;
    }
    switch (k) {
        case 0:
            if (b.max_chunks) {
                hipLaunchKernelGGL(k_scan, dim3(b.max_chunks, b.nimg), dim3(kScanThreads), 0, s, b);  // (fills sub_seg)
            } else if (b.nsub) {  // no entropy-coded bytes at all: no k_scan to fill the piece slots
                const hipError_t e = hipMemsetAsync(b.sub_seg, 0xFF, size_t(b.nsub) * 4, s);
                if (e != hipSuccess) return e;
            }
            break;
        case 1: hipLaunchKernelGGL(k_index, dim3(b.nimg), dim3(64), 0, s, b); break;
        case 2:
            if (b.max_chunks) hipLaunchKernelGGL(k_compact, dim3(b.max_chunks, b.nimg), dim3(kScanThreads), 0, s, b);
            break;
        case 3: {
            if (!b.nsub || b.small_fold) break;
            if (b.piece_plan) hipLaunchKernelGGL(k_pieceplan, dim3(1), dim3(kPlanThreads), 0, s, b);
            hipLaunchKernelGGL(k_subplan, dim3(b.nimg), dim3(64), 0, s, b);
            break;
        }
        case 4:
            if (b.nsub >= kSmallPieceLanes)
                hipLaunchKernelGGL(k_piece<kPieceThreads>, dim3(b.nsub / kPieceThreads), dim3(kPieceThreads), lds, s, b);
            else if (b.nsub)
                hipLaunchKernelGGL(k_piece<64>, dim3(b.nsub / 64), dim3(64), piece_lds_bytes(b.max_slots, 64), s, b);
            break;
        case 5:
            if (b.skip_redo) break;  // (diagnostics)
            if (b.nsub && (b.big_chain || b.small_fold))
                hipLaunchKernelGGL(k_redo<true>, dim3(b.nsub / kRedoThreads), dim3(kRedoThreads),
                                   size_t(b.max_slots) * sizeof(HuffLut) + kRedoLds, s, b);
            else if (b.nsub)
                hipLaunchKernelGGL(k_redo<false>, dim3(b.nsub / kRedoThreads), dim3(kRedoThreads), kRewalkLds, s, b);
            break;
        case 6:
            if (!b.nseg) break;
            hipLaunchKernelGGL(k_chain, dim3((b.nseg + 3) / 4), dim3(256), 0, s, b);
            if (b.nchain && b.big_chain) {
                const size_t lds_big = size_t(b.max_slots) * sizeof(HuffLut) + kBigLds;
                const hipError_t e = allow_lds_big(lds_big);
                if (e != hipSuccess) return e;
                hipLaunchKernelGGL(k_chain_big, dim3(b.nchain), dim3(kBigThreads), lds_big, s, b);
            }
            else if (b.nchain)
                hipLaunchKernelGGL(k_chain_fix, dim3(b.nchain / kRedoThreads), dim3(kRedoThreads), kRewalkLds, s, b);
            break;
        case 7:
            if (b.nsub) hipLaunchKernelGGL(k_gather, dim3((b.nsub + 255) / 256), dim3(256), 0, s, b);  // 64 pieces per wave
            break;
        case 8:
            if (!b.max_tiles) break;
            hipLaunchKernelGGL(k_dc_sum, dim3((b.max_tiles + 4 * kDcTilesPerWave - 1) / (4 * kDcTilesPerWave), b.nimg),
                               dim3(256), 0, s, b);
            hipLaunchKernelGGL(k_dc_scan, dim3(b.nimg), dim3(64), 0, s, b);
            break;
        case 9:
            if (!b.max_tiles) break;
            // one launch per sampling layout present in the batch (k_idct_color<M> is specialised)
            if (b.mode_cnt[kModeGen])
                hipLaunchKernelGGL(k_idct_color<kModeGen>, dim3(b.mode_max_tiles[kModeGen], b.mode_cnt[kModeGen]), dim3(kIdctThreads), 0, s, b);
            if (b.mode_cnt[kMode420])
                hipLaunchKernelGGL(k_idct_color<kMode420>, dim3(b.mode_max_tiles[kMode420], b.mode_cnt[kMode420]), dim3(kIdctThreads), 0, s, b);
            if (b.mode_cnt[kMode422])
                hipLaunchKernelGGL(k_idct_color<kMode422>, dim3(b.mode_max_tiles[kMode422], b.mode_cnt[kMode422]), dim3(kIdctThreads), 0, s, b);
            if (b.mode_cnt[kMode444])
                hipLaunchKernelGGL(k_idct_color<kMode444>, dim3(b.mode_max_tiles[kMode444], b.mode_cnt[kMode444]), dim3(kIdctThreads), 0, s, b);
            hipLaunchKernelGGL(k_idct_color_exact, dim3(1024), dim3(kIdctThreads), 0, s, b);
            break;
        case 10:
            if (b.fancy && b.max_fancy_wgs) {  // one launch per sampling layout present in the batch
                const dim3 g(b.max_fancy_wgs & 0xFFFFu, b.max_fancy_wgs >> 16, 1);
                if (b.mode_cnt[kModeGen])
                    hipLaunchKernelGGL(k_colour_fancy<kModeGen>, dim3(g.x, g.y, b.mode_cnt[kModeGen]), dim3(kFancyThreads), 0, s, b);
                if (b.mode_cnt[kMode420])
                    hipLaunchKernelGGL(k_colour_fancy<kMode420>, dim3(g.x, g.y, b.mode_cnt[kMode420]), dim3(kFancyThreads), 0, s, b);
                if (b.mode_cnt[kMode422])
                    hipLaunchKernelGGL(k_colour_fancy<kMode422>, dim3(g.x, g.y, b.mode_cnt[kMode422]), dim3(kFancyThreads), 0, s, b);
                if (b.mode_cnt[kMode444])
                    hipLaunchKernelGGL(k_colour_fancy<kMode444>, dim3(g.x, g.y, b.mode_cnt[kMode444]), dim3(kFancyThreads), 0, s, b);
            }
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_test_idct(const int32_t* in_zz, int32_t* out, int n, int exact_only, hipStream_t s) {
    hipLaunchKernelGGL(k_test_idct, dim3((n + 63) / 64), dim3(64), 0, s, in_zz, out, n, exact_only);
    return hipGetLastError();
}

hipError_t launch_test_color(const int32_t* ycc, uint8_t* rgb, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_test_color, dim3((n + 255) / 256), dim3(256), 0, s, ycc, rgb, n);
    return hipGetLastError();
}

hipError_t launch_copy16(const void* src, void* dst, size_t bytes, hipStream_t s) {
    const size_t n16 = bytes / 16;
    const size_t per = size_t(kCopyThreads) * kCopyPer;
    hipLaunchKernelGGL(k_copy16, dim3(uint32_t((n16 + per - 1) / per)), dim3(kCopyThreads), 0, s,
                       static_cast<const copy_v4*>(src), static_cast<copy_v4*>(dst), n16);
    return hipGetLastError();
}

}  // namespace jd
