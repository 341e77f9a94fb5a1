// jd_internal.hpp — data layout shared by the host runtime and the gfx950 kernels.
//
// Everything a kernel reads is described here; see DESIGN.md §4 for the HBM layout of a batch.
#pragma once

#include <stdint.h>

#include "jd.h"

namespace jd {

// Fast Huffman lookup width: one LDS read resolves every code of <= kLutBits bits (and, when the
// magnitude bits fit too, the coefficient value).  Longer codes take the canonical slow path.
#ifndef JD_LUT_BITS
#define JD_LUT_BITS 10
#endif
constexpr int kLutBits = JD_LUT_BITS;
constexpr int kLutSize = 1 << kLutBits;

#if defined(__HIPCC__)
#define JD_HD __host__ __device__
#else
#define JD_HD
#endif

// Symbol entry of the rare path (32 bits; jd_kernels.hip huff_slow / the piece walks' rare branch):
//     bits 0..4   L    bits the symbol consumes, code + magnitude (0: code longer than kLutBits)
//     bit  5      sz16 DC size 16 (the sz field then 0)
//     bit  6      emit AC coefficient stored (size != 0)
//     bits 8..14  adv  advance of the coefficient index z (the last position decoded, DC = 0):
//                      DC 0, AC run + 1 (ZRL 16), EOB 64.  A block ends when z + adv >= 63, and
//                      a coefficient lands at z + adv unless that is past 63 (parser.cpp:120-131:
//                      its magnitude bits are consumed, the value dropped, the block ends)
//     bit  15     dc   DC symbol
//     bits 16..19 sz   magnitude bits (DC: symbol, AC: symbol & 15; a DC size above 16 is corrupt)
//     bit  7      bad  corrupt code (slow path only)
//   The coefficient is EXTEND(the last sz of the L bits).
constexpr uint32_t kEntEmit = 1u << 6, kEntDc = 1u << 15, kEntBad = 1u << 7, kEntSz16 = 1u << 5;

// Entry of a code of length l for symbol sym; 0 when it cannot be represented: l + sz > 31 (a DC
// size 16 behind a 16-bit code), or a DC size beyond 16 bits.  Baseline DC sizes are <= 11, but
// the reference reads a DC size as it comes (parser.cpp:106-108, 16 bits into a uint16_t) and the
// oracle takes up to 16 (jdoracle.c decode_block): a size-16 difference spans +-65535 (a block
// record's DC field has 17 bits, jd_kernels.hip block_rec).
JD_HD inline uint32_t lut_entry(uint32_t l, uint32_t sym, bool is_dc) {
    const uint32_t sz = is_dc ? sym : (sym & 15u);
    if (sz > 16u || l + sz > 31u || l == 0u) return 0u;
    if (is_dc) return (l + sz) | kEntDc | ((sz & 15u) << 16) | ((sz >> 4) << 5);
    const uint32_t adv = sym == 0u ? 64u : (sym >> 4) + 1u;
    return (l + sz) | (sz ? kEntEmit : 0u) | (adv << 8) | (sz << 16);
}

// Device Huffman table (built on the host from a DHT table, uploaded once, cached by content).
// fast[i] is the 64-bit entry {lo, hi} for the next kLutBits stream bits = i, laid out so that the
// piece walks use its fields as instruction operands (v_bfe_i32 takes its offset from lo[4:0] and
// its width from hi[4:0]):
//   lo  bits 0..4   o1   32 - L1: offset in the 32-bit peek of the first symbol's magnitude
//       bit  5      DC   DC symbol
//       bit  6      E1   the first symbol stores a coefficient (AC, size != 0); bit 6 so that
//                        lo & ~zn & 64 is its emit test (zn < 64)
//       bit  7      E2   the second symbol stores a coefficient (tested against zn << 1)
//       bit  8      P    a second AC symbol follows within the index (pair)
//       bits 9..13  L1   bits of the first symbol, code + magnitude (<= 31)
//       bit  15     R    rare: hi holds the 32-bit entry above << kRareShift (0: a code longer than
//                        kLutBits; the shift keeps hi's adv fields 0, so a rare entry the walk does not
//                        resolve in this iteration leaves the decoder state unchanged);
//                        codes longer than kLutBits, AC magnitudes of 10 bits or more (they need an
//                        escaped slot), DC sizes above 11.  lo = R alone (no flags, no pair)
//       bits 16..31 M1   int16: the coefficient is s - (M1 ^ (s >> 31)) for s = the magnitude bits
//                        sign-extended (v_bfe_i32 of width w1): M1 = 2^sz - 1 when the magnitude
//                        reaches beyond the index, else w1 = 0 and M1 = -value
//   hi  bits 0..4   w1   magnitude bits still to extract (0 when the index resolves the value)
//       bits 5..11  adv1 advance of z by the first symbol (DC 0, AC run + 1, ZRL 16, EOB 64)
//       bits 12..18 adv2 the same for the second symbol
//       bits 19..22 L12  bits of the pair, L1 + the second symbol's code + magnitude (<= kLutBits)
//       bits 23..31 v2   int9: its value (|v2| <= 255: its magnitude has at most 8 bits)
//   Codes longer than kLutBits take the canonical slow path:
//   lim[l]     : left-justified 16-bit limit; a code has length l iff peek16 < lim[l] (and not
//                < lim[l-1]) — the canonical DECODE procedure of JPEG Annex F.2.2.3
//   lim[19]    : 1 for a DC table
//   base[l]    : valptr[l] - mincode[l]; vals[] the symbols in code order
struct alignas(16) HuffLut {
    uint32_t fast[2 * kLutSize];  // {lo, hi} pairs
    uint32_t lim[20];
    int32_t base[20];
    uint8_t vals[256];
};
static_assert(sizeof(HuffLut) % 16 == 0, "HuffLut must stay 16-byte aligned");
constexpr int kLutWords = int(sizeof(HuffLut) / 4);
constexpr uint32_t kLoDc = 1u << 5, kLoE1 = 1u << 6, kLoE2 = 1u << 7, kLoPair = 1u << 8, kLoRare = 1u << 15;
constexpr uint32_t kLoL1Shift = 9;
constexpr uint32_t kRareShift = 12;  // the 20-bit rare entry (lut_entry) sits in hi bits 12..31

// Maximum Huffman tables a table set (one workgroup of the Huffman kernel) stages into LDS.
constexpr int kSlotsPerSet = 6;

// Per table set: which cached LUT each slot holds and which slot each component uses.
struct TableSet {
    int32_t lut[kSlotsPerSet];  // index into the LUT array (-1 = unused)
    uint8_t dc_slot[4];
    uint8_t ac_slot[4];
    int32_t nslots;
    int32_t set_lut0;  // first of this set's nslots LUTs in BatchDev::set_luts (k_redo reads them there)
};

// Per image of a batch (device array, one entry per decodable image).
struct alignas(16) ImgDesc {
    uint64_t jpeg;     // device address of the file bytes
    uint64_t rgb;      // device address of the H*W*3 uint8 output
    uint64_t comp;     // device address of this image's un-stuffed entropy-coded data
    uint32_t len;      // file length in bytes
    uint32_t ecs_off;  // first ECS byte
    uint32_t width, height;
    uint32_t mcux, mcuy;
    uint32_t ncomp, hmax, vmax, bpm;  // bpm = blocks per MCU
    uint32_t block_pattern;           // component of MCU block b at bits 2b..2b+1
    uint32_t restart_interval;        // MCUs per interval (0 = single segment)
    uint32_t seg_base, nseg;          // this image's segments in the global segment list
    uint64_t block_base;              // first global block index
    uint32_t tableset;
    uint32_t chunk_base, nchunks;     // 16 KiB scan chunks of this image's ECS
    uint32_t sub_base, sub_cap;       // this image's share of its table set's piece-slot range (upper
                                      // bound of its pieces; k_subplan allocates them densely)
    uint32_t tile_mcus;               // MCU columns per IDCT/colour tile
    uint32_t tile_mrows;              // MCU rows per tile: always 1 (a tile is a run of MCUs of one
                                      // MCU row, tile_mcus * bpm <= 64; the DC prediction relies on it)
    uint32_t tiles_x, tiles_y;        // tiles per image row / column
    uint32_t lg_mw, lg_mh;            // log2 of the MCU width / height in pixels
    uint8_t h[4], v[4];
    uint16_t qslot[4];                // quant table of each component (index into batch Q array)
    uint8_t comp_block0[4];           // first MCU block of each component
    uint8_t shx[4], shy[4];           // log2(hmax / h[c]), log2(vmax / v[c])
    uint32_t tile_base;               // first tile of this image in BatchDev::tile_dc
    uint64_t planes;                  // fancy upsampling: device address of the int16 component planes
    uint32_t qmask;                   // k_idct_color's range test of quantised AC coefficients (bits
                                      // k..15 and 16+k..31: |c| <= 2^(k-1), 2^(k-1) * max step < 2^16)
    uint32_t entry_cap;               // AC-entry slots of this image (entry indices are image-relative):
                                      // its pieces' regions, then spare regions for re-walks
    uint64_t entry_base;              // first AC-entry slot of this image in BatchDev::entries
    uint32_t rw_div;                  // walk bits per region word the regions are sized for (region_words):
                                      // jd_plan.cpp region_divisor (worst case) or kOptRegionDiv
    uint32_t rw_slack;                // region words per piece beyond plen / rw_div (region_words)
    uint32_t rsv_[2];
};
static_assert(sizeof(ImgDesc) % 16 == 0, "ImgDesc must stay 16-byte aligned");

// Per-block result of the Huffman decode (sparse coefficient representation):
//   entry_start = index of the block's first AC-entry slot (16-bit units), relative to its image's
//                 ImgDesc::entry_base (32-bit units)
//   cnt_dc      = slots << kCntShift | escape flag (kCntEsc) | DC difference & kDcMask: the quantised
//                 DC difference as a 24-bit two's complement value; k_idct_color predicts the DC
// AC entry slot (16 bits) = value << 6 | zig-zag index (1..63) for |value| <= 511; a larger value
// (an AC size of 10 or more: rare below quality 95) takes two slots, 0x8000 | zig-zag index, then
// the value as int16, and sets the block's escape flag.
constexpr uint32_t kCntShift = 25, kCntEsc = 1u << 24, kDcMask = 0xFFFFFFu;
struct BlockInfo {
    uint32_t entry_start;
    uint32_t cnt_dc;
};

// A break in the raw ECS found by the scan: FF followed by RSTn, or a terminating marker.  One word
// (a 16 KiB chunk can hold 8 192 of them: the pool is kScanCap words per chunk, twice the ECS):
//   bits 0..13   byte offset of the FF in its scan chunk
//   bits 14..27  stuffed zero bytes in [chunk start, FF) (<= 8 192)
//   bit  31      terminating marker
struct Break {
    uint32_t w;
};
JD_HD inline Break brk_make(uint32_t rel, uint32_t drops, uint32_t term) { return Break{rel | (drops << 14) | (term << 31)}; }
JD_HD inline uint32_t brk_rel(Break k) { return k.w & 0x3FFFu; }
JD_HD inline uint32_t brk_drops(Break k) { return (k.w >> 14) & 0x3FFFu; }
JD_HD inline bool brk_term(Break k) { return (k.w >> 31) != 0u; }

constexpr uint32_t kInvalidImage = 0xFFFFFFFFu;

// Huffman decode geometry: every interval is cut into pieces of piece_bits un-stuffed bits, one
// lane each; a piece's walk synchronises from piece_overlap bits before its start (jd_kernels.hip
// k_piece; reference: parallelHuffManDecode, cuda-decoder/src/parser.cu:132-208).  4:2:0 MCU
// phase needs a few thousand bits to lock: speculative starts failed 45 % / 12 % / 0.6 % of the
// time at 1024 / 2048 / 4096 bits on the bench images (tools/jd_trace.py emulate()).  16384-bit
// pieces (the warm-up is a fifth of a lane's walk) measured best against 8192 / 24576 / 32768 on
// C2, C3 and C5 once consecutive batches overlap (their longer tails are hidden).
#ifndef JD_PIECE_BITS
#define JD_PIECE_BITS 16384
#endif
#ifndef JD_PIECE_OVERLAP
#define JD_PIECE_OVERLAP 4096
#endif
constexpr uint32_t kPieceBits = JD_PIECE_BITS;
constexpr uint32_t kPieceOverlap = JD_PIECE_OVERLAP;
constexpr uint32_t kMinPieceBits = 512;      // adaptive floor (small batches)
constexpr uint64_t kPieceTarget = 65536;    // pieces wanted per batch before shrinking stops
#ifndef JD_PIECE_THREADS
#define JD_PIECE_THREADS 512
#endif
// One workgroup shares one copy of its table set in LDS (four 8.4 KB tables for 4:2:0 + 76 B per
// lane: two 512-lane workgroups per CU, 16 waves).
constexpr int kPieceThreads = JD_PIECE_THREADS;
// Batches with fewer piece lanes than this run k_piece in 64-lane workgroups.
#ifndef JD_SMALL_PIECE_LANES
#define JD_SMALL_PIECE_LANES 16384
#endif
constexpr uint32_t kSmallPieceLanes = JD_SMALL_PIECE_LANES;
// k_chain leaves intervals of more pieces to k_chain_big (wave-parallel re-walk rounds and counts),
// which the host launches instead of k_chain_fix when an image's ECS may hold that many pieces
constexpr uint32_t kBigInterval = 256;

// Scan / compaction geometry: each chunk is 16 KiB of one image's ECS, 256 threads x 64 bytes.
constexpr int kScanThreads = 256;
constexpr int kScanBytesPerThread = 64;
constexpr int kScanChunk = kScanThreads * kScanBytesPerThread;
constexpr int kScanCap = kScanChunk / 2;  // a break takes 2 bytes: a chunk cannot hold more
constexpr uint32_t kBrkSlack = 16;        // optimistic break slots beyond the batch's most intervals
static_assert(kScanChunk <= 16384, "Break: 14-bit chunk offsets and drop counts");

#ifndef JD_CP_MAX
#define JD_CP_MAX 8
#endif
constexpr int kCpMax = JD_CP_MAX;  // checkpoints per piece (k_redo / k_chain_fix joins)
constexpr int kCpRecords = kCpMax + 1;

// Speculative-walk checkpoints, kCpRecords per piece slot: kCpMax checkpoints, then the totals.
//   checkpoint: {bit of an MCU boundary, MCUs and AC entries written up to it (entries = offset in
//                the piece's region), the walk's MCU index of its first error between the previous
//                checkpoint (or the start) and this one (kNoError: none)}
//   totals:     {end, MCUs, AC entries, first error after the last checkpoint}
// (piece_join: tail << 24 | checkpoints << 16, tail = the walk's MCUs begun in the data's last byte)
// A re-walk from the true start that reaches a checkpoint's bit at an MCU boundary is in the
// speculative walk's state there, so it joins it: the piece is then the re-walk's blocks followed
// by the speculative walk's blocks from that checkpoint on (two segments, k_gather), and its first
// error is the re-walk's or the speculative walk's first after that checkpoint (the speculative
// walk's first error overall may lie before, in bits it decoded out of sync).
struct alignas(16) CpRec {
    uint32_t bit, mcus, ents, flags;
};
constexpr uint32_t kNoError = 0xFFFFFFFFu;
// piece_emcu: the MCUs before the piece's first error, or, >= kTailErr, no error and kNoError - it
// of its MCUs began in the data's last byte (an interval ending at RSTn may end before them: k_chain)
constexpr uint32_t kTailErr = kNoError - 15u;

// Per-piece output region (image-relative AC-entry slots): AC entries ascend from its start, one
// 32-bit record per block (AC-entry count << 16 | 16-bit DC difference) descends from its end.  A
// block (one word) and an emitted entry (half a word) each take at least a table-dependent number
// of walk bits (jd_plan.cpp region_divisor: at least 2 for any tables, 4 for the standard Annex K
// tables), so a piece of plen bits fills at most plen / div + kRegionSlack words: the MCU that
// straddles the piece's end (<= 10 blocks x 64) and one window round past the data end (<= 272), see
// jd_kernels.hip walk_piece, whose region guard stops a walk (as an error) before it could overrun.
constexpr uint32_t kRegionSlack = 1040;
// Optimistic regions (the default plan): sized for kOptRegionDiv walk bits per word
// (C2's streams average 13), with a slack of the image's own largest MCU (64 words a block) plus one
// window round (kRoundItemsMax).  A walk whose region fills up stops at the region guard and flags
// its image kStOverflow; the host then decodes that image again with the worst-case plan
// (jd_runtime.cpp run_retries), so a dense stream costs time, never correctness.
constexpr uint32_t kOptRegionDiv = 8u;
constexpr uint32_t kRoundItemsMax = 152u;  // >= jd_kernels.hip kRoundItems (static_assert there)
JD_HD inline uint32_t opt_region_slack(uint32_t bpm) { return 64u * bpm + kRoundItemsMax + 8u; }
// Entry quads are stored in pairs (32 bytes, one HBM write granule) into 32-byte aligned regions:
// a lane's region line stays open for ~60 walk iterations and is written back piecemeal when the
// L2 (4 MB per XCD, ~32 K lanes each streaming into their own lines) evicts it, each 16-byte quad
// costing a 32-byte write (C2: k_piece WRITE_SIZE 3.98 -> 2.30 GB per launch).
constexpr uint32_t kRegionAlign = 8u;  // words
JD_HD inline uint32_t region_words(uint32_t plen, uint32_t div = 2u, uint32_t slack = kRegionSlack) {
    return ((plen + div - 1u) / div + slack + kRegionAlign - 1u) & ~(kRegionAlign - 1u);
}

constexpr int kIdctThreads = 64;      // one wave per IDCT/colour tile
#ifndef JD_TILE_BLOCKS
#define JD_TILE_BLOCKS 60
#endif
constexpr int kTileMaxBlocks = JD_TILE_BLOCKS;   // blocks per IDCT/colour tile (one lane each; k_idct_color's LDS)

// k_colour_fancy's workgroup (fancy upsampling): kFancyW x kFancyH-pixel bands, kFancyBands of them
// stacked vertically (the next band's window is fetched while the current one is coloured).  The
// host sizes the grid from the same constants (jd_runtime.cpp launch_batch).
#ifndef JD_FANCY_BANDS
#define JD_FANCY_BANDS 8
#endif
constexpr uint32_t kFancyW = 128, kFancyH = 16, kFancyBands = JD_FANCY_BANDS;
constexpr uint32_t kFancyRowsPerWg = kFancyH * kFancyBands;

// Per-image status bits written by kernels (atomicOr); host maps them to jd_status.
constexpr uint32_t kStCorrupt = 1u;     // bad code / overrun / DC range
constexpr uint32_t kStRstMissing = 2u;  // fewer RST markers than intervals
constexpr uint32_t kStRstOrder = 4u;    // RSTn numbering wrong
constexpr uint32_t kStOverflow = 8u;    // an optimistic pool was too small for the image (a piece region,
                                        // or a chunk's break list before the ECS end): decode it again
                                        // with the worst-case plan (jd_runtime.cpp run_retries)

// Per IDCT/colour tile: k_dc_sum's aggregate (sums of the DC differences of components 0..2 after
// the tile's last interval start, flag = it has one), which k_dc_scan turns into the components'
// DC predictors at the tile's first block (flag 0).
struct alignas(16) DcPred {
    int32_t p0, p1, p2, flag;
};

struct TileRef {
    uint32_t img, tile;
};

// BatchDev::counters after the first four (jd_stats): pieces k_redo re-walked; intervals k_chain_fix /
// k_chain_big fixed, their rounds (a serial k_chain_fix pass counts one) and re-walked pieces, and the
// k_chain_big intervals that stopped early at a right piece with an error
constexpr int kCtrRedo = 4, kCtrFixIntervals = 5, kCtrFixRounds = 6, kCtrFixRewalks = 7, kCtrFixEarly = 8;
constexpr int kNumCounters = 10;

struct BatchDev {
    const ImgDesc* imgs;
    uint32_t nimg;
    const HuffLut* luts;
    const TableSet* tablesets;
    const HuffLut* set_luts;  // every table set's LUTs, contiguous per set (global-memory lookups)
    const uint16_t* qtabs;        // 64 x uint16 per quant table, zig-zag order
    // segments (restart intervals)
    const uint32_t* seg_img;      // image of each segment
    uint32_t* seg_cstart;         // first un-stuffed byte of each segment (image-relative)
    uint32_t* seg_cend;           // end of each segment's data (image-relative, un-stuffed)
    uint32_t* seg_sub_base;       // first piece slot of each segment
    uint32_t* seg_nsub;           // pieces of each segment
    uint32_t nseg;
    // pieces (per image a slot capacity of ceil(ECS bits / piece_bits) + nseg, padded)
    uint32_t* sub_seg;            // segment of each piece slot (kInvalidImage = unused)
    uint32_t nsub;                // multiple of kPieceThreads
    const uint32_t* wg_tableset;  // table set of each k_piece workgroup
    uint32_t* ts_cursor;          // next free piece slot of each table set's range: k_subplan packs the
                                  // pieces of the batch's images densely from its start (whole waves
                                  // of the range's tail stay unused and exit at once)
    const uint32_t* img_order;    // images in table-set order (the host's piece-slot ranges)
    uint32_t* img_cand;           // k_index (large batches): pieces of each image at k_pieceplan's 16
                                  // candidate piece sizes
    uint32_t* img_base;           // k_pieceplan: first piece slot of each image
    uint32_t max_slots;           // LUT slots staged per workgroup
    uint32_t piece_bits, piece_overlap;
    uint32_t piece_plan;          // k_pieceplan: resident piece lanes (0: use piece_bits as is)
    uint32_t* seg_ent;            // k_subplan: first region word of each segment's pieces (image-relative)
    unsigned long long* img_pool; // k_subplan: next free region word of each image (re-walk regions; 64-bit: never wraps)
    uint32_t no_pool;             // 1: re-walks always write over their own region (tests, JD_SPARE_PIECES=0)
    uint32_t* piece_bit;          // first bit of the piece (an MCU boundary; kNoPiece: none found)
    uint32_t* piece_end;          // first MCU boundary at/after the piece's nominal end (or data end)
    uint32_t* piece_nmcu;         // MCUs walked (chain: MCUs the piece contributes)
    uint32_t* piece_nent;         // AC entries written
    uint32_t* piece_emcu;         // MCUs before the first error (kNoError: none)
    uint32_t* piece_abase;        // first word of the region holding segment A (image-relative)
    uint32_t* piece_amcu;         // MCUs in segment A
    uint32_t* piece_join;         // checkpoints recorded << 16 | (segment B = own region from
                                  // checkpoint join - 1; 0 = none)
    uint32_t* piece_mcu0;         // chain: first MCU of the piece within its segment
    uint32_t* seg_fix;            // k_chain: 1 = the interval needs k_chain_fix / k_chain_big
    uint32_t big_chain;           // a small batch (no piece plan) whose intervals may have more than
                                  // kBigInterval pieces: k_chain_big, and re-walks with LDS tables
    uint32_t small_fold;          // small batch (no piece plan): k_compact's first workgroups run the subplan
    CpRec* piece_cp;              // kCpRecords per piece slot (CpRec)
    const uint32_t* chain_seg;    // k_chain_fix: segment of each lane, grouped by table set
    uint32_t nchain;              // multiple of kPieceThreads
    const uint32_t* chain_wg_tableset;
    // scan / compaction
    uint32_t max_chunks;
    uint32_t* chunk_nbrk;         // breaks per chunk
    uint32_t* chunk_drops;        // stuffed zero bytes per chunk
    uint32_t* chunk_coff;         // un-stuffed offset of each chunk's first byte
    Break* chunk_brk;             // brk_cap per chunk
    uint32_t brk_cap;             // break slots per chunk: kScanCap (worst case), or the batch's most
                                  // restart intervals + kBrkSlack (every RSTn and the EOI of a valid
                                  // stream; k_index flags kStOverflow when a chunk before the ECS end
                                  // held more)
    // outputs
    BlockInfo* blocks;
    uint32_t* entries;
    uint64_t entries_cap;         // entry slots allocated
    uint32_t* status;             // per image
    unsigned long long* counters; // kNumCounters: [0] AC entries written, [1] slow_tiles entries, [2] k_idct_color's
                                  // tile queue, [3] k_pieceplan's choice, then the re-walk counters (kCtr*), [4] k_piece workgroups started (walk order)
    uint32_t max_tiles;
    TileRef* slow_tiles;          // (image, tile) k_idct_color left to k_idct_color_exact; count in counters[1]
    uint32_t total_tiles;
    DcPred* tile_dc;              // per tile: k_dc_sum aggregates, then (k_dc_scan) the DC predictors
                                  // of components 0..2 at the tile's first block
    // fancy upsampling (JD_FLAG_FANCY_UPSAMPLING): k_idct_color writes component planes to HBM
    // (ImgDesc::planes), k_colour_fancy filters and colours them
    // k_idct_color<M>: the batch's images of each sampling layout (kModeGen, kMode420, kMode422,
    // kMode444 in jd_kernels.hip): mode_imgs[mode_off[m] .. + mode_cnt[m]), at most mode_max_tiles[m] tiles
    const uint32_t* mode_imgs;
    uint32_t mode_off[4], mode_cnt[4], mode_max_tiles[4];
    unsigned long long* stamps;   // diagnostic builds (JD_STAMP): 8 s_memtime stamps per IDCT tile, else null
    uint32_t fancy;
    uint32_t max_fancy_wgs;       // k_colour_fancy bands per image: x in bits 0..15, y in 16..31
    uint32_t fix_round_cap;       // diagnostics (JD_FIX_ROUND_CAP): k_chain_big gives up (corrupt) after this many rounds; 0: never
    uint32_t skip_redo;           // diagnostics (JD_SKIP_REDO): no k_redo (the speculative starts stay as k_piece left them)
};

}  // namespace jd
