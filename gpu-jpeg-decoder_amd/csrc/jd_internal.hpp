// jd_internal.hpp — data layout shared by the host runtime and the gfx950 kernels.
//
// Everything a kernel reads is described here; see DESIGN.md §4 for the HBM layout of a batch.
#pragma once

#include <stdint.h>

#include "jd.h"

namespace jd {

// Fast Huffman lookup width: one LDS read resolves every code of <= kLutBits bits (and, when the
// magnitude bits fit too, the coefficient value).  Longer codes take the canonical slow path.
constexpr int kLutBits = 10;
constexpr int kLutSize = 1 << kLutBits;

// Device Huffman table (built on the host from a DHT table, uploaded once, cached by content).
//   fast[i]: entry for the next kLutBits stream bits = i
//     bits 0..4  : bits to consume (0 = slow path)
//     bit  5     : value-complete (magnitude bits already included in the count)
//     bits 8..15 : symbol (DC: size s; AC: run<<4 | size)
//     bits 16..31: int16 coefficient value when value-complete
//   lim[l]     : left-justified 16-bit limit; a code has length l iff peek16 < lim[l] (and not
//                < lim[l-1]) — the canonical DECODE procedure of JPEG Annex F.2.2.3
//   base[l]    : valptr[l] - mincode[l]
struct alignas(16) HuffLut {
    uint32_t fast[kLutSize];
    uint32_t lim[20];
    int32_t base[20];
    uint8_t vals[256];
};
static_assert(sizeof(HuffLut) % 16 == 0, "HuffLut must stay 16-byte aligned");
constexpr uint32_t kLutFlagComplete = 32u;

// Maximum Huffman tables a table set (one workgroup of the Huffman kernel) stages into LDS.
constexpr int kSlotsPerSet = 6;

// Per table set: which cached LUT each slot holds and which slot each component uses.
struct TableSet {
    int32_t lut[kSlotsPerSet];  // index into the LUT array (-1 = unused)
    uint8_t dc_slot[4];
    uint8_t ac_slot[4];
    int32_t nslots;
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
    uint32_t sub_base, sub_cap;       // this image's range in the subsequence list (upper bound)
    uint32_t tile_mcus;               // MCU columns per IDCT/colour tile
    uint32_t tile_mrows;              // MCU rows per tile (tile_mcus * tile_mrows * bpm <= 64)
    uint32_t tiles_x, tiles_y;        // tiles per image row / column
    uint32_t lg_mw, lg_mh;            // log2 of the MCU width / height in pixels
    uint8_t h[4], v[4];
    uint16_t qslot[4];                // quant table of each component (index into batch Q array)
    uint8_t comp_block0[4];           // first MCU block of each component
    uint8_t shx[4], shy[4];           // log2(hmax / h[c]), log2(vmax / v[c])
    uint32_t pad[1];
};

// Per-block result of the Huffman kernel (sparse coefficient representation):
//   entry_start = index of the block's first AC entry in the entry array
//   cnt_dc      = (number of AC entries << 16) | (uint16)DC   (DC un-predicted, still quantised)
// AC entry = (int16 value << 16) | zig-zag index (1..63).
struct BlockInfo {
    uint32_t entry_start;
    uint32_t cnt_dc;
};

// A break in the raw ECS found by the scan: FF followed by RSTn, or a terminating marker.
//   pos  : byte position in the file
//   info : (stuffed zero bytes in [chunk start, pos) << 1) | is_terminator
struct Break {
    uint32_t pos;
    uint32_t info;
};

constexpr uint32_t kInvalidImage = 0xFFFFFFFFu;

// Self-synchronising decode: every restart interval (segment) is cut into subsequences of
// kSubBits bits of un-stuffed data, one lane each (reference:
// parallelHuffManDecode, cuda-decoder/src/parser.cu:132-208).  A decoder state is
//   p  : segment-relative bit position of the next symbol
//   sk : (bi << 16) | (k << 8) | ncur   — block-in-MCU, coefficient index (0 = DC next),
//        AC entries already emitted for the current block
constexpr int kSubBits = 512;
struct SubState {
    uint32_t p;
    uint32_t sk;
};
struct SubCount {  // decoded from a subsequence's true entry state
    uint32_t blocks;   // DC symbols (block starts)
    uint32_t entries;  // non-zero AC entries
    int32_t dc[3];     // sum of DC differences per component
    uint32_t pad;
};
struct SubEntry {  // verified entry state + prefix sums within the segment
    uint32_t p, sk;
    uint32_t blk;      // segment-relative index of the next block to start
    uint32_t ent;      // global index of the next AC entry
    int32_t pred[3];   // DC predictors
    uint32_t pad;
};

// Scan / compaction geometry: each chunk is 16 KiB of one image's ECS, 256 threads x 64 bytes.
constexpr int kScanThreads = 256;
constexpr int kScanBytesPerThread = 64;
constexpr int kScanChunk = kScanThreads * kScanBytesPerThread;
constexpr int kScanCap = kScanChunk / 2;  // a break takes 2 bytes: a chunk cannot hold more

constexpr int kHuffThreads = 256;
constexpr int kSegThreads = 64;  // k_seg workgroup: one lane per restart interval
// An image is decoded interval-per-lane (k_seg) when it has at least this many restart
// intervals; otherwise (no DRI, or very long intervals) by the self-synchronising passes.
constexpr uint32_t kMinLaneSegments = 4;
constexpr int kIdctThreads = 64;      // one wave per IDCT/colour tile
constexpr int kTileMaxBlocks = 64;   // blocks per IDCT/colour tile (one lane each)

// Per-image status bits written by kernels (atomicOr); host maps them to jd_status.
constexpr uint32_t kStCorrupt = 1u;     // bad code / overrun / DC range
constexpr uint32_t kStRstMissing = 2u;  // fewer RST markers than intervals
constexpr uint32_t kStRstOrder = 4u;    // RSTn numbering wrong

struct BatchDev {
    const ImgDesc* imgs;
    uint32_t nimg;
    const HuffLut* luts;
    const TableSet* tablesets;
    const uint16_t* qtabs;        // 64 x uint16 per quant table, zig-zag order
    // segments (restart intervals)
    const uint32_t* seg_img;      // image of each segment
    uint32_t* seg_cstart;         // first un-stuffed byte of each segment (image-relative)
    uint32_t* seg_cend;           // end of each segment's data (image-relative, un-stuffed)
    const uint32_t* seg_entry;    // first AC-entry slot of each segment
    uint32_t* seg_sub_base;       // first subsequence of each segment
    uint32_t* seg_nsub;           // subsequences of each segment
    uint32_t nseg;
    // subsequences
    uint32_t* sub_seg;            // segment of each subsequence (kInvalidImage = unused)
    uint32_t nsub;                // multiple of kHuffThreads
    const uint32_t* wg_tableset;  // table set of each decode workgroup (kHuffThreads subsequences)
    uint32_t max_slots;           // LUT slots staged per decode workgroup
    SubState* exit_spec;          // pass 0 exits (speculative entries)
    SubState* exit_cnt;           // pass 1 exits
    SubCount* sub_cnt;            // pass 1 counts
    SubEntry* sub_entry;          // chain output
    // restart-interval lanes (images with DRI, decoded by k_seg)
    const uint32_t* seg_lane;     // segment of each lane (kInvalidImage = padding)
    uint32_t nseg_lane;           // multiple of kSegThreads
    const uint32_t* lane_wg_tableset;  // table set of each k_seg workgroup
    // scan / compaction
    uint32_t max_chunks;
    uint32_t* chunk_nbrk;         // breaks per chunk
    uint32_t* chunk_drops;        // stuffed zero bytes per chunk
    uint32_t* chunk_coff;         // un-stuffed offset of each chunk's first byte
    Break* chunk_brk;             // kScanCap per chunk
    // outputs
    BlockInfo* blocks;
    uint32_t* entries;
    uint64_t entries_cap;         // entry slots allocated
    uint32_t* status;             // per image
    unsigned long long* counters; // [0] AC entries written
    uint32_t max_tiles;
};

}  // namespace jd
