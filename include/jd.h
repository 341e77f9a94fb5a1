/*
 * jd.h — C ABI of the MI355X-native batched JPEG decoder (libjdamd.so).
 *
 * This is the drop-in boundary for the reference's decode(file/bitstream) -> RGB path.  The
 * reference exposes that path as C++ free functions plus two CUDA kernels
 * (/root/reference/cuda-decoder/src/parser.h:49-55) and, on the CPU side, the class
 * JPEGParser{ctor(path), extract(), decode(), write()} (/root/reference/cpp-decoder/src/parser.h:42-69).
 * Each entry point below names the reference interface it replaces.  Everything is plain C:
 * pointers, sizes, status codes; no exceptions cross this boundary and no torch types appear.
 *
 * Output format: interleaved uint8 RGB, H*W*3 bytes, row-major (the reference writes the same
 * values as three int planes in a text `.array` file — jd_write_array reproduces that file).
 *
 * Threading: a jd_ctx belongs to one host thread and one HIP device.  Calls on one context are
 * ordered: the memcpy helpers and jd_synchronize run after every batch the context has launched
 * (pending jd_decode_batch_async work included, on whichever stream it runs).  jd_parse and
 * jd_write_array are reentrant and context-free.
 */
#ifndef JD_H
#define JD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JD_ABI_VERSION 8

typedef enum jd_status {
    JD_OK = 0,
    JD_ERR_INVALID_ARG = 1, /* NULL pointer, bad size, bad device                             */
    JD_ERR_CORRUPT = 2,     /* malformed stream (bad Huffman code, missing RSTn, overrun ...)   */
    JD_ERR_UNSUPPORTED = 3, /* progressive / arithmetic / 12-bit / CMYK / multi-scan input      */
    JD_ERR_TRUNCATED = 4,   /* file ends inside the headers                                     */
    JD_ERR_HIP = 5,         /* a HIP runtime call failed (reference: checkCudaError throws,
                               cuda-decoder/src/parser.cu:317-321)                              */
    JD_ERR_NOMEM = 6,       /* device or host allocation failed                                 */
    JD_ERR_CAPACITY = 7,    /* batch exceeds the context's limits                               */
    JD_ERR_IO = 8           /* file could not be read / written                                 */
} jd_status;

typedef struct jd_ctx jd_ctx;

/* jd_opts.flags */
#define JD_FLAG_TIMING 1u /* record hipEvents around every kernel launch (jd_get_stats) */
/* Entropy-decode piece size.  Default: pieces of at least 16384 bits (kPieceBits) with a 4096-bit
 * warm-up; for large batches the device-side planner (k_pieceplan) grows them up to ~2x so the
 * pieces fill whole rounds of resident lanes.  Results are identical for every setting; the flags
 * exist so tests can stress the two extremes of the piece-parallel decode. */
#define JD_FLAG_FORCE_SYNC 2u  /* 1024-bit pieces: many speculative starts, exercises re-walks */
#define JD_FLAG_FORCE_LANES 4u /* one piece per restart interval (the whole scan if no DRI) */
/* Small batches (under ~64 K pieces of 16384 bits) use shorter pieces by default, down to 512 bits
 * with a 2x-piece warm-up; this flag keeps 16384-bit pieces / 4096-bit warm-up for every batch
 * (k_pieceplan may still grow them for large batches). */
#define JD_FLAG_FULL_PIECES 16u
/* Chroma upsampling: replicate (default; the semantics pinned in DESIGN.md §2) or, with this flag,
 * libjpeg's triangular "fancy" filter for 2x1, 2x2 and 1x2 ratios (closer to libjpeg-turbo /
 * Pillow output; an option beyond the reference, which has no subsampled chroma at all). */
#define JD_FLAG_FANCY_UPSAMPLING 8u
/* jd_decode_batch_async leaves two batches in flight instead of one: a call collects the batch
 * launched two calls before it, so results[], rgb and jpeg_dev buffers of batch k stay in use until
 * call k + 2 returns (or jd_decode_wait).  Measured 3-4 % slower on the bench configs (DESIGN.md
 * §4.5); an explicit opt-in because it changes when a caller may reuse those buffers. */
#define JD_FLAG_ASYNC_DEPTH2 32u
/* Device pools.  By default a batch's scratch is sized for the data it is likely to hold: piece
 * regions of sparse coefficients for 8 walk bits per 32-bit word (real streams take 10-14) and
 * scan break lists for the batch's restart intervals.  An image that overflows one is decoded again
 * with worst-case pools before its batch is reported (jd_stats.retried_images): the results are the
 * same, the pools about half as large.  This flag plans every batch with worst-case pools (no retry
 * can happen; about twice the device memory).  At async depth 2 a batch with host-memory inputs is
 * always planned with worst-case pools (its inputs' device copy does not outlive its slot's next
 * launch, which precedes its collection). */
#define JD_FLAG_WORST_CASE_POOLS 64u

typedef struct jd_opts {
    unsigned flags;
    int parse_threads; /* host parse workers for jd_decode_batch; 0 = auto (hardware threads) */
} jd_opts;

/* Subsampling classes reported by jd_parse. */
#define JD_SS_GRAY 0
#define JD_SS_444 1
#define JD_SS_422 2
#define JD_SS_420 3
#define JD_SS_440 4
#define JD_SS_OTHER 5

typedef struct jd_header {
    int width, height, ncomp;
    int h[4], v[4], tq[4];
    int hmax, vmax, mcux, mcuy, blocks_per_mcu;
    int restart_interval; /* MCUs per restart interval, 0 = none (DRI absent) */
    int subsampling;      /* JD_SS_* */
    uint64_t ecs_offset;  /* first byte of the entropy-coded segment */
} jd_header;

/* One batch item.  `jpeg` (host) is always required: headers are parsed on the host.
 * `jpeg_dev` may point at a device copy of the same bytes (already resident in HBM); when NULL the
 * library uploads the file itself.  `rgb` receives H*W*3 bytes; it is a device pointer when the
 * batch call's rgb_on_device is non-zero, otherwise a host pointer. */
typedef struct jd_item {
    const uint8_t* jpeg;
    const uint8_t* jpeg_dev;
    size_t len;
    uint8_t* rgb;
} jd_item;

typedef struct jd_result {
    int status; /* jd_status of this image; a bad image never poisons the rest of the batch */
    int width, height;
} jd_result;

/* Context: owns the device pools, stream, events and table caches.
 * Replaces the reference's allocate() (cuda-decoder/src/parser.cu:324-358). */
jd_status jd_ctx_create(jd_ctx** ctx, int hip_device, const jd_opts* opts);
/* Replaces clean() (cuda-decoder/src/parser.cu:684-700). */
jd_status jd_ctx_destroy(jd_ctx* ctx);

/* Header parse only, host, reentrant.  Replaces the marker walk of extract()
 * (cuda-decoder/src/parser.cu:360-471, cpp-decoder/src/parser.cpp:24-103). */
jd_status jd_parse(const uint8_t* jpeg, size_t len, jd_header* hdr);

/* decode(bitstream) -> RGB for one image.  Replaces extract()+decodeKernel<<<1,T>>>+write's D2H
 * (cuda-decoder/main.cu:7-40, parser.cu:577-611) and JPEGParser::extract()+decode()
 * (cpp-decoder/src/parser.cpp:24-195).  rgb must hold H*W*3 bytes. */
jd_status jd_decode(jd_ctx* ctx, const uint8_t* jpeg, size_t len, uint8_t* rgb, int rgb_on_device,
                    int* width, int* height);

/* Same, reading the file.  Mirrors the CLI `decoder <jpeg>` (cpp-decoder/main.cpp:5-16). */
jd_status jd_decode_file(jd_ctx* ctx, const char* path, uint8_t* rgb, size_t rgb_capacity,
                         int rgb_on_device, int* width, int* height);

/* Batched decode of independent images.  Replaces batchDecodeKernel<<<N,T>>>(DeviceData*)
 * (cuda-decoder/src/parser.cu:663-682, driven by benchmark_thoughput/benchmark.cu:43-93).
 * hip_stream: hipStream_t to order the work on, or NULL for the context's own stream.  The call
 * returns after the batch completes; per-image status in results[i].  The context's scratch pools
 * are ordered by stream only: a call on another stream than the one of still-pending
 * jd_decode_batch_async launches first collects them (jd_decode_wait).  Any n: the library
 * launches the batch in sub-batches of at most 65535 items (and of at most a device-pool budget of
 * sparse coefficients), each collected before the next. */
jd_status jd_decode_batch(jd_ctx* ctx, const jd_item* items, int n, jd_result* results,
                          int rgb_on_device, void* hip_stream);

/* Pipelined form of jd_decode_batch with device outputs (rgb are device pointers): returns once
 * the batch is launched, after collecting the batch launched before it, so the host parses and
 * plans batch k+1 (and stages its host inputs) while the GPU decodes batch k.  Inputs may be
 * device-resident (jpeg_dev) or host memory (jpeg_dev NULL): host inputs are copied into the
 * launching slot's pinned staging by the context's host workers before the call returns, and
 * uploaded by an H2D on that slot's stream, which overlaps the other slot's kernels.  results[],
 * the rgb buffers and the jpeg_dev buffers must stay valid and unused by other calls until the
 * batch is collected: by the next jd_decode_batch_async call (the second next with
 * JD_FLAG_ASYNC_DEPTH2, which leaves two batches in flight), by a jd_decode_batch call, or by
 * jd_decode_wait; host jpeg buffers only until the call returns, unless they lie in a range
 * registered with jd_host_register (then until the batch is collected). */
jd_status jd_decode_batch_async(jd_ctx* ctx, const jd_item* items, int n, jd_result* results,
                                void* hip_stream);
/* Collects every launched batch (fills their results). */
jd_status jd_decode_wait(jd_ctx* ctx);

/* Registers a caller-owned host range (page-locks it for DMA; hipHostRegister) for inputs: a
 * batch item whose `jpeg` bytes lie in a registered range and that has no `jpeg_dev` is uploaded
 * straight from it, neighbouring files in one DMA, without the copy into the context's pinned
 * staging.  Unlike staged inputs, such bytes are read after jd_decode_batch_async returns: they
 * must stay unchanged until the batch is collected.  The reference copies each image to the
 * device inside its host loop (cuda-decoder/src/parser.cu:441-467, driven per image by
 * benchmark_thoughput/benchmark.cu:49-60); this replaces that copy for callers that keep their
 * files in one arena.  Ranges may not overlap.  jd_host_unregister waits for the context's
 * in-flight batches before unlocking; jd_ctx_destroy unregisters what is left. */
jd_status jd_host_register(jd_ctx* ctx, void* ptr, size_t bytes);
jd_status jd_host_unregister(jd_ctx* ctx, void* ptr);
/* The same for an arena the library allocates (hipHostMalloc pinned memory) for the caller to
 * read its files into: inputs in it are uploaded straight from it.  jd_host_free waits for the
 * context's in-flight batches before freeing; jd_ctx_destroy frees what is left. */
jd_status jd_host_alloc(jd_ctx* ctx, size_t bytes, void** ptr);
jd_status jd_host_free(jd_ctx* ctx, void* ptr);

/* `.array` text writer: "H W\n", then R, G, B planes as space-terminated decimal ints, one plane
 * per line, no trailing newline.  Replaces JPEGParser::write() (cpp-decoder/src/parser.cpp:197-209)
 * and the CUDA write() (cuda-decoder/src/parser.cu:702-744). */
jd_status jd_write_array(const char* path, const uint8_t* rgb, int width, int height);

/* Binary PPM (P6) writer: "P6\n<W> <H>\n255\n" then the interleaved RGB bytes — the format of the
 * reference's libjpeg comparison outputs (testing/jpeglib_output_ppm/<name>.ppm, read back by
 * jpeglib-implementation/process_ppm.py into `.array` files for testing/compare.py). */
jd_status jd_write_ppm(const char* path, const uint8_t* rgb, int width, int height);

const char* jd_status_str(jd_status st);
int jd_abi_version(void);
/* Text of the most recent HIP failure on this context ("" if none). */
const char* jd_ctx_last_error(jd_ctx* ctx);

/* Device-memory helpers for FFI callers that bring no allocator of their own (ctypes tests). */
jd_status jd_device_alloc(jd_ctx* ctx, size_t bytes, void** dptr);
jd_status jd_device_free(jd_ctx* ctx, void* dptr);
jd_status jd_memcpy_h2d(jd_ctx* ctx, void* dst_dev, const void* src_host, size_t bytes);
jd_status jd_memcpy_d2h(jd_ctx* ctx, void* dst_host, const void* src_dev, size_t bytes);
jd_status jd_synchronize(jd_ctx* ctx);

/* Per-kernel timing (JD_FLAG_TIMING).
 * Kernels: 0 k_scan, 1 k_index, 2 k_compact, 3 k_subplan, 4 k_piece, 5 k_redo, 6 k_chain,
 * 7 k_gather, 8 k_dc_pred, 9 k_idct_color, 10 k_colour_fancy. */
#define JD_NUM_KERNELS 11
typedef struct jd_stats {
    int launches[JD_NUM_KERNELS];
    double total_ms[JD_NUM_KERNELS]; /* hipEvent time, summed over launches                     */
    double bytes[JD_NUM_KERNELS];    /* algorithmic bytes moved, summed          */
    double batches, images, pixels, ecs_bytes, blocks, segments, subsequences;
    /* host wall time (ms, summed): 0 header parse, 1 plan + plan upload, 2 staging of host-memory
     * inputs (parallel memcpy into pinned memory + H2D issue), 3 waiting for batches to finish */
    double host_ms[4];
    double h2d_bytes; /* host-memory input bytes uploaded */
    double h2d_registered_bytes; /* file bytes uploaded straight from registered ranges (no staging copy) */
    /* speculative decode: pieces k_redo re-walked; intervals whose starts still
     * disagreed after it (k_chain_fix / k_chain_big), their re-walk rounds and re-walked pieces, and
     * the k_chain_big intervals that stopped early at a right piece with an error (corrupt data or
     * trailing bytes) */
    double redo_pieces, fix_intervals, fix_rounds, fix_rewalks, fix_early;
    /* images decoded again with worst-case pools after overflowing an optimistic one
     * (JD_FLAG_WORST_CASE_POOLS); the retry's batch counts in batches, images, pixels and the
     * kernel figures like any other */
    double retried_images;
} jd_stats;
jd_status jd_get_stats(jd_ctx* ctx, jd_stats* out);
jd_status jd_reset_stats(jd_ctx* ctx);
const char* jd_kernel_name(int k);
/* Device memory the context's pools hold now and at most since creation (bytes; pools are
 * grow-only: the piece regions of the largest batch dominate). */
jd_status jd_device_bytes(jd_ctx* ctx, uint64_t* current, uint64_t* peak);

#ifdef __cplusplus
}
#endif
#endif /* JD_H */
