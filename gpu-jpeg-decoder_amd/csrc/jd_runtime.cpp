// jd_runtime.cpp — context, batch planning and the C ABI of libjdamd.so.
//
// A batch flows through: host header parse (C++ threads) -> plan (tables de-duplicated, segments,
// tiles, offsets) -> one H2D copy of the plan -> four kernels on the context stream -> per-image
// status D2H.  Device buffers are grow-only pools owned by the context, so steady-state batches do
// no allocation.  Replaces the reference's per-image extract()/allocate()/clean() cycle
// (cuda-decoder/benchmark_thoughput/benchmark.cu:49-93) which cudaMalloc'ed every image.
#include <emmintrin.h>
#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdio.h>
#include <chrono>
#include <cstdlib>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <array>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "jd.h"
#include "jd_internal.hpp"
#include "jd_kernels.hpp"
#include "jd_parse.hpp"
#include "jd_plan.hpp"
#include "jd_test.h"

using namespace jd;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};


inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Host-input staging copy into pinned memory with streaming (non-temporal) stores: the staging
// buffer is only read again by the H2D DMA, so its lines need not be fetched (no read-for-
// ownership) nor kept in the caches.  dst is 16-byte aligned (staging offsets are 256-B aligned,
// pieces 1 MiB apart); the fence makes the stores globally visible before the worker reports done.
void stage_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    if (i < n) memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

// roctx range over a host phase (parse / plan / launch / collect), visible in rocprofv3
// --marker-trace next to the kernels; the analogue of the reference's NVTX ranges
// (cuda-decoder/benchmark/benchmark.cu:41,70).
struct Range {
    explicit Range(const char* what) { roctxRangePushA(what); }
    ~Range() { roctxRangePop(); }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;
};

struct CachedLut {
    HuffSpec spec;
    bool is_dc;
};

// Persistent host workers for the per-image header work (a thread spawn per call would cost more
// than the parsing): run(n, fn) calls fn(0..n-1) across the workers and the caller.
class Pool {
   public:
    explicit Pool(int nworkers) {
        for (int i = 0; i < nworkers; i++) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(int n, const std::function<void(int)>& fn) {
        if (th_.empty() || n <= 1) {
            for (int i = 0; i < n; i++) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> l(m_);
            fn_ = &fn;
            n_ = n;
            next_ = 0;
            active_ = int(th_.size());
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return active_ == 0; });
    }

   private:
    void work() {
        for (int i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> l(m_);
        while (true) {
            cv_.wait(l, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            l.unlock();
            work();
            l.lock();
            if (--active_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0, active_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace

// One of the context's two device-scratch slots.  Each owns the device scratch of the batch it
// runs and, unless the caller names a stream, its own stream, so one batch's first kernels run
// beside the other slot's latency-bound tail (re-walks, chain, DC scan) and big kernels.  A slot is
// reused by every second launch; the work of consecutive launches on one slot is ordered by its
// stream, so batch k+2 can be planned and enqueued while batch k still runs.
struct Slot {
    hipStream_t stream = nullptr;                // this slot's internal stream
    DevBuf d_plan, d_brk, d_blocks, d_entries, d_comp, d_planes, d_stamps;  // device scratch of the batch
    void* plan_host = nullptr;                   // pinned staging of the slot's plan blob
    size_t plan_cap = 0;
    void* in_host = nullptr;                     // pinned staging of the slot's host-memory JPEG inputs
    size_t in_cap = 0;
    DevBuf d_input;                              // device copy of those inputs
    hipEvent_t h2d_done = nullptr;               // after the slot's latest host-input copies
    hipEvent_t plan_done = nullptr;              // after the slot's latest plan upload
    bool h2d_recorded = false, plan_recorded = false;
    // JD_IDCT_STREAM=1 (experiment): the colour stage on a stream of its own (JD_IDCT_PRIO), entered
    // and left through events, so that its waves can be given another dispatch priority
    hipStream_t istream = nullptr;
    hipEvent_t ev_tail = nullptr, ev_idct = nullptr;
};

// One launched batch whose results are not collected yet.  jd_decode_batch_async returns with the
// newest async_depth launches in flight: 1 by default (the previous launch is collected before the
// call returns); with JD_FLAG_ASYNC_DEPTH2 the host parses, plans and enqueues batch k+2 on its slot's
// stream (behind batch k) before it waits for batch k.  That starts batch k+2's front-end the
// moment batch k ends, but the two slots' walks then often run together, and the step measured
// 3-4 % slower.
struct Pending {
    bool active = false;
    uint64_t seq = 0;                           // launch order
    int slot = 0;                               // the slot it runs on
    jd_result* results = nullptr;
    int lo = 0, hi = 0;
    std::vector<jd_status> pst;                 // per item lo..hi: host-side status
    std::vector<int> w, h;                      // per item
    std::vector<int> item_of_img;
    std::vector<std::array<uint64_t, 3>> host_copies;  // {host dst, device src, bytes} (host output)
    uint32_t nimg = 0;
    void* host = nullptr;                       // pinned: u64 counters[4], then u32 status[nimg]
    size_t host_cap = 0;
    hipEvent_t done = nullptr;
    hipEvent_t ev[JD_NUM_KERNELS][2] = {};
    bool timing = false, fancy = false;
    double blocks = 0, pixels = 0, ecs = 0, nsub = 0, nseg = 0, chunks = 0, tiles = 0, piece_bits = 0, piece_overlap = 0;
    double t_plan = 0, t_upload = 0;
    // what a retry needs (run_retries): the items, their parsed headers and device bytes (dev_addr:
    // the caller's jpeg_dev, or the slot's copy of a host input, which stays until the slot's next
    // launch, i.e. past this batch's collection at async depth 1), and whether the plan was the worst case
    std::vector<jd_item> items;
    std::vector<ParsedJpeg> parsed;
    std::vector<uint64_t> dev_addr;
    int rgb_on_device = 1;
    bool worst = false;
};
// launch records (>= the async depth + 2: a record is reused 4 launches later)
constexpr int kNumPending = 4;
// timing slot of k_idct_color (jd_kernel_name): the colour stage starts here
constexpr int kIdctSlot = 9;
// batches of at most this many images without a piece plan fold the subplan into k_compact
// (jd_kernels.hip subplan_image: a launch saved on a small batch's critical path)
constexpr uint32_t kSmallFoldImages = 64;

struct jd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    unsigned flags = 0;
    int parse_threads = 1;
    std::unique_ptr<Pool> pool;  // parse_threads - 1 workers
    bool host_timing = false;  // JD_HOST_TIMING=1: per-batch host phase times on stderr
    std::string last_error;

    // Huffman LUT cache (content-addressed, grows across calls)
    std::unordered_multimap<uint64_t, int> lut_by_hash;
    std::vector<CachedLut> lut_specs;
    std::vector<HuffLut> lut_host;
    DevBuf lut_dev;
    size_t lut_dev_count = 0;

    // output pool shared by the slots (host outputs: collected before reuse); host inputs are
    // staged per slot (Pending::in_host / d_input), so host-input batches pipeline too
    DevBuf output;

    Slot slots[2];
    Pending pend[kNumPending];
    int slot = 0;                        // the slot the next launch uses
    uint64_t seq = 0;                    // launches so far (the next launch's record: pend[seq % kNumPending])
    int async_depth = 1;                 // batches jd_decode_batch_async leaves in flight (2: JD_FLAG_ASYNC_DEPTH2)
    const void* last_stream = nullptr;  // caller stream of the pending launches (nullptr: the slots' own)
    uint64_t max_batch_entries = 0;     // AC-entry slots per launched sub-batch (JD_MAX_BATCH_ENTRIES)
    int max_batch_images = 0;           // items per launched sub-batch (JD_MAX_BATCH_IMAGES)
    int64_t spare_pieces = -1;          // spare re-walk regions per image (JD_SPARE_PIECES; -1: default)
    // Pools: optimistic by default (piece regions at kOptRegionDiv bits per word, break lists of the
    // batch's most intervals); an image that overflows one is decoded again with the worst-case plan
    // (run_retries).  worst: the plan being built is the worst case (a retry, or every batch with
    // JD_FLAG_WORST_CASE_POOLS); brk_cap_force: JD_BRK_CAP (tests: break slots per chunk of
    // optimistic plans, to force the break-list overflow).
    bool worst = false, worst_always = false;
    uint32_t brk_cap_force = 0;
    struct Retry {
        jd_item item;
        ParsedJpeg pj;
        jd_result* res;
        int rgb_on_device;
    };
    std::vector<Retry> retry;  // overflowed images of collected batches, not yet decoded again
    int64_t piece_overlap = -1;         // warm-up bits (JD_PIECE_OVERLAP_BITS; -1: default)
    uint32_t min_piece_bits = kMinPieceBits;  // small batches' shortest pieces (JD_MIN_PIECE_BITS: a test knob)
    bool fixed_pieces = false;          // JD_FIXED_PIECES: keep the host's piece size (no k_pieceplan)
    size_t stage_chunk = size_t(128) << 20;  // host-input H2D chunk (JD_STAGE_CHUNK_MB; 0: one copy per batch)
    bool stage_nt = true;                     // streaming-store staging copy (JD_STAGE_NT=0: memcpy)
    // caller-owned host ranges registered with jd_host_register (page-locked, DMA-readable): host
    // inputs lying in one are uploaded straight from it, without the staging copy
    std::vector<std::pair<uintptr_t, uintptr_t>> host_regs;  // [begin, end), sorted by begin
    std::vector<uintptr_t> host_owned;  // the ranges jd_host_alloc allocated (hipHostMalloc)
    // Host-input copies of consecutive batches run one after the other (JD_H2D_SERIAL=0: as their
    // streams allow): two batches' DMAs interleaved on the link each took twice as long, delaying
    // both batches' kernels
    bool h2d_serial = true;
    hipEvent_t last_h2d = nullptr;  // the h2d_done event of the batch whose copies were issued last
    jd_stats stats{};

    std::vector<ParsedJpeg> parsed;
    std::vector<jd_status> pst;

    // last batch (jd_debug_fetch)
    BatchDev last{};
    uint64_t last_blocks = 0, last_entries = 0;
    std::vector<uint64_t> last_entry_base;  // per image (jd_debug_fetch 20)
    std::vector<uint32_t> last_rw_div;      // per image (jd_debug_fetch 21)
    std::vector<uint32_t> last_rw_slack;    // per image (jd_debug_fetch 22)
    uint64_t dev_bytes = 0, dev_peak = 0;   // device pool bytes held now / at most (jd_device_bytes)
};

namespace {

jd_status hip_fail(jd_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) ctx->last_error = std::string(what) + ": " + hipGetErrorString(e);
    return JD_ERR_HIP;
}

#define HIPCHK(ctx, call)                                         \
    do {                                                          \
        hipError_t e_ = (call);                                   \
        if (e_ != hipSuccess) return hip_fail((ctx), e_, #call);  \
    } while (0)

// Waits for everything this context has in flight: the pending batches (their done events, on
// the slot streams or a caller stream) and the context stream.  Unlike hipDeviceSynchronize it
// does not stall the caller's unrelated streams.
hipError_t quiesce(jd_ctx* ctx) {
    hipError_t r = hipSuccess;
    for (Pending& pd : ctx->pend)
        if (pd.active) {
            const hipError_t e = hipEventSynchronize(pd.done);
            if (e != hipSuccess) r = e;
        }
    if (ctx->stream) {
        const hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) r = e;
    }
    return r;
}

// Makes the context stream wait for the pending batches (jd.h: calls on one context are ordered).
hipError_t order_after_pending(jd_ctx* ctx) {
    for (Pending& pd : ctx->pend)
        if (pd.active) {
            const hipError_t e = hipStreamWaitEvent(ctx->stream, pd.done, 0);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

hipError_t ensure_dev(jd_ctx* ctx, DevBuf& b, size_t bytes) {
    if (bytes <= b.cap) return hipSuccess;
    const size_t n = std::max(bytes, b.cap + b.cap / 2);
    if (b.p) {
        (void)quiesce(ctx);  // a launched batch may still use it (jd_decode_batch_async)
        (void)hipFree(b.p);
        ctx->dev_bytes -= b.cap;
    }
    b.p = nullptr;
    b.cap = 0;
    hipError_t e = hipMalloc(&b.p, n);
    if (e == hipSuccess) {
        b.cap = n;
        ctx->dev_bytes += n;
        ctx->dev_peak = std::max(ctx->dev_peak, ctx->dev_bytes);
    }
    return e;
}


int lut_id(jd_ctx* ctx, const HuffSpec& s, bool is_dc, uint64_t h) {
    auto range = ctx->lut_by_hash.equal_range(h);
    for (auto it = range.first; it != range.second; ++it) {
        const CachedLut& c = ctx->lut_specs[size_t(it->second)];
        if (c.is_dc == is_dc && c.spec.nvals == s.nvals && !memcmp(c.spec.counts, s.counts, 17) &&
            !memcmp(c.spec.vals, s.vals, size_t(s.nvals)))
            return it->second;
    }
    HuffLut lut;  // the piece walks' format (pair fields: second symbol's bits and run/size byte)
    if (!build_lut(s, is_dc, &lut)) return -1;
    const int id = int(ctx->lut_host.size());
    ctx->lut_host.push_back(lut);
    ctx->lut_specs.push_back(CachedLut{s, is_dc});
    ctx->lut_by_hash.emplace(h, id);
    return id;
}

jd_status sync_luts(jd_ctx* ctx) {
    if (ctx->lut_dev_count == ctx->lut_host.size()) return JD_OK;
    HIPCHK(ctx, ensure_dev(ctx, ctx->lut_dev, ctx->lut_host.size() * sizeof(HuffLut)));
    HIPCHK(ctx, hipMemcpyAsync(ctx->lut_dev.p, ctx->lut_host.data(), ctx->lut_host.size() * sizeof(HuffLut),
                               hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->lut_dev_count = ctx->lut_host.size();
    return JD_OK;
}

void parse_all(jd_ctx* ctx, const jd_item* items, int n) {
    Range r("jd_parse");
    ctx->parsed.resize(size_t(n));
    ctx->pst.resize(size_t(n));
    constexpr int kPer = 16;  // images per work item
    ctx->pool->run((n + kPer - 1) / kPer, [&](int t) {
        for (int i = t * kPer; i < std::min(n, (t + 1) * kPer); i++) {
            ParsedJpeg& pj = ctx->parsed[i];
            ctx->pst[i] = parse_jpeg(items[i].jpeg, items[i].len, &pj);
            if (ctx->pst[i] != JD_OK) continue;
            for (int c = 0; c < pj.hdr.ncomp; c++) {
                pj.hdc[c] = hash_huff(pj.dc[pj.td[c]], true);
                pj.hac[c] = hash_huff(pj.ac[pj.ta[c]], false);
            }
        }
    });
}

struct Plan {
    std::vector<ImgDesc> imgs;
    std::vector<int> item_of_img;
    std::vector<TableSet> tablesets;
    std::vector<uint16_t> qtabs;
    std::vector<uint32_t> seg_img, wg_tableset;
    std::vector<uint32_t> ts_slot0;  // first piece slot of each table set's range (k_subplan allocates from it)
    std::vector<uint32_t> img_order;  // images in table-set order (k_pieceplan's dense allocation)
    uint32_t piece_bits = kPieceBits, piece_overlap = kPieceOverlap;
    std::vector<uint32_t> chain_seg, chain_wg_tableset;  // k_chain lanes, grouped by table set
    uint32_t total_chunks = 0, max_chunks = 0, max_tiles = 0, total_tiles = 0, max_slots = 1, nsub = 0, brk_cap = kScanCap;
    uint64_t total_blocks = 0, total_entry_cap = 0, comp_bytes = 0;
    double pixels = 0, ecs_bytes = 0;
    std::vector<uint32_t> mode_imgs;  // images grouped by sampling layout (k_idct_color<M>)
    uint32_t mode_off[4] = {0, 0, 0, 0}, mode_cnt[4] = {0, 0, 0, 0}, mode_max_tiles[4] = {0, 0, 0, 0};
};

// Largest item prefix [lo, hi) whose sparse-coefficient words stay within the context's
// max_batch_entries (default kMaxBatchEntries; entry indices are image-relative, this only bounds
// the pool, 4 B per word; estimated at full-size pieces) and that holds at most max_batch_images
// items (default kMaxBatchImages: the per-image kernels index images by the grid's y dimension,
// at most 65535).  JD_MAX_BATCH_ENTRIES / JD_MAX_BATCH_IMAGES override them (tests force
// multi-way splits).  12 G words (48 GB of entry pool per slot, two slots: a third of the 288 GB):
// the reference's own 3000-image batch (ref444, ~9 G words reserved) runs as one launch (at 8 G it
// was split in two, and the pipelined rate fell below the kernel-only one).
constexpr uint64_t kMaxBatchEntries = 12ull << 30;
constexpr int kMaxBatchImages = 65535;
int batch_split(jd_ctx* ctx, int lo, int n, const jd_item* items) {
    const uint64_t limit = ctx->max_batch_entries;
    uint64_t cap = 0;
    int hi = lo;
    for (; hi < n; hi++) {
        if (hi - lo >= ctx->max_batch_images) break;
        if (ctx->pst[hi] != JD_OK) continue;
        const jd_header& h = ctx->parsed[hi].hdr;
        // (at async depth 2 a batch with host inputs is planned with worst-case pools: launch_batch)
        const RegionSizing rs = region_sizing(ctx->parsed[hi], ctx->worst || ctx->worst_always || ctx->async_depth == 2);
        const uint64_t w = entry_words(items[hi].len - h.ecs_offset, image_segments(h), kPieceBits, -1, rs.div, rs.slack);
        if (hi > lo && cap + w > limit) break;
        cap += w;
    }
    return hi;
}

jd_status build_plan(jd_ctx* ctx, const jd_item* items, int lo, int hi, const std::vector<uint64_t>& dev_addr,
                     const std::vector<uint64_t>& out_addr, bool worst, Plan& P) {
    const auto tb0 = std::chrono::steady_clock::now();
    auto tbms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count(); };
    // 1. sequential: table sets and quant tables (de-duplicated across the batch), bases
    std::map<std::array<int, 7>, int> ts_index;
    std::map<std::array<uint16_t, 64>, int> q_index;
    std::vector<PlanImg> pim;
    pim.reserve(size_t(hi - lo));
    // images of one encoder repeat their tables: the previous image's lookups are tried first
    const ParsedJpeg* prev = nullptr;
    int prev_ts = -1;
    uint16_t prev_qslot[3] = {0, 0, 0};
    uint64_t block_cursor = 0, comp_cursor = 0;
    uint32_t seg_cursor = 0, chunk_cursor = 0;
    for (int it = lo; it < hi; it++) {
        if (ctx->pst[it] != JD_OK) continue;
        const ParsedJpeg& pj = ctx->parsed[it];
        const jd_header& h = pj.hdr;
        // jd_plan.hpp kMaxImageEntryWords, at the shortest pieces a batch holding it can get
        const uint64_t ecs_img = items[it].len - h.ecs_offset;
        const uint32_t pmin = (ctx->flags & JD_FLAG_FORCE_SYNC)    ? 1024u
                              : (ctx->flags & JD_FLAG_FORCE_LANES) ? 0x40000000u
                              : (ctx->flags & JD_FLAG_FULL_PIECES) ? kPieceBits
                                                                   : adaptive_piece_bits(ecs_img * 8, ctx->min_piece_bits);
        const bool forced = (ctx->flags & (JD_FLAG_FORCE_SYNC | JD_FLAG_FORCE_LANES | JD_FLAG_FULL_PIECES)) != 0;
        // (the worst-case plan must fit: an optimistic one may be retried with it)
        const RegionSizing rs = region_sizing(pj, true);
        if (!image_fits(ecs_img, h, pmin, forced ? pmin : kPieceBits, ctx->spare_pieces, rs.div, rs.slack)) {
            ctx->pst[it] = JD_ERR_CAPACITY;
            continue;
        }
        bool same_tables = prev && prev->hdr.ncomp == h.ncomp;
        for (int c = 0; same_tables && c < h.ncomp; c++) {
            const HuffSpec &d0 = pj.dc[pj.td[c]], &d1 = prev->dc[prev->td[c]];
            const HuffSpec &a0 = pj.ac[pj.ta[c]], &a1 = prev->ac[prev->ta[c]];
            same_tables = pj.hdc[c] == prev->hdc[c] && pj.hac[c] == prev->hac[c] && d0.nvals == d1.nvals &&
                          a0.nvals == a1.nvals && !memcmp(d0.counts, d1.counts, 17) && !memcmp(a0.counts, a1.counts, 17) &&
                          !memcmp(d0.vals, d1.vals, d0.nvals) && !memcmp(a0.vals, a1.vals, a0.nvals);
        }
        int ts = same_tables ? prev_ts : -1;
        if (ts < 0) {
            std::array<int, 7> key{};
            key[0] = h.ncomp;
            bool ok = true;
            for (int c = 0; c < h.ncomp; c++) {
                key[1 + c] = lut_id(ctx, pj.dc[pj.td[c]], true, pj.hdc[c]);
                key[4 + c] = lut_id(ctx, pj.ac[pj.ta[c]], false, pj.hac[c]);
                if (key[1 + c] < 0 || key[4 + c] < 0) ok = false;
            }
            if (!ok) {
                ctx->pst[it] = JD_ERR_CORRUPT;
                continue;
            }
            auto f = ts_index.find(key);
            if (f != ts_index.end()) {
                ts = f->second;
            } else {
                TableSet t;
                for (int s = 0; s < kSlotsPerSet; s++) t.lut[s] = -1;
                memset(t.dc_slot, 0, sizeof(t.dc_slot));
                memset(t.ac_slot, 0, sizeof(t.ac_slot));
                int nslot = 0;
                auto slot_of = [&](int id) {
                    for (int s = 0; s < nslot; s++)
                        if (t.lut[s] == id) return s;
                    t.lut[nslot] = id;
                    return nslot++;
                };
                for (int c = 0; c < h.ncomp; c++) {
                    t.dc_slot[c] = uint8_t(slot_of(key[1 + c]));
                    t.ac_slot[c] = uint8_t(slot_of(key[4 + c]));
                }
                t.nslots = nslot;
                P.max_slots = std::max(P.max_slots, uint32_t(nslot));
                ts = int(P.tablesets.size());
                P.tablesets.push_back(t);
                ts_index.emplace(key, ts);
            }
        }
        PlanImg pi;
        pi.item = it;
        pi.ts = ts;
        for (int c = 0; c < h.ncomp; c++) {
            if (prev && c < prev->hdr.ncomp && !memcmp(pj.q[h.tq[c]], prev->q[prev->hdr.tq[c]], 128)) {
                pi.qslot[c] = prev_qslot[c];
                continue;
            }
            std::array<uint16_t, 64> q;
            memcpy(q.data(), pj.q[h.tq[c]], sizeof(q));
            auto fq = q_index.find(q);
            int qi;
            if (fq == q_index.end()) {
                qi = int(P.qtabs.size() / 64);
                P.qtabs.insert(P.qtabs.end(), q.begin(), q.end());
                q_index.emplace(q, qi);
            } else {
                qi = fq->second;
            }
            pi.qslot[c] = uint16_t(qi);
        }
        for (int c = 0; c < h.ncomp && c < 3; c++) prev_qslot[c] = pi.qslot[c];
        prev = &pj;
        prev_ts = ts;
        const uint64_t nmcu = uint64_t(h.mcux) * h.mcuy;
        pi.nseg = image_segments(h);
        pi.seg_base = seg_cursor;
        seg_cursor += pi.nseg;
        pi.block_base = block_cursor;
        block_cursor += nmcu * uint64_t(h.blocks_per_mcu);
        const uint64_t a0 = (dev_addr[it] + uint64_t(h.ecs_offset)) & ~uint64_t(15);
        pi.nchunks = uint32_t((dev_addr[it] + items[it].len - a0 + kScanChunk - 1) / kScanChunk);
        pi.chunk_base = chunk_cursor;
        chunk_cursor += pi.nchunks;
        pi.comp = comp_cursor;
        comp_cursor += align_up(size_t(items[it].len - h.ecs_offset) + 64, 256);
        P.max_chunks = std::max(P.max_chunks, pi.nchunks);
        P.pixels += double(h.width) * h.height;
        P.ecs_bytes += double(items[it].len - h.ecs_offset);
        pim.push_back(pi);
    }
    P.total_blocks = block_cursor;
    P.total_chunks = chunk_cursor;
    P.comp_bytes = comp_cursor;
    const double tb_imgs = tbms();
    // 2. parallel: image descriptors and segment lists
    const size_t nimg = pim.size();
    P.imgs.resize(nimg);
    P.item_of_img.resize(nimg);
    P.seg_img.resize(seg_cursor);
    constexpr int kPer = 32;
    ctx->pool->run(int((nimg + kPer - 1) / kPer), [&](int t) {
        for (size_t i = size_t(t) * kPer; i < std::min(nimg, size_t(t + 1) * kPer); i++) {
            const PlanImg& pi = pim[i];
            const ParsedJpeg& pj = ctx->parsed[pi.item];
            ImgDesc& d = P.imgs[i];
            fill_desc(pj, items[pi.item], dev_addr[pi.item], out_addr[pi.item], pi, d, worst);
            P.item_of_img[i] = pi.item;
            for (uint32_t k = 0; k < d.nseg; k++) P.seg_img[d.seg_base + k] = uint32_t(i);
        }
    });
    std::vector<uint32_t> by_mode[4];
    for (size_t i = 0; i < P.imgs.size(); i++) {
        ImgDesc& d = P.imgs[i];
        d.tile_base = P.total_tiles;
        P.total_tiles += d.tiles_x * d.tiles_y;
        P.max_tiles = std::max(P.max_tiles, d.tiles_x * d.tiles_y);
        const uint32_t m = image_mode(d);
        by_mode[m].push_back(uint32_t(i));
        P.mode_max_tiles[m] = std::max(P.mode_max_tiles[m], d.tiles_x * d.tiles_y);
    }
    for (int m = 0; m < 4; m++) {
        P.mode_off[m] = uint32_t(P.mode_imgs.size());
        P.mode_cnt[m] = uint32_t(by_mode[m].size());
        P.mode_imgs.insert(P.mode_imgs.end(), by_mode[m].begin(), by_mode[m].end());
    }
    const double tb_segs = tbms();
    // 3. piece slots: per image ceil(ECS bits / piece_bits) + nseg (interval lengths are only known
    // on the GPU), grouped by table set so each k_piece workgroup stages one table set
    std::vector<uint32_t> order(nimg);
    for (size_t i = 0; i < order.size(); i++) order[i] = uint32_t(i);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return pim[a].ts < pim[b].ts; });
    // Piece size: kPieceBits for full batches; a small batch (one image, a few) gets shorter pieces
    // so it still spreads over ~kPieceTarget lanes — a lane walks piece_bits + overlap bits, so
    // single-image latency falls with the piece size while the overlap (sync distance) is fixed.
    uint64_t ecs_bits = 0;
    for (const ImgDesc& d : P.imgs) ecs_bits += uint64_t(d.len - d.ecs_off) * 8;
    const uint32_t adaptive = (ctx->flags & JD_FLAG_FULL_PIECES) ? kPieceBits : adaptive_piece_bits(ecs_bits, ctx->min_piece_bits);
    P.piece_bits = (ctx->flags & JD_FLAG_FORCE_SYNC) ? 1024u : (ctx->flags & JD_FLAG_FORCE_LANES) ? 0x40000000u : adaptive;
    // shorter pieces also get a shorter warm-up: a lane that has not synchronised by then is
    // re-walked (k_redo / k_chain_big), which costs less than every lane walking 4096 extra bits.
    // Three pieces' worth: on the reference's single-image sizes (4:4:4 q95, 200^2 .. 2000^2) as fast
    // as two at 200^2 and 10 % faster at 2000^2 (fewer failed starts for k_chain_big's rounds); four
    // were slower on small images (profiles/r05v_*)
    P.piece_overlap = (ctx->flags & (JD_FLAG_FORCE_SYNC | JD_FLAG_FORCE_LANES)) ? kPieceOverlap
                                                                             : std::min(kPieceOverlap, 3 * adaptive);
    if (ctx->piece_overlap >= 0) P.piece_overlap = uint32_t(ctx->piece_overlap);
    uint64_t sub = 0, entry_cursor = 0;
    P.chain_seg.reserve(seg_cursor + kPieceThreads * P.tablesets.size());
    P.ts_slot0.assign(P.tablesets.size(), 0u);
    P.img_order = order;
    for (size_t oi = 0; oi < order.size();) {
        const int ts = pim[order[oi]].ts;
        P.ts_slot0[ts] = uint32_t(sub);
        for (; oi < order.size() && pim[order[oi]].ts == ts; oi++) {
            ImgDesc& d = P.imgs[order[oi]];
            d.sub_base = uint32_t(sub);
            d.sub_cap = uint32_t(piece_slots(d.len - d.ecs_off, d.nseg, P.piece_bits));
            d.entry_base = entry_cursor;
            const uint64_t words = entry_words(d.len - d.ecs_off, d.nseg, P.piece_bits, ctx->spare_pieces, d.rw_div, d.rw_slack);
            if (words > kMaxImageEntryWords) return JD_ERR_CAPACITY;  // image_fits checked every piece size
            d.entry_cap = uint32_t(words);
            entry_cursor += align_up(size_t(d.entry_cap), kRegionAlign);
            sub += d.sub_cap;
            for (uint32_t k = 0; k < d.nseg; k++) P.chain_seg.push_back(d.seg_base + k);
        }
        sub = align_up(sub, kPieceThreads);
        while (P.wg_tableset.size() < sub / kPieceThreads) P.wg_tableset.push_back(uint32_t(ts));
        while (P.chain_seg.size() % kPieceThreads) P.chain_seg.push_back(kInvalidImage);
        while (P.chain_wg_tableset.size() < P.chain_seg.size() / kPieceThreads) P.chain_wg_tableset.push_back(uint32_t(ts));
    }
    if (ctx->host_timing) std::fprintf(stderr, "plan imgs %.3f descs %.3f pieces %.3f ms\n", tb_imgs, tb_segs - tb_imgs, tbms() - tb_segs);
    if (sub > 0x7FFFFFFFull) return JD_ERR_CAPACITY;
    P.nsub = uint32_t(sub);

    P.total_entry_cap = entry_cursor;
    // break slots per scan chunk: every RSTn and the EOI of a valid stream fit in the batch's most
    // intervals + kBrkSlack (k_index flags a chunk before the ECS end that held more)
    uint32_t most_seg = 0;
    for (const ImgDesc& d : P.imgs) most_seg = std::max(most_seg, d.nseg);
    P.brk_cap = worst ? uint32_t(kScanCap) : std::min<uint32_t>(kScanCap, most_seg + kBrkSlack);
    if (!worst && ctx->brk_cap_force) P.brk_cap = std::min<uint32_t>(P.brk_cap, ctx->brk_cap_force);
    return JD_OK;
}

template <typename T>
size_t put(std::vector<uint8_t>& blob, const std::vector<T>& v) {
    const size_t off = align_up(blob.size(), 256);
    blob.resize(off + std::max<size_t>(v.size() * sizeof(T), 16));
    if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

// Device-only scratch laid out after the uploaded part: only the offset advances (no host bytes).
size_t reserve(size_t& end, size_t bytes) {
    const size_t off = align_up(end, 256);
    end = off + std::max<size_t>(bytes, 16);
    return off;
}

jd_status finish_batch(jd_ctx* ctx, Pending& pd);
jd_status run_retries(jd_ctx* ctx, void* hip_stream);

// Grow-only pinned buffer of a pending slot (the slot is idle when this is called).
hipError_t ensure_pinned(void*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    const size_t n = std::max(bytes, cap + cap / 2);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
    if (e == hipSuccess) cap = n;
    return e;
}

// Parses nothing (parse_all did), plans items [lo, hi), uploads the plan and launches every kernel
// on stream s into the context's current pending slot, which it leaves active; finish_batch
// collects it.
// The registered range holding address a (index into host_regs), or -1.
int reg_range(const jd_ctx* ctx, uintptr_t a) {
    const auto& r = ctx->host_regs;
    auto it = std::upper_bound(r.begin(), r.end(), a, [](uintptr_t x, const std::pair<uintptr_t, uintptr_t>& y) { return x < y.first; });
    if (it == r.begin()) return -1;
    --it;
    return a < it->second ? int(it - r.begin()) : -1;
}
// Whether [p, p + n) lies in one registered range.
bool host_registered(const jd_ctx* ctx, const uint8_t* p, size_t n) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const int k = reg_range(ctx, a);
    return k >= 0 && n <= ctx->host_regs[size_t(k)].second - a;
}

jd_status launch_batch(jd_ctx* ctx, const jd_item* items, int lo, int hi, jd_result* results, int rgb_on_device,
                       hipStream_t s) {
    Slot& sl = ctx->slots[ctx->slot];
    Pending& pd = ctx->pend[ctx->seq % kNumPending];
    if (pd.active) {  // (the async depth keeps fewer batches in flight: normally collected already)
        jd_status fst = finish_batch(ctx, pd);
        if (fst == JD_OK) fst = run_retries(ctx, s);  // (before this launch reuses a slot)
        if (fst != JD_OK) return fst;
    }
    // The slot's previous batch (launched two calls ago) may still run: its device scratch is
    // reused in stream order; its pinned staging only once its copies are done (below).
    // An error return after the host inputs' H2D copies were queued (plan capacity, a HIP failure)
    // leaves the slot inactive, so nothing else would wait for them: wait here, before the staging
    // buffers can be refilled or freed by a later call.
    struct StagingGuard {
        hipStream_t s = nullptr;
        ~StagingGuard() {
            if (s) (void)hipStreamSynchronize(s);
        }
    } staging;
    // 1. inputs and outputs on the device
    std::vector<uint64_t> dev_addr(size_t(hi), 0), out_addr(size_t(hi), 0);
    // Host-memory inputs in a registered range (jd_host_register) are uploaded straight from it,
    // in spans of neighbouring files (one DMA per span); the others are staged (below).
    std::vector<int> reg_items;
    std::vector<char> registered(size_t(hi), 0);
    if (!ctx->host_regs.empty())
        for (int i = lo; i < hi; i++)
            if (ctx->pst[i] == JD_OK && !items[i].jpeg_dev && host_registered(ctx, items[i].jpeg, items[i].len)) {
                registered[size_t(i)] = 1;
                reg_items.push_back(i);
            }
    struct Span { uintptr_t lo, hi; size_t off; };
    std::vector<Span> spans;
    size_t in_bytes = 0, reg_bytes = 0, out_bytes = 0;
    if (!reg_items.empty()) {
        std::sort(reg_items.begin(), reg_items.end(), [&](int a, int b) { return items[a].jpeg < items[b].jpeg; });
        // A gap between neighbouring files is copied along only while it is small against the span
        // (at most 4 KiB, or an eighth of the span so far): sparse files in a large arena move their
        // own bytes, not the arena's.
        constexpr uintptr_t kSpanGap = uintptr_t(4) << 10;
        for (int i : reg_items) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(items[i].jpeg), e = a + items[i].len;
            const bool merge = !spans.empty() && reg_range(ctx, a) == reg_range(ctx, spans.back().lo) &&
                               (a <= spans.back().hi + std::max(kSpanGap, (spans.back().hi - spans.back().lo) / 8));
            if (!merge)
                spans.push_back({a, e, 0});
            else
                spans.back().hi = std::max(spans.back().hi, e);
        }
    }
    for (int i = lo; i < hi; i++) {
        if (ctx->pst[i] != JD_OK) continue;
        if (!items[i].jpeg_dev && !registered[size_t(i)]) in_bytes += align_up(items[i].len + 64, 256);
        if (!rgb_on_device) out_bytes += align_up(size_t(ctx->parsed[i].hdr.width) * ctx->parsed[i].hdr.height * 3, 256);
    }
    for (Span& sp : spans) {  // after the staged inputs in the slot's device input pool
        sp.off = in_bytes + reg_bytes;
        reg_bytes += align_up(size_t(sp.hi - sp.lo) + 64, 256);
    }
    if (in_bytes + reg_bytes) HIPCHK(ctx, ensure_dev(ctx, sl.d_input, in_bytes + reg_bytes));
    if (in_bytes + reg_bytes && ctx->h2d_serial && ctx->last_h2d && ctx->last_h2d != sl.h2d_done)
        HIPCHK(ctx, hipStreamWaitEvent(s, ctx->last_h2d, 0));
    if (reg_bytes) {
        uint8_t* const dbase = static_cast<uint8_t*>(sl.d_input.p);
        for (const Span& sp : spans)  // (in JD_STAGE_CHUNK_MB pieces, as the staged copies)
            for (uintptr_t c = sp.lo; c < sp.hi; c += std::min<uintptr_t>(ctx->stage_chunk, sp.hi - c)) {
                staging.s = s;
                HIPCHK(ctx, hipMemcpyAsync(dbase + sp.off + (c - sp.lo), reinterpret_cast<const void*>(c),
                                           std::min<uintptr_t>(ctx->stage_chunk, sp.hi - c), hipMemcpyHostToDevice, s));
            }
        size_t k = 0;  // reg_items ascend by address, as the spans do
        for (int i : reg_items) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(items[i].jpeg);
            while (a >= spans[k].hi) k++;
            dev_addr[i] = reinterpret_cast<uint64_t>(dbase) + spans[k].off + (a - spans[k].lo);
        }
        ctx->stats.h2d_bytes += double(reg_bytes);  // what moves (spans, gaps included)
        for (int i : reg_items) ctx->stats.h2d_registered_bytes += double(items[i].len);  // the files' own bytes
    }
    if (in_bytes) {
        // Host-memory inputs: copied into this slot's pinned staging by the host workers in
        // parallel (pieces of at most 1 MiB), chunk by chunk; each chunk's H2D is issued on the
        // slot's stream as soon as it is staged, so the DMA of chunk c overlaps the copy of chunk
        // c + 1, and both overlap the other slot's kernels.  The slot is idle
        // here (collected above).
        Range r("jd_stage_inputs");
        const auto ts0 = std::chrono::steady_clock::now();
        if (sl.h2d_recorded) HIPCHK(ctx, hipEventSynchronize(sl.h2d_done));  // the slot's last DMA read it
        HIPCHK(ctx, ensure_pinned(sl.in_host, sl.in_cap, in_bytes));
        struct Piece { const uint8_t* src; size_t off, n; };
        std::vector<Piece> pieces;
        constexpr size_t kStagePiece = size_t(1) << 20;
        size_t off = 0;
        for (int i = lo; i < hi; i++) {
            if (ctx->pst[i] != JD_OK || items[i].jpeg_dev || registered[size_t(i)]) continue;
            for (size_t k = 0; k < items[i].len; k += kStagePiece)
                pieces.push_back({items[i].jpeg + k, off + k, std::min(kStagePiece, items[i].len - k)});
            dev_addr[i] = reinterpret_cast<uint64_t>(sl.d_input.p) + off;
            off += align_up(items[i].len + 64, 256);
        }
        uint8_t* const stage = static_cast<uint8_t*>(sl.in_host);
        uint8_t* const dstage = static_cast<uint8_t*>(sl.d_input.p);
        const size_t kStageChunk = ctx->stage_chunk;  // H2D granularity (JD_STAGE_CHUNK_MB)
        for (size_t p0 = 0; p0 < pieces.size();) {
            size_t p1 = p0 + 1;
            while (p1 < pieces.size() && pieces[p1].off + pieces[p1].n - pieces[p0].off <= kStageChunk) p1++;
            ctx->pool->run(int(p1 - p0), [&](int k) {
                const Piece& q = pieces[p0 + size_t(k)];
                if (ctx->stage_nt) stage_copy(stage + q.off, q.src, q.n);
                else memcpy(stage + q.off, q.src, q.n);
            });
            const size_t c0 = pieces[p0].off, c1 = (p1 < pieces.size()) ? pieces[p1].off : in_bytes;
            staging.s = s;
            HIPCHK(ctx, hipMemcpyAsync(dstage + c0, stage + c0, c1 - c0, hipMemcpyHostToDevice, s));
            p0 = p1;
        }
        ctx->stats.host_ms[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
        ctx->stats.h2d_bytes += double(in_bytes);
    }
    if (in_bytes + reg_bytes) {
        HIPCHK(ctx, hipEventRecord(sl.h2d_done, s));
        sl.h2d_recorded = true;
        if (ctx->h2d_serial) ctx->last_h2d = sl.h2d_done;
    }
    for (int i = lo; i < hi; i++)
        if (ctx->pst[i] == JD_OK && items[i].jpeg_dev) dev_addr[i] = reinterpret_cast<uint64_t>(items[i].jpeg_dev);
    if (out_bytes) HIPCHK(ctx, ensure_dev(ctx, ctx->output, out_bytes));
    {
        size_t off = 0;
        for (int i = lo; i < hi; i++) {
            if (ctx->pst[i] != JD_OK) continue;
            if (rgb_on_device) {
                out_addr[i] = reinterpret_cast<uint64_t>(items[i].rgb);
            } else {
                out_addr[i] = reinterpret_cast<uint64_t>(ctx->output.p) + off;
                off += align_up(size_t(ctx->parsed[i].hdr.width) * ctx->parsed[i].hdr.height * 3, 256);
            }
        }
    }

    // 2. plan
    std::unique_ptr<Range> rng(new Range("jd_plan"));
    const auto tp0 = std::chrono::steady_clock::now();
    auto tms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count(); };
    // Optimistic pools unless this is a retry (or the caller asked for worst-case pools), or a batch
    // with host inputs at async depth 2: the slot's copy of them may be replaced by its next launch
    // before this batch is collected, and a retry would have nothing to read.
    const bool worst = ctx->worst || ctx->worst_always || (ctx->async_depth == 2 && in_bytes + reg_bytes > 0);
    Plan P;
    jd_status st = build_plan(ctx, items, lo, hi, dev_addr, out_addr, worst, P);
    const double t_plan = tms();
    if (st != JD_OK) return st;
    st = sync_luts(ctx);
    if (st != JD_OK) return st;
    const uint32_t nimg = uint32_t(P.imgs.size());
    if (nimg) {
        HIPCHK(ctx, ensure_dev(ctx, sl.d_comp, std::max<size_t>(16, P.comp_bytes)));
        for (ImgDesc& d : P.imgs) d.comp += reinterpret_cast<uint64_t>(sl.d_comp.p);
        const bool fancy = (ctx->flags & JD_FLAG_FANCY_UPSAMPLING) != 0;
        uint32_t max_fancy_wgs = 0;
        if (fancy) {  // int16 component planes over the padded MCU grid, 256-B aligned per image
            std::vector<size_t> poff(P.imgs.size());
            size_t tot = 0;
            for (size_t i = 0; i < P.imgs.size(); i++) {
                const ImgDesc& d = P.imgs[i];
                size_t n = 0;
                for (uint32_t c = 0; c < d.ncomp; c++) n += size_t(d.mcux * d.h[c] * 8) * (d.mcuy * d.v[c] * 8) * 2;
                poff[i] = tot;
                tot += align_up(n, 256);
                // k_colour_fancy's grid: kFancyW x kFancyRowsPerWg-pixel workgroups (kFancyBands bands
                // of kFancyH rows; x in the low 16 bits, y in the high)
                max_fancy_wgs = std::max<uint32_t>(max_fancy_wgs & 0xFFFFu, (d.width + kFancyW - 1) / kFancyW) |
                                (std::max<uint32_t>(max_fancy_wgs >> 16, (d.height + kFancyRowsPerWg - 1) / kFancyRowsPerWg) << 16);
            }
            HIPCHK(ctx, ensure_dev(ctx, sl.d_planes, std::max<size_t>(16, tot)));
            for (size_t i = 0; i < P.imgs.size(); i++)
                P.imgs[i].planes = reinterpret_cast<uint64_t>(sl.d_planes.p) + poff[i];
        }
        std::vector<uint8_t> blob;
        const size_t nseg = P.seg_img.size();
        const size_t nsub = P.nsub;
        // every table set's LUTs once more, contiguous per set: k_redo looks them up in global
        // memory (so its small workgroups need no LDS for tables)
        std::vector<HuffLut> set_luts;
        for (TableSet& t : P.tablesets) {
            t.set_lut0 = int32_t(set_luts.size());
            for (int k = 0; k < t.nslots; k++) set_luts.push_back(ctx->lut_host[size_t(t.lut[k])]);
        }
        const size_t o_imgs = put(blob, P.imgs);
        const size_t o_ts = put(blob, P.tablesets);
        const size_t o_setluts = put(blob, set_luts);
        const size_t o_q = put(blob, P.qtabs);
        const size_t o_segimg = put(blob, P.seg_img);
        const size_t o_wgts = put(blob, P.wg_tableset);
        const size_t o_chain = put(blob, P.chain_seg);
        const size_t o_chts = put(blob, P.chain_wg_tableset);
        const size_t o_modes = put(blob, P.mode_imgs);
        const size_t o_status = put(blob, std::vector<uint32_t>(nimg, 0));
        const size_t o_ctr = put(blob, std::vector<unsigned long long>(kNumCounters, 0));  // BatchDev::counters
        const size_t o_tscur = put(blob, P.ts_slot0);
        const size_t o_order = put(blob, P.img_order);
        const size_t upload = blob.size();
        // device-written scratch after the uploaded part (no initialisation needed)
        size_t end = upload;
        const size_t o_cstart = reserve(end, nseg * 4);
        const size_t o_cend = reserve(end, nseg * 4);
        const size_t o_nbrk = reserve(end, size_t(P.total_chunks) * 4);
        const size_t o_drops = reserve(end, size_t(P.total_chunks) * 4);
        const size_t o_coff = reserve(end, size_t(P.total_chunks) * 4);
        const size_t o_ssb = reserve(end, nseg * 4);
        const size_t o_sns = reserve(end, nseg * 4);
        const size_t o_subseg = reserve(end, nsub * 4);
        const size_t o_segent = reserve(end, nseg * 4);
        const size_t o_pool = reserve(end, size_t(nimg) * 8);
        const size_t o_cand = reserve(end, size_t(nimg) * 16 * 4);
        const size_t o_ibase = reserve(end, size_t(nimg) * 4);
        size_t o_piece[9];
        for (int q = 0; q < 9; q++) o_piece[q] = reserve(end, nsub * 4);
        const size_t o_cp = reserve(end, nsub * kCpRecords * sizeof(CpRec));
        const size_t o_fix = reserve(end, nseg * 4);
        const size_t o_tdc = reserve(end, size_t(P.total_tiles) * sizeof(DcPred));
        const size_t o_slow = reserve(end, size_t(P.total_tiles) * 8);
        HIPCHK(ctx, ensure_dev(ctx, sl.d_plan, end));
        if (sl.plan_recorded) HIPCHK(ctx, hipEventSynchronize(sl.plan_done));  // the slot's last plan upload
        HIPCHK(ctx, ensure_pinned(sl.plan_host, sl.plan_cap, upload));
        memcpy(sl.plan_host, blob.data(), upload);
        HIPCHK(ctx, hipMemcpyAsync(sl.d_plan.p, sl.plan_host, upload, hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipEventRecord(sl.plan_done, s));
        sl.plan_recorded = true;
        HIPCHK(ctx, ensure_dev(ctx, sl.d_brk, std::max<size_t>(16, size_t(P.total_chunks) * P.brk_cap * sizeof(Break))));
        HIPCHK(ctx, ensure_dev(ctx, sl.d_blocks, std::max<size_t>(16, P.total_blocks * sizeof(BlockInfo))));
        HIPCHK(ctx, ensure_dev(ctx, sl.d_entries, P.total_entry_cap * 4 + 64));  // +64: 16-byte over-reads

        uint8_t* base = static_cast<uint8_t*>(sl.d_plan.p);
        BatchDev b;
        memset(&b, 0, sizeof(b));
        b.imgs = reinterpret_cast<const ImgDesc*>(base + o_imgs);
        b.nimg = nimg;
        b.luts = static_cast<const HuffLut*>(ctx->lut_dev.p);
        b.tablesets = reinterpret_cast<const TableSet*>(base + o_ts);
        b.set_luts = reinterpret_cast<const HuffLut*>(base + o_setluts);
        b.qtabs = reinterpret_cast<const uint16_t*>(base + o_q);
        b.seg_img = reinterpret_cast<const uint32_t*>(base + o_segimg);
        b.seg_cstart = reinterpret_cast<uint32_t*>(base + o_cstart);
        b.seg_cend = reinterpret_cast<uint32_t*>(base + o_cend);
        b.seg_ent = reinterpret_cast<uint32_t*>(base + o_segent);
        b.img_pool = reinterpret_cast<unsigned long long*>(base + o_pool);
        b.nseg = uint32_t(nseg);
        b.seg_sub_base = reinterpret_cast<uint32_t*>(base + o_ssb);
        b.seg_nsub = reinterpret_cast<uint32_t*>(base + o_sns);
        b.sub_seg = reinterpret_cast<uint32_t*>(base + o_subseg);
        b.nsub = uint32_t(nsub);
        b.wg_tableset = reinterpret_cast<const uint32_t*>(base + o_wgts);
        b.ts_cursor = reinterpret_cast<uint32_t*>(base + o_tscur);
        b.img_order = reinterpret_cast<const uint32_t*>(base + o_order);
        b.img_cand = reinterpret_cast<uint32_t*>(base + o_cand);
        b.img_base = reinterpret_cast<uint32_t*>(base + o_ibase);
        b.chain_seg = reinterpret_cast<const uint32_t*>(base + o_chain);
        b.nchain = uint32_t(P.chain_seg.size());
        b.chain_wg_tableset = reinterpret_cast<const uint32_t*>(base + o_chts);
        b.piece_bits = P.piece_bits;
        // large batches: k_pieceplan picks the piece size (>= piece_bits) that fits the pieces to
        // whole rounds of k_piece's resident lanes
        b.piece_plan = (P.piece_bits == kPieceBits && !(ctx->flags & (JD_FLAG_FORCE_SYNC | JD_FLAG_FORCE_LANES)) &&
                        !ctx->fixed_pieces) ? piece_lanes_resident(huffman_lds_bytes(P.max_slots)) : 0u;
        b.no_pool = ctx->spare_pieces == 0 ? 1u : 0u;
        b.small_fold = (b.piece_plan == 0 && P.total_chunks > 0 && nimg <= kSmallFoldImages) ? 1u : 0u;
        if (!b.piece_plan) {  // small batches only (a large batch keeps k_chain_fix and its small footprint
                              // beside the other batch's kernels): an interval holds at most its image's
                              // ECS bits, in pieces of at least P.piece_bits
            uint64_t most = 0;
            for (const ImgDesc& d : P.imgs) most = std::max<uint64_t>(most, (uint64_t(d.len - d.ecs_off) * 8 + P.piece_bits - 1) / P.piece_bits);
            b.big_chain = most > kBigInterval ? 1u : 0u;
        }
        b.piece_overlap = P.piece_overlap;
        uint32_t* pc[9];
        for (int q = 0; q < 9; q++) pc[q] = reinterpret_cast<uint32_t*>(base + o_piece[q]);
        b.piece_bit = pc[0];
        b.piece_end = pc[1];
        b.piece_nmcu = pc[2];
        b.piece_nent = pc[3];
        b.piece_mcu0 = pc[4];
        b.piece_emcu = pc[5];
        b.piece_abase = pc[6];
        b.piece_amcu = pc[7];
        b.piece_join = pc[8];
        b.piece_cp = reinterpret_cast<CpRec*>(base + o_cp);
        b.seg_fix = reinterpret_cast<uint32_t*>(base + o_fix);
        b.tile_dc = reinterpret_cast<DcPred*>(base + o_tdc);
        b.slow_tiles = reinterpret_cast<TileRef*>(base + o_slow);
        b.total_tiles = P.total_tiles;
        b.max_slots = P.max_slots;
        b.max_chunks = P.max_chunks;
        b.chunk_nbrk = reinterpret_cast<uint32_t*>(base + o_nbrk);
        b.chunk_drops = reinterpret_cast<uint32_t*>(base + o_drops);
        b.chunk_coff = reinterpret_cast<uint32_t*>(base + o_coff);
        b.chunk_brk = static_cast<Break*>(sl.d_brk.p);
        b.brk_cap = P.brk_cap;
        b.blocks = static_cast<BlockInfo*>(sl.d_blocks.p);
        b.entries = static_cast<uint32_t*>(sl.d_entries.p);
        b.entries_cap = (sl.d_entries.cap - 64) / 4;  // last 64 B: padding for 16-byte over-reads
        b.status = reinterpret_cast<uint32_t*>(base + o_status);
        b.counters = reinterpret_cast<unsigned long long*>(base + o_ctr);
        b.max_tiles = P.max_tiles;
        b.mode_imgs = reinterpret_cast<const uint32_t*>(base + o_modes);
        for (int m = 0; m < 4; m++) {
            b.mode_off[m] = P.mode_off[m];
            b.mode_cnt[m] = P.mode_cnt[m];
            b.mode_max_tiles[m] = P.mode_max_tiles[m];
        }
        if (std::getenv("JD_STAMPS")) {  // diagnostic builds (JD_STAMP): per-tile phase stamps
            HIPCHK(ctx, ensure_dev(ctx, sl.d_stamps, size_t(P.total_tiles) * 64));
            HIPCHK(ctx, hipMemsetAsync(sl.d_stamps.p, 0, size_t(P.total_tiles) * 64, s));
            b.stamps = static_cast<unsigned long long*>(sl.d_stamps.p);
        }
        b.fancy = fancy ? 1u : 0u;
        b.max_fancy_wgs = max_fancy_wgs;
        if (const char* e = std::getenv("JD_FIX_ROUND_CAP")) b.fix_round_cap = uint32_t(std::strtoul(e, nullptr, 0));
        b.skip_redo = std::getenv("JD_SKIP_REDO") ? 1u : 0u;

        ctx->last = b;
        ctx->last_blocks = P.total_blocks;
        ctx->last_entries = P.total_entry_cap;
        ctx->last_entry_base.resize(P.imgs.size());
        ctx->last_rw_div.resize(P.imgs.size());
        ctx->last_rw_slack.resize(P.imgs.size());
        for (size_t i = 0; i < P.imgs.size(); i++) {
            ctx->last_entry_base[i] = P.imgs[i].entry_base;
            ctx->last_rw_div[i] = P.imgs[i].rw_div;
            ctx->last_rw_slack[i] = P.imgs[i].rw_slack;
        }
        const bool timing = (ctx->flags & JD_FLAG_TIMING) != 0;
        const double t_upload = tms();
        rng.reset(new Range("jd_launch"));
        double t_k[JD_NUM_KERNELS];
        const bool split = sl.istream != nullptr && s == sl.stream;  // (a caller stream orders everything)
        for (int k = 0; k < JD_NUM_KERNELS; k++) {
            hipStream_t ks = s;
            if (split && k >= kIdctSlot) {
                if (k == kIdctSlot) {
                    HIPCHK(ctx, hipEventRecord(sl.ev_tail, s));
                    HIPCHK(ctx, hipStreamWaitEvent(sl.istream, sl.ev_tail, 0));
                }
                ks = sl.istream;
            }
            if (timing) HIPCHK(ctx, hipEventRecord(pd.ev[k][0], ks));
            HIPCHK(ctx, launch_kernel(k, b, ks));
            if (timing) HIPCHK(ctx, hipEventRecord(pd.ev[k][1], ks));
            t_k[k] = tms();
        }
        if (split) {  // the slot's later work (status readback, the next batch) after the colour stage
            HIPCHK(ctx, hipEventRecord(sl.ev_idct, sl.istream));
            HIPCHK(ctx, hipStreamWaitEvent(s, sl.ev_idct, 0));
        }
        if (ctx->host_timing) {
            std::fprintf(stderr, "host launch returns:");
            for (int k = 0; k < JD_NUM_KERNELS; k++) std::fprintf(stderr, " %.3f", t_k[k]);
            std::fprintf(stderr, "\n");
        }
        constexpr size_t kCtrBytes = kNumCounters * 8;
        HIPCHK(ctx, ensure_pinned(pd.host, pd.host_cap, kCtrBytes + size_t(nimg) * 4));
        HIPCHK(ctx, hipMemcpyAsync(pd.host, b.counters, kCtrBytes, hipMemcpyDeviceToHost, s));
        HIPCHK(ctx, hipMemcpyAsync(static_cast<uint8_t*>(pd.host) + kCtrBytes, b.status, nimg * 4, hipMemcpyDeviceToHost, s));
        pd.timing = timing;
        pd.fancy = fancy;
        pd.blocks = double(P.total_blocks);
        pd.pixels = P.pixels;
        pd.ecs = P.ecs_bytes;
        pd.nsub = double(nsub);
        pd.nseg = double(nseg);
        pd.chunks = double(P.total_chunks);
        pd.tiles = double(P.total_tiles);
        pd.piece_bits = double(P.piece_bits);
        pd.piece_overlap = double(P.piece_overlap);
        pd.t_plan = t_plan;
        pd.t_upload = t_upload - t_plan;
        ctx->stats.host_ms[1] += t_upload;  // plan + plan upload
    }
    pd.nimg = nimg;
    pd.item_of_img = P.item_of_img;
    pd.results = results;
    pd.lo = lo;
    pd.hi = hi;
    pd.pst.assign(ctx->pst.begin() + lo, ctx->pst.begin() + hi);
    pd.w.resize(size_t(hi - lo));
    pd.h.resize(size_t(hi - lo));
    pd.host_copies.clear();
    for (int i = lo; i < hi; i++) {
        pd.w[i - lo] = ctx->parsed[i].hdr.width;
        pd.h[i - lo] = ctx->parsed[i].hdr.height;
        if (!rgb_on_device && out_addr[i] && items[i].rgb && ctx->pst[i] == JD_OK)
            pd.host_copies.push_back({reinterpret_cast<uint64_t>(items[i].rgb), out_addr[i],
                                      uint64_t(ctx->parsed[i].hdr.width) * ctx->parsed[i].hdr.height * 3});
    }
    pd.worst = worst;
    pd.rgb_on_device = rgb_on_device;
    if (!worst) {  // (a worst-case batch is never retried)
        pd.items.assign(items + lo, items + hi);
        pd.dev_addr.assign(dev_addr.begin() + lo, dev_addr.begin() + hi);
        if (lo == 0 && size_t(hi) == ctx->parsed.size())
            std::swap(pd.parsed, ctx->parsed);  // (the call's last use of them: parse_all refills ctx->parsed)
        else
            pd.parsed.assign(ctx->parsed.begin() + lo, ctx->parsed.begin() + hi);
    }
    HIPCHK(ctx, hipEventRecord(pd.done, s));
    pd.active = true;
    pd.seq = ctx->seq++;
    pd.slot = ctx->slot;
    staging.s = nullptr;  // the slot's done event now covers the copies
    ctx->slot ^= 1;
    return JD_OK;
}

// Waits for a launched batch and collects it: per-image status (a kernel's corrupt flag
// overrides OK), results, host copies of RGB, statistics.
jd_status finish_batch(jd_ctx* ctx, Pending& pd) {
    if (!pd.active) return JD_OK;
    pd.active = false;
    Range r("jd_collect");
    const auto tw0 = std::chrono::steady_clock::now();
    HIPCHK(ctx, hipEventSynchronize(pd.done));
    ctx->stats.host_ms[3] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count();
    const uint32_t nimg = pd.nimg;
    if (nimg) {
        const unsigned long long* ctr = static_cast<const unsigned long long*>(pd.host);
        const uint32_t* status = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(pd.host) + kNumCounters * 8);
        for (uint32_t i = 0; i < nimg; i++) {
            if (!status[i]) continue;
            const size_t k = size_t(pd.item_of_img[i] - pd.lo);
            pd.pst[k] = JD_ERR_CORRUPT;  // (until a retry decodes it)
            if ((status[i] & kStOverflow) && !pd.worst) {  // an optimistic pool was too small: decode it again
                jd_item it = pd.items[k];
                it.jpeg_dev = reinterpret_cast<const uint8_t*>(pd.dev_addr[k]);
                ctx->retry.push_back(jd_ctx::Retry{it, pd.parsed[k], pd.results + pd.lo + k, pd.rgb_on_device});
            }
        }
        if (ctx->host_timing)
            std::fprintf(stderr, "host plan %.3f upload %.3f wait %.3f ms\n", pd.t_plan, pd.t_upload,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count());

        // algorithmic bytes per kernel
        jd_stats& S = ctx->stats;
        const double entries = double(ctr[0]);  // 16-bit AC-entry slots
        const double blocks = pd.blocks, ecs = pd.ecs, nsegd = pd.nseg;
        double nsubd = pd.nsub;
        const bool fancy = pd.fancy;
        // k_pieceplan's choice (counters[3] = pieces << 32 | piece bits), else the host's
        const double piece_bits = (ctr[3] & 0xFFFFFFFFull) ? double(ctr[3] & 0xFFFFFFFFull) : pd.piece_bits;
        if (ctr[3] >> 32) nsubd = double(ctr[3] >> 32);
        pd.piece_bits = piece_bits;
        const double overlap_factor = (piece_bits + pd.piece_overlap) / piece_bits;
        const double bytes[JD_NUM_KERNELS] = {
            ecs,                                               // k_scan: read the ECS once
            pd.chunks * 12 + nsegd * 8,                        // k_index: per-chunk counters, boundaries
            2 * ecs,                                           // k_compact: read + write the ECS
            nsubd * 4 + nsegd * 16,                            // k_subplan: piece map
            ecs * std::min(overlap_factor, 2.0) + blocks * 4 + entries * 2 + nsubd * 32,  // k_piece: bits incl.
                                                               // warm-up in, records + AC entries + counts out
            nsubd * 8,                                         // k_redo: start/end check per piece
            nsubd * 20,                                        // k_chain: counts in, first MCU / count out
            blocks * 12 + nsubd * 24,                          // k_gather: records in, BlockInfo out
            blocks * 8 + pd.tiles * 48,                        // k_dc_pred: BlockInfo read, tile sums, scan
            blocks * 8 + entries * 2 + (fancy ? blocks * 128 : pd.pixels * 3),  // k_idct_color: coefficients
                                                                                 // in, RGB (fancy: planes) out
            fancy ? blocks * 128 + pd.pixels * 3 : 0.0};       // k_colour_fancy: planes in, RGB out
        for (int k = 0; k < JD_NUM_KERNELS; k++) {
            if (k == 10 && !fancy) continue;  // k_colour_fancy runs only with the flag
            S.launches[k]++;
            S.bytes[k] += bytes[k];
            if (pd.timing) {
                float ms = 0;
                HIPCHK(ctx, hipEventElapsedTime(&ms, pd.ev[k][0], pd.ev[k][1]));
                S.total_ms[k] += ms;
            }
        }
        S.batches += 1;
        S.images += nimg;
        S.pixels += pd.pixels;
        S.ecs_bytes += pd.ecs;
        S.blocks += blocks;
        S.segments += nsegd;
        S.subsequences += nsubd;
        S.redo_pieces += double(ctr[kCtrRedo]);
        S.fix_intervals += double(ctr[kCtrFixIntervals]);
        S.fix_rounds += double(ctr[kCtrFixRounds]);
        S.fix_rewalks += double(ctr[kCtrFixRewalks]);
        S.fix_early += double(ctr[kCtrFixEarly]);
    }
    for (int i = pd.lo; i < pd.hi; i++) {
        const jd_status st = pd.pst[size_t(i - pd.lo)];
        pd.results[i].status = st;
        const bool dims = st == JD_OK || st == JD_ERR_CORRUPT;
        pd.results[i].width = dims ? pd.w[size_t(i - pd.lo)] : 0;
        pd.results[i].height = dims ? pd.h[size_t(i - pd.lo)] : 0;
    }
    if (!pd.host_copies.empty()) {
        for (const auto& c : pd.host_copies)
            HIPCHK(ctx, hipMemcpy(reinterpret_cast<void*>(c[0]), reinterpret_cast<const void*>(c[1]), c[2],
                                  hipMemcpyDeviceToHost));
    }
    return JD_OK;
}

// Collects launched batches, oldest first, until at most `keep` are left in flight.
jd_status collect_until(jd_ctx* ctx, int keep) {
    while (true) {
        Pending* oldest = nullptr;
        int active = 0;
        for (Pending& pd : ctx->pend)
            if (pd.active) {
                active++;
                if (!oldest || pd.seq < oldest->seq) oldest = &pd;
            }
        if (active <= keep) return JD_OK;
        const jd_status st = finish_batch(ctx, *oldest);
        if (st != JD_OK) return st;
    }
}

// Collects every launched batch, oldest first.
jd_status finish_all(jd_ctx* ctx) { return collect_until(ctx, 0); }

// Decodes again, with worst-case pools, the images of collected batches that overflowed an
// optimistic one (kStOverflow), and fills their results.  Called right after every collection
// point, before anything else is launched: the retry reads a host input's copy in its slot's
// device input pool, which the slot's next launch would replace.  The retry runs as synchronous
// batches on the next launch's slot, which holds no batch at async depth 1 (the collected ones ran
// there), while the other slot's batch keeps running; otherwise every batch is collected first.
// The images' parsed headers and device bytes were kept with their batch (Pending), so nothing is
// read from the caller's host buffers, which may have been reused since; the caller's own parse
// results (decode_batch's further sub-batches) are kept aside meanwhile.
jd_status run_retries(jd_ctx* ctx, void* hip_stream) {
    if (ctx->worst || ctx->retry.empty()) return JD_OK;  // (a retry's own batches are never retried)
    std::vector<ParsedJpeg> keep_parsed;
    std::vector<jd_status> keep_pst;
    keep_parsed.swap(ctx->parsed);
    keep_pst.swap(ctx->pst);
    jd_status st = JD_OK;
    while (st == JD_OK && !ctx->retry.empty()) {
        int active = 0;
        bool next_busy = false;
        for (const Pending& pd : ctx->pend)
            if (pd.active) {
                active++;
                next_busy = next_busy || pd.slot == ctx->slot;
            }
        if (active > 1 || next_busy) st = finish_all(ctx);  // (may add retries)
        if (st != JD_OK) break;
        const int keep_slot = ctx->slot;
        std::vector<jd_ctx::Retry> r;
        r.swap(ctx->retry);
        for (int mode = 0; mode < 2 && st == JD_OK; mode++) {
            std::vector<size_t> idx;
            for (size_t j = 0; j < r.size(); j++)
                if ((r[j].rgb_on_device != 0) == (mode != 0)) idx.push_back(j);
            if (idx.empty()) continue;
            const int m = int(idx.size());
            std::vector<jd_item> items(static_cast<size_t>(m));
            std::vector<jd_result> res(static_cast<size_t>(m));
            ctx->parsed.resize(size_t(m));
            ctx->pst.assign(size_t(m), JD_OK);
            for (int j = 0; j < m; j++) {
                items[size_t(j)] = r[idx[size_t(j)]].item;
                ctx->parsed[size_t(j)] = r[idx[size_t(j)]].pj;
            }
            ctx->worst = true;
            for (int lo = 0; lo < m && st == JD_OK;) {
                const int hi = batch_split(ctx, lo, m, items.data());
                ctx->slot = keep_slot;
                hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->slots[ctx->slot].stream;
                st = launch_batch(ctx, items.data(), lo, hi, res.data(), mode, s);
                if (st == JD_OK) st = finish_batch(ctx, ctx->pend[(ctx->seq - 1) % kNumPending]);
                lo = hi;
            }
            ctx->slot = keep_slot;  // (the other slot's batch, if any, stays the older one in flight)
            ctx->worst = false;
            if (st != JD_OK) break;
            for (int j = 0; j < m; j++) *r[idx[size_t(j)]].res = res[size_t(j)];
            ctx->stats.retried_images += double(m);
        }
    }
    ctx->parsed.swap(keep_parsed);
    ctx->pst.swap(keep_pst);
    return st;
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

int jd_abi_version(void) { return JD_ABI_VERSION; }

const char* jd_status_str(jd_status st) {
    switch (st) {
        case JD_OK: return "ok";
        case JD_ERR_INVALID_ARG: return "invalid argument";
        case JD_ERR_CORRUPT: return "corrupt stream";
        case JD_ERR_UNSUPPORTED: return "unsupported JPEG variant";
        case JD_ERR_TRUNCATED: return "truncated file";
        case JD_ERR_HIP: return "HIP runtime error";
        case JD_ERR_NOMEM: return "out of memory";
        case JD_ERR_CAPACITY: return "batch exceeds capacity";
        case JD_ERR_IO: return "I/O error";
    }
    return "unknown status";
}

const char* jd_ctx_last_error(jd_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

const char* jd_kernel_name(int k) {
    static const char* names[JD_NUM_KERNELS] = {"k_scan",  "k_index", "k_compact", "k_subplan",    "k_piece",       "k_redo",
                                                "k_chain", "k_gather", "k_dc_pred", "k_idct_color", "k_colour_fancy"};
    return (k >= 0 && k < JD_NUM_KERNELS) ? names[k] : "?";
}

jd_status jd_ctx_create(jd_ctx** out, int hip_device, const jd_opts* opts) {
    if (!out) return JD_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || hip_device < 0 || hip_device >= ndev) return JD_ERR_INVALID_ARG;
    jd_ctx* ctx = new jd_ctx();
    ctx->device = hip_device;
    ctx->flags = opts ? opts->flags : 0u;
    int pt = opts ? opts->parse_threads : 0;
    if (pt <= 0) pt = int(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    ctx->parse_threads = pt;
    ctx->pool.reset(new Pool(pt - 1));
    ctx->host_timing = std::getenv("JD_HOST_TIMING") != nullptr;
    ctx->max_batch_entries = kMaxBatchEntries;
    if (const char* e = std::getenv("JD_MAX_BATCH_ENTRIES")) {
        const unsigned long long v = std::strtoull(e, nullptr, 0);
        if (v > 0) ctx->max_batch_entries = v;
    }
    ctx->max_batch_images = kMaxBatchImages;
    if (const char* e = std::getenv("JD_MAX_BATCH_IMAGES")) {
        const long v = std::strtol(e, nullptr, 0);
        if (v > 0 && v < kMaxBatchImages) ctx->max_batch_images = int(v);
    }
    // test knobs: fewer spare regions (re-walks fall back to their own region, no join) and a
    // shorter warm-up (many speculative starts fail)
    if (const char* e = std::getenv("JD_SPARE_PIECES")) ctx->spare_pieces = std::strtoll(e, nullptr, 0);
    if (const char* e = std::getenv("JD_FIXED_PIECES")) ctx->fixed_pieces = std::strtoll(e, nullptr, 0) != 0;
    if (const char* e = std::getenv("JD_PIECE_OVERLAP_BITS")) ctx->piece_overlap = std::strtoll(e, nullptr, 0);
    if (const char* e = std::getenv("JD_MIN_PIECE_BITS")) {  // a power of two in [64, kPieceBits]
        const long long v = std::strtoll(e, nullptr, 0);
        if (v >= 64 && v <= kPieceBits && (v & (v - 1)) == 0) ctx->min_piece_bits = uint32_t(v);
    }
    if (const char* e = std::getenv("JD_STAGE_NT")) ctx->stage_nt = std::strtoll(e, nullptr, 0) != 0;
    if (const char* e = std::getenv("JD_H2D_SERIAL")) ctx->h2d_serial = std::strtoll(e, nullptr, 0) != 0;
    ctx->async_depth = (ctx->flags & JD_FLAG_ASYNC_DEPTH2) ? 2 : 1;  // an explicit opt-in
    ctx->worst_always = (ctx->flags & JD_FLAG_WORST_CASE_POOLS) != 0;
    if (const char* e = std::getenv("JD_WORST_CASE_POOLS")) ctx->worst_always = ctx->worst_always || std::strtoll(e, nullptr, 0) != 0;
    if (const char* e = std::getenv("JD_BRK_CAP")) ctx->brk_cap_force = uint32_t(std::strtoul(e, nullptr, 0));
    if (const char* e = std::getenv("JD_STAGE_CHUNK_MB")) {
        const long long mb = std::strtoll(e, nullptr, 0);
        ctx->stage_chunk = mb > 0 ? size_t(mb) << 20 : ~size_t(0);
    }
    if (hipSetDevice(hip_device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return JD_ERR_HIP;
    }
    // experiment knobs: JD_SLOT_PRIO / JD_IDCT_PRIO = 1 (greatest priority) or -1 (least); JD_IDCT_STREAM=1
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    auto prio_of = [&](const char* env) {
        const char* e = std::getenv(env);
        const long v = e ? std::strtol(e, nullptr, 0) : 0;
        return v > 0 ? prio_greatest : v < 0 ? prio_least : 0;
    };
    const bool idct_stream = std::getenv("JD_IDCT_STREAM") && std::strtol(std::getenv("JD_IDCT_STREAM"), nullptr, 0) != 0;

    for (Slot& sl : ctx->slots) {
        bool ok = hipStreamCreateWithPriority(&sl.stream, hipStreamNonBlocking, prio_of("JD_SLOT_PRIO")) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&sl.h2d_done, hipEventDisableTiming) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&sl.plan_done, hipEventDisableTiming) == hipSuccess;
        if (ok && idct_stream) {
            ok = hipStreamCreateWithPriority(&sl.istream, hipStreamNonBlocking, prio_of("JD_IDCT_PRIO")) == hipSuccess;
            ok = ok && hipEventCreateWithFlags(&sl.ev_tail, hipEventDisableTiming) == hipSuccess;
            ok = ok && hipEventCreateWithFlags(&sl.ev_idct, hipEventDisableTiming) == hipSuccess;
        }
        if (!ok) {
            jd_ctx_destroy(ctx);
            return JD_ERR_HIP;
        }
    }
    for (Pending& pd : ctx->pend) {
        bool ok = hipEventCreateWithFlags(&pd.done, hipEventDisableTiming) == hipSuccess;
        for (int k = 0; k < JD_NUM_KERNELS; k++)
            for (int j = 0; j < 2; j++) ok = ok && hipEventCreate(&pd.ev[k][j]) == hipSuccess;
        if (!ok) {
            jd_ctx_destroy(ctx);
            return JD_ERR_HIP;
        }
    }
    *out = ctx;
    return JD_OK;
}

jd_status jd_ctx_destroy(jd_ctx* ctx) {
    if (!ctx) return JD_ERR_INVALID_ARG;
    (void)hipSetDevice(ctx->device);
    (void)quiesce(ctx);
    for (DevBuf* b : {&ctx->lut_dev, &ctx->output})
        if (b->p) (void)hipFree(b->p);
    for (Slot& sl : ctx->slots) {
        for (DevBuf* b : {&sl.d_plan, &sl.d_brk, &sl.d_blocks, &sl.d_entries, &sl.d_comp, &sl.d_planes, &sl.d_stamps,
                          &sl.d_input})
            if (b->p) (void)hipFree(b->p);
        if (sl.in_host) (void)hipHostFree(sl.in_host);
        if (sl.plan_host) (void)hipHostFree(sl.plan_host);
        if (sl.stream) (void)hipStreamDestroy(sl.stream);
        if (sl.h2d_done) (void)hipEventDestroy(sl.h2d_done);
        if (sl.plan_done) (void)hipEventDestroy(sl.plan_done);
        if (sl.istream) (void)hipStreamDestroy(sl.istream);
        if (sl.ev_tail) (void)hipEventDestroy(sl.ev_tail);
        if (sl.ev_idct) (void)hipEventDestroy(sl.ev_idct);
    }
    for (Pending& pd : ctx->pend) {
        if (pd.host) (void)hipHostFree(pd.host);
        if (pd.done) (void)hipEventDestroy(pd.done);
        for (int k = 0; k < JD_NUM_KERNELS; k++)
            for (int j = 0; j < 2; j++)
                if (pd.ev[k][j]) (void)hipEventDestroy(pd.ev[k][j]);
    }
    for (const auto& r : ctx->host_regs) {
        void* p = reinterpret_cast<void*>(r.first);
        if (std::find(ctx->host_owned.begin(), ctx->host_owned.end(), r.first) != ctx->host_owned.end())
            (void)hipHostFree(p);
        else
            (void)hipHostUnregister(p);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return JD_OK;
}

jd_status jd_host_register(jd_ctx* ctx, void* ptr, size_t bytes) {
    if (!ctx || !ptr || !bytes) return JD_ERR_INVALID_ARG;
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr), e = a + bytes;
    for (const auto& r : ctx->host_regs)
        if (a < r.second && r.first < e) return JD_ERR_INVALID_ARG;  // overlaps a registered range
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    ctx->host_regs.insert(std::upper_bound(ctx->host_regs.begin(), ctx->host_regs.end(), std::make_pair(a, e)),
                          std::make_pair(a, e));
    return JD_OK;
}

// Removes a registered (owned = false) or allocated (owned = true) range.
static jd_status host_release(jd_ctx* ctx, void* ptr, bool owned) {
    if (!ctx || !ptr) return JD_ERR_INVALID_ARG;
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    auto it = std::find_if(ctx->host_regs.begin(), ctx->host_regs.end(),
                           [&](const std::pair<uintptr_t, uintptr_t>& r) { return r.first == a; });
    auto ow = std::find(ctx->host_owned.begin(), ctx->host_owned.end(), a);
    if (it == ctx->host_regs.end() || (ow != ctx->host_owned.end()) != owned) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, quiesce(ctx));  // a launched batch may still be reading it
    ctx->host_regs.erase(it);
    if (owned) {
        ctx->host_owned.erase(ow);
        HIPCHK(ctx, hipHostFree(ptr));
    } else {
        HIPCHK(ctx, hipHostUnregister(ptr));
    }
    return JD_OK;
}

jd_status jd_host_unregister(jd_ctx* ctx, void* ptr) { return host_release(ctx, ptr, false); }

jd_status jd_host_alloc(jd_ctx* ctx, size_t bytes, void** ptr) {
    if (!ctx || !bytes || !ptr) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    void* p = nullptr;
    HIPCHK(ctx, hipHostMalloc(&p, bytes, hipHostMallocDefault));
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    ctx->host_regs.insert(std::upper_bound(ctx->host_regs.begin(), ctx->host_regs.end(), std::make_pair(a, a + bytes)),
                          std::make_pair(a, a + bytes));
    ctx->host_owned.push_back(a);
    *ptr = p;
    return JD_OK;
}

jd_status jd_host_free(jd_ctx* ctx, void* ptr) { return host_release(ctx, ptr, true); }

jd_status jd_parse(const uint8_t* jpeg, size_t len, jd_header* hdr) {
    if (!jpeg || !hdr) return JD_ERR_INVALID_ARG;
    ParsedJpeg* p = new ParsedJpeg();
    jd_status st = parse_jpeg(jpeg, len, p);
    *hdr = p->hdr;
    delete p;
    return st;
}

namespace {
// Parse on the host, then plan + launch every sub-batch; async leaves the last one launched
// (each launch first collects the batch two launches back, whose slot it reuses).
jd_status decode_batch(jd_ctx* ctx, const jd_item* items, int n, jd_result* results, int rgb_on_device,
                       void* hip_stream, bool async) {
    if (!ctx || n < 0 || (n > 0 && (!items || !results))) return JD_ERR_INVALID_ARG;
    for (int i = 0; i < n; i++)
        if (!items[i].jpeg || items[i].len > 0xFFFFFFF0ull) return JD_ERR_INVALID_ARG;
    if (hipSetDevice(ctx->device) != hipSuccess) return JD_ERR_HIP;
    // Without a caller stream each slot runs on its own stream; a caller stream orders both slots.
    // Switching streams first collects the pending batches.
    if (hip_stream != ctx->last_stream) {
        jd_status st = finish_all(ctx);
        if (st == JD_OK) st = run_retries(ctx, const_cast<void*>(ctx->last_stream));  // (on their own stream)
        if (st != JD_OK) return st;
        ctx->last_stream = hip_stream;
    }
    // The output pool is shared by the slots: with host outputs, collect first, and collect every
    // sub-batch before launching the next.  Host inputs are staged per slot and pipeline.
    if (!rgb_on_device) {
        jd_status st = finish_all(ctx);
        if (st == JD_OK) st = run_retries(ctx, hip_stream);
        if (st != JD_OK) return st;
        async = false;
    }
    const auto t0 = std::chrono::steady_clock::now();
    parse_all(ctx, items, n);
    const double t_parse = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->stats.host_ms[0] += t_parse;
    if (ctx->host_timing) std::fprintf(stderr, "host parse %.3f ms\n", t_parse);
    for (int lo = 0; lo < n;) {
        const int hi = batch_split(ctx, lo, n, items);
        hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->slots[ctx->slot].stream;
        jd_status st = launch_batch(ctx, items, lo, hi, results, rgb_on_device, s);
        if (st != JD_OK) return st;
        // async: the newest async_depth launches stay in flight (with 2, this launch was enqueued
        // behind the batch two launches back on its slot's stream before that batch is waited
        // for); otherwise collect this sub-batch before the next one reuses the staging and
        // output pools
        st = collect_until(ctx, async ? ctx->async_depth : 0);
        if (st == JD_OK) st = run_retries(ctx, hip_stream);  // (before the next sub-batch reuses a slot)
        if (st != JD_OK) return st;
        lo = hi;
    }
    if (!async) {
        jd_status st = finish_all(ctx);
        if (st == JD_OK) st = run_retries(ctx, hip_stream);
        if (st != JD_OK) return st;
    }
    return JD_OK;
}
}  // namespace

jd_status jd_decode_batch(jd_ctx* ctx, const jd_item* items, int n, jd_result* results, int rgb_on_device,
                          void* hip_stream) {
    return decode_batch(ctx, items, n, results, rgb_on_device, hip_stream, false);
}

jd_status jd_decode_batch_async(jd_ctx* ctx, const jd_item* items, int n, jd_result* results, void* hip_stream) {
    return decode_batch(ctx, items, n, results, 1, hip_stream, true);
}

jd_status jd_decode_wait(jd_ctx* ctx) {
    if (!ctx) return JD_ERR_INVALID_ARG;
    if (hipSetDevice(ctx->device) != hipSuccess) return JD_ERR_HIP;
    const jd_status st = finish_all(ctx);
    if (st != JD_OK) return st;
    return run_retries(ctx, const_cast<void*>(ctx->last_stream));
}

jd_status jd_decode(jd_ctx* ctx, const uint8_t* jpeg, size_t len, uint8_t* rgb, int rgb_on_device, int* width,
                    int* height) {
    if (!ctx || !jpeg || !rgb) return JD_ERR_INVALID_ARG;
    jd_item it{jpeg, nullptr, len, rgb};
    jd_result r{};
    jd_status st = jd_decode_batch(ctx, &it, 1, &r, rgb_on_device, nullptr);
    if (st != JD_OK) return st;
    if (width) *width = r.width;
    if (height) *height = r.height;
    return jd_status(r.status);
}

jd_status jd_decode_file(jd_ctx* ctx, const char* path, uint8_t* rgb, size_t rgb_capacity, int rgb_on_device,
                         int* width, int* height) {
    if (!ctx || !path) return JD_ERR_INVALID_ARG;
    FILE* f = fopen(path, "rb");
    if (!f) return JD_ERR_IO;
    std::vector<uint8_t> data;
    uint8_t tmp[1 << 16];
    size_t got;
    while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) data.insert(data.end(), tmp, tmp + got);
    fclose(f);
    jd_header h;
    jd_status st = jd_parse(data.data(), data.size(), &h);
    if (st != JD_OK) return st;
    if (width) *width = h.width;
    if (height) *height = h.height;
    if (!rgb) return JD_OK;  // header query
    if (rgb_capacity < size_t(h.width) * h.height * 3) return JD_ERR_CAPACITY;
    return jd_decode(ctx, data.data(), data.size(), rgb, rgb_on_device, width, height);
}

jd_status jd_write_array(const char* path, const uint8_t* rgb, int width, int height) {
    if (!path || !rgb || width <= 0 || height <= 0) return JD_ERR_INVALID_ARG;
    FILE* f = fopen(path, "wb");
    if (!f) return JD_ERR_IO;
    fprintf(f, "%d %d\n", height, width);  // parser.cpp:203
    const size_t npx = size_t(width) * height;
    std::string line;
    line.reserve(npx * 4);
    for (int c = 0; c < 3; c++) {  // parser.cpp:204-208: R, G, B planes
        line.clear();
        char buf[8];
        for (size_t i = 0; i < npx; i++) {
            int n = snprintf(buf, sizeof(buf), "%d ", rgb[i * 3 + c]);
            line.append(buf, size_t(n));
        }
        if (c < 2) line.push_back('\n');
        fwrite(line.data(), 1, line.size(), f);
    }
    fclose(f);
    return JD_OK;
}

jd_status jd_write_ppm(const char* path, const uint8_t* rgb, int width, int height) {
    if (!path || !rgb || width <= 0 || height <= 0) return JD_ERR_INVALID_ARG;
    FILE* f = fopen(path, "wb");
    if (!f) return JD_ERR_IO;
    fprintf(f, "P6\n%d %d\n255\n", width, height);
    const size_t n = size_t(width) * height * 3;
    const bool ok = fwrite(rgb, 1, n, f) == n;
    return (fclose(f) == 0 && ok) ? JD_OK : JD_ERR_IO;
}

jd_status jd_device_alloc(jd_ctx* ctx, size_t bytes, void** dptr) {
    if (!ctx || !dptr) return JD_ERR_INVALID_ARG;
    (void)hipSetDevice(ctx->device);
    HIPCHK(ctx, hipMalloc(dptr, std::max<size_t>(bytes, 1)));
    return JD_OK;
}

jd_status jd_device_free(jd_ctx* ctx, void* dptr) {
    if (!ctx) return JD_ERR_INVALID_ARG;
    if (dptr) HIPCHK(ctx, hipFree(dptr));
    return JD_OK;
}

jd_status jd_memcpy_h2d(jd_ctx* ctx, void* dst, const void* src, size_t n) {
    if (!ctx || (n && (!dst || !src))) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, order_after_pending(ctx));  // an in-flight batch may still read dst
    HIPCHK(ctx, hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return JD_OK;
}

jd_status jd_memcpy_d2h(jd_ctx* ctx, void* dst, const void* src, size_t n) {
    if (!ctx || (n && (!dst || !src))) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, order_after_pending(ctx));  // an in-flight batch may still write src
    HIPCHK(ctx, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return JD_OK;
}

jd_status jd_synchronize(jd_ctx* ctx) {
    if (!ctx) return JD_ERR_INVALID_ARG;
    jd_status st = finish_all(ctx);
    if (st == JD_OK) st = run_retries(ctx, const_cast<void*>(ctx->last_stream));  // (collected batches' overflows)
    if (st != JD_OK) return st;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return JD_OK;
}

jd_status jd_get_stats(jd_ctx* ctx, jd_stats* out) {
    if (!ctx || !out) return JD_ERR_INVALID_ARG;
    *out = ctx->stats;
    return JD_OK;
}

jd_status jd_reset_stats(jd_ctx* ctx) {
    if (!ctx) return JD_ERR_INVALID_ARG;
    ctx->stats = jd_stats{};
    return JD_OK;
}

jd_status jd_debug_fetch(jd_ctx* ctx, int what, void* dst, size_t cap, size_t* nbytes) {
    if (!ctx || !nbytes) return JD_ERR_INVALID_ARG;
    const BatchDev& b = ctx->last;
    const void* src = nullptr;
    size_t n = 0;
    switch (what) {
        case 0: src = b.blocks; n = ctx->last_blocks * sizeof(BlockInfo); break;
        case 1: src = b.seg_cstart; n = size_t(b.nseg) * 4; break;
        case 2: src = b.seg_cend; n = size_t(b.nseg) * 4; break;
        case 3: src = b.seg_sub_base; n = size_t(b.nseg) * 4; break;
        case 4: src = b.seg_nsub; n = size_t(b.nseg) * 4; break;
        case 5: src = b.piece_bit; n = size_t(b.nsub) * 4; break;
        case 6: src = b.piece_end; n = size_t(b.nsub) * 4; break;
        case 7: src = b.piece_nmcu; n = size_t(b.nsub) * 4; break;
        case 8: src = b.piece_nent; n = size_t(b.nsub) * 4; break;
        case 9: src = b.sub_seg; n = size_t(b.nsub) * 4; break;
        case 10: src = b.status; n = size_t(b.nimg) * 4; break;
        case 11: src = b.entries; n = ctx->last_entries * 4; break;
        case 12: src = b.piece_mcu0; n = size_t(b.nsub) * 4; break;
        case 13: src = b.piece_abase; n = size_t(b.nsub) * 4; break;
        case 14: src = b.piece_cp; n = size_t(b.nsub) * kCpRecords * sizeof(CpRec); break;
        case 15: src = b.stamps; n = b.stamps ? size_t(b.total_tiles) * 64 : 0; break;
        case 16: src = b.piece_emcu; n = size_t(b.nsub) * 4; break;
        case 17: src = b.piece_amcu; n = size_t(b.nsub) * 4; break;
        case 18: src = b.piece_join; n = size_t(b.nsub) * 4; break;
        case 19: src = b.seg_ent; n = size_t(b.nseg) * 4; break;
        case 20:  // per image of the last batch: ImgDesc::entry_base (u64, 32-bit words), host copy
            *nbytes = ctx->last_entry_base.size() * 8;
            if (dst) memcpy(dst, ctx->last_entry_base.data(), std::min(*nbytes, cap));
            return JD_OK;
        case 21:  // per image of the last batch: ImgDesc::rw_div (u32), host copy
            *nbytes = ctx->last_rw_div.size() * 4;
            if (dst) memcpy(dst, ctx->last_rw_div.data(), std::min(*nbytes, cap));
            return JD_OK;
        case 22:  // per image of the last batch: ImgDesc::rw_slack (u32), host copy
            *nbytes = ctx->last_rw_slack.size() * 4;
            if (dst) memcpy(dst, ctx->last_rw_slack.data(), std::min(*nbytes, cap));
            return JD_OK;
        default: return JD_ERR_INVALID_ARG;
    }
    *nbytes = n;
    if (dst && src && n) {
        HIPCHK(ctx, quiesce(ctx));  // the last batch ran on a slot's stream
        HIPCHK(ctx, hipMemcpy(dst, src, std::min(n, cap), hipMemcpyDeviceToHost));
    }
    return JD_OK;
}

jd_status jd_test_idct(jd_ctx* ctx, const int32_t* in_dev, int32_t* out_dev, int nblocks) {
    if (!ctx || !in_dev || !out_dev || nblocks < 0) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, launch_test_idct(in_dev, out_dev, nblocks, 0, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return JD_OK;
}

jd_status jd_test_idct_exact(jd_ctx* ctx, const int32_t* in_dev, int32_t* out_dev, int nblocks) {
    if (!ctx || !in_dev || !out_dev || nblocks < 0) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, launch_test_idct(in_dev, out_dev, nblocks, 1, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return JD_OK;
}

jd_status jd_test_color(jd_ctx* ctx, const int32_t* ycc_dev, uint8_t* rgb_dev, int n) {
    if (!ctx || !ycc_dev || !rgb_dev || n < 0) return JD_ERR_INVALID_ARG;
    HIPCHK(ctx, launch_test_color(ycc_dev, rgb_dev, n, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return JD_OK;
}

jd_status jd_device_bytes(jd_ctx* ctx, uint64_t* current, uint64_t* peak) {
    if (!ctx) return JD_ERR_INVALID_ARG;
    if (current) *current = ctx->dev_bytes;
    if (peak) *peak = ctx->dev_peak;
    return JD_OK;
}

jd_status jd_test_copy_peak(jd_ctx* ctx, const void* src, void* dst, size_t bytes, int reps, double* gbs) {
    if (!ctx || !src || !dst || !gbs || reps <= 0 || bytes == 0 || bytes % 16) return JD_ERR_INVALID_ARG;
    (void)hipSetDevice(ctx->device);
    HIPCHK(ctx, order_after_pending(ctx));
    hipEvent_t e0, e1;
    HIPCHK(ctx, hipEventCreate(&e0));
    HIPCHK(ctx, hipEventCreate(&e1));
    hipError_t e = launch_copy16(src, dst, bytes, ctx->stream);  // warm-up
    if (e == hipSuccess) e = hipEventRecord(e0, ctx->stream);
    for (int r = 0; r < reps && e == hipSuccess; r++) e = launch_copy16(src, dst, bytes, ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(e1, ctx->stream);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (e != hipSuccess) return hip_fail(ctx, e, "jd_test_copy_peak");
    *gbs = ms > 0 ? 2.0 * double(bytes) * reps / (double(ms) * 1e-3) / 1e9 : 0.0;
    return JD_OK;
}

}  // extern "C"
