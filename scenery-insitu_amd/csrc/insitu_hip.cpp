// insitu_hip.cpp -- host side of libinsitu_hip.so: the C ABI declared in include/insitu_hip.h.
//
// Owns the per-rank device state of the in-situ frame (bricks, transfer function, sub-VDI
// send/receive blocks, octree counters, composited strip, gathered image) and orders the
// four stages on one HIP stream:
//   render    -> VDIGenerator.comp+AccumulateVDI.comp / VolumeRaycaster.comp+AccumulatePlainImage.comp
//   exchange  -> distributeVDIs' MPI_Alltoall (DistributedVolumes.kt:860), here RCCL send/recv
//                of contiguous screen-strip blocks over xGMI
//   composite -> PlainImageCompositor.comp / VDI flatten (VDIGenerator.comp:147-185)
//   gather    -> gatherCompositedVDIs' MPI_Gather (DistributedVolumes.kt:903), RCCL to rank 0
#include "insitu_hip.h"
#include "insitu_kernels.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#pragma clang fp contract(off)

using namespace insitu;

namespace {

thread_local std::string g_create_error;

struct Brick {
    void* d = nullptr;
    size_t bytes = 0;
    int dtype = -1;
    int dims[3] = {0, 0, 0};
    float im[16];
    bool valid = false;
};

size_t dtype_size(int dt) { return dt == INSITU_U8 ? 1 : (dt == INSITU_U16 ? 2 : 4); }

// float mat4 product with the same operation order as the shaders' `A * B` (and the oracle)
void mat4_mul_f(const float* a, const float* b, float* out) {
    float t[16];
    for (int c = 0; c < 4; ++c) {
        const float x = b[c * 4 + 0], y = b[c * 4 + 1], z = b[c * 4 + 2], w = b[c * 4 + 3];
        for (int r = 0; r < 4; ++r)
            t[c * 4 + r] = std::fmaf(a[12 + r], w, std::fmaf(a[8 + r], z, std::fmaf(a[4 + r], y, a[r] * x)));
    }
    std::memcpy(out, t, sizeof t);
}

// general 4x4 inverse in double, rounded to float (column-major in and out)
bool mat4_inverse(const float* m, float* out) {
    double a[4][8];
    for (int r = 0; r < 4; ++r) {
        for (int c = 0; c < 4; ++c) a[r][c] = (double)m[c * 4 + r];
        for (int c = 0; c < 4; ++c) a[r][4 + c] = (r == c) ? 1.0 : 0.0;
    }
    for (int col = 0; col < 4; ++col) {
        int piv = col;
        for (int r = col + 1; r < 4; ++r)
            if (std::fabs(a[r][col]) > std::fabs(a[piv][col])) piv = r;
        if (a[piv][col] == 0.0) return false;
        if (piv != col)
            for (int c = 0; c < 8; ++c) std::swap(a[piv][c], a[col][c]);
        const double inv = 1.0 / a[col][col];
        for (int c = 0; c < 8; ++c) a[col][c] *= inv;
        for (int r = 0; r < 4; ++r) {
            if (r == col) continue;
            const double f = a[r][col];
            for (int c = 0; c < 8; ++c) a[r][c] -= f * a[col][c];
        }
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) out[c * 4 + r] = (float)a[r][4 + c];
    return true;
}

}  // namespace

struct insitu_local_group {
    std::vector<insitu_ctx*> ranks;
};

// tuning knobs of the VDI generator (insitu_set_option; seeded from the environment at create)
struct Tuning {
    long long exact_search = 0;
    long long search_depth = 0;
    long long long_samples = 384;   // measured optimum
    long long round_batch = 28;     // round 5: 28 vs 20, three A/Bs on one box each: search -0.1 to -0.2 ms
    long long search_oversub = 6;   // measured: one brick per GPU (N=8) 12.2 -> 10.9 ms, N=1..4 unchanged
    long long pipe_oversub = 3;     // pipelined frames (their search overlaps the next first pass): emulated N=8
                                    // share 4.62 -> 4.18 ms/frame, N=4 6.11 -> 5.62, N=1..2 unchanged
    long long pipe_search_rays = 2048;   // pipelined frames: queued rays per searching block (0: the full grid)
    long long tile_order = 1;       // sampling tiles longest-first
    long long super_tile = 1;       // ... by the longest ray of super-tiles of this many tiles per edge
    long long regroup = 1;          // search: deeper tree groups for the rays left once the queue is drained
    long long exact_tile_keys = 0;  // 1: tile keys from all 64 rays of a tile (0: 16 of them)
};

// hipEvent slots of a frame (insitu_ctx::ev): [0] render start, [1] render end (send buffers ready),
// [2] exchange end, [3] composite end, [4] gather end, [5] sample / search split, [6] compaction start,
// [7] (local group) this rank's copies out of its peers' buffers are done -- recorded after its exchange and
// its gather; a peer's next render/composite waits on it before rewriting them, [8] exchange counts in,
// [9] payload start, [10] the root's image copied to the host buffer of insitu_gather, [11] (pipelined) the
// frame's completion is done: its slot may be rendered into again, [12] compaction end, [13] (pipelined)
// search end: the next frame's sampling may start (trigger mode 0)
constexpr int kFrameEvents = 14;

// The generator's per-frame buffers and the frame's camera, events and stage flags.  Pipelined frames
// (insitu_frame_pipelined) render frame k+1 into one set while frame k is composited from the other: the
// insitu_ctx members listed in swap_slot hold the set of the frame the stage functions work on, `alt` holds
// the other (swap_slot exchanges them).  Unpipelined contexts use one set (alt stays empty).
struct FrameSlot {
    float4* vcol_send = nullptr;
    float2* vdep_send = nullptr;
    uint32_t* octree = nullptr;
    uint8_t* passes = nullptr;
    uint16_t* seg_pending = nullptr;
    uint16_t* seg_steps = nullptr;
    GenCounters* counters = nullptr;
    PendingRay* queue = nullptr;
    float* cache = nullptr;
    uint32_t cache_chunks = 0;
    uint32_t cache_grow_to = 0;
    bool cache_sized = false;
    GenCounters* h_ctr = nullptr;
    bool h_ctr_pending = false;
    bool h_ctr_valid = false;
    bool search_launched = false;
    uint32_t* tile_keys = nullptr;
    uint32_t* tile_ids = nullptr;
    unsigned char* sort_tmp = nullptr;
    float ipv[16] = {}, pv[16] = {}, view[16] = {};
    bool rendered = false, composited = false, exchanged = false;
    bool pipelined = false;   // rendered by insitu_frame_pipelined (compaction runs with the completion)
    hipStream_t search_stream = nullptr;   // pipelined: the slot's search, finish and counter copy run here
    int flag_index = 1;                    // pipelined: the slot's drain trigger, insitu_ctx::pipe_flag[flag_index]
    hipEvent_t ev[kFrameEvents] = {};
    bool ev_valid[kFrameEvents] = {};
};

struct insitu_ctx {
    insitu_config cfg{};
    insitu_local_group* group = nullptr;   // in-process rank group (test transport), else RCCL
    int W = 0, H = 0, S = 0, N = 1, rank = 0, B = 1, V = 1, mode = INSITU_MODE_VDI;
    int BV = 1;   // sub-VDIs per rank: B, or 1 when the bricks are the volumes of one VDI (merge_bricks)
    int strip_w = 0, strip_tiles = 0, rows = 0, ncx = 0, ncy = 0;
    size_t blockE = 0;      // VDI entries per (strip, brick) block
    size_t plainBlock = 0;  // pixels per (strip, brick) block in plain mode
    size_t stripPx = 0;     // pixels of one composited strip
    hipStream_t stream = nullptr;
    bool own_stream = false;
    ncclComm_t comm = nullptr;
    std::vector<Brick> bricks;
    float* d_tf = nullptr;
    float* d_cmap = nullptr;
    int n_tf = 0, n_cm = 0;
    float cmag = 1.0f;                  // TransferDesc::cmag of the current LUTs
    float conv_scale = 1.0f, conv_offset = 0.0f;
    float4* d_vcol_send = nullptr;
    float2* d_vdep_send = nullptr;
    float4* d_vcol_recv = nullptr;
    float2* d_vdep_recv = nullptr;
    uint32_t* d_octree = nullptr;
    uint8_t* d_passes = nullptr;
    uint16_t* d_seg_pending = nullptr;  // per brick and pixel: supersegments awaiting vdi_finish_kernel
    uint16_t* d_seg_steps = nullptr;    // per sub-VDI entry: step count of a deferred colour
    uint32_t* d_pcol_send = nullptr;
    uint32_t* d_pdep_send = nullptr;
    uint32_t* d_pcol_recv = nullptr;
    uint32_t* d_pdep_recv = nullptr;
    uint32_t* d_strip = nullptr;
    uint32_t* d_gather = nullptr;
    uint32_t* d_image = nullptr;
    float4* d_ref_col = nullptr;        // reference-layout staging for insitu_distribute_vdis: send | recv
    float* d_ref_dep = nullptr;
    uint16_t* d_ref_cnt = nullptr;      // per source strip [y][xl] counts of the host-buffer path's lists
    bool lists_from_reference = false;  // the last composite input came through insitu_distribute_vdis
    // variable-length exchange (N > 1, VDI mode): compact messages per destination
    float4* d_ccol_send = nullptr;      // [d] regions of B*blockE entries
    float2* d_cdep_send = nullptr;
    uint8_t* d_meta_send = nullptr;     // [d] regions of meta_bytes
    uint8_t* d_meta_recv = nullptr;     // [s]
    uint32_t* d_cursor = nullptr;       // [d] entries packed for d | [N + s] entries received from s
    uint32_t* h_tot = nullptr;          // pinned copy of d_cursor
    size_t meta_bytes = 0;
    bool camera_set = false;
    float* d_cache = nullptr;           // per-sample raymarch cache (32-byte chunks of 4 samples)
    void* d_staging = nullptr;          // host-buffer brick uploads (kept: re-ingest every N frames)
    size_t staging_bytes = 0;
    GenCounters* d_counters = nullptr;  // cache cursor + search queue counters
    PendingRay* d_queue = nullptr;      // rays queued for the search kernel (B*W*H)
    uint32_t cache_chunks = 0;
    // default-sized caches grow to the measured demand: the frame's cursor (chunks asked for) is
    // copied to pinned h_ctr at the end of every render, read after the next synchronisation
    bool cache_adaptive = false;
    size_t cache_max_chunks = 0;        // growth limit (45 % of the HBM free at create, 2^32 chunks)
    uint32_t cache_grow_to = 0;         // > cache_chunks: reallocate before the next render
    GenCounters* h_ctr = nullptr;       // pinned copy of d_counters (valid after a synchronisation)
    bool cache_sized = false;           // the default cache was sized from a frame's measured demand
    bool h_ctr_pending = false;         // h_ctr's copy was enqueued and not yet observed after a synchronisation
    bool h_ctr_valid = false;           // h_ctr holds the last render's counters (observed after a synchronisation)
    int num_cus = 256;
    int search_blocks = 0;
    int search_lanes = 0;               // resident lanes of the search grid for the LUT sizes below
    int search_lanes_tf = -1, search_lanes_cm = -1;
    Tuning tune;
    bool search_launched = false;       // a render ran the persistent search kernel (fault flag valid)
    unsigned long long* d_dbg = nullptr;   // INSITU_DEBUG_RAYS: per-round search timing
    uint32_t* d_tile_keys = nullptr;       // longest-tiles-first order: keys / ids (2 x B*tiles each)
    uint32_t* d_tile_ids = nullptr;
    unsigned char* d_sort_tmp = nullptr;   // hipcub temporary storage
    size_t sort_tmp_bytes = 0;
    size_t dbg_entries = 0;
    std::string dbg_path;
    bool dbg_pending = false;
    long long last_exchange_bytes = 0, last_exchange_entries = 0;
    bool composite_vdi = false;         // VDICompositor output instead of the RGBA flatten
    int S_out = 0;
    size_t cblockE = 0;                 // composited-VDI entries per strip block (S_out slots)
    float4* d_cvdi_col = nullptr;       // this rank's composited strip (non-root ranks)
    float2* d_cvdi_dep = nullptr;
    float4* d_gvdi_col = nullptr;       // root: gathered composited strips [rank][block]
    float2* d_gvdi_dep = nullptr;
    uint16_t* d_cvdi_cnt = nullptr;     // per pixel of this rank's composited strip: slots written (non-root ranks)
    uint16_t* d_gvdi_cnt = nullptr;     // root: the gathered counts [rank][y][x_local]
    uint8_t* d_cpasses = nullptr;       // compositor search passes of the strip
    float4* d_cseq = nullptr;           // VDICompositor merge cache (kCompEntryF4 float4 per entry)
    unsigned long long* d_cseq_cursor = nullptr;
    unsigned long long* h_cseq_demand = nullptr;   // pinned: the last composite's demand (entries), written
                                                   // by an async copy; read only by cache_observe after a sync
    bool cseq_pending = false;          // that copy is enqueued and not yet observed
    unsigned long long cseq_demand = 0; // the demand observed after the last composite's synchronisation
    unsigned long long cseq_cap = 0;    // capacity (entries)
    unsigned long long cseq_max = 0;    // growth limit (entries): 20 % of the HBM free at create
    float ipv[16], pv[16], view[16];
    bool rendered = false, composited = false;
    bool exchanged = false;             // the compositor's input lists are complete (VDI set readable)
    bool slot_pipelined = false;        // this slot's frame was rendered by insitu_frame_pipelined
    hipStream_t slot_search_stream = nullptr;   // pipelined: this slot's search stream (FrameSlot::search_stream)
    int slot_flag_index = 0;            // pipelined: this slot's trigger flag (FrameSlot::flag_index)
    hipEvent_t ev[kFrameEvents] = {};   // (kFrameEvents above)
    bool ev_valid[kFrameEvents] = {};
    // cross-frame pipelining (insitu_frame_pipelined, DistributedVolumeRenderer.kt:530-542: the composite is
    // one frame stale): the other frame's buffers, the sampling and completion streams, the trigger flag
    FrameSlot alt;
    bool pipe_ready = false;            // alt allocated, streams created
    bool pipe_inflight = false;         // alt holds a rendered frame whose completion is pending
    bool completing = false;            // insitu_frame_pipelined is running the stages of the frame one behind
    bool ingest_batch = false;          // re-ingests since the last render: ev_ingest0 marks their start
    hipEvent_t ev_ingest0 = nullptr, ev_ingest = nullptr;   // the last batch of re-ingests (start, end)
    hipEvent_t ev_gate = nullptr;       // pipelined: `stream`'s work so far, waited for by the next first pass
    hipStream_t pipe_sample = nullptr;  // the first pass of every pipelined frame (low priority)
    hipStream_t pipe_comp = nullptr;    // exchange, composite, gather of the frame one behind (high priority)
    hipStream_t s_sample = nullptr;     // where insitu_render puts its first pass (null: `stream`)
    // search-drain triggers, one per slot (device memory, written at system scope): a slot's frames are
    // sequential, so its flag only grows -- two slots' searches may overlap and drain in either order
    unsigned long long* pipe_flag = nullptr;
    unsigned long long pipe_seq = 0;    // frames rendered by the pipeline (the value each search stores)
    long long pipe_frames = 0;          // frame index of the next pipelined render
    int pipe_trigger = 2;               // 0: after the previous search; 1: at its queue drain; 2: none (default:
                                        // the search keeps only the blocks its queue needs)
    bool pipe_wait_value = true;        // hipStreamWaitValue64 works here (else mode 1 falls back to 0)
    // the trigger of the frame insitu_render is enqueuing, placed between its prepare (counters, tile keys and
    // their sort: the slot's own buffers) and its sampling kernel, so the prepare's launches run ahead of it
    unsigned long long* trig_flag = nullptr;         // wait for *trig_flag >= trig_value (mode 1) ...
    unsigned long long trig_value = 0;
    hipEvent_t trig_event = nullptr;                 // ... or for this event (mode 0)
    std::string err;
};

namespace {

int fail(insitu_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    else g_create_error = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(ctx, -3, std::string(#expr " failed: ") + hipGetErrorString(e_));          \
    } while (0)

#define NCCLCHK(ctx, expr)                                                                         \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return fail(ctx, -4, std::string(#expr " failed: ") + ncclGetErrorString(r_));         \
    } while (0)

template <typename T>
int dev_alloc(insitu_ctx* c, T** p, size_t count) {
    if (count == 0) { *p = nullptr; return 0; }
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess)
        return fail(c, -5, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed: " + hipGetErrorString(e));
    return 0;
}

void release(insitu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    // every stream first: a pipelined frame left in flight (no insitu_pipeline_flush) still runs on the sampling,
    // search and completion streams and reads the buffers, events and trigger flags freed below (each of its
    // waits has its producer enqueued ahead of it, so these synchronisations end)
    for (hipStream_t st : {c->stream, c->pipe_sample, c->slot_search_stream, c->alt.search_stream, c->pipe_comp})
        if (st) (void)hipStreamSynchronize(st);
    for (auto& b : c->bricks)
        if (b.d) (void)hipFree(b.d);
    void* ptrs[] = {c->d_tf, c->d_cmap, c->d_vcol_send, c->d_vdep_send, c->d_vcol_recv, c->d_vdep_recv,
                    c->d_octree, c->d_passes, c->d_seg_pending, c->d_seg_steps, c->d_pcol_send, c->d_pdep_send, c->d_pcol_recv, c->d_pdep_recv,
                    c->d_strip, c->d_gather, c->d_image, c->d_cache, c->d_counters, c->d_queue, c->d_cvdi_col, c->d_cvdi_dep, c->d_gvdi_col, c->d_gvdi_dep, c->d_cvdi_cnt, c->d_gvdi_cnt, c->d_cpasses, c->d_cseq, c->d_cseq_cursor, c->d_ref_col, c->d_ref_dep,
                    c->d_dbg, c->d_tile_keys, c->d_tile_ids, c->d_sort_tmp, c->d_ref_cnt, c->d_ccol_send, c->d_cdep_send, c->d_meta_send, c->d_meta_recv, c->d_cursor, c->d_staging};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    {   // the other frame slot (pipelined contexts)
        FrameSlot& a = c->alt;
        void* aptrs[] = {a.vcol_send, a.vdep_send, a.octree, a.passes, a.seg_pending, a.seg_steps, a.counters, a.queue,
                         a.cache, a.tile_keys, a.tile_ids, a.sort_tmp};
        for (void* p : aptrs)
            if (p) (void)hipFree(p);
        for (auto& e : a.ev)
            if (e) (void)hipEventDestroy(e);
        if (a.h_ctr) (void)hipHostFree(a.h_ctr);
    }
    if (c->ev_ingest) (void)hipEventDestroy(c->ev_ingest);
    if (c->ev_ingest0) (void)hipEventDestroy(c->ev_ingest0);
    if (c->ev_gate) (void)hipEventDestroy(c->ev_gate);
    if (c->pipe_flag) (void)hipFree(c->pipe_flag);
    for (hipStream_t st : {c->slot_search_stream, c->alt.search_stream})
        if (st) (void)hipStreamDestroy(st);
    if (c->pipe_sample) (void)hipStreamDestroy(c->pipe_sample);
    if (c->pipe_comp) (void)hipStreamDestroy(c->pipe_comp);
    if (c->h_tot) (void)hipHostFree(c->h_tot);
    if (c->h_ctr) (void)hipHostFree(c->h_ctr);
    if (c->h_cseq_demand) (void)hipHostFree(c->h_cseq_demand);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->group && c->rank < (int)c->group->ranks.size() && c->group->ranks[c->rank] == c) c->group->ranks[c->rank] = nullptr;
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
}

bool is_root(const insitu_ctx* c) { return c->rank == 0; }

// exchange the current frame slot's members with `alt` (FrameSlot)
void swap_slot(insitu_ctx* c) {
    FrameSlot& a = c->alt;
    std::swap(c->d_vcol_send, a.vcol_send);
    std::swap(c->d_vdep_send, a.vdep_send);
    std::swap(c->d_octree, a.octree);
    std::swap(c->d_passes, a.passes);
    std::swap(c->d_seg_pending, a.seg_pending);
    std::swap(c->d_seg_steps, a.seg_steps);
    std::swap(c->d_counters, a.counters);
    std::swap(c->d_queue, a.queue);
    std::swap(c->d_cache, a.cache);
    std::swap(c->cache_chunks, a.cache_chunks);
    std::swap(c->cache_grow_to, a.cache_grow_to);
    std::swap(c->cache_sized, a.cache_sized);
    std::swap(c->h_ctr, a.h_ctr);
    std::swap(c->h_ctr_pending, a.h_ctr_pending);
    std::swap(c->h_ctr_valid, a.h_ctr_valid);
    std::swap(c->search_launched, a.search_launched);
    std::swap(c->d_tile_keys, a.tile_keys);
    std::swap(c->d_tile_ids, a.tile_ids);
    std::swap(c->d_sort_tmp, a.sort_tmp);
    std::swap(c->ipv, a.ipv);
    std::swap(c->pv, a.pv);
    std::swap(c->view, a.view);
    std::swap(c->rendered, a.rendered);
    std::swap(c->composited, a.composited);
    std::swap(c->exchanged, a.exchanged);
    std::swap(c->slot_pipelined, a.pipelined);
    std::swap(c->slot_search_stream, a.search_stream);
    std::swap(c->slot_flag_index, a.flag_index);
    std::swap(c->ev, a.ev);
    std::swap(c->ev_valid, a.ev_valid);
}

// the stream the current slot's readbacks run on: a pipelined frame in flight keeps `stream` busy with the
// next frame's search, the completion stream holds nothing of it
hipStream_t read_stream(const insitu_ctx* c) { return c->pipe_inflight ? c->pipe_comp : c->stream; }

// points c->stream at `s` for a scope: the stage and readback functions enqueue on c->stream
struct StreamScope {
    insitu_ctx* c;
    hipStream_t saved;
    StreamScope(insitu_ctx* c_, hipStream_t s) : c(c_), saved(c_->stream) { c->stream = s; }
    ~StreamScope() { c->stream = saved; }
};

// after a stream synchronisation: the last render's cache demand (h_ctr) decides whether a
// default-sized cache grows before the next render
void cache_observe(insitu_ctx* c) {
    if (c->cseq_pending) {   // the compositor merge cache's demand (insitu_composite grows it)
        c->cseq_pending = false;
        c->cseq_demand = *c->h_cseq_demand;
    }
    if (!c->h_ctr_pending) return;
    c->h_ctr_pending = false;
    c->h_ctr_valid = true;
    if (!c->cache_adaptive || c->h_ctr->march_rays == 0) return;
    const unsigned long long want = c->h_ctr->cache_cursor + c->h_ctr->cache_cursor / 4;
    const size_t to = std::min((size_t)want, c->cache_max_chunks);
    if (to > c->cache_chunks) c->cache_grow_to = (uint32_t)to;
}

// (re)allocate the sample cache to `chunks` 32-byte units; on failure nothing is left allocated and the
// error is returned
hipError_t cache_realloc(insitu_ctx* c, size_t chunks) {
    if (c->d_cache) (void)hipFree(c->d_cache);
    c->d_cache = nullptr;
    c->cache_chunks = 0;
    hipError_t e = hipMalloc(&c->d_cache, chunks * 32);
    if (e != hipSuccess) {
        if (c->d_cache) (void)hipFree(c->d_cache);
        c->d_cache = nullptr;
        (void)hipGetLastError();
        return e;
    }
    c->cache_chunks = (uint32_t)chunks;
    return hipSuccess;
}

// after a stream synchronisation: did a persistent kernel of the last render hit its wall-clock bound?
int check_fault(insitu_ctx* c) {
    cache_observe(c);   // (a pending copy of the frame's counters reached h_ctr: we are after a synchronisation)
    if (!c->d_counters || !c->search_launched) return 0;
    uint32_t f = 0;
    if (c->h_ctr_valid) f = c->h_ctr->fault;
    else if (hipMemcpy(&f, &c->d_counters->fault, sizeof f, hipMemcpyDeviceToHost) != hipSuccess) f = 1;
    if (f) return fail(c, -6, "VDI search kernel exceeded its loop bound (internal error)");
    return 0;
}

// this rank's composited-VDI strip block (the root composites straight into its gather slot)
float4* cvdi_col(const insitu_ctx* c) { return c->rank == 0 ? c->d_gvdi_col : c->d_cvdi_col; }
float2* cvdi_dep(const insitu_ctx* c) { return c->rank == 0 ? c->d_gvdi_dep : c->d_cvdi_dep; }
uint16_t* cvdi_cnt(const insitu_ctx* c) { return c->rank == 0 ? c->d_gvdi_cnt : c->d_cvdi_cnt; }

void record_on(insitu_ctx* c, int i, hipStream_t s) {
    if (hipEventRecord(c->ev[i], s) == hipSuccess) c->ev_valid[i] = true;
}
void record(insitu_ctx* c, int i) { record_on(c, i, c->stream); }

// N > 1, VDI mode: pack the stored supersegments of the current slot's blocks bound for the other ranks into
// the compact messages (vdi_compact_kernel), on `stream`, between events [6] and [12]
hipError_t compact_enqueue(insitu_ctx* c) {
    record(c, 6);
    hipError_t e = hipMemsetAsync(c->d_cursor, 0, sizeof(uint32_t) * (size_t)c->N, c->stream);
    if (e != hipSuccess) return e;
    CompactParams cp{};
    cp.col = c->d_vcol_send;
    cp.dep = c->d_vdep_send;
    cp.pend = c->d_seg_pending;
    cp.pend_stride = (size_t)c->W * (size_t)c->H;
    cp.W = c->W; cp.H = c->H; cp.S = c->S; cp.B = c->BV; cp.nstrips = c->N; cp.strip_w = c->strip_w;
    cp.strip_tiles = c->strip_tiles; cp.ytiles = (c->H + 7) / 8; cp.skip_d = c->rank;
    cp.blockE = c->blockE;
    cp.out_col = c->d_ccol_send;
    cp.out_dep = c->d_cdep_send;
    cp.out_meta = c->d_meta_send;
    cp.meta_bytes = c->meta_bytes;
    cp.cursor = c->d_cursor;
    e = launch_vdi_compact(cp, c->stream);
    if (e == hipSuccess) record(c, 12);
    return e;
}

// local group: before this rank rewrites buffers its peers copy from (send blocks, counts, strips),
// order its stream after the peers' last reads of them (write-after-read across streams)
hipError_t wait_peer_reads(insitu_ctx* c) {
    if (!c->group) return hipSuccess;
    for (const insitu_ctx* q : c->group->ranks) {
        if (!q || q == c || !q->ev_valid[7]) continue;
        hipError_t e = hipStreamWaitEvent(c->stream, q->ev[7], 0);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// allocate one frame slot's generator buffers (VDI mode): send blocks, octree counters, pass counts, pending
// counts and step counts, generator counters, and -- with a sample cache of `chunks` 32-byte units -- the
// cache, the search queue, the pinned counter copy and the tile-order keys; plus the slot's events
int alloc_slot(insitu_ctx* c, FrameSlot& f, size_t chunks) {
    int rc = 0;
    for (auto& ev : f.ev)
        if (!ev && hipEventCreate(&ev) != hipSuccess) return fail(c, -3, "hipEventCreate failed");
    const size_t sendE = (size_t)c->N * (size_t)c->BV * c->blockE;
    const size_t px = (size_t)c->BV * (size_t)c->W * (size_t)c->H;
    if ((rc = dev_alloc(c, &f.vcol_send, sendE)) || (rc = dev_alloc(c, &f.vdep_send, sendE))) return rc;
    const size_t oct = (size_t)c->BV * (size_t)c->S * (size_t)c->ncx * (size_t)c->ncy;
    if ((rc = dev_alloc(c, &f.octree, oct ? oct : 1))) return rc;
    if ((rc = dev_alloc(c, &f.seg_pending, px)) || (rc = dev_alloc(c, &f.seg_steps, sendE))) return rc;
    // per-pixel supersegment counts: empty until the first render (the slots are not zero-filled)
    if (hipMemset(f.seg_pending, 0, sizeof(uint16_t) * px) != hipSuccess)
        return fail(c, -3, "hipMemset of the supersegment counts failed");
    if (c->cfg.keep_passes && (rc = dev_alloc(c, &f.passes, px))) return rc;
    // generator counters, zeroed here so the fault flag reads 0 before any render (the host-buffer path
    // never renders)
    if ((rc = dev_alloc(c, &f.counters, 1))) return rc;
    if (hipMemset(f.counters, 0, sizeof(GenCounters)) != hipSuccess)
        return fail(c, -3, "hipMemset of the generator counters failed");
    if (chunks == 0) return 0;
    if ((rc = dev_alloc(c, &f.cache, chunks * 8)) || (rc = dev_alloc(c, &f.queue, (size_t)c->B * (size_t)c->W * (size_t)c->H)))
        return rc;
    if (hipHostMalloc((void**)&f.h_ctr, sizeof(GenCounters), 0) != hipSuccess)
        return fail(c, -5, "hipHostMalloc of the generator counters failed");
    std::memset(f.h_ctr, 0, sizeof(GenCounters));
    f.cache_chunks = (uint32_t)chunks;
    // longest-tiles-first order of the sampling kernel: keys, ids and the sort's scratch (the key keeps 24
    // bits of tile position; super-tiles of up to 4x4 tiles pad the grid, so larger frames keep the order
    // only with super_tile 1: insitu_set_option checks that)
    const size_t ntile = (size_t)c->B * (size_t)((c->H + 7) / 8) * (size_t)c->N * (size_t)c->strip_tiles;
    if (ntile < ((size_t)1 << 24)) {
        size_t tb = 0;
        if (sort_tiles_desc(nullptr, tb, nullptr, nullptr, nullptr, nullptr, (int)ntile, nullptr) != hipSuccess)
            return fail(c, -3, "hipcub radix sort: temporary storage query failed");
        if ((rc = dev_alloc(c, &f.tile_keys, 2 * ntile)) || (rc = dev_alloc(c, &f.tile_ids, 2 * ntile)) ||
            (rc = dev_alloc(c, &f.sort_tmp, tb + 1)))
            return rc;
        c->sort_tmp_bytes = tb;
    }
    return 0;
}

// the padded tile count of super-tiles of `sup` tiles per edge: the sort key keeps 24 bits of tile position
size_t padded_tiles(const insitu_ctx* c, int sup) {
    return (size_t)c->B * (size_t)((((c->H + 7) / 8) + sup - 1) / sup * sup) *
           (size_t)((c->N * c->strip_tiles + sup - 1) / sup * sup);
}

}  // namespace

extern "C" {

int insitu_abi_version(void) { return INSITU_ABI_VERSION; }

int insitu_local_group_create(int nranks, insitu_local_group** out) {
    if (!out || nranks < 1 || nranks > kMaxLists) return fail(nullptr, -1, "insitu_local_group_create: bad arguments");
    *out = new insitu_local_group();
    (*out)->ranks.assign((size_t)nranks, nullptr);
    return 0;
}

void insitu_local_group_destroy(insitu_local_group* g) { delete g; }

int insitu_comm_id(void* out, size_t cap) {
    if (!out || cap < sizeof(ncclUniqueId)) return fail(nullptr, -1, "insitu_comm_id: buffer too small");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(nullptr, -4, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(out, &id, sizeof id);
    return 0;
}

const char* insitu_last_error(const insitu_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int insitu_create(const insitu_config* cfg, insitu_ctx** out) {
    if (!cfg || !out) return fail(nullptr, -1, "insitu_create: null argument");
    *out = nullptr;
    const insitu_config& k = *cfg;
    if (k.nranks < 1 || k.rank < 0 || k.rank >= k.nranks) return fail(nullptr, -1, "insitu_create: bad rank/nranks");
    if (k.width <= 0 || k.height <= 0) return fail(nullptr, -1, "insitu_create: bad window size");
    if (k.mode != INSITU_MODE_VDI && k.mode != INSITU_MODE_PLAIN) return fail(nullptr, -1, "insitu_create: bad mode");
    if (k.bricks_per_rank < 1 || k.bricks_per_rank > kMaxBricks)
        return fail(nullptr, -1, "insitu_create: bricks_per_rank must be in [1," + std::to_string(kMaxBricks) + "]");
    if (k.nranks * k.bricks_per_rank > kMaxLists)
        return fail(nullptr, -1, "insitu_create: nranks*bricks_per_rank exceeds " + std::to_string(kMaxLists));
    if (k.mode == INSITU_MODE_VDI && (k.max_supersegments < 1 || k.max_supersegments > 255))
        return fail(nullptr, -1, "insitu_create: max_supersegments must be in [1,255]");
    if (k.mode == INSITU_MODE_VDI && k.width % k.nranks != 0)
        return fail(nullptr, -1, "insitu_create: width must divide evenly into nranks screen strips");
    if (k.mode == INSITU_MODE_PLAIN && k.height % k.nranks != 0)
        return fail(nullptr, -1, "insitu_create: height (texture dim1) must divide evenly into nranks strips");
    if (k.nranks > 1 && !k.comm_id && !k.local_group)
        return fail(nullptr, -1, "insitu_create: comm_id (or local_group) required when nranks > 1");
    if (k.local_group && ((int)k.local_group->ranks.size() != k.nranks || k.local_group->ranks[k.rank]))
        return fail(nullptr, -1, "insitu_create: local_group size differs from nranks, or rank already taken");
    if (k.composite_vdi && k.mode != INSITU_MODE_VDI)
        return fail(nullptr, -1, "insitu_create: composite_vdi needs VDI mode");
    if (k.merge_bricks && k.mode != INSITU_MODE_VDI)
        return fail(nullptr, -1, "insitu_create: merge_bricks needs VDI mode");
    if (k.max_output_supersegments < 0 || k.max_output_supersegments > 255)
        return fail(nullptr, -1, "insitu_create: max_output_supersegments must be in [0,255]");
    if (k.faithful & ~(INSITU_FAITHFUL_COMPOSITOR_NDC_X | INSITU_FAITHFUL_PLAIN_NUM_PROCESSES))
        return fail(nullptr, -1, "insitu_create: unknown faithful bits");

    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return fail(nullptr, -2, "insitu_create: no HIP device available");
    if (k.device < 0 || k.device >= ndev) return fail(nullptr, -2, "insitu_create: device index out of range");
    e = hipSetDevice(k.device);
    if (e != hipSuccess) return fail(nullptr, -2, std::string("hipSetDevice: ") + hipGetErrorString(e));

    insitu_ctx* c = new insitu_ctx();
    c->cfg = k;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, k.device) == hipSuccess && prop.multiProcessorCount > 0)
            c->num_cus = prop.multiProcessorCount;
    }
    c->cfg.comm_id = nullptr;
    c->W = k.width; c->H = k.height; c->N = k.nranks; c->rank = k.rank; c->B = k.bricks_per_rank;
    c->BV = (k.mode == INSITU_MODE_VDI && k.merge_bricks) ? 1 : c->B;
    c->V = c->N * c->BV; c->mode = k.mode;
    c->S = (k.mode == INSITU_MODE_VDI) ? k.max_supersegments : 1;
    c->bricks.resize(c->B);
    int rc = 0;
    auto bail = [&](int code) { std::string m = c->err; release(c); delete c; g_create_error = m; return code; };
    if (k.stream) {
        c->stream = (hipStream_t)k.stream;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            c->err = "hipStreamCreate failed";
            return bail(-3);
        }
        c->own_stream = true;
    }
    for (auto& ev : c->ev)
        if (hipEventCreate(&ev) != hipSuccess) { c->err = "hipEventCreate failed"; return bail(-3); }
    if (hipEventCreate(&c->ev_ingest0) != hipSuccess || hipEventCreate(&c->ev_ingest) != hipSuccess ||
        hipEventCreate(&c->ev_gate) != hipSuccess) {
        c->err = "hipEventCreate failed";
        return bail(-3);
    }

    if (c->mode == INSITU_MODE_VDI) {
        c->strip_w = c->W / c->N;
        c->strip_tiles = (c->strip_w + 7) / 8;
        c->blockE = (size_t)c->strip_tiles * (size_t)c->S * (size_t)c->H * 8;
        c->stripPx = (size_t)c->H * (size_t)c->strip_w;
        c->ncx = c->W / 8; c->ncy = c->H / 8;
        const size_t sendE = (size_t)c->N * (size_t)c->BV * c->blockE;
        if (c->N > 1) {
            // compact exchange: send regions per destination, receive regions per source, meta blocks
            c->meta_bytes = compact_meta_bytes(c->BV, c->strip_tiles, (c->H + 7) / 8);
            if ((rc = dev_alloc(c, &c->d_vcol_recv, sendE)) || (rc = dev_alloc(c, &c->d_vdep_recv, sendE)) ||
                (rc = dev_alloc(c, &c->d_ccol_send, sendE)) || (rc = dev_alloc(c, &c->d_cdep_send, sendE)) ||
                (rc = dev_alloc(c, &c->d_meta_send, (size_t)c->N * c->meta_bytes)) ||
                (rc = dev_alloc(c, &c->d_meta_recv, (size_t)c->N * c->meta_bytes)) ||
                (rc = dev_alloc(c, &c->d_cursor, 2 * (size_t)c->N)))
                return bail(rc);
            // received counts/offsets read as empty lists until the first exchange fills them
            if (hipMemset(c->d_meta_recv, 0, (size_t)c->N * c->meta_bytes) != hipSuccess) {
                c->err = "hipMemset of the exchange meta blocks failed";
                return bail(-3);
            }
            if (hipHostMalloc((void**)&c->h_tot, 2 * sizeof(uint32_t) * (size_t)c->N, 0) != hipSuccess) {
                c->err = "hipHostMalloc of the exchange totals failed";
                return bail(-5);
            }
        }
        size_t chunks = 0;
        bool start_knob = false;
        if (k.sample_cache_mb >= 0) {
            // default: 512 B (64 samples of 8 B) per pixel per brick to start with (config 2 asks for
            // 4.1 GB = 250 B per pixel per brick), grown after a frame
            // whose rays did not fit to 1.25x that frame's demand, up to 45 % of the HBM free at create
            // (this is an in-situ library: the simulation shares the GPU, so the cache takes what the
            // frames need, not what is free).  Rays that do not fit are searched by re-sampling (same
            // results, slower) and counted (insitu_stats.rays_uncached).  sample_cache_mb > 0 fixes it.
            size_t freeb = 0, totalb = 0;
            if (hipMemGetInfo(&freeb, &totalb) != hipSuccess) freeb = (size_t)32 << 30;
            c->cache_max_chunks = std::min(freeb / 20 * 9 / 32, (size_t)0xffffffffu);
            size_t bytes = (size_t)k.sample_cache_mb << 20;
            if (k.sample_cache_mb == 0) {
                bytes = std::min((size_t)c->B * (size_t)c->W * (size_t)c->H * 512, c->cache_max_chunks * 32);
                c->cache_adaptive = true;
            }
            chunks = std::min(bytes / 32, (size_t)0xffffffffu);
            if (const char* v = std::getenv("INSITU_CACHE_START_CHUNKS")) {
                // test knob: a default-sized cache that starts at this size, below the first frame's
                // demand (no first-frame sizing), so the growth path runs (tests/test_gpu_parity.py)
                if (c->cache_adaptive && std::atoll(v) > 0) {
                    chunks = std::min((size_t)std::atoll(v), c->cache_max_chunks);
                    start_knob = true;
                }
            }
            if (chunks > 0) c->search_blocks = c->num_cus * 8;   // 32 waves per CU; waves that find the queue drained exit
        }
        // the frame slot's buffers, allocated into `alt` and swapped in (a pipelined context allocates the
        // second slot at its first pipelined frame)
        rc = alloc_slot(c, c->alt, chunks);
        swap_slot(c);
        if (rc) return bail(rc);
        if (chunks > 0 && start_knob) c->cache_sized = true;
        if (const char* dbg = std::getenv("INSITU_DEBUG_RAYS")) {   // diagnostics (tools/ray_timing.py)
            if (c->d_queue) {
                c->dbg_entries = (size_t)c->BV * (size_t)c->W * (size_t)c->H;
                if ((rc = dev_alloc(c, &c->d_dbg, c->dbg_entries * 4))) return bail(rc);
                c->dbg_path = dbg;
            }
        }
        if (is_root(c)) {
            if ((rc = dev_alloc(c, &c->d_gather, (size_t)c->N * c->stripPx)) ||
                (rc = dev_alloc(c, &c->d_image, (size_t)c->W * (size_t)c->H)))
                return bail(rc);
        } else if ((rc = dev_alloc(c, &c->d_strip, c->stripPx))) {
            return bail(rc);
        }
        if (k.composite_vdi) {
            c->composite_vdi = true;
            c->S_out = k.max_output_supersegments > 0 ? k.max_output_supersegments : c->S;
            c->cblockE = (size_t)c->strip_tiles * (size_t)c->S_out * (size_t)c->H * 8;
            if ((rc = dev_alloc(c, &c->d_cpasses, c->stripPx))) return bail(rc);
            // merge cache of the compositor: an eighth of the V*S entries per pixel to start with, grown to
            // a composite's demand when it did not fit (the waves that found no room merge every pass)
            // growth budget: 20 % of the HBM free at create (the simulation and the sample cache share the GPU)
            size_t freeb = 0, totalb = 0;
            if (hipMemGetInfo(&freeb, &totalb) != hipSuccess) freeb = (size_t)32 << 30;
            c->cseq_max = std::max<unsigned long long>(64ull * 64ull, (unsigned long long)(freeb / 5 / (16 * kCompEntryF4)));
            c->cseq_cap = std::min(c->cseq_max, std::max<unsigned long long>(
                64ull * 64ull, (unsigned long long)c->V * c->stripPx * (unsigned long long)c->S / 8));
            if ((rc = dev_alloc(c, &c->d_cseq, (size_t)kCompEntryF4 * (size_t)c->cseq_cap)) || (rc = dev_alloc(c, &c->d_cseq_cursor, 1)))
                return bail(rc);
            if (hipHostMalloc((void**)&c->h_cseq_demand, sizeof(unsigned long long), 0) != hipSuccess) {
                c->err = "hipHostMalloc of the compositor demand failed";
                return bail(-5);
            }
            *c->h_cseq_demand = 0;
            if (is_root(c)) {
                if ((rc = dev_alloc(c, &c->d_gvdi_col, (size_t)c->N * c->cblockE)) ||
                    (rc = dev_alloc(c, &c->d_gvdi_dep, (size_t)c->N * c->cblockE)) ||
                    (rc = dev_alloc(c, &c->d_gvdi_cnt, (size_t)c->N * c->stripPx)))
                    return bail(rc);
            } else if ((rc = dev_alloc(c, &c->d_cvdi_col, c->cblockE)) || (rc = dev_alloc(c, &c->d_cvdi_dep, c->cblockE)) ||
                       (rc = dev_alloc(c, &c->d_cvdi_cnt, c->stripPx))) {
                return bail(rc);
            }
        }
    } else {
        c->rows = c->H / c->N;
        c->plainBlock = (size_t)c->rows * (size_t)c->W;
        c->stripPx = c->plainBlock;
        const size_t sendPx = (size_t)c->N * (size_t)c->B * c->plainBlock;
        if ((rc = dev_alloc(c, &c->d_pcol_send, sendPx)) || (rc = dev_alloc(c, &c->d_pdep_send, sendPx))) return bail(rc);
        if (c->N > 1)
            if ((rc = dev_alloc(c, &c->d_pcol_recv, sendPx)) || (rc = dev_alloc(c, &c->d_pdep_recv, sendPx))) return bail(rc);
        if (is_root(c)) {
            if ((rc = dev_alloc(c, &c->d_gather, (size_t)c->N * c->stripPx))) return bail(rc);
        } else if ((rc = dev_alloc(c, &c->d_strip, c->stripPx))) {
            return bail(rc);
        }
    }
    if (k.local_group) {
        c->group = k.local_group;
        c->group->ranks[c->rank] = c;
    } else if (c->N > 1) {
        ncclUniqueId id;
        std::memcpy(&id, k.comm_id, sizeof id);
        ncclResult_t r = ncclCommInitRank(&c->comm, c->N, id, c->rank);
        if (r != ncclSuccess) {
            c->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            c->comm = nullptr;
            return bail(-4);
        }
    }
    {   // tuning seeds from the environment (tools/knob_sweep.sh); insitu_set_option overrides
        const struct { const char* name; int opt; } names[] = {
            {"INSITU_EXACT_SEARCH", INSITU_OPT_EXACT_SEARCH}, {"INSITU_SEARCH_DEPTH", INSITU_OPT_SEARCH_DEPTH},
            {"INSITU_LONG_SAMPLES", INSITU_OPT_LONG_SAMPLES}, {"INSITU_ROUND_BATCH", INSITU_OPT_ROUND_BATCH},
            {"INSITU_SEARCH_OVERSUB", INSITU_OPT_SEARCH_OVERSUB}, {"INSITU_TILE_ORDER", INSITU_OPT_TILE_ORDER},
            {"INSITU_SUPER_TILE", INSITU_OPT_SUPER_TILE}, {"INSITU_REGROUP", INSITU_OPT_REGROUP},
            {"INSITU_EXACT_TILE_KEYS", INSITU_OPT_EXACT_TILE_KEYS}, {"INSITU_PIPE_TRIGGER", INSITU_OPT_PIPE_TRIGGER},
            {"INSITU_PIPE_OVERSUB", INSITU_OPT_PIPE_OVERSUB}, {"INSITU_PIPE_SEARCH_RAYS", INSITU_OPT_PIPE_SEARCH_RAYS}};
        for (const auto& nm : names) {
            if (const char* v = std::getenv(nm.name)) {
                if (insitu_set_option(c, nm.opt, std::atoll(v)) != 0) {
                    c->err = std::string("insitu_create: ") + nm.name + "=" + v + " out of range";
                    return bail(-1);
                }
            }
        }
    }
    *out = c;
    return 0;
}

int insitu_set_option(insitu_ctx* c, int option, long long v) {
    if (!c) return fail(nullptr, -1, "insitu_set_option: null context");
    Tuning& t = c->tune;
    switch (option) {
    case INSITU_OPT_EXACT_SEARCH:
        if (v != 0 && v != 1) break;
        t.exact_search = v;
        return 0;
    case INSITU_OPT_SEARCH_DEPTH:
        if (v < 0 || v > 6) break;
        t.search_depth = v;
        return 0;
    case INSITU_OPT_LONG_SAMPLES:
        if (v < 0 || v > 0xffffffffll) break;
        t.long_samples = v;
        return 0;
    case INSITU_OPT_ROUND_BATCH:
        if (v < 1 || v > 64) break;
        t.round_batch = v;
        return 0;
    case INSITU_OPT_SEARCH_OVERSUB:
        if (v < 1 || v > 64) break;
        t.search_oversub = v;
        return 0;
    case INSITU_OPT_TILE_ORDER:
        if (v != 0 && v != 1) break;
        t.tile_order = v;
        return 0;
    case INSITU_OPT_SUPER_TILE:
        if (v != 1 && v != 2 && v != 4) break;
        if (v > 1 && c->mode == INSITU_MODE_VDI && padded_tiles(c, (int)v) >= ((size_t)1 << 24))
            return fail(c, -1, "insitu_set_option: super-tiles of " + std::to_string(v) +
                                   " tiles pad this frame's tile grid past the sort key's 24 bits of position");
        t.super_tile = v;
        return 0;
    case INSITU_OPT_REGROUP:
        if (v != 0 && v != 1) break;
        t.regroup = v;
        return 0;
    case INSITU_OPT_EXACT_TILE_KEYS:
        if (v != 0 && v != 1) break;
        t.exact_tile_keys = v;
        return 0;
    case INSITU_OPT_PIPE_TRIGGER:
        if (v < 0 || v > 2) break;
        c->pipe_trigger = (int)v;
        return 0;
    case INSITU_OPT_PIPE_OVERSUB:
        if (v < 1 || v > 64) break;
        t.pipe_oversub = v;
        return 0;
    case INSITU_OPT_PIPE_SEARCH_RAYS:
        if (v < 0 || v > (1ll << 24)) break;
        t.pipe_search_rays = v;
        return 0;

    default:
        return fail(c, -1, "insitu_set_option: unknown option " + std::to_string(option));
    }
    return fail(c, -1, "insitu_set_option: value " + std::to_string(v) + " out of range for option " +
                           std::to_string(option));
}

void insitu_destroy(insitu_ctx* ctx) {
    release(ctx);
    delete ctx;
}

void* insitu_stream(insitu_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int insitu_set_brick(insitu_ctx* c, int slot, const void* data, int dtype, const int dims[3], const float model[16],
                     int data_on_device) {
    if (!c) return fail(nullptr, -1, "insitu_set_brick: null context");
    if (slot < 0 || slot >= c->B) return fail(c, -1, "insitu_set_brick: slot out of range");
    if (!data || !dims || !model) return fail(c, -1, "insitu_set_brick: null argument");
    if (dtype != INSITU_U8 && dtype != INSITU_U16 && dtype != INSITU_F32) return fail(c, -1, "insitu_set_brick: bad dtype");
    if (dims[0] < 1 || dims[1] < 1 || dims[2] < 1) return fail(c, -1, "insitu_set_brick: bad dims");
    const size_t vox = (size_t)dims[0] * (size_t)dims[1] * (size_t)dims[2];
    if (vox >= (size_t)1 << 32) return fail(c, -1, "insitu_set_brick: brick exceeds 2^32 voxels");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    Brick& b = c->bricks[slot];
    const size_t nb = (size_t)((dims[0] + 7) / 8) * (size_t)((dims[1] + 7) / 8) * (size_t)((dims[2] + 7) / 8);
    if (nb * 729 >= (size_t)1 << 32) return fail(c, -1, "insitu_set_brick: blocked brick exceeds 2^32 voxels");
    const size_t bytes = nb * 729 * dtype_size(dtype);   // blocked layout with halo (insitu_sampling.h)
    if (b.bytes != bytes) {
        if (b.d) HIPCHK(c, hipFree(b.d));
        b.d = nullptr;
        b.bytes = 0;
        HIPCHK(c, hipMalloc(&b.d, bytes));
        b.bytes = bytes;
    }
    if (!mat4_inverse(model, b.im)) return fail(c, -1, "insitu_set_brick: model matrix is singular");
    b.dtype = dtype;
    std::memcpy(b.dims, dims, sizeof b.dims);
    b.valid = false;
    // a pipelined frame in flight may still sample this brick (its first pass, and its search re-samples rays
    // without cache space): the ingest waits for that frame's search
    if (c->pipe_inflight && c->alt.ev_valid[13]) HIPCHK(c, hipStreamWaitEvent(c->stream, c->alt.ev[13], 0));
    if (!c->ingest_batch) {   // the first re-ingest since the last render: the batch's GPU time starts here
        HIPCHK(c, hipEventRecord(c->ev_ingest0, c->stream));
        c->ingest_batch = true;
    }
    if (data_on_device) {
        // in-situ: the simulation's device array is read in place by the ingest kernel
        HIPCHK(c, launch_brick_ingest(data, b.d, dtype, dims[0], dims[1], dims[2], c->stream));
        HIPCHK(c, hipEventRecord(c->ev_ingest, c->stream));
    } else {
        // the staging buffer is kept across calls: the reference re-uploads every grid every 20 frames
        // (DistributedVolumeRenderer.kt:521-527); a pinned source makes the copy a DMA at link speed
        const size_t src_bytes = vox * dtype_size(dtype);
        if (c->staging_bytes < src_bytes) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            if (c->d_staging) HIPCHK(c, hipFree(c->d_staging));
            c->d_staging = nullptr;
            c->staging_bytes = 0;
            HIPCHK(c, hipMalloc(&c->d_staging, src_bytes));
            c->staging_bytes = src_bytes;
        }
        hipError_t e = hipMemcpyAsync(c->d_staging, data, src_bytes, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = launch_brick_ingest(c->d_staging, b.d, dtype, dims[0], dims[1], dims[2], c->stream);
        if (e == hipSuccess) e = hipEventRecord(c->ev_ingest, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);   // host buffer may be reused by the caller
        if (e != hipSuccess) return fail(c, -3, std::string("insitu_set_brick: ") + hipGetErrorString(e));
    }
    b.valid = true;
    return 0;
}

int insitu_set_transfer(insitu_ctx* c, const float* tf, int n_tf, const float* cmap, int n_cm, float conv_scale,
                        float conv_offset) {
    if (!c) return fail(nullptr, -1, "insitu_set_transfer: null context");
    if (!tf || !cmap || n_tf < 1 || n_cm < 1 || n_tf > 8192 || n_cm > 4096)
        return fail(c, -1, "insitu_set_transfer: bad LUTs (1..8192 tf texels, 1..4096 colour texels)");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    {   // the generator kernels stage the LUTs in LDS beside their own per-block state: refuse LUTs that would
        // not fit a block here rather than fail at the next kernel launch
        int max_lds = 0;
        HIPCHK(c, hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, c->cfg.device));
        const size_t need = vdi_generator_lds_bytes(n_tf, n_cm);
        if (c->mode == INSITU_MODE_VDI && max_lds > 0 && need > (size_t)max_lds)
            return fail(c, -1, "insitu_set_transfer: LUTs of " + std::to_string(n_tf) + " + " + std::to_string(n_cm) +
                                   " texels need " + std::to_string(need) + " bytes of LDS per block; the device has " +
                                   std::to_string(max_lds));
    }
    if (n_tf != c->n_tf) {
        if (c->d_tf) HIPCHK(c, hipFree(c->d_tf));
        c->d_tf = nullptr;
        HIPCHK(c, hipMalloc(&c->d_tf, sizeof(float) * n_tf));
        c->n_tf = n_tf;
    }
    if (n_cm != c->n_cm) {
        if (c->d_cmap) HIPCHK(c, hipFree(c->d_cmap));
        c->d_cmap = nullptr;
        HIPCHK(c, hipMalloc(&c->d_cmap, sizeof(float) * 4 * n_cm));
        c->n_cm = n_cm;
    }
    // the colour bound of the filtered decisions' margin (vdi_generate.hip, filter_margin)
    double cm_max = 0.0, tf_max = 0.0;
    bool finite = true;
    for (int i = 0; i < n_cm; ++i)
        for (int k = 0; k < 3; ++k) {
            finite = finite && std::isfinite(cmap[4 * i + k]);
            cm_max = std::max(cm_max, (double)std::fabs(cmap[4 * i + k]));
        }
    for (int i = 0; i < n_tf; ++i) {
        finite = finite && std::isfinite(tf[i]);
        tf_max = std::max(tf_max, (double)std::fabs(tf[i]));
    }
    const double cb = std::max({1.0, 2.0 * cm_max, 2.0 * cm_max * tf_max});
    c->cmag = (finite && cb < 1.0e6) ? (float)cb : std::numeric_limits<float>::infinity();   // inf: exact path only
    if (c->pipe_ready)   // a pipelined frame in flight reads the LUTs
        if (int rc = insitu_synchronize(c)) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_tf, tf, sizeof(float) * n_tf, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_cmap, cmap, sizeof(float) * 4 * n_cm, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->conv_scale = conv_scale;
    c->conv_offset = conv_offset;
    return 0;
}

static BrickDesc brick_desc(const insitu_ctx* c, const Brick& b) {
    BrickDesc d;
    d.data = b.d;
    d.dtype = b.dtype;
    d.nx = b.dims[0]; d.ny = b.dims[1]; d.nz = b.dims[2];
    d.nbx = (d.nx + 7) / 8; d.nby = (d.ny + 7) / 8; d.nbz = (d.nz + 7) / 8;
    std::memcpy(d.im, b.im, sizeof d.im);
    const float norm = b.dtype == INSITU_U8 ? 1.0f / 255.0f : (b.dtype == INSITU_U16 ? 1.0f / 65535.0f : 1.0f);
    d.conv_k = c->conv_scale * norm;
    d.conv_off = c->conv_offset;
    return d;
}

int insitu_set_camera(insitu_ctx* c, const insitu_camera* cam) {
    if (!c) return fail(nullptr, -1, "insitu_set_camera: null context");
    if (!cam) return fail(c, -1, "insitu_set_camera: null camera");
    float iv[16], ip[16];
    if (cam->has_inverses) {
        std::memcpy(iv, cam->inv_view, sizeof iv);
        std::memcpy(ip, cam->inv_proj, sizeof ip);
    } else if (!mat4_inverse(cam->view, iv) || !mat4_inverse(cam->proj, ip)) {
        return fail(c, -1, "insitu_set_camera: view or projection matrix is singular");
    }
    mat4_mul_f(iv, ip, c->ipv);                // VDIGenerator.comp:289 (ipvG of accumulateSupseg)
    mat4_mul_f(cam->proj, cam->view, c->pv);   // VDIGenerator.comp:290
    std::memcpy(c->view, cam->view, sizeof c->view);
    c->camera_set = true;
    return 0;
}

int insitu_render(insitu_ctx* c, const insitu_camera* cam) {
    if (!c) return fail(nullptr, -1, "insitu_render: null context");
    if (!cam) return fail(c, -1, "insitu_render: null camera");
    if (c->pipe_inflight && !c->s_sample)
        return fail(c, -1, "insitu_render: a pipelined frame is in flight (insitu_pipeline_flush first)");
    if (!c->d_tf) return fail(c, -1, "insitu_render: transfer function not set");
    for (int b = 0; b < c->B; ++b) {
        if (!c->bricks[b].valid) return fail(c, -1, "insitu_render: brick slot " + std::to_string(b) + " not set");
        if (c->bricks[b].dtype != c->bricks[0].dtype)
            return fail(c, -1, "insitu_render: all bricks of a rank must share one voxel type");
    }
    if (!(cam->nw > 0.0f)) return fail(c, -1, "insitu_render: nw must be > 0");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    int rc = insitu_set_camera(c, cam);
    if (rc) return rc;
    TransferDesc xf{c->d_tf, c->n_tf, c->d_cmap, c->n_cm, c->cmag};
    HIPCHK(c, wait_peer_reads(c));
    c->ingest_batch = false;
    // the first pass runs on s_sample (a pipelined frame: the sampling stream, behind the trigger the caller
    // enqueued there), the search and the rest on `stream`
    hipStream_t ss = c->s_sample ? c->s_sample : c->stream;
    const bool pipelined = c->s_sample != nullptr;
    hipStream_t sr = pipelined ? c->slot_search_stream : c->stream;   // the search and what follows it
    c->slot_pipelined = pipelined;
    if (!pipelined) record_on(c, 0, ss);   // (pipelined: at the trigger, below)
    if (c->mode == INSITU_MODE_VDI) {
        const size_t oct = (size_t)c->BV * (size_t)c->S * (size_t)c->ncx * (size_t)c->ncy;
        if (oct) HIPCHK(c, hipMemsetAsync(c->d_octree, 0, oct * sizeof(uint32_t), ss));   // GridCellsToZero.comp
        if (c->cache_grow_to > c->cache_chunks) {   // the last frame of this slot's rays did not all fit
            const size_t grow = c->cache_grow_to, old = c->cache_chunks;
            c->cache_grow_to = 0;   // (cleared first: a failure below is not retried every frame)
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipStreamSynchronize(ss));
            HIPCHK(c, hipStreamSynchronize(sr));
            if (cache_realloc(c, grow) != hipSuccess) {
                // keep what fits (the rest re-samples): half the request, never less than the cache
                // that worked, and at most that from now on
                const size_t keep = std::max(old, grow / 2);
                if (cache_realloc(c, keep) != hipSuccess) HIPCHK(c, cache_realloc(c, old));
                c->cache_max_chunks = c->cache_chunks;
            }
        }
        VdiGenParams p{};
        for (int b = 0; b < c->B; ++b) p.bricks[b] = brick_desc(c, c->bricks[b]);
        p.xfer = xf;
        std::memcpy(p.ipv, c->ipv, sizeof p.ipv);
        std::memcpy(p.pv, c->pv, sizeof p.pv);
        std::memcpy(p.view, c->view, sizeof p.view);
        p.nw = cam->nw;
        p.tmax = cam->tmax;
        p.W = c->W; p.H = c->H; p.S = c->S;
        p.strip_w = c->strip_w; p.strip_tiles = c->strip_tiles; p.nstrips = c->N; p.B = c->BV;
        p.nvolumes = c->BV != c->B ? c->B : 0;
        p.ytiles = (c->H + 7) / 8;
        p.color = c->d_vcol_send;
        p.depth = c->d_vdep_send;
        p.octree = c->d_octree;
        p.octree_stride = (size_t)c->S * (size_t)c->ncx * (size_t)c->ncy;
        p.passes = c->d_passes;
        p.passes_stride = (size_t)c->W * (size_t)c->H;
        p.seg_pending = c->d_seg_pending;
        p.seg_steps = c->d_seg_steps;
        p.ncx = c->ncx; p.ncy = c->ncy;
        p.interval_size = (20.0f - 0.1f) / (float)c->S;   // VDIGenerator.comp:241-247
        p.cache = c->d_cache;
        p.split_event = c->ev[5];
        c->ev_valid[5] = true;
        p.cache_chunks = c->cache_chunks;
        p.ctr = c->d_counters;
        p.queue = c->d_queue;
        p.queue_cap = (uint32_t)((size_t)c->BV * (size_t)c->W * (size_t)c->H);
        // longest-first, coarsely: rays with many samples (most work per pass, and the ones with
        // 20+ passes) are searched before the rest, so the frame does not end waiting for a long
        // ray popped late; within each class the queue keeps the sampling kernel's tile order
        p.long_samples = (uint32_t)c->tune.long_samples;
        p.round_batch = (int)c->tune.round_batch;   // (group mode ends rounds at once)
        p.search_blocks = c->search_blocks;
        if (pipelined && c->tune.pipe_search_rays > 0) {
            // the search beside the next frame's first pass: one to two blocks per CU by the queue length, the
            // rest of each CU's wave slots left to that first pass
            p.search_blocks = std::min(c->search_blocks, 2 * c->num_cus);
            p.search_block_rays = (int)c->tune.pipe_search_rays;
            p.search_min_blocks = std::min(p.search_blocks, c->num_cus);
        }
        p.search_oversub = (int)(pipelined ? c->tune.pipe_oversub : c->tune.search_oversub);
        p.search_depth = (int)c->tune.search_depth;
        p.regroup = (int)c->tune.regroup;
        p.exact_search = (int)c->tune.exact_search;
        if (c->d_cache && (c->search_lanes_tf != c->n_tf || c->search_lanes_cm != c->n_cm)) {
            // lanes the search grid keeps resident on this device with these LUT sizes (LDS)
            HIPCHK(c, vdi_search_resident_lanes(c->n_tf, c->n_cm, c->cfg.device, &c->search_lanes));
            c->search_lanes_tf = c->n_tf;
            c->search_lanes_cm = c->n_cm;
        }
        p.search_lanes = std::min(c->search_lanes, p.search_blocks * 256);
        if (c->tune.tile_order && c->d_tile_keys) {
            p.tile_keys = c->d_tile_keys;
            p.super_tile = (int)c->tune.super_tile;
            p.tile_len_exact = (int)c->tune.exact_tile_keys;
            p.tile_ids = c->d_tile_ids;
            p.sort_tmp = c->d_sort_tmp;
            p.sort_tmp_bytes = c->sort_tmp_bytes;
        }
        if (pipelined && c->d_cache && c->pipe_flag && c->pipe_trigger == 1) {
            p.pipe_flag = c->pipe_flag + c->slot_flag_index;   // this search's queue drain starts the next first pass
            p.pipe_seq = c->pipe_seq;
        }
        // counters zeroed, tile keys (and, on a default cache's first frame, the frame's cache demand) sorted
        p.measure_cache = (c->cache_adaptive && !c->cache_sized && p.nvolumes == 0) ? 1 : 0;
        HIPCHK(c, launch_vdi_prepare(p, ss));
        p.prepared = 1;
        if (p.measure_cache && c->d_cache && p.tile_ids) {
            // the first frame of a default-sized cache: wait for the demand the tile keys measured and
            // size the cache to it (later frames grow it from their own demand, cache_observe)
            unsigned long long need = 0;
            HIPCHK(c, hipMemcpyAsync(&need, &c->d_counters->cache_need, sizeof need, hipMemcpyDeviceToHost, ss));
            HIPCHK(c, hipStreamSynchronize(ss));
            c->cache_sized = true;
            const size_t want = std::min((size_t)(need + need / 4 + 64), c->cache_max_chunks);
            if (want > c->cache_chunks) HIPCHK(c, cache_realloc(c, want));
            p.cache = c->d_cache;
            p.cache_chunks = c->cache_chunks;
        }
        if (pipelined) {
            // the trigger (insitu_frame_pipelined): the prepare above only touches this slot's buffers, so its
            // small launches are already queued when the previous frame's search lets the first pass start;
            // the frame's render time and latency count from here
            if (c->trig_flag)
                HIPCHK(c, hipStreamWaitValue64(ss, c->trig_flag, c->trig_value, hipStreamWaitValueGte));
            else if (c->trig_event)
                HIPCHK(c, hipStreamWaitEvent(ss, c->trig_event, 0));
            record_on(c, 0, ss);
        }
        if (c->d_dbg && !pipelined) {
            HIPCHK(c, hipMemsetAsync(c->d_dbg, 0, c->dbg_entries * 32, ss));
            p.debug_rays = c->d_dbg;
            p.debug_cap = (uint32_t)std::min(c->dbg_entries, (size_t)0xffffffffu);
            c->dbg_pending = true;   // written to INSITU_DEBUG_RAYS at the next insitu_synchronize
        }
        HIPCHK(c, launch_vdi_sample(p, ss));
        if (ss != sr) HIPCHK(c, hipStreamWaitEvent(sr, c->ev[5], 0));        HIPCHK(c, launch_vdi_search(p, sr));
        c->search_launched = c->d_cache != nullptr;
        if (pipelined) {
            // the next frame's trigger: the search is over (mode 0), or -- the flag's safety net when no wave
            // crossed the trigger point (an empty queue) -- its value is reached (mode 1)
            record_on(c, 13, sr);
            if (p.pipe_flag) HIPCHK(c, hipStreamWriteValue64(sr, p.pipe_flag, c->pipe_seq, 0));
        }
        HIPCHK(c, launch_vdi_finish(p, sr));
        if (c->h_ctr) {   // the frame's counters, read on the host after the next synchronisation
            HIPCHK(c, hipMemcpyAsync(c->h_ctr, c->d_counters, sizeof(GenCounters), hipMemcpyDeviceToHost, sr));
            c->h_ctr_pending = true;
            c->h_ctr_valid = false;
        }
        // variable-length exchange: the stored supersegments of the blocks bound for the other
        // ranks are packed as part of producing the send buffers (timed as the exchange); a pipelined frame
        // packs them with its completion, where the compact buffers are free
        if (c->N > 1 && !pipelined) HIPCHK(c, compact_enqueue(c));
        c->lists_from_reference = false;
    } else {
        PlainGenParams p{};
        for (int b = 0; b < c->B; ++b) p.bricks[b] = brick_desc(c, c->bricks[b]);
        p.xfer = xf;
        std::memcpy(p.ipv, c->ipv, sizeof p.ipv);
        p.nw = cam->nw; p.fwnw = cam->fwnw; p.tmax = cam->tmax;
        p.dim0 = c->W; p.dim1 = c->H; p.rows = c->rows;
        p.nstrips = c->N; p.B = c->B;
        p.color = c->d_pcol_send;
        p.depth = c->d_pdep_send;
        HIPCHK(c, launch_plain_generate(p, c->stream));
    }
    record_on(c, 1, sr);
    c->rendered = true;
    c->composited = false;
    c->exchanged = false;
    return 0;
}

int insitu_exchange(insitu_ctx* c) {
    if (!c) return fail(nullptr, -1, "insitu_exchange: null context");
    if (c->pipe_inflight && !c->completing)
        return fail(c, -1, "insitu_exchange: a pipelined frame is in flight (insitu_pipeline_flush first)");
    if (!c->rendered) return fail(c, -1, "insitu_exchange: nothing rendered");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    c->last_exchange_entries = 0;
    c->last_exchange_bytes = 0;
    if (c->N > 1 && c->mode == INSITU_MODE_VDI) {
        // variable-length exchange of the compact messages (VDICompositingTest.kt:251-305, 360-415:
        // counts first, then MPI_Alltoallv): totals to every peer, the host learns the receive sizes,
        // then grouped send/recv of the meta blocks and of exactly the packed entries
        const size_t region = (size_t)c->BV * c->blockE;
        uint32_t* send_tot = c->h_tot;
        uint32_t* recv_tot = c->h_tot + c->N;
        if (c->group) {   // in-process: the peers packed their blocks in their renders (event [1])
            for (int p = 0; p < c->N; ++p) {
                if (p == c->rank) continue;
                const insitu_ctx* q = c->group->ranks[p];
                if (!q) return fail(c, -1, "insitu_exchange: local group rank " + std::to_string(p) + " missing");
                if (!q->rendered || !q->ev_valid[1]) return fail(c, -1, "insitu_exchange: local group rank " + std::to_string(p) + " has not rendered");
                HIPCHK(c, hipStreamWaitEvent(c->stream, q->ev[1], 0));
                HIPCHK(c, hipMemcpyAsync(recv_tot + p, q->d_cursor + c->rank, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
            }
            HIPCHK(c, hipMemcpyAsync(send_tot, c->d_cursor, sizeof(uint32_t) * (size_t)c->N, hipMemcpyDeviceToHost, c->stream));
            record(c, 8);
            HIPCHK(c, hipStreamSynchronize(c->stream));
            record(c, 9);
            for (int p = 0; p < c->N; ++p) {
                if (p == c->rank) continue;
                const insitu_ctx* q = c->group->ranks[p];
                HIPCHK(c, hipMemcpyAsync(c->d_meta_recv + (size_t)p * c->meta_bytes, q->d_meta_send + (size_t)c->rank * q->meta_bytes,
                                         c->meta_bytes, hipMemcpyDeviceToDevice, c->stream));
                const size_t n = recv_tot[p];
                if (n == 0) continue;
                HIPCHK(c, hipMemcpyAsync(c->d_vcol_recv + (size_t)p * region, q->d_ccol_send + (size_t)c->rank * region,
                                         n * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
                HIPCHK(c, hipMemcpyAsync(c->d_vdep_recv + (size_t)p * region, q->d_cdep_send + (size_t)c->rank * region,
                                         n * sizeof(float2), hipMemcpyDeviceToDevice, c->stream));
            }
        } else {
            NCCLCHK(c, ncclGroupStart());
            for (int p = 0; p < c->N; ++p) {
                if (p == c->rank) continue;
                NCCLCHK(c, ncclSend(c->d_cursor + p, 1, ncclUint32, p, c->comm, c->stream));
                NCCLCHK(c, ncclRecv(c->d_cursor + c->N + p, 1, ncclUint32, p, c->comm, c->stream));
            }
            NCCLCHK(c, ncclGroupEnd());
            HIPCHK(c, hipMemcpyAsync(c->h_tot, c->d_cursor, 2 * sizeof(uint32_t) * (size_t)c->N, hipMemcpyDeviceToHost,
                                     c->stream));
            // the host learns the receive sizes: the stream idles from here ([8]) until the payload
            // group is enqueued ([9]) -- reported as insitu_stats.ms_exchange_sync
            record(c, 8);
            HIPCHK(c, hipStreamSynchronize(c->stream));
            record(c, 9);
            NCCLCHK(c, ncclGroupStart());
            for (int p = 0; p < c->N; ++p) {
                if (p == c->rank) continue;
                NCCLCHK(c, ncclSend(c->d_meta_send + (size_t)p * c->meta_bytes, c->meta_bytes, ncclUint8, p, c->comm, c->stream));
                NCCLCHK(c, ncclRecv(c->d_meta_recv + (size_t)p * c->meta_bytes, c->meta_bytes, ncclUint8, p, c->comm, c->stream));
                if (send_tot[p]) {
                    NCCLCHK(c, ncclSend(c->d_ccol_send + (size_t)p * region, (size_t)send_tot[p] * 4, ncclFloat32, p, c->comm, c->stream));
                    NCCLCHK(c, ncclSend(c->d_cdep_send + (size_t)p * region, (size_t)send_tot[p] * 2, ncclFloat32, p, c->comm, c->stream));
                }
                if (recv_tot[p]) {
                    NCCLCHK(c, ncclRecv(c->d_vcol_recv + (size_t)p * region, (size_t)recv_tot[p] * 4, ncclFloat32, p, c->comm, c->stream));
                    NCCLCHK(c, ncclRecv(c->d_vdep_recv + (size_t)p * region, (size_t)recv_tot[p] * 2, ncclFloat32, p, c->comm, c->stream));
                }
            }
            NCCLCHK(c, ncclGroupEnd());
        }
        for (int p = 0; p < c->N; ++p) {
            if (p == c->rank) continue;
            c->last_exchange_entries += send_tot[p];
            c->last_exchange_bytes += (long long)c->meta_bytes + (long long)send_tot[p] * (long long)(sizeof(float4) + sizeof(float2));
        }
    } else if (c->N > 1 && c->group) {   // plain mode, in-process: pull the block each peer rendered for my strip
        for (int p = 0; p < c->N; ++p) {
            if (p == c->rank) continue;
            const insitu_ctx* q = c->group->ranks[p];
            if (!q) return fail(c, -1, "insitu_exchange: local group rank " + std::to_string(p) + " missing");
            if (!q->rendered || !q->ev_valid[1]) return fail(c, -1, "insitu_exchange: local group rank " + std::to_string(p) + " has not rendered");
            // the peer's render runs on its own stream (and maybe device): order my copies after it
            HIPCHK(c, hipStreamWaitEvent(c->stream, q->ev[1], 0));
            const size_t n = (size_t)c->B * c->plainBlock;
            const size_t src = (size_t)c->rank * n, dst = (size_t)p * n;
            HIPCHK(c, hipMemcpyAsync(c->d_pcol_recv + dst, q->d_pcol_send + src, n * 4, hipMemcpyDeviceToDevice, c->stream));
            HIPCHK(c, hipMemcpyAsync(c->d_pdep_recv + dst, q->d_pdep_send + src, n * 4, hipMemcpyDeviceToDevice, c->stream));
        }
        c->last_exchange_bytes = (long long)(c->N - 1) * (long long)c->B * (long long)c->plainBlock * 8;
    } else if (c->N > 1) {   // plain mode: one rgba8 colour + depth texel per pixel, fixed-size blocks
        NCCLCHK(c, ncclGroupStart());
        for (int p = 0; p < c->N; ++p) {
            if (p == c->rank) continue;
            const size_t e = (size_t)p * (size_t)c->B * c->plainBlock, n = (size_t)c->B * c->plainBlock;
            NCCLCHK(c, ncclSend(c->d_pcol_send + e, n, ncclUint32, p, c->comm, c->stream));
            NCCLCHK(c, ncclRecv(c->d_pcol_recv + e, n, ncclUint32, p, c->comm, c->stream));
            NCCLCHK(c, ncclSend(c->d_pdep_send + e, n, ncclUint32, p, c->comm, c->stream));
            NCCLCHK(c, ncclRecv(c->d_pdep_recv + e, n, ncclUint32, p, c->comm, c->stream));
        }
        NCCLCHK(c, ncclGroupEnd());
        c->last_exchange_bytes = (long long)(c->N - 1) * (long long)c->B * (long long)c->plainBlock * 8;
    }
    if (c->group) record(c, 7);
    record(c, 2);
    c->exchanged = true;
    return 0;
}

namespace {
// list v (source s = v / B, brick b = v % B) of this rank's strip, as the compositors read it
VdiList list_of(const insitu_ctx* c, int v) {
    const int s = v / c->BV, b = v % c->BV;
    VdiList L{};
    if (c->lists_from_reference) {   // host-buffer path: reference layout converted to slots (B == 1)
        const size_t slot = (size_t)s * c->blockE;
        L.col = (s == c->rank ? c->d_vcol_send : c->d_vcol_recv) + slot;
        L.dep = (s == c->rank ? c->d_vdep_send : c->d_vdep_recv) + slot;
        L.cnt16 = c->d_ref_cnt + (size_t)s * c->stripPx;
        L.cnt_pitch = c->strip_w;
        L.cnt_x0 = 0;
    } else if (s == c->rank) {       // my own strip: the generator's slots and counts
        const size_t e = ((size_t)c->rank * (size_t)c->BV + (size_t)b) * c->blockE;
        L.col = c->d_vcol_send + e;
        L.dep = c->d_vdep_send + e;
        L.cnt16 = c->d_seg_pending + (size_t)b * (size_t)c->W * (size_t)c->H;
        L.cnt_pitch = c->W;
        L.cnt_x0 = c->rank * c->strip_w;
    } else {                         // the compact message source s sent
        const size_t tiles = (size_t)c->strip_tiles * (size_t)((c->H + 7) / 8);
        const size_t region = (size_t)c->BV * c->blockE;
        L.col = c->d_vcol_recv + (size_t)s * region;
        L.dep = c->d_vdep_recv + (size_t)s * region;
        const uint8_t* meta = c->d_meta_recv + (size_t)s * c->meta_bytes;
        L.cnt8 = meta + (size_t)b * tiles * 64;
        L.toff = reinterpret_cast<const uint32_t*>(meta + (size_t)c->BV * tiles * 64) + (size_t)b * tiles;
    }
    return L;
}
}  // namespace

int insitu_composite(insitu_ctx* c) {
    if (!c) return fail(nullptr, -1, "insitu_composite: null context");
    if (c->pipe_inflight && !c->completing)
        return fail(c, -1, "insitu_composite: a pipelined frame is in flight (insitu_pipeline_flush first)");
    if (!c->rendered) return fail(c, -1, "insitu_composite: nothing rendered");
    // with N > 1 the peers' lists arrive in insitu_exchange: without it the compact-message offsets
    // of the receive buffers are not this frame's (or never written)
    if (c->N > 1 && !c->exchanged) return fail(c, -1, "insitu_composite: call insitu_exchange first (nranks > 1)");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, wait_peer_reads(c));   // (local group: the root's gather of the last strip)
    uint32_t* out = is_root(c) ? c->d_gather + (size_t)c->rank * c->stripPx : c->d_strip;
    if (c->mode == INSITU_MODE_VDI && c->composite_vdi) {
        CompositeParams p{};   // VDICompositor.comp (DistributedVolumes.kt:424-439)
        p.V = c->V; p.S = c->S; p.S_out = c->S_out; p.H = c->H; p.W = c->W;
        p.strip_w = c->strip_w; p.strip_tiles = c->strip_tiles; p.x_offset = c->rank * c->strip_w;
        std::memcpy(p.ipv, c->ipv, sizeof p.ipv);
        for (int v = 0; v < c->V; ++v) p.lists[v] = list_of(c, v);
        p.out_color = cvdi_col(c);
        p.out_depth = cvdi_dep(c);
        p.out_count = cvdi_cnt(c);
        p.ndc_local = (c->cfg.faithful & INSITU_FAITHFUL_COMPOSITOR_NDC_X) ? 1 : 0;
        p.passes = c->d_cpasses;
        p.exact = (int)c->tune.exact_search;
        if (c->d_cseq) {
            // the previous composite's demand (observed after that frame's synchronisation) grows the
            // cache, up to the budget taken at create; the waves that find no room merge every pass
            const unsigned long long dem = c->cseq_demand, old = c->cseq_cap;
            if (dem > old && old < c->cseq_max) {
                const unsigned long long want = std::min(dem + dem / 4, c->cseq_max);
                HIPCHK(c, hipStreamSynchronize(c->stream));
                HIPCHK(c, hipFree(c->d_cseq));
                c->d_cseq = nullptr;
                c->cseq_cap = 0;
                // the request, else half of it, else the cache that worked (and that size from now on)
                for (unsigned long long sz : {want, std::max(old, want / 2), old}) {
                    if (sz && hipMalloc(&c->d_cseq, (size_t)sz * 16 * kCompEntryF4) == hipSuccess) {
                        c->cseq_cap = sz;
                        break;
                    }
                    (void)hipGetLastError();
                    c->d_cseq = nullptr;
                }
                if (c->cseq_cap < want) c->cseq_max = c->cseq_cap;
                if (!c->d_cseq) return fail(c, -5, "insitu_composite: re-allocating the merge cache failed");
            }
            if (c->d_cseq) {
                HIPCHK(c, hipMemsetAsync(c->d_cseq_cursor, 0, sizeof(unsigned long long), c->stream));
                p.seq = c->d_cseq;
                p.seq_cursor = c->d_cseq_cursor;
                p.seq_cap = c->cseq_cap;
            }
        }
        HIPCHK(c, launch_vdi_composite(p, c->stream));
        if (p.seq) {
            HIPCHK(c, hipMemcpyAsync(c->h_cseq_demand, c->d_cseq_cursor, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                     c->stream));
            c->cseq_pending = true;   // observed after the next synchronisation (cache_observe)
        }
    } else if (c->mode == INSITU_MODE_VDI) {
        FlattenParams p{};
        p.V = c->V; p.S = c->S; p.H = c->H; p.W = c->W;
        p.strip_w = c->strip_w; p.strip_tiles = c->strip_tiles; p.x_offset = c->rank * c->strip_w;
        std::memcpy(p.ipv, c->ipv, sizeof p.ipv);
        for (int v = 0; v < c->V; ++v) p.lists[v] = list_of(c, v);
        p.out = out;
        HIPCHK(c, launch_vdi_flatten(p, c->stream));
    } else {
        PlainCompParams p{};
        p.V = c->V; p.dim0 = c->W; p.rows = c->rows;
        // PlainImageCompositor.comp:43 as written composites numProcesses = dim0 / rows lists (those past
        // the received ones read as empty): the first min(numProcesses, V)
        if (c->cfg.faithful & INSITU_FAITHFUL_PLAIN_NUM_PROCESSES) p.V = std::min(c->V, c->W / c->rows);
        for (int v = 0; v < c->V; ++v) {
            const int s = v / c->B, b = v % c->B;
            if (s == c->rank) {
                const size_t e = ((size_t)c->rank * (size_t)c->B + (size_t)b) * c->plainBlock;
                p.colors[v] = c->d_pcol_send + e;
                p.depths[v] = c->d_pdep_send + e;
            } else {
                const size_t r = ((size_t)s * (size_t)c->B + (size_t)b) * c->plainBlock;
                p.colors[v] = c->d_pcol_recv + r;
                p.depths[v] = c->d_pdep_recv + r;
            }
        }
        p.out = out;
        HIPCHK(c, launch_plain_composite(p, c->stream));
    }
    record(c, 3);
    c->composited = true;
    return 0;
}

int insitu_gather(insitu_ctx* c, void* host_out, size_t cap) {
    if (!c) return fail(nullptr, -1, "insitu_gather: null context");
    if (c->pipe_inflight && !c->completing)
        return fail(c, -1, "insitu_gather: a pipelined frame is in flight (insitu_pipeline_flush first)");
    if (!c->composited) return fail(c, -1, "insitu_gather: nothing composited");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (c->N > 1 && c->group) {   // in-process: the root pulls every peer's strip
        if (is_root(c)) {
            for (int p = 1; p < c->N; ++p) {
                const insitu_ctx* q = c->group->ranks[p];
                if (!q) return fail(c, -1, "insitu_gather: local group rank " + std::to_string(p) + " missing");
                if (!q->composited || !q->ev_valid[3]) return fail(c, -1, "insitu_gather: local group rank " + std::to_string(p) + " has not composited");
                HIPCHK(c, hipStreamWaitEvent(c->stream, q->ev[3], 0));   // the peer's composite, its stream
                if (c->composite_vdi) {
                    HIPCHK(c, hipMemcpyAsync(c->d_gvdi_col + (size_t)p * c->cblockE, q->d_cvdi_col, c->cblockE * sizeof(float4),
                                             hipMemcpyDeviceToDevice, c->stream));
                    HIPCHK(c, hipMemcpyAsync(c->d_gvdi_dep + (size_t)p * c->cblockE, q->d_cvdi_dep, c->cblockE * sizeof(float2),
                                             hipMemcpyDeviceToDevice, c->stream));
                    HIPCHK(c, hipMemcpyAsync(c->d_gvdi_cnt + (size_t)p * c->stripPx, q->d_cvdi_cnt, c->stripPx * sizeof(uint16_t),
                                             hipMemcpyDeviceToDevice, c->stream));
                } else {
                    HIPCHK(c, hipMemcpyAsync(c->d_gather + (size_t)p * c->stripPx, q->d_strip, c->stripPx * 4,
                                             hipMemcpyDeviceToDevice, c->stream));
                }
            }
        }
    } else if (c->N > 1 && c->composite_vdi) {   // MPI_Gather of the composited VDIs (DistributedVolumes.kt:903)
        NCCLCHK(c, ncclGroupStart());
        if (is_root(c)) {
            for (int p = 1; p < c->N; ++p) {
                NCCLCHK(c, ncclRecv(c->d_gvdi_col + (size_t)p * c->cblockE, c->cblockE * 4, ncclFloat32, p, c->comm,
                                    c->stream));
                NCCLCHK(c, ncclRecv(c->d_gvdi_dep + (size_t)p * c->cblockE, c->cblockE * 2, ncclFloat32, p, c->comm,
                                    c->stream));
                NCCLCHK(c, ncclRecv(c->d_gvdi_cnt + (size_t)p * c->stripPx, c->stripPx * sizeof(uint16_t), ncclUint8, p,
                                    c->comm, c->stream));
            }
        } else {
            NCCLCHK(c, ncclSend(c->d_cvdi_col, c->cblockE * 4, ncclFloat32, 0, c->comm, c->stream));
            NCCLCHK(c, ncclSend(c->d_cvdi_dep, c->cblockE * 2, ncclFloat32, 0, c->comm, c->stream));
            NCCLCHK(c, ncclSend(c->d_cvdi_cnt, c->stripPx * sizeof(uint16_t), ncclUint8, 0, c->comm, c->stream));
        }
        NCCLCHK(c, ncclGroupEnd());
    } else if (c->N > 1) {
        NCCLCHK(c, ncclGroupStart());
        if (is_root(c)) {
            for (int p = 1; p < c->N; ++p)
                NCCLCHK(c, ncclRecv(c->d_gather + (size_t)p * c->stripPx, c->stripPx, ncclUint32, p, c->comm, c->stream));
        } else {
            NCCLCHK(c, ncclSend(c->d_strip, c->stripPx, ncclUint32, 0, c->comm, c->stream));
        }
        NCCLCHK(c, ncclGroupEnd());
    }
    if (is_root(c) && c->composite_vdi) {
        // the root's image: each gathered composited strip flattened front to back (accumulateSupseg)
        for (int p = 0; p < c->N; ++p) {
            FlattenParams f{};
            f.V = 1; f.S = c->S_out; f.H = c->H; f.W = c->W;
            f.strip_w = c->strip_w; f.strip_tiles = c->strip_tiles; f.x_offset = p * c->strip_w;
            std::memcpy(f.ipv, c->ipv, sizeof f.ipv);
            f.lists[0].col = c->d_gvdi_col + (size_t)p * c->cblockE;
            f.lists[0].dep = c->d_gvdi_dep + (size_t)p * c->cblockE;
            f.lists[0].cnt16 = c->d_gvdi_cnt + (size_t)p * c->stripPx;   // (slots past the count: not written)
            f.lists[0].cnt_pitch = c->strip_w;
            f.lists[0].cnt_x0 = 0;
            f.out = c->d_gather + (size_t)p * c->stripPx;
            HIPCHK(c, launch_vdi_flatten(f, c->stream));
        }
    }
    if (is_root(c) && c->mode == INSITU_MODE_VDI)
        HIPCHK(c, launch_assemble_columns(c->d_gather, c->N, c->H, c->strip_w, c->d_image, c->stream));
    if (c->group && is_root(c)) record(c, 7);
    record(c, 4);
    if (is_root(c) && host_out) {
        const size_t bytes = (size_t)c->W * (size_t)c->H * 4;
        if (cap < bytes) return fail(c, -1, "insitu_gather: output buffer too small");
        const void* src = c->mode == INSITU_MODE_VDI ? (const void*)c->d_image : (const void*)c->d_gather;
        HIPCHK(c, hipMemcpyAsync(host_out, src, bytes, hipMemcpyDeviceToHost, c->stream));
        record(c, 10);
    } else {
        c->ev_valid[10] = false;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return check_fault(c);
}

int insitu_frame(insitu_ctx* c, const insitu_camera* cam, void* host_out, size_t cap) {
    int rc;
    if ((rc = insitu_render(c, cam))) return rc;
    if ((rc = insitu_exchange(c))) return rc;
    if ((rc = insitu_composite(c))) return rc;
    return insitu_gather(c, host_out, cap);
}

namespace {

// the second frame slot, the sampling and completion streams and the trigger flag (first pipelined frame)
int pipeline_setup(insitu_ctx* c) {
    if (c->pipe_ready) return 0;
    int lo = 0, hi = 0;
    HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi));   // (greatest priority = numerically smallest)
    // the next frame's first pass fills what the search leaves idle: low priority; the completion of the frame
    // one behind is short and sets the latency: high priority
    HIPCHK(c, hipStreamCreateWithPriority(&c->pipe_sample, hipStreamNonBlocking, lo));
    HIPCHK(c, hipStreamCreateWithPriority(&c->pipe_comp, hipStreamNonBlocking, hi));
    // a search stream per slot: frame k+1's search starts as soon as its first pass is done, beside frame k's
    // search tail and finish (one stream would order it after them)
    HIPCHK(c, hipStreamCreateWithFlags(&c->slot_search_stream, hipStreamNonBlocking));
    HIPCHK(c, hipStreamCreateWithFlags(&c->alt.search_stream, hipStreamNonBlocking));
    int can_wait = 0;
    if (hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, c->cfg.device) != hipSuccess) can_wait = 0;
    c->pipe_wait_value = can_wait != 0;
    if (c->pipe_wait_value) {
        if (int rc = dev_alloc(c, &c->pipe_flag, 2)) return rc;
        HIPCHK(c, hipMemset(c->pipe_flag, 0, 2 * sizeof(unsigned long long)));
    }
    // the second slot starts with the cache size the first one has reached
    if (int rc = alloc_slot(c, c->alt, c->cache_chunks)) return rc;
    c->alt.cache_sized = c->cache_sized;
    c->pipe_ready = true;
    return 0;
}

// the stages of the current slot's frame after its render, on the completion stream: compaction (N > 1),
// exchange, composite, gather (+ the root's image to host_out); blocks until they are done
int pipeline_complete(insitu_ctx* c, void* host_out, size_t cap) {
    StreamScope scope(c, c->pipe_comp);
    c->completing = true;
    int rc = 0;
    if (c->ev_valid[1] && hipStreamWaitEvent(c->stream, c->ev[1], 0) != hipSuccess)
        rc = fail(c, -3, "insitu_frame_pipelined: hipStreamWaitEvent failed");
    if (!rc && c->N > 1) {
        hipError_t e = compact_enqueue(c);
        if (e != hipSuccess) rc = fail(c, -3, std::string("vdi_compact_kernel: ") + hipGetErrorString(e));
    }
    if (!rc) rc = insitu_exchange(c);
    if (!rc) rc = insitu_composite(c);
    if (!rc) {
        record(c, 11);   // (recorded before gather's synchronisation: the slot may be rendered into after it)
        rc = insitu_gather(c, host_out, cap);
    }
    c->completing = false;
    return rc;
}

}  // namespace

int insitu_frame_pipelined(insitu_ctx* c, const insitu_camera* cam, void* host_out, size_t cap, long long* done_frame) {
    if (!c) return fail(nullptr, -1, "insitu_frame_pipelined: null context");
    if (done_frame) *done_frame = -1;
    if (c->mode != INSITU_MODE_VDI) return fail(c, -1, "insitu_frame_pipelined: VDI mode only");
    if (c->group) return fail(c, -1, "insitu_frame_pipelined: not with a local group (stages run rank by rank)");
    if (!c->d_cache) return fail(c, -1, "insitu_frame_pipelined: needs the sample cache (sample_cache_mb >= 0)");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (int rc = pipeline_setup(c)) return rc;
    // 1. frame k into the current slot (its last frame is completed: ev[11] was synchronised)
    hipStream_t ss = c->pipe_sample;
    if (c->ev_valid[11]) HIPCHK(c, hipStreamWaitEvent(ss, c->ev[11], 0));
    // everything enqueued on `stream` before this call -- brick ingests (a re-ingest behind the frame in flight
    // waits for that frame's search), LUT uploads, and before the first pipelined frame whatever the context did
    // unpipelined -- is ordered before this frame's first pass: the sampling stream is not `stream`
    HIPCHK(c, hipEventRecord(c->ev_gate, c->stream));
    HIPCHK(c, hipStreamWaitEvent(ss, c->ev_gate, 0));
    if (c->pipe_inflight) {
        // the trigger of this frame's first pass: the previous frame's search (in `alt`) drains its queue
        // (mode 1), or ends (mode 0); mode 2 starts it once the previous first pass is done (stream order)
        // (enqueued by insitu_render after this frame's prepare)
        int mode = c->pipe_trigger;
        if (mode == 1 && !c->pipe_wait_value) mode = 0;
        if (mode == 1) {
            c->trig_flag = c->pipe_flag + c->alt.flag_index;
            c->trig_value = c->pipe_seq;
        } else if (mode == 0 && c->alt.ev_valid[13]) {
            c->trig_event = c->alt.ev[13];
        }
    }
    c->pipe_seq++;
    c->s_sample = ss;
    int rc = insitu_render(c, cam);
    c->s_sample = nullptr;
    c->trig_flag = nullptr;
    c->trig_event = nullptr;
    if (rc) return rc;
    const long long k = c->pipe_frames++;
    // 2. the frame one behind (in `alt`): exchange, composite, gather -- while frame k renders
    swap_slot(c);
    const bool behind = c->pipe_inflight;
    c->pipe_inflight = true;   // (the slot now in `alt`: frame k)
    if (!behind) return 0;
    rc = pipeline_complete(c, host_out, cap);
    if (rc) return rc;
    if (done_frame) *done_frame = k - 1;
    return 0;
}

int insitu_pipeline_flush(insitu_ctx* c, void* host_out, size_t cap, long long* done_frame) {
    if (!c) return fail(nullptr, -1, "insitu_pipeline_flush: null context");
    if (done_frame) *done_frame = -1;
    if (!c->pipe_inflight) return 0;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    swap_slot(c);   // the frame in flight becomes current
    int rc = pipeline_complete(c, host_out, cap);
    c->pipe_inflight = false;
    if (rc) return rc;
    if (done_frame) *done_frame = c->pipe_frames - 1;
    return 0;
}

int insitu_synchronize(insitu_ctx* c) {
    if (!c) return fail(nullptr, -1, "insitu_synchronize: null context");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (hipStream_t st : {c->pipe_sample, c->pipe_comp, c->slot_search_stream, c->alt.search_stream})
        if (st) HIPCHK(c, hipStreamSynchronize(st));
    if (c->dbg_pending) {   // diagnostics: the last render's per-round search timing, all launches
        c->dbg_pending = false;
        std::vector<unsigned long long> h(c->dbg_entries * 4);
        GenCounters gc{};
        HIPCHK(c, hipMemcpy(h.data(), c->d_dbg, h.size() * 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(&gc, c->d_counters, sizeof gc, hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen(c->dbg_path.c_str(), "wb")) {   // sizeof counters, counters, the non-empty entries
            const uint32_t hdr = (uint32_t)sizeof gc;
            std::fwrite(&hdr, sizeof hdr, 1, f);
            std::fwrite(&gc, sizeof gc, 1, f);
            for (size_t i = 0; i < c->dbg_entries; ++i)
                if (h[4 * i + 1]) std::fwrite(&h[4 * i], 32, 1, f);
            std::fclose(f);
        }
    }
    return check_fault(c);
}

size_t insitu_buffer_bytes(const insitu_ctx* c, int which) {
    if (!c) return 0;
    const size_t px = (size_t)c->W * (size_t)c->H;
    switch (which) {
    case INSITU_BUF_VDI_COLOR: return c->mode == INSITU_MODE_VDI ? px * (size_t)c->S * 16 : 0;
    case INSITU_BUF_VDI_DEPTH: return c->mode == INSITU_MODE_VDI ? px * (size_t)c->S * 8 : 0;
    case INSITU_BUF_OCTREE: return c->mode == INSITU_MODE_VDI ? (size_t)c->ncx * c->ncy * c->S * 4 : 0;
    case INSITU_BUF_PASSES: return (c->mode == INSITU_MODE_VDI && c->d_passes) ? px : 0;
    case INSITU_BUF_PLAIN_COLOR:
    case INSITU_BUF_PLAIN_DEPTH: return c->mode == INSITU_MODE_PLAIN ? px * 4 : 0;
    case INSITU_BUF_STRIP: return c->stripPx * 4;
    case INSITU_BUF_IMAGE: return is_root(c) ? px * 4 : 0;
    case INSITU_BUF_COMPOSITED_COLOR: return c->composite_vdi ? c->stripPx * (size_t)c->S_out * 16 : 0;
    case INSITU_BUF_COMPOSITED_DEPTH: return c->composite_vdi ? c->stripPx * (size_t)c->S_out * 8 : 0;
    case INSITU_BUF_GATHERED_COLOR: return (c->composite_vdi && is_root(c)) ? px * (size_t)c->S_out * 16 : 0;
    case INSITU_BUF_GATHERED_DEPTH: return (c->composite_vdi && is_root(c)) ? px * (size_t)c->S_out * 8 : 0;
    case INSITU_BUF_COMPOSITE_PASSES: return c->composite_vdi ? c->stripPx : 0;
    case INSITU_BUF_RECEIVED_COLOR: return (c->mode == INSITU_MODE_VDI && c->exchanged) ? (size_t)c->V * c->stripPx * c->S * 16 : 0;
    case INSITU_BUF_RECEIVED_DEPTH: return (c->mode == INSITU_MODE_VDI && c->exchanged) ? (size_t)c->V * c->stripPx * c->S * 8 : 0;
    default: return 0;
    }
}

int insitu_read(insitu_ctx* c, int which, int slot, void* host_out, size_t cap) {
    if (!c) return fail(nullptr, -1, "insitu_read: null context");
    StreamScope scope(c, read_stream(c));   // (a pipelined frame in flight: the completed frame's slot)
    if (!host_out) return fail(c, -1, "insitu_read: null output");
    const size_t need = insitu_buffer_bytes(c, which);
    if (need == 0) return fail(c, -1, "insitu_read: buffer not available in this mode/rank");
    if (cap < need) return fail(c, -1, "insitu_read: output buffer too small");
    const bool per_brick = which <= INSITU_BUF_PLAIN_DEPTH;
    if (per_brick && (slot < 0 || slot >= (c->mode == INSITU_MODE_VDI ? c->BV : c->B)))
        return fail(c, -1, "insitu_read: slot out of range");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (int rc = check_fault(c)) return rc;
    switch (which) {
    case INSITU_BUF_VDI_COLOR:
    case INSITU_BUF_VDI_DEPTH: {
        const size_t n = (size_t)c->W * (size_t)c->H * (size_t)c->S;
        float4* rc = nullptr;
        float* rd = nullptr;
        HIPCHK(c, hipMalloc(&rc, n * sizeof(float4)));
        if (hipMalloc(&rd, n * 2 * sizeof(float)) != hipSuccess) {
            (void)hipFree(rc);
            return fail(c, -5, "insitu_read: scratch allocation failed");
        }
        hipError_t e = launch_vdi_to_reference(c->d_vcol_send, c->d_vdep_send, c->d_seg_pending,
                                               (size_t)c->W * (size_t)c->H, (size_t)c->strip_w, (size_t)c->W, c->W, 0, c->W,
                                               c->H, c->S, c->strip_w, c->strip_tiles, c->BV, slot, rc, rd, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(host_out, which == INSITU_BUF_VDI_COLOR ? (void*)rc : (void*)rd, need,
                               hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(rc);
        (void)hipFree(rd);
        if (e != hipSuccess) return fail(c, -3, std::string("insitu_read: ") + hipGetErrorString(e));
        return 0;
    }
    case INSITU_BUF_OCTREE:
        HIPCHK(c, hipMemcpy(host_out, c->d_octree + (size_t)slot * (need / 4), need, hipMemcpyDeviceToHost));
        return 0;
    case INSITU_BUF_PASSES:
        HIPCHK(c, hipMemcpy(host_out, c->d_passes + (size_t)slot * need, need, hipMemcpyDeviceToHost));
        return 0;
    case INSITU_BUF_PLAIN_COLOR:
    case INSITU_BUF_PLAIN_DEPTH: {
        const uint32_t* src = which == INSITU_BUF_PLAIN_COLOR ? c->d_pcol_send : c->d_pdep_send;
        for (int d = 0; d < c->N; ++d)
            HIPCHK(c, hipMemcpy((uint8_t*)host_out + (size_t)d * c->plainBlock * 4,
                                src + ((size_t)d * (size_t)c->B + (size_t)slot) * c->plainBlock, c->plainBlock * 4,
                                hipMemcpyDeviceToHost));
        return 0;
    }
    case INSITU_BUF_STRIP: {
        const uint32_t* src = is_root(c) ? c->d_gather + (size_t)c->rank * c->stripPx : c->d_strip;
        HIPCHK(c, hipMemcpy(host_out, src, need, hipMemcpyDeviceToHost));
        return 0;
    }
    case INSITU_BUF_IMAGE: {
        const void* src = c->mode == INSITU_MODE_VDI ? (const void*)c->d_image : (const void*)c->d_gather;
        HIPCHK(c, hipMemcpy(host_out, src, need, hipMemcpyDeviceToHost));
        return 0;
    }
    case INSITU_BUF_COMPOSITED_COLOR:
    case INSITU_BUF_COMPOSITED_DEPTH:
    case INSITU_BUF_GATHERED_COLOR:
    case INSITU_BUF_GATHERED_DEPTH: {
        const bool gathered = which == INSITU_BUF_GATHERED_COLOR || which == INSITU_BUF_GATHERED_DEPTH;
        const bool colour = which == INSITU_BUF_COMPOSITED_COLOR || which == INSITU_BUF_GATHERED_COLOR;
        const int width = gathered ? c->W : c->strip_w;
        const size_t n = (size_t)width * (size_t)c->H * (size_t)c->S_out;
        float4* rc = nullptr;
        float* rd = nullptr;
        HIPCHK(c, hipMalloc(&rc, n * sizeof(float4)));
        if (hipMalloc(&rd, n * 2 * sizeof(float)) != hipSuccess) {
            (void)hipFree(rc);
            return fail(c, -5, "insitu_read: scratch allocation failed");
        }
        // gathered: N blocks [rank] of one strip each; a single strip: one block
        // (the slots past each pixel's count are not written by the compositor: zeros here)
        hipError_t e = launch_vdi_to_reference(gathered ? c->d_gvdi_col : cvdi_col(c), gathered ? c->d_gvdi_dep : cvdi_dep(c),
                                               gathered ? c->d_gvdi_cnt : cvdi_cnt(c), 0, c->stripPx, (size_t)c->strip_w,
                                               width, 0, width, c->H, c->S_out, c->strip_w, c->strip_tiles, 1, 0, rc, rd,
                                               c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(host_out, colour ? (void*)rc : (void*)rd, need, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(rc);
        (void)hipFree(rd);
        if (e != hipSuccess) return fail(c, -3, std::string("insitu_read: ") + hipGetErrorString(e));
        return 0;
    }
    case INSITU_BUF_COMPOSITE_PASSES:
        HIPCHK(c, hipMemcpy(host_out, c->d_cpasses, need, hipMemcpyDeviceToHost));
        return 0;
    case INSITU_BUF_RECEIVED_COLOR:
    case INSITU_BUF_RECEIVED_DEPTH: {   // block v = list v of the compositor (source-major)
        const size_t n = c->stripPx * (size_t)c->S;
        float4* rc = nullptr;
        float2* rd = nullptr;
        HIPCHK(c, hipMalloc(&rc, n * sizeof(float4)));
        if (hipMalloc(&rd, n * sizeof(float2)) != hipSuccess) {
            (void)hipFree(rc);
            return fail(c, -5, "insitu_read: scratch allocation failed");
        }
        const bool colour = which == INSITU_BUF_RECEIVED_COLOR;
        const size_t blk = colour ? n * sizeof(float4) : n * sizeof(float2);
        hipError_t e = hipSuccess;
        for (int v = 0; v < c->V && e == hipSuccess; ++v) {
            e = launch_vdi_list_to_reference(list_of(c, v), c->S, c->H, c->strip_w, c->strip_tiles, rc, rd, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync((uint8_t*)host_out + (size_t)v * blk, colour ? (void*)rc : (void*)rd, blk,
                                   hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        }
        (void)hipFree(rc);
        (void)hipFree(rd);
        if (e != hipSuccess) return fail(c, -3, std::string("insitu_read: ") + hipGetErrorString(e));
        return 0;
    }
    default: return fail(c, -1, "insitu_read: unknown buffer");
    }
}

int insitu_read_region(insitu_ctx* c, int which, int slot, int x0, int x1, void* host_out, size_t cap) {
    if (!c) return fail(nullptr, -1, "insitu_read_region: null context");
    StreamScope scope(c, read_stream(c));   // (a pipelined frame in flight: the completed frame's slot)
    if (!host_out) return fail(c, -1, "insitu_read_region: null output");
    if (c->mode != INSITU_MODE_VDI) return fail(c, -1, "insitu_read_region: VDI mode only");
    if (which != INSITU_BUF_VDI_COLOR && which != INSITU_BUF_VDI_DEPTH && which != INSITU_BUF_PASSES)
        return fail(c, -1, "insitu_read_region: buffer must be VDI colour, VDI depth or passes");
    if (slot < 0 || slot >= c->BV) return fail(c, -1, "insitu_read_region: slot out of range");
    if (x0 < 0 || x1 > c->W || x0 >= x1) return fail(c, -1, "insitu_read_region: bad column range");
    const size_t nx = (size_t)(x1 - x0);
    const size_t n = nx * (size_t)c->H * (size_t)c->S;
    const size_t need = which == INSITU_BUF_VDI_COLOR ? n * 16 : (which == INSITU_BUF_VDI_DEPTH ? n * 8 : nx * (size_t)c->H);
    if (cap < need) return fail(c, -1, "insitu_read_region: output buffer too small");
    if (which == INSITU_BUF_PASSES && !c->d_passes) return fail(c, -1, "insitu_read_region: context keeps no pass counts");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (int rc = check_fault(c)) return rc;
    if (which == INSITU_BUF_PASSES) {   // (H, x1-x0) rows of the (H, W) pass counts
        HIPCHK(c, hipMemcpy2D(host_out, nx, c->d_passes + (size_t)slot * (size_t)c->W * (size_t)c->H + (size_t)x0,
                              (size_t)c->W, nx, (size_t)c->H, hipMemcpyDeviceToHost));
        return 0;
    }
    void* scratch = nullptr;
    HIPCHK(c, hipMalloc(&scratch, n * (which == INSITU_BUF_VDI_COLOR ? 16 : 8)));
    float4* rc_ = which == INSITU_BUF_VDI_COLOR ? (float4*)scratch : nullptr;
    float* rd_ = which == INSITU_BUF_VDI_DEPTH ? (float*)scratch : nullptr;
    hipError_t e = hipSuccess;
    // the kernel writes both outputs: give the unused one a throwaway buffer
    void* other = nullptr;
    e = hipMalloc(&other, n * (which == INSITU_BUF_VDI_COLOR ? 8 : 16));
    if (e == hipSuccess) {
        if (!rc_) rc_ = (float4*)other;
        else rd_ = (float*)other;
        e = launch_vdi_to_reference(c->d_vcol_send, c->d_vdep_send, c->d_seg_pending, (size_t)c->W * (size_t)c->H,
                                    (size_t)c->strip_w, (size_t)c->W, c->W, x0, (int)nx, c->H, c->S, c->strip_w,
                                    c->strip_tiles, c->BV, slot, rc_, rd_, c->stream);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(host_out, scratch, need, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(scratch);
    if (other) (void)hipFree(other);
    if (e != hipSuccess) return fail(c, -3, std::string("insitu_read_region: ") + hipGetErrorString(e));
    return 0;
}

int insitu_get_stats(insitu_ctx* c, insitu_stats* out) {
    if (!c || !out) return fail(c, -1, "insitu_get_stats: null argument");
    StreamScope scope(c, read_stream(c));   // (a pipelined frame in flight: the completed frame's slot)
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    cache_observe(c);
    std::memset(out, 0, sizeof *out);
    float* slots[4] = {&out->ms_render, &out->ms_exchange, &out->ms_composite, &out->ms_gather};
    for (int i = 0; i < 4; ++i) {
        if (c->ev_valid[i] && c->ev_valid[i + 1]) {
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]) == hipSuccess) *slots[i] = ms;
        }
    }
    if (c->ev_valid[4] && c->ev_valid[10]) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, c->ev[4], c->ev[10]) == hipSuccess) out->ms_image_d2h = ms;
    }
    out->cache_bytes = (long long)c->cache_chunks * 32;
    out->exchange_bytes = c->last_exchange_bytes;
    out->exchange_entries = c->last_exchange_entries;
    if (c->mode == INSITU_MODE_VDI && c->d_counters) {
        // the render's pinned copy when it has arrived: a synchronous copy out of device memory is a blit kernel,
        // and with a pipelined frame's persistent search holding every CU it waited ~2 ms for a slot (the 8-GPU
        // share's trace: the host's next frame call, and so the next first pass, came that much late)
        GenCounters gc{};
        if (c->h_ctr_valid) gc = *c->h_ctr;
        else HIPCHK(c, hipMemcpy(&gc, c->d_counters, sizeof gc, hipMemcpyDeviceToHost));
        out->rays_searched = (long long)gc.queue_count + (long long)gc.queue_short;
        out->rays_uncached = (long long)gc.march_rays + (long long)gc.cap_overflow;
        out->cache_demand_bytes = (long long)gc.cache_cursor * 32;
        out->search_regroups = (int)gc.regroups;
    }
    if (c->mode == INSITU_MODE_VDI && c->N > 1 && c->ev_valid[8] && c->ev_valid[9]) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, c->ev[8], c->ev[9]) == hipSuccess) out->ms_exchange_sync = ms;
    }
    if (c->mode == INSITU_MODE_VDI && c->N > 1 && c->ev_valid[6] && c->ev_valid[12]) {   // compaction: exchange
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, c->ev[6], c->ev[12]) == hipSuccess) {
            out->ms_compact = ms;
            if (!c->slot_pipelined) {   // (a pipelined frame packs after its render, in its exchange span)
                out->ms_render -= ms;
                out->ms_exchange += ms;
            }
        }
    }
    if (c->slot_pipelined && c->ev_valid[1] && c->ev_valid[6] && c->N > 1) {   // exchange from its compaction
        float ms = 0.0f;
        if (c->ev_valid[2] && hipEventElapsedTime(&ms, c->ev[6], c->ev[2]) == hipSuccess) out->ms_exchange = ms;
    }
    {   // latency: render start to the image on the host (or the gather's end)
        const int end = c->ev_valid[10] ? 10 : 4;
        float ms = 0.0f;
        if (c->ev_valid[0] && c->ev_valid[end] && hipEventElapsedTime(&ms, c->ev[0], c->ev[end]) == hipSuccess)
            out->ms_latency = ms;
    }
    out->pipelined = c->slot_pipelined ? 1 : 0;
    {   // the last batch of re-ingests, once it is done (a pipelined loop does not wait for it)
        float ms = 0.0f;
        if (hipEventQuery(c->ev_ingest) == hipSuccess && hipEventElapsedTime(&ms, c->ev_ingest0, c->ev_ingest) == hipSuccess)
            out->ms_ingest = ms;
        (void)hipGetLastError();
    }
    out->ms_sample = out->ms_render;
    if (c->mode == INSITU_MODE_VDI && c->ev_valid[5] && c->ev_valid[0] && c->ev_valid[1]) {
        float a = 0.0f, b = 0.0f;
        if (hipEventElapsedTime(&a, c->ev[0], c->ev[5]) == hipSuccess &&
            hipEventElapsedTime(&b, c->ev[5], c->ev[1]) == hipSuccess) {
            out->ms_sample = a;
            out->ms_search = b - out->ms_compact;
        }
    }
    return 0;
}

int insitu_pass_stats(insitu_ctx* c, double* mean_passes, long long* rays_hit) {
    if (!c || !mean_passes || !rays_hit) return fail(c, -1, "insitu_pass_stats: null argument");
    StreamScope scope(c, read_stream(c));   // (a pipelined frame in flight: the completed frame's slot)
    if (!c->d_passes || c->mode != INSITU_MODE_VDI) return fail(c, -1, "insitu_pass_stats: needs VDI mode + keep_passes");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<uint8_t> h((size_t)c->BV * (size_t)c->W * (size_t)c->H);
    HIPCHK(c, hipMemcpy(h.data(), c->d_passes, h.size(), hipMemcpyDeviceToHost));
    long long hit = 0, sum = 0;
    for (uint8_t v : h)
        if (v) { ++hit; sum += v; }
    *rays_hit = hit;
    *mean_passes = hit ? (double)sum / (double)hit : 0.0;
    return 0;
}

int insitu_distribute_vdis(insitu_ctx* c, const void* subVDIColor, const void* subVDIDepth, long long sizePerProcess,
                           int commSize, void* recvColor, void* recvDepth) {
    if (!c) return fail(nullptr, -1, "insitu_distribute_vdis: null context");
    if (!subVDIColor || !subVDIDepth) return fail(c, -1, "insitu_distribute_vdis: null sub-VDI buffer");
    if (commSize != c->N) return fail(c, -1, "insitu_distribute_vdis: commSize differs from the context's nranks");
    if (c->BV != 1) return fail(c, -1, "insitu_distribute_vdis: the host-buffer path carries one sub-VDI per rank");
    if (!c->camera_set) return fail(c, -1, "insitu_distribute_vdis: call insitu_set_camera (VDI metadata) first");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (c->mode == INSITU_MODE_PLAIN) {
        // rgba8 (dim0, dim1) colour + encoded depth; blocks of rows*dim0 texels (DistributedVolumeRenderer.kt:577)
        if (sizePerProcess != (long long)c->plainBlock * 4)
            return fail(c, -1, "insitu_distribute_vdis: plain sizePerProcess must be H*W*4/commSize bytes");
        const size_t bytes = (size_t)c->N * c->plainBlock * 4;
        HIPCHK(c, hipMemcpyAsync(c->d_pcol_send, subVDIColor, bytes, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_pdep_send, subVDIDepth, bytes, hipMemcpyHostToDevice, c->stream));
        c->rendered = true;
        int rc = insitu_exchange(c);
        if (rc) return rc;
        for (int s = 0; s < c->N; ++s) {   // the received set, source-major (compositeVDIs' VDISetColour)
            const size_t blk = c->plainBlock;
            const uint32_t* sc = s == c->rank ? c->d_pcol_send + (size_t)c->rank * blk : c->d_pcol_recv + (size_t)s * blk;
            const uint32_t* sd = s == c->rank ? c->d_pdep_send + (size_t)c->rank * blk : c->d_pdep_recv + (size_t)s * blk;
            if (recvColor) HIPCHK(c, hipMemcpyAsync((uint32_t*)recvColor + (size_t)s * blk, sc, blk * 4, hipMemcpyDeviceToHost, c->stream));
            if (recvDepth) HIPCHK(c, hipMemcpyAsync((uint32_t*)recvDepth + (size_t)s * blk, sd, blk * 4, hipMemcpyDeviceToHost, c->stream));
        }
        rc = insitu_composite(c);
        if (rc) return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return 0;
    }
    // VDI mode: colour (S,H,W) rgba32f + depth (2S,H,W) r32f, x slowest; block j = columns of strip j
    const size_t blkE = (size_t)c->strip_w * (size_t)c->H * (size_t)c->S;   // supersegments per block
    if (sizePerProcess != (long long)(blkE * 4))
        return fail(c, -1, "insitu_distribute_vdis: VDI sizePerProcess must be H*W*S*4/commSize floats");
    const size_t allE = blkE * (size_t)c->N;
    if (!c->d_ref_col) {
        HIPCHK(c, hipMalloc(&c->d_ref_col, 2 * allE * sizeof(float4)));
        HIPCHK(c, hipMalloc(&c->d_ref_dep, 2 * allE * 2 * sizeof(float)));
        HIPCHK(c, hipMalloc(&c->d_ref_cnt, (size_t)c->N * c->stripPx * sizeof(uint16_t)));
    }
    float4* send_c = c->d_ref_col;
    float4* recv_c = c->d_ref_col + allE;
    float* send_d = c->d_ref_dep;
    float* recv_d = c->d_ref_dep + 2 * allE;
    HIPCHK(c, hipMemcpyAsync(send_c, subVDIColor, allE * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(send_d, subVDIDepth, allE * 2 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(recv_c + (size_t)c->rank * blkE, send_c + (size_t)c->rank * blkE, blkE * sizeof(float4),
                             hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(recv_d + (size_t)c->rank * 2 * blkE, send_d + (size_t)c->rank * 2 * blkE,
                             blkE * 2 * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
    if (c->N > 1 && c->group) {
        return fail(c, -1, "insitu_distribute_vdis: the host-buffer path needs RCCL ranks (not a local group)");
    } else if (c->N > 1) {   // MPI_Alltoall of InVis.cpp -> grouped RCCL send/recv of contiguous strip blocks
        NCCLCHK(c, ncclGroupStart());
        for (int p = 0; p < c->N; ++p) {
            if (p == c->rank) continue;
            NCCLCHK(c, ncclSend(send_c + (size_t)p * blkE, blkE * 4, ncclFloat32, p, c->comm, c->stream));
            NCCLCHK(c, ncclRecv(recv_c + (size_t)p * blkE, blkE * 4, ncclFloat32, p, c->comm, c->stream));
            NCCLCHK(c, ncclSend(send_d + (size_t)p * 2 * blkE, blkE * 2, ncclFloat32, p, c->comm, c->stream));
            NCCLCHK(c, ncclRecv(recv_d + (size_t)p * 2 * blkE, blkE * 2, ncclFloat32, p, c->comm, c->stream));
        }
        NCCLCHK(c, ncclGroupEnd());
    }
    if (recvColor) HIPCHK(c, hipMemcpyAsync(recvColor, recv_c, allE * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    if (recvDepth) HIPCHK(c, hipMemcpyAsync(recvDepth, recv_d, allE * 2 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    // uploadForCompositing (DistributedVolumes.kt:945-998): the received set feeds the compositor
    for (int s = 0; s < c->N; ++s) {
        const size_t slot = s == c->rank ? (size_t)c->rank * c->blockE : (size_t)s * c->blockE;
        float4* dc = (s == c->rank ? c->d_vcol_send : c->d_vcol_recv) + slot;
        float2* dd = (s == c->rank ? c->d_vdep_send : c->d_vdep_recv) + slot;
        HIPCHK(c, launch_vdi_from_reference(recv_c + (size_t)s * blkE, recv_d + (size_t)s * 2 * blkE, c->H, c->S,
                                            c->strip_w, c->strip_tiles, dc, dd, c->d_ref_cnt + (size_t)s * c->stripPx,
                                            c->stream));
    }
    c->rendered = true;
    c->exchanged = true;
    c->lists_from_reference = true;
    int rc = insitu_composite(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int insitu_gather_composited_vdi_set(insitu_ctx* c, long long compositedVDILen, int root, int myRank, int commSize,
                                     void* gatherColor, void* gatherDepth) {
    if (!c) return fail(nullptr, -1, "insitu_gather_composited_vdi_set: null context");
    if (!c->composite_vdi) return fail(c, -1, "insitu_gather_composited_vdi_set: context has composite_vdi == 0");
    if (root != 0) return fail(c, -1, "insitu_gather_composited_vdi_set: root must be 0");
    if (myRank != c->rank || commSize != c->N)
        return fail(c, -1, "insitu_gather_composited_vdi_set: rank/commSize differ from the context");
    if (compositedVDILen != (long long)(c->stripPx * (size_t)c->S_out * 4))
        return fail(c, -1, "insitu_gather_composited_vdi_set: compositedVDILen must be H*W*S_out*4/commSize floats");
    int rc = insitu_gather(c, nullptr, 0);
    if (rc) return rc;
    if (is_root(c)) {
        const size_t cb = insitu_buffer_bytes(c, INSITU_BUF_GATHERED_COLOR);
        if (gatherColor && (rc = insitu_read(c, INSITU_BUF_GATHERED_COLOR, 0, gatherColor, cb))) return rc;
        if (gatherDepth && (rc = insitu_read(c, INSITU_BUF_GATHERED_DEPTH, 0, gatherDepth, cb / 2))) return rc;
    }
    return 0;
}

int insitu_gather_composited_vdis(insitu_ctx* c, int root, long long subVDILen, int myRank, int commSize,
                                  void* gatherOut, size_t cap) {
    if (!c) return fail(nullptr, -1, "insitu_gather_composited_vdis: null context");
    if (root != 0) return fail(c, -1, "insitu_gather_composited_vdis: root must be 0");
    if (myRank != c->rank || commSize != c->N)
        return fail(c, -1, "insitu_gather_composited_vdis: rank/commSize differ from the context");
    if (subVDILen != (long long)c->stripPx * 4)
        return fail(c, -1, "insitu_gather_composited_vdis: subVDILen must be the rgba8 strip size H*W*4/commSize");
    return insitu_gather(c, gatherOut, cap);
}

}  // extern "C"
