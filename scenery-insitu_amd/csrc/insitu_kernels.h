// insitu_kernels.h -- kernel parameter blocks and launch entry points (host <-> device).
//
// Device VDI layout (DESIGN.md "Data layout in HBM"): for every (destination strip d,
// local brick b) one contiguous block of E = strip_tiles*S*H*8 supersegment entries,
// entry index ((xt*S + i)*H + y)*8 + xx with xt = x_local/8, xx = x_local%8.  A wave
// owns one 8x8 pixel tile, so the 64 lanes writing slot i of their pixels store 64
// consecutive entries (1 KiB colour, 512 B depth).  Blocks are ordered [d][b] so the
// exchange is one equal-count all-to-all of contiguous blocks.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace insitu {

enum VoxelType { VOX_U8 = 0, VOX_U16 = 1, VOX_F32 = 2 };

struct BrickDesc {
    const void* data;  // blocked layout with halo (insitu_sampling.h): 9^3-voxel blocks, device memory
    int dtype;
    int nx, ny, nz;
    int nbx, nby, nbz; // blocks per axis (ceil(n/8))
    float im[16];      // inverse model (world -> voxel space)
    float conv_k;      // convert scale with the unorm normalisation folded in
    float conv_off;
};

struct TransferDesc {
    const float* tf;    // n_tf alpha texels
    int n_tf;
    const float* cmap;  // n_cm rgba texels
    int n_cm;
    float cmag;         // max(1, 2C, 2CA): C = max |colour-map rgb|, A = max |TF| (filtered-decision margin)
};

constexpr int kMaxBricks = 8;   // bricks (sub-VDIs) one rank renders in one launch

// A ray whose first raymarch pass closed more than S supersegments, queued by
// vdi_sample_kernel for vdi_search_kernel (vdi_generate.hip).
struct PendingRay {
    uint32_t pix;         // gy * W + gx
    uint32_t b;           // local brick slot
    uint32_t chunk;       // first 32-byte cache chunk (4 samples) of the ray
    uint32_t n;           // cached (in-brick) samples
    float step_first;     // ray parameter `step` of the first cached sample (the running sum of VG:447)
    uint32_t last_final;  // 1 if the last cached sample is the ray's last sample
    float low, high, mid; // threshold search state after the passes run in vdi_sample_kernel
    uint32_t iter_found;  // passes done (bits 0-7) | threshold found (bit 8)
    // Segmentation intervals (lo, hi] in squared-difference space: every squared threshold in the
    // interval makes the same supersegment decisions as the pass that ran at `low` (seg_low) or at
    // `high` (seg_high), so a pass at such a threshold has that pass's outcome without running
    float seg_low[2], seg_high[2];
    uint32_t n_high;      // supersegments closed by the pass at `high`
    uint32_t nsteps;      // merged volumes: the ray's numSteps (a sample is `last` at step nsteps - 1)
};

// per-render counters of the VDI generator, zeroed before every render
struct GenCounters {
    unsigned long long cache_cursor;   // cache chunks handed out
    uint32_t queue_count;              // long rays queued for the search kernel (from the queue's front)
    uint32_t queue_head;               // rays taken by the search kernel
    uint32_t fault;                    // set when a persistent kernel hit its wall-clock bound (never expected)
    uint32_t queue_short;              // short rays queued (from the queue's back)
    uint32_t march_rays;               // rays without cache space (searched by re-sampling the brick)
    uint32_t cap_overflow;             // merged volumes: rays that outgrew their per-ray cache cap (in place
                                       // too; a bigger cache does not help them, so they do not grow it)
    unsigned long long cache_need;     // cache chunks the frame's rays ask for (vdi_tile_len_kernel)
    uint32_t regroups;                 // search: wave regroups (diagnostics, tools/ray_timing.py)
    // cross-frame pipelining (insitu_frame_pipelined): the wave whose queue claim drains the queue stores
    // pipe_seq to *pipe_flag (system scope, seen by the command processor), and the next frame's sampling,
    // enqueued behind hipStreamWaitValue64 on its own stream, starts in this search's tail.  Written after
    // the zeroing by hipStreamWriteValue64 (launch_vdi_prepare); null: not pipelined
    unsigned long long* pipe_flag;
    unsigned long long pipe_seq;
};

struct VdiGenParams {
    BrickDesc bricks[kMaxBricks];  // all local bricks; blockIdx.y selects one (or: the volumes of one VDI)
    int nvolumes;                  // > 0: bricks[0..nvolumes) are the volumes of ONE VDI (B == 1)
    size_t octree_stride;        // counters per brick
    size_t passes_stride;        // bytes per brick
    TransferDesc xfer;
    float ipv[16];
    float pv[16];
    float view[16];
    float nw, tmax;
    int W, H, S;
    int strip_w, strip_tiles, nstrips, B;
    int ytiles;
    float4* color;      // send buffer base (block [0][0])
    float2* depth;
    uint32_t* octree;   // (S, H/8, W/8) counters of brick 0; brick b at + b*octree_stride
    uint8_t* passes;    // H*W pass counts of brick 0 (may be null); brick b at + b*passes_stride
    uint16_t* seg_pending;  // H*W per brick (passes_stride): kPendingCount bits = supersegments stored
                            // for the pixel (<= S); | kPendingDeferred when their colours are raw curV
                            // (see seg_steps); | kPendingCounted when their octree cells are counted
                            // already (otherwise vdi_finish_kernel counts them)
    uint16_t* seg_steps;    // per supersegment entry (color's layout): step count of a deferred colour
    float* cache;       // per-sample cache in 32-byte chunks of 4 samples {LUT coord x4, opacity x4}
                        // (merged volumes: 64-byte slots of two chunk units, with the 4 samples'
                        // step indices, vdi_generate.hip MergedChunkStore); null = off
    uint32_t cache_chunks;              // capacity (32-byte units)
    GenCounters* ctr;                   // per-render counters (zeroed by launch_vdi_generate)
    PendingRay* queue;                  // capacity queue_cap = B*W*H
    uint32_t queue_cap;
    uint32_t long_samples;              // rays with at least this many cached samples are searched first
    int round_batch;                    // a wave ends rounds once this many lanes (or all) have finished
    int search_blocks;                  // grid of the persistent search kernel
    // > 0 (pipelined frames): only the first clamp(ceil(queue / search_block_rays), search_min_blocks,
    // search_blocks) blocks search, the rest leave at once -- their wave slots go to the next frame's first pass
    int search_block_rays;
    int search_min_blocks;
    int search_lanes;                   // lanes of that grid resident at once (vdi_search_resident_lanes)
    int search_oversub;                 // queue length x group size allowed per resident lane
    int search_depth;                   // tree levels per replay round; 0 = chosen from the queue
    int regroup;                        // 1: deeper trees for the rays left once the queue is drained
    hipEvent_t split_event;             // recorded between the two kernels when non-null
    int exact_search;                   // 1: every supersegment decision by the exact contract path
                                        // (default 0: filtered decisions, identical results)
    unsigned long long* debug_rays;     // diagnostics (INSITU_DEBUG_RAYS): per search round
                                        // {pop, done, passes | n << 8 | group << 24, pix | brick << 32};
                                        // may be null
    uint32_t debug_cap;                 // entries of debug_rays
    int ncx, ncy;
    float interval_size;
    // longest tiles first (vdi_tile_order): per (brick, tile) a sort key -- the tile's longest ray
    // in 16-sample classes, then the XCD order -- and the sorted (brick, tile) ids the sampling
    // kernel walks; null = the plain XCD order
    uint32_t* tile_keys;     // 2 x B*tiles (in, sorted out)
    uint32_t* tile_ids;      // 2 x B*tiles (in, sorted out)
    void* sort_tmp;          // hipcub temporary storage
    size_t sort_tmp_bytes;
    int super_tile;          // tiles per super-tile edge of the sort key (1, 2 or 4; vdi_tile_len_kernel)
    int tile_len_exact;      // 1: keys from every ray of a tile (else 16 of its 64 rays, vdi_tile_len_sub_kernel)
    int prepared;            // counters zeroed and tile keys sorted already (launch_vdi_prepare)
    int measure_cache;       // vdi_tile_len_kernel sums the frame's cache demand into ctr->cache_need
    unsigned long long* pipe_flag;   // pipelined frames: stored into ctr by launch_vdi_prepare (GenCounters)
    unsigned long long pipe_seq;
};

constexpr uint32_t kPendingCount = 0xffu;
constexpr uint32_t kPendingDeferred = 0x100u;
constexpr uint32_t kPendingCounted = 0x200u;

struct PlainGenParams {
    BrickDesc bricks[kMaxBricks];   // all local bricks (blockIdx.y selects one)
    TransferDesc xfer;
    float ipv[16];
    float nw, fwnw, tmax;
    int dim0, dim1;     // texture size (gid.x < dim0, gid.y < dim1)
    int rows;           // dim1 / nstrips
    int nstrips, B;
    uint32_t* color;    // send buffer base, packed rgba8: [d][b][rows][dim0]
    uint32_t* depth;
};

constexpr int kMaxLists = 32;   // max sub-VDIs (virtual ranks) merged per pixel

// One sub-VDI list set of a screen strip, as the compositors read it.  Two layouts:
//  * slotted (cnt8 == null): the generator's strip block [xt][i][y][xx] of S slots, entry of slot i
//    of pixel (xl, y) at ((xt*S + i)*H + y)*8 + xx; the pixel's supersegment count from cnt16
//    (& kPendingCount) at [y*cnt_pitch + cnt_x0 + xl], or S when cnt16 is null (zero-filled blocks).
//    Slots past the count are never read.
//  * compact (cnt8 != null): what the variable-length exchange moves -- per 8x8 tile (index
//    xt*ytiles + yt) the 64 pixel counts cnt8[tile*64 + lane] and the first entry toff[tile]; a
//    tile's entries pixel-major (the pixel's lists at toff + exclusive prefix of the counts).
struct VdiList {
    const float4* col;
    const float2* dep;
    const uint16_t* cnt16;
    int cnt_pitch, cnt_x0;
    const uint8_t* cnt8;
    const uint32_t* toff;
};

struct FlattenParams {
    VdiList lists[kMaxLists];     // V lists, merged in list order on ties (determineNextSupseg)
    int V, S, H, W;
    int strip_w, strip_tiles, x_offset;
    float ipv[16];
    uint32_t* out;                // packed rgba8, row-major (H, strip_w)
};

// VDICompositor.comp over this rank's strip (re-supersegmenting compositor)
struct CompositeParams {
    VdiList lists[kMaxLists];     // V lists (S slots at most each)
    int V, S, S_out, H, W;
    int strip_w, strip_tiles, x_offset;
    float ipv[16];
    float4* out_color;            // composited strip block [xt][i][y][xx], S_out slots
    float2* out_depth;
    uint16_t* out_count;          // per pixel [y][x_local] the slots written (<= S_out); the slots past it are
                                  // not zero-filled (every reader is bounded by it).  null: zero-filled slots
    int ndc_local;                // 1: ndc_x from the strip-local column (VDICompositor.comp:204 as written)
    uint8_t* passes;              // (H, strip_w) search passes, may be null
    // merge cache: every pixel's merged supersegment sequence with its pass-independent opacity,
    // kCompEntryF4 float4 per entry ({start, end, adjusted alpha, -}, colour; the replay recomputes the
    // world positions from the depths), entry k of lane l of a wave at base + 64k + l; a wave that finds
    // no room merges on every pass instead (exact decisions).  null = off
    float4* seq;
    unsigned long long* seq_cursor;   // entries handed out (zeroed before the launch); the demand
    unsigned long long seq_cap;       // capacity in entries
    int exact;                        // 1: every decision by the exact contract path (filtered: same results)
};
constexpr int kCompEntryF4 = 2;   // float4 per merge-cache entry (32 bytes)

struct PlainCompParams {
    const uint32_t* colors[kMaxLists];  // V device pointers to (rows, dim0) rgba8 blocks
    const uint32_t* depths[kMaxLists];
    int V, dim0, rows;
    uint32_t* out;                  // (rows, dim0)
};

// counters zeroed, tile keys (with the frame's cache demand in ctr->cache_need) and their sort;
// launch_vdi_generate runs it itself unless p.prepared
hipError_t launch_vdi_prepare(const VdiGenParams& p, hipStream_t s);
hipError_t launch_vdi_generate(const VdiGenParams& p, hipStream_t s);   // launch_vdi_sample + launch_vdi_search
// the two halves of a render: the first pass over the bricks (sampling or merge kernel; records p.split_event)
// and the persistent threshold search over the queued rays -- on different streams when frames are pipelined
hipError_t launch_vdi_sample(const VdiGenParams& p, hipStream_t s);
hipError_t launch_vdi_search(const VdiGenParams& p, hipStream_t s);
// tile_order.hip: descending radix sort of (key, id) pairs (hipcub); tmp == null queries tmp_bytes
hipError_t sort_tiles_desc(void* tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                           const uint32_t* ids_in, uint32_t* ids_out, int n, hipStream_t s);
hipError_t launch_vdi_finish(const VdiGenParams& p, hipStream_t s);   // all local bricks, one lane per pixel
// LDS bytes of the search kernel and the lanes its grid keeps resident on `device` for that LDS
hipError_t vdi_search_resident_lanes(int n_tf, int n_cm, int device, int* lanes);
// the most LDS any generator kernel asks for with LUTs of these sizes (sampling, merge and search kernels)
size_t vdi_generator_lds_bytes(int n_tf, int n_cm);
hipError_t launch_plain_generate(const PlainGenParams& p, hipStream_t s);
hipError_t launch_vdi_flatten(const FlattenParams& p, hipStream_t s);
hipError_t launch_plain_composite(const PlainCompParams& p, hipStream_t s);
hipError_t launch_vdi_composite(const CompositeParams& p, hipStream_t s);
// root: [d][H][strip_w] strips -> row-major (H, W) image
hipError_t launch_assemble_columns(const uint32_t* strips, int nstrips, int H, int strip_w, uint32_t* image,
                                   hipStream_t s);
// reference-layout strip block (strip_w, H, S) of one source -> our [xt][i][y][xx] block, with the
// per-pixel counts ([y][xl], the slots before the first empty start, as determineNextSupseg reads them)
hipError_t launch_vdi_from_reference(const float4* ref_color, const float* ref_depth, int H, int S, int strip_w,
                                     int strip_tiles, float4* color, float2* depth, uint16_t* counts,
                                     hipStream_t s);
// Variable-length exchange: pack the stored supersegments of every strip block bound
// for another rank (d != skip_d) into per-destination compact messages: meta [b][tiles] {counts u8 x64}
// then [b][tiles] first entries u32; entries pixel-major per tile, placed by one atomic per tile on the
// destination's cursor (cursor[d] = entries packed for d).
struct CompactParams {
    const float4* col;            // slotted send blocks [d][b]
    const float2* dep;
    const uint16_t* pend;         // per brick [y][x] counts (& kPendingCount), stride pend_stride
    size_t pend_stride;
    int W, H, S, B, nstrips, strip_w, strip_tiles, ytiles, skip_d;
    size_t blockE;                // entries per slotted block
    float4* out_col;              // [d] regions of capacity B*blockE entries
    float2* out_dep;
    uint8_t* out_meta;            // [d] regions of meta_bytes
    size_t meta_bytes;
    uint32_t* cursor;             // [d], zeroed before the launch
};
hipError_t launch_vdi_compact(const CompactParams& p, hipStream_t s);
// one compositor input list -> its reference-layout block (the received set, SetOfVDI dumps)
hipError_t launch_vdi_list_to_reference(const VdiList& L, int S, int H, int strip_w, int strip_tiles, float4* ref_color,
                                        float2* ref_depth, hipStream_t s);
// bytes of one destination's meta block: B bricks x tiles x (64 counts + 4-byte first entry)
inline size_t compact_meta_bytes(int B, int strip_tiles, int ytiles) {
    return (size_t)B * (size_t)strip_tiles * (size_t)ytiles * (64 + 4);
}
// simulation array (x-fastest, dims n) -> blocked layout of insitu_sampling.h
hipError_t launch_brick_ingest(const void* src, void* dst, int dtype, int nx, int ny, int nz, hipStream_t s);
// reference-layout readback of one brick's VDI, columns [x0, x0+nx): colour (S,H,nx) rgba32f, depth
// (2S,H,nx) r32f; slots past the pixel's count (pend: per brick [y][x], stride pend_stride; null = all
// S slots stored) read as zero
hipError_t launch_vdi_to_reference(const float4* color, const float2* depth, const uint16_t* pend, size_t pend_stride,
                                   size_t pend_dstride, size_t pend_pitch, int W, int x0, int nx, int H, int S, int strip_w,
                                   int strip_tiles, int B, int b, float4* ref_color, float* ref_depth, hipStream_t s);

}  // namespace insitu
