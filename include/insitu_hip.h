/*
 * insitu_hip.h -- C ABI of libinsitu_hip.so, the MI355X-native replacement for the
 * native half of scenery-insitu's distributed VDI volume-rendering path.
 *
 * In the reference, the Kotlin host (DistributedVolumeRenderer.kt / DistributedVolumes.kt)
 * renders sub-VDIs with Vulkan compute shaders, reads them back to host ByteBuffers and
 * hands them to external native code (OpenFPM's InVis.cpp, README.md:19) through
 *   external fun distributeVDIs(...)        DistributedVolumeRenderer.kt:112, DistributedVolumes.kt:136-137
 *   external fun gatherCompositedVDIs(...)  DistributedVolumeRenderer.kt:113, DistributedVolumes.kt:138-139
 * which run MPI_Alltoall / MPI_Gather and call back into Kotlin (compositeVDIs :684,
 * uploadForCompositing DistributedVolumes.kt:945, streamImage :726).
 *
 * Here the whole frame stays on the GPU: insitu_render replaces the Vulkan dispatch of
 * VDIGenerator.comp+AccumulateVDI.comp (or VolumeRaycaster.comp+AccumulatePlainImage.comp),
 * insitu_exchange replaces distributeVDIs' MPI_Alltoall (RCCL over xGMI, device buffers),
 * insitu_composite replaces the compositor dispatch (PlainImageCompositor.comp, or the VDI
 * flatten of VDIGenerator.comp:147-185 in VDICompositor.comp:58-91 order), and
 * insitu_gather replaces gatherCompositedVDIs' MPI_Gather.  The reference-shaped entry
 * points at the bottom keep the exact Kotlin argument lists for a JNI shim
 * (INTEGRATION.md).
 *
 * Conventions: 0 = success, negative = error (insitu_last_error() has the text).  A context
 * is owned by one thread.  Calls are ordered on the context's HIP stream; insitu_gather,
 * insitu_read and insitu_synchronize block.  Matrices are column-major float[16] (GLSL/JOML).
 */
#ifndef INSITU_HIP_H
#define INSITU_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INSITU_ABI_VERSION 8
#define INSITU_COMM_ID_BYTES 128

typedef struct insitu_ctx insitu_ctx;
/* In-process rank group: the contexts of all ranks live in one process (on any devices) and the
 * exchange/gather copy device to device instead of RCCL.  Used to run the multi-rank data path
 * on one GPU (RCCL refuses two ranks per device); each stage must then be called for every rank
 * before the next stage starts (render all, exchange all, composite all, gather all). */
typedef struct insitu_local_group insitu_local_group;

enum insitu_mode {
    INSITU_MODE_PLAIN = 0, /* DistributedVolumeRenderer.kt: generateVDIs = false (:78)  */
    INSITU_MODE_VDI = 1    /* DistributedVolumes.kt:      generateVDIs = true  (:88)  */
};

enum insitu_dtype { INSITU_U8 = 0, INSITU_U16 = 1, INSITU_F32 = 2 };

enum insitu_buf {
    INSITU_BUF_VDI_COLOR = 0,   /* brick `slot`: (S,H,W) rgba32f, reference layout (DistributedVolumes.kt:349-358) */
    INSITU_BUF_VDI_DEPTH = 1,   /* brick `slot`: (2S,H,W) r32f (DistributedVolumes.kt:360-368)                    */
    INSITU_BUF_OCTREE = 2,      /* brick `slot`: (W/8,H/8,S) r32ui OctreeCells (DistributedVolumes.kt:342,370-374)  */
    INSITU_BUF_PASSES = 3,      /* brick `slot`: H*W uint8 raymarch passes per pixel (needs keep_passes)          */
    INSITU_BUF_PLAIN_COLOR = 4, /* brick `slot`: (dim0,dim1) rgba8 OutputSubVDIColor (DistributedVolumeRenderer.kt:214) */
    INSITU_BUF_PLAIN_DEPTH = 5, /* brick `slot`: (dim0,dim1) rgba8 OutputSubVDIDepth (EncodeFloatRGBA(tnear))      */
    INSITU_BUF_STRIP = 6,       /* this rank's composited strip, rgba8 (VDI: H x W/P row-major; plain: rows x dim0) */
    INSITU_BUF_IMAGE = 7,       /* root: gathered full image rgba8, row-major (H,W) / (dim1,dim0)                  */
    /* composite_vdi contexts (VDICompositor.comp output, DistributedVolumes.kt:423-431):              */
    INSITU_BUF_COMPOSITED_COLOR = 8,  /* this rank's strip: (S_out,H,W/P) rgba32f CompositedVDIColor     */
    INSITU_BUF_COMPOSITED_DEPTH = 9,  /* this rank's strip: (2S_out,H,W/P) r32f CompositedVDIDepth       */
    INSITU_BUF_GATHERED_COLOR = 10,   /* root: (S_out,H,W) rgba32f, the gathered composited VDI          */
    INSITU_BUF_GATHERED_DEPTH = 11,   /* root: (2S_out,H,W) r32f                                         */
    INSITU_BUF_COMPOSITE_PASSES = 12, /* this rank's strip: H*(W/P) uint8 compositor search passes      */
    /* VDI mode, after insitu_exchange (or insitu_distribute_vdis): the set this rank composites, in the
     * reference layout -- nranks * bricks source-major blocks of (S,H,W/P) rgba32f / (2S,H,W/P) r32f,
     * empty slots zero: what allToAllColorPointer holds and uploadForCompositing receives
     * (DistributedVolumes.kt:945), dumped as SetOfVDI{n}_ndc_col / _ndc_depth (:974-975)        */
    INSITU_BUF_RECEIVED_COLOR = 13,
    INSITU_BUF_RECEIVED_DEPTH = 14
};

typedef struct insitu_config {
    int rank;              /* DistributedVolumes.rank (:104)                               */
    int nranks;            /* commSize (:103)                                              */
    int device;            /* nodeRank -> scenery.Renderer.DeviceId (:450-451)             */
    int width, height;     /* window W,H; plain mode: texture dims (dim0, dim1)             */
    int max_supersegments; /* maxSupersegments S (DistributedVolumes.kt:99); plain: 1      */
    int mode;              /* enum insitu_mode                                              */
    int bricks_per_rank;   /* bricks (volumes) rendered by this rank; each is one sub-VDI   */
    const void* comm_id;   /* INSITU_COMM_ID_BYTES from insitu_comm_id() on rank 0; NULL if nranks == 1 */
    void* stream;          /* hipStream_t to run on; NULL -> the context creates one        */
    int keep_passes;       /* record per-pixel raymarch pass counts (INSITU_BUF_PASSES)     */
    int sample_cache_mb;   /* VDI mode: HBM for the per-sample raymarch cache, MiB; 0 = default
                              (512 B per pixel per brick at first, grown after a frame whose rays did
                              not fit to 1.25x that frame's demand, at most 45 % of the HBM free at
                              create), > 0 = fixed size, < 0 = off */
    int composite_vdi;     /* VDI mode: 0 = insitu_composite flattens the merged lists to RGBA
                              (accumulateSupseg, VDIGenerator.comp:147-185); 1 = VDICompositor.comp:
                              re-supersegment them into a composited VDI of max_output_supersegments
                              per pixel, gathered to rank 0 (DistributedVolumes.kt:903)         */
    int max_output_supersegments; /* maxOutputSupersegments S_out (DistributedVolumes.kt:100); 0 -> S */
    insitu_local_group* local_group; /* non-NULL: in-process rank group instead of RCCL (comm_id unused) */
    int faithful;          /* bit mask of enum insitu_faithful: reproduce a reference quirk instead of the
                              default (corrected) behaviour, for parity with the shaders as written */
    int merge_bricks;      /* VDI mode: 1 = the rank's bricks are the volumes of ONE sub-VDI, as
                              VDIGenerator.comp renders all of a rank's grids ($repeat over volumes,
                              :333-347; several grids per compute partner, DistributedVolumeRenderer.kt:57-63);
                              0 = every brick is its own sub-VDI (a virtual rank).  Merged volumes run
                              the threshold search through the per-sample cache too (64-byte slots that
                              carry each sample's step index)                   */
} insitu_config;

/* Reference quirks (default off: the corrected behaviour). */
enum insitu_faithful {
    /* VDICompositor.comp:204: ndc_x from gl_GlobalInvocationID.x, the strip-LOCAL column, over the
     * full window width (default: the pixel's global column; the two agree on rank 0 only) */
    INSITU_FAITHFUL_COMPOSITOR_NDC_X = 1,
    /* PlainImageCompositor.comp:43: numProcesses = imageSize.r / imageSize.g = dim0 * nranks / dim1
     * (default: every list; the two agree for square windows) */
    INSITU_FAITHFUL_PLAIN_NUM_PROCESSES = 2
};

typedef struct insitu_camera {
    float view[16];     /* LightParameters.ViewMatrices[0]                                 */
    float proj[16];     /* LightParameters.ProjectionMatrix (Vulkan-corrected, DistributedVolumes.kt:67-79) */
    float inv_view[16]; /* InverseViewMatrices[0]  (used when has_inverses != 0)           */
    float inv_proj[16]; /* InverseProjectionMatrix (used when has_inverses != 0)           */
    int has_inverses;   /* 0 -> computed here in double precision                          */
    float nw;           /* VolumeManager shaderProperties["nw"] (DistributedVolumes.kt:713) */
    float fwnw;         /* plain mode only (VolumeRaycaster.comp:133-139)                   */
    float tmax;         /* getMaxDepth(): 1.0 = no opaque geometry                          */
} insitu_camera;

typedef struct insitu_stats {
    float ms_render, ms_exchange, ms_composite, ms_gather; /* HIP-event times of the last frame */
    float ms_sample, ms_search;  /* VDI render split: first-pass sampling kernel / threshold-search kernel */
    /* VDI render counters of the last frame (all local bricks): */
    long long rays_searched;     /* rays queued for the threshold search after the first pass        */
    long long rays_uncached;     /* rays that hit a brick but got no per-sample cache space: searched
                                    by re-sampling the brick every pass (same results, slower)       */
    long long cache_bytes;       /* capacity of the per-sample cache                                 */
    long long exchange_bytes;    /* bytes this rank sent to peers in the last exchange (VDI mode:
                                    the compact messages -- counts, tile offsets, stored entries)     */
    long long exchange_entries;  /* supersegment entries this rank sent to peers (VDI mode)          */
    float ms_compact;            /* VDI mode, nranks > 1: packing the stored supersegments bound for
                                    the peers (counted in ms_exchange, not in ms_render)              */
    float ms_exchange_sync;      /* VDI mode, nranks > 1: GPU idle time of the exchange's host round trip
                                    (the receive sizes reach the host before the payload is enqueued) */
    long long cache_demand_bytes; /* per-sample cache the last render's rays asked for (fits when
                                    <= cache_bytes; a default-sized cache grows to it)               */
    int search_regroups;         /* VDI mode: waves of the threshold search that re-formed their lanes into
                                    deeper search trees once the queue was drained (INSITU_OPT_REGROUP) */
    float ms_image_d2h;          /* root: copy of the final image to the host buffer of insitu_gather
                                    (what streamImage receives, DistributedVolumeRenderer.kt:726); 0 when
                                    no host buffer was passed                                          */
    float ms_latency;            /* render start to the image on the host (or the gather's end) of the
                                    frame: with insitu_frame_pipelined it spans the next frame's start   */
    int pipelined;               /* 1: the frame was rendered by insitu_frame_pipelined (its render starts
                                    at its trigger: its prepare was queued ahead of it)   */
    float ms_ingest;             /* GPU time of the last batch of insitu_set_brick re-ingests (the bricks set
                                    between two renders; 0 until one has completed)                     */
} insitu_stats;

/* Tuning and diagnostics options (insitu_set_option); the defaults are the measured optimum. */
enum insitu_option {
    INSITU_OPT_EXACT_SEARCH = 0,   /* 1: every supersegment decision by the exact contract path
                                      (default 0: filtered decisions -- identical results)         */
    INSITU_OPT_SEARCH_DEPTH = 1,   /* 0 = from the queue length; 1..6 tree levels per replay round */
    INSITU_OPT_LONG_SAMPLES = 2,   /* rays with at least this many samples are searched first      */
    INSITU_OPT_ROUND_BATCH = 3,    /* 1..64: lanes that end a search round together                */
    INSITU_OPT_SEARCH_OVERSUB = 4, /* 1..64: queue length x group size per resident search lane    */
    INSITU_OPT_TILE_ORDER = 5,     /* 1 (default): sampling tiles longest-first; 0: plain XCD order */
    /* 6 and 7 (ABI 6: the fused generator modes, measured slower and removed in ABI 7) are rejected */
    INSITU_OPT_SUPER_TILE = 8,     /* 1, 2 or 4: the longest-first order sorts super-tiles of this many
                                      tiles per edge, a super-tile's tiles kept together (one XCD's L2) */
    INSITU_OPT_REGROUP = 9,        /* 1 (default): once the search queue is drained, a wave deals its lanes
                                      out again so the rays left get deeper search trees; 0: off        */
    INSITU_OPT_EXACT_TILE_KEYS = 10, /* 1: the longest-first order keys a tile by all 64 of its rays;
                                      0 (default): by 16 of them (frames that size the cache: all)      */
    /* insitu_frame_pipelined: when frame k+1's first pass (the sampling kernel) may start beside frame k */
    INSITU_OPT_PIPE_TRIGGER = 11,  /* 0: after frame k's threshold search; 1: when frame k's search queue is
                                      drained (its tail: the rays in flight); 2 (default): at once (after
                                      frame k's first pass, sharing the GPU with its whole search, whose
                                      grid leaves it wave slots: INSITU_OPT_PIPE_SEARCH_RAYS)              */
    INSITU_OPT_PIPE_OVERSUB = 12,  /* 1..64: INSITU_OPT_SEARCH_OVERSUB of pipelined frames (default 3; their
                                      search shares the GPU with the next frame's first pass, so fewer
                                      speculative tree lanes pay: DESIGN.md 5.1)                          */
    INSITU_OPT_PIPE_SEARCH_RAYS = 13 /* pipelined frames: queued rays per searching block of the threshold
                                      search, which then keeps one to two blocks per CU and leaves the other
                                      wave slots to the next frame's first pass (default 2048; 0 = the full
                                      persistent grid, as unpipelined frames)                              */
};

int insitu_abi_version(void);
/* ncclUniqueId for a multi-rank context; call on rank 0 and broadcast the bytes. */
int insitu_comm_id(void* out, size_t cap);
int insitu_create(const insitu_config* cfg, insitu_ctx** out);
int insitu_local_group_create(int nranks, insitu_local_group** out);
void insitu_local_group_destroy(insitu_local_group* g);
void insitu_destroy(insitu_ctx* ctx);
/* last error of ctx, or of the last failed insitu_create when ctx == NULL */
const char* insitu_last_error(const insitu_ctx* ctx);

/* Brick upload: replaces addVolume/updateVolume (DistributedVolumes.kt:147-250) and
 * updateData (DistributedVolumeRenderer.kt:136-160).  data is x-fastest dims[0]*dims[1]*dims[2]
 * voxels; data_on_device != 0 means `data` is a device pointer (in-situ zero-copy source, read
 * in place on the context's stream: the work that produced it must be complete, or run on
 * cfg.stream).  model = world matrix of the volume (position, pixelToWorldRatio, origin). */
int insitu_set_brick(insitu_ctx* ctx, int slot, const void* data, int dtype, const int dims[3],
                     const float model[16], int data_on_device);
/* Transfer function (alpha LUT), colour map (rgba LUT) and converter (display range):
 * raw = normalised_voxel * conv_scale + conv_offset, normalised_voxel = v/255, v/65535 or v. */
int insitu_set_transfer(insitu_ctx* ctx, const float* tf, int n_tf, const float* cmap_rgba, int n_cm,
                        float conv_scale, float conv_offset);

/* Camera of the frame (the VDI metadata's view/projection; DistributedVolumes.kt:718-723).
 * insitu_render sets it too; the host-buffer path needs it before insitu_distribute_vdis. */
int insitu_set_camera(insitu_ctx* ctx, const insitu_camera* cam);
int insitu_render(insitu_ctx* ctx, const insitu_camera* cam);   /* all local bricks        */
int insitu_exchange(insitu_ctx* ctx);                          /* screen-strip all-to-all */
int insitu_composite(insitu_ctx* ctx);                         /* sort-last merge of strip */
/* Gather the strips on rank 0.  Root copies the (H,W) rgba8 image to host_out when non-NULL
 * (cap >= W*H*4); other ranks ignore host_out. */
int insitu_gather(insitu_ctx* ctx, void* host_out, size_t cap);
int insitu_frame(insitu_ctx* ctx, const insitu_camera* cam, void* host_out, size_t cap);
/* Pipelined frames, the reference's own loop (DistributedVolumeRenderer.kt:530-542, 577, 602-603: the
 * composite it reads is one frame stale): enqueue frame k's render (camera `cam`) and, while it runs, complete
 * frame k-1 -- exchange, composite, gather, the root's image to host_out -- and return when that is done, with
 * *done_frame = k-1 (-1 for the first call; frames count from 0 per context).  Frame k's first pass runs on
 * a second stream and starts in frame k-1's search tail (INSITU_OPT_PIPE_TRIGGER), so the GPU does not idle
 * between frames.  insitu_read / insitu_read_region / insitu_get_stats / insitu_pass_stats then describe
 * frame k-1.  The second frame's buffers are allocated at the first call (VDI mode, sample cache on, not
 * with a local group).  insitu_set_brick between calls is ordered before the next render; the unpipelined
 * stage calls fail while a frame is in flight. */
int insitu_frame_pipelined(insitu_ctx* ctx, const insitu_camera* cam, void* host_out, size_t cap,
                           long long* done_frame);
/* Complete the frame in flight (as insitu_frame_pipelined's second half); *done_frame = its index, or -1
 * when none was in flight. */
int insitu_pipeline_flush(insitu_ctx* ctx, void* host_out, size_t cap, long long* done_frame);
int insitu_synchronize(insitu_ctx* ctx);
/* Copy a buffer to host in the reference layout (enum insitu_buf). */
int insitu_read(insitu_ctx* ctx, int which, int slot, void* host_out, size_t cap);
size_t insitu_buffer_bytes(const insitu_ctx* ctx, int which);
/* Columns [x0, x1) of brick `slot`'s VDI in the reference layout: INSITU_BUF_VDI_COLOR (x1-x0, H, S)
 * rgba32f, INSITU_BUF_VDI_DEPTH (x1-x0, H, 2S) r32f (x slowest, as (S,H,W) images), or
 * INSITU_BUF_PASSES (H, x1-x0) uint8 -- parity checks of frames too large to read whole. */
int insitu_read_region(insitu_ctx* ctx, int which, int slot, int x0, int x1, void* host_out, size_t cap);
int insitu_get_stats(insitu_ctx* ctx, insitu_stats* out);
/* Set a tuning option (enum insitu_option) for the following renders; -1 on an unknown option or
 * a value out of range.  Environment variables INSITU_<OPTION NAME> (INSITU_EXACT_SEARCH,
 * INSITU_SEARCH_DEPTH, ..., INSITU_PIPE_TRIGGER) seed the values when the context is created (tuning scripts). */
int insitu_set_option(insitu_ctx* ctx, int option, long long value);
/* Mean raymarch passes over rays that hit a brick, and the number of such rays, of the last
 * render over all local bricks (needs keep_passes; reads the pass buffer back). */
int insitu_pass_stats(insitu_ctx* ctx, double* mean_passes, long long* rays_hit);
void* insitu_stream(insitu_ctx* ctx);

/* ---- reference-shaped entry points (host ByteBuffers, reference layouts) ----
 * distributeVDIs(subVDIColor, subVDIDepth, sizePerProcess, commSize, colPointer, depthPointer,
 * mpiPointer), DistributedVolumes.kt:136-137 / DistributedVolumeRenderer.kt:112: all-to-all of
 * the host sub-VDI (VDI mode: sizePerProcess = H*W*S*4/commSize floats of colour per
 * destination, depth = half of that; plain mode: bytes of rgba8 per destination, same for
 * depth), received blocks written to recvColor/recvDepth (the native-owned
 * allToAllColorPointer/allToAllDepthPointer), then the composite of this rank's strip is run on
 * the GPU from them (what compositeVDIs/uploadForCompositing trigger). */
int insitu_distribute_vdis(insitu_ctx* ctx, const void* subVDIColor, const void* subVDIDepth,
                           long long sizePerProcess, int commSize, void* recvColor, void* recvDepth);

/* gatherCompositedVDIs(compositedVDIColor, compositedVDIDepth, compositedVDILen, root, myRank, commSize,
 * colPointer, depthPointer, mpiPointer), DistributedVolumes.kt:138-139 / :903-904 (composite_vdi
 * contexts): gathers the composited VDI strips on root 0; compositedVDILen = H*W*S_out*4/commSize
 * floats of colour per rank.  The root's gatherColor receives (S_out,H,W) rgba32f and gatherDepth
 * (2S_out,H,W) r32f (the native-owned gatherColorPointer/gatherDepthPointer); other ranks pass NULL. */
int insitu_gather_composited_vdi_set(insitu_ctx* ctx, long long compositedVDILen, int root, int myRank, int commSize,
                                     void* gatherColor, void* gatherDepth);

/* gatherCompositedVDIs(compositedVDIColor, root, subVDILen, myRank, commSize, ...)
 * (DistributedVolumeRenderer.kt:113, :602-603): gathers the composited rgba8 strips on root 0
 * (subVDILen = H*W*4/commSize bytes); the root's full image goes to gatherOut (what streamImage
 * receives, DistributedVolumeRenderer.kt:726).  Requires bricks_per_rank == 1 like the reference. */
int insitu_gather_composited_vdis(insitu_ctx* ctx, int root, long long subVDILen, int myRank, int commSize,
                                  void* gatherOut, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
