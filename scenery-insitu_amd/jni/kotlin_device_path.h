/*
 * kotlin_device_path.h -- the device-resident frame of libinsitu_hip.so driven with the Kotlin host's own
 * arguments: what the Vulkan dispatch of scenery-insitu's two renderer classes becomes.
 *
 * In the reference the JVM uploads every grid into a scenery Volume (GPU texture) and lets the
 * VolumeManager dispatch VDIGenerator.comp / VolumeRaycaster.comp every frame; a postRenderLambda reads
 * the sub-VDI textures back and hands the host buffers to distributeVDIs / gatherCompositedVDIs:
 *
 *   DistributedVolumeRenderer.updateData(partnerNo, numGrids, grids, origins, gridDims, domainDims)
 *                                                                      DistributedVolumeRenderer.kt:136-160
 *   DistributedVolumeRenderer.updateVolumes() every 20 frames          :521-527, :656-681
 *   DistributedVolumes.addVolume(volumeID, dimensions, pos, is16bit)   DistributedVolumes.kt:147-236
 *   DistributedVolumes.updateVolume(volumeID, buffer)                  :238-245
 *   the per-frame Vulkan dispatch + postRenderLambdas + distributeVDIs + gatherCompositedVDIs
 *                                                                      DistributedVolumes.kt:736-904,
 *                                                                      DistributedVolumeRenderer.kt:450-654
 *   DistributedVolumeRenderer.streamImage(image) on the root           :726
 *
 * Here the grid goes straight to insitu_set_brick (host ByteBuffer through the kept staging buffer, or
 * -- in situ -- the simulation's device pointer, read in place) and ONE call per frame runs render ->
 * exchange -> composite -> gather on the GPU (insitu_frame); the root's image lands in a host buffer
 * that the JNI layer hands to streamImage.  The JNI adaptor (insitu_jni.cpp) and the C harness
 * (tests/c_harness/kotlin_units_harness.c, checked against the oracle) share these bodies.
 */
#ifndef INSITU_KOTLIN_DEVICE_PATH_H
#define INSITU_KOTLIN_DEVICE_PATH_H

#include <string.h>

#include "insitu_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The world matrix of a scenery Volume placed the way the Kotlin host places its grids: origin
 * FrontBottomLeft at `pos`, pixelToWorldRatio world units per voxel (DistributedVolumes.kt:159-165,
 * DistributedVolumeRenderer.kt:351-369): world = pos + pixelToWorld * voxel.  Column-major. */
static inline void kt_volume_model(const float pos[3], float pixelToWorld, float model[16]) {
    memset(model, 0, 16 * sizeof(float));
    model[0] = model[5] = model[10] = pixelToWorld;
    model[12] = pos[0];
    model[13] = pos[1];
    model[14] = pos[2];
    model[15] = 1.0f;
}

/* Grid i of updateData's arrays: its voxel extent (gridDims: start xyz, end xyz per grid, inclusive)
 * and world matrix (origins: voxel offsets, scaled by pixelToWorld as DistributedVolumeRenderer.kt:351-352
 * does before positioning the volume). */
static inline void kt_grid_brick(const int* origins, const int* gridDims, int i, float pixelToWorld, int dims[3],
                                 float model[16]) {
    const int* g = gridDims + 6 * i;
    dims[0] = g[3] - g[0] + 1;
    dims[1] = g[4] - g[1] + 1;
    dims[2] = g[5] - g[2] + 1;
    const float pos[3] = {(float)origins[3 * i] * pixelToWorld, (float)origins[3 * i + 1] * pixelToWorld,
                          (float)origins[3 * i + 2] * pixelToWorld};
    kt_volume_model(pos, pixelToWorld, model);
}

/* updateData / updateVolumes: every grid of this rank becomes brick slot i (u16 voxels, as the
 * reference's asShortBuffer reads them); grids[i] is host memory (on_device == 0: the ByteBuffer's
 * address) or a device pointer of the simulation (on_device != 0).  0 or the failing call's code. */
static inline int kt_update_data(insitu_ctx* c, int numGrids, const void* const* grids, int on_device,
                                 const int* origins, const int* gridDims, float pixelToWorld) {
    for (int i = 0; i < numGrids; ++i) {
        int dims[3];
        float model[16];
        kt_grid_brick(origins, gridDims, i, pixelToWorld, dims, model);
        const int rc = insitu_set_brick(c, i, grids[i], INSITU_U16, dims, model, on_device);
        if (rc) return rc;
    }
    return 0;
}

/* addVolume + updateVolume: the volume's voxels (u8 or u16, DistributedVolumes.kt:155-159) into slot
 * volumeID at pos with pixelToWorld. */
static inline int kt_update_volume(insitu_ctx* c, int volumeID, const void* data, int on_device, const int dims[3],
                                   int is16bit, const float pos[3], float pixelToWorld) {
    float model[16];
    kt_volume_model(pos, pixelToWorld, model);
    return insitu_set_brick(c, volumeID, data, is16bit ? INSITU_U16 : INSITU_U8, dims, model, on_device);
}

/* The camera of a frame from the Kotlin side's matrices: view = cam.spatial().getTransformation(),
 * projection = cam.spatial().projection with applyVulkanCoordinateSystem() applied, and their inverses
 * as the renderer's uniforms carry them (JOML Matrix4f.invert(), DistributedVolumes.kt:718-723); NULL
 * inverses are computed here in double precision.  nw / fwnw: the VolumeManager's shader properties. */
static inline void kt_camera(const float view[16], const float projection[16], const float* inv_view,
                             const float* inv_projection, float nw, float fwnw, insitu_camera* cam) {
    memset(cam, 0, sizeof *cam);
    memcpy(cam->view, view, sizeof cam->view);
    memcpy(cam->proj, projection, sizeof cam->proj);
    cam->has_inverses = (inv_view && inv_projection) ? 1 : 0;
    if (cam->has_inverses) {
        memcpy(cam->inv_view, inv_view, sizeof cam->inv_view);
        memcpy(cam->inv_proj, inv_projection, sizeof cam->inv_proj);
    }
    cam->nw = nw;
    cam->fwnw = fwnw;
    cam->tmax = 1.0f;   /* getMaxDepth(): no opaque geometry in front of the volumes */
}

/* One frame: render -> exchange -> composite -> gather; the root's (H, W) rgba8 image goes to `image`
 * (cap >= W*H*4), what streamImage receives.  Other ranks pass NULL. */
static inline int kt_frame(insitu_ctx* c, const float view[16], const float projection[16], const float* inv_view,
                           const float* inv_projection, float nw, float fwnw, void* image, size_t cap) {
    insitu_camera cam;
    kt_camera(view, projection, inv_view, inv_projection, nw, fwnw, &cam);
    return insitu_frame(c, &cam, image, cap);
}

/* insituFramePipelined: the reference's own loop, one frame stale (DistributedVolumeRenderer.kt:530-542 composites
 * the previous render frame while it distributes the current one): this call's camera starts a render and the
 * previous frame completes; *done = the completed frame's index (-1 on the first call), `image` holds its image
 * on the root.  kt_frame_flush completes the frame still in flight (insitu_frame_pipelined / _flush). */
static inline int kt_frame_pipelined(insitu_ctx* c, const float view[16], const float projection[16],
                                     const float* inv_view, const float* inv_projection, float nw, float fwnw,
                                     void* image, size_t cap, long long* done) {
    insitu_camera cam;
    kt_camera(view, projection, inv_view, inv_projection, nw, fwnw, &cam);
    return insitu_frame_pipelined(c, &cam, image, cap, done);
}
static inline int kt_frame_flush(insitu_ctx* c, void* image, size_t cap, long long* done) {
    return insitu_pipeline_flush(c, image, cap, done);
}

#ifdef __cplusplus
}
#endif
#endif
