/*
 * kotlin_units.h -- the argument units of the reference's Kotlin `external` functions, in one place.
 *
 * The Kotlin host computes every size it hands to native code from the window and the supersegment
 * counts; the JNI adaptor (insitu_jni.cpp) and the C harness test (tests/c_harness/) both take their
 * sizes from here, so the units the harness checks against libinsitu_hip.so are the ones the
 * adaptor passes on.
 *
 *   DistributedVolumes.distributeVDIs          DistributedVolumes.kt:860   H*W*S*4/commSize        floats of colour per destination
 *   DistributedVolumes.gatherCompositedVDIs    DistributedVolumes.kt:903   H*W*S_out*4*layers/commSize floats of colour per rank
 *   DistributedVolumeRenderer.distributeVDIs   DistributedVolumeRenderer.kt:577  H*W*S*4/commSize  (plain: S = 1, bytes of rgba8)
 *   DistributedVolumeRenderer.gatherCompositedVDIs  DistributedVolumeRenderer.kt:602  H*W*S_out*4*layers/commSize (plain: bytes)
 *
 * Colour entries are rgba32f (VDI) or rgba8 (plain); VDI depth is (2S,H,W) r32f, i.e. half the
 * floats of the colour; plain depth is rgba8-encoded (EncodeFloatRGBA), the same bytes as the colour.
 */
#ifndef INSITU_KOTLIN_UNITS_H
#define INSITU_KOTLIN_UNITS_H

#ifdef __cplusplus
extern "C" {
#endif

/* sizePerProcess of distributeVDIs (Kotlin Int arithmetic: the product is formed first, then divided) */
static inline long long kt_size_per_process(int W, int H, int S, int commSize) {
    return (long long)H * W * S * 4 / commSize;
}

/* the length argument of both gatherCompositedVDIs (numLayers = 1 in the reference's runs) */
static inline long long kt_gather_len(int W, int H, int S_out, int num_layers, int commSize) {
    return (long long)H * W * S_out * 4 * num_layers / commSize;
}

/* bytes of the received set the native side hands back (allToAllColorPointer / the VDISetColour of
 * compositeVDIs, DistributedVolumeRenderer.kt:684; uploadForCompositing, DistributedVolumes.kt:945) */
static inline long long kt_recv_colour_bytes(int vdi, long long sizePerProcess, int commSize) {
    return sizePerProcess * commSize * (vdi ? 4 : 1);   /* VDI: floats; plain: bytes */
}
static inline long long kt_recv_depth_bytes(int vdi, long long sizePerProcess, int commSize) {
    return vdi ? sizePerProcess * commSize * 4 / 2 : sizePerProcess * commSize;
}

/* bytes of the gathered composited VDI on the root (gatherColorPointer / gatherDepthPointer) */
static inline long long kt_gather_colour_bytes(long long len, int commSize) { return len * commSize * 4; }
static inline long long kt_gather_depth_bytes(long long len, int commSize) { return len * commSize * 4 / 2; }

#ifdef __cplusplus
}
#endif
#endif
