// insitu_jni.cpp -- JNI adaptor: the four Kotlin `external` functions of scenery-insitu's distributed
// volume path, implemented over libinsitu_hip.so's C ABI (include/insitu_hip.h) instead of the MPI
// half of OpenFPM's InVis.cpp (README.md:19).
//
//   DistributedVolumes.distributeVDIs(subVDIColor, subVDIDepth, sizePerProcess, commSize,
//                                     colPointer, depthPointer, mpiPointer)       DistributedVolumes.kt:136-137
//   DistributedVolumes.gatherCompositedVDIs(compositedVDIColor, compositedVDIDepth, compositedVDILen,
//                                     root, myRank, commSize, colPointer, depthPointer, mpiPointer)
//                                                                                    DistributedVolumes.kt:138-139
//   DistributedVolumeRenderer.distributeVDIs(subVDIColor, subVDIDepth?, sizePerProcess, commSize,
//                                     generateVDIS)                                 DistributedVolumeRenderer.kt:112
//   DistributedVolumeRenderer.gatherCompositedVDIs(compositedVDIColor, root, subVDILen, myRank,
//                                     commSize, generateVDIS, saveFiles)             DistributedVolumeRenderer.kt:113
//
// and the Kotlin callbacks the native side makes after them, as InVis.cpp does:
//   uploadForCompositing(vdiSetColour, vdiSetDepth)                 DistributedVolumes.kt:945
//   compositeVDIs(VDISetColour, VDISetDepth, sizePerProcess)        DistributedVolumeRenderer.kt:684
//   streamImage(image)                                              DistributedVolumeRenderer.kt:726
//
// Which context: the launcher that starts the JVM (the OpenFPM side) creates one insitu_ctx per rank
// (insitu_create with the ncclUniqueId broadcast over its own MPI communicator) and either passes
// its address as the `mpiPointer` Long -- the slot through which InVis.cpp handed Kotlin its MPI
// communicator -- or registers it with insitu_jni_set_context() for DistributedVolumeRenderer, whose
// externals carry no pointer.  The composite already runs on the GPU inside insitu_distribute_vdis,
// so the callbacks receive the exchanged set only for dumps and bookkeeping (vdisComposited).
//
// Sizes come from kotlin_units.h, the header the C harness test (tests/c_harness/) checks against
// the library.  Built only when a JDK is present: `make -C scenery-insitu_amd jni` (JAVA_HOME).
//
// The device-resident frame (replacing the Vulkan dispatch, not only the MPI half): externals a
// maintainer adds to the two Kotlin classes (INTEGRATION.md lists the declarations and the calls
// that replace the VolumeManager dispatch and the postRenderLambdas), over kotlin_device_path.h,
// whose bodies the C harness drives against the oracle:
//   DistributedVolumeRenderer.insituUpdateData(numGrids, grids, origins, gridDims, pixelToWorld)
//       updateData / updateVolumes (:136-160, :656-681): the OpenFPM grids' ByteBuffers -> bricks
//   DistributedVolumeRenderer.insituUpdateDataDevice(numGrids, devicePointers, origins, gridDims, pixelToWorld)
//       the same for a simulation whose grids live on the GPU (read in place, no host copy)
//   DistributedVolumeRenderer.insituFrame(view, projection, invView, invProjection, nw, fwnw)
//   DistributedVolumeRenderer.insituFramePipelined(view, projection, invView, invProjection, nw, fwnw): Long
//   DistributedVolumeRenderer.insituFrameFlush(): Long
//       one frame on the GPU; the root then calls streamImage(image) (:726)
//   DistributedVolumes.insituUpdateVolume(volumeID, buffer, dimensions, pos, is16bit, pixelToWorld, mpiPointer)
//       addVolume + updateVolume (DistributedVolumes.kt:147-245)
//   DistributedVolumes.insituFrame(view, projection, invView, invProjection, nw, colPointer, depthPointer, mpiPointer)
//       one frame (VDICompositor output); the root's gathered composited VDI lands in
//       gatherColorPointer / gatherDepthPointer, as gatherCompositedVDIs leaves it (:903-904)
#include <jni.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "insitu_hip.h"
#include "kotlin_device_path.h"
#include "kotlin_units.h"

namespace {

insitu_ctx* g_ctx = nullptr;   // DistributedVolumeRenderer's context (insitu_jni_set_context)

struct NativeBuffers {         // what InVis.cpp allocates for DistributedVolumeRenderer
    std::vector<unsigned char> recv_colour, recv_depth, image;
};
std::mutex g_mu;
std::unordered_map<insitu_ctx*, NativeBuffers> g_buffers;

NativeBuffers& buffers_of(insitu_ctx* c) {
    std::lock_guard<std::mutex> lock(g_mu);
    return g_buffers[c];
}

insitu_ctx* context_of(jlong mpiPointer) {
    return mpiPointer ? reinterpret_cast<insitu_ctx*>(mpiPointer) : g_ctx;
}

// the reference logs and carries on; a failed frame here raises in the Kotlin caller instead
void throw_error(JNIEnv* env, insitu_ctx* c, const char* what) {
    if (env->ExceptionCheck()) return;
    jclass k = env->FindClass("java/lang/RuntimeException");
    std::string msg = std::string(what) + ": " + insitu_last_error(c);
    if (k) env->ThrowNew(k, msg.c_str());
}

void* direct(JNIEnv* env, jobject buf) { return buf ? env->GetDirectBufferAddress(buf) : nullptr; }

void call_void(JNIEnv* env, jobject self, const char* name, const char* sig, jobject a, jobject b) {
    jclass k = env->GetObjectClass(self);
    jmethodID m = env->GetMethodID(k, name, sig);
    if (!m) return;   // NoSuchMethodError pending
    env->CallVoidMethod(self, m, a, b);
}

bool floats16(JNIEnv* env, jfloatArray a, float out[16]) {
    if (!a || env->GetArrayLength(a) != 16) return false;
    env->GetFloatArrayRegion(a, 0, 16, out);
    return true;
}

// updateData's grid arrays: numGrids grids, 3 origin and 6 extent ints each
bool grid_arrays(JNIEnv* env, jint numGrids, jintArray origins, jintArray gridDims, std::vector<jint>& o,
                 std::vector<jint>& g) {
    if (numGrids < 1 || !origins || !gridDims || env->GetArrayLength(origins) < 3 * numGrids ||
        env->GetArrayLength(gridDims) < 6 * numGrids)
        return false;
    o.resize((size_t)3 * numGrids);
    g.resize((size_t)6 * numGrids);
    env->GetIntArrayRegion(origins, 0, 3 * numGrids, o.data());
    env->GetIntArrayRegion(gridDims, 0, 6 * numGrids, g.data());
    return true;
}

// a frame's camera: view and projection (Vulkan-corrected), their inverses (null: computed natively)
bool frame_matrices(JNIEnv* env, jfloatArray view, jfloatArray projection, jfloatArray invView,
                    jfloatArray invProjection, float v[16], float p[16], float iv[16], float ip[16], bool& inverses) {
    if (!floats16(env, view, v) || !floats16(env, projection, p)) return false;
    inverses = invView && invProjection;
    if (inverses && (!floats16(env, invView, iv) || !floats16(env, invProjection, ip))) return false;
    return true;
}

}  // namespace

extern "C" {

// Register DistributedVolumeRenderer's context (its externals carry no pointer); NULL unregisters.
JNIEXPORT void insitu_jni_set_context(insitu_ctx* ctx) { g_ctx = ctx; }

// ---------------------------------------------------------------- DistributedVolumes (VDI mode)
JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumes_distributeVDIs(
        JNIEnv* env, jobject self, jobject subVDIColor, jobject subVDIDepth, jint sizePerProcess, jint commSize,
        jlong colPointer, jlong depthPointer, jlong mpiPointer) {
    insitu_ctx* c = context_of(mpiPointer);
    void* col = direct(env, subVDIColor);
    void* dep = direct(env, subVDIDepth);
    if (!c || !col || !dep) {
        throw_error(env, c, "distributeVDIs: no context or a non-direct ByteBuffer");
        return;
    }
    // allToAllColorPointer / allToAllDepthPointer: the received set, source-major (native-owned)
    if (insitu_distribute_vdis(c, col, dep, sizePerProcess, commSize, reinterpret_cast<void*>(colPointer),
                               reinterpret_cast<void*>(depthPointer)) != 0) {
        throw_error(env, c, "distributeVDIs");
        return;
    }
    const jlong cb = kt_recv_colour_bytes(1, sizePerProcess, commSize);
    const jlong db = kt_recv_depth_bytes(1, sizePerProcess, commSize);
    jobject setC = env->NewDirectByteBuffer(reinterpret_cast<void*>(colPointer), cb);
    jobject setD = env->NewDirectByteBuffer(reinterpret_cast<void*>(depthPointer), db);
    call_void(env, self, "uploadForCompositing", "(Ljava/nio/ByteBuffer;Ljava/nio/ByteBuffer;)V", setC, setD);
}

JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumes_gatherCompositedVDIs(
        JNIEnv* env, jobject /*self*/, jobject /*compositedVDIColor*/, jobject /*compositedVDIDepth*/,
        jint compositedVDILen, jint root, jint myRank, jint commSize, jlong colPointer, jlong depthPointer,
        jlong mpiPointer) {
    // the composited strip is already in HBM (the composite ran in distributeVDIs); the Kotlin
    // buffers fetched from the compositor textures are not needed.  Root receives the (S_out,H,W)
    // colour and (2S_out,H,W) depth into gatherColorPointer / gatherDepthPointer.
    insitu_ctx* c = context_of(mpiPointer);
    const bool is_root = myRank == root;
    if (!c || insitu_gather_composited_vdi_set(c, compositedVDILen, root, myRank, commSize,
                                               is_root ? reinterpret_cast<void*>(colPointer) : nullptr,
                                               is_root ? reinterpret_cast<void*>(depthPointer) : nullptr) != 0)
        throw_error(env, c, "gatherCompositedVDIs");
}

// ---------------------------------------------------------- DistributedVolumeRenderer (plain mode)
JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_distributeVDIs(
        JNIEnv* env, jobject self, jobject subVDIColor, jobject subVDIDepth, jint sizePerProcess, jint commSize,
        jboolean generateVDIS) {
    insitu_ctx* c = g_ctx;
    void* col = direct(env, subVDIColor);
    void* dep = direct(env, subVDIDepth);   // null when generateVDIS (no separate depth texture, :498-501)
    if (!c || !col || !dep) {
        throw_error(env, c, "distributeVDIs: no context, a non-direct ByteBuffer, or no depth buffer "
                            "(a VDI context needs the separate depth: use DistributedVolumes)");
        return;
    }
    const int vdi = generateVDIS ? 1 : 0;
    NativeBuffers& nb = buffers_of(c);
    nb.recv_colour.resize((size_t)kt_recv_colour_bytes(vdi, sizePerProcess, commSize));
    nb.recv_depth.resize((size_t)kt_recv_depth_bytes(vdi, sizePerProcess, commSize));
    if (insitu_distribute_vdis(c, col, dep, sizePerProcess, commSize, nb.recv_colour.data(), nb.recv_depth.data()) != 0) {
        throw_error(env, c, "distributeVDIs");
        return;
    }
    jobject setC = env->NewDirectByteBuffer(nb.recv_colour.data(), (jlong)nb.recv_colour.size());
    jobject setD = env->NewDirectByteBuffer(nb.recv_depth.data(), (jlong)nb.recv_depth.size());
    jclass k = env->GetObjectClass(self);
    jmethodID m = env->GetMethodID(k, "compositeVDIs", "(Ljava/nio/ByteBuffer;Ljava/nio/ByteBuffer;I)V");
    if (m) env->CallVoidMethod(self, m, setC, setD, sizePerProcess);
}

JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_gatherCompositedVDIs(
        JNIEnv* env, jobject self, jobject /*compositedVDIColor*/, jint root, jint subVDILen, jint myRank,
        jint commSize, jboolean /*generateVDIS*/, jboolean /*saveFiles*/) {
    insitu_ctx* c = g_ctx;
    if (!c) {
        throw_error(env, c, "gatherCompositedVDIs: no context (insitu_jni_set_context)");
        return;
    }
    NativeBuffers& nb = buffers_of(c);
    const bool is_root = myRank == root;
    nb.image.resize(is_root ? (size_t)subVDILen * (size_t)commSize : 0);
    if (insitu_gather_composited_vdis(c, root, subVDILen, myRank, commSize, is_root ? nb.image.data() : nullptr,
                                      nb.image.size()) != 0) {
        throw_error(env, c, "gatherCompositedVDIs");
        return;
    }
    if (is_root) {   // streamImage(image), DistributedVolumeRenderer.kt:726
        jobject img = env->NewDirectByteBuffer(nb.image.data(), (jlong)nb.image.size());
        jclass k = env->GetObjectClass(self);
        jmethodID m = env->GetMethodID(k, "streamImage", "(Ljava/nio/ByteBuffer;)V");
        if (m) env->CallVoidMethod(self, m, img);
    }
}

// ------------------------------------------------ device-resident frame (replaces the Vulkan dispatch)
JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_insituUpdateData(
        JNIEnv* env, jobject /*self*/, jint numGrids, jobjectArray grids, jintArray origins, jintArray gridDims,
        jfloat pixelToWorld) {
    insitu_ctx* c = g_ctx;
    std::vector<jint> o, g;
    if (!c || !grids || env->GetArrayLength(grids) < numGrids || !grid_arrays(env, numGrids, origins, gridDims, o, g)) {
        throw_error(env, c, "insituUpdateData: no context or inconsistent grid arrays");
        return;
    }
    std::vector<const void*> ptr((size_t)numGrids);
    for (jint i = 0; i < numGrids; ++i) {
        // u16 voxels over the grid's inclusive extent (kt_grid_brick): the buffer must hold all of them
        const jint* e = g.data() + 6 * (size_t)i;
        const long long nx = (long long)e[3] - e[0] + 1, ny = (long long)e[4] - e[1] + 1, nz = (long long)e[5] - e[2] + 1;
        jobject b = env->GetObjectArrayElement(grids, i);
        ptr[(size_t)i] = direct(env, b);
        const long long cap = b ? (long long)env->GetDirectBufferCapacity(b) : -1;
        if (b) env->DeleteLocalRef(b);
        if (!ptr[(size_t)i]) {
            throw_error(env, c, "insituUpdateData: a grid is not a direct ByteBuffer");
            return;
        }
        if (nx <= 0 || ny <= 0 || nz <= 0 || cap < nx * ny * nz * 2) {
            throw_error(env, c, "insituUpdateData: a grid's buffer is smaller than its extent (u16 voxels)");
            return;
        }
    }
    if (kt_update_data(c, numGrids, ptr.data(), 0, o.data(), g.data(), pixelToWorld) != 0)
        throw_error(env, c, "insituUpdateData");
}

JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_insituUpdateDataDevice(
        JNIEnv* env, jobject /*self*/, jint numGrids, jlongArray devicePointers, jintArray origins, jintArray gridDims,
        jfloat pixelToWorld) {
    insitu_ctx* c = g_ctx;
    std::vector<jint> o, g;
    if (!c || !devicePointers || env->GetArrayLength(devicePointers) < numGrids ||
        !grid_arrays(env, numGrids, origins, gridDims, o, g)) {
        throw_error(env, c, "insituUpdateDataDevice: no context or inconsistent grid arrays");
        return;
    }
    std::vector<jlong> dp((size_t)numGrids);
    env->GetLongArrayRegion(devicePointers, 0, numGrids, dp.data());
    std::vector<const void*> ptr((size_t)numGrids);
    for (jint i = 0; i < numGrids; ++i) ptr[(size_t)i] = reinterpret_cast<const void*>(dp[(size_t)i]);
    if (kt_update_data(c, numGrids, ptr.data(), 1, o.data(), g.data(), pixelToWorld) != 0)
        throw_error(env, c, "insituUpdateDataDevice");
}

JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_insituFrame(
        JNIEnv* env, jobject self, jfloatArray view, jfloatArray projection, jfloatArray invView,
        jfloatArray invProjection, jfloat nw, jfloat fwnw) {
    insitu_ctx* c = g_ctx;
    float v[16], p[16], iv[16], ip[16];
    bool inverses = false;
    if (!c || !frame_matrices(env, view, projection, invView, invProjection, v, p, iv, ip, inverses)) {
        throw_error(env, c, "insituFrame: no context or a camera matrix that is not 16 floats");
        return;
    }
    NativeBuffers& nb = buffers_of(c);
    const size_t bytes = insitu_buffer_bytes(c, INSITU_BUF_IMAGE);   // root: W*H*4, other ranks 0
    nb.image.resize(bytes);
    if (kt_frame(c, v, p, inverses ? iv : nullptr, inverses ? ip : nullptr, nw, fwnw, bytes ? nb.image.data() : nullptr,
                 bytes) != 0) {
        throw_error(env, c, "insituFrame");
        return;
    }
    if (bytes) {   // streamImage(image), DistributedVolumeRenderer.kt:726
        jobject img = env->NewDirectByteBuffer(nb.image.data(), (jlong)bytes);
        jclass k = env->GetObjectClass(self);
        jmethodID m = env->GetMethodID(k, "streamImage", "(Ljava/nio/ByteBuffer;)V");
        if (m) env->CallVoidMethod(self, m, img);
    }
}

// private external fun insituFramePipelined(view, projection, invView, invProjection, nw, fwnw): Long -- the
// frame loop one frame stale (DistributedVolumeRenderer.kt:530-542): starts this camera's render, completes the
// previous frame and hands its image to streamImage on the root; returns the completed frame's index (-1 first)
JNIEXPORT jlong JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_insituFramePipelined(
        JNIEnv* env, jobject self, jfloatArray view, jfloatArray projection, jfloatArray invView,
        jfloatArray invProjection, jfloat nw, jfloat fwnw) {
    insitu_ctx* c = g_ctx;
    float v[16], p[16], iv[16], ip[16];
    bool inverses = false;
    if (!c || !frame_matrices(env, view, projection, invView, invProjection, v, p, iv, ip, inverses)) {
        throw_error(env, c, "insituFramePipelined: no context or a camera matrix that is not 16 floats");
        return -1;
    }
    NativeBuffers& nb = buffers_of(c);
    const size_t bytes = insitu_buffer_bytes(c, INSITU_BUF_IMAGE);   // root: W*H*4, other ranks 0
    nb.image.resize(bytes);
    long long done = -1;
    if (kt_frame_pipelined(c, v, p, inverses ? iv : nullptr, inverses ? ip : nullptr, nw, fwnw,
                           bytes ? nb.image.data() : nullptr, bytes, &done) != 0) {
        throw_error(env, c, "insituFramePipelined");
        return -1;
    }
    if (bytes && done >= 0) {   // streamImage(image) of the completed frame, DistributedVolumeRenderer.kt:726
        jobject img = env->NewDirectByteBuffer(nb.image.data(), (jlong)bytes);
        jclass k = env->GetObjectClass(self);
        jmethodID m = env->GetMethodID(k, "streamImage", "(Ljava/nio/ByteBuffer;)V");
        if (m) env->CallVoidMethod(self, m, img);
    }
    return (jlong)done;
}

// private external fun insituFrameFlush(): Long -- completes the pipelined frame in flight (streamImage on the root)
JNIEXPORT jlong JNICALL Java_graphics_scenery_insitu_DistributedVolumeRenderer_insituFrameFlush(JNIEnv* env, jobject self) {
    insitu_ctx* c = g_ctx;
    if (!c) {
        throw_error(env, c, "insituFrameFlush: no context");
        return -1;
    }
    NativeBuffers& nb = buffers_of(c);
    const size_t bytes = insitu_buffer_bytes(c, INSITU_BUF_IMAGE);
    nb.image.resize(bytes);
    long long done = -1;
    if (kt_frame_flush(c, bytes ? nb.image.data() : nullptr, bytes, &done) != 0) {
        throw_error(env, c, "insituFrameFlush");
        return -1;
    }
    if (bytes && done >= 0) {
        jobject img = env->NewDirectByteBuffer(nb.image.data(), (jlong)bytes);
        jclass k = env->GetObjectClass(self);
        jmethodID m = env->GetMethodID(k, "streamImage", "(Ljava/nio/ByteBuffer;)V");
        if (m) env->CallVoidMethod(self, m, img);
    }
    return (jlong)done;
}

JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumes_insituUpdateVolume(
        JNIEnv* env, jobject /*self*/, jint volumeID, jobject buffer, jintArray dimensions, jfloatArray pos,
        jboolean is16bit, jfloat pixelToWorld, jlong mpiPointer) {
    insitu_ctx* c = context_of(mpiPointer);
    const void* data = direct(env, buffer);
    if (!c || !data || !dimensions || !pos || env->GetArrayLength(dimensions) != 3 || env->GetArrayLength(pos) != 3) {
        throw_error(env, c, "insituUpdateVolume: no context, a non-direct ByteBuffer or bad dimensions/pos");
        return;
    }
    jint d[3];
    float p[3];
    env->GetIntArrayRegion(dimensions, 0, 3, d);
    env->GetFloatArrayRegion(pos, 0, 3, p);
    const int dims[3] = {d[0], d[1], d[2]};
    const long long need = (long long)dims[0] * dims[1] * dims[2] * (is16bit ? 2 : 1);
    if (env->GetDirectBufferCapacity(buffer) < need) {
        throw_error(env, c, "insituUpdateVolume: buffer smaller than the volume");
        return;
    }
    if (kt_update_volume(c, volumeID, data, 0, dims, is16bit ? 1 : 0, p, pixelToWorld) != 0)
        throw_error(env, c, "insituUpdateVolume");
}

JNIEXPORT void JNICALL Java_graphics_scenery_insitu_DistributedVolumes_insituFrame(
        JNIEnv* env, jobject /*self*/, jfloatArray view, jfloatArray projection, jfloatArray invView,
        jfloatArray invProjection, jfloat nw, jlong colPointer, jlong depthPointer, jlong mpiPointer) {
    insitu_ctx* c = context_of(mpiPointer);
    float v[16], p[16], iv[16], ip[16];
    bool inverses = false;
    if (!c || !frame_matrices(env, view, projection, invView, invProjection, v, p, iv, ip, inverses)) {
        throw_error(env, c, "insituFrame: no context or a camera matrix that is not 16 floats");
        return;
    }
    if (kt_frame(c, v, p, inverses ? iv : nullptr, inverses ? ip : nullptr, nw, 0.0f, nullptr, 0) != 0) {
        throw_error(env, c, "insituFrame");
        return;
    }
    // the root's gathered composited VDI (S_out,H,W) rgba32f / (2S_out,H,W) r32f, where
    // gatherCompositedVDIs leaves it (gatherColorPointer / gatherDepthPointer)
    const size_t cb = insitu_buffer_bytes(c, INSITU_BUF_GATHERED_COLOR);
    if (cb && colPointer && insitu_read(c, INSITU_BUF_GATHERED_COLOR, 0, reinterpret_cast<void*>(colPointer), cb) != 0) {
        throw_error(env, c, "insituFrame: gathered colour");
        return;
    }
    const size_t db = insitu_buffer_bytes(c, INSITU_BUF_GATHERED_DEPTH);
    if (db && depthPointer && insitu_read(c, INSITU_BUF_GATHERED_DEPTH, 0, reinterpret_cast<void*>(depthPointer), db) != 0)
        throw_error(env, c, "insituFrame: gathered depth");
}

}  // extern "C"
