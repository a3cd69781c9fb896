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
#include <jni.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "insitu_hip.h"
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

}  // extern "C"
