/* jni.h stand-in for a SYNTAX-ONLY compile check of scenery-insitu_amd/jni/insitu_jni.cpp in an image
 * without a JDK (tests/test_jni_syntax.py runs g++ -fsyntax-only).  It declares just the JNI subset the
 * adaptor uses, with the JDK's names and signatures; nothing here is defined, linked or executed --
 * the real adaptor is built against a JDK's jni.h by `make -C scenery-insitu_amd jni`. */
#ifndef INSITU_JNI_STUB_H
#define INSITU_JNI_STUB_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef float jfloat;
typedef jint jsize;
class _jobject {};
class _jclass : public _jobject {};
class _jarray : public _jobject {};
class _jobjectArray : public _jarray {};
class _jintArray : public _jarray {};
class _jlongArray : public _jarray {};
class _jfloatArray : public _jarray {};
typedef _jobject* jobject;
typedef _jclass* jclass;
typedef _jarray* jarray;
typedef _jobjectArray* jobjectArray;
typedef _jintArray* jintArray;
typedef _jlongArray* jlongArray;
typedef _jfloatArray* jfloatArray;
struct _jmethodID;
typedef _jmethodID* jmethodID;
struct JNIEnv {
    jclass FindClass(const char* name);
    jclass GetObjectClass(jobject obj);
    jmethodID GetMethodID(jclass clazz, const char* name, const char* sig);
    void CallVoidMethod(jobject obj, jmethodID methodID, ...);
    jint ThrowNew(jclass clazz, const char* msg);
    jboolean ExceptionCheck();
    jobject NewDirectByteBuffer(void* address, jlong capacity);
    void* GetDirectBufferAddress(jobject buf);
    jlong GetDirectBufferCapacity(jobject buf);
    jsize GetArrayLength(jarray array);
    jobject GetObjectArrayElement(jobjectArray array, jsize index);
    void GetIntArrayRegion(jintArray array, jsize start, jsize len, jint* buf);
    void GetLongArrayRegion(jlongArray array, jsize start, jsize len, jlong* buf);
    void GetFloatArrayRegion(jfloatArray array, jsize start, jsize len, jfloat* buf);
    void DeleteLocalRef(jobject localRef);
};
#endif
