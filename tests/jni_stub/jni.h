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
class _jobject {};
class _jclass : public _jobject {};
typedef _jobject* jobject;
typedef _jclass* jclass;
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
};
#endif
