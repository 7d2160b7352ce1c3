/*
 * Test-only stand-in for <jni.h> (this image has no JDK).  Declares exactly the
 * JNIEnv functions jleveldb_amd/jni/jlcrc_jni.c calls, with the JNI
 * specification's signatures, so tests/cpp/jni_harness.c can drive the adapter
 * through a fake JVM (tests/test_jni.py).  The real build uses the JDK's jni.h
 * (jleveldb_amd/jni/Makefile); nothing here is part of the product.
 */
#ifndef JLCRC_TEST_JNI_H
#define JLCRC_TEST_JNI_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jobjectArray;

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jint (*ThrowNew)(JNIEnv *env, jclass cls, const char *msg);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    void *(*GetPrimitiveArrayCritical)(JNIEnv *env, jarray array, jboolean *is_copy);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv *env, jarray array, void *carray, jint mode);
    jstring (*NewStringUTF)(JNIEnv *env, const char *utf);
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
    void (*GetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, jlong *buf);
    void (*GetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, jint *buf);
    void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
    void (*SetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, const jlong *buf);
    void (*SetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, const jint *buf);
    jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
    void (*DeleteLocalRef)(JNIEnv *env, jobject obj);
};
#endif
