/*
 * jlcrc_jni.c — JNI adapter from the reference's Java checksum surface to the
 * C-ABI (include/jlcrc.h).  Built only where a JDK provides jni.h
 * (`make -C jleveldb_amd/jni JAVA_HOME=...`); this image has no JDK.
 *
 * Java side: jleveldb_amd/jni/java/com/tchaicatkovsky/jleveldb/util/Crc32CNative.java
 * (static natives) used by the patched Crc32C statics and by the batching shim
 * at the four call sites, see INTEGRATION.md.
 *
 * The scalar statics (host work of a few microseconds) pin their heap array with
 * GetPrimitiveArrayCritical for the call only; the batch entry points that do
 * device work copy heap arrays in and out instead, so no JVM array stays pinned
 * across a kernel.  Direct ByteBuffers (mmap'd .ldb / .log regions) are passed
 * zero-copy via GetDirectBufferAddress (the C-ABI never retains pointers).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/jlcrc.h"

#define JFN(name) Java_com_tchaicatkovsky_jleveldb_util_Crc32CNative_##name

static void throw_(JNIEnv *env, const char *cls, const char *msg) {
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg);
}

static int range_ok(JNIEnv *env, jbyteArray a, jint off, jint n) {
    jsize len = (*env)->GetArrayLength(env, a);
    if (off < 0 || n < 0 || off > len - n) {
        throw_(env, "java/lang/ArrayIndexOutOfBoundsException", "Crc32C range");
        return 0;
    }
    return 1;
}

/* static long value(byte[] data, int offset, int n) — Crc32C.java:85-89 */
JNIEXPORT jlong JNICALL JFN(value)(JNIEnv *env, jclass cls, jbyteArray data, jint off, jint n) {
    (void)cls;
    if (!range_ok(env, data, off, n)) return 0;
    uint8_t *p = (*env)->GetPrimitiveArrayCritical(env, data, NULL);
    uint32_t v = jl_crc32c_value(p + off, (size_t)n);
    (*env)->ReleasePrimitiveArrayCritical(env, data, p, JNI_ABORT);
    return (jlong)v;
}

/* static long extend(long initCrc, byte[] data, int offset, int n) — Crc32C.java:43-48 */
JNIEXPORT jlong JNICALL JFN(extend)(JNIEnv *env, jclass cls, jlong init, jbyteArray data, jint off, jint n) {
    (void)cls;
    if (!range_ok(env, data, off, n)) return 0;
    uint8_t *p = (*env)->GetPrimitiveArrayCritical(env, data, NULL);
    uint32_t v = jl_crc32c_extend((uint32_t)init, p + off, (size_t)n);
    (*env)->ReleasePrimitiveArrayCritical(env, data, p, JNI_ABORT);
    return (jlong)v;
}

/* instance update(byte[],int,int) on the bit-flipped state — Crc32C.java:119-162 */
JNIEXPORT jint JNICALL JFN(update)(JNIEnv *env, jclass cls, jint state, jbyteArray data, jint off, jint n) {
    (void)cls;
    if (!range_ok(env, data, off, n)) return state;
    uint8_t *p = (*env)->GetPrimitiveArrayCritical(env, data, NULL);
    uint32_t v = jl_crc32c_update((uint32_t)state, p + off, (size_t)n);
    (*env)->ReleasePrimitiveArrayCritical(env, data, p, JNI_ABORT);
    return (jint)v;
}

JNIEXPORT jint JNICALL JFN(init)(JNIEnv *env, jclass cls, jint device) {
    (void)env; (void)cls;
    return jl_init(device);
}

/* jl_set_option: the call-size dispatch thresholds (JL_OPT_HOST_THRESHOLD,
 * JL_OPT_LOG_HOST_THRESHOLD) and the other engine options */
JNIEXPORT jint JNICALL JFN(setOption)(JNIEnv *env, jclass cls, jint option, jlong value) {
    (void)env; (void)cls;
    return jl_set_option(option, (int64_t)value);
}

JNIEXPORT jlong JNICALL JFN(getOption)(JNIEnv *env, jclass cls, jint option) {
    (void)env; (void)cls;
    return (jlong)jl_get_option(option);
}

JNIEXPORT jstring JNICALL JFN(lastError)(JNIEnv *env, jclass cls) {
    (void)cls;
    return (*env)->NewStringUTF(env, jl_last_error());
}

/* Batched TableFormat.readBlock checksum test over an mmap'd table (direct
 * ByteBuffer): status[i] = 1 ok / 0 "block checksum mismatch".  The handle
 * arrays are copied out (Get*ArrayRegion) and the statuses copied back: no JVM
 * array stays pinned (GetPrimitiveArrayCritical would stall the collector)
 * across the device work. */
JNIEXPORT jint JNICALL JFN(tableVerify)(JNIEnv *env, jclass cls, jobject file, jlongArray off, jintArray size,
                                         jbyteArray status) {
    (void)cls;
    uint8_t *f = (*env)->GetDirectBufferAddress(env, file);
    jlong cap = (*env)->GetDirectBufferCapacity(env, file);
    jsize n = (*env)->GetArrayLength(env, off);
    if (!f || cap < 0 || (*env)->GetArrayLength(env, size) != n || (*env)->GetArrayLength(env, status) != n) {
        throw_(env, "java/lang/IllegalArgumentException", "tableVerify arguments");
        return JL_ERR_INVALID;
    }
    uint64_t *o = malloc((size_t)n * 8 + 1);
    uint32_t *s = malloc((size_t)n * 4 + 1);
    uint8_t *st = malloc((size_t)n + 1);
    int r = JL_ERR_NOMEM;
    if (o && s && st) {
        (*env)->GetLongArrayRegion(env, off, 0, n, (jlong *)o);
        (*env)->GetIntArrayRegion(env, size, 0, n, (jint *)s);
        r = jl_table_verify(f, (uint64_t)cap, o, s, (uint64_t)n, st);
        if (r == JL_OK) (*env)->SetByteArrayRegion(env, status, 0, n, (const jbyte *)st);
    }
    free(st);
    free(s);
    free(o);
    return r;
}

/* Several tables at once (a compaction's inputs, jl_tables_verify): files[t]
 * are direct ByteBuffers (mmap'd .ldb), table t's handles are off/size[first[t]
 * .. first[t+1]) (first has files.length + 1 entries).  status[i] = 1 ok / 0
 * "block checksum mismatch".  Arrays copied in and out as in tableVerify; each
 * element's local reference is released as soon as its address is taken. */
JNIEXPORT jint JNICALL JFN(tablesVerify)(JNIEnv *env, jclass cls, jobjectArray files, jlongArray first,
                                          jlongArray off, jintArray size, jbyteArray status) {
    (void)cls;
    jsize nt = (*env)->GetArrayLength(env, files), n = (*env)->GetArrayLength(env, off);
    if ((*env)->GetArrayLength(env, first) != nt + 1 || (*env)->GetArrayLength(env, size) != n ||
        (*env)->GetArrayLength(env, status) != n) {
        throw_(env, "java/lang/IllegalArgumentException", "tablesVerify arguments");
        return JL_ERR_INVALID;
    }
    const uint8_t **fp = malloc((size_t)nt * sizeof(*fp) + 1);
    uint64_t *fb = malloc((size_t)nt * 8 + 1), *fi = malloc(((size_t)nt + 1) * 8);
    uint64_t *o = malloc((size_t)n * 8 + 1);
    uint32_t *s = malloc((size_t)n * 4 + 1);
    uint8_t *st = malloc((size_t)n + 1);
    int r = JL_ERR_NOMEM;
    if (fp && fb && fi && o && s && st) {
        r = JL_OK;
        for (jsize t = 0; t < nt && r == JL_OK; t++) {
            jobject b = (*env)->GetObjectArrayElement(env, files, t);
            fp[t] = b ? (*env)->GetDirectBufferAddress(env, b) : NULL;
            jlong cap = b ? (*env)->GetDirectBufferCapacity(env, b) : -1;
            if (b) (*env)->DeleteLocalRef(env, b);
            if (!fp[t] || cap < 0) {
                throw_(env, "java/lang/IllegalArgumentException", "tablesVerify: not a direct buffer");
                r = JL_ERR_INVALID;
            }
            fb[t] = (uint64_t)cap;
        }
        if (r == JL_OK) {
            (*env)->GetLongArrayRegion(env, first, 0, nt + 1, (jlong *)fi);
            (*env)->GetLongArrayRegion(env, off, 0, n, (jlong *)o);
            (*env)->GetIntArrayRegion(env, size, 0, n, (jint *)s);
            if (fi[nt] != (uint64_t)n) {
                throw_(env, "java/lang/IllegalArgumentException", "tablesVerify: first[n] != handles");
                r = JL_ERR_INVALID;
            } else {
                r = jl_tables_verify((uint64_t)nt, fp, fb, fi, o, s, st);
                if (r == JL_OK) (*env)->SetByteArrayRegion(env, status, 0, n, (const jbyte *)st);
            }
        }
    }
    free(st);
    free(s);
    free(o);
    free(fi);
    free(fb);
    free((void *)fp);
    return r;
}

/* Block handles of a whole .ldb image (direct ByteBuffer): data blocks in
 * index order, meta blocks, metaindex, index (jl_table_block_handles).  Returns
 * the handle count — larger than the arrays when they are too short (grow and
 * call again) — or a negative error (JL_ERR_CORRUPT: message in lastError()). */
JNIEXPORT jlong JNICALL JFN(tableBlockHandles)(JNIEnv *env, jclass cls, jobject file, jlongArray off,
                                               jintArray size, jbyteArray kind) {
    (void)cls;
    uint8_t *f = (*env)->GetDirectBufferAddress(env, file);
    jlong cap = (*env)->GetDirectBufferCapacity(env, file);
    jsize n = (*env)->GetArrayLength(env, off);
    if (!f || cap < 0 || (*env)->GetArrayLength(env, size) != n || (*env)->GetArrayLength(env, kind) != n) {
        throw_(env, "java/lang/IllegalArgumentException", "tableBlockHandles arguments");
        return JL_ERR_INVALID;
    }
    uint64_t got = 0;
    uint64_t *o = malloc((size_t)n * 8 + 1);
    uint32_t *s = malloc((size_t)n * 4 + 1);
    uint8_t *k = malloc((size_t)n + 1);
    int r = JL_ERR_NOMEM;
    if (o && s && k) {
        r = jl_table_block_handles(f, (uint64_t)cap, o, s, k, (uint64_t)n, &got);
        if (r == JL_OK) {
            (*env)->SetLongArrayRegion(env, off, 0, (jsize)got, (const jlong *)o);
            (*env)->SetIntArrayRegion(env, size, 0, (jsize)got, (const jint *)s);
            (*env)->SetByteArrayRegion(env, kind, 0, (jsize)got, (const jbyte *)k);
        }
    }
    free(k);
    free(s);
    free(o);
    return (r == JL_OK || r == JL_ERR_CAPACITY) ? (jlong)got : (jlong)r;
}

/* Batched LogReader verification of a whole .log / MANIFEST image (direct
 * ByteBuffer): fills events as 16-byte jl_log_event records into `events`
 * (a direct ByteBuffer); returns the event count — larger than the buffer holds
 * when it is too small (nothing usable was written: grow it to the count and
 * call again, as for tableBlockHandles) — or a negative error. */
JNIEXPORT jlong JNICALL JFN(logVerify)(JNIEnv *env, jclass cls, jobject log, jboolean checksum, jobject events) {
    (void)cls;
    uint8_t *l = (*env)->GetDirectBufferAddress(env, log);
    jlong bytes = (*env)->GetDirectBufferCapacity(env, log);
    jl_log_event *ev = (*env)->GetDirectBufferAddress(env, events);
    jlong evcap = (*env)->GetDirectBufferCapacity(env, events) / (jlong)sizeof(jl_log_event);
    if (!l || !ev || bytes < 0 || evcap < 0) {
        throw_(env, "java/lang/IllegalArgumentException", "logVerify arguments");
        return JL_ERR_INVALID;
    }
    uint64_t n = 0;
    int r = jl_log_verify(l, (uint64_t)bytes, checksum ? 1 : 0, ev, (uint64_t)evcap, &n);
    return (r == JL_OK || r == JL_ERR_CAPACITY) ? (jlong)n : (jlong)r;
}
