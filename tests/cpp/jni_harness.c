/*
 * jni_harness.c — drives the JNI adapter (jleveldb_amd/jni/jlcrc_jni.c) through
 * a fake JVM: a JNIEnv function table over test-owned "Java" arrays and direct
 * buffers (tests/cpp/jni_stub/jni.h).  Test infrastructure only (no JDK here).
 *
 * The fake JVM enforces the JNI rules the adapter must keep: no JNI call while
 * an exception is pending or inside a GetPrimitiveArrayCritical region (other
 * than its release), region copies inside the array's bounds and of the
 * array's element type, every critical region released, with JNI_ABORT on the
 * read-only scalar paths.
 *
 *   jni_harness cpu <sstable.bin>           scalar statics, range errors, block-handle
 *                                           walk with its grow-and-retry protocol,
 *                                           argument checks, device entry points
 *                                           failing cleanly without a GPU
 *   jni_harness gpu <sstable.bin> <log>     tableVerify / logVerify on the device
 *                                           equal the C-ABI calls (and flips are seen)
 * Prints "OK <checks>" and exits 0, or reports the first failures and exits 1.
 * Reference surface: Crc32C.java:43-48,85-93,119-162 (J/util); call sites
 * TableBuilder.java:313-317, TableFormat.java:211-212, LogWriter.java:147-148,
 * LogReader.java:357-358.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/jlcrc.h"

#define JFN(name) Java_com_tchaicatkovsky_jleveldb_util_Crc32CNative_##name
jlong JFN(value)(JNIEnv *, jclass, jbyteArray, jint, jint);
jlong JFN(extend)(JNIEnv *, jclass, jlong, jbyteArray, jint, jint);
jint JFN(update)(JNIEnv *, jclass, jint, jbyteArray, jint, jint);
jint JFN(init)(JNIEnv *, jclass, jint);
jint JFN(setOption)(JNIEnv *, jclass, jint, jlong);
jlong JFN(getOption)(JNIEnv *, jclass, jint);
jstring JFN(lastError)(JNIEnv *, jclass);
jint JFN(tableVerify)(JNIEnv *, jclass, jobject, jlongArray, jintArray, jbyteArray);
jlong JFN(tableBlockHandles)(JNIEnv *, jclass, jobject, jlongArray, jintArray, jbyteArray);
jlong JFN(logVerify)(JNIEnv *, jclass, jobject, jboolean, jobject);
jint JFN(tablesVerify)(JNIEnv *, jclass, jobjectArray, jlongArray, jlongArray, jintArray, jbyteArray);

/* ------------------------------------------------------------- fake JVM */
enum { K_BYTE = 1, K_INT, K_LONG, K_DIRECT, K_HEAPBUF, K_CLASS, K_STRING, K_OBJARRAY };
struct _jobject {
    int kind;
    jsize len;   /* elements (arrays) */
    void *data;  /* elements, or the direct buffer's memory */
    jlong cap;   /* direct buffer capacity */
    char text[256];
};

static int g_fail, g_checks;
static char g_exc[256];  /* pending exception class ("" = none) */
static int g_critical;   /* open critical regions */
static int g_abort_release;
static int g_local_refs;  /* element references handed out and not yet deleted */

#define CHECK(cond, ...)                                                        \
    do {                                                                        \
        g_checks++;                                                             \
        if (!(cond)) {                                                          \
            g_fail++;                                                           \
            fprintf(stderr, "%s:%d: ", __FILE__, __LINE__);                     \
            fprintf(stderr, __VA_ARGS__);                                       \
            fputc('\n', stderr);                                                \
        }                                                                       \
    } while (0)

static void jni_rule(const char *fn, int allowed_in_critical) {
    CHECK(g_exc[0] == 0, "JNI %s called with exception %s pending", fn, g_exc);
    CHECK(allowed_in_critical || g_critical == 0, "JNI %s called inside a critical region", fn);
}

static struct _jobject g_classes[8];
static int g_nclasses;
static jclass f_FindClass(JNIEnv *env, const char *name) {
    (void)env;
    jni_rule("FindClass", 0);
    jclass c = &g_classes[g_nclasses++ % 8];
    c->kind = K_CLASS;
    snprintf(c->text, sizeof c->text, "%s", name);
    return c;
}
static jint f_ThrowNew(JNIEnv *env, jclass cls, const char *msg) {
    (void)env;
    (void)msg;
    jni_rule("ThrowNew", 0);
    CHECK(cls && cls->kind == K_CLASS, "ThrowNew without a class");
    snprintf(g_exc, sizeof g_exc, "%s", cls->text);
    return 0;
}
static jsize f_GetArrayLength(JNIEnv *env, jarray a) {
    (void)env;
    jni_rule("GetArrayLength", 0);
    CHECK(a && (a->kind == K_BYTE || a->kind == K_INT || a->kind == K_LONG || a->kind == K_OBJARRAY),
          "GetArrayLength of a non-array");
    return a ? a->len : 0;
}
static void *f_GetCritical(JNIEnv *env, jarray a, jboolean *is_copy) {
    (void)env;
    jni_rule("GetPrimitiveArrayCritical", 1);
    if (is_copy) *is_copy = JNI_FALSE;
    g_critical++;
    return a->data;
}
static void f_ReleaseCritical(JNIEnv *env, jarray a, void *p, jint mode) {
    (void)env;
    CHECK(g_critical > 0 && p == a->data, "ReleasePrimitiveArrayCritical without its Get");
    if (mode == JNI_ABORT) g_abort_release++;
    g_critical--;
}
static struct _jobject g_strings[4];
static int g_nstrings;
static jstring f_NewStringUTF(JNIEnv *env, const char *s) {
    (void)env;
    jni_rule("NewStringUTF", 0);
    jstring o = &g_strings[g_nstrings++ % 4];
    o->kind = K_STRING;
    snprintf(o->text, sizeof o->text, "%s", s ? s : "");
    return o;
}
static void *f_GetDirectBufferAddress(JNIEnv *env, jobject b) {
    (void)env;
    jni_rule("GetDirectBufferAddress", 0);
    return (b && b->kind == K_DIRECT) ? b->data : NULL;  /* heap buffers: NULL, as the JVM */
}
static jlong f_GetDirectBufferCapacity(JNIEnv *env, jobject b) {
    (void)env;
    jni_rule("GetDirectBufferCapacity", 0);
    return (b && b->kind == K_DIRECT) ? b->cap : -1;
}
static int region_ok(const char *fn, jarray a, int kind, jsize start, jsize len) {
    jni_rule(fn, 0);
    CHECK(a && a->kind == kind, "%s on an array of another element type", fn);
    if (!a || a->kind != kind) return 0;
    if (start < 0 || len < 0 || start > a->len - len) {
        snprintf(g_exc, sizeof g_exc, "java/lang/ArrayIndexOutOfBoundsException");
        CHECK(0, "%s out of bounds: start %d len %d of %d", fn, start, len, a->len);
        return 0;
    }
    return 1;
}
static void f_GetLongRegion(JNIEnv *env, jlongArray a, jsize s, jsize n, jlong *buf) {
    (void)env;
    if (region_ok("GetLongArrayRegion", a, K_LONG, s, n)) memcpy(buf, (jlong *)a->data + s, (size_t)n * 8);
}
static void f_GetIntRegion(JNIEnv *env, jintArray a, jsize s, jsize n, jint *buf) {
    (void)env;
    if (region_ok("GetIntArrayRegion", a, K_INT, s, n)) memcpy(buf, (jint *)a->data + s, (size_t)n * 4);
}
static void f_SetByteRegion(JNIEnv *env, jbyteArray a, jsize s, jsize n, const jbyte *buf) {
    (void)env;
    if (region_ok("SetByteArrayRegion", a, K_BYTE, s, n)) memcpy((jbyte *)a->data + s, buf, (size_t)n);
}
static void f_SetLongRegion(JNIEnv *env, jlongArray a, jsize s, jsize n, const jlong *buf) {
    (void)env;
    if (region_ok("SetLongArrayRegion", a, K_LONG, s, n)) memcpy((jlong *)a->data + s, buf, (size_t)n * 8);
}
static void f_SetIntRegion(JNIEnv *env, jintArray a, jsize s, jsize n, const jint *buf) {
    (void)env;
    if (region_ok("SetIntArrayRegion", a, K_INT, s, n)) memcpy((jint *)a->data + s, buf, (size_t)n * 4);
}

static jobject f_GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
    (void)env;
    jni_rule("GetObjectArrayElement", 0);
    CHECK(a && a->kind == K_OBJARRAY && i >= 0 && i < a->len, "GetObjectArrayElement out of bounds");
    g_local_refs++;
    return ((jobject *)a->data)[i];
}
static void f_DeleteLocalRef(JNIEnv *env, jobject o) {
    (void)env;
    (void)o;
    g_local_refs--;
}

static const struct JNINativeInterface_ g_fns = {
    f_FindClass,      f_ThrowNew,        f_GetArrayLength,          f_GetCritical,   f_ReleaseCritical,
    f_NewStringUTF,   f_GetDirectBufferAddress, f_GetDirectBufferCapacity, f_GetLongRegion, f_GetIntRegion,
    f_SetByteRegion,  f_SetLongRegion,   f_SetIntRegion,            f_GetObjectArrayElement, f_DeleteLocalRef,
};
static JNIEnv g_env_v = &g_fns;
static JNIEnv *const env = &g_env_v;

static struct _jobject *array(int kind, jsize n) {
    struct _jobject *o = calloc(1, sizeof *o);
    size_t el = kind == K_BYTE ? 1 : kind == K_INT ? 4 : 8;
    o->kind = kind;
    o->len = n;
    o->data = calloc((size_t)(n ? n : 1), el);
    return o;
}
static struct _jobject *direct(void *p, jlong cap) {
    struct _jobject *o = calloc(1, sizeof *o);
    o->kind = K_DIRECT;
    o->data = p;
    o->cap = cap;
    return o;
}
static void release(struct _jobject *o) {
    if (!o) return;
    if (o->kind != K_DIRECT) free(o->data);
    free(o);
}
/* takes the pending exception (the Java caller would see it thrown) */
static int took(const char *cls) {
    int ok = strcmp(g_exc, cls) == 0;
    g_exc[0] = 0;
    return ok;
}

static uint8_t *read_file(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc((size_t)sz + 1);
    *n = fread(b, 1, (size_t)sz, f);
    fclose(f);
    return b;
}

/* --------------------------------------------------------------- checks */
static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return g_rng;
}

/* value / extend / update over random ranges equal the C-ABI scalars; bad
 * ranges throw ArrayIndexOutOfBoundsException and touch nothing */
static void scalars(void) {
    struct _jobject *a = array(K_BYTE, 5000);
    for (int i = 0; i < a->len; i++) ((uint8_t *)a->data)[i] = (uint8_t)rnd();
    const uint8_t *d = a->data;
    for (int t = 0; t < 2000; t++) {
        jint off = (jint)(rnd() % 5001), n = (jint)(rnd() % (uint64_t)(5001 - off));
        uint32_t init = (uint32_t)rnd();
        CHECK((uint32_t)JFN(value)(env, NULL, a, off, n) == jl_crc32c_value(d + off, (size_t)n), "value %d %d", off, n);
        CHECK((uint32_t)JFN(extend)(env, NULL, (jlong)init, a, off, n) == jl_crc32c_extend(init, d + off, (size_t)n),
              "extend %d %d", off, n);
        CHECK((uint32_t)JFN(update)(env, NULL, (jint)init, a, off, n) == jl_crc32c_update(init, d + off, (size_t)n),
              "update %d %d", off, n);
        CHECK(g_exc[0] == 0 && g_critical == 0, "scalar left state behind");
    }
    /* Crc32C.java:29 / TestCrc32C.java:63: value(32 x 0) = 0x8a9136aa */
    struct _jobject *z = array(K_BYTE, 32);
    CHECK((uint32_t)JFN(value)(env, NULL, z, 0, 32) == 0x8a9136aau, "value(32 x 0)");
    const jint bad[][2] = {{-1, 1}, {0, -1}, {5000, 1}, {4990, 11}, {0x7fffffff, 1}, {1, 0x7fffffff}, {-5, -5}};
    for (size_t i = 0; i < sizeof bad / sizeof bad[0]; i++) {
        const int before = g_abort_release;
        CHECK(JFN(value)(env, NULL, a, bad[i][0], bad[i][1]) == 0 && took("java/lang/ArrayIndexOutOfBoundsException"),
              "value(%d, %d) did not throw AIOOBE", bad[i][0], bad[i][1]);
        CHECK(JFN(extend)(env, NULL, 7, a, bad[i][0], bad[i][1]) == 0 && took("java/lang/ArrayIndexOutOfBoundsException"),
              "extend(%d, %d) did not throw AIOOBE", bad[i][0], bad[i][1]);
        CHECK(JFN(update)(env, NULL, 1234, a, bad[i][0], bad[i][1]) == 1234 &&
                  took("java/lang/ArrayIndexOutOfBoundsException"),
              "update(%d, %d) did not throw AIOOBE or changed the state", bad[i][0], bad[i][1]);
        CHECK(g_abort_release == before, "a bad range still entered the critical region");
    }
    CHECK(g_abort_release >= 6000, "scalar critical regions not released with JNI_ABORT");
    release(a);
    release(z);
}

/* tableBlockHandles: every capacity from 0 up, the grow-and-retry protocol of
 * Crc32CShims.verifyTable, equal to jl_table_block_handles; bad arguments */
static void handles(const uint8_t *sst, size_t sst_n) {
    uint64_t want_n = 0;
    CHECK(jl_table_block_handles(sst, sst_n, NULL, NULL, NULL, 0, &want_n) == JL_ERR_CAPACITY && want_n > 2,
          "sstable fixture has %llu handles", (unsigned long long)want_n);
    uint64_t *wo = malloc(want_n * 8);
    uint32_t *ws = malloc(want_n * 4);
    uint8_t *wk = malloc(want_n);
    CHECK(jl_table_block_handles(sst, sst_n, wo, ws, wk, want_n, &want_n) == JL_OK, "C-ABI handles");
    uint8_t *copy = malloc(sst_n);
    memcpy(copy, sst, sst_n);
    struct _jobject *buf = direct(copy, (jlong)sst_n);
    for (jsize cap = 0; cap <= (jsize)want_n + 3; cap++) {
        struct _jobject *o = array(K_LONG, cap), *s = array(K_INT, cap), *k = array(K_BYTE, cap);
        for (jsize i = 0; i < cap; i++) ((jlong *)o->data)[i] = -7;
        jlong n = JFN(tableBlockHandles)(env, NULL, buf, o, s, k);
        CHECK(n == (jlong)want_n && g_exc[0] == 0, "cap %d: returned %lld", cap, (long long)n);
        if ((uint64_t)cap < want_n) {
            CHECK(((cap == 0) || ((jlong *)o->data)[0] == -7), "cap %d: short arrays were written", cap);
        } else {
            for (uint64_t i = 0; i < want_n; i++)
                CHECK((uint64_t)((jlong *)o->data)[i] == wo[i] && (uint32_t)((jint *)s->data)[i] == ws[i] &&
                          (uint8_t)((jbyte *)k->data)[i] == wk[i],
                      "cap %d: handle %llu differs", cap, (unsigned long long)i);
            for (jsize i = (jsize)want_n; i < cap; i++) CHECK(((jlong *)o->data)[i] == -7, "wrote past the count");
        }
        release(o);
        release(s);
        release(k);
    }
    /* the shim's grow-and-retry: 64 first, then exactly n */
    {
        struct _jobject *o = array(K_LONG, 1), *s = array(K_INT, 1), *k = array(K_BYTE, 1);
        jlong n = JFN(tableBlockHandles)(env, NULL, buf, o, s, k);
        release(o), release(s), release(k);
        o = array(K_LONG, (jsize)n), s = array(K_INT, (jsize)n), k = array(K_BYTE, (jsize)n);
        CHECK(JFN(tableBlockHandles)(env, NULL, buf, o, s, k) == n && ((jlong *)o->data)[n - 1] == (jlong)wo[n - 1],
              "grow and retry");
        release(o), release(s), release(k);
    }
    /* a corrupted footer: the reference's Status text through lastError */
    copy[sst_n - 1] ^= 0xff;
    {
        struct _jobject *o = array(K_LONG, 64), *s = array(K_INT, 64), *k = array(K_BYTE, 64);
        jlong n = JFN(tableBlockHandles)(env, NULL, buf, o, s, k);
        jstring msg = JFN(lastError)(env, NULL);
        CHECK(n == JL_ERR_CORRUPT && strstr(msg->text, "bad magic number"), "corrupt table: %lld %s", (long long)n,
              msg->text);
        release(o), release(s), release(k);
    }
    copy[sst_n - 1] ^= 0xff;
    /* mismatched array lengths and a heap (non-direct) buffer: IllegalArgumentException */
    {
        struct _jobject *o = array(K_LONG, 8), *s = array(K_INT, 7), *k = array(K_BYTE, 8);
        CHECK(JFN(tableBlockHandles)(env, NULL, buf, o, s, k) == JL_ERR_INVALID &&
                  took("java/lang/IllegalArgumentException"), "mismatched arrays");
        struct _jobject heap = {K_HEAPBUF, 0, copy, (jlong)sst_n, ""};
        release(s);
        s = array(K_INT, 8);
        CHECK(JFN(tableBlockHandles)(env, NULL, &heap, o, s, k) == JL_ERR_INVALID &&
                  took("java/lang/IllegalArgumentException"), "heap buffer");
        struct _jobject *st = array(K_BYTE, 8);
        CHECK(JFN(tableVerify)(env, NULL, &heap, o, s, st) == JL_ERR_INVALID &&
                  took("java/lang/IllegalArgumentException"), "tableVerify heap buffer");
        release(st);
        st = array(K_BYTE, 3);
        CHECK(JFN(tableVerify)(env, NULL, buf, o, s, st) == JL_ERR_INVALID &&
                  took("java/lang/IllegalArgumentException"), "tableVerify short status");
        CHECK(JFN(logVerify)(env, NULL, &heap, 1, buf) == JL_ERR_INVALID && took("java/lang/IllegalArgumentException"),
              "logVerify heap buffer");
        release(st), release(o), release(s), release(k);
    }
    release(buf);
    free(copy);
    free(wo);
    free(ws);
    free(wk);
}

/* device entry points: without a GPU they fail with JL_ERR_NO_DEVICE (no
 * exception, nothing written); with one they equal the C-ABI */
static void device_paths(const uint8_t *sst, size_t sst_n, const uint8_t *log, size_t log_n, int gpu) {
    uint64_t n = 0;
    (void)jl_table_block_handles(sst, sst_n, NULL, NULL, NULL, 0, &n);
    uint64_t *wo = malloc(n * 8);
    uint32_t *ws = malloc(n * 4);
    (void)jl_table_block_handles(sst, sst_n, wo, ws, NULL, n, &n);
    uint8_t *copy = malloc(sst_n);
    memcpy(copy, sst, sst_n);
    struct _jobject *buf = direct(copy, (jlong)sst_n);
    struct _jobject *o = array(K_LONG, (jsize)n), *s = array(K_INT, (jsize)n), *st = array(K_BYTE, (jsize)n);
    memcpy(o->data, wo, n * 8);
    memcpy(s->data, ws, n * 4);
    memset(st->data, 9, n);
    jint r = JFN(tableVerify)(env, NULL, buf, o, s, st);
    if (!gpu) {
        CHECK(r == JL_ERR_NO_DEVICE && g_exc[0] == 0 && ((uint8_t *)st->data)[0] == 9, "tableVerify without a GPU: %d", r);
    } else {
        uint8_t *want = malloc(n);
        CHECK(r == JL_OK && jl_table_verify(sst, sst_n, wo, ws, n, want) == JL_OK && memcmp(want, st->data, n) == 0,
              "tableVerify differs from jl_table_verify (%d)", r);
        for (uint64_t i = 0; i < n; i++) CHECK(want[i] == 1, "clean table block %llu fails", (unsigned long long)i);
        copy[wo[0] + ws[0] / 2] ^= 0x10;  /* a flip in the first block */
        CHECK(JFN(tableVerify)(env, NULL, buf, o, s, st) == JL_OK && ((uint8_t *)st->data)[0] == 0 &&
                  (n < 2 || ((uint8_t *)st->data)[1] == 1), "flipped block not seen");
        free(want);
    }
    release(o), release(s), release(st);
    /* tablesVerify: the same table three times (a compaction's inputs), one flip in the second copy */
    {
        uint8_t *c2 = malloc(sst_n);
        memcpy(c2, sst, sst_n);
        c2[wo[n - 1] + 1] ^= 0x04;  /* a byte of the index block */
        struct _jobject *b1 = direct((void *)sst, (jlong)sst_n), *b2 = direct(c2, (jlong)sst_n);
        struct _jobject *fa = array(K_OBJARRAY, 3);
        fa->data = realloc(fa->data, 3 * sizeof(jobject));
        ((jobject *)fa->data)[0] = b1, ((jobject *)fa->data)[1] = b2, ((jobject *)fa->data)[2] = b1;
        struct _jobject *fi = array(K_LONG, 4), *to = array(K_LONG, (jsize)(3 * n)), *tz = array(K_INT, (jsize)(3 * n)),
                        *tst = array(K_BYTE, (jsize)(3 * n));
        for (int t = 0; t < 4; t++) ((jlong *)fi->data)[t] = (jlong)(t * n);
        for (int t = 0; t < 3; t++) {
            memcpy((jlong *)to->data + t * n, wo, n * 8);
            memcpy((jint *)tz->data + t * n, ws, n * 4);
        }
        jint rr = JFN(tablesVerify)(env, NULL, fa, fi, to, tz, tst);
        CHECK(g_local_refs == 0, "tablesVerify leaked %d local references", g_local_refs);
        if (!gpu) {
            CHECK(rr == JL_ERR_NO_DEVICE && g_exc[0] == 0, "tablesVerify without a GPU: %d", rr);
        } else {
            CHECK(rr == JL_OK, "tablesVerify: %d", rr);
            for (uint64_t i = 0; i < 3 * n; i++)
                CHECK(((uint8_t *)tst->data)[i] == (i == 2 * n - 1 ? 0 : 1), "tablesVerify status %llu", (unsigned long long)i);
        }
        ((jlong *)fi->data)[3] = (jlong)(3 * n - 1);  /* first[n] must equal the handle count */
        CHECK(JFN(tablesVerify)(env, NULL, fa, fi, to, tz, tst) == JL_ERR_INVALID &&
                  took("java/lang/IllegalArgumentException") && g_local_refs == 0, "tablesVerify bad first");
        struct _jobject heap = {K_HEAPBUF, 0, c2, (jlong)sst_n, ""};
        ((jobject *)fa->data)[1] = &heap;
        ((jlong *)fi->data)[3] = (jlong)(3 * n);
        CHECK(JFN(tablesVerify)(env, NULL, fa, fi, to, tz, tst) == JL_ERR_INVALID &&
                  took("java/lang/IllegalArgumentException") && g_local_refs == 0, "tablesVerify heap buffer");
        release(fi), release(to), release(tz), release(tst), release(fa), release(b1), release(b2);
        free(c2);
    }
    release(buf);
    free(copy);
    free(wo);
    free(ws);
    if (!log) return;
    /* logVerify: events into a direct buffer, equal to jl_log_verify */
    uint64_t cap = log_n / 7 + 2;
    jl_log_event *ev = calloc(cap, sizeof *ev), *want = calloc(cap, sizeof *want);
    struct _jobject *lb = direct((void *)log, (jlong)log_n), *eb = direct(ev, (jlong)(cap * sizeof *ev));
    for (int checksum = 0; checksum < 2; checksum++) {
        jlong got = JFN(logVerify)(env, NULL, lb, (jboolean)checksum, eb);
        if (!gpu) {
            CHECK(got == JL_ERR_NO_DEVICE && g_exc[0] == 0, "logVerify without a GPU: %lld", (long long)got);
            continue;
        }
        uint64_t wn = 0;
        CHECK(jl_log_verify(log, log_n, checksum, want, cap, &wn) == JL_OK && got == (jlong)wn &&
                  memcmp(ev, want, wn * sizeof *ev) == 0, "logVerify differs from jl_log_verify (checksum %d)", checksum);
        if (checksum && wn > 1) {
            int bad = 0;
            for (uint64_t i = 0; i < wn; i++) bad += want[i].kind == JL_LOG_BAD_CRC;
            CHECK(bad >= 1, "the log's flipped record is not BAD_CRC");
        }
    }
    if (gpu) {  /* an event buffer too small: the full count comes back (grow and retry) */
        struct _jobject *small = direct(ev, 16 * 3);
        uint64_t wn = 0;
        (void)jl_log_verify(log, log_n, 1, want, cap, &wn);
        CHECK(JFN(logVerify)(env, NULL, lb, 1, small) == (jlong)wn && wn > 3 && g_exc[0] == 0, "short event buffer");
        release(small);
    }
    release(lb), release(eb);
    free(ev);
    free(want);
}

/* ------------------------------------------------------------------ dump mode
 * What the Java side of Crc32CShims sees, written to a file for
 * tests/test_jni.py to compare with the oracle (not with the C-ABI):
 *   table:  Crc32CShims.verifyTable — tableBlockHandles from 64 entries with
 *           grow-and-retry, then tableVerify over the exact handles
 *           (TableFormat.java:211-212 for every block of Table.open)
 *   tables: a compaction's inputs (VersionSet.java:820-823) — each table's
 *           handles, then one tablesVerify call over all of them
 *   log:    Crc32CShims.verifyLog — its capacity guess, logVerify, one grow to
 *           the reported count, and its decoding of the 16-B little-endian
 *           events (Crc32CShims.java:153-158), restated here byte by byte
 *           (LogReader.java:297-383 for every physical record) */
static FILE *g_out;
static void put(const void *p, size_t n) { CHECK(fwrite(p, 1, n, g_out) == n, "short write"); }

/* Crc32CShims.verifyTable's handle walk: the count, arrays of exactly that length */
static jlong shim_handles(struct _jobject *buf, struct _jobject **o, struct _jobject **s, struct _jobject **k) {
    *o = array(K_LONG, 64), *s = array(K_INT, 64), *k = array(K_BYTE, 64);
    jlong n = JFN(tableBlockHandles)(env, NULL, buf, *o, *s, *k);
    if (n > 64) {
        release(*o), release(*s), release(*k);
        *o = array(K_LONG, (jsize)n), *s = array(K_INT, (jsize)n), *k = array(K_BYTE, (jsize)n);
        n = JFN(tableBlockHandles)(env, NULL, buf, *o, *s, *k);
    }
    CHECK(n >= 0 && g_exc[0] == 0, "tableBlockHandles: %lld %s", (long long)n, JFN(lastError)(env, NULL)->text);
    if (n >= 0) (*o)->len = (*s)->len = (*k)->len = (jsize)n; /* Arrays.copyOf(.., n) */
    return n;
}

static int dump_table(const char *path) {
    size_t fn = 0;
    uint8_t *f = read_file(path, &fn);
    if (!f) return 2;
    struct _jobject *buf = direct(f, (jlong)fn), *o, *s, *k;
    const jlong n = shim_handles(buf, &o, &s, &k);
    struct _jobject *ok = array(K_BYTE, (jsize)(n > 0 ? n : 0));
    const jint rc = n >= 0 ? JFN(tableVerify)(env, NULL, buf, o, s, ok) : -1;
    CHECK(rc == JL_OK && g_exc[0] == 0, "tableVerify: %d", rc);
    const uint64_t nn = n > 0 ? (uint64_t)n : 0;
    put(&nn, 8);
    put(o->data, nn * 8), put(s->data, nn * 4), put(k->data, nn), put(ok->data, nn);
    release(o), release(s), release(k), release(ok), release(buf);
    free(f);
    return 0;
}

static int dump_tables(int nt, char **paths) {
    uint8_t **f = calloc((size_t)nt, sizeof *f);
    struct _jobject **b = calloc((size_t)nt, sizeof *b);
    struct _jobject *fa = array(K_OBJARRAY, nt), *fi = array(K_LONG, nt + 1);
    fa->data = realloc(fa->data, (size_t)nt * sizeof(jobject));
    jlong total = 0;
    struct _jobject **ho = calloc((size_t)nt, sizeof *ho), **hs = calloc((size_t)nt, sizeof *hs);
    for (int t = 0; t < nt; t++) {
        size_t fn = 0;
        if (!(f[t] = read_file(paths[t], &fn))) return 2;
        b[t] = direct(f[t], (jlong)fn);
        ((jobject *)fa->data)[t] = b[t];
        struct _jobject *k;
        ((jlong *)fi->data)[t] = total;
        const jlong n = shim_handles(b[t], &ho[t], &hs[t], &k);
        release(k);
        total += n > 0 ? n : 0;
    }
    ((jlong *)fi->data)[nt] = total;
    struct _jobject *o = array(K_LONG, (jsize)total), *s = array(K_INT, (jsize)total), *st = array(K_BYTE, (jsize)total);
    for (int t = 0; t < nt; t++) {
        const jlong a = ((jlong *)fi->data)[t], m = ((jlong *)fi->data)[t + 1] - a;
        memcpy((jlong *)o->data + a, ho[t]->data, (size_t)m * 8);
        memcpy((jint *)s->data + a, hs[t]->data, (size_t)m * 4);
        release(ho[t]), release(hs[t]);
    }
    const jint rc = JFN(tablesVerify)(env, NULL, fa, fi, o, s, st);
    CHECK(rc == JL_OK && g_exc[0] == 0 && g_local_refs == 0, "tablesVerify: %d", rc);
    const uint64_t T = (uint64_t)nt;
    put(&T, 8);
    put(fi->data, (T + 1) * 8);
    put(o->data, (size_t)total * 8), put(s->data, (size_t)total * 4), put(st->data, (size_t)total);
    for (int t = 0; t < nt; t++) release(b[t]), free(f[t]);
    release(fa), release(fi), release(o), release(s), release(st);
    free(f), free(b), free(ho), free(hs);
    return 0;
}

/* ByteBuffer.order(LITTLE_ENDIAN).getLong / getInt / get of the shim's decode */
static uint64_t le(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = n - 1; i >= 0; i--) v = v << 8 | p[i];
    return v;
}

static int dump_log(const char *path, int checksum) {
    size_t ln = 0;
    uint8_t *l = read_file(path, &ln);
    if (!l) return 2;
    struct _jobject *lb = direct(l, (jlong)ln);
    const int64_t size = (int64_t)ln, imax = 2147483647;
    int64_t cap = size / 7 + 2;
    if (cap > (imax - 15) / 16) cap = (imax - 15) / 16;
    if (cap > (size / 512 > 1024 ? size / 512 : 1024)) cap = size / 512 > 1024 ? size / 512 : 1024;
    uint8_t *eb = calloc((size_t)cap, 16);
    struct _jobject *ev = direct(eb, 16 * cap);
    jlong n = JFN(logVerify)(env, NULL, lb, (jboolean)checksum, ev);
    const int grew = n > cap;
    if (n > cap) { /* the count came back: grow once */
        release(ev);
        free(eb);
        cap = n;
        eb = calloc((size_t)cap, 16);
        ev = direct(eb, 16 * cap);
        n = JFN(logVerify)(env, NULL, lb, (jboolean)checksum, ev);
    }
    CHECK(n >= 0 && n <= cap && g_exc[0] == 0, "logVerify: %lld", (long long)n);
    const uint64_t nn = n > 0 ? (uint64_t)n : 0;
    put(&nn, 8);
    const uint64_t g = (uint64_t)grew;
    put(&g, 8);
    for (uint64_t i = 0; i < nn; i++) {
        const uint8_t *e = eb + 16 * i;
        /* new LogEvent(getLong(b), getInt(b + 8), get(b + 12) & 0xff, get(b + 13) & 0xff) */
        const uint64_t offset = le(e, 8);
        const uint32_t length = (uint32_t)le(e + 8, 4);
        const uint8_t type = e[12], kind = e[13];
        const jl_log_event back = {offset, length, type, kind, 0};
        CHECK(memcmp(&back, e, 14) == 0, "event %llu: the shim's decode does not round-trip", (unsigned long long)i);
        uint8_t rec[16] = {0};
        memcpy(rec, &offset, 8), memcpy(rec + 8, &length, 4), rec[12] = type, rec[13] = kind;
        put(rec, 16);
    }
    release(ev), release(lb);
    free(eb);
    free(l);
    return 0;
}

static int dump(int argc, char **argv) {
    /* dump[-default] <out> table <sst> | tables <sst>... | log <log> <checksum 0|1> */
    if (argc < 5) return 2;
    jint r = JFN(init)(env, NULL, 0);
    CHECK(r == JL_OK, "init returned %d", r);
    if (strcmp(argv[1], "dump") == 0) { /* every call on the device (the shim's thresholds at 0) */
        CHECK(JFN(setOption)(env, NULL, JL_OPT_HOST_THRESHOLD, 0) == JL_OK, "threshold 0");
        CHECK(JFN(setOption)(env, NULL, JL_OPT_LOG_HOST_THRESHOLD, 0) == JL_OK, "log threshold 0");
    }
    if (!(g_out = fopen(argv[2], "wb"))) return 2;
    int rc = 2;
    if (strcmp(argv[3], "table") == 0) rc = dump_table(argv[4]);
    else if (strcmp(argv[3], "tables") == 0) rc = dump_tables(argc - 4, argv + 4);
    else if (strcmp(argv[3], "log") == 0 && argc > 5) rc = dump_log(argv[4], atoi(argv[5]));
    fclose(g_out);
    CHECK(g_critical == 0 && g_exc[0] == 0, "left a critical region open or an exception pending");
    if (rc) return rc;
    if (g_fail) {
        fprintf(stderr, "FAILED %d of %d\n", g_fail, g_checks);
        return 1;
    }
    printf("OK %d\n", g_checks);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && strncmp(argv[1], "dump", 4) == 0) return dump(argc, argv);
    if (argc < 3) {
        fprintf(stderr, "usage: jni_harness cpu|gpu <sstable.bin> [log]\n"
                        "       jni_harness dump|dump-default <out> table <sst> | tables <sst>... | log <log> <0|1>\n");
        return 2;
    }
    const int gpu = strcmp(argv[1], "gpu") == 0;
    size_t sst_n = 0, log_n = 0;
    uint8_t *sst = read_file(argv[2], &sst_n), *log = argc > 3 ? read_file(argv[3], &log_n) : NULL;
    if (!sst || (argc > 3 && !log)) {
        fprintf(stderr, "cannot read inputs\n");
        return 2;
    }
    jint r = JFN(init)(env, NULL, 0);
    CHECK(gpu ? r == JL_OK : r == JL_ERR_NO_DEVICE, "init returned %d", r);
    if (!gpu) CHECK(strstr(JFN(lastError)(env, NULL)->text, "no HIP device") != NULL, "lastError after init");
    /* options through JNI (the dispatch thresholds the shim sets from system properties) */
    const jlong thr0 = JFN(getOption)(env, NULL, JL_OPT_HOST_THRESHOLD);
    CHECK(JFN(setOption)(env, NULL, JL_OPT_HOST_THRESHOLD, 12345) == JL_OK &&
              JFN(getOption)(env, NULL, JL_OPT_HOST_THRESHOLD) == 12345, "setOption / getOption");
    CHECK(JFN(setOption)(env, NULL, JL_OPT_LOG_HOST_THRESHOLD, -2) == JL_ERR_INVALID && g_exc[0] == 0, "bad option value");
    CHECK(JFN(setOption)(env, NULL, JL_OPT_LOG_HOST_THRESHOLD, JL_HOST_THRESHOLD_AUTO) == JL_OK, "auto threshold");
    CHECK(JFN(setOption)(env, NULL, JL_OPT_HOST_THRESHOLD, 0) == JL_OK, "threshold 0");
    CHECK(JFN(setOption)(env, NULL, JL_OPT_LOG_HOST_THRESHOLD, 0) == JL_OK, "log threshold 0");
    (void)thr0;
    scalars();
    handles(sst, sst_n);
    device_paths(sst, sst_n, log, log_n, gpu);
    CHECK(g_critical == 0 && g_exc[0] == 0, "left a critical region open or an exception pending");
    free(sst);
    free(log);
    if (g_fail) {
        fprintf(stderr, "FAILED %d of %d\n", g_fail, g_checks);
        return 1;
    }
    printf("OK %d\n", g_checks);
    return 0;
}
