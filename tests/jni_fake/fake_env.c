/*
 * TEST-ONLY fake JNIEnv for tests/test_jni_shim.py: backs the function-table members declared in
 * tests/jni_fake/jni.h with plain C objects (byte/int arrays, direct buffers, strings), records a
 * pending exception the way a JVM would (ThrowNew, an out-of-range GetByteArrayRegion), counts
 * critical sections, and can make the shim's malloc (compiled with -Dmalloc=bkd_test_malloc) or a
 * GetPrimitiveArrayCritical fail on demand. Linked with the shim into one test library; Python
 * calls the Java_* natives through ctypes with the env pointer returned by fake_env().
 */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_BYTES = 1, K_INTS, K_DIRECT, K_STRING, K_CLASS, K_LONGS, K_OBJECTS };

struct _jobject {
    int kind;
    void* data;
    jsize len;
};

static char g_pending[256];
static int g_critical_depth, g_critical_total, g_critical_fail, g_malloc_fail, g_malloc_calls;

static void set_pending(const char* cls, const char* msg) {
    if (g_pending[0]) return; /* the first exception stays pending, as in a JVM */
    strncpy(g_pending, cls, sizeof g_pending - 1);
    strncat(g_pending, ": ", sizeof g_pending - strlen(g_pending) - 1);
    strncat(g_pending, msg ? msg : "", sizeof g_pending - strlen(g_pending) - 1);
}

static struct _jobject* new_obj(int kind, const void* data, size_t bytes, jsize len) {
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof *o);
    o->kind = kind;
    o->len = len;
    if (kind == K_DIRECT) {
        o->data = (void*)data;
    } else {
        o->data = malloc(bytes ? bytes : 1);
        if (bytes) memcpy(o->data, data, bytes);
    }
    return o;
}

static jclass j_find_class(JNIEnv* env, const char* name) {
    (void)env;
    return new_obj(K_CLASS, name, strlen(name) + 1, 0);
}

static jint j_throw_new(JNIEnv* env, jclass cls, const char* msg) {
    (void)env;
    set_pending(cls && cls->kind == K_CLASS ? (const char*)cls->data : "?", msg);
    return 0;
}

static jboolean j_exception_check(JNIEnv* env) {
    (void)env;
    return g_pending[0] ? JNI_TRUE : JNI_FALSE;
}

static jsize j_get_array_length(JNIEnv* env, jarray a) {
    (void)env;
    return a ? a->len : 0;
}

static void j_get_byte_array_region(JNIEnv* env, jbyteArray a, jsize start, jsize len, jbyte* buf) {
    (void)env;
    if (start < 0 || len < 0 || (int64_t)start + len > (int64_t)a->len) {
        set_pending("java/lang/ArrayIndexOutOfBoundsException", "region");
        return;
    }
    memcpy(buf, (const jbyte*)a->data + start, (size_t)len);
}

static void* j_get_critical(JNIEnv* env, jarray a, jboolean* is_copy) {
    (void)env;
    if (is_copy) *is_copy = JNI_FALSE;
    if (g_critical_fail) {
        --g_critical_fail;
        set_pending("java/lang/OutOfMemoryError", "critical");
        return NULL;
    }
    ++g_critical_depth;
    ++g_critical_total;
    return a->data;
}

static void j_release_critical(JNIEnv* env, jarray a, void* p, jint mode) {
    (void)env;
    (void)a;
    (void)p;
    (void)mode;
    --g_critical_depth;
}

static void* j_direct_address(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->data : NULL;
}

static jstring j_new_string_utf(JNIEnv* env, const char* s) {
    (void)env;
    return new_obj(K_STRING, s, strlen(s) + 1, (jsize)strlen(s));
}

static jobject j_get_object_array_element(JNIEnv* env, jobjectArray a, jsize i) {
    (void)env;
    if (i < 0 || i >= a->len) {
        set_pending("java/lang/ArrayIndexOutOfBoundsException", "element");
        return NULL;
    }
    return ((jobject*)a->data)[i];
}

static void j_get_long_array_region(JNIEnv* env, jlongArray a, jsize start, jsize len, jlong* buf) {
    (void)env;
    if (start < 0 || len < 0 || (int64_t)start + len > (int64_t)a->len) {
        set_pending("java/lang/ArrayIndexOutOfBoundsException", "region");
        return;
    }
    memcpy(buf, (const jlong*)a->data + start, (size_t)len * sizeof(jlong));
}

static int g_local_refs_deleted;
static void j_delete_local_ref(JNIEnv* env, jobject o) {
    (void)env;
    (void)o;
    ++g_local_refs_deleted;  /* the objects stay owned by the test */
}

static const struct JNINativeInterface_ g_table = {
    j_find_class,   j_throw_new,        j_exception_check, j_get_array_length, j_get_byte_array_region,
    j_get_critical, j_release_critical, j_direct_address,  j_new_string_utf,   j_get_object_array_element,
    j_get_long_array_region, j_delete_local_ref,
};
static JNIEnv g_env = &g_table;

/* ---- hooks for the test (ctypes) ---- */
JNIEXPORT JNIEnv* fake_env(void) { return &g_env; }
JNIEXPORT jobject fake_byte_array(const void* data, jsize len) { return new_obj(K_BYTES, data, (size_t)len, len); }
JNIEXPORT jobject fake_int_array(const int32_t* data, jsize len) {
    return new_obj(K_INTS, data, (size_t)len * sizeof(int32_t), len);
}
JNIEXPORT jobject fake_long_array(const int64_t* data, jsize len) {
    return new_obj(K_LONGS, data, (size_t)len * sizeof(int64_t), len);
}
/* a byte[][]: the element objects stay owned by the caller (fake_free frees only the array itself) */
JNIEXPORT jobject fake_object_array(const jobject* elems, jsize len) {
    return new_obj(K_OBJECTS, elems, (size_t)len * sizeof(jobject), len);
}
JNIEXPORT int fake_local_refs_deleted(void) { return g_local_refs_deleted; }
JNIEXPORT jobject fake_direct_buffer(void* addr) { return new_obj(K_DIRECT, addr, 0, 0); }
JNIEXPORT const char* fake_string(jobject s) { return s && s->kind == K_STRING ? (const char*)s->data : NULL; }
JNIEXPORT void fake_free(jobject o) {
    if (!o) return;
    if (o->kind != K_DIRECT) free(o->data);
    free(o);
}
JNIEXPORT const char* fake_pending(void) { return g_pending; }
JNIEXPORT void fake_clear(void) { g_pending[0] = 0; }
JNIEXPORT int fake_critical_depth(void) { return g_critical_depth; }
JNIEXPORT int fake_critical_total(void) { return g_critical_total; }
JNIEXPORT void fake_fail_critical(int times) { g_critical_fail = times; }
JNIEXPORT void fake_fail_malloc(int times) { g_malloc_fail = times; }
JNIEXPORT int fake_malloc_calls(void) { return g_malloc_calls; }

/* the shim's malloc/free (it is compiled with -Dmalloc=bkd_test_malloc -Dfree=bkd_test_free) */
void* bkd_test_malloc(size_t n) {
    ++g_malloc_calls;
    if (g_malloc_fail) {
        --g_malloc_fail;
        return NULL;
    }
    return malloc(n);
}
void bkd_test_free(void* p) { free(p); }
