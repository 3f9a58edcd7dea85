/*
 * TEST-ONLY stand-in for a JDK's <jni.h>: just the JNI types and the JNIEnv function-table members
 * that native/jni/bkdigest_jni.c calls, so that the CPU suite can compile the shim with -Wall -Werror
 * and drive every native through a fake JNIEnv (tests/jni_fake/fake_env.c, tests/test_jni_shim.py).
 * It is never used to build a library a JVM loads: the Makefile in native/jni requires a real JDK.
 * Types follow the JNI specification ("JNI Types and Data Structures"): jint is 32-bit, jlong
 * 64-bit, jboolean an unsigned 8-bit value, jsize a jint; the function table is reached as
 * (*env)->Fn(env, ...) from C.
 */
#ifndef BKD_TEST_FAKE_JNI_H
#define BKD_TEST_FAKE_JNI_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

/* the members the shim uses, by name (the real table has ~230, in a fixed order) */
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
    jboolean (*ExceptionCheck)(JNIEnv* env);
    jsize (*GetArrayLength)(JNIEnv* env, jarray array);
    void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void* (*GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode);
    void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
    jobject (*GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
    void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
    void (*DeleteLocalRef)(JNIEnv* env, jobject ref);
};

#endif
