/*
 * Declaration-level stand-in for <jni.h>, TEST INFRASTRUCTURE ONLY: the
 * build image has no JDK, so tests/test_jni_shim.py compiles
 * integration/jni/lda_jni.c against these declarations to check its calls'
 * types and arities (-fsyntax-only; nothing is linked or run).  The types and
 * the nine JNIEnv functions the shim calls are restated from the JNI
 * specification (Java Native Interface Specification, "JNI Types and Data
 * Structures" and "JNI Functions"); the function-table layout of a real JDK is
 * not reproduced, so this header is never used to build the shim.
 */
#ifndef LDA_TEST_STUB_JNI_H
#define LDA_TEST_STUB_JNI_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef signed char jbyte;
typedef unsigned char jboolean;
typedef unsigned short jchar;
typedef short jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jint* (*GetIntArrayElements)(JNIEnv* env, jintArray array, jboolean* isCopy);
  jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
  jdouble* (*GetDoubleArrayElements)(JNIEnv* env, jdoubleArray array, jboolean* isCopy);
  void (*ReleaseIntArrayElements)(JNIEnv* env, jintArray array, jint* elems, jint mode);
  void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
  void (*ReleaseDoubleArrayElements)(JNIEnv* env, jdoubleArray array, jdouble* elems, jint mode);
};
#endif
