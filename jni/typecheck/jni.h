/*
 * jni/typecheck/jni.h -- NOT a JDK header and never used to build a library.
 *
 * The JDK's jni.h is absent from this image.  This file declares, from the JNI specification
 * (JDK 8 "Java Native Interface Specification", chapters 3-4), only the types and the eight
 * JNIEnv functions jni/jrq_jni.c uses, with their specified C signatures, so that the CPU test
 * suite can type-check the glue (`gcc -fsyntax-only`, tests/test_jni.py).  The function table
 * here has none of the real one's layout; object code from it would be wrong, so the Makefile
 * only ever runs -fsyntax-only against it.  A real build uses -I$JAVA_HOME/include.
 */
#ifndef JRQ_TYPECHECK_JNI_H
#define JRQ_TYPECHECK_JNI_H

#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jintArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    void (*DeleteLocalRef)(JNIEnv *env, jobject obj);
    jstring (*NewStringUTF)(JNIEnv *env, const char *utf);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
    void (*GetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, jint *buf);
    jobject (*NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

#endif
