/*
 * jni.h subset for a compile check of jni/vproxy_component_secure_GpuClassifier.c
 * in an image without a JDK (test infrastructure only).  The types and the
 * function-table entries the shim calls, as the JNI specification defines
 * them (Java Native Interface Specification, chapter 4 "JNI Functions");
 * the entries the shim does not use are opaque padding of the same width,
 * so every used slot keeps its specified index.  A real JDK header replaces
 * this one in jni/Makefile.
 */
#ifndef VC_TEST_JNI_H
#define VC_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef uint16_t jchar;
typedef jint jsize;

struct _jobject;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    void *reserved0, *reserved1, *reserved2, *reserved3;
    void *GetVersion, *DefineClass;                                      /* 4, 5 */
    jclass (*FindClass)(JNIEnv *env, const char *name);                  /* 6 */
    void *slots7_13[7];                                                  /* 7 .. 13 */
    jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);        /* 14 */
    void *slots15_166[152];                                              /* 15 .. 166 */
    jstring (*NewStringUTF)(JNIEnv *env, const char *utf);               /* 167 */
    void *slot168;                                                       /* 168 */
    const char *(*GetStringUTFChars)(JNIEnv *env, jstring s, jboolean *isCopy);   /* 169 */
    void (*ReleaseStringUTFChars)(JNIEnv *env, jstring s, const char *chars);     /* 170 */
    void *slot171, *slot172;                                             /* 171, 172 */
    jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray a, jsize i);       /* 173 */
    void *slots174_229[56];                                              /* 174 .. 229 */
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);           /* 230 */
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);          /* 231 */
};

#endif
