/* Minimal stand-in for a JDK's <jni.h>, used ONLY by tests/test_jni_shim.py to syntax-check
 * java/jni/titan_gpu_olap_jni.c with gcc where no JDK exists: the shim's calls into the C-ABI
 * (include/titan_gpu_olap.h) are type-checked against the real header, and its JNI calls
 * against these declarations, which follow the JNI specification's signatures (C binding:
 * JNIEnv is a pointer to the function table, calls are (*env)->Fn(env, ...)).  Only the
 * functions the shim uses are declared, so a new JNI call in the shim fails the test until it
 * is declared here with its specified signature. */
#ifndef TGO_TEST_JNI_STUB_H
#define TGO_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
    jsize (*GetArrayLength)(JNIEnv* env, jarray array);
    jobjectArray (*NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
    void (*SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
    jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
    jintArray (*NewIntArray)(JNIEnv* env, jsize len);
    jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
    jdoubleArray (*NewDoubleArray)(JNIEnv* env, jsize len);
    jint* (*GetIntArrayElements)(JNIEnv* env, jintArray array, jboolean* isCopy);
    jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
    jdouble* (*GetDoubleArrayElements)(JNIEnv* env, jdoubleArray array, jboolean* isCopy);
    void (*ReleaseIntArrayElements)(JNIEnv* env, jintArray array, jint* elems, jint mode);
    void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
    void (*ReleaseDoubleArrayElements)(JNIEnv* env, jdoubleArray array, jdouble* elems, jint mode);
    void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
    void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
    void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
    void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
    void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
};

#endif
