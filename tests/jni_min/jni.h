/* jni.h (minimal) -- test infrastructure, not product.
 *
 * The image has no JDK, so tests/test_jni_syntax.py type-checks
 * java/jni/hbam_jni.c against this header: the JNI primitive and reference
 * types as the JNI specification defines them for C (chapter 3, "JNI Types
 * and Data Structures": in C every reference type is jobject), the constants
 * the glue uses (chapter 4 / 5 return codes and versions, the array release
 * modes), and the entries of the JNIEnv function table (chapter 4) and the
 * JavaVM invocation table (chapter 5) that the glue calls, with the
 * specification's parameter lists.  Table order does not matter to a syntax
 * check, so only the members the glue names are declared.
 */
#ifndef HBAM_TEST_JNI_MIN_H
#define HBAM_TEST_JNI_MIN_H

#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNIIMPORT
#define JNICALL

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
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;
typedef jarray jcharArray;
typedef jarray jshortArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

struct _jmethodID;
typedef struct _jmethodID *jmethodID;
struct _jfieldID;
typedef struct _jfieldID *jfieldID;

#define JNI_FALSE 0
#define JNI_TRUE 1

#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_EDETACHED (-2)
#define JNI_EVERSION (-3)

#define JNI_COMMIT 1
#define JNI_ABORT 2

#define JNI_VERSION_1_6 0x00010006

struct JNINativeInterface_;
struct JNIInvokeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
typedef const struct JNIInvokeInterface_ *JavaVM;

struct JNINativeInterface_ {
  jclass(JNICALL *FindClass)(JNIEnv *env, const char *name);
  jint(JNICALL *ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
  void(JNICALL *ExceptionClear)(JNIEnv *env);
  jobject(JNICALL *NewGlobalRef)(JNIEnv *env, jobject obj);
  void(JNICALL *DeleteGlobalRef)(JNIEnv *env, jobject gref);
  void(JNICALL *DeleteLocalRef)(JNIEnv *env, jobject obj);
  jclass(JNICALL *GetObjectClass)(JNIEnv *env, jobject obj);
  jmethodID(JNICALL *GetMethodID)(JNIEnv *env, jclass clazz, const char *name, const char *sig);
  jint(JNICALL *CallIntMethod)(JNIEnv *env, jobject obj, jmethodID methodID, ...);
  jstring(JNICALL *NewStringUTF)(JNIEnv *env, const char *utf);
  const char *(JNICALL *GetStringUTFChars)(JNIEnv *env, jstring str, jboolean *isCopy);
  void(JNICALL *ReleaseStringUTFChars)(JNIEnv *env, jstring str, const char *chars);
  jsize(JNICALL *GetArrayLength)(JNIEnv *env, jarray array);
  jobjectArray(JNICALL *NewObjectArray)(JNIEnv *env, jsize len, jclass clazz, jobject init);
  void(JNICALL *SetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index, jobject val);
  jbyteArray(JNICALL *NewByteArray)(JNIEnv *env, jsize len);
  jlongArray(JNICALL *NewLongArray)(JNIEnv *env, jsize len);
  jbyte *(JNICALL *GetByteArrayElements)(JNIEnv *env, jbyteArray array, jboolean *isCopy);
  jint *(JNICALL *GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
  void(JNICALL *ReleaseByteArrayElements)(JNIEnv *env, jbyteArray array, jbyte *elems, jint mode);
  void(JNICALL *ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
  void(JNICALL *GetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, jlong *buf);
  void(JNICALL *SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
  void(JNICALL *SetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, const jlong *buf);
  jint(JNICALL *GetJavaVM)(JNIEnv *env, JavaVM **vm);
  jboolean(JNICALL *ExceptionCheck)(JNIEnv *env);
  jobject(JNICALL *NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
  void *(JNICALL *GetDirectBufferAddress)(JNIEnv *env, jobject buf);
  jlong(JNICALL *GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};

struct JNIInvokeInterface_ {
  jint(JNICALL *DetachCurrentThread)(JavaVM *vm);
  jint(JNICALL *GetEnv)(JavaVM *vm, void **penv, jint version);
  jint(JNICALL *AttachCurrentThreadAsDaemon)(JavaVM *vm, void **penv, void *args);
};

#endif
