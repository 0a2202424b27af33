/* tests/jni_stub/jni.h -- TYPE-CHECK STUB ONLY.  This image has no JDK, so
 * tests/test_jni_shim.py runs `gcc -fsyntax-only -DHAVE_JNI` on
 * adam_amd/csrc/bqsr_jni.c against this file: the JNI types and the
 * JNIEnv function-table entries the shim calls, with the signatures of the
 * JNI specification (Java Native Interface Specification, chapter 4).
 * Nothing is ever linked or run against it; the real build uses
 * $JAVA_HOME/include/jni.h. */
#ifndef BQSR_TEST_JNI_STUB_H
#define BQSR_TEST_JNI_STUB_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef double jdouble;
typedef jint jsize;
struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;
typedef jobject jthrowable;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
  jstring (*NewString)(JNIEnv* env, const jchar* unicode, jsize len);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jobjectArray (*NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
  jobject (*GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  void (*SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
  jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
  jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
  void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
  void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
  void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
};
#endif
