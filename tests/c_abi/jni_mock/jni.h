/* Test double of the JDK's <jni.h> for tests/c_abi/jni_consumer.c: the JNI types and the
 * JNIEnv functions integration/jni/eegfx_jni.c calls, with the JNI specification's signatures,
 * so that file compiles and RUNS under a mock environment without a JVM (the image has no JDK).
 * It is not the JDK header: the function table holds only those entries, so a native that called
 * any other JNIEnv function -- GetPrimitiveArrayCritical included -- would not compile here.
 * Both sides (eegfx_jni.c and jni_consumer.c) are compiled against this file; the real build
 * (make -C integration jni) uses $JAVA_HOME/include/jni.h. */
#ifndef EEGFX_TEST_JNI_MOCK_H_
#define EEGFX_TEST_JNI_MOCK_H_

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
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
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jdoubleArray;
typedef jarray jintArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jsize(JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
  void(JNICALL* GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len,
                                      jdouble* buf);
  void(JNICALL* SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len,
                                      const jdouble* buf);
  void(JNICALL* SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len,
                                   const jint* buf);
  jobject(JNICALL* GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  jstring(JNICALL* NewStringUTF)(JNIEnv* env, const char* utf);
  const char*(JNICALL* GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void(JNICALL* ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
};

#endif
