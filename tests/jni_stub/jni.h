/* Minimal JNI declarations -- TEST INFRASTRUCTURE ONLY: lets tests/test_java_binding.py syntax-check jni/gwo_jni.c
 * (types, arity, every JNIEnv call it makes) in an image without a JDK.  Not a JDK header and never used to
 * build the shim (`make jni` requires a real JAVA_HOME). */
#include <stdint.h>
typedef int32_t jint; typedef int64_t jlong; typedef int8_t jbyte; typedef uint8_t jboolean; typedef uint16_t jchar;
typedef jint jsize; typedef void *jobject; typedef jobject jclass, jstring, jarray, jobjectArray, jlongArray, jintArray, jcharArray, jbyteArray;
#define JNI_ABORT 2
#define JNIEXPORT
#define JNICALL
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  void *(*GetDirectBufferAddress)(JNIEnv*, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void (*DeleteLocalRef)(JNIEnv*, jobject);
  jboolean (*ExceptionCheck)(JNIEnv*);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  jlong *(*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
  void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
  jint *(*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  jobjectArray (*NewObjectArray)(JNIEnv*, jsize, jclass, jobject);
  jstring (*NewString)(JNIEnv*, const jchar*, jsize);
  void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  jbyte *(*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
};
