/*
 * cep_jni.c — JNI binding of libcep.so (include/cep.h) for
 * org.apache.flink.streaming.siddhi.gpu.CepNative (flink-siddhi_amd/java/).
 *
 * Build next to libcep.so on a host with a JDK (none exists in this image,
 * so this file ships as source):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -I../../include cep_jni.c -L.. -lcep -Wl,-rpath,'$ORIGIN' -o libcep_jni.so
 *
 * Every function is a thin marshalling layer: Java strings to UTF-8, direct
 * ByteBuffers to their addresses (no copies; libcep copies host batches before
 * returning), status codes back as ints.  The output callback runs on the
 * calling Java thread inside cep_flush, as StreamCallback.receive runs inside
 * InputHandler.send (operator/StreamOutputHandler.java:63).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cep.h"

#define FN(name) Java_org_apache_flink_streaming_siddhi_gpu_CepNative_##name

static const char* utf(JNIEnv* env, jstring s) { return s ? (*env)->GetStringUTFChars(env, s, NULL) : NULL; }
static void unutf(JNIEnv* env, jstring s, const char* p) {
  if (s && p) (*env)->ReleaseStringUTFChars(env, s, p);
}
static void set_err(JNIEnv* env, jobjectArray err, const char* msg) {
  if (err && (*env)->GetArrayLength(env, err) > 0)
    (*env)->SetObjectArrayElement(env, err, 0, (*env)->NewStringUTF(env, msg));
}

/* ---- cep_operator --------------------------------------------------------- */
JNIEXPORT jlong JNICALL FN(operatorCreate)(JNIEnv* env, jclass cls, jint device, jlongArray options,
                                           jobjectArray err) {
  cep_options o;
  cep_default_options(&o);
  o.device = device;
  jlong v[6] = {16, 1 << 20, 1 << 22, 1, 0, 0};
  const jsize n = options ? (*env)->GetArrayLength(env, options) : 0;
  if (n > 0) (*env)->GetLongArrayRegion(env, options, 0, n < 6 ? n : 6, v);
  o.pending_slots = (int32_t)v[0];
  o.key_capacity = v[1];
  o.chunk_events = v[2];
  o.ordered_output = (int32_t)v[3];
  o.late_policy = (int32_t)v[4];
  o.sparse_keys = (int32_t)v[5];
  o.omit_seq = 1; /* StreamOutputHandler never reads the arrival numbers */
  char msg[2048] = {0};
  cep_operator* op = cep_operator_create(&o, msg, sizeof msg);
  if (!op) set_err(env, err, msg);
  return (jlong)(intptr_t)op;
}

JNIEXPORT void JNICALL FN(operatorDestroy)(JNIEnv* env, jclass cls, jlong op) {
  cep_operator_destroy((cep_operator*)(intptr_t)op);
}

static jint plan_call(JNIEnv* env, jlong op, jstring id, jstring plan, int kind) {
  const char* i = utf(env, id);
  const char* p = utf(env, plan);
  cep_operator* o = (cep_operator*)(intptr_t)op;
  int rc = kind == 0 ? cep_operator_add_plan(o, i, p) : kind == 1 ? cep_operator_update_plan(o, i, p)
                                                                  : cep_operator_remove_plan(o, i);
  unutf(env, plan, p);
  unutf(env, id, i);
  return rc;
}

JNIEXPORT jint JNICALL FN(operatorAddPlan)(JNIEnv* env, jclass cls, jlong op, jstring id, jstring plan) {
  return plan_call(env, op, id, plan, 0);
}
JNIEXPORT jint JNICALL FN(operatorUpdatePlan)(JNIEnv* env, jclass cls, jlong op, jstring id, jstring plan) {
  return plan_call(env, op, id, plan, 1);
}
JNIEXPORT jint JNICALL FN(operatorRemovePlan)(JNIEnv* env, jclass cls, jlong op, jstring id) {
  return plan_call(env, op, id, NULL, 2);
}

JNIEXPORT jint JNICALL FN(operatorEnable)(JNIEnv* env, jclass cls, jlong op, jstring id, jboolean on) {
  const char* i = utf(env, id);
  const int rc = cep_operator_enable((cep_operator*)(intptr_t)op, i, on ? 1 : 0);
  unutf(env, id, i);
  return rc;
}

JNIEXPORT jlong JNICALL FN(operatorPlan)(JNIEnv* env, jclass cls, jlong op, jstring id) {
  const char* i = utf(env, id);
  cep_app* a = cep_operator_plan((cep_operator*)(intptr_t)op, i);
  unutf(env, id, i);
  return (jlong)(intptr_t)a;
}

JNIEXPORT jint JNICALL FN(operatorIntern)(JNIEnv* env, jclass cls, jlong op, jstring s) {
  const char* p = utf(env, s);
  const int32_t id = cep_operator_intern((cep_operator*)(intptr_t)op, p ? p : "");
  unutf(env, s, p);
  return id;
}

JNIEXPORT jstring JNICALL FN(operatorLookup)(JNIEnv* env, jclass cls, jlong op, jint id) {
  const char* s = cep_operator_lookup((cep_operator*)(intptr_t)op, id);
  return s ? (*env)->NewStringUTF(env, s) : NULL;
}

JNIEXPORT jstring JNICALL FN(operatorLastError)(JNIEnv* env, jclass cls, jlong op) {
  const char* s = cep_operator_last_error((cep_operator*)(intptr_t)op);
  return (*env)->NewStringUTF(env, s ? s : "");
}

/* ---- plan-level ------------------------------------------------------------- */
JNIEXPORT jstring JNICALL FN(planInputStreams)(JNIEnv* env, jclass cls, jstring plan) {
  const char* p = utf(env, plan);
  char buf[8192] = {0};
  const int rc = cep_plan_input_streams(p, buf, sizeof buf);
  unutf(env, plan, p);
  return (*env)->NewStringUTF(env, rc == CEP_OK ? buf : "");
}

JNIEXPORT jint JNICALL FN(validate)(JNIEnv* env, jclass cls, jstring plan, jobjectArray err) {
  const char* p = utf(env, plan);
  char msg[2048] = {0};
  const int rc = cep_validate(p, msg, sizeof msg);
  unutf(env, plan, p);
  if (rc != CEP_OK) set_err(env, err, msg);
  return rc;
}

/* ---- one plan's runtime ------------------------------------------------------ */
JNIEXPORT jint JNICALL FN(streamSchema)(JNIEnv* env, jclass cls, jlong app, jstring sid, jobjectArray names,
                                        jintArray types, jintArray nout) {
  const char* s = utf(env, sid);
  cep_attr at[64];
  int n = 0;
  const int rc = cep_stream_schema((cep_app*)(intptr_t)app, s, at, 64, &n);
  unutf(env, sid, s);
  if (rc != CEP_OK) return rc;
  const jsize cap = (*env)->GetArrayLength(env, names);
  if (n > cap) n = cap;
  for (int i = 0; i < n; ++i) {
    (*env)->SetObjectArrayElement(env, names, i, (*env)->NewStringUTF(env, at[i].name));
    const jint t = at[i].type;
    (*env)->SetIntArrayRegion(env, types, i, 1, &t);
  }
  const jint jn = n;
  (*env)->SetIntArrayRegion(env, nout, 0, 1, &jn);
  return CEP_OK;
}

JNIEXPORT jint JNICALL FN(input)(JNIEnv* env, jclass cls, jlong app, jstring sid) {
  const char* s = utf(env, sid);
  const int h = cep_input((cep_app*)(intptr_t)app, s);
  unutf(env, sid, s);
  return h;
}

/* Output callback: one RowSink per (runtime, output stream), held as a global
 * reference for the runtime's lifetime (the Java operator keeps the sinks). */
typedef struct {
  JavaVM* vm;
  jobject sink;
  int failed;   /* receive threw: no more JNI work until the exception reaches Java */
  jmethodID receive;
  jclass bb;
  int ncols;
  int width[64];   /* element bytes per output column (include/cep.h layouts) */
} sink_ctx;

static int type_width(int t) { return t == CEP_LONG || t == CEP_DOUBLE ? 8 : t == CEP_BOOL ? 1 : 4; }

static void emit(void* user, const cep_rows* rows) {
  sink_ctx* c = (sink_ctx*)user;
  JNIEnv* env = NULL;
  if ((*c->vm)->GetEnv(c->vm, (void**)&env, JNI_VERSION_1_8) != JNI_OK || !env) return;
  /* An exception thrown by an earlier receive is still pending: JNI calls
   * other than the exception functions are undefined until it returns to Java
   * (when cep_flush returns), so later callbacks of this flush do nothing. */
  if (c->failed || (*env)->ExceptionCheck(env)) {
    c->failed = 1;
    return;
  }
  const jlong n = rows->n;
  jobject ts = (*env)->NewDirectByteBuffer(env, (void*)rows->ts, n * 8);
  jobjectArray cols = (*env)->NewObjectArray(env, rows->ncols, c->bb, NULL);
  for (int i = 0; i < rows->ncols && i < c->ncols; ++i) {
    jobject b = (*env)->NewDirectByteBuffer(env, (void*)rows->cols[i], n * c->width[i]);
    (*env)->SetObjectArrayElement(env, cols, i, b);
    (*env)->DeleteLocalRef(env, b);
  }
  (*env)->CallVoidMethod(env, c->sink, c->receive, n, ts, cols);
  if ((*env)->ExceptionCheck(env)) {
    c->failed = 1;   /* DeleteLocalRef is allowed with a pending exception */
  }
  (*env)->DeleteLocalRef(env, cols);
  (*env)->DeleteLocalRef(env, ts);
}

JNIEXPORT jint JNICALL FN(setCallback)(JNIEnv* env, jclass cls, jlong app, jstring out, jobject sink) {
  sink_ctx* c = (sink_ctx*)calloc(1, sizeof(sink_ctx));
  if (!c) return CEP_E_ARG;
  (*env)->GetJavaVM(env, &c->vm);
  c->sink = (*env)->NewGlobalRef(env, sink);
  jclass sc = (*env)->GetObjectClass(env, sink);
  c->receive = (*env)->GetMethodID(env, sc, "receive", "(JLjava/nio/ByteBuffer;[Ljava/nio/ByteBuffer;)V");
  c->bb = (jclass)(*env)->NewGlobalRef(env, (*env)->FindClass(env, "java/nio/ByteBuffer"));
  const char* o = utf(env, out);
  cep_attr at[64];
  int rc = cep_stream_schema((cep_app*)(intptr_t)app, o, at, 64, &c->ncols);
  for (int i = 0; rc == CEP_OK && i < c->ncols; ++i) c->width[i] = type_width(at[i].type);
  if (rc == CEP_OK) rc = cep_set_callback((cep_app*)(intptr_t)app, o, emit, c);
  unutf(env, out, o);
  return rc;
}

static jint batch_call(JNIEnv* env, jlong app, jint input, jlong n, jobject ts, jobject stream, jobjectArray cols,
                       int buffer) {
  const jsize nc = cols ? (*env)->GetArrayLength(env, cols) : 0;
  const void* ptrs[64];
  if (nc > 64) return CEP_E_ARG;
  for (jsize i = 0; i < nc; ++i) {
    jobject b = (*env)->GetObjectArrayElement(env, cols, i);
    ptrs[i] = (*env)->GetDirectBufferAddress(env, b);
    (*env)->DeleteLocalRef(env, b);
  }
  cep_batch bt;
  memset(&bt, 0, sizeof bt);
  bt.n = n;
  bt.ts = (const int64_t*)(*env)->GetDirectBufferAddress(env, ts);
  bt.stream = stream ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, stream) : NULL;
  bt.input = input;
  bt.ncols = nc;
  bt.cols = ptrs;
  bt.on_device = 0;
  cep_app* a = (cep_app*)(intptr_t)app;
  return buffer ? cep_buffer_batch(a, &bt) : cep_send_batch(a, &bt);
}

JNIEXPORT jint JNICALL FN(sendBatch)(JNIEnv* env, jclass cls, jlong app, jint input, jlong n, jobject ts,
                                     jobject stream, jobjectArray cols) {
  return batch_call(env, app, input, n, ts, stream, cols, 0);
}

JNIEXPORT jint JNICALL FN(bufferBatch)(JNIEnv* env, jclass cls, jlong app, jint input, jlong n, jobject ts,
                                       jobject stream, jobjectArray cols) {
  return batch_call(env, app, input, n, ts, stream, cols, 1);
}

JNIEXPORT jint JNICALL FN(watermark)(JNIEnv* env, jclass cls, jlong app, jlong mark) {
  return cep_watermark((cep_app*)(intptr_t)app, mark);
}

/* A RowSink exception propagates to Java when this returns; the sinks'
 * failed flags are per sink, so a sink that threw stays silent for the rest of
 * the operator's life (the Flink task fails on the exception anyway). */
JNIEXPORT jint JNICALL FN(flush)(JNIEnv* env, jclass cls, jlong app) { return cep_flush((cep_app*)(intptr_t)app); }

JNIEXPORT jbyteArray JNICALL FN(snapshot)(JNIEnv* env, jclass cls, jlong app) {
  uint8_t* buf = NULL;
  size_t len = 0;
  if (cep_snapshot((cep_app*)(intptr_t)app, &buf, &len) != CEP_OK) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)len);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)len, (const jbyte*)buf);
  cep_free(buf);
  return out;
}

JNIEXPORT jint JNICALL FN(restore)(JNIEnv* env, jclass cls, jlong app, jbyteArray state) {
  const jsize len = (*env)->GetArrayLength(env, state);
  jbyte* p = (*env)->GetByteArrayElements(env, state, NULL);
  const int rc = cep_restore((cep_app*)(intptr_t)app, (const uint8_t*)p, (size_t)len);
  (*env)->ReleaseByteArrayElements(env, state, p, JNI_ABORT);
  return rc;
}

JNIEXPORT jstring JNICALL FN(lastError)(JNIEnv* env, jclass cls, jlong app) {
  const char* s = cep_last_error((cep_app*)(intptr_t)app);
  return (*env)->NewStringUTF(env, s ? s : "");
}
