/* bqsr_jni.c -- the JVM side of the drop-in boundary: the JNI shim a Spark
 * executor loads (System.loadLibrary("adam_bqsr_jni")) to run the two
 * partition bodies of RecalibrateBaseQualities (computeTable's per-partition
 * fold, RecalibrateBaseQualities.scala:52-64, and applyTable's per-partition
 * map, :66-76) through libadam_bqsr.so (include/adam_bqsr.h).  Java
 * declarations and the Scala call sites: INTEGRATION.md §1-2.
 *
 * Two layers:
 *  - the core (always compiled, plain C over the C ABI, no JNI types): the
 *    status -> Java exception mapping and the observe / finalize / apply
 *    sequences the JNI entry points run.  __graft_entry__.build() compiles it
 *    into adam_amd/libadam_bqsr_jni.so and the tests call it through ctypes.
 *  - the JNI entry points (#ifdef HAVE_JNI): argument marshalling only
 *    (direct ByteBuffers -> bqsr_records, long[] <-> table words, UTF-16
 *    quality strings -> java.lang.String).  This image has no JDK; the
 *    maintainer's build is
 *      gcc -shared -fPIC -DHAVE_JNI -I$JAVA_HOME/include -I$JAVA_HOME/include/linux
 *          -Iinclude adam_amd/csrc/bqsr_jni.c -Ladam_amd -ladam_bqsr -o libadam_bqsr_jni.so
 *    (tests/test_jni_shim.py type-checks this branch against the JNI calls it
 *    uses, see tests/jni_stub/jni.h).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/adam_bqsr.h"

#if defined(__GNUC__)
#define BQSR_JNI_API __attribute__((visibility("default")))
#else
#define BQSR_JNI_API
#endif

/* The exception class the Scala reference raises where the library reports
 * `s` (the reference file:line of each is on the status in adam_bqsr.h). */
BQSR_JNI_API const char* bqsr_jni_exception_class(bqsr_status s) {
  switch (s) {
    case BQSR_OK:
      return NULL;
    case BQSR_ERR_NULL_RG:
    case BQSR_ERR_NULL_FIELD:
      return "java/lang/NullPointerException";
    case BQSR_ERR_MD_PARSE:
      return "java/lang/IllegalArgumentException";
    case BQSR_ERR_CIGAR_SHORT:
      return "java/lang/IndexOutOfBoundsException";
    case BQSR_ERR_BAD_REVCOMP_BASE:
    case BQSR_ERR_MISSING_KEY:
    case BQSR_ERR_CIGAR_INVALID:
      return "java/util/NoSuchElementException";
    case BQSR_ERR_EMPTY_TABLE:
      return "java/lang/UnsupportedOperationException";
    case BQSR_ERR_QUAL_RANGE:
    case BQSR_ERR_SEQ_SHORT:
      return "java/lang/ArrayIndexOutOfBoundsException";
    case BQSR_ERR_INVALID_ARG:
      return "java/lang/IllegalArgumentException";
    default: /* DEVICE, UNSUPPORTED, SAM_PARSE: no reference counterpart */
      return "java/lang/RuntimeException";
  }
}

/* applyTable recalibrates mapped, primary, non-duplicate reads
 * (RecalibrateBaseQualities.scala:70-72); others are returned unchanged. */
BQSR_JNI_API int bqsr_jni_eligible(uint32_t flags) {
  return (flags & BQSR_F_MAPPED) && (flags & BQSR_F_PRIMARY) && !(flags & BQSR_F_DUPLICATE);
}

/* computeTable's seqOp over one partition: the partition's table words
 * (bqsr_table_words(d) int64) and its expectedMismatch. */
BQSR_JNI_API bqsr_status bqsr_jni_observe(bqsr_context* ctx, const bqsr_sites* sites, const bqsr_records* r,
                                          bqsr_dims d, int64_t* words, double* em) {
  bqsr_table* t = NULL;
  if (!words || !em) return BQSR_ERR_INVALID_ARG;
  bqsr_status st = bqsr_observe_records(ctx, r, sites, d, &t, em);
  if (st != BQSR_OK) return st;
  st = bqsr_table_download(t, words);
  bqsr_table_destroy(t);
  return st;
}

/* finalizeTable on the driver's merged words (RecalTable.++ already applied
 * by the caller: an int64 sum, and the em fold in partition order). */
BQSR_JNI_API bqsr_status bqsr_jni_finalize(bqsr_context* ctx, const int64_t* words, bqsr_dims d, double em,
                                           bqsr_lut** out) {
  bqsr_table* t = NULL;
  if (!words || !out) return BQSR_ERR_INVALID_ARG;
  *out = NULL;
  bqsr_status st = bqsr_table_create(ctx, d, NULL, &t);
  if (st == BQSR_OK) st = bqsr_table_upload(t, words);
  if (st == BQSR_OK) st = bqsr_finalize(ctx, t, em, out);
  bqsr_table_destroy(t);
  return st;
}

/* applyTable's map over one partition: out_chars[qual_offset[i] ..
 * + out_len[i]) is read i's new quality string as Java chars; pass-through
 * reads get out_len -1 (the JNI layer returns null for them: the record is
 * kept unchanged). */
BQSR_JNI_API bqsr_status bqsr_jni_apply(bqsr_context* ctx, const bqsr_lut* l, const bqsr_records* r,
                                        uint16_t* out_chars, int32_t* out_len) {
  if (!r || !out_chars || !out_len) return BQSR_ERR_INVALID_ARG;
  bqsr_status st = bqsr_apply_records(ctx, r, l, out_chars, (uint32_t*)out_len);
  if (st != BQSR_OK) return st;
  for (int64_t i = 0; i < r->n_reads; ++i)
    if (!bqsr_jni_eligible(r->flags[i])) out_len[i] = -1;
  return BQSR_OK;
}

#ifdef HAVE_JNI
#include <jni.h>

#define JFN(name) Java_edu_berkeley_cs_amplab_adam_rdd_recalibration_HipBqsr_##name

static void rethrow(JNIEnv* env, bqsr_status s) {
  jclass k = (*env)->FindClass(env, bqsr_jni_exception_class(s));
  if (k) (*env)->ThrowNew(env, k, bqsr_last_error());
}

#define BUF(b) ((*env)->GetDirectBufferAddress(env, (b)))

/* the partition's columns, filled on the JVM side by HipBqsr.Columns.pack
 *  as direct native-order ByteBuffers */
static bqsr_records columns(JNIEnv* env, jint n, jobject flags, jobject rg, jobject contig, jobject start,
                            jobject so, jobject s, jobject qo, jobject q, jobject co, jobject c, jobject mo,
                            jobject m) {
  bqsr_records r;
  r.n_reads = n;
  r.flags = (const uint32_t*)BUF(flags);
  r.rg_id = (const int32_t*)BUF(rg);
  r.contig_id = (const int32_t*)BUF(contig);
  r.start = (const int64_t*)BUF(start);
  r.seq_offset = (const uint64_t*)BUF(so);
  r.seq = (const uint8_t*)BUF(s);
  r.qual_offset = (const uint64_t*)BUF(qo);
  r.qual = (const uint8_t*)BUF(q);
  r.cigar_offset = (const uint64_t*)BUF(co);
  r.cigar = (const uint32_t*)BUF(c);
  r.md_offset = (const uint64_t*)BUF(mo);
  r.md = (const uint8_t*)BUF(m);
  return r;
}

JNIEXPORT jlong JNICALL JFN(contextCreate)(JNIEnv* env, jclass k, jint device) {
  bqsr_context* c = NULL;
  bqsr_status s = bqsr_context_create(device, &c);
  (void)k;
  if (s != BQSR_OK) rethrow(env, s);
  return (jlong)(intptr_t)c;
}

/* SnpTable (Map[String, Set[Long]], SnpTable.scala:12-47) as contig names and
 * one long[] of VCF POS values per contig (as stored: quirk Q7) */
JNIEXPORT jlong JNICALL JFN(sitesCreate)(JNIEnv* env, jclass k, jlong ctx, jobjectArray contigs,
                                         jobjectArray pos) {
  const jsize nc = (*env)->GetArrayLength(env, contigs);
  const char** names = calloc((size_t)nc + 1, sizeof(char*));
  const int64_t** p = calloc((size_t)nc + 1, sizeof(int64_t*));
  uint64_t* n = calloc((size_t)nc + 1, sizeof(uint64_t));
  jstring* js = calloc((size_t)nc + 1, sizeof(jstring));
  jlongArray* ja = calloc((size_t)nc + 1, sizeof(jlongArray));
  bqsr_sites* out = NULL;
  bqsr_status st = (names && p && n && js && ja) ? BQSR_OK : BQSR_ERR_INVALID_ARG;
  (void)k;
  for (jsize i = 0; st == BQSR_OK && i < nc; ++i) {
    js[i] = (jstring)(*env)->GetObjectArrayElement(env, contigs, i);
    ja[i] = (jlongArray)(*env)->GetObjectArrayElement(env, pos, i);
    names[i] = (*env)->GetStringUTFChars(env, js[i], NULL);
    n[i] = (uint64_t)(*env)->GetArrayLength(env, ja[i]);
    p[i] = (const int64_t*)(*env)->GetLongArrayElements(env, ja[i], NULL);
  }
  if (st == BQSR_OK) st = bqsr_sites_create((bqsr_context*)(intptr_t)ctx, names, p, n, (int32_t)nc, &out);
  for (jsize i = 0; js && ja && i < nc; ++i) {
    if (names && names[i]) (*env)->ReleaseStringUTFChars(env, js[i], names[i]);
    if (p && p[i]) (*env)->ReleaseLongArrayElements(env, ja[i], (jlong*)p[i], JNI_ABORT);
  }
  free(names);
  free(p);
  free(n);
  free(js);
  free(ja);
  if (st != BQSR_OK) rethrow(env, st);
  return (jlong)(intptr_t)out;
}

JNIEXPORT jlongArray JNICALL JFN(observe)(JNIEnv* env, jclass k, jlong ctx, jlong sites, jint n, jobject flags,
                                          jobject rg, jobject contig, jobject start, jobject so, jobject s,
                                          jobject qo, jobject q, jobject co, jobject c, jobject mo, jobject m,
                                          jint n_rg, jint max_len, jdoubleArray em_out) {
  bqsr_records r = columns(env, n, flags, rg, contig, start, so, s, qo, q, co, c, mo, m);
  bqsr_dims d;
  double em = 0.0;
  (void)k;
  d.n_rg = n_rg;
  d.max_len = max_len;
  jlongArray out = (*env)->NewLongArray(env, (jsize)bqsr_table_words(d));
  if (!out) return NULL; /* OutOfMemoryError pending */
  jlong* w = (*env)->GetLongArrayElements(env, out, NULL);
  bqsr_status st = bqsr_jni_observe((bqsr_context*)(intptr_t)ctx, (const bqsr_sites*)(intptr_t)sites, &r, d,
                                    (int64_t*)w, &em);
  (*env)->ReleaseLongArrayElements(env, out, w, st == BQSR_OK ? 0 : JNI_ABORT);
  if (st != BQSR_OK) {
    rethrow(env, st);
    return NULL;
  }
  (*env)->SetDoubleArrayRegion(env, em_out, 0, 1, &em);
  return out;
}

JNIEXPORT jlong JNICALL JFN(finalizeTable)(JNIEnv* env, jclass k, jlong ctx, jlongArray words, jint n_rg,
                                           jint max_len, jdouble em) {
  bqsr_dims d;
  bqsr_lut* l = NULL;
  (void)k;
  d.n_rg = n_rg;
  d.max_len = max_len;
  jlong* w = (*env)->GetLongArrayElements(env, words, NULL);
  bqsr_status st = bqsr_jni_finalize((bqsr_context*)(intptr_t)ctx, (const int64_t*)w, d, em, &l);
  (*env)->ReleaseLongArrayElements(env, words, w, JNI_ABORT);
  if (st != BQSR_OK) {
    rethrow(env, st);
    return 0;
  }
  return (jlong)(intptr_t)l;
}

JNIEXPORT jobjectArray JNICALL JFN(apply)(JNIEnv* env, jclass k, jlong ctx, jlong lut, jint n, jobject flags,
                                          jobject rg, jobject contig, jobject start, jobject so, jobject s,
                                          jobject qo, jobject q, jobject co, jobject c, jobject mo, jobject m) {
  bqsr_records r = columns(env, n, flags, rg, contig, start, so, s, qo, q, co, c, mo, m);
  const uint64_t nq = r.qual_offset[n];
  uint16_t* chars = malloc(sizeof(uint16_t) * (nq ? nq : 1));
  int32_t* len = malloc(sizeof(int32_t) * (n ? (size_t)n : 1));
  jobjectArray out = NULL;
  (void)k;
  bqsr_status st = (chars && len) ? bqsr_jni_apply((bqsr_context*)(intptr_t)ctx, (const bqsr_lut*)(intptr_t)lut,
                                                   &r, chars, len)
                                  : BQSR_ERR_INVALID_ARG;
  if (st != BQSR_OK) {
    rethrow(env, st);
  } else {
    out = (*env)->NewObjectArray(env, n, (*env)->FindClass(env, "java/lang/String"), NULL);
    for (jint i = 0; out && i < n; ++i) {
      if (len[i] < 0) continue; /* null: the record is returned unchanged */
      jstring js = (*env)->NewString(env, (const jchar*)(chars + r.qual_offset[i]), (jsize)len[i]);
      (*env)->SetObjectArrayElement(env, out, i, js);
      (*env)->DeleteLocalRef(env, js);
    }
  }
  free(chars);
  free(len);
  return out;
}

JNIEXPORT void JNICALL JFN(lutDestroy)(JNIEnv* env, jclass k, jlong lut) {
  (void)env;
  (void)k;
  bqsr_lut_destroy((bqsr_lut*)(intptr_t)lut);
}

/* streamed partitions */
JNIEXPORT jlong JNICALL JFN(stage)(JNIEnv* env, jclass k, jlong ctx, jint n, jobject flags, jobject rg,
                                   jobject contig, jobject start, jobject so, jobject s, jobject qo, jobject q,
                                   jobject co, jobject c, jobject mo, jobject m) {
  bqsr_records r = columns(env, n, flags, rg, contig, start, so, s, qo, q, co, c, mo, m);
  bqsr_staged* st = NULL;
  (void)k;
  bqsr_status x = bqsr_stage_records((bqsr_context*)(intptr_t)ctx, &r, &st);
  if (x != BQSR_OK) rethrow(env, x);
  return (jlong)(intptr_t)st; /* pinned, link format: the direct buffers may be dropped now */
}

JNIEXPORT jlong JNICALL JFN(batchFromStaged)(JNIEnv* env, jclass k, jlong ctx, jlong st) {
  bqsr_batch* b = NULL;
  (void)k;
  bqsr_status x = bqsr_batch_create_staged((bqsr_context*)(intptr_t)ctx, (const bqsr_staged*)(intptr_t)st, &b);
  if (x != BQSR_OK) rethrow(env, x);
  return (jlong)(intptr_t)b;
}

JNIEXPORT void JNICALL JFN(upload)(JNIEnv* env, jclass k, jlong b, jlong st, jlong copy_stream) {
  (void)k;
  bqsr_status x = bqsr_batch_upload_async((bqsr_batch*)(intptr_t)b, (const bqsr_staged*)(intptr_t)st,
                                          (void*)(intptr_t)copy_stream);
  if (x != BQSR_OK) rethrow(env, x);
}

JNIEXPORT void JNICALL JFN(stagedFree)(JNIEnv* env, jclass k, jlong st) {
  (void)env;
  (void)k;
  bqsr_staged_destroy((bqsr_staged*)(intptr_t)st);
}
#endif /* HAVE_JNI */
