/* hbam_jni.c -- JNI glue between org.seqdoop.hadoop_bam.gpu.HbamNative and
 * libhbam.so (include/hbam.h).  Plain C over the C ABI: copies Java arrays in
 * and out, wraps the library's pinned host columns as direct ByteBuffers and
 * maps status codes to the exceptions the replaced Java methods throw.
 *
 * Build (with a JDK):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       java/jni/hbam_jni.c -Lhadoop-bam_amd/lib -lhbam -o libhbam_jni.so
 * Not built in this repository (the image has no jni.h); every entry point it
 * calls is exercised through ctypes by tests/.
 */
#include <jni.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hbam.h"

#define FN(name) JNICALL Java_org_seqdoop_hadoop_1bam_gpu_HbamNative_##name
#define CTX(h) ((hbam_ctx *)(intptr_t)(h))

static void throw_for(JNIEnv *env, int rc, const char *msg) {
  const char *cls = rc == HBAM_E_ARG      ? "java/lang/IllegalArgumentException"
                    : rc == HBAM_E_FORMAT ? "htsjdk/samtools/SAMFormatException"
                    : rc == HBAM_E_TRUNC  ? "htsjdk/samtools/FileTruncatedException"
                                          : "java/io/IOException";
  jclass c = (*env)->FindClass(env, cls);
  if (!c) return; /* NoClassDefFoundError already pending */
  (*env)->ThrowNew(env, c, msg && *msg ? msg : "libhbam error");
}

static jbyteArray to_bytes(JNIEnv *env, const uint8_t *p, uint64_t n) {
  jbyteArray a = (*env)->NewByteArray(env, (jsize)n);
  if (a && n) (*env)->SetByteArrayRegion(env, a, 0, (jsize)n, (const jbyte *)p);
  return a;
}

/* long[] -> malloc'd uint64_t[] (caller frees); NULL + pending exception on failure */
static uint64_t *from_longs(JNIEnv *env, jlongArray a, jsize *n) {
  *n = a ? (*env)->GetArrayLength(env, a) : 0;
  uint64_t *v = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(*n ? *n : 1));
  if (!v) {
    throw_for(env, HBAM_E_NOMEM, "out of memory");
    return NULL;
  }
  if (*n) (*env)->GetLongArrayRegion(env, a, 0, *n, (jlong *)v);
  return v;
}

static jlongArray to_longs(JNIEnv *env, const uint64_t *v, jsize n) {
  jlongArray a = (*env)->NewLongArray(env, n);
  if (a && n) (*env)->SetLongArrayRegion(env, a, 0, n, (const jlong *)v);
  return a;
}

/* the 16 columns of a batch as direct buffers (HbamNative column order) */
static jobjectArray wrap_batch(JNIEnv *env, const hbam_batch *b) {
  jclass bb = (*env)->FindClass(env, "java/nio/ByteBuffer");
  jobjectArray out = (*env)->NewObjectArray(env, 16, bb, NULL);
  if (!out) return NULL;
  const void *cols[16] = {b->key,     b->voff,        b->ref_id,   b->pos,  b->l_read_name, b->mapq,
                          b->bin,     b->n_cigar,     b->flag,     b->l_seq, b->next_ref_id, b->next_pos,
                          b->tlen,    b->rest_off,    b->rest_len, b->data};
  static const uint64_t width[15] = {8, 8, 4, 4, 1, 1, 2, 2, 2, 4, 4, 4, 4, 8, 4};
  for (int i = 0; i < 16; ++i) {
    const uint64_t bytes = i == 15 ? b->data_len : b->n * width[i];
    jobject buf = (*env)->NewDirectByteBuffer(env, (void *)(cols[i] ? cols[i] : (const void *)b), (jlong)bytes);
    if (!buf) return NULL;
    (*env)->SetObjectArrayElement(env, out, i, buf);
    (*env)->DeleteLocalRef(env, buf);
  }
  return out;
}

JNIEXPORT jlong FN(open)(JNIEnv *env, jclass c, jstring path, jint device, jboolean crc, jint stringency,
                         jlong window, jlong batch) {
  const char *p = (*env)->GetStringUTFChars(env, path, NULL);
  if (!p) return 0;
  hbam_opts o = {device, crc ? 1 : 0, stringency, 0, (uint64_t)window, (uint64_t)batch};
  hbam_ctx *ctx = NULL;
  int rc = hbam_open(p, &o, &ctx);
  (*env)->ReleaseStringUTFChars(env, path, p);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(ctx));
    if (ctx) hbam_close(ctx);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

/* ---- hbam_open_reader: a HbamNative.PositionedReader behind hbam_read_fn ---- */
struct jreader {
  JavaVM *vm;
  jobject reader;     /* global ref */
  jmethodID read;     /* int read(long, ByteBuffer) */
  hbam_ctx *ctx;
  struct jreader *next;
};
static struct jreader *g_readers = NULL; /* the readers of open ctxs, freed by close */
static pthread_mutex_t g_readers_mu = PTHREAD_MUTEX_INITIALIZER;

/* A library thread that calls a reader is attached here as a daemon, and
 * detached when it exits: the thread-specific value below holds its JavaVM,
 * and the key's destructor runs DetachCurrentThread at thread exit (the JNI
 * rule: a native thread detaches before it exits).  The library starts a
 * staging thread per window and its copy pool threads live as long as the
 * process; both exit through the destructor. */
static pthread_key_t g_attach_key;
static pthread_once_t g_attach_once = PTHREAD_ONCE_INIT;
static void detach_at_exit(void *vm) {
  if (vm) (*(JavaVM *)vm)->DetachCurrentThread((JavaVM *)vm);
}
static void make_attach_key(void) { (void)pthread_key_create(&g_attach_key, detach_at_exit); }

/* hbam_read_fn: called from library threads */
static int64_t jreader_read(void *user, uint64_t off, void *dst, uint64_t len) {
  struct jreader *r = (struct jreader *)user;
  JNIEnv *env = NULL;
  if ((*r->vm)->GetEnv(r->vm, (void **)&env, JNI_VERSION_1_6) != JNI_OK) {
    if ((*r->vm)->AttachCurrentThreadAsDaemon(r->vm, (void **)&env, NULL) != JNI_OK) return -1;
    (void)pthread_once(&g_attach_once, make_attach_key);
    (void)pthread_setspecific(g_attach_key, r->vm); /* detached by detach_at_exit */
  }
  uint64_t done = 0;
  while (done < len) { /* direct buffers hold < 2 GiB */
    const uint64_t n = len - done < (1u << 30) ? len - done : (1u << 30);
    jobject buf = (*env)->NewDirectByteBuffer(env, (uint8_t *)dst + done, (jlong)n);
    if (!buf) {
      (*env)->ExceptionClear(env);
      return -1;
    }
    const jint got = (*env)->CallIntMethod(env, r->reader, r->read, (jlong)(off + done), buf);
    (*env)->DeleteLocalRef(env, buf);
    if ((*env)->ExceptionCheck(env)) { /* the reader's IOException: HBAM_E_IO */
      (*env)->ExceptionClear(env);
      return -1;
    }
    if (got <= 0) break; /* end of file */
    done += (uint64_t)got;
    if ((uint64_t)got < n) break;
  }
  return (int64_t)done;
}

JNIEXPORT jlong FN(openReader)(JNIEnv *env, jclass c, jlong size, jobject reader, jboolean parallel, jint device,
                               jboolean crc, jint stringency, jlong window, jlong batch) {
  struct jreader *r = (struct jreader *)calloc(1, sizeof *r);
  jclass rc_cls = reader ? (*env)->GetObjectClass(env, reader) : NULL;
  if (!r || !rc_cls || (*env)->GetJavaVM(env, &r->vm) != 0) {
    free(r);
    throw_for(env, reader ? HBAM_E_NOMEM : HBAM_E_ARG, reader ? "out of memory" : "null reader");
    return 0;
  }
  r->read = (*env)->GetMethodID(env, rc_cls, "read", "(JLjava/nio/ByteBuffer;)I");
  if (!r->read) {
    free(r);
    return 0; /* NoSuchMethodError pending */
  }
  r->reader = (*env)->NewGlobalRef(env, reader);
  hbam_opts o = {device, crc ? 1 : 0, stringency, parallel ? 1 : 0, (uint64_t)window, (uint64_t)batch};
  hbam_ctx *ctx = NULL;
  int rc = hbam_open_reader((uint64_t)size, jreader_read, r, &o, &ctx);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(ctx));
    if (ctx) hbam_close(ctx);
    (*env)->DeleteGlobalRef(env, r->reader);
    free(r);
    return 0;
  }
  r->ctx = ctx;
  pthread_mutex_lock(&g_readers_mu);
  r->next = g_readers;
  g_readers = r;
  pthread_mutex_unlock(&g_readers_mu);
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void FN(close)(JNIEnv *env, jclass c, jlong h) {
  hbam_close(CTX(h)); /* joins the ctx's threads: no read after this */
  pthread_mutex_lock(&g_readers_mu);
  struct jreader **pp = &g_readers, *r = NULL;
  while (*pp && (*pp)->ctx != CTX(h)) pp = &(*pp)->next;
  if (*pp) {
    r = *pp;
    *pp = r->next;
  }
  pthread_mutex_unlock(&g_readers_mu);
  if (r) {
    (*env)->DeleteGlobalRef(env, r->reader);
    free(r);
  }
}

JNIEXPORT jlongArray FN(header)(JNIEnv *env, jclass c, jlong h) {
  hbam_header_info hi;
  int rc = hbam_header(CTX(h), &hi);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
    return NULL;
  }
  uint64_t v[4] = {(uint64_t)(int64_t)hi.n_ref, (uint64_t)(int64_t)hi.l_text, hi.first_record_voff, hi.file_size};
  return to_longs(env, v, 4);
}

JNIEXPORT jstring FN(headerText)(JNIEnv *env, jclass c, jlong h) {
  hbam_header_info hi;
  int rc = hbam_header(CTX(h), &hi);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
    return NULL;
  }
  /* the text is Latin-1/ASCII SAM; NewStringUTF needs a NUL-terminated copy */
  char *t = (char *)malloc((size_t)hi.l_text + 1);
  if (!t) {
    throw_for(env, HBAM_E_NOMEM, "out of memory");
    return NULL;
  }
  memcpy(t, hi.text, (size_t)hi.l_text);
  t[hi.l_text] = 0;
  jstring s = (*env)->NewStringUTF(env, t);
  free(t);
  return s;
}

JNIEXPORT void FN(prefetch)(JNIEnv *env, jclass c, jlong h, jlong lo, jlong hi) {
  int rc = hbam_prefetch(CTX(h), (uint64_t)lo, (uint64_t)hi);
  if (rc != HBAM_OK) throw_for(env, rc, hbam_last_error(CTX(h)));
}

JNIEXPORT jobjectArray FN(decodeSpan)(JNIEnv *env, jclass c, jlong h, jlong vs, jlong ve, jlong max_records,
                                      jlongArray cursor) {
  hbam_batch b;
  memset(&b, 0, sizeof b);
  int rc = hbam_decode_span(CTX(h), (uint64_t)vs, (uint64_t)ve, (uint64_t)max_records, &b);
  if (rc != HBAM_OK && b.n == 0) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
    return NULL;
  }
  /* records before a failing one are delivered; next_voff points at it, so
   * the next call (BAMRecordReader's next nextKeyValue) throws */
  if (cursor && (*env)->GetArrayLength(env, cursor) > 0) {
    jlong nv = (jlong)b.next_voff;
    (*env)->SetLongArrayRegion(env, cursor, 0, 1, &nv);
  }
  return wrap_batch(env, &b);
}

JNIEXPORT jlong FN(readerPosition)(JNIEnv *env, jclass c, jlong h, jlong i) {
  uint64_t pos = 0;
  int rc = hbam_reader_position(CTX(h), (uint64_t)i, &pos);
  if (rc != HBAM_OK) throw_for(env, rc, hbam_last_error(CTX(h)));
  return (jlong)pos;
}

JNIEXPORT jbyteArray FN(splittingIndex)(JNIEnv *env, jclass c, jlong h, jint g) {
  uint8_t *buf = NULL;
  uint64_t len = 0;
  int rc = hbam_build_splitting_index(CTX(h), g, &buf, &len);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
    return NULL;
  }
  jbyteArray a = to_bytes(env, buf, len);
  hbam_free(buf);
  return a;
}

JNIEXPORT jbyteArray FN(splittingIndexForRecords)(JNIEnv *env, jclass c, jint device, jlongArray voffs, jint g,
                                                  jlong file_size) {
  jsize n;
  uint64_t *v = from_longs(env, voffs, &n);
  if (!v) return NULL;
  hbam_opts o = {device, 0, HBAM_STRICT, 0, 0, 0};
  uint8_t *buf = NULL;
  uint64_t len = 0;
  int rc = hbam_splitting_index_for_records(&o, v, (uint64_t)n, g, (uint64_t)file_size, &buf, &len);
  free(v);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(NULL));
    return NULL;
  }
  jbyteArray a = to_bytes(env, buf, len);
  hbam_free(buf);
  return a;
}

static jlongArray guess_starts(JNIEnv *env, jlong h, jint header_n_ref, jlongArray begs, jlongArray ends) {
  jsize n, m;
  uint64_t *b = from_longs(env, begs, &n);
  if (!b) return NULL;
  uint64_t *e = from_longs(env, ends, &m);
  if (!e) {
    free(b);
    return NULL;
  }
  jlongArray r = NULL;
  if (m != n) {
    throw_for(env, HBAM_E_ARG, "begs and ends differ in length");
  } else {
    uint64_t *out = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n ? n : 1));
    int rc = out ? hbam_guess_record_starts_hdr(CTX(h), header_n_ref, b, e, (uint64_t)n, out) : HBAM_E_NOMEM;
    if (rc != HBAM_OK) throw_for(env, rc, hbam_last_error(CTX(h)));
    else r = to_longs(env, out, n);
    free(out);
  }
  free(b);
  free(e);
  return r;
}

JNIEXPORT jlongArray FN(guessRecordStarts)(JNIEnv *env, jclass c, jlong h, jlongArray begs, jlongArray ends) {
  return guess_starts(env, h, -1, begs, ends);
}

JNIEXPORT jlongArray FN(guessRecordStartsHdr)(JNIEnv *env, jclass c, jlong h, jint header_n_ref, jlongArray begs,
                                              jlongArray ends) {
  return guess_starts(env, h, header_n_ref, begs, ends);
}

JNIEXPORT jlongArray FN(getSplits)(JNIEnv *env, jclass c, jlong h, jlongArray starts, jlongArray lengths,
                                   jbyteArray sbi, jbyteArray bai) {
  jsize n, m;
  uint64_t *s = from_longs(env, starts, &n);
  if (!s) return NULL;
  uint64_t *l = from_longs(env, lengths, &m);
  if (!l) {
    free(s);
    return NULL;
  }
  jlongArray r = NULL;
  jbyte *ib = sbi ? (*env)->GetByteArrayElements(env, sbi, NULL) : NULL;
  const jsize ilen = sbi ? (*env)->GetArrayLength(env, sbi) : 0;
  jbyte *bb = bai ? (*env)->GetByteArrayElements(env, bai, NULL) : NULL;
  const jsize blen = bai ? (*env)->GetArrayLength(env, bai) : 0;
  uint64_t *vs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n ? n : 1));
  uint64_t *ve = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n ? n : 1));
  uint64_t nout = 0;
  int rc = m != n ? HBAM_E_ARG
           : (!vs || !ve)
               ? HBAM_E_NOMEM
               : hbam_get_splits_bai(CTX(h), s, l, (uint64_t)n, (const uint8_t *)ib, (uint64_t)ilen,
                                     (const uint8_t *)bb, (uint64_t)blen, vs, ve, &nout);
  if (ib) (*env)->ReleaseByteArrayElements(env, sbi, ib, JNI_ABORT);
  if (bb) (*env)->ReleaseByteArrayElements(env, bai, bb, JNI_ABORT);
  if (rc == HBAM_E_STATE) {  /* where BAMInputFormat.addBAISplits dereferences null */
    jclass npe = (*env)->FindClass(env, "java/lang/NullPointerException");
    if (npe) (*env)->ThrowNew(env, npe, hbam_last_error(CTX(h)));
  } else if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
  } else {
    uint64_t *pairs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(2 * nout + 1));
    if (!pairs) {
      throw_for(env, HBAM_E_NOMEM, "out of memory");
    } else {
      for (uint64_t i = 0; i < nout; ++i) {
        pairs[2 * i] = vs[i];
        pairs[2 * i + 1] = ve[i];
      }
      r = to_longs(env, pairs, (jsize)(2 * nout));
      free(pairs);
    }
  }
  free(vs);
  free(ve);
  free(s);
  free(l);
  return r;
}

JNIEXPORT jlong FN(encodeWritables)(JNIEnv *env, jclass c, jlong h, jobject out, jlongArray offs) {
  uint64_t len = 0;
  uint8_t *dst = out ? (uint8_t *)(*env)->GetDirectBufferAddress(env, out) : NULL;
  const uint64_t cap = out ? (uint64_t)(*env)->GetDirectBufferCapacity(env, out) : 0;
  uint64_t *o = NULL;
  jsize no = 0;
  if (out && offs) {
    no = (*env)->GetArrayLength(env, offs);
    o = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(no ? no : 1));
    if (!o) {
      throw_for(env, HBAM_E_NOMEM, "out of memory");
      return -1;
    }
  }
  int rc = hbam_encode_writables(CTX(h), dst, cap, o, &len);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
  } else if (o && no) {
    (*env)->SetLongArrayRegion(env, offs, 0, no, (const jlong *)o);
  }
  free(o);
  return (jlong)len;
}

JNIEXPORT jlong FN(openCodec)(JNIEnv *env, jclass c, jint device) {
  hbam_opts o = {device, 0, HBAM_STRICT, 0, 0, 0};
  hbam_ctx *ctx = NULL;
  int rc = hbam_open_codec(&o, &ctx);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(ctx));
    if (ctx) hbam_close(ctx);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT jobjectArray FN(decodeWritables)(JNIEnv *env, jclass c, jlong h, jobject buf, jlongArray offs) {
  jsize n;
  uint64_t *o = from_longs(env, offs, &n);
  if (!o) return NULL;
  const void *p = (*env)->GetDirectBufferAddress(env, buf);
  const uint64_t len = (uint64_t)(*env)->GetDirectBufferCapacity(env, buf);
  hbam_batch b;
  memset(&b, 0, sizeof b);
  int rc = p ? hbam_decode_writables(CTX(h), p, len, o, (uint64_t)n, &b) : HBAM_E_ARG;
  free(o);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(CTX(h)));
    return NULL;
  }
  return wrap_batch(env, &b);
}

JNIEXPORT jbyteArray FN(bgzfCompress)(JNIEnv *env, jclass c, jint device, jobject payload, jintArray lens,
                                      jint level, jboolean eof) {
  hbam_opts o = {device, 0, HBAM_STRICT, 0, 0, 0};
  const void *p = (*env)->GetDirectBufferAddress(env, payload);
  const uint64_t plen = (uint64_t)(*env)->GetDirectBufferCapacity(env, payload);
  const jsize nb = lens ? (*env)->GetArrayLength(env, lens) : 0;
  jint *l = lens ? (*env)->GetIntArrayElements(env, lens, NULL) : NULL;
  uint8_t *buf = NULL;
  uint64_t len = 0;
  int rc = p ? hbam_bgzf_compress(&o, p, plen, (const uint32_t *)l, (uint64_t)nb, 0, level,
                                  eof ? HBAM_BGZF_EOF : 0, &buf, &len)
             : HBAM_E_ARG;
  if (l) (*env)->ReleaseIntArrayElements(env, lens, l, JNI_ABORT);
  if (rc != HBAM_OK) {
    throw_for(env, rc, hbam_last_error(NULL));
    return NULL;
  }
  jbyteArray a = to_bytes(env, buf, len);
  hbam_free(buf);
  return a;
}

JNIEXPORT jlong FN(getKey)(JNIEnv *env, jclass c, jint ref, jint start) { return (jlong)hbam_get_key(ref, start); }

JNIEXPORT jlong FN(getKey0)(JNIEnv *env, jclass c, jint ref, jint start0) { return (jlong)hbam_get_key0(ref, start0); }

JNIEXPORT jlong FN(murmurhash3)(JNIEnv *env, jclass c, jbyteArray key, jint seed) {
  const jsize n = (*env)->GetArrayLength(env, key);
  jbyte *k = (*env)->GetByteArrayElements(env, key, NULL);
  if (!k) return 0;
  const int64_t h = hbam_murmurhash3(k, (uint64_t)n, seed);
  (*env)->ReleaseByteArrayElements(env, key, k, JNI_ABORT);
  return (jlong)h;
}

JNIEXPORT jlong FN(releaseCachedMemory)(JNIEnv *env, jclass c) { return (jlong)hbam_release_cached_memory(); }
