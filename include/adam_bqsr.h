/*
 * adam_bqsr.h -- C ABI of the MI355X-native BQSR (base quality score
 * recalibration) path.  This is the drop-in boundary that replaces the two
 * JVM function bodies of ADAM's RecalibrateBaseQualities:
 *
 *   observe : RecalibrateBaseQualities.computeTable  (the per-partition
 *             `aggregate` fold)      adam-core/.../rdd/RecalibrateBaseQualities.scala:52-64
 *   apply   : RecalibrateBaseQualities.applyTable    (the per-partition
 *             `map(recalibrate)`)    adam-core/.../rdd/RecalibrateBaseQualities.scala:66-76
 *
 * The driver-side pieces stay host-side and are exported separately:
 *   merge    : RecalTable.++          adam-core/.../rdd/recalibration/RecalTable.scala:90-108
 *   finalize : RecalTable.finalizeTable                  RecalTable.scala:117-126
 *   sites    : SnpTable (known-site mask)   adam-core/.../models/SnpTable.scala:12-47
 *
 * The public Scala API in front of these bodies is unchanged:
 *   AdamRecordRDDFunctions.adamBQSR(dbSNP: SnpTable)  core/rdd/AdamRDDFunctions.scala:104-107
 *   `adam transform -recalibrate_base_qualities [-dbsnp_sites f]` cli/Transform.scala:47-50
 * (INTEGRATION.md shows the JNI stubs a maintainer adds to those closures.)
 *
 * Conventions
 *  - plain C, POD structs, no torch / HIP types in any signature; `stream`
 *    arguments are a hipStream_t passed as void* (NULL = the library's own
 *    per-thread stream);
 *  - the library owns every handle and the device memory behind it; every
 *    handle has a *_destroy;
 *  - every function returns a bqsr_status; on failure bqsr_last_error()
 *    returns a thread-local message and, for data errors, the index of the
 *    first offending read (in read order) is reported through
 *    bqsr_last_error_read();
 *  - all exports are re-entrant: Spark local[N] calls observe/apply from N
 *    task threads at once.  merge/finalize are single-threaded driver calls.
 */
#ifndef ADAM_BQSR_H
#define ADAM_BQSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BQSR_ABI_VERSION 1

/* Status codes.  Data errors mirror the JVM exception the reference throws
 * on the same input (it fails the whole Spark job). */
typedef enum bqsr_status {
  BQSR_OK = 0,
  BQSR_ERR_NULL_RG = 1,          /* NullPointerException, QualByRG: StandardCovariate.scala:28            */
  BQSR_ERR_MD_PARSE = 2,         /* IllegalArgumentException, MdTag.apply: MdTag.scala:52,75              */
  BQSR_ERR_CIGAR_SHORT = 3,      /* IndexOutOfBoundsException, referencePositions(o): RichADAMRecord.scala:191 */
  BQSR_ERR_BAD_REVCOMP_BASE = 4, /* NoSuchElementException, COMPL_MP(b): StandardCovariate.scala:70       */
  BQSR_ERR_EMPTY_TABLE = 5,      /* UnsupportedOperationException("empty.reduceLeft"): RecalTable.scala:123 */
  BQSR_ERR_MISSING_KEY = 6,      /* NoSuchElementException, readGroupCounts/qualByRGCounts: RecalTable.scala:129,135 */
  BQSR_ERR_QUAL_RANGE = 7,       /* ArrayIndexOutOfBoundsException, phredToErrorProbability: PhredUtils.scala:32 */
  BQSR_ERR_NULL_FIELD = 8,       /* NullPointerException on a null qual/sequence/cigar/start/referenceName */
  BQSR_ERR_SEQ_SHORT = 9,        /* ArrayIndexOutOfBoundsException: covariate arrays shorter than the quals */
  BQSR_ERR_CIGAR_INVALID = 10,   /* NoSuchElementException: zero-length M/X/=/S element (Range.last)     */
  BQSR_ERR_INVALID_ARG = 11,     /* bad call: null pointer, inconsistent sizes, dims mismatch            */
  BQSR_ERR_DEVICE = 12,          /* HIP runtime failure                                                  */
  BQSR_ERR_UNSUPPORTED = 13,     /* input outside what the device path handles          */
  BQSR_ERR_SAM_PARSE = 14        /* malformed SAM text where read_sam / SAMRecordConverter throws (adam_sam.h) */
} bqsr_status;

/* ADAMRecord boolean fields (adam-format/.../adam.avdl:28-38) and null-ness
 * of the optional fields BQSR dereferences.  A field absent in the record is
 * a 0 bit. */
enum {
  BQSR_F_PAIRED = 1u << 0,         /* readPaired          */
  BQSR_F_MAPPED = 1u << 1,         /* readMapped          */
  BQSR_F_NEG_STRAND = 1u << 2,     /* readNegativeStrand  */
  BQSR_F_SECOND_OF_PAIR = 1u << 3, /* secondOfPair        */
  BQSR_F_PRIMARY = 1u << 4,        /* primaryAlignment    */
  BQSR_F_DUPLICATE = 1u << 5,      /* duplicateRead       */
  BQSR_F_HAS_RG = 1u << 8,         /* recordGroupId != null        */
  BQSR_F_HAS_MD = 1u << 9,         /* mismatchingPositions != null */
  BQSR_F_HAS_QUAL = 1u << 10,      /* qual != null                 */
  BQSR_F_HAS_SEQ = 1u << 11,       /* sequence != null             */
  BQSR_F_HAS_CIGAR = 1u << 12,     /* cigar != null                */
  BQSR_F_HAS_START = 1u << 13,     /* start != null                */
  BQSR_F_HAS_REFNAME = 1u << 14    /* referenceName != null        */
};

/* BAM CIGAR op codes (len << 4 | op), the samtools CigarOperator order. */
enum { BQSR_CIGAR_M = 0, BQSR_CIGAR_I = 1, BQSR_CIGAR_D = 2, BQSR_CIGAR_N = 3, BQSR_CIGAR_S = 4,
       BQSR_CIGAR_H = 5, BQSR_CIGAR_P = 6, BQSR_CIGAR_EQ = 7, BQSR_CIGAR_X = 8 };

/* Contig id meaning "referenceName is not a SnpTable contig" (not masked,
 * SnpTable.scala:21-22 catches the lookup failure). */
#define BQSR_CONTIG_UNKNOWN (-1)

/* One partition of ADAMRecords flattened to columns: what the JNI shim fills
 * from the Spark partition iterator.  Strings are byte columns addressed by
 * [n_reads+1] offset arrays (Arrow layout). */
typedef struct bqsr_records {
  int64_t n_reads;
  const uint32_t* flags;        /* [n] BQSR_F_* bits                                   */
  const int32_t* rg_id;         /* [n] recordGroupId (RecordGroupDictionary index)    */
  const int32_t* contig_id;     /* [n] index into the bqsr_sites contig list, or BQSR_CONTIG_UNKNOWN */
  const int64_t* start;         /* [n] 0-based alignment start                         */
  const uint64_t* seq_offset;   /* [n+1] into seq                                      */
  const uint8_t* seq;           /* sequence bytes (ASCII)                              */
  const uint64_t* qual_offset;  /* [n+1] into qual                                     */
  const uint8_t* qual;          /* quality chars, phred+33 (ASCII)                     */
  const uint64_t* cigar_offset; /* [n+1] into cigar                                    */
  const uint32_t* cigar;        /* BAM-encoded CIGAR elements (len<<4 | op)            */
  const uint64_t* md_offset;    /* [n+1] into md                                       */
  const uint8_t* md;            /* MD:Z strings                                        */
} bqsr_records;

/* Dense covariate-table dimensions.  The reference's RecalTable is a
 * HashMap[qualByRG key -> Array(cycle map, context map)]; the dense form has
 *   K = 60*(n_rg-1) + 128 keys (q + 60*rg, RecalTable key aliasing kept),
 *   C = 2*max_len + 1 cycle slots (cycle c -> c + max_len),
 *   X = 21 context slots (ctx x -> x + 4, x in [-4, 16]). */
typedef struct bqsr_dims {
  int32_t n_rg;    /* read groups (max recordGroupId + 1) */
  int32_t max_len; /* longest sequence                   */
} bqsr_dims;

typedef struct bqsr_context bqsr_context; /* device, streams, static tables  */
typedef struct bqsr_sites bqsr_sites;     /* known sites (SnpTable)          */
typedef struct bqsr_batch bqsr_batch;     /* device-resident packed reads    */
typedef struct bqsr_table bqsr_table;     /* device-resident count table     */
typedef struct bqsr_lut bqsr_lut;         /* finalized table / apply tables  */

/* ---- library / errors ---------------------------------------------------- */
int bqsr_abi_version(void);
const char* bqsr_last_error(void);
int64_t bqsr_last_error_read(void);
const char* bqsr_status_name(bqsr_status s);

/* Open the library on a HIP device (one context per device / rank). */
bqsr_status bqsr_context_create(int device, bqsr_context** out);
void bqsr_context_destroy(bqsr_context* ctx);

/* Layout knobs of a context, for tests and A/B measurements (no reference
 * counterpart; results are identical under every setting).  They take effect
 * on batches created afterwards.  The defaults are the measured choices
 * (DESIGN.md §3).
 *   BQSR_TUNE_ORDER     -1 auto (read-group buckets for several read groups
 *                        or quals beyond one window), 0 read order, 1 buckets
 *   BQSR_TUNE_FRONTS    -1 auto, 0 none, f > 0: f fronts of bucketed batches
 *   BQSR_TUNE_KEYMAJOR   0 off (default: the copy costs ~17 cfg4 jobs of its
 *                        saving), 1 key-major copy of bucketed batches
 *   BQSR_TUNE_FUSED_PREP 0 only: a prep kernel of its own (the form with
 *                        prep inside the observe kernel was measured slower
 *                        and removed; 1 is refused)
 *   BQSR_TUNE_BGZF       1 BAM ingest inflates BGZF on the device (default:
 *                        each block decoded to symbols by a thread, then
 *                        assembled and CRC-checked in LDS by a workgroup;
 *                        a file it cannot take -- a block that does not
 *                        inflate or check, a record chain it cannot prove --
 *                        falls back to 0), 0 on up to 16 host threads */
enum { BQSR_TUNE_ORDER = 1, BQSR_TUNE_FRONTS = 2, BQSR_TUNE_KEYMAJOR = 3, BQSR_TUNE_FUSED_PREP = 4, BQSR_TUNE_BGZF = 5 };
bqsr_status bqsr_context_tune(bqsr_context* ctx, int knob, int64_t value);

/* ---- known sites (SnpTable.apply(File) + broadcast, SnpTable.scala:32-47,
 *      AdamRDDFunctions.scala:105) ------------------------------------------ */
/* positions are the VCF POS values exactly as stored (no -1: quirk Q7).  Each
 * contig's list may be unsorted / contain duplicates. */
bqsr_status bqsr_sites_create(bqsr_context* ctx, const char* const* contigs, const int64_t* const* pos,
                              const uint64_t* n, int32_t n_contigs, bqsr_sites** out);
void bqsr_sites_destroy(bqsr_sites* s);

/* ---- reads --------------------------------------------------------------- */
/* Pack a record partition into the device layout (4-bit base codes, phred
 * bytes, 16+24 B per-read metadata, CIGAR, MD) and upload it. */
bqsr_status bqsr_batch_create(bqsr_context* ctx, const bqsr_records* recs, void* stream, bqsr_batch** out);
void bqsr_batch_destroy(bqsr_batch* b);
int64_t bqsr_batch_reads(const bqsr_batch* b);
int64_t bqsr_batch_bases(const bqsr_batch* b);
bqsr_dims bqsr_batch_dims(const bqsr_batch* b);
/* Measurement: redo the layout a bucketed batch builds once at creation
 * (piece-key sort, key-major copy of quals and codes) into its buffers
 * (allocated with the batch) and report its wall time in *ms (-1: the batch
 * has no such layout).  Synchronous on `stream`. */
bqsr_status bqsr_batch_relayout(bqsr_batch* b, void* stream, double* ms);
/* The same layout's cost when the batch was created, split into the
 * allocation of its buffers and its kernels (wall ms, each synchronised;
 * -1 when the batch built none). */
bqsr_status bqsr_batch_layout_times(const bqsr_batch* b, double* alloc_ms, double* build_ms);

/* Caller-owned device buffers already in the packed layout (used by the
 * benchmark, which synthesises reads directly in HBM).  Layout documented in
 * DESIGN.md §"Data layout in HBM".  No copy; buffers must outlive the batch. */
typedef struct bqsr_device_reads {
  int64_t n_reads;
  int64_t n_slots;        /* total base slots (sum of max(Ls, Lq) per read)           */
  const void* meta;       /* [n] 16-B records {u64 slot; u16 lq; u16 ls; u16 flags; u16 rg} */
  const void* align;      /* [n] 24-B records {i64 start; u32 cigar_off; u32 md_off; i32 contig; u16 n_cigar; u16 md_len} */
  const uint8_t* qual;    /* [n_slots + 32] phred bytes (qual char - 33, as Java byte);
                             the 32 bytes past the end must be readable (16-B loads) */
  const uint8_t* bases;   /* [(n_slots+1)/2 + 32] 4-bit codes A0 C1 G2 T3 N4 other5,
                             low nibble first; 32 readable bytes of padding likewise */
  const uint32_t* cigar;  /* BAM elements; 32 readable bytes of padding past the end     */
  const uint8_t* md;      /* MD bytes; 32 readable bytes of padding past the end        */
  bqsr_dims dims;
  int32_t slots_aligned;  /* nonzero: every slot is a multiple of 16 and each read's
                             slot range is max(Ls, Lq) rounded up to 16 (the layout
                             bqsr_batch_create builds); the per-base passes then use
                             aligned 16-B accesses                                    */
} bqsr_device_reads;
bqsr_status bqsr_batch_wrap_device(bqsr_context* ctx, const bqsr_device_reads* dev, bqsr_batch** out);

/* ---- streamed partitions (BASELINE cfg5: partitions streamed from the host
 *      with the H2D copy of one overlapping the kernels of another) ---------
 * Replaces, per Spark task, the hand-over of one partition of
 * `RecalibrateBaseQualities.computeTable`'s input (RecalibrateBaseQualities.scala:52-64)
 * when the JNI side streams partitions rather than calling bqsr_batch_create
 * per partition.  bqsr_stage_records packs the partition once into pinned host
 * memory in the device layout; bqsr_batch_create_staged allocates matching
 * device columns (no copy); bqsr_batch_upload_async enqueues the H2D copies on
 * `stream` without a host sync (the caller orders its compute stream after it
 * with an event).  A batch may be re-uploaded from the same staged partition
 * any number of times; each upload invalidates the batch's prep results.  Any
 * other staged partition (even one of the same shape) is refused with
 * BQSR_ERR_INVALID_ARG: the batch's launch parameters come from its own. */
typedef struct bqsr_staged bqsr_staged;
bqsr_status bqsr_stage_records(bqsr_context* ctx, const bqsr_records* recs, bqsr_staged** out);
void bqsr_staged_destroy(bqsr_staged* s);
int64_t bqsr_staged_bytes(const bqsr_staged* s);
int64_t bqsr_staged_reads(const bqsr_staged* s);
int64_t bqsr_staged_bases(const bqsr_staged* s);
bqsr_status bqsr_batch_create_staged(bqsr_context* ctx, const bqsr_staged* s, bqsr_batch** out);
bqsr_status bqsr_batch_upload_async(bqsr_batch* b, const bqsr_staged* s, void* stream);

/* ---- table --------------------------------------------------------------- */
/* int64 words of a dense table: [touched K][obs K*(C+X)][mm K*(C+X)]. */
int64_t bqsr_table_words(bqsr_dims d);
/* Zeroed table in library memory, or over caller device memory (e.g. a torch
 * tensor that takes part in an RCCL all-reduce) when `device_words` != NULL. */
bqsr_status bqsr_table_create(bqsr_context* ctx, bqsr_dims d, void* device_words, bqsr_table** out);
void bqsr_table_destroy(bqsr_table* t);
bqsr_dims bqsr_table_dims(const bqsr_table* t);
void* bqsr_table_device_ptr(bqsr_table* t);
/* Copy to / from host int64 arrays in the word layout above. */
bqsr_status bqsr_table_download(const bqsr_table* t, int64_t* host_words);
bqsr_status bqsr_table_upload(bqsr_table* t, const int64_t* host_words);

/* ---- observe: computeTable's per-partition fold ------------------------- */
/* Folds every usable read (readMapped && primaryAlignment && !duplicateRead &&
 * mismatchingPositions != null, RecalibrateBaseQualities.scala:29-32) of the
 * batch into `table` (added to its counts) and returns the partition's
 * expectedMismatch, folded from 0.0 in read/base order exactly as Spark's
 * per-partition foldLeft does (RecalTable.scala:61).  `sites` may be NULL
 * (SnpTable()). */
bqsr_status bqsr_observe(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, bqsr_table* table,
                         double* expected_mismatch, void* stream);

/* Host-records convenience form of the survey's `bqsr_observe(soa, sites,
 * out_partial, out_em)`: packs, uploads, observes into a fresh table. */
bqsr_status bqsr_observe_records(bqsr_context* ctx, const bqsr_records* recs, const bqsr_sites* sites,
                                 bqsr_dims dims, bqsr_table** out_partial, double* out_expected_mismatch);

/* ---- merge: RecalTable.++ on the driver ---------------------------------- */
/* acc += part (int64, exact); *acc_em = *acc_em + part_em (the caller owns
 * the merge order, H1 in SURVEY.md).  Dims must match. */
bqsr_status bqsr_table_merge(bqsr_table* acc, const bqsr_table* part, double* acc_em, double part_em);

/* ---- finalize: RecalTable.finalizeTable ---------------------------------- */
/* Returns BQSR_ERR_EMPTY_TABLE where the reference throws
 * UnsupportedOperationException("empty.reduceLeft"). */
bqsr_status bqsr_finalize(bqsr_context* ctx, const bqsr_table* t, double expected_mismatch, bqsr_lut** out);
void bqsr_lut_destroy(bqsr_lut* l);
/* Finalized statistics (RecalTable fields): average reported error, global
 * counts, and per-read-group counts ((key-1)/60 grouping). */
typedef struct bqsr_final_stats {
  double average_reported_error;
  double global_error;
  int64_t global_obs, global_mm;
  int32_t n_groups; /* group slots reported in rg_obs/rg_mm (index r + 1; slot 0 = group -1 unused) */
} bqsr_final_stats;
bqsr_status bqsr_lut_stats(const bqsr_lut* l, bqsr_final_stats* out);
/* getErrorRateShifts for one base covariate (RecalTable.scala:128-152):
 * shifts[0..3] = readGroupDelta, qualScoreDelta, cycleDelta, contextDelta;
 * *new_q = errorProbabilityToPhred(fold).  qual_by_rg = q + 60*rg. */
bqsr_status bqsr_lut_shifts(const bqsr_lut* l, int32_t qual_by_rg, int32_t qual, int32_t cycle, int32_t context,
                            double shifts[4], int32_t* new_q);

/* ---- apply: applyTable's per-partition map -------------------------------- */
/* Device form.  For every read: eligible reads (mapped && primary && !dup,
 * RecalibrateBaseQualities.scala:69) get new quality chars
 * (char)(Q+33) for read offsets [st, end) written at out_qual[slot+st ..
 * slot+end) (low byte), with out_start[r] = st, out_len[r] = end-st;
 * ineligible reads are passed through (out_start 0, out_len Lq, chars copied).
 * Codes that do not fit a byte (Q+33 > 255 after Java's (char) narrowing) are
 * reported through the exception list: (slot index, 16-bit code) pairs;
 * *n_exceptions counts them (the list holds at most max_exceptions).
 * All output pointers are device pointers. */
bqsr_status bqsr_apply(bqsr_context* ctx, bqsr_batch* b, const bqsr_lut* l, uint8_t* out_qual,
                       uint32_t* out_start, uint32_t* out_len, uint64_t* exceptions, int64_t max_exceptions,
                       int64_t* n_exceptions, void* stream);

/* Host-records form: out_qual is host uint16_t[qual_offset[n]] (Java chars),
 * read r's new qual string is out_qual[qual_offset[r] .. + out_len[r]). */
bqsr_status bqsr_apply_records(bqsr_context* ctx, const bqsr_records* recs, const bqsr_lut* l,
                               uint16_t* out_qual, uint32_t* out_len);

/* ---- asynchronous / staged device API -------------------------------------
 * The calls above synchronise.  These enqueue on `stream` and return at once,
 * so a driver can keep a whole BQSR job on the device (the benchmark and the
 * multi-GPU path use them; RCCL collectives go between the stages). */
enum { BQSR_STAGE_RESET = 1, BQSR_STAGE_KERNEL = 2, BQSR_STAGE_FOLD = 4, BQSR_STAGE_PREP = 8,
       BQSR_STAGE_LUT = 16, BQSR_STAGE_NO_LUT = 32 };
/* apply stages: RESET clears its error words, KERNEL builds the pieces' char
 * tables (bqsr_apply_chars) and runs the apply kernel; LUT builds the char
 * tables only, KERNEL | NO_LUT runs the kernel on tables an earlier LUT
 * stage built for the same LUT (so a caller can time the kernel alone). */
/* observe stages: RESET clears the error word, PREP is the per-read prep
 * kernel (trimming, CIGAR/MD/known-site masks, validation), KERNEL the
 * observe kernel, FOLD the expectedMismatch fold (result at
 * bqsr_batch_em_device_ptr). */
bqsr_status bqsr_observe_stage(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, bqsr_table* t,
                               int32_t stages, void* stream);
bqsr_status bqsr_observe_async(bqsr_context* ctx, bqsr_batch* b, const bqsr_sites* sites, bqsr_table* t,
                               void* stream);
/* waits for the stream, returns the data error (if any) and the partition's expectedMismatch */
bqsr_status bqsr_observe_result(bqsr_batch* b, double* expected_mismatch, void* stream);
void* bqsr_batch_em_device_ptr(bqsr_batch* b);
bqsr_status bqsr_table_zero_async(bqsr_table* t, void* stream);
/* finalize into *out.  *out must be NULL or a LUT returned by an earlier
 * finalize: one of the same dims and context is reused (no allocation), any
 * other is destroyed and replaced. */
bqsr_status bqsr_finalize_async(bqsr_context* ctx, const bqsr_table* t, double expected_mismatch, bqsr_lut** out,
                                void* stream);
bqsr_status bqsr_finalize_result(bqsr_lut* l, void* stream);
/* as bqsr_finalize_async, with the expectedMismatch read on the device (one
 * double at em_device: bqsr_batch_em_device_ptr, or the rank-order fold of
 * the all-gathered values), so observe -> finalize -> apply needs no host
 * round trip */
bqsr_status bqsr_finalize_device(bqsr_context* ctx, const bqsr_table* t, const double* em_device, bqsr_lut** out,
                                 void* stream);
/* copy the batch's expectedMismatch (one double) to a device buffer, on `stream` */
bqsr_status bqsr_batch_em_copy_async(bqsr_batch* b, double* dst_device, void* stream);
/* RecalTable.++ of n partitions' expectedMismatch in the given order
 * (RecalTable.scala:90-108): *out_device = ((0.0 + ems[0]) + ems[1]) + ...,
 * computed on the device on `stream` (ems_device: n doubles).  The multi-rank
 * and streamed paths gather every partition's value and fold them in global
 * partition order with this. */
bqsr_status bqsr_em_fold_async(bqsr_context* ctx, const double* ems_device, int64_t n, double* out_device,
                               void* stream);
/* apply stages: RESET clears the error word and exception count, KERNEL the
 * apply kernel; PREP (re)runs the prep kernel, which also runs by itself when
 * observe has not prepared this batch */
bqsr_status bqsr_apply_stage(bqsr_context* ctx, bqsr_batch* b, const bqsr_lut* l, uint8_t* out_qual,
                             uint32_t* out_start, uint32_t* out_len, uint64_t* exceptions, int64_t max_exceptions,
                             int32_t stages, void* stream);
bqsr_status bqsr_apply_async(bqsr_context* ctx, bqsr_batch* b, const bqsr_lut* l, uint8_t* out_qual,
                             uint32_t* out_start, uint32_t* out_len, uint64_t* exceptions, int64_t max_exceptions,
                             void* stream);
bqsr_status bqsr_apply_result(bqsr_batch* b, int64_t* n_exceptions, void* stream);

/* ---- introspection --------------------------------------------------------- */
/* LDS window of the covariate table a batch's launches privatise: read group
 * rg_lo, quals q_lo.. (chosen from the packed quals; settable for device batches). */
bqsr_status bqsr_batch_set_window(bqsr_batch* b, int32_t q_lo, int32_t rg_lo);
int32_t bqsr_batch_reads_per_tile(const bqsr_batch* b);
/* base slots of the packed layout (sum over reads of max(Ls, Lq) rounded up to 16): the size of
 * apply's out_qual */
int64_t bqsr_batch_slots(const bqsr_batch* b);
/* read-group counts of a finalized table, group r at (r >= -1): 1 found, 0 absent, -1 error */
int bqsr_lut_group(const bqsr_lut* l, int32_t r, int64_t* obs, int64_t* mm);
/* the errorProbabilityToPhred threshold table the apply kernel uses:
 * out[i] = largest p with phred(p) >= qmin + i; returns the entry count */
int32_t bqsr_phred_threshold_table(double* out, int32_t cap, int32_t* qmin);

/* A copy by a kernel on `stream` (either side may be pinned host memory the
 * device can address): the streamed path's D2H of results, which then runs
 * beside the DMA engines' H2D of the next partitions instead of sharing them
 * (tools/link_probe.hip).  Any size; 16-B aligned buffers move in 16-B
 * pieces, unaligned ones byte by byte.  Replaces, for the JNI side, the memcpy of a partition's
 * output buffers back into the executor's direct buffers. */
bqsr_status bqsr_copy_async(bqsr_context* ctx, void* dst, const void* src, int64_t bytes, void* stream);
/* The same for a size the device holds: bytes = min(*count * scale, max_bytes)
 * (count a u32 or u64, count_bytes 4 / 8) -- the compacted outputs below,
 * whose length the host does not know when it enqueues the copy. */
bqsr_status bqsr_copy_dyn_async(bqsr_context* ctx, void* dst, const void* src, const void* count, int32_t count_bytes,
                                int64_t scale, int64_t max_bytes, void* stream);
/* A partition's apply outputs compacted for the trip to the host (the JNI
 * side's result buffers hold just the new quality strings, Q13):
 * chars[offsets[r] .. offsets[r + 1]) = the out_len[r] chars of read r
 * (device buffers: chars >= the batch's slots, offsets u32 [n + 1]); with
 * `lengths` (u16 [n], may be NULL) also each read's char count -- what a
 * caller ships instead of the offsets (half the bytes; the offsets are its
 * prefix sum).  The exception list's entries are rewritten to (position in
 * chars) << 16 | char.  Enqueued on `stream` after the apply stage;
 * bqsr_batch_exception_count_ptr is the device word holding the exception
 * count (for bqsr_copy_dyn_async). */
bqsr_status bqsr_compact_outputs_async(bqsr_context* ctx, bqsr_batch* b, const uint8_t* out_qual,
                                       const uint32_t* out_start, const uint32_t* out_len, uint64_t* exceptions,
                                       int64_t max_exceptions, uint8_t* chars, uint32_t* offsets, uint16_t* lengths,
                                       void* stream);
const void* bqsr_batch_exception_count_ptr(const bqsr_batch* b);

/* One job's launches with the fewest host round trips (what bench.py's step
 * runs): the table zeroed and the batch's error words reset in one kernel
 * (replaces bqsr_table_zero_async and the BQSR_STAGE_RESET stages), and, after
 * the stages, every status of the job fetched in one transfer: the observe
 * error, expectedMismatch, finalize's EMPTY_TABLE, the apply error and the
 * exception count, raised in the reference's order. */
bqsr_status bqsr_job_reset_async(bqsr_batch* b, bqsr_table* t, void* stream);
bqsr_status bqsr_job_result(bqsr_batch* b, bqsr_lut* l, double* expected_mismatch, int64_t* n_exceptions,
                            void* stream);
/* Multi-rank jobs (one partition per rank, in rank order): the reference's
 * job fails with the first error of the first failing partition
 * (RecalibrateBaseQualities.scala:63,75 -- a Spark job aborts on its first
 * failed task).  export writes the batch's observe and apply error keys,
 * rebased to global read indices (reads before this rank's = read_base), as
 * two int64 at dst_device (no error = INT64_MAX); the caller all-reduces them
 * with MIN over the ranks and imports the result, so bqsr_job_result raises
 * the same error (global read index) on every rank. */
/* Pipelined jobs (streamed partitions, adam_amd/stream.py): the batch's
 * status of one job -- observe error, expectedMismatch, finalize's
 * EMPTY_TABLE, apply error, exception count -- snapshot on `stream` into
 * pinned slot `slot` (< 4) without a sync; after the caller has waited for
 * the stream past that point, bqsr_job_status_get returns the part's status
 * (0 observe, 1 finalize, 2 apply), so the job's errors are raised in the
 * reference's order while the next job already runs. */
bqsr_status bqsr_job_status_async(bqsr_batch* b, bqsr_lut* l, int32_t slot, void* stream);
bqsr_status bqsr_job_status_get(const bqsr_batch* b, int32_t slot, int32_t part, double* expected_mismatch,
                                int64_t* n_exceptions);
bqsr_status bqsr_job_errors_export_async(bqsr_batch* b, int64_t read_base, int64_t* dst_device, void* stream);
bqsr_status bqsr_job_errors_import_async(bqsr_batch* b, const int64_t* src_device, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ADAM_BQSR_H */
