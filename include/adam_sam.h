/*
 * adam_sam.h -- SAM text into and out of the device around the BQSR path
 * (SURVEY.md §8 rows f1, f2, f3), part of libadam_bqsr.so.
 *
 *   ingest  : sc.adamLoad of a SAM file          adam-core/.../rdd/AdamContext.scala:122-137
 *             SAMRecordConverter.convert         adam-core/.../converters/SAMRecordConverter.scala:26-144
 *             RecordGroupDictionary (sorted ids) adam-core/.../models/RecordGroupDictionary.scala:36-43
 *             with the BQSR column projection    adam-core/.../projections/ADAMRecordField.scala:28-71
 *   output  : the recalibrated records written back (adamSave,
 *             adam-core/.../rdd/AdamRDDFunctions.scala:37-56) -- here as SAM
 *             text: every record's QUAL field replaced by the string
 *             RecalUtil.recalibrate built (trimmed length, Q13; Java chars
 *             as UTF-8, Q14), every other byte of the record kept
 *   dedup   : MarkDuplicates (adam-core/.../rdd/MarkDuplicates.scala:24-111),
 *             the `-mark_duplicate_reads` step `transform` runs before BQSR
 *             (adam-cli/.../cli/Transform.scala:73-76)
 *
 * Same conventions as adam_bqsr.h (bqsr_status results, bqsr_last_error(),
 * library-owned handles with *_destroy, `stream` = hipStream_t as void*).
 */
#ifndef ADAM_SAM_H
#define ADAM_SAM_H

#include "adam_bqsr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A parsed SAM file: the text and the record columns, in device memory. */
typedef struct bqsr_sam bqsr_sam;

/* Parse a whole SAM file (header + records) as read_sam does
 * (adam_amd/records.py, the SAMRecordConverter semantics): start = POS - 1
 * when RNAME is a header @SQ name and POS != 0; flag bits only when the flag
 * word is non-zero (quirk Q2); MD:Z -> mismatchingPositions; RG:Z -> the
 * index of the name among the sorted @RG IDs; referenceName ids in order of
 * first appearance.  Header lines are parsed on the host, records on the
 * device (line split, field split, CIGAR text -> BAM u32 elements).
 * `text` is host memory (pinned or not).  BQSR_ERR_SAM_PARSE where the
 * reference's parser throws (fewer than 11 fields, a tag without two ':', a
 * malformed CIGAR or FLAG / POS); BQSR_ERR_UNSUPPORTED for header lines after
 * the first record and lone '\r' bytes. */
bqsr_status bqsr_sam_parse(bqsr_context* ctx, const char* text, int64_t n_bytes, void* stream, bqsr_sam** out);
void bqsr_sam_destroy(bqsr_sam* s);
/* BAM bytes (BGZF) -> the same parse bqsr_sam_parse builds from the SAM
 * text of the same records (AdamContext.scala:122-137 adamBamLoad,
 * SAMRecordConverter.scala:26-144): BGZF blocks inflated (and their CRC32
 * checked) by host threads; on the device every record becomes its SAM text
 * line (integer tag types as "i", floats by Java's Float.toString, arrays as
 * B:t,...) and the lines go through the SAM record parser.  So every call
 * on a SAM parse -- rewrite, text download, MarkDuplicates, ADAM columns --
 * serves BAM input too. */
bqsr_status bqsr_bam_parse(bqsr_context* ctx, const uint8_t* bam, int64_t n_bytes, void* stream, bqsr_sam** out);

typedef struct bqsr_sam_counts {
  int64_t n_reads;     /* records (empty lines skipped)   */
  int64_t seq_bytes;   /* Σ SEQ field lengths            */
  int64_t qual_bytes;  /* Σ QUAL field lengths           */
  int64_t cigar_ops;   /* Σ CIGAR elements               */
  int64_t md_bytes;    /* Σ MD:Z value lengths           */
  int64_t text_bytes;  /* the SAM text (input, or the rewritten text after bqsr_sam_rewrite_quals) */
  int32_t n_ref_names; /* distinct referenceNames used    */
  int32_t n_read_groups;
} bqsr_sam_counts;
bqsr_status bqsr_sam_get_counts(const bqsr_sam* s, bqsr_sam_counts* out);
/* referenceName i (ref_index order: first appearance in the records) */
const char* bqsr_sam_ref_name(const bqsr_sam* s, int32_t i);

/* The record columns (bqsr_records layout; ref_index as RecordBatch keeps it:
 * index into the bqsr_sam_ref_name list, -1 when referenceName is null). */
typedef struct bqsr_sam_columns {
  uint32_t* flags;
  int32_t* rg_id;
  int32_t* ref_index;
  int64_t* start;
  uint64_t* seq_offset;
  uint8_t* seq;
  uint64_t* qual_offset;
  uint8_t* qual;
  uint64_t* cigar_offset;
  uint32_t* cigar;
  uint64_t* md_offset;
  uint8_t* md;
} bqsr_sam_columns;
/* device pointers of the columns (valid while `s` lives) */
bqsr_status bqsr_sam_device_columns(const bqsr_sam* s, bqsr_sam_columns* out);
/* copy the columns to caller-allocated host arrays sized by bqsr_sam_get_counts */
bqsr_status bqsr_sam_download(const bqsr_sam* s, const bqsr_sam_columns* dst);

/* The parse's records as a BQSR batch, packed on the device: the layout,
 * launch window and read order bqsr_batch_create builds from the same
 * records' host columns (bqsr_sam_download), without the columns leaving the
 * device.  ref_contig[i] = the bqsr_sites contig index of referenceName i
 * (bqsr_sam_ref_name order) or BQSR_CONTIG_UNKNOWN; n_ref may be 0 (no known
 * sites).  The batch owns its columns (the parse may be destroyed).
 * BQSR_ERR_UNSUPPORTED as bqsr_batch_create (fields beyond 65535, a
 * recordGroupId beyond 65535, reads longer than the device path takes). */
bqsr_status bqsr_sam_batch_create(bqsr_context* ctx, const bqsr_sam* s, const int32_t* ref_contig, int32_t n_ref,
                                  void* stream, bqsr_batch** out);

/* ADAMRecord Parquet (§8 f1/f2): adamLoad with the BQSR projection
 * (core/rdd/AdamContext.scala:139-161, projections/Projection.scala:10-34) as
 * Arrow decodes it on the host -- the column buffers uploaded as they are and
 * turned into the parse layout on the device.  One bqsr_arrow_chunk per Arrow
 * record batch (array offsets 0); a NULL column is all null.  String columns:
 * int32 offsets [n+1], UTF-8 bytes, validity bitmap (NULL: all valid); chars
 * are Java chars (a 4-byte UTF-8 sequence is a surrogate pair): a qual char c
 * enters as the byte c & 0xFF, a sequence / MD char as min(c, 0xFF) (as
 * adam_amd/parquet.py).  CIGAR strings are parsed by samtools
 * TextCigarCodec's rules (BQSR_ERR_SAM_PARSE, read index, when malformed).
 * reference = referenceName dictionary indices (the caller's dictionary; the
 * ref_contig map of bqsr_arrow_batch_create is indexed by them).  Booleans: a
 * null reads as false. */
typedef struct bqsr_arrow_strings {
  const int32_t* offsets;
  const uint8_t* data;
  const uint8_t* validity;
} bqsr_arrow_strings;
typedef struct bqsr_arrow_chunk {
  int64_t n_reads;
  bqsr_arrow_strings sequence, qual, cigar, md; /* md = mismatchingPositions */
  const int32_t* reference;
  const uint8_t* reference_validity;
  const int64_t* start;
  const uint8_t* start_validity;
  const int32_t* record_group; /* recordGroupId */
  const uint8_t* record_group_validity;
  /* readPaired, readMapped, readNegativeStrand, secondOfPair, primaryAlignment, duplicateRead */
  const uint8_t* bools[6];
  const uint8_t* bools_validity[6];
  /* MarkDuplicates only (NULL otherwise): readName; referenceId (NULL: the
   * referenceName index); library = 1 + the rank of recordGroupLibrary among
   * the input's sorted distinct libraries, 0 for null */
  bqsr_arrow_strings read_name;
  const int32_t* reference_id;
  const uint8_t* reference_id_validity;
  const int32_t* library;
} bqsr_arrow_chunk;
typedef struct bqsr_arrow bqsr_arrow;
bqsr_status bqsr_arrow_load(bqsr_context* ctx, const bqsr_arrow_chunk* chunks, int32_t n_chunks, void* stream,
                            bqsr_arrow** out);
void bqsr_arrow_destroy(bqsr_arrow* a);
int64_t bqsr_arrow_reads(const bqsr_arrow* a);
/* the records as a BQSR batch (as bqsr_sam_batch_create) */
bqsr_status bqsr_arrow_batch_create(bqsr_context* ctx, const bqsr_arrow* a, const int32_t* ref_contig, int32_t n_ref,
                                    void* stream, bqsr_batch** out);
/* The qual column after apply (adamSave of the recalibrated records): per
 * read the recalibrated chars as UTF-8 (pass-through reads keep their input
 * string; null where the input had none and nothing was written), built on
 * the device; prepare returns the byte count, column copies the Arrow
 * buffers (int32 offsets [n+1], bytes, validity bitmap) to the host.  b ==
 * NULL keeps every input string. */
bqsr_status bqsr_arrow_qual_prepare(bqsr_context* ctx, bqsr_arrow* a, const bqsr_batch* b, const uint8_t* out_qual,
                                    const uint32_t* out_start, const uint32_t* out_len, const uint64_t* exceptions,
                                    int64_t n_exceptions, void* stream, int64_t* n_bytes);
bqsr_status bqsr_arrow_qual_column(const bqsr_arrow* a, int32_t* offsets, uint8_t* data, uint8_t* validity);
/* MarkDuplicates over the reads (bqsr_sam_mark_duplicates' rules; readName
 * and library from the chunk columns): the duplicateRead bits of the
 * records (and of the batches built after) set or cleared */
bqsr_status bqsr_arrow_mark_duplicates(bqsr_context* ctx, bqsr_arrow* a, int64_t* n_duplicates);
/* the reads' flag bit `flag` (a BQSR_F_* value) as an Arrow boolean bitmap */
bqsr_status bqsr_arrow_flag_bitmap(const bqsr_arrow* a, uint32_t flag, uint8_t* bitmap);

/* Output (§8 f2): replace every record's QUAL field by its recalibrated
 * string.  out_qual / out_start / out_len / exceptions are the device
 * buffers bqsr_apply_async wrote for batch `b`, built from this parse's
 * records in read order (b's slot of read r = its qual chars' base).
 * Recalibrated reads get the chars of [out_start, out_start + out_len) as
 * UTF-8 (chars above 0xFF from the exception list); pass-through reads keep
 * their QUAL bytes; with b == NULL every QUAL field is kept.  After
 * bqsr_sam_mark_duplicates the FLAG fields are rewritten too (0x400 = the
 * duplicateRead MarkDuplicates gave the read).  The header is kept, empty
 * lines are dropped and every record ends with '\n'.  The new text
 * replaces the parse's on the device. */
bqsr_status bqsr_sam_rewrite_quals(bqsr_context* ctx, bqsr_sam* s, const bqsr_batch* b, const uint8_t* out_qual,
                                   const uint32_t* out_start, const uint32_t* out_len, const uint64_t* exceptions,
                                   int64_t n_exceptions, void* stream);
/* copy the (rewritten) SAM text to host memory of at least counts.text_bytes */
bqsr_status bqsr_sam_text_download(const bqsr_sam* s, char* dst);

/* ADAMRecord columns (§8 f2: adamSave of SAMRecordConverter's records,
 * core/rdd/AdamRDDFunctions.scala:37-56, converters/SAMRecordConverter.scala:
 * 26-144) of records [r0, r0 + n) of the parse, from its current text (after
 * bqsr_sam_rewrite_quals: the recalibrated QUAL and MarkDuplicates' FLAG).
 * Record-level columns in Arrow layout, built on the device:
 *   strings (int32 offsets [n+1], bytes, validity bitmap): readName, sequence,
 *     cigar (re-encoded, "*" when empty), qual, mismatchingPositions (MD),
 *     attributes (every tag but MD as TG:T:value, descending binary tag,
 *     tab-joined; "" without tags);
 *   int32 (+ validity): referenceId, mapq, mateReferenceId, recordGroupId;
 *   int64 (+ validity): start, mateAlignmentStart;
 *   bitmaps: readPaired, properPair, readMapped, mateMapped,
 *     readNegativeStrand, mateNegativeStrand, firstOfPair, secondOfPair,
 *     primaryAlignment, failedVendorQualityChecks, duplicateRead.
 * Bitmaps are Arrow's (bit r of word r / 64, LSB first).  The columns that
 * depend only on the read group or the @SQ entry (referenceName,
 * recordGroup*, referenceLength / Url, mate*) come from the header text by
 * index (bqsr_sam_header_text).  An H or B tag, or an 'i' tag outside Int,
 * gives BQSR_ERR_UNSUPPORTED (the reference's attribute conversion throws).
 * prepare: pass 1 and the sizes; columns: pass 2 and the copies into the
 * caller's host buffers (NULL pointers skip a column). */
typedef struct bqsr_adam_sizes {
  int64_t n_reads;
  int64_t str_bytes[6];
  int64_t bitmap_words; /* u64 words of each bitmap */
} bqsr_adam_sizes;
typedef struct bqsr_adam_host {
  int32_t* str_offsets[6];
  uint8_t* str_bytes[6];
  uint64_t* str_valid[6];
  int32_t* i32[4];
  int64_t* i64[2];
  uint64_t* int_valid[6]; /* referenceId, mapq, mateReferenceId, recordGroupId, start, mateAlignmentStart */
  uint64_t* bools[11];
} bqsr_adam_host;
bqsr_status bqsr_sam_adam_prepare(bqsr_context* ctx, bqsr_sam* s, int64_t r0, int64_t n, void* stream,
                                  bqsr_adam_sizes* out);
bqsr_status bqsr_sam_adam_columns(bqsr_context* ctx, bqsr_sam* s, const bqsr_adam_host* dst, void* stream);
/* The ADAM columns' qual from an apply's outputs for batch `b` (built from
 * this parse in read order) instead of the text's QUAL, as
 * bqsr_sam_rewrite_quals would write them (pass-through reads keep theirs),
 * without rewriting the text; the device buffers must outlive the following
 * prepare / columns calls.  b == NULL: the text's QUAL again.  After
 * MarkDuplicates the duplicateRead column follows its bits either way. */
bqsr_status bqsr_sam_adam_set_quals(bqsr_context* ctx, bqsr_sam* s, const bqsr_batch* b, const uint8_t* out_qual,
                                    const uint32_t* out_start, const uint32_t* out_len, const uint64_t* exceptions,
                                    int64_t n_exceptions, void* stream);
/* the header lines of the parse (SAM input, or a BAM's header text) */
bqsr_status bqsr_sam_header_text(const bqsr_sam* s, char* dst, int64_t cap, int64_t* len);

/* MarkDuplicates (§8 f3): adam-core/.../rdd/MarkDuplicates.scala:24-111 over
 * SingleReadBucket (models/SingleReadBucket.scala:27-37: reads grouped by
 * (recordGroupId, readName)) and ReferencePositionPair
 * (models/ReferencePositionPair.scala:27-63: the buckets' 5' positions,
 * RichADAMRecord.scala:77-118).  Buckets grouped by (left position,
 * library), then by right position; the best-scoring bucket of a group
 * (score = Σ quals >= 15 of its primary reads, :37-39) keeps its primary
 * reads, every other mapped read of the group is a duplicate, unmapped reads
 * never are.  Ties go to the bucket seen first (Spark leaves their order to
 * its shuffle).  Host C++: a grouping step in front of the device passes. */
typedef struct bqsr_dup_reads {
  int64_t n_reads;
  const char* const* read_name; /* [n] readName (NULL = null)                      */
  const char* const* library;   /* [n] recordGroupLibrary (NULL = null)            */
  const uint32_t* flags;        /* [n] BQSR_F_* (PAIRED, MAPPED, NEG_STRAND, PRIMARY, HAS_RG) */
  const uint8_t* mate_mapped;   /* [n] mateMapped                                  */
  const int32_t* rg_id;         /* [n] recordGroupId (when BQSR_F_HAS_RG)          */
  const int32_t* reference_id;  /* [n] referenceId                                 */
  const int64_t* start;         /* [n] 0-based start                               */
  const uint64_t* qual_offset;  /* [n+1] */
  const uint8_t* qual;          /* phred+33 chars                                  */
  const uint64_t* cigar_offset; /* [n+1] */
  const uint32_t* cigar;        /* BAM-encoded elements                            */
} bqsr_dup_reads;
/* dup[r] = the duplicateRead value MarkDuplicates gives read r */
bqsr_status bqsr_mark_duplicates(const bqsr_dup_reads* reads, uint8_t* dup);
/* The same over a parse (readName = QNAME, referenceId = the @SQ index,
 * mateMapped from FLAG 0x8, library = the read group's LB); the parse's
 * flags column gets BQSR_F_DUPLICATE set or cleared accordingly, as
 * `transform -mark_duplicate_reads` does before BQSR. */
bqsr_status bqsr_sam_mark_duplicates(bqsr_sam* s, int64_t* n_duplicates);

/* MarkDuplicates across the partitions of one input (the reference's
 * groupBy spans every partition of the RDD, MarkDuplicates.scala:43-58).
 * add: one partition's parse (partitions in input order, each parsed with
 * the same header); its reads get global indices after those added before.
 * Per read the set keeps a compact record on the device (two 64-bit hashes
 * of (rg, QNAME), class, packed 5' position, score, library rank; 31 bytes),
 * so partitions need not stay resident.  finish: buckets, groups and the
 * duplicate bit of every read (the passes of bqsr_sam_mark_duplicates);
 * records are released.  apply: a parse of partition `part` (the same text
 * as added) gets its reads' duplicateRead bits, as bqsr_sam_mark_duplicates
 * leaves them.  Reads of different partitions share a bucket when both
 * hashes agree (names are not compared across partitions: a 128-bit
 * collision would merge two buckets).  BQSR_ERR_UNSUPPORTED for more than
 * 2^32 - 1 reads or positions / libraries beyond the packed keys;
 * BQSR_ERR_INVALID_ARG for partitions whose headers name other libraries. */
typedef struct bqsr_dup_set bqsr_dup_set;
bqsr_status bqsr_dup_set_create(bqsr_context* ctx, int64_t reads_hint, bqsr_dup_set** out);
bqsr_status bqsr_dup_set_add(bqsr_dup_set* d, const bqsr_sam* s);
bqsr_status bqsr_dup_set_finish(bqsr_dup_set* d, int64_t* n_duplicates);
bqsr_status bqsr_dup_set_apply(bqsr_dup_set* d, int64_t part, bqsr_sam* s, int64_t* n_duplicates);
void bqsr_dup_set_destroy(bqsr_dup_set* d);

/* adamSave's GZIP part files (AdamRDDFunctions.scala:37-48 through
 * parquet-mr; ParquetArgs.scala:27: GZIP by default).  `in` is a Parquet file
 * written UNCOMPRESSED (Arrow's writer: schema, encodings, dictionary pages,
 * statistics), here rewritten to `path` with every page a gzip member:
 * the columns named in `huffman_cols` (comma-separated top-level names, e.g.
 * "qual,sequence") as one dynamic-Huffman DEFLATE block of literals, the
 * others by libdeflate (zlib when absent) at `level` (zlib's default 6 is
 * Hadoop's GzipCodec); page headers, column-chunk metadata and the footer
 * re-encoded with the new sizes and offsets.  Data page v1 and dictionary
 * pages; no page index, bloom filter or external column chunks
 * (BQSR_ERR_INVALID_ARG otherwise).  `threads` compress pages in parallel.
 * *out_len: bytes written. */
bqsr_status bqsr_parquet_gzip(const uint8_t* in, int64_t in_len, const char* path, int32_t level,
                              const char* huffman_cols, int32_t threads, int64_t* out_len);
/* One gzip member of n bytes into out (cap bytes; *out_len the size, also
 * when it does not fit): huffman != 0 the literal-only Huffman block, else
 * libdeflate / zlib at `level` (tests). */
bqsr_status bqsr_gzip_bytes(const uint8_t* in, int64_t n, int32_t huffman, int32_t level, uint8_t* out, int64_t cap,
                            int64_t* out_len);

#ifdef __cplusplus
}
#endif

#endif /* ADAM_SAM_H */
