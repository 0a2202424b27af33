// bqsr_internal.h -- device data layout and kernel parameter blocks shared by
// the HIP kernels (bqsr_kernels.hip) and the host side (bqsr_capi.cpp).
// Layout rationale: DESIGN.md "Data layout in HBM".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/adam_bqsr.h"

namespace bqsr {

// ---- per-read records (SoA of fixed-size records) --------------------------
// 16 B: what the per-base passes need.
struct ReadMeta {
  uint64_t slot;   // first base slot of the read in qual[] / bases[]
  uint16_t lq;     // quality length (Lq)
  uint16_t ls;     // sequence length (Ls)
  uint16_t flags;  // BQSR_F_* (bits 0-5, 8-14) | kSeqOther
  uint16_t rg;     // recordGroupId
};
static_assert(sizeof(ReadMeta) == 16, "ReadMeta must be 16 B");

// 24 B: alignment fields, read by the prep kernel only.
struct ReadAlign {
  int64_t start;       // 0-based alignment start
  uint32_t cigar_off;  // into cigar[]
  uint32_t md_off;     // into md[]
  int32_t contig;      // index into the known-site contigs, <0 unknown
  uint16_t n_cigar;
  uint16_t md_len;
};
static_assert(sizeof(ReadAlign) == 24, "ReadAlign must be 24 B");

// 8 B per read, written by the prep kernel for the observe / apply passes.
// Invariant: on the device a ReadInfo is read and written as ONE aligned
// 64-bit access (info_load / info_store).  A bucketed batch's fold runs on a
// second stream beside bqsr_observe_chunks, which writes deferred trims back
// (kInfoTrim -> the resolved range) while the fold kernels read the same
// words: a torn read (new fl without kInfoTrim, old st = en = 0) would drop
// the read from the fold.  Both sides resolve a kInfoTrim word to the same
// value, so either whole word is correct.
struct alignas(8) ReadInfo {
  uint16_t st;  // qualityStartOffset
  uint16_t en;  // qualityEndOffset, or the offset of the read's first error
  uint16_t fl;  // kInfo* bits
  uint16_t pad;
};
static_assert(sizeof(ReadInfo) == 8 && alignof(ReadInfo) == 8, "ReadInfo must be one aligned 8-B word");
__device__ __forceinline__ ReadInfo info_load(const ReadInfo* p) {
  const uint64_t v = __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return ReadInfo{(uint16_t)v, (uint16_t)(v >> 16), (uint16_t)(v >> 32), (uint16_t)(v >> 48)};
}
__device__ __forceinline__ void info_store(ReadInfo* p, ReadInfo x) {
  const uint64_t v = (uint64_t)x.st | ((uint64_t)x.en << 16) | ((uint64_t)x.fl << 32) | ((uint64_t)x.pad << 48);
  __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr uint16_t kInfoObs = 1;        // usable, valid: its bases go into the table
constexpr uint16_t kInfoObsCheck = 2;   // usable, fails at `en`: bases before it are only qual-checked
constexpr uint16_t kInfoApp = 4;        // eligible for recalibration, valid
constexpr uint16_t kInfoAppCheck = 8;   // eligible, fails at `en`: bases before it only checked
constexpr uint16_t kInfoNeg = 16;       // readNegativeStrand
constexpr uint16_t kInfoSecond = 32;    // readPaired && secondOfPair (DiscreteCycle negates)
constexpr uint16_t kInfoPass = 64;      // not eligible: quality string passed through
constexpr uint16_t kInfoCycNeg = 128;   // (tile record only) cycle cell decreases with the slot
constexpr uint16_t kInfoTrim = 256;     // st / en not computed yet (prep's lock-step path reads no
                                        // quals): the first pass over the read's quals trims it
                                        // (resolve_info), observe writes the result back
constexpr uint16_t kInfoNoBits = 512;   // the read has no masked / mismatch bit (prep's common-read
                                        // path): the per-base passes do not load its slot-bitmap words

// packer-derived flag: the sequence holds a byte outside "ACGTN"
// (BaseContext.simpleReverseComplement throws on it for reverse reads,
// StandardCovariate.scala:55-57,70).
constexpr uint16_t kSeqOther = 1u << 15;

// 4-bit base codes
constexpr uint8_t kCodeA = 0, kCodeC = 1, kCodeG = 2, kCodeT = 3, kCodeN = 4, kCodeOther = 5;

constexpr int kMaxQ = 60;      // RecalUtil.Constants.MAX_REASONABLE_QSCORE
constexpr int kCtxSlots = 21;  // contexts -4..16
constexpr uint32_t kCtxTab = 4096;            // context table entries per strand (3 codes of 4 bits)
constexpr int kCtxTabBytes = 2 * kCtxTab * 2;  // both strands, u16 entries (LDS of the per-base passes)
constexpr int kQBins = 128;    // qual values 0..127 (Java byte >= 0)

// Read tiles: `reads_per_tile` consecutive reads (<= 64) whose base slots fit
// in kTileSlots.  Tiles are the unit of the expectedMismatch fold (per-tile
// qual histograms); the per-base passes split the batch into per-workgroup
// ranges of whole tiles and give each lane one read.
constexpr int kTileSlots = 4096;
constexpr int kMaxTileReads = 64;
constexpr int kMaxFoldBlocks = 1024;  // workgroups of the per-base passes (one per CU)
constexpr int kWaves = 16;  // waves per workgroup of the per-base passes (1024 threads)
constexpr int kBlockThreads = 64 * kWaves;
constexpr int kMkWords = kWaves * 64;  // LDS of the lane-per-chunk walk: one marker word per lane
constexpr int kMaxReadLen = 4096;  // longest read the device path takes
constexpr int kColumnPad = 32;     // readable bytes past the end of the qual / bases columns
constexpr int kRedSlabs = 16;      // slabs one bqsr_window_reduce thread sums (grid y splits the rest)

// Error reporting: u64 words, atomicMin of
//   read << 28 | read_offset << 8 | rank << 4 | code
// so the first failing read (read order), and within it the first failing
// base / step, wins -- the exception the JVM would raise first.
constexpr uint64_t kNoError = ~0ull;
__host__ __device__ inline uint64_t err_key(uint64_t read, uint32_t o, uint32_t rank, uint32_t code) {
  return (read << 28) | ((uint64_t)(o & 0xFFFFF) << 8) | ((uint64_t)(rank & 0xF) << 4) | (code & 0xF);
}
// ranks at one read offset, in the order ReadCovariates.next evaluates them
enum : uint32_t {
  kRankCtor = 0,   // constructor: qual / RG / sequence / reverse complement
  kRankCigar = 1,  // referencePositions (null cigar/start, empty range, index past the end)
  kRankMd = 2,     // mdEvent parse
  kRankSnp = 3,    // SnpTable: null referenceName
  kRankCov = 4,    // BaseCovariates: covariate arrays shorter than the quals
  kRankTable = 5   // RecalTable += / getErrorRateShifts
};
// error words of a batch
enum { kErrObs = 0, kErrAppPrep = 1, kErrAppKern = 2, kNExc = 3, kErrWords = 4 };
constexpr int kJobStatusWords = 16;  // bqsr_job_result: error words, em, FinalOut
constexpr int kStatusSlots = 4;      // bqsr_job_status_async: snapshots of pipelined jobs

// ---- known sites -------------------------------------------------------------
struct SitesDev {
  const int64_t* pos;          // all contigs' sorted unique positions
  const uint64_t* off;         // [n_contigs + 1]
  const uint32_t* bucket;      // per contig: first site index (relative) with pos >= base + (b << shift)
  const uint64_t* bucket_off;  // [n_contigs + 1] into bucket
  const int64_t* bucket_base;  // [n_contigs] position of bucket 0 (min pos)
  // per contig a bitmap of site positions (bit p - bm_base = a site at raw POS
  // p); a contig whose bitmap would be too sparse has none (bm_off equal)
  const uint64_t* bm;
  const uint64_t* bm_off;      // [n_contigs + 1] words into bm
  const int64_t* bm_base;      // [n_contigs] position of bit 0 (a multiple of 64)
  int32_t n_contigs;
  int32_t shift;
};

// ---- table geometry ----------------------------------------------------------
struct TableGeom {
  int32_t K;      // 60*(n_rg-1) + 128
  int32_t C;      // 2*L + 1
  int32_t L;      // max_len
  int32_t cells;  // C + 21
};

// LDS window of the covariate table: rows (rg_lo, q_lo .. q_lo+qw-1).
struct Window {
  int32_t qw;
  int32_t q_lo;
  int32_t rg_lo;
};

struct ReadsDev {
  const ReadMeta* meta;
  const ReadAlign* align;
  const uint8_t* qual;
  const uint8_t* bases;
  const uint32_t* cigar;
  const uint8_t* md;
  int64_t n_reads;
  int64_t n_slots;  // base slots of the batch (qual[] holds n_slots bytes, bases[] n_slots nibbles)
  int32_t reads_per_tile;
  int64_t n_tiles;
  int32_t slots_aligned;  // every read's slot is a multiple of 16 and its slot range is padded to 16
                          // (slot_span): the per-base passes then walk 16-aligned chunks
};
// slots a read takes in the packed layout (bqsr_batch_create pads to 16)
__host__ __device__ inline uint64_t slot_span(uint64_t lq, uint64_t ls) {
  const uint64_t sl = lq > ls ? lq : ls;
  return (sl + 15) & ~(uint64_t)15;
}

// Slot bitmap: u64 word i covers base slots 32i .. 32i+31 of the batch, bit j
// of the low half = slot 32i+j is masked, of the high half = it mismatches.
struct PrepParams {
  ReadsDev rd;
  SitesDev sites;
  ReadInfo* info;      // [n_reads]
  uint64_t* sbits;     // [n_slots / 32 + 4]: each workgroup clears its reads' words first, or (store_words) pass 1 writes them whole
  int32_t store_words; // pass 1 stores every sbits word (reads of <= 128 bases), no zeroing, no atomics
  uint64_t* bnd;       // store_words: per wavefront of pass 1 [bits, word] its first read's share of the word the previous wavefront stored
  unsigned long long* err;  // error words
  uint32_t* work;      // [n_reads] reads bqsr_prep_kernel left to bqsr_prep_complex, per workgroup segment
  uint32_t* n_work;    // [workgroups] their count per segment
};

// Read order of the per-base passes.  With one read group whose table rows
// fit the LDS windows, the passes walk the batch in read order (perm ==
// nullptr).  Otherwise reads are bucketed by key = 2 * read group + mate
// class (a device counting sort, bqsr_key_*): sorted position i holds read
// perm[i], and key_off[k] .. key_off[k+1] are the positions of key k.  The
// mate class (readPaired && secondOfPair) decides the sign of DiscreteCycle,
// so a key's reads only use half of the cycle cells: cycles 1..L (cells
// L+1..2L) for class 0, -L..-1 (cells 0..L-1) for class 1 -- the windows
// hold that half only (WinGeom).  Workgroup w takes the positions [a_w,
// a_w+1) (tile-aligned, wg_begin) and walks them as "pieces", one per key it
// meets, with that key's rows in its LDS window: a piece's counts go to slab
// (w + k).  (w + k is unique: the key is nondecreasing along the order.)
struct OrderDev {
  const uint32_t* perm;    // [n_reads] or nullptr (identity, one piece per workgroup, group = Window::rg_lo)
  const int64_t* key_off;  // [n_keys + 1]
  int32_t n_keys;          // 2 * n_rg when bucketed
  // fronts (n_base > 0): keys are (front, base key) = front * n_base + base
  // key, a front being a contiguous share of the read indices, and workgroup
  // w of the chunk-walk passes takes key w whole -- so the workgroups of one
  // front sweep the same read range together and share its cache lines
  // (bqsr_capi.cpp fronts()).  0: keys are base keys, ranges by wg_begin.
  int32_t n_base = 0;
  // key-major copy (bqsr_capi.cpp layout_build): when set, the bucketed
  // passes read quals / base codes from a copy laid out in perm order -- the
  // read at sorted position p at kslot[p] -- so a piece's reads are
  // contiguous; the ReadsDev they get points at that copy, and the slot
  // bitmap and outputs stay at the read's own slot (LaneRead::oslot)
  const uint64_t* kslot = nullptr;
};

struct ObserveParams {
  ReadsDev rd;
  OrderDev ord;
  ReadInfo* info;  // read; trimmed ranges left to observe (kInfoTrim) are written back
  const uint64_t* sbits;  // PrepParams::sbits
  TableGeom g;
  Window w;
  int64_t* touched;  // [K]
  int64_t* obs;      // [K*cells]
  int64_t* mm;       // [K*cells]
  uint32_t* part;      // [n_blocks + n_keys - 1][part_stride] per-piece window counts (obs, mm, touched)
  int32_t part_stride; // 2*qw*wcells + qw, wcells = WinGeom::cw + 21
  uint32_t* hq_block;  // [n_blocks][128] per-block qual histogram of folded bases (identity order; bucketed
                       // batches: bqsr_fold_hist)
  unsigned long long* err;
  int32_t n_blocks;
  int32_t wcells;      // window row length: WinGeom::cw + 21
  int32_t lane_shift;  // lane-per-chunk kernels: log2(lanes per read)
  int32_t orow;        // bqsr_observe_lean: LDS obs row words (nc copies of the cycle and 43 context cells), 2 mod 4
  int32_t nc;          // bqsr_observe_lean: copies of a row's counters (<= 4)
  int32_t rows_all;    // bqsr_observe_lean: every qual of the batch is a window row (host histogram)
};

// ---- expectedMismatch fold (bqsr_fold.hip) ----
constexpr int32_t kFoldNoBase = INT32_MIN;  // FoldBlock::e of a block without folded bases
constexpr int kSegBinades = 32;             // binades a candidate block's tiles are tabulated at
constexpr double kFoldTie = -1.0, kFoldUnknown = -2.0;
constexpr int kFoldMaxSegs = 64;            // segments per candidate block (the rest: one fallback segment)
enum : int32_t { kSegRun = 0, kSegEvent = 1, kSegGlobal = 2 };

// per fold block (one observe workgroup's range of tiles), bqsr_fold_plan
struct FoldBlock {
  double r0, r1;  // real sum of the folded quals before / after the block (approximate)
  double inc;     // event-free block: its exact increment at binade e, in units 2^(e-52)
  int32_t e;      // event-free: the binade the whole block stays in
  int32_t cidx;   // candidate index (bqsr_fold_segs workgroup), -1 when event-free
};
static_assert(sizeof(FoldBlock) == 32, "FoldBlock is 4 words");

// a run of tiles of a candidate block, bqsr_fold_segs
struct FoldSeg {
  int64_t inc;         // kSegRun: exact increment at binade e; kSegEvent: element count
  int32_t t0, t1;      // tiles t0 .. t1
  int32_t e;           // kSegRun: the binade; kSegEvent: the lowest binade >= kFoldSeqLimit it may start in
  int32_t kind;        // kSegRun / kSegEvent (quals at streams + off) / kSegGlobal (folded from the columns)
  int64_t off;
};
static_assert(sizeof(FoldSeg) == 32, "FoldSeg is 4 words");

struct FoldParams {
  ReadsDev rd;
  const ReadInfo* info;
  const uint32_t* hq_block;  // [n_blocks][128] qual histograms of the folded bases, read order
  const double* pow10;       // phredToErrorProbabilityCache[0..127]
  int32_t n_blocks;
  FoldBlock* blk;            // [n_blocks]
  int32_t* cand_list;        // [n_blocks] candidate blocks in block order
  int32_t* n_cand;
  double* delta;             // relative bound of |exact - real| partial sums
  double* rtile;             // [n_tiles] candidate blocks' tiles: real sum
  int32_t* ntile;            //           folded bases
  double* dtile;             //           [kSegBinades] exact increments at the block's binades eb0 ..
                             //           (kFoldTie / kFoldUnknown when a qual ties / not exact)
  FoldSeg* seg;              // segments of all candidate blocks, each block's consecutive
  int32_t* seg_base;         // [n_blocks] candidate c's first segment
  int32_t* nseg;             // [n_blocks] and count
  uint32_t* seg_used;
  uint8_t* streams;          // event segments' quals in fold order, each segment 64-B aligned
  double* csum;              // [stream_cap / 64][2] per 64 quals of a stream: exact increment at the
                             // segment's binades e, e + 1 (kFoldTie / kFoldUnknown sentinels)
  int64_t stream_cap;
  unsigned long long* stream_used;
  double* em_out;            // [1]
  uint32_t* qmask;           // [4] the histograms' bins holding a base (apply skips its
                             // clean-row test for folded reads when they all lie in clean rows)
};

// errorProbabilityToPhred by buckets: p's binade (unbiased exponent
// kQbElo..kQbEhi) and top 5 mantissa bits select a bucket holding at most one
// phred threshold: Q = p <= qb_thr[b] ? qb_q[b] : qb_q[b] - 1.  Other p take
// the full threshold table (thr).
constexpr int kQbElo = -48;
constexpr int kQbEhi = 3;
constexpr int kQbBits = 5;
constexpr int kQbN = (kQbEhi - kQbElo + 1) << kQbBits;

struct ApplyParams {
  ReadsDev rd;
  OrderDev ord;
  const ReadInfo* info;
  TableGeom g;
  Window w;               // qw rows of the per-piece char table
  int32_t n_rg;
  const double* s1;       // [n_rg*128][C]  a2 + cycleDelta
  const double* d2;       // [n_rg*128][21] contextDelta
  const uint8_t* rq_ok;   // [n_rg*128]     key touched && read group present
  const uint8_t* key_ok;  // [K]  touched
  const uint8_t* grp_ok;  // [n_groups] group r exists at index r+1
  int32_t n_groups;
  const double* thr;      // phred thresholds, see PhredThresholds
  int32_t thr_qmin;       // Q value of thr[0]
  int32_t thr_n;
  const double* qb_thr;   // [kQbN]
  const int16_t* qb_q;    // [kQbN]
  uint8_t* out_qual;      // [n_slots]; slots outside the recalibrated ranges are scratch
  uint32_t* out_start;
  uint32_t* out_len;
  unsigned long long* exc;  // (slot << 16 | code16)
  int64_t max_exc;
  unsigned long long* n_exc;
  unsigned long long* err;
  int32_t lane_shift;  // lane-per-chunk kernel: log2(lanes per read)
  int32_t outs_apart;  // the per-read outputs (out_start / out_len) by bqsr_apply_outs in read order, not the walk
  const uint8_t* chars;   // [n_keys][piece_stride] the pieces' char tables (bqsr_apply_chars)
  int64_t piece_stride;   // bytes per piece: qw * cw * 21 rounded up to 16
  uint32_t* rowbad;       // [n_keys][4] rows of a piece's char table holding a 0 entry (bit per row)
  const uint32_t* qmask;  // [4] qual bins of the batch's folded bases (FoldParams::qmask), or null
};

// finalize results read back by the host
struct FinalOut {
  int64_t g_obs, g_mm;
  double avg, global_error;
  int32_t any_key;
  int32_t pad;
};
// bqsr_job_status_kernel's host words: error words, expectedMismatch, FinalOut
static_assert(kErrWords + 1 + sizeof(FinalOut) / 8 <= (size_t)kJobStatusWords, "job status words overflow");
static_assert(sizeof(FinalOut) % 8 == 0, "FinalOut is whole words");

// errorProbabilityToPhred step function: thr[i] = the largest p > 0 whose
// javaD2I(-10*log10(p)) >= thr_qmin + i.  Q(p) = max{n : p <= thr[n - qmin]}.
constexpr int kThrQmin = -3100;
constexpr int kThrQmax = 3300;
constexpr int kThrN = kThrQmax - kThrQmin + 1;

}  // namespace bqsr
